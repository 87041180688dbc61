# Re-verify the final library build: the p-estimate suites, the bench tests, smoke and the
# p bench line (which now reads profiles/r05/p)
set -o pipefail
out=gpurun_out/r05/verify; mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_psweep.py tests/test_gpu_pflow.py tests/test_gpu_dwr.py tests/test_gpu_bench.py tests/test_gpu_sweep.py > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --indicator p > $out/bench_p.json 2> $out/bench_p.err || { tail $out/bench_p.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench_p.json')); r=d['roofline']; print('%.4g' % d['value'], r['launch_us'], r['traffic'], r['traffic_source'], d['roofline_fp64'].get('pmc_issued_frac'))"
echo all-done
