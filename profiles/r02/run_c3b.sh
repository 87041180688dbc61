# config-3: tests + bench (after the tile-width / SGPR changes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decisions.py tests/test_gpu_nonlinear.py tests/test_gpu_checkpoint.py -v --timeout 240 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_c3.log | head -20; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > gpurun_out/bench_c3_$i.json 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3_$i.json')); print('c3', d['value'], 'adj', d['roofline']['launch_us'], d['roofline']['frac'], 'fwd', d['roofline_fwd']['launch_us'], d['roofline_fwd']['frac'])"
done
