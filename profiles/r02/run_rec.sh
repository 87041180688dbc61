# jump-record sweep pair: parity tests, then the headline bench with the record and with
# snapshots on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/rec; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rec.py tests/test_gpu_eta_modes.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread > gpurun_out/rec/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/rec/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/rec/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  for r in jumps snapshots; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --record $r > gpurun_out/rec/bench_${r}_$i.json 2> gpurun_out/rec/bench.err || { tail -5 gpurun_out/rec/bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/rec/bench_${r}_$i.json')); print('$r', '%.4g' % d['value'], 'ms', '%.4f' % d['ms_per_step'], 'adj', '%.2f' % d['roofline']['launch_us'], '%.3f' % d['roofline']['frac'], 'fwd', '%.2f' % d['roofline_fwd']['launch_us'], '%.3f' % d['roofline_fwd']['frac'], 'idx', d['refine_index'])"
  done
done
