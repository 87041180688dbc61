# Final library: whole GPU suite + smoke; the record default at K = 2^20, 2^21, 2^22 (how the
# per-launch fill/drain and the partial last round of workgroups weigh at each size).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/f3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
for k in 1048576 2097152 4194304; do
  timeout -k 10 300 python bench.py --K $k --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_K$k.json 2> $OUT/err_K$k || { tail -5 $OUT/err_K$k; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('K', sys.argv[2], '%.4g'%d['value'], 'adj %.1f fwd %.1f'%(d['roofline']['launch_us'],d['roofline_fwd']['launch_us']))" $OUT/bench_K$k.json $k
done
