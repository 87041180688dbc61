# Closing GPU pass (round 2): every GPU test, the driver's bench command, the rocprof /
# PMC collection of the default (jump-record) bench, the snapshot bench for comparison, and
# SQ counters of the record kernels.   bash profiles/r02/run_final.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/final/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_driver.json 2> gpurun_out/final/bench_driver.err || { tail -20 gpurun_out/final/bench_driver.err; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --record snapshots > gpurun_out/final/bench_snapshots.json 2> gpurun_out/final/bench_snap.err || { tail -20 gpurun_out/final/bench_snap.err; exit 1; }
bash profiles/r02/collect.sh || exit 1
bash profiles/r02/collect_sq.sh fwd_rec fwd_rec --nsteps 20 || exit 1
bash profiles/r02/collect_sq.sh adj_rec adj_rec --nsteps 20 || exit 1
python3 -c "
import json
for f in ('bench_driver', 'bench_snapshots'):
  d = json.load(open('gpurun_out/final/%s.json' % f))
  print(f, '%.4g' % d['value'], 'adj', '%.2f' % d['roofline']['launch_us'], '%.3f' % d['roofline']['frac'], 'fwd', '%.2f' % d['roofline_fwd']['launch_us'], '%.3f' % d['roofline_fwd']['frac'])
"
