# Round 3 full pass on the 8-byte record + Np = 9 pair tiles: the whole GPU suite, smoke, the
# driver bench (N = 4) and N = 8, and a rocprof kernel-stats profile of the driver command.
set -o pipefail
OUT=gpurun_out/r03/full1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -m gpu tests/ -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --N 8 --no-cpu-baseline > $OUT/bench_N8.json 2> $OUT/bench_N8.err || { tail $OUT/bench_N8.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_rocprof.json 2> $OUT/rocprof.err || { tail $OUT/rocprof.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_N8', 'bench_rocprof'):
  d = json.load(open('$OUT/%s.json' % f)); print(f, d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['launch_steps'], d['launch_steps_fwd'])"
find $OUT/prof -name "*kernel_stats.csv" | head -2
