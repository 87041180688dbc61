# Round 3 full pass on the Horner-form pair kernels: the whole GPU suite, smoke, the driver
# bench (N = 4) and N = 8, then rocprof kernel stats + PMC traffic (profiles/r03/collect.sh).
set -o pipefail
OUT=gpurun_out/r03/full2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -m gpu tests/ -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --N 8 --no-cpu-baseline > $OUT/bench_N8.json 2> $OUT/bench_N8.err || { tail $OUT/bench_N8.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_N8'):
  d = json.load(open('$OUT/%s.json' % f)); print(f, d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['launch_steps'], d['launch_steps_fwd'])"
bash profiles/r03/collect.sh || exit 1
