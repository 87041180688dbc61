# Round 3: the 8-byte jump record + pair tiles at Np = 9.  GPU tests of the record path, the A/B
# of the sweep shapes, and the driver bench at N = 4 and N = 8.
set -o pipefail
OUT=gpurun_out/r03/rec8; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_golden_stages.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u profiles/r03/ab_rec.py --rounds 9 > $OUT/ab.json 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
timeout -k 10 300 python -u profiles/r03/ab_rec.py --rounds 7 --N 8 --variants 20:10,10:10,10:10:1,5:5:1,20:20 > $OUT/ab_N8.json 2> $OUT/ab_N8.err || { tail $OUT/ab_N8.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r03/rec8/ab.json", "gpurun_out/r03/rec8/ab_N8.json"):
  d = json.load(open(f))
  for k, v in d["results"].items(): print(d["N"], k, v["fwd_us"], v["adj_us"], v["sweep_us"], f"{v['dof_updates_per_s']:.4g}", v["bit_identical_to_first_same_steps"])
PY
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --N 8 --no-cpu-baseline > $OUT/bench_N8.json 2> $OUT/bench_N8.err || { tail $OUT/bench_N8.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_N8'):
  d = json.load(open('$OUT/%s.json' % f)); print(f, d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['launch_steps'], d['launch_steps_fwd'])"
