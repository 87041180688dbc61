set -o pipefail
OUT=gpurun_out/r03/full3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
for n in 1 2 6 8; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --N $n --no-cpu-baseline > $OUT/bench_N$n.json 2> $OUT/bench_N$n.err || { tail $OUT/bench_N$n.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 --K 65536 --ics 1024 > $OUT/bench_config4.json 2> $OUT/bench_config4.err || { tail $OUT/bench_config4.err; exit 1; }
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03/full3/bench_*.json")):
  d = json.load(open(f))
  print(f.split("/")[-1], f"{d['value']:.4g}", round(d["ms_per_step"], 4), d["roofline"]["kernel"][:40], (d.get("dataflow") or {}).get("refine_in_launch"), (d.get("cpu_baseline") or {}).get("value"))
PY
