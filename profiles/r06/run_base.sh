# Round-6 baseline on today's box: config-3 bench (2 runs) and the headline bench
set -o pipefail
out=gpurun_out/r06/base; mkdir -p $out
timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu-baseline > $out/c3_1.json 2> $out/c3_1.err || { tail $out/c3_1.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu-baseline > $out/c3_2.json 2> $out/c3_2.err || { tail $out/c3_2.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/head.json 2> $out/head.err || { tail $out/head.err; exit 1; }
python3 - <<'PY'
import json
for f in ("c3_1", "c3_2", "head"):
  d = json.loads(open(f"gpurun_out/r06/base/{f}.json").read().strip().splitlines()[-1])
  print(f, d["value"], d["roofline"].get("launch_us"), d.get("roofline_fwd", {}).get("launch_us"))
PY
echo all-done
