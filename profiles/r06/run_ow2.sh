# Round 6: remaining parity tests of the first pass, then interleaved config-3 bench A/B
# (DG_NL_EXCHANGE 0/1) and the headline
set -o pipefail
out=gpurun_out/r06/ow2; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_psweep.py -k "trace or fallback" > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
for i in 1 2; do
  for e in 0 1; do
    DG_NL_EXCHANGE=$e timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu-baseline > $out/c3_e${e}_$i.json 2> $out/c3_e${e}_$i.err || { tail $out/c3_e${e}_$i.err; exit 1; }
  done
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/head.json 2> $out/head.err || { tail $out/head.err; exit 1; }
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/ow2/*.json")):
  d = json.loads(open(f).read().strip().splitlines()[-1])
  r = d["roofline"]
  print(f, "%.4g" % d["value"], r.get("kernel", "")[:40], "launch %.1f" % r["launch_us"],
        "fwd %.1f" % d["roofline_fwd"]["launch_us"] if d.get("roofline_fwd") else "", d["refine_index"])
PY
echo all-done
