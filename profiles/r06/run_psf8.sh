# Round 6: the p one-launch sweep with 8-step forward blocks (the plan's 8 steps per launch;
# VERDICT r05 item 3) -- bit-identity vs the chains at 4 and 8 steps, the p full-size tests,
# then an interleaved bench A/B (DG_P_SWEEP_FWD=4 forces the old 4-step forward blocks)
set -o pipefail
out=gpurun_out/r06/psf8; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_psweep.py tests/test_gpu_dwr.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
for i in 1 2 3; do
  for f in 4 8; do
    DG_P_SWEEP_FWD=$f timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --indicator p > $out/p_f${f}_$i.json 2> $out/p_f${f}_$i.err || { tail $out/p_f${f}_$i.err; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/psf8/p_*.json")):
  d = json.loads(open(f).read().strip().splitlines()[-1])
  print(f, "%.4g" % d["value"], "launch %.1f" % d["roofline"]["launch_us"], d.get("refine_index"), d.get("refine_margin", {}).get("decided") if isinstance(d.get("refine_margin"), dict) else d.get("refine_margin"))
PY
echo all-done
