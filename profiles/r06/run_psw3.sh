# Round 6: the p one-launch sweep on 768-element tiles (DG_P_SWEEP_W=3, 12 waves, 2 workgroups
# per CU) -- bit-identity vs the chains (the whole psweep test file under the env), then an
# interleaved bench A/B (--indicator p)
set -o pipefail
out=gpurun_out/r06/psw3; mkdir -p $out
DG_P_SWEEP_W=3 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_psweep.py -k "not trace_buffer" > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
for i in 1 2 3; do
  for w in 0 3; do
    DG_P_SWEEP_W=$w timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin --indicator p > $out/p_w${w}_$i.json 2> $out/p_w${w}_$i.err || { tail $out/p_w${w}_$i.err; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/psw3/p_*.json")):
  d = json.loads(open(f).read().strip().splitlines()[-1])
  print(f, "%.4g" % d["value"], "launch %.1f" % d["roofline"]["launch_us"], d.get("refine_index"))
PY
echo all-done
