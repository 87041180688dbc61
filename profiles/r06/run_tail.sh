# Round 6: a 5-step tail adjoint block in the headline dataflow sweep (DG_SWEEP_ADJ_TAIL=5) --
# bit-identity vs equal blocks, then interleaved headline bench A/B (tail 0 / 5)
set -o pipefail
out=gpurun_out/r06/tail; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sweep.py -k "tail or equals_launch_chains or refine_equals" > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
for i in 1 2 3; do
  for t in 0 5; do
    DG_SWEEP_ADJ_TAIL=$t timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/head_t${t}_$i.json 2> $out/head_t${t}_$i.err || { tail $out/head_t${t}_$i.err; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/tail/head_*.json")):
  d = json.loads(open(f).read().strip().splitlines()[-1])
  print(f, "%.4g" % d["value"], "launch %.1f" % d["roofline"]["launch_us"], d["dataflow"]["blocks_adj"], d["dataflow"]["work_items"], d.get("refine_index"))
PY
echo all-done
