# Round 6: config-3 kernels on overlapped waves -- bit-identity vs the workgroup tiles, the
# full-size bench-path oracle test, then interleaved config-3 bench A/B (DG_NL_EXCHANGE 0/1)
set -o pipefail
out=gpurun_out/r06/ow1; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_nl_exchange.py tests/test_gpu_nonlinear.py tests/test_gpu_decisions.py tests/test_gpu_psweep.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
for i in 1 2; do
  for e in 0 1; do
    DG_NL_EXCHANGE=$e timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu-baseline > $out/c3_e${e}_$i.json 2> $out/c3_e${e}_$i.err || { tail $out/c3_e${e}_$i.err; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/ow1/c3_*.json")):
  d = json.loads(open(f).read().strip().splitlines()[-1])
  print(f, "%.4g" % d["value"], "adj %.1f" % d["roofline"]["launch_us"], "fwd %.1f" % d["roofline_fwd"]["launch_us"], d["refine_index"])
PY
echo all-done
