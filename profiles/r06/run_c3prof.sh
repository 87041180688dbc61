# Round 6: config-3 PMC passes for both exchanges (workgroup tiles = default, overlapped waves)
set -o pipefail
DG_NL_EXCHANGE=0 bash profiles/r06/collect_c3.sh gpurun_out/r06/config3 > gpurun_out/c3prof0.log 2>&1 || { tail -20 gpurun_out/c3prof0.log; exit 1; }
DG_NL_EXCHANGE=1 bash profiles/r06/collect_c3.sh gpurun_out/r06/config3_ow > gpurun_out/c3prof1.log 2>&1 || { tail -20 gpurun_out/c3prof1.log; exit 1; }
python3 - <<'PY'
import json
for d in ("config3", "config3_ow"):
  p = json.load(open(f"gpurun_out/r06/{d}/pmc.json"))
  for k, v in p["kernels"].items():
    if ", false" in k:
      print(d, k, {a: round(b, 3) if isinstance(b, float) else b for a, b in v.items()})
PY
echo all-done
