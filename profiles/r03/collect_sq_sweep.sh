# SQ counters of the dataflow launch (k_sweep_rp) under the driver bench (2 timed steps):
# wave cycles, waits, VALU activity and the issued fp64 VALU instructions, in two passes
# (<= 8 SQ counters each, nothing traced besides).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/r03/sq"; mkdir -p "$OUT"
B="$GRAFT_REPO_ROOT/bench.py"
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_sweep_rp" in k:
      agg["k_sweep_rp"][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {c: sum(v) / len(v) for c, v in agg["k_sweep_rp"].items()}
w = res.get("SQ_WAVES", 1.0)
per_wave = {c: res[c] / w for c in res if c.startswith("SQ_INSTS") or c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE") or c == "SQ_WAVE_CYCLES" or c == "SQ_BUSY_CYCLES"}
fl = 64.0 * (2 * res.get("SQ_INSTS_VALU_FMA_F64", 0) + res.get("SQ_INSTS_VALU_ADD_F64", 0) + res.get("SQ_INSTS_VALU_MUL_F64", 0))
summary = {"per_launch": res, "per_wave": per_wave, "fp64_flops_issued_per_launch": fl,
           "wait_any_frac_of_wave_cycles": res.get("SQ_WAIT_ANY", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1),
           "valu_active_frac_of_wave_cycles": res.get("SQ_ACTIVE_INST_VALU", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1)}
json.dump(summary, open(out + "/sq_summary.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
PY
