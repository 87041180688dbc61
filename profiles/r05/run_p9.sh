# Why the one-launch p-estimate is slower: kernel stats + SQ passes of k_adjp_flow
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
export DG_P_HORNER=3 DG_P_FLOW=1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05/pflow1"; mkdir -p "$OUT"
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -- python3 "$B" --steps 20 --warmup 5 --no-cpu-baseline --no-margin --indicator p > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/sq$i" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline --no-margin --indicator p > "$OUT/sq$i.log" 2>&1 || { echo "sq pass $i failed"; tail -3 "$OUT/sq$i.log"; exit 1; }
done
STATS=$(find "$OUT/prof" -name '*kernel_stats.csv' -print -quit)
cp "$STATS" "$OUT/kernel_stats.csv"
python3 profiles/r04/sq_reduce.py "$OUT" k_adjp_flow > /dev/null || exit 1
python3 - <<'PY'
import csv, json
rows = list(csv.DictReader(open('gpurun_out/r05/pflow1/kernel_stats.csv')))
for r in rows[:8]:
  print('%-60s %6s %8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
d = json.load(open('gpurun_out/r05/pflow1/sq_summary.json'))
print({k: round(v, 1) for k, v in d['per_wave'].items()})
print(d['wait_any_frac_of_wave_cycles'], d['valu_active_frac_of_wave_cycles'], d['per_launch']['SQ_WAVE_CYCLES'] / d['per_launch']['GRBM_GUI_ACTIVE'])
PY
echo all-done
