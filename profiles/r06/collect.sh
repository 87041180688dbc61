# Round-6 profile (as profiles/r05/collect.sh) of one bench configuration: rocprofv3 kernel stats of the bench command,
# HBM traffic (FETCH_SIZE and WRITE_SIZE, separate --pmc passes, nothing else traced), and
# two SQ passes (<= 8 SQ counters each) for the dominant kernel; then the JSON summaries the
# bench line reads (profiles/summarize.py, profiles/r04/sq_reduce.py).
#   bash profiles/r06/collect.sh TAG KERNEL_SUBSTRING [extra bench args...]   (GPU box, repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; KSUB=$2; shift 2
OUT="$GRAFT_REPO_ROOT/gpurun_out/r06/$TAG"; mkdir -p "$OUT"
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -- python3 "$B" --steps 20 --warmup 5 --no-cpu-baseline --no-margin "$@" > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
grep '^{' "$OUT/prof.log" > "$OUT/bench_under_rocprof.json" || true
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline --no-margin "$@" > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; tail -5 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline --no-margin "$@" > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; tail -5 "$OUT/pmc_write.log"; exit 1; }
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/sq$i" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline --no-margin "$@" > "$OUT/sq$i.log" 2>&1 || { echo "sq pass $i failed"; tail -3 "$OUT/sq$i.log"; exit 1; }
done
STATS=$(find "$OUT/prof" -name '*kernel_stats.csv' -print -quit)
FETCH=$(find "$OUT/pmc_fetch" -name '*counter_collection.csv' -print -quit)
WRITE=$(find "$OUT/pmc_write" -name '*counter_collection.csv' -print -quit)
cp "$STATS" "$OUT/kernel_stats.csv"
python3 - "$OUT/bench_under_rocprof.json" > "$OUT/meta.txt" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config"]
print(c["N"], c["K"], c.get("trajectories_per_gpu", 1), d.get("steps_per_launch", 0), c.get("record", "jumps"), d.get("indicator", "jump"), d.get("tile_width", 1))
PY
read N K BATCH SPL REC IND TW < "$OUT/meta.txt"
python3 profiles/summarize.py --stats "$STATS" --fetch "$FETCH" --write "$WRITE" --out "$OUT/summary.json" --traffic-json "$OUT/pmc_traffic.json" --N $N --K $K --batch $BATCH --record $REC --steps-per-launch $SPL --indicator $IND --tile-width $TW > /dev/null || exit 1
python3 profiles/r04/sq_reduce.py "$OUT" "$KSUB" > /dev/null || exit 1
# the dataflow kernel's signature (instantiation + occupancy target) the bench matches on
python3 - "$OUT/bench_under_rocprof.json" "$OUT/pmc_traffic.json" <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
t = json.load(open(sys.argv[2]))
t["sweep_kernel"] = (b.get("dataflow") or {}).get("kernel")
json.dump(t, open(sys.argv[2], "w"), indent=1)
PY
echo "collected $TAG"
