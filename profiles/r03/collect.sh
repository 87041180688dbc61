# Round-3 profile of the driver's bench command: rocprofv3 kernel stats, then HBM traffic
# (FETCH_SIZE and WRITE_SIZE in separate --pmc passes, nothing else traced), then the JSON
# summary + the per-launch traffic file bench.py reads (profiles/r03/pmc_traffic.json).
#   bash profiles/r02/collect.sh [extra bench args...]      (GPU box, repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/r03/collect"; mkdir -p "$OUT"
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -- python3 "$B" --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
grep '^{' "$OUT/prof.log" > "$OUT/bench_under_rocprof.json" || true
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline "$@" > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; tail -5 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -- python3 "$B" --steps 2 --warmup 1 --no-converge --no-cpu-baseline "$@" > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; tail -5 "$OUT/pmc_write.log"; exit 1; }
STATS=$(find "$OUT/prof" -name '*kernel_stats.csv' -print -quit)
FETCH=$(find "$OUT/pmc_fetch" -name '*counter_collection.csv' -print -quit)
WRITE=$(find "$OUT/pmc_write" -name '*counter_collection.csv' -print -quit)
cp "$STATS" "$OUT/kernel_stats.csv"
REC=jumps
case " $* " in *" --record snapshots "*) REC=snapshots;; esac
# the bench line under rocprof names the sweep's steps per launch
SPL=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['steps_per_launch'])" "$OUT/bench_under_rocprof.json")
python3 profiles/summarize.py --stats "$STATS" --fetch "$FETCH" --write "$WRITE" --out "$OUT/summary.json" --traffic-json "$OUT/pmc_traffic.json" --record $REC --steps-per-launch $SPL > /dev/null && echo collected
