# Config 3 (bench.py --config 3) on the round-6 tree: bench line, rocprof kernel stats, HBM
# traffic (FETCH_SIZE, WRITE_SIZE passes) and the SQ fp64 / wait counters per kernel ->
# $OUT/pmc.json (profiles/r06/config3/pmc.json is what the bench's config-3 line reads).
# usage: bash profiles/r06/collect_c3.sh OUTDIR   (env DG_NL_EXCHANGE passes through)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/${1:-gpurun_out/r06/config3}"; mkdir -p "$OUT"
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 300 python3 -u "$B" --config 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -- python3 "$B" --config 3 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -- python3 "$B" --config 3 --steps 2 --warmup 1 --no-converge --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; tail -5 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -- python3 "$B" --config 3 --steps 2 --warmup 1 --no-converge --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; tail -5 "$OUT/pmc_write.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES --output-format csv -d "$OUT/pmc_sq" -- python3 "$B" --config 3 --steps 2 --warmup 1 --no-converge --no-cpu-baseline > "$OUT/pmc_sq.log" 2>&1 || { echo "pmc sq failed"; tail -5 "$OUT/pmc_sq.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$OUT/pmc_wait" -- python3 "$B" --config 3 --steps 2 --warmup 1 --no-converge --no-cpu-baseline > "$OUT/pmc_wait.log" 2>&1 || { echo "pmc wait failed"; tail -5 "$OUT/pmc_wait.log"; }
STATS=$(find "$OUT/prof" -name '*kernel_stats.csv' -print -quit); cp "$STATS" "$OUT/kernel_stats.csv"
FETCH=$(find "$OUT/pmc_fetch" -name '*counter_collection.csv' -print -quit)
WRITE=$(find "$OUT/pmc_write" -name '*counter_collection.csv' -print -quit)
SQ=$(find "$OUT/pmc_sq" -name '*counter_collection.csv' -print -quit)
WAIT=$(find "$OUT/pmc_wait" -name '*counter_collection.csv' -print -quit)
python3 profiles/r06/summarize_c3.py --stats "$OUT/kernel_stats.csv" --fetch "$FETCH" --write "$WRITE" --sq "$SQ" --wait "$WAIT" --out "$OUT/pmc.json"
