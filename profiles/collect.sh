# Round profile: bench line, rocprofv3 kernel stats, and HBM traffic (FETCH_SIZE and
# WRITE_SIZE in separate passes, no tracing besides --pmc), then the JSON summary.
#   bash profiles/collect.sh <tag>      (run on the GPU box from the repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed"; tail -20 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
# the bench's own step counts (the default run minus the CPU baseline, which follows the
# timed region), so the kernel averages compare with the bench line's launch_us
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof_$TAG.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$TAG.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$TAG.log" 2>&1 || { echo "pmc write failed"; exit 1; }
echo collected
