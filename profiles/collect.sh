set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err || { echo "bench failed $?"; exit 1; }
cat gpurun_out/bench_r1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r1" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch_r1" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_r1.log 2>&1 || { echo "pmc fetch failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write_r1" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_r1.log 2>&1 || { echo "pmc write failed $?"; exit 1; }
find gpurun_out -name "*.csv" | head -50
