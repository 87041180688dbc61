# Round 3: the p-estimate bench line + rocprof kernel stats, the default line, and the new
# GPU tests not yet run.  Usage (GPU box): bash profiles/r03/run_bench_p.sh
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "tests/test_gpu_nonlinear.py::test_full_size_config3_adjoint_and_indicator" tests/test_gpu_bench.py -v --timeout 300 --timeout-method thread > gpurun_out/r03/tests2.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03/bench_jump.json 2> gpurun_out/r03/bench_jump.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --indicator p > gpurun_out/r03/bench_p.json 2> gpurun_out/r03/bench_p.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/prof_p -o run -- python3 bench.py --steps 20 --warmup 5 --indicator p --no-cpu-baseline > gpurun_out/r03/bench_p_rocprof.json 2> gpurun_out/r03/rocprof_p.err || exit 1
echo done
