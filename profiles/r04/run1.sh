# Round 4, GPU pass 1: the argmax reproducer, the new parity/watchdog tests, the driver bench.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 60 ./profiles/probes/argmax_phi_copy > gpurun_out/r04/argmax_probe.txt 2>&1; echo "probe exit $?" >> gpurun_out/r04/argmax_probe.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sweep.py tests/test_gpu_eta_modes.py tests/test_gpu_bench.py \
  "tests/test_gpu_full_size.py::test_full_size_dataflow_sweep_refine" \
  "tests/test_gpu_full_size.py::test_full_size_bench_workload" \
  "tests/test_gpu_full_size.py::test_full_size_dataflow_config4_shape" \
  > gpurun_out/r04/pytest1.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r04/pytest1.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/bench1.json 2> gpurun_out/r04/bench1.err || { echo "bench failed"; tail -20 gpurun_out/r04/bench1.err; exit 1; }
echo all-done
