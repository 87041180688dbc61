# Persistent dataflow sweep (product library): correctness first, then A/B against the
# round-3 library (base) and the capped one-workgroup-per-item kernel (occ), then a trace.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sweep.py \
  "tests/test_gpu_full_size.py::test_full_size_dataflow_sweep_refine" \
  "tests/test_gpu_full_size.py::test_full_size_dataflow_config4_shape" > gpurun_out/r04/pers_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04/pers_tests.log; exit 1; }
tail -2 gpurun_out/r04/pers_tests.log
bash profiles/r04/ab_libs.sh gpurun_out/r04/ab2 adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so adjoint-ode-adaptivity_amd/lib/ab/libdgadv_occ.so adjoint-ode-adaptivity_amd/lib/libdgadv.so || exit 1
timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_pers > gpurun_out/r04/trace_pers.txt 2>&1 || exit 1
echo all-done
