# 12-wave workgroups (1536-element tiles) for the dataflow sweep vs 8-wave (occ = product) vs
# the round-3 library; correctness of the variant first.
set -o pipefail
mkdir -p gpurun_out/r04
W12=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_w12.so
DG_LIB_PATH=$W12 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sweep.py -k "equals_launch_chains or refine_equals or watchdog" > gpurun_out/r04/w12_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04/w12_tests.log; exit 1; }
tail -1 gpurun_out/r04/w12_tests.log
bash profiles/r04/ab_libs.sh gpurun_out/r04/ab4 adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so adjoint-ode-adaptivity_amd/lib/libdgadv.so $W12 || exit 1
DG_LIB_PATH=$W12 timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_w12 > gpurun_out/r04/trace_w12.txt 2>&1 || exit 1
echo all-done
