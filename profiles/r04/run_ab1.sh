set -o pipefail
mkdir -p gpurun_out/r04
NI=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_ni.so
DG_LIB_PATH=$NI timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sweep.py > gpurun_out/r04/ni_sweep_tests.log 2>&1 || { echo "ni tests failed"; tail -30 gpurun_out/r04/ni_sweep_tests.log; exit 1; }
tail -2 gpurun_out/r04/ni_sweep_tests.log
bash profiles/r04/ab_libs.sh gpurun_out/r04/ab1 adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so adjoint-ode-adaptivity_amd/lib/ab/libdgadv_occ.so $NI || exit 1
DG_LIB_PATH=$NI timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_ni > gpurun_out/r04/trace_ni.txt 2>&1 || exit 1
echo all-done
