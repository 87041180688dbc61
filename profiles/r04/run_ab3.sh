# Isolate the persistent kernel's slowdown: the one-workgroup-per-item kernel calling the item
# as a non-inlined function (call), vs the inlined one (occ), vs persistent (product).
set -o pipefail
mkdir -p gpurun_out/r04
CALL=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_call.so
DG_LIB_PATH=$CALL timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sweep.py -k "equals_launch_chains or refine_equals" > gpurun_out/r04/call_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04/call_tests.log; exit 1; }
tail -1 gpurun_out/r04/call_tests.log
for v in call occ; do
  DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_$v.so timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_$v > gpurun_out/r04/trace_$v.txt 2>&1 || exit 1
done
timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_pers2 > gpurun_out/r04/trace_pers2.txt 2>&1 || exit 1
grep sweep_us gpurun_out/r04/trace_call.txt gpurun_out/r04/trace_occ.txt gpurun_out/r04/trace_pers2.txt
echo all-done
