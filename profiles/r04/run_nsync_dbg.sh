set -o pipefail
out=gpurun_out/r04/nsync; mkdir -p $out
DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_nsync.so timeout -k 10 400 python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_rec.py tests/test_gpu_sweep.py -k "record_pair_equals or dataflow_equals" > $out/pytest_dbg.log 2>&1; echo "exit $?"
grep -E "PASS|FAIL|passed|failed" $out/pytest_dbg.log | tail -40
