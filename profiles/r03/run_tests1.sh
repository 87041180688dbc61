mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dwr.py tests/test_gpu_rec.py tests/test_gpu_ties.py tests/test_gpu_config1.py "tests/test_gpu_nonlinear.py::test_full_size_config3_adjoint_and_indicator" -v -s --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke1.log 2>&1; echo "smoke rc=$?"; fi
tail -5 gpurun_out/smoke1.log
grep -E "PASS|FAIL|ERROR|passed|failed|effectivity gpu" gpurun_out/t1.log | tail -80
