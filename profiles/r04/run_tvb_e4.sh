set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sweep.py > gpurun_out/r04/pytest_tvb_e4.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04/pytest_tvb_e4.log; exit 1; }
tail -3 gpurun_out/r04/pytest_tvb_e4.log
bash profiles/r04/run_e4b.sh
