# config-3: parity tests, then A/B of the product library against variants (same box)
#   bash profiles/r02/run_c3ab.sh <tag> <variant.so>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decisions.py tests/test_gpu_nonlinear.py tests/test_gpu_checkpoint.py -v --timeout 240 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_c3.log | head -20; exit $rc; }
TAG=$1; shift
bash profiles/r02/ab_libs.sh "$TAG" "$@" -- --config 3
