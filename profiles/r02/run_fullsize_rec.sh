set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fs; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_full_size.py -k record_default > gpurun_out/fs/pytest.log 2>&1 || { tail -30 gpurun_out/fs/pytest.log; exit 1; }
tail -2 gpurun_out/fs/pytest.log
