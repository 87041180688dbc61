set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rec.py > gpurun_out/pytest_rec.log 2>&1 || { tail -30 gpurun_out/pytest_rec.log; exit 1; }
tail -3 gpurun_out/pytest_rec.log
bash profiles/r02/ab_env.sh pair "" "DG_REC_LANE_ELEMENTS=2" "DG_REC_LANE_ELEMENTS=2 DG_REC_TILE_WIDTH=1"
