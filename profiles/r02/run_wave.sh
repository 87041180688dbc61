# Wave-tile record forward (8 elements per lane, no barriers): bit-identity, then A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/wv; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rec.py -k "wave_tiles" > gpurun_out/wv/pytest.log 2>&1 || { tail -30 gpurun_out/wv/pytest.log; exit 1; }
tail -1 gpurun_out/wv/pytest.log
bash profiles/r02/ab_env.sh wave "" "DG_REC_LANE_ELEMENTS=8" "DG_REC_LANE_ELEMENTS=8 DG_REC_STEPS_PER_LAUNCH=5"
