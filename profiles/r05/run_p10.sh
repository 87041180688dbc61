# One-launch p-estimate with the snapshot loads issued before the producer poll: parity, then
# A/B against the chain at 20 steps (4-step blocks) and at 16 steps (8-step blocks, 512 tiles)
set -o pipefail
out=gpurun_out/r05/p10; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pflow.py tests/test_gpu_dwr.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/ab20 "--indicator p" "DG_P_HORNER=3" "DG_P_HORNER=3 DG_P_FLOW=1" || exit 1
bash profiles/r05/ab_env.sh $out/ab16 "--indicator p --nsteps 16" "DG_P_HORNER=3 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=8" "DG_P_HORNER=3 DG_P_FLOW=1 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=8" "DG_P_HORNER=3 DG_P_FLOW=1" || exit 1
echo all-done
