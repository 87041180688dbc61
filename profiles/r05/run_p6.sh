# Tile fill of the Horner estimate: 4855 256-element tiles fill 5 or 6 workgroups per CU in 4
# rounds (the last 16-80 % full); 512-element tiles at 6 waves per SIMD (GL: 80 VGPRs) fill 3.
set -o pipefail
out=gpurun_out/r05/p6; mkdir -p $out
DG_P_HORNER=3 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py --deselect tests/test_gpu_dwr.py::test_full_size_p_estimate > $out/pytest.log 2>&1; rc=$?
# -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_HORNER=1" "DG_P_HORNER=3" "DG_P_HORNER=3 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=4" "DG_P_HORNER=3 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=8" "DG_P_HORNER=1 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=4" || exit 1
echo all-done
