# pipelined Horner p-estimate (k_adj_pq, the new default): parity, then A/B against the plain
# Horner kernel (DG_P_HORNER=1), both tile widths, and the 8-step forward on 512-element tiles
set -o pipefail
out=gpurun_out/r05/p3; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
F8="DG_TILE_WIDTH=2 DG_STEPS_PER_LAUNCH=8"
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_HORNER=1 DG_P_TILE_WIDTH=1 $F8" "DG_P_HORNER=2 DG_P_TILE_WIDTH=1 $F8" "DG_P_HORNER=2 $F8" "DG_P_HORNER=2 DG_P_TILE_WIDTH=1" || exit 1
echo all-done
