# Is the one-launch estimate's speed tied to DG_P_HORNER=3?  A/B on one box
set -o pipefail
out=gpurun_out/r05/p13; mkdir -p $out
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_FLOW=1" "DG_P_HORNER=3 DG_P_FLOW=1" "DG_P_HORNER=3" "DG_P_HORNER=1" "DG_P_FLOW=1 DG_P_TILE_WIDTH=2" || exit 1
echo all-done
