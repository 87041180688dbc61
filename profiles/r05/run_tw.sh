# The whole p sweep launch on 256- vs 512-element tiles (A/B, one box)
set -o pipefail
out=gpurun_out/r05/tw; mkdir -p $out
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_TILE_WIDTH=2" "DG_P_TILE_WIDTH=1" || exit 1
echo all-done
