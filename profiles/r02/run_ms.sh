# Steps per launch of the pair-tile record sweeps (20-step sweeps): 8 (8+8+4) vs 10 (10+10) at
# tile widths 1 and 2, 16 (16+4) and 20 (one launch) at width 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash profiles/r02/ab_env.sh ms "" "DG_REC_STEPS_PER_LAUNCH=10" "DG_REC_TILE_WIDTH=2" "DG_REC_TILE_WIDTH=2 DG_REC_STEPS_PER_LAUNCH=10" "DG_REC_TILE_WIDTH=2 DG_REC_STEPS_PER_LAUNCH=16" "DG_REC_TILE_WIDTH=2 DG_REC_STEPS_PER_LAUNCH=20"
