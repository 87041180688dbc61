set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash profiles/r02/ab_env.sh rpp "DG_REC_LANE_ELEMENTS=2 DG_REC_TILE_WIDTH=1 DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_base.so" "DG_REC_LANE_ELEMENTS=2 DG_REC_TILE_WIDTH=1 DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_roll.so" "DG_REC_LANE_ELEMENTS=2 DG_REC_TILE_WIDTH=1 DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_prio1.so" "DG_REC_LANE_ELEMENTS=2 DG_REC_TILE_WIDTH=1 DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_prio3.so" "DG_REC_LANE_ELEMENTS=2 DG_REC_TILE_WIDTH=1 DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_rollprio1.so"
