# Pair adjoint occupancy variants (A/B): 6 waves/SIMD (80 VGPRs, 3 spills), record prefetch
# issued mid-step, both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash profiles/r02/ab_env.sh adjocc "" "DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_w6.so" "DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_late.so" "DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/var_latew6.so"
