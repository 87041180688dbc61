# p-estimate shapes: Horner kernel on 256-element tiles, 8 steps per launch, the 6-waves-per-SIMD
# variant, and the forward snapshot kernel at 8 steps per launch on 512-element tiles
set -o pipefail
out=gpurun_out/r05/p2; mkdir -p $out
L6=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_ph6.so
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_TILE_WIDTH=1" "DG_P_STEPS_PER_LAUNCH=8" "DG_LIB_PATH=$L6" "DG_LIB_PATH=$L6 DG_P_TILE_WIDTH=1" "DG_P_TILE_WIDTH=1 DG_TILE_WIDTH=2 DG_STEPS_PER_LAUNCH=8" || exit 1
echo all-done
