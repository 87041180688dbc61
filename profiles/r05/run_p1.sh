# p-estimate in Horner form (k_adj_ph): parity vs the oracle, then bench --indicator p A/B:
# round-3 stage loop (DG_P_HORNER=0) vs Horner on 512- and 256-element tiles vs Horner capped
# at 6 waves per SIMD (variant library)
set -o pipefail
out=gpurun_out/r05/p1; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_HORNER=0" "DG_P_HORNER=1" "DG_P_TILE_WIDTH=1" "DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_ph6.so" "DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_ph6.so DG_P_TILE_WIDTH=1" "DG_P_STEPS_PER_LAUNCH=8" || exit 1
echo all-done
