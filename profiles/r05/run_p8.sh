# The p-estimate as one dataflow launch (k_adjp_flow): its parity tests, the DWR and sweep
# suites (shared dataflow primitives moved to dg_flow.h), then an A/B of the p bench.
set -o pipefail
out=gpurun_out/r05/p8; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pflow.py tests/test_gpu_dwr.py tests/test_gpu_sweep.py > $out/pytest.log 2>&1; rc=$?
tail -5 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_HORNER=3" "DG_P_HORNER=3 DG_P_FLOW=1" "DG_P_HORNER=3 DG_P_FLOW=1 DG_P_TILE_WIDTH=2" "DG_P_HORNER=3 DG_P_FLOW=1 DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=8" || exit 1
echo all-done
