# Snapshot tiles loaded straight into LDS in the Horner estimate (DG_P_HORNER=3): parity of
# the DWR tests under it, then an A/B against the register prefetch (DG_P_HORNER=1)
set -o pipefail
out=gpurun_out/r05/p5; mkdir -p $out
DG_P_HORNER=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_HORNER=1" "DG_P_HORNER=3" || exit 1
echo all-done
