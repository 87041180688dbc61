# Overlapped waves with ds_bpermute lane shifts: parity, then A/B at N = 1, 2, 4
set -o pipefail
out=gpurun_out/r05/ovl3; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sweep.py -k "overlapped" > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/n1 "--N 1" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1" "DG_SWEEP_EXCHANGE=1 DG_SWEEP_WAVES=16" || exit 1
bash profiles/r05/ab_env.sh $out/n2 "--N 2" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1" || exit 1
bash profiles/r05/ab_env.sh $out/n4 "" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1" || exit 1
echo all-done
