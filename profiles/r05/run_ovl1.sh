# Overlapped-wave tiles (DG_SWEEP_EXCHANGE=1): parity against the launch chains, then A/B at
# N = 4 (headline) and N = 1.
set -o pipefail
out=gpurun_out/r05/ovl1; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sweep.py -k "overlapped" > $out/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" $out/pytest.log | tail -20
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/n4 "" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1" || exit 1
bash profiles/r05/ab_env.sh $out/n1 "--N 1" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1" || exit 1
echo all-done
