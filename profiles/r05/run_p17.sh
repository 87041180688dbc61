# The p sweep as one dataflow launch by default: its tests, the p bench A/B (the whole sweep,
# the estimate's dataflow launch alone, the chains), then its profile
set -o pipefail
out=gpurun_out/r05/p17; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_psweep.py tests/test_gpu_pflow.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_SWEEP=1" "DG_P_SWEEP=0" "DG_P_SWEEP=0 DG_P_FLOW=0" || exit 1
echo all-done
