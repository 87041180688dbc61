# The whole p sweep launch on 1024-element tiles (DG_P_SWEEP_W4=1, experiment): parity, A/B
set -o pipefail
out=gpurun_out/r05/w4; mkdir -p $out
DG_P_SWEEP_W4=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_psweep.py > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; exit 1; }
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_SWEEP_W4=0" "DG_P_SWEEP_W4=1" || exit 1
echo all-done
