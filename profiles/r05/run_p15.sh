# The p sweep as one dataflow launch (k_psweep): parity against the chains, regression of the
# DWR / pflow / parity suites, then a probe timing the three forms
set -o pipefail
out=gpurun_out/r05/p15; mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_psweep.py tests/test_gpu_pflow.py tests/test_gpu_dwr.py tests/test_gpu_parity.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
timeout -k 10 300 python profiles/r05/probes/psweep_time.py > $out/time.json 2> $out/time.err || { tail $out/time.err; exit 1; }
cat $out/time.json
echo all-done
