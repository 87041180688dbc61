# Round 6: the whole GPU suite + smoke on the current tree
set -o pipefail
out=gpurun_out/r06/full; mkdir -p $out
timeout -k 10 1100 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/ > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
echo all-done
