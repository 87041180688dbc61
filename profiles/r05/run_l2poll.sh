# The producer poll's first read from L2 (dg_flow.h ld_l2): the dataflow suites, then A/B of
# the p bench and the headline bench against the library without it (ablib/libdgadv_r05a.so)
set -o pipefail
out=gpurun_out/r05/l2poll; mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_psweep.py tests/test_gpu_pflow.py tests/test_gpu_sweep.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; exit 1; }
bash profiles/r05/ab_env.sh $out/ab_p "--indicator p" "DG_LIB_PATH=$PWD/profiles/r05/ablib/libdgadv_r05a.so" "DG_X=1" || exit 1
bash profiles/r05/ab_env.sh $out/ab_h "" "DG_LIB_PATH=$PWD/profiles/r05/ablib/libdgadv_r05a.so" "DG_X=1" || exit 1
echo all-done
