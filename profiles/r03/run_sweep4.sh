# Dataflow sweep with the monotonic take counter (no generation load, no exit counter):
# its tests, a trace, and the A/B against the launch chains (+ the plain-store timing variant).
set -o pipefail
OUT=gpurun_out/r03/sweep4; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_sweep.log 2>&1
rc=$?; tail -3 $OUT/tests_sweep.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/r03/sweep_trace.py --out $OUT > $OUT/trace.txt 2>&1 || { tail $OUT/trace.txt; exit 1; }
tail -2 $OUT/trace.txt
X=adjoint-ode-adaptivity_amd/lib/exp
bash profiles/r03/ab_sweep.sh $OUT/ab lc=DG_REC_SWEEP=0 df=- plainst=DG_LIB_PATH=$X/libdgadv_plainst.so
