# Dataflow sweep + fused refine decision + side-stream result copy: tests, then the block
# shapes and occupancy A/B, then rocprof of the driver command.
set -o pipefail
OUT=gpurun_out/r03/sweep5; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error" $OUT/tests.log | head -20; exit 1; }
X=adjoint-ode-adaptivity_amd/lib/exp
bash profiles/r03/ab_sweep.sh $OUT/ab df=- lc=DG_REC_SWEEP=0 f10=DG_REC_FWD_STEPS_PER_LAUNCH=10 a5=DG_REC_STEPS_PER_LAUNCH=5,DG_REC_FWD_STEPS_PER_LAUNCH=20 f10a5=DG_REC_STEPS_PER_LAUNCH=5,DG_REC_FWD_STEPS_PER_LAUNCH=10 w6=DG_LIB_PATH=$X/libdgadv_w6.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
STATS=$(find $OUT/prof -name '*kernel_stats.csv' -print -quit); cp "$STATS" $OUT/kernel_stats.csv; head -6 $OUT/kernel_stats.csv | cut -c1-200
grep '^{' $OUT/prof.log > $OUT/bench_under_rocprof.json || true
