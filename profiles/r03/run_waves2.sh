# Dataflow launch workgroup sizes (DG_SWEEP_WAVES: 8 default = 16 of the 20 wave slots the
# 88-VGPR bodies leave per CU; 5, 10 fill all 20; 6 fills 18), 20- and 10-step forward blocks.
set -o pipefail
OUT=gpurun_out/r03/waves2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit 1; }
bash profiles/r03/ab_sweep.sh $OUT/ab w8=- w5=DG_SWEEP_WAVES=5 w10=DG_SWEEP_WAVES=10 w10f10=DG_SWEEP_WAVES=10,DG_REC_FWD_STEPS_PER_LAUNCH=10 w6f10=DG_SWEEP_WAVES=6,DG_REC_FWD_STEPS_PER_LAUNCH=10 w5f10=DG_SWEEP_WAVES=5,DG_REC_FWD_STEPS_PER_LAUNCH=10
