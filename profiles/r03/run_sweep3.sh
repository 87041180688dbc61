# Dataflow sweep diagnosis: per-item timeline (dg_plan_sweep_trace) and timing-only variants
# (plain stores instead of write-through; no dependency waits -- both give wrong results,
# timing only), natural occupancy (w5) vs forced 6 waves/SIMD (product build here).
set -o pipefail
OUT=gpurun_out/r03/sweep3; mkdir -p $OUT; export TMPDIR=/tmp
X=adjoint-ode-adaptivity_amd/lib/exp
timeout -k 10 120 python -u profiles/r03/sweep_trace.py --out $OUT > $OUT/trace_w6.txt 2>&1 || { tail $OUT/trace_w6.txt; exit 1; }
DG_LIB_PATH=$X/libdgadv_w5.so timeout -k 10 120 python -u profiles/r03/sweep_trace.py --out $OUT/w5 > $OUT/trace_w5.txt 2>&1 || { tail $OUT/trace_w5.txt; exit 1; }
head -60 $OUT/trace_w5.txt
bash profiles/r03/ab_sweep.sh $OUT/ab lc=DG_REC_SWEEP=0 w6=- w5=DG_LIB_PATH=$X/libdgadv_w5.so plainst=DG_LIB_PATH=$X/libdgadv_plainst.so nowait=DG_LIB_PATH=$X/libdgadv_nowait.so
