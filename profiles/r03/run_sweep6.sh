# Dataflow sweep + fused refine written straight to pinned host memory: tests, the driver
# bench twice (and the launch chains once), then rocprof kernel stats + PMC traffic.
set -o pipefail
OUT=gpurun_out/r03/sweep6; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_bench.py tests/test_gpu_full_size.py tests/test_gpu_ties.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAIL" $OUT/tests.log | head -20; exit 1; }
bash profiles/r03/ab_sweep.sh $OUT/ab df=- lc=DG_REC_SWEEP=0 || exit 1
bash profiles/r03/collect.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r03/collect/summary.json'))
for k,v in list(d.items())[:4]: print(k, {kk: round(vv,1) if isinstance(vv,float) else vv for kk,vv in v.items()})"
cat gpurun_out/r03/collect/pmc_traffic.json
