# Round 3: first GPU pass of the dataflow sweep (dg_lserk4_sweep_rec).  Its own tests first
# (bit-identity to the launch chains), then the suites that run it through EnsembleSweep,
# then bench A/B (DG_REC_SWEEP=1 default vs 0 = launch chains) and a rocprof kernel-stats pass.
set -o pipefail
OUT=gpurun_out/r03/sweep1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_parity.py::test_ensemble_sweep_graph_matches_eager -x -v --timeout 120 --timeout-method thread > $OUT/tests_sweep.log 2>&1
rc=$?; echo "sweep tests rc=$rc"; grep -E "passed|failed|PASS|FAIL" $OUT/tests_sweep.log | tail -25; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_ties.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_more.log 2>&1
rc=$?; echo "more tests rc=$rc"; tail -5 $OUT/tests_more.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_df_$i.json 2> $OUT/bench_df_$i.err || { tail $OUT/bench_df_$i.err; exit 1; }
  DG_REC_SWEEP=0 timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_lc_$i.json 2> $OUT/bench_lc_$i.err || { tail $OUT/bench_lc_$i.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03/sweep1/bench_*.json")):
  d = json.load(open(f))
  print(f.split("/")[-1], f"{d['value']:.4g}", d["ms_per_step"], d["roofline"]["launch_us"], (d.get("roofline_fwd") or {}).get("launch_us"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
STATS=$(find $OUT/prof -name '*kernel_stats.csv' -print -quit); cp "$STATS" $OUT/kernel_stats.csv; head -8 $OUT/kernel_stats.csv | cut -c1-220
