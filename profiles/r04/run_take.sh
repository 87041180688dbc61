# Take counter vs workgroup-id items: sweep tests under the id mode, per-item traces (8/12
# waves, both modes), interleaved bench A/B; then the N = 1 / N = 8 profiles
set -o pipefail
out=gpurun_out/r04/take; mkdir -p $out
DG_SWEEP_TAKE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sweep.py tests/test_gpu_full_size.py > $out/pytest_take1.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_take1.log; exit 1; }
tail -2 $out/pytest_take1.log
for m in 0 1; do for w in 8 12; do
  DG_SWEEP_TAKE=$m DG_SWEEP_WAVES=$w timeout -k 10 120 python profiles/r03/sweep_trace.py --out $out/t$m > $out/trace_t${m}_w$w.txt 2>&1 || { echo "trace failed"; tail -5 $out/trace_t${m}_w$w.txt; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1], 'untraced %.1f traced %.1f' % (d['sweep_us_untraced'], d['sweep_us_traced']), {k: (round(v['wait_mean'],2), round(v['compute_mean'],1), round(v['last_done'],1)) for k,v in d['phases'].items()}, 'inflight', d['timeline_5us']['in_flight'][:6])
" $out/t$m/trace_N4_f20_w$w.json
done; done
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/$tag.json 2> $out/$tag.err || { echo "bench $tag failed"; tail -5 $out/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], '%.1f us' % d['roofline']['launch_us'])" $out/$tag.json
}
for rep in 1 2; do
  run t0w8_$rep DG_SWEEP_TAKE=0 || exit 1
  run t1w8_$rep DG_SWEEP_TAKE=1 || exit 1
  run t0w12_$rep DG_SWEEP_TAKE=0 DG_SWEEP_WAVES=12 || exit 1
  run t1w12_$rep DG_SWEEP_TAKE=1 DG_SWEEP_WAVES=12 || exit 1
done
echo bench-done
bash profiles/r04/collect.sh N1 k_sweep_rp --N 1 || exit 1
DG_SWEEP_WAVES=8 bash profiles/r04/collect.sh N8 k_sweep_rp --N 8 || exit 1
echo all-done
