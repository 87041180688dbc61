# config-5 shape A/B on the dataflow sweep: N = 1, 2 with 8/12/16-wave tiles, N = 6, and N = 8
# on the launch-per-block default vs dataflow launches (8 waves f20/a10, 4 waves f10/a10)
set -o pipefail
out=gpurun_out/r04/perN; mkdir -p $out
run() {
  tag=$1; n=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/$tag.json 2> $out/$tag.err || { echo "bench $tag failed"; tail -5 $out/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:60], '%.1f us' % d['roofline']['launch_us'], '%.1f ms/step' % d['ms_per_step'])" $out/$tag.json
}
for rep in 1 2; do
  run N1_w8_$rep 1 || exit 1
  run N1_w12_$rep 1 DG_SWEEP_WAVES=12 || exit 1
  run N1_w16_$rep 1 DG_SWEEP_WAVES=16 || exit 1
  run N2_w12_$rep 2 DG_SWEEP_WAVES=12 || exit 1
  run N2_w16_$rep 2 DG_SWEEP_WAVES=16 || exit 1
  run N4_w16_$rep 4 DG_SWEEP_WAVES=16 || exit 1
  run N6_base_$rep 6 || exit 1
  run N6_w12_$rep 6 DG_SWEEP_WAVES=12 || exit 1
  run N8_base_$rep 8 || exit 1
  run N8_w8_$rep 8 DG_SWEEP_WAVES=8 || exit 1
  run N8_w4f10_$rep 8 DG_SWEEP_WAVES=4 DG_REC_FWD_STEPS_PER_LAUNCH=10 || exit 1
done
echo all-done
