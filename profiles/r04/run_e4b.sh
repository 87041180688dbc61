set -o pipefail
mkdir -p gpurun_out/r04/e4b
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin $BARGS > gpurun_out/r04/e4b/$tag.json 2> gpurun_out/r04/e4b/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/r04/e4b/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:70], '%.1f us' % d['roofline']['launch_us'])" gpurun_out/r04/e4b/$tag.json
}
for rep in 1 2; do
  BARGS="--N 1"
  run N1_e2_$rep DG_SWEEP_LANE_ELEMENTS=2 || exit 1
  run N1_e4w8_$rep DG_SWEEP_LANE_ELEMENTS=4 DG_SWEEP_WAVES=8 || exit 1
  BARGS="--N 2"
  run N2_e2_$rep DG_SWEEP_LANE_ELEMENTS=2 || exit 1
  run N2_e4w8_$rep DG_SWEEP_LANE_ELEMENTS=4 DG_SWEEP_WAVES=8 || exit 1
done
echo all-done
mkdir -p gpurun_out/r04/n4shape
for rep in 1 2; do
  for cfg in "base" "w12 DG_SWEEP_WAVES=12" "f10 DG_REC_FWD_STEPS_PER_LAUNCH=10" "w12f10 DG_SWEEP_WAVES=12 DG_REC_FWD_STEPS_PER_LAUNCH=10"; do
    set -- $cfg; tag=$1; shift
    env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin > gpurun_out/r04/n4shape/${tag}_$rep.json 2> gpurun_out/r04/n4shape/${tag}_$rep.err || { echo "bench $tag failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], '%.1f us' % d['roofline']['launch_us'])" gpurun_out/r04/n4shape/${tag}_$rep.json
  done
done
echo all-done2
