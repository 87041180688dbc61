# Four elements per lane at N = 1, 2 (DG_SWEEP_LANE_ELEMENTS=4): correctness, then the bench.
set -o pipefail
mkdir -p gpurun_out/r04/e4
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sweep.py -k "four_elements or wide_dataflow or equals_launch_chains" > gpurun_out/r04/e4/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04/e4/tests.log; exit 1; }
tail -1 gpurun_out/r04/e4/tests.log
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin $BARGS > gpurun_out/r04/e4/$tag.json 2> gpurun_out/r04/e4/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/r04/e4/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:70], '%.1f us' % d['roofline']['launch_us'])" gpurun_out/r04/e4/$tag.json
}
for rep in 1 2; do
  BARGS="--N 1"
  run N1_e2_$rep DG_SWEEP_LANE_ELEMENTS=2 || exit 1
  run N1_e4w8_$rep DG_SWEEP_LANE_ELEMENTS=4 DG_SWEEP_WAVES=8 || exit 1
  run N1_e4w4_$rep DG_SWEEP_LANE_ELEMENTS=4 DG_SWEEP_WAVES=4 || exit 1
  BARGS="--N 2"
  run N2_e2_$rep DG_SWEEP_LANE_ELEMENTS=2 || exit 1
  run N2_e4w8_$rep DG_SWEEP_LANE_ELEMENTS=4 DG_SWEEP_WAVES=8 || exit 1
  run N2_e4w4_$rep DG_SWEEP_LANE_ELEMENTS=4 DG_SWEEP_WAVES=4 || exit 1
done
echo all-done
