# Operator blocks re-read from the kernarg segment at Np >= 6 (no SGPR spill to VGPR lanes):
# parity of the record sweeps and the dataflow launch, then config-5 benches at N = 6, 8
set -o pipefail
out=gpurun_out/r04/opreload; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sweep.py tests/test_gpu_full_size.py tests/test_gpu_parity.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
run() {
  tag=$1; n=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/$tag.json 2> $out/$tag.err || { echo "bench $tag failed"; tail -5 $out/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:60], '%.1f us' % d['roofline']['launch_us'])" $out/$tag.json
}
for rep in 1 2; do
  run N8_base_$rep 8 || exit 1
  run N8_w8_$rep 8 DG_SWEEP_WAVES=8 || exit 1
  run N6_base_$rep 6 || exit 1
  run N4_w12_$rep 4 DG_SWEEP_WAVES=12 || exit 1
done
echo all-done
