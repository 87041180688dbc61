# N = 1, 2: 8-wave tiles with 8 waves per SIMD (SGPRs <= 80: 4 workgroups per CU) against the
# default 12-wave tiles and the 6-wave-per-SIMD 8-wave tiles, alternating on one box
set -o pipefail
out=gpurun_out/r04/wpe8; mkdir -p $out
run() {
  tag=$1; n=$2; lib=$3; shift 3
  env DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_$lib.so "$@" timeout -k 10 200 python bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/$tag.json 2> $out/$tag.err || { echo "bench $tag failed"; tail -5 $out/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], '%.1f us' % d['roofline']['launch_us'])" $out/$tag.json
}
for rep in 1 2; do for n in 1 2; do
  run N${n}_base_w12_$rep $n base || exit 1
  run N${n}_base_w8_$rep $n base DG_SWEEP_WAVES=8 || exit 1
  run N${n}_wpe8_w8_$rep $n wpe8 DG_SWEEP_WAVES=8 || exit 1
done; done
echo all-done
