# N = 8 on the dataflow launch with 8-wave (1024-element) tiles in both directions (the
# odd-first adjoint volume order brought the Np = 9 sweep kernel to 127 VGPRs: 2 workgroups
# per CU), against its launch chains; and repeated N = 1 / N = 4 pairs of 8 vs 12 waves.
set -o pipefail
mkdir -p gpurun_out/r04/waves2
run() {  # tag, env..., -- bench args
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin $BARGS > gpurun_out/r04/waves2/$tag.json 2> gpurun_out/r04/waves2/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/r04/waves2/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:70], '%.1f us' % d['roofline']['launch_us'])" gpurun_out/r04/waves2/$tag.json
}
BARGS="--N 8"
run N8_chain DG_REC_SWEEP=0 || exit 1
run N8_df8 DG_SWEEP_WAVES=8 || exit 1
run N8_chain_w2 DG_REC_SWEEP=0 DG_REC_TILE_WIDTH=2 || exit 1
run N8_df8_b DG_SWEEP_WAVES=8 || exit 1
for rep in 1 2; do
  BARGS="--N 1"; run N1_w0_$rep DG_SWEEP_WAVES=0 || exit 1; run N1_w12_$rep DG_SWEEP_WAVES=12 || exit 1
  BARGS="--N 4"; run N4_w0_$rep DG_SWEEP_WAVES=0 || exit 1; run N4_w12_$rep DG_SWEEP_WAVES=12 || exit 1
done
echo all-done
