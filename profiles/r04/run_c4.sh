# config 4 shape on one GPU (1024 ICs x K = 65,536): 12-wave default vs 8-wave tiles, alternating
set -o pipefail
out=gpurun_out/r04/c4; mkdir -p $out
for rep in 1 2; do for w in 0 8; do
  DG_SWEEP_WAVES=$w timeout -k 10 300 python bench.py --K 65536 --ics 1024 --steps 5 --warmup 2 --no-cpu-baseline --no-margin > $out/w${w}_$rep.json 2> $out/w${w}_$rep.err || { echo "bench failed"; tail -5 $out/w${w}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:70], '%.1f us' % d['roofline']['launch_us'])" $out/w${w}_$rep.json
done; done
echo all-done
