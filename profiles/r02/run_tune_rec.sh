# Config 5 with the round-2 record default (pair tiles, 10 steps per launch; Np = 9: one
# element per lane, 2 steps): one bench line and one rocprof kernel-stats summary per N.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/tune10; mkdir -p $OUT; export TMPDIR=/tmp
for n in 1 2 4 6 8; do
  timeout -k 10 300 python bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_N$n.json 2> $OUT/bench_N$n.err || { tail -5 $OUT/bench_N$n.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_N$n -- python3 bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_N$n.log 2>&1 || { tail -5 $OUT/prof_N$n.log; exit 1; }
  cp "$(find $OUT/prof_N$n -name '*kernel_stats.csv' -print -quit)" $OUT/kernel_stats_N$n.csv
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('N', sys.argv[2], '%.4g'%d['value'], 'adj %.1f fwd %.1f'%(d['roofline']['launch_us'],d['roofline_fwd']['launch_us']), 'hbm %.3f/%.3f'%(d['roofline']['frac'],d['roofline_fwd']['frac']), 'fp64 %.3f/%.3f'%(d['roofline_fp64']['adj_frac'],d['roofline_fp64']['fwd_frac']), d['roofline']['kernel'])" $OUT/bench_N$n.json $n
done
