# Config 5 (N sweep at K = 2^20): one bench line and one rocprofv3 kernel-stats summary per N
# with the plan's default per-N shape.   bash profiles/r02/perN.sh "1 2 4 6 8"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/perN"; mkdir -p "$OUT"
for N in ${1:-1 2 4 6 8}; do
  timeout -k 10 200 python bench.py --N $N --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/bench_N$N.json" 2> "$OUT/bench_N$N.err" || { echo "bench N=$N failed"; tail -3 "$OUT/bench_N$N.err"; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_N$N" -- python3 "$GRAFT_REPO_ROOT/bench.py" --N $N --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_N$N.log" 2>&1 || { echo "rocprof N=$N failed"; tail -3 "$OUT/prof_N$N.log"; exit 1; }
  cp "$(find "$OUT/prof_N$N" -name '*kernel_stats.csv' -print -quit)" "$OUT/kernel_stats_N$N.csv"
  python3 -c "
import json; d=json.load(open('$OUT/bench_N$N.json')); r,g=d['roofline'],d['roofline_fwd']
print('N=$N', f\"value {d['value']:.4g} spl {d['steps_per_launch']} fwd {g['launch_us']:.1f}us frac {g['frac']:.3f} adj {r['launch_us']:.1f}us frac {r['frac']:.3f}\")"
done
