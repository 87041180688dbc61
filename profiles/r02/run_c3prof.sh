# Config-3 profiles of the final round-2 kernels: bench line, rocprof kernel stats, SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/c3prof"; mkdir -p "$OUT"
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
cp "$(find "$OUT/prof" -name '*kernel_stats.csv' -print -quit)" "$OUT/kernel_stats.csv"
bash profiles/r02/collect_sq.sh c3_adj adj --physics burgers_limited --nonuniform --K 4194304 --nsteps 4 > /dev/null || exit 1
bash profiles/r02/collect_sq.sh c3_fwd fwd --physics burgers_limited --nonuniform --K 4194304 --nsteps 4 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('c3', '%.4g' % d['value'], 'adj', '%.1f' % d['roofline']['launch_us'], '%.3f' % d['roofline']['frac'], 'fwd', '%.1f' % d['roofline_fwd']['launch_us'], '%.3f' % d['roofline_fwd']['frac'])"
head -8 "$OUT/kernel_stats.csv" | cut -c1-160
