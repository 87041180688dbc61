# Jump-record sweep shapes per N: bench line per (tile width, steps per launch)
#   bash profiles/r02/tune_rec.sh "4" "1:4 2:8 2:4 1:2"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/tune_rec"; mkdir -p "$OUT"
for N in ${1:-4}; do
  for shape in ${2:-1:4 2:8 2:4 1:2}; do
    tw=${shape%%:*}; spl=${shape##*:}
    f="$OUT/bench_N${N}_tw${tw}_spl${spl}.json"
    DG_REC_TILE_WIDTH=$tw DG_REC_STEPS_PER_LAUNCH=$spl timeout -k 10 200 python bench.py --N $N --steps 50 --warmup 5 --no-cpu-baseline > "$f" 2> "$OUT/err" || { echo "bench N=$N $shape failed"; tail -3 "$OUT/err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$f')); r,g=d['roofline'],d['roofline_fwd']
print('N=$N tw=$tw spl=$spl', f\"value {d['value']:.4g} launches {d['launch_steps']} fwd {g['launch_us']:.1f}us {g['frac']:.3f} adj {r['launch_us']:.1f}us {r['frac']:.3f}\")"
  done
done
