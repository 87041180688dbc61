# Record-sweep shapes per N next to the snapshot sweep's default (config 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/tune_rec"; mkdir -p "$OUT"
for N in 1 2 6; do
  bash profiles/r02/tune_rec.sh "$N" "2:8 2:4 1:4" || exit 1
done
bash profiles/r02/tune_rec.sh "8" "2:2 1:2" || exit 1
for N in 1 2 6 8; do
  timeout -k 10 200 python bench.py --N $N --steps 50 --warmup 5 --no-cpu-baseline --record snapshots > "$OUT/bench_N${N}_snap.json" 2> "$OUT/err" || { tail -3 "$OUT/err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_N${N}_snap.json'))
print('N=$N snapshots', f\"value {d['value']:.4g}\")"
done
