# A/B of plan settings on one box: the driver's bench command under each environment setting,
# alternating.   bash profiles/r05/ab_env.sh OUTDIR "EXTRA BENCH ARGS" "VAR=a" "VAR=b" ...
set -o pipefail
out=$1; shift
args=$1; shift
mkdir -p $out
for rep in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e" | tr ' =/' '___')
    env $e timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-margin $args > $out/${tag}_$rep.json 2> $out/${tag}_$rep.err || { echo "bench $tag failed"; tail -20 $out/${tag}_$rep.err; exit 1; }
  done
done
python - "$out" "$@" <<'PY'
import json, sys
out = sys.argv[1]
for e in sys.argv[2:]:
  tag = e.replace(" ", "_").replace("=", "_").replace("/", "_")
  vals = []
  for rep in (1, 2):
    d = json.load(open(f"{out}/{tag}_{rep}.json"))
    vals.append((d["value"], d["roofline"]["launch_us"]))
  print(e, " ".join("%.4g (%.1f us)" % v for v in vals))
PY
