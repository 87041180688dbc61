# A/B of library variants on one box: the driver's bench command per variant, alternating.
#   bash profiles/r04/ab_libs.sh OUTDIR lib1 lib2 ...   (paths relative to the repo root)
set -o pipefail
out=$1; shift
mkdir -p $out
for rep in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    DG_LIB_PATH=$lib timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/${tag}_$rep.json 2> $out/${tag}_$rep.err || { echo "bench $tag failed"; tail -20 $out/${tag}_$rep.err; exit 1; }
  done
done
python - "$out" "$@" <<'PY'
import json, os, sys
out = sys.argv[1]
for lib in sys.argv[2:]:
  tag = os.path.basename(lib)[:-3]
  vals = []
  for rep in (1, 2):
    d = json.load(open(f"{out}/{tag}_{rep}.json"))
    vals.append((d["value"], d["roofline"]["launch_us"]))
  print(tag, " ".join("%.4g (%.1f us)" % v for v in vals))
PY
