# A/B of dataflow-sweep variants against the launch chains on one box: bench.py (driver
# command shape) per variant, alternating, two rounds.  Variants: tag=ENV... (DG_LIB_PATH
# picks an experiment library under lib/exp/).   bash profiles/r03/ab_sweep.sh <outdir> tag=VAR=val,VAR=val ...
set -o pipefail
OUT=$1; shift; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do
  for v in "$@"; do
    tag=${v%%=*}; envs=${v#*=}
    ( IFS=','; for kv in $envs; do [ -n "$kv" ] && [ "$kv" != "-" ] && export "$kv"; done
      timeout -k 10 200 python -u bench.py --gpus 1 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/${tag}_$i.json 2> $OUT/${tag}_$i.err ) || { echo "$tag failed"; tail -5 $OUT/${tag}_$i.err; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
  d = json.load(open(f))
  print(f.split("/")[-1], f"{d['value']:.4g}", round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["launch_us"], 1), (d.get("roofline_fwd") or {}).get("launch_us"))
PY
