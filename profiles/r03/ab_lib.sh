# A/B of the in-tree library against an experiment build (lib/exp), alternating processes,
# with profiles/r03/ab_rec.py.   bash profiles/r03/ab_lib.sh <tag> [ab_rec.py args]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/r03/ab; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u profiles/r03/ab_rec.py --rounds 9 "$@" > $OUT/${TAG}_base_$i.json 2> $OUT/${TAG}_base_$i.err || { tail $OUT/${TAG}_base_$i.err; exit 1; }
  timeout -k 10 200 python -u profiles/r03/ab_rec.py --rounds 9 "$@" --lib adjoint-ode-adaptivity_amd/lib/exp/libdgadv.so > $OUT/${TAG}_exp_$i.json 2> $OUT/${TAG}_exp_$i.err || { tail $OUT/${TAG}_exp_$i.err; exit 1; }
done
python3 - "$TAG" <<'PY'
import json, glob, sys
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/r03/ab/{tag}_*.json")):
  d = json.load(open(f))
  for k, v in d["results"].items():
    print(f.split("/")[-1], k, v["fwd_us"], v["adj_us"], v["sweep_us"], f"{v['dof_updates_per_s']:.4g}")
PY
