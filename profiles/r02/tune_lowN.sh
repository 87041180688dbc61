# Low-N launch shapes: bench lines per N and plan shape (env overrides
# of dg_plan_create: DG_TILE_WIDTH, DG_STEPS_PER_LAUNCH, DG_LANE_ELEMENTS).
#   bash profiles/r02/tune_lowN.sh "1 2" [variant.so]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tune; export TMPDIR=/tmp
NS=${1:-"1 2"}
[ -n "$2" ] && export DG_LIB_PATH="$GRAFT_REPO_ROOT/$2"
for N in $NS; do
  for CFG in "default" "DG_STEPS_PER_LAUNCH=8" "DG_TILE_WIDTH=1" "DG_LANE_ELEMENTS=4" "DG_LANE_ELEMENTS=8" "DG_LANE_ELEMENTS=4 DG_STEPS_PER_LAUNCH=8" "DG_LANE_ELEMENTS=8 DG_STEPS_PER_LAUNCH=8"; do
    TAG="N${N}_$(echo $CFG | tr ' =' '_-')"
    if [ "$CFG" == "default" ]; then E=""; else E="$CFG"; fi
    env $E timeout -k 10 200 python bench.py --N $N --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/tune/$TAG.json 2> gpurun_out/tune/$TAG.err || { echo "$TAG failed"; tail -3 gpurun_out/tune/$TAG.err; continue; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tune/N*.json")):
    try:
        d = json.load(open(f))
    except Exception:
        continue
    r, g = d["roofline"], d["roofline_fwd"]
    print(f.split("/")[-1][:-5], f"value {d['value']:.4g} ms {d['ms_per_step']:.4f} spl {d['steps_per_launch']}",
          f"fwd {g['launch_us']:.1f}us frac {g['frac']:.3f}  adj {r['launch_us']:.1f}us frac {r['frac']:.3f}")
PY
