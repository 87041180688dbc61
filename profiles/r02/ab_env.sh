# A/B of plan shapes set through environment overrides, on one box: the bench (driver command,
# no CPU baseline) once per variant, twice over.
#   bash profiles/r02/ab_env.sh <tag> "<VAR=val ...>" "<VAR=val ...>" ... [-- extra bench args]
# An empty string is the product default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab; export TMPDIR=/tmp
TAG=$1; shift
VARS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for rep in 1 2; do
  i=0
  for V in "${VARS[@]}"; do
    env $V timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" \
      > gpurun_out/ab/${TAG}_v${i}_$rep.json 2>gpurun_out/ab/${TAG}_v${i}_$rep.err || exit 1
    echo "$TAG v$i rep$rep ($V) done"
    i=$((i+1))
  done
done
python3 - "$TAG" "${VARS[@]}" <<'PY'
import json, glob, sys
tag, vars_ = sys.argv[1], sys.argv[2:]
for f in sorted(glob.glob(f"gpurun_out/ab/{tag}_*.json")):
    d = json.load(open(f))
    i = int(f.split("_v")[-1].split("_")[0])
    print(f.split("/")[-1], repr(vars_[i]), f"{d['value']:.4g}", "adj", f"{d['roofline']['launch_us']:.2f}",
          "fwd", f"{d['roofline_fwd']['launch_us']:.2f}", "step_ms", f"{d['ms_per_step']:.4f}")
PY
