# A/B of library variants on the same box: the bench (driver command, no CPU baseline) with
# the product library and with each variant given as DG_LIB_PATH.
#   bash profiles/r02/ab_libs.sh <tag> <variant.so>... [-- extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab; export TMPDIR=/tmp
TAG=$1; shift
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab/${TAG}_base_$rep.json 2>/dev/null || exit 1
  i=0
  for L in "${LIBS[@]}"; do
    i=$((i+1))
    DG_LIB_PATH="$GRAFT_REPO_ROOT/$L" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab/${TAG}_v${i}_$rep.json 2>/dev/null || exit 1
  done
done
python3 - "$TAG" <<'PY'
import json, glob, sys
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/ab/{tag}_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], f"{d['value']:.4g}", "adj", f"{d['roofline']['launch_us']:.2f}",
          "fwd", f"{d['roofline_fwd']['launch_us']:.2f}", "step_ms", f"{d['ms_per_step']:.4f}")
PY
