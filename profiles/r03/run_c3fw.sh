#!/bin/bash
# Config-3 forward with one exchange per limited stage (nl_stage_fw): decision/nonlinear GPU
# tests, then an A/B of bench.py --config 3: product vs the two-exchange forward
# (variants/libdg_head.so) vs the one-exchange forward capped at 8 waves/SIMD (libdg_w8.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/c3fw; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decisions.py tests/test_gpu_nonlinear.py -x -q \
  --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
V=$GRAFT_REPO_ROOT/adjoint-ode-adaptivity_amd/lib/variants
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $OUT/new_$rep.json 2> $OUT/new_$rep.err || { tail $OUT/new_$rep.err; exit 1; }
  DG_LIB_PATH=$V/libdg_head.so timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $OUT/head_$rep.json 2> $OUT/head_$rep.err || { tail $OUT/head_$rep.err; exit 1; }
  DG_LIB_PATH=$V/libdg_w8.so timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $OUT/w8_$rep.json 2> $OUT/w8_$rep.err || { tail $OUT/w8_$rep.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/c3fw/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], f"{d['value']:.4g}", "adj_us", f"{d['roofline']['launch_us']:.1f}",
          "fwd_us", f"{d['roofline_fwd']['launch_us']:.1f}", "fwd_frac", f"{d['roofline_fwd']['frac']:.3f}",
          "ref", d.get("refine_index"))
PY
