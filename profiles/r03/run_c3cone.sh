#!/bin/bash
# Config-3 adjoint on narrow-cone tiles (troubled tiles listed for k_adj_nl_wide): the
# decision/nonlinear GPU tests, then an A/B of bench.py --config 3 against the previous
# kernel (lib/variants/libdg_c3old.so) on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/c3cone; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decisions.py tests/test_gpu_nonlinear.py -x -q \
  --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $OUT/new_$rep.json 2> $OUT/new_$rep.err || { tail $OUT/new_$rep.err; exit 1; }
  DG_LIB_PATH=$GRAFT_REPO_ROOT/adjoint-ode-adaptivity_amd/lib/variants/libdg_c3old.so \
    timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $OUT/old_$rep.json 2> $OUT/old_$rep.err || { tail $OUT/old_$rep.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/c3cone/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], f"{d['value']:.4g}", "adj_us", f"{d['roofline']['launch_us']:.1f}",
          "frac", f"{d['roofline']['frac']:.3f}", "fwd_us", f"{d['roofline_fwd']['launch_us']:.1f}",
          "K_final", d.get("K_final"), "ref", d.get("refine_index"))
PY
# kernel stats of the new library
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -- python3 bench.py --config 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
STATS=$(find $GRAFT_REPO_ROOT/$OUT/prof -name '*kernel_stats.csv' -print -quit); cp "$STATS" $OUT/kernel_stats.csv
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/c3cone/kernel_stats.csv")))[:6]:
    print(r["Name"][:70], r["Calls"], f'{float(r["AverageNs"])/1e3:.1f} us', f'{float(r["Percentage"]):.1f}%')
PY
