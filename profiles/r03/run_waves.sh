# Round 3: wide pair-tile workgroups (DG_TUNE_REC_*_WAVES) A/B, the fixed config-3 window test,
# and the record tests.  Usage (GPU box): bash profiles/r03/run_waves.sh
set -o pipefail
OUT=gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_nonlinear.py::test_full_size_config3_adjoint_and_indicator" tests/test_gpu_rec.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_waves.log 2>&1 || { tail -30 $OUT/tests_waves.log; exit 1; }
tail -1 $OUT/tests_waves.log
timeout -k 10 300 python -u profiles/r03/ab_rec.py --rounds 9 > $OUT/ab_waves_1.json 2> $OUT/ab_waves_1.err || { tail $OUT/ab_waves_1.err; exit 1; }
timeout -k 10 300 python -u profiles/r03/ab_rec.py --rounds 9 --variants 20:10:0:0,20:10:12:10,10:10:10:10,10:10:12:12,20:10:16:10,20:10:10:12 > $OUT/ab_waves_2.json 2> $OUT/ab_waves_2.err || { tail $OUT/ab_waves_2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r03/ab_waves_1.json", "gpurun_out/r03/ab_waves_2.json"):
  d = json.load(open(f))
  for k, v in d["results"].items(): print(k, v["fwd_us"], v["adj_us"], v["sweep_us"], f"{v['dof_updates_per_s']:.4g}", v["bit_identical_to_first_same_steps"])
PY
