# 512-element dataflow tiles: their tests, then config 5's N = 8 (Np = 9) with the dataflow
# launch (both directions on 512-element tiles, 10-step blocks) against the launch chains
# (forward 1024-element tiles 20 steps, adjoint 512-element tiles 10 + 10), and N = 4 on 512.
set -o pipefail
OUT=gpurun_out/r03/np9; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit 1; }
for i in 1 2; do
  DG_REC_SWEEP=0 timeout -k 10 200 python -u bench.py --N 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/n8_lc_$i.json 2> $OUT/n8_lc_$i.err || { tail -5 $OUT/n8_lc_$i.err; exit 1; }
  DG_REC_FWD_TILE_WIDTH=1 DG_REC_FWD_STEPS_PER_LAUNCH=10 timeout -k 10 200 python -u bench.py --N 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/n8_df_$i.json 2> $OUT/n8_df_$i.err || { tail -5 $OUT/n8_df_$i.err; exit 1; }
  DG_REC_TILE_WIDTH=1 DG_REC_FWD_STEPS_PER_LAUNCH=10 timeout -k 10 200 python -u bench.py --N 4 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/n4_w1_$i.json 2> $OUT/n4_w1_$i.err || { tail -5 $OUT/n4_w1_$i.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03/np9/*.json")):
  d = json.load(open(f))
  print(f.split("/")[-1], f"{d['value']:.4g}", round(d["ms_per_step"] * 1e3, 1), d["roofline"]["kernel"][:50])
PY
