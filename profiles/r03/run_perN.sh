# Round 3: per-N A/B of the record sweep shapes with the 8-byte record (config 5).
set -o pipefail
OUT=gpurun_out/r03/perN; mkdir -p $OUT; export TMPDIR=/tmp
for N in 8 1 2 6 4; do
  timeout -k 10 300 python -u profiles/r03/ab_rec.py --rounds 9 --N $N --variants 20:10,10:10,20:20,16:16,10:10:1,8:8:1,5:5:1,4:4:1 > $OUT/ab_N$N.json 2> $OUT/ab_N$N.err || { tail $OUT/ab_N$N.err; exit 1; }
  echo "N=$N done"
done
python3 - <<'PY'
import json
for N in (1, 2, 4, 6, 8):
  d = json.load(open(f"gpurun_out/r03/perN/ab_N{N}.json"))
  best = max(d["results"].items(), key=lambda kv: kv[1]["dof_updates_per_s"])
  for k, v in d["results"].items(): print(N, k, v["fwd_us"], v["adj_us"], v["sweep_us"], f"{v['dof_updates_per_s']:.4g}", v["bit_identical_to_first_same_steps"])
  print("best", N, best[0])
PY
