# Round-5 final pass: the whole GPU suite, smoke, the driver bench (headline) and the p bench,
# then the p sweep's profile (kernel stats, PMC traffic, SQ passes)
set -o pipefail
out=gpurun_out/r05/final; mkdir -p $out
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --indicator p > $out/bench_p.json 2> $out/bench_p.err || { tail $out/bench_p.err; exit 1; }
bash profiles/r05/collect.sh p k_psweep --indicator p || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/r05/final/bench.json", "gpurun_out/r05/final/bench_p.json"):
  d = json.load(open(f))
  r = d["roofline"]
  print(f.split("/")[-1], "%.4g" % d["value"], "%.3f ms" % d["ms_per_step"], "%.1f us" % r["launch_us"], r.get("traffic_source"), d.get("cpu_baseline", {}).get("value"))
t = json.load(open("gpurun_out/r05/p/pmc_traffic.json")); print({k: t.get(k) for k in ("adj_kernel", "adj_bytes_per_launch", "p_flow", "p_sweep", "tile_width")})
s = json.load(open("gpurun_out/r05/p/sq_summary.json")); print(s["kernel"], s["wait_any_frac_of_wave_cycles"], s["fp64_flops_issued_per_launch"])
PY
echo main-done
# A/B (round 5, since removed): two queue items per workgroup in the p sweep launch
# (k_psweep2, DG_P_SWEEP_PAIR=1)
DG_P_SWEEP_PAIR=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_psweep.py > $out/pytest_pair.log 2>&1; rc=$?
tail -2 $out/pytest_pair.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/ab_env.sh $out/ab_pair "--indicator p" "DG_P_SWEEP_PAIR=0" "DG_P_SWEEP_PAIR=1" || exit 1
echo pair-done
