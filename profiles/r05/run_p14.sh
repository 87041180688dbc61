# p-estimate defaults (dataflow launch on 512-element tiles, direct-to-LDS chain): DWR/pflow/
# sweep suites, the p bench and its profile (kernel stats, PMC traffic, SQ), the headline bench
set -o pipefail
out=gpurun_out/r05/p14; mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pflow.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --indicator p > $out/bench_p.json 2> $out/bench_p.err || { tail $out/bench_p.err; exit 1; }
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
bash profiles/r05/collect.sh p k_adjp_flow --indicator p || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/r05/p14/bench_p.json", "gpurun_out/r05/p14/bench.json"):
  d = json.load(open(f))
  r = d["roofline"]
  print(f.split("/")[-1], "%.4g" % d["value"], "%.3f ms" % d["ms_per_step"], "%.1f us" % r["launch_us"], r.get("kernel", "")[:60], d.get("cpu_baseline", {}).get("value"))
t = json.load(open("gpurun_out/r05/p/pmc_traffic.json")); print({k: t[k] for k in ("adj_kernel", "adj_bytes_per_launch", "p_flow", "tile_width")})
s = json.load(open("gpurun_out/r05/p/sq_summary.json")); print(s["kernel"], s["wait_any_frac_of_wave_cycles"], s["fp64_flops_issued_per_launch"])
PY
echo all-done
