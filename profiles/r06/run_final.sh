# Round 6, final: the whole GPU suite + smoke on the committed tree, then the driver's bench
# command and the config-3 / p lines
set -o pipefail
out=gpurun_out/r06/${FINAL_TAG:-final}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest -q --timeout 500 --timeout-method thread -m gpu tests/ > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config 3 > $out/bench_c3.json 2> $out/bench_c3.err || { tail $out/bench_c3.err; exit 1; }
timeout -k 10 300 python bench.py --indicator p > $out/bench_p.json 2> $out/bench_p.err || { tail $out/bench_p.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench", "bench_c3", "bench_p"):
  d = json.loads(open(f"gpurun_out/r06/{__import__('os').environ.get('FINAL_TAG', 'final')}/{f}.json").read().strip().splitlines()[-1])
  r = d["roofline"]
  print(f, "%.4g" % d["value"], r.get("bound"), "frac %.3f" % r["frac"], "traffic", r.get("traffic"), "cpu", d.get("cpu_baseline", {}).get("value"))
PY
echo all-done
