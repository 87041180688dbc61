# After the round-5 first commit: the dataflow sweep suite (incl. overlapped waves, the
# refine-loop scratch test, the watchdog), ABI + eta modes, the full-size dataflow parity,
# then the driver bench.
set -o pipefail
out=gpurun_out/r05/gpu1; mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sweep.py tests/test_gpu_eta_modes.py tests/test_gpu_full_size.py > $out/pytest.log 2>&1; rc=$?
grep -E "FAIL|passed|failed|Error" $out/pytest.log | tail -15
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['metric'], '%.4g' % d['value'], d['roofline']['traffic'], d['roofline']['traffic_source'], d['dataflow']['kernel'])"
echo all-done
