#!/bin/bash
# Final GPU pass of round 3: the candidate-kernel shape probe, every -m gpu test, smoke(), the
# driver bench and the exchange-cost timing.
set -o pipefail
OUT=gpurun_out/r03/final; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python3 profiles/r03/dbg_cand.py > $OUT/dbg_cand.log 2>&1 || { tail $OUT/dbg_cand.log; exit 1; }
echo "probe: $(grep -c OK $OUT/dbg_cand.log) OK, $(grep -c BAD $OUT/dbg_cand.log) BAD"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['cpu_baseline']['value'])"
timeout -k 10 200 python3 profiles/r03/exchange_cost.py > $OUT/exchange_cost.json 2> $OUT/exchange_cost.err || { tail $OUT/exchange_cost.err; exit 1; }
cat $OUT/exchange_cost.json
