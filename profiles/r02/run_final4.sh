# Closing run with the size-aware forward default: the whole GPU suite, smoke, the driver's
# bench command, config 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/f4; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_driver.json'));print('driver', d['value'], d['launch_steps_fwd'], d['launch_steps'], d['roofline']['traffic'])"
timeout -k 10 300 python bench.py --K 65536 --ics 1024 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_config4.json 2> $OUT/err4 || { tail -5 $OUT/err4; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_config4.json'));print('config4', d['value'], d['launch_steps_fwd'], d['launch_steps'])"
