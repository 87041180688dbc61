# Forward record sweep in one 20-step launch, adjoint 10 + 10 (the new default): the whole GPU
# suite, smoke, the driver's bench command twice with an A/B against both-at-10, rocprof + PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/f20; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_driver.json'));print('driver', d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['roofline_fwd']['kernel'], d['launch_steps_fwd'])"
bash profiles/r02/ab_env.sh f20 "" "DG_REC_FWD_STEPS_PER_LAUNCH=10" || exit 1
bash profiles/r02/collect.sh || exit 1
