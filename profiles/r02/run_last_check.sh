set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/lc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_driver.json'));print('driver', d['value'])"
