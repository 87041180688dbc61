# Pair tiles as the record default: full GPU suite, the driver's bench command, per-N A/B
# against the one-element-per-lane record kernels (the previous default shape).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pd; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pd/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pd/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pd/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/pd/bench_driver.json 2> gpurun_out/pd/bench_driver.err || { tail -20 gpurun_out/pd/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/pd/bench_driver.json'));print('driver', d['value'], d['roofline']['kernel'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['roofline_fp64'])"
for n in 1 2 6; do
  bash profiles/r02/ab_env.sh pdN$n "" "DG_REC_LANE_ELEMENTS=1 DG_REC_TILE_WIDTH=2" -- --N $n || exit 1
done
bash profiles/r02/run_ms.sh || exit 1
