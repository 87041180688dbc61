# Round-2 pair tiles, 10 steps per launch (the new record default): driver bench x2, rocprof
# kernel stats + PMC traffic of the driver command, per-N shapes, SQ counters, config 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/p10; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rec.py tests/test_gpu_eta_modes.py tests/test_gpu_bench.py > gpurun_out/p10/pytest.log 2>&1 || { tail -30 gpurun_out/p10/pytest.log; exit 1; }
tail -1 gpurun_out/p10/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/p10/smoke.log 2>&1 || { tail -20 gpurun_out/p10/smoke.log; exit 1; }
cat gpurun_out/p10/smoke.log | tail -3
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/p10/bench_driver_$r.json 2> gpurun_out/p10/bench_driver_$r.err || { tail -20 gpurun_out/p10/bench_driver_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p10/bench_driver_$r.json'));print('driver', d['value'], d['roofline']['kernel'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['roofline']['frac'])"
done
bash profiles/r02/collect.sh || exit 1
for n in 1 2 6; do
  bash profiles/r02/ab_env.sh p10N$n "" "DG_REC_TILE_WIDTH=1" "DG_REC_TILE_WIDTH=1 DG_REC_STEPS_PER_LAUNCH=8" -- --N $n || exit 1
done
bash profiles/r02/collect_sq.sh p10fwd fwd_rec || true
bash profiles/r02/collect_sq.sh p10adj adj_rec || true
timeout -k 10 300 python bench.py --K 65536 --ics 1024 --steps 10 --warmup 3 > gpurun_out/p10/bench_config4.json 2> gpurun_out/p10/bench_config4.err || { tail -20 gpurun_out/p10/bench_config4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/p10/bench_config4.json'));print('config4', d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'])"
