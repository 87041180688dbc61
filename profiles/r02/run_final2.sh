# Closing check of the pair-tile default: the whole GPU suite, smoke(), the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/f2; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/f2/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/f2/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/f2/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f2/smoke.log 2>&1 || { tail -20 gpurun_out/f2/smoke.log; exit 1; }
grep smoke gpurun_out/f2/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/f2/bench_driver.json 2> gpurun_out/f2/bench_driver.err || { tail -20 gpurun_out/f2/bench_driver.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/f2/bench_driver.json'));print('driver', d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline_fp64']['adj_frac'], d['cpu_baseline']['value'])"
timeout -k 10 120 ./profiles/probes/fp64_mix > gpurun_out/f2/fp64_mix.jsonl && cat gpurun_out/f2/fp64_mix.jsonl
timeout -k 10 60 ./profiles/probes/fp64_peak >> gpurun_out/f2/fp64_mix.jsonl && tail -1 gpurun_out/f2/fp64_mix.jsonl
