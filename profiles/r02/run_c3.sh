# config-3 and low-N checks after the decision-record / metric-folding change
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decisions.py tests/test_gpu_nonlinear.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_eta_modes.py -v --timeout 240 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_c3.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3.json')); print('c3', d['value'], 'adj', d['roofline']['launch_us'], d['roofline']['frac'], 'fwd', d['roofline_fwd']['launch_us'], d['roofline_fwd']['frac'])"
bash profiles/r02/tune_lowN.sh "1 2"
