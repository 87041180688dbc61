set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/final_pytest.log; exit 1; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash profiles/collect.sh r01h || exit 1
timeout -k 10 400 python bench.py --config 3 > gpurun_out/final_c3.json 2> gpurun_out/final_c3.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof_c3 -- python3 bench.py --config 3 --no-cpu-baseline > gpurun_out/final_prof_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --K 65536 --ics 1024 > gpurun_out/final_c4.json 2> gpurun_out/final_c4.err || exit 1
echo all-done
