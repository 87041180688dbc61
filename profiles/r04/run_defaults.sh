# New sweep defaults (12-wave tiles at Np <= 5, 8-wave dataflow at Np = 9, operator blocks
# re-read at Np >= 6): GPU test files of the sweep paths, config-5 benches, the headline and
# N = 8 profiles
set -o pipefail
out=gpurun_out/r04/defaults; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sweep.py tests/test_gpu_full_size.py tests/test_gpu_bench.py tests/test_gpu_eta_modes.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for n in 1 2 4 6 8; do
  timeout -k 10 200 python bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/N$n.json 2> $out/N$n.err || { echo "bench N$n failed"; tail -5 $out/N$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:60], '%.1f us' % d['roofline']['launch_us'])" $out/N$n.json
done
bash profiles/r04/collect.sh headline_w12 k_sweep_rp || exit 1
bash profiles/r04/collect.sh N8_dflow k_sweep_rp --N 8 || exit 1
echo all-done
