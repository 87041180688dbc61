set -o pipefail
out=gpurun_out/r04/np2; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sweep.py tests/test_gpu_full_size.py tests/test_gpu_rec.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for rep in 1 2; do
timeout -k 10 200 python bench.py --N 1 --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/N1_$rep.json 2> $out/N1_$rep.err || { echo "bench failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:60], '%.1f us' % d['roofline']['launch_us'])" $out/N1_$rep.json
done
bash profiles/r04/collect.sh N1_w8 k_sweep_rp --N 1 || exit 1
echo all-done
