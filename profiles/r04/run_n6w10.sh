# N = 6 (Np = 7): 10-wave tiles at 5 waves per SIMD against the 8-wave default, alternating
set -o pipefail
out=gpurun_out/r04/n6w10; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sweep.py -k "wide" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do for w in 0 10; do
  DG_SWEEP_WAVES=$w timeout -k 10 200 python bench.py --N 6 --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/w${w}_$rep.json 2> $out/w${w}_$rep.err || { echo "bench failed"; tail -5 $out/w${w}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:60], '%.1f us' % d['roofline']['launch_us'])" $out/w${w}_$rep.json
done; done
echo all-done
