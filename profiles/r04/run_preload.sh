# p-estimate (k_adj_p) with its constants re-read from the kernarg segment (NPL >= 5) against
# the previous library: parity under the variant, then bench --indicator p alternating
set -o pipefail
out=gpurun_out/r04/preload; mkdir -p $out
DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_preload.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do for lib in base preload; do
  DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_$lib.so timeout -k 10 300 python bench.py --indicator p --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/${lib}_$rep.json 2> $out/${lib}_$rep.err || { echo "bench failed"; tail -5 $out/${lib}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:50], '%.1f us' % d['roofline']['launch_us'])" $out/${lib}_$rep.json
done; done
echo all-done
