# Neighbour-wave level hand-off (DG_NSYNC=1) vs the workgroup barrier: parity under the variant
# library, then the driver bench alternating (and N = 8, N = 1)
set -o pipefail
out=gpurun_out/r04/nsync; mkdir -p $out
DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_nsync.so timeout -k 10 300 python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_rec.py tests/test_gpu_sweep.py -k "record_pair_equals or dataflow_equals or wide" > $out/pytest.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" $out/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
bash profiles/r04/ab_libs.sh $out adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so adjoint-ode-adaptivity_amd/lib/ab/libdgadv_nsync.so || exit 1
for n in 8 1; do for lib in base nsync; do
  DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_$lib.so timeout -k 10 200 python bench.py --N $n --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/N${n}_$lib.json 2> $out/N${n}_$lib.err || { echo "bench N$n $lib failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], '%.1f us' % d['roofline']['launch_us'])" $out/N${n}_$lib.json
done; done
echo all-done
