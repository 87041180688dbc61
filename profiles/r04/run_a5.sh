# Headline shape with 5-step adjoint blocks on 12-wave tiles (shorter drain, less adjoint halo,
# 4 adjoint blocks) against the default 10 + 10, alternating on one box
set -o pipefail
out=gpurun_out/r04/a5; mkdir -p $out
DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_a5.so DG_SWEEP_WAVES=12 DG_REC_STEPS_PER_LAUNCH=5 DG_REC_FWD_STEPS_PER_LAUNCH=20 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "tests/test_gpu_full_size.py::test_full_size_dataflow_sweep_refine" -k "4" > $out/pytest.log 2>&1; tail -3 $out/pytest.log
for rep in 1 2; do
  DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/base_$rep.json 2> $out/base_$rep.err || exit 1
  DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_a5.so DG_SWEEP_WAVES=12 DG_REC_STEPS_PER_LAUNCH=5 DG_REC_FWD_STEPS_PER_LAUNCH=20 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin > $out/a5_$rep.json 2> $out/a5_$rep.err || { tail -5 $out/a5_$rep.err; exit 1; }
  for t in base a5; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:70], '%.1f us' % d['roofline']['launch_us'])" $out/${t}_$rep.json; done
done
echo all-done
