# Wide dataflow tiles (DG_SWEEP_WAVES 12 / 16) per N: correctness, then the driver bench per
# N and tile (config 5 shape: K = 2^20, 20 + 20 steps).
set -o pipefail
mkdir -p gpurun_out/r04/waves
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sweep.py -k "wide_dataflow" > gpurun_out/r04/waves/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r04/waves/tests.log; exit 1; }
tail -1 gpurun_out/r04/waves/tests.log
for N in 8 1 4 2 6; do
  for W in 0 12 16; do
    if [ $W = 16 ] && [ $N -gt 4 ]; then continue; fi
    DG_SWEEP_WAVES=$W timeout -k 10 200 python bench.py --N $N --steps 20 --warmup 5 --no-cpu-baseline --no-margin > gpurun_out/r04/waves/N${N}_w$W.json 2> gpurun_out/r04/waves/N${N}_w$W.err || { echo "bench N=$N W=$W failed"; tail -5 gpurun_out/r04/waves/N${N}_w$W.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'][:60], '%.1f us' % d['roofline']['launch_us'])" gpurun_out/r04/waves/N${N}_w$W.json
  done
done
echo all-done
