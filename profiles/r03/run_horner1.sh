# Round 3: the Horner-form pair kernels.  Parity tests of the record path (some assert
# bit-identity with the LSERK stage-loop kernels and are expected to change), then the A/B
# against the LSERK build (lib/exp) and the driver bench.
set -o pipefail
OUT=gpurun_out/r03/horner; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_rec.py tests/test_gpu_ties.py tests/test_gpu_eta_modes.py -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" $OUT/tests.log | tail -3; grep -E "^FAILED" $OUT/tests.log | head -30
bash profiles/r03/ab_lib.sh horner --variants 20:10,10:10 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json
d = json.load(open('$OUT/bench.json')); print('bench', d['value'], d['roofline']['launch_us'], d['roofline_fwd']['launch_us'])"
