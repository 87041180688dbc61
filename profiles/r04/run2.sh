# Round 4, GPU pass 1 (+ A/B): the argmax reproducer, the new parity/watchdog tests, the
# driver bench with the product library (k_sweep_rp capped at 6 waves/SIMD, odd-first adjoint
# volume order) against the round-3 library (lib/ab/libdgadv_base.so), alternating.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 60 ./profiles/probes/argmax_phi_copy > gpurun_out/r04/argmax_probe.txt 2>&1; echo "probe exit $?" >> gpurun_out/r04/argmax_probe.txt
BASE=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04/ab_new_$i.json 2> gpurun_out/r04/ab_new_$i.err || { echo "bench new failed"; tail -20 gpurun_out/r04/ab_new_$i.err; exit 1; }
  DG_LIB_PATH=$BASE timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04/ab_base_$i.json 2> gpurun_out/r04/ab_base_$i.err || { echo "bench base failed"; tail -20 gpurun_out/r04/ab_base_$i.err; exit 1; }
done
python - <<'PY'
import json
for tag in ("new_1", "base_1", "new_2", "base_2"):
  d = json.load(open(f"gpurun_out/r04/ab_{tag}.json"))
  print(tag, "%.4g" % d["value"], "launch us %.1f" % d["roofline"]["launch_us"], d["refine_decision"]["decided"] if d.get("refine_decision") else None)
PY
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sweep.py tests/test_gpu_eta_modes.py tests/test_gpu_bench.py \
  "tests/test_gpu_full_size.py::test_full_size_dataflow_sweep_refine" \
  "tests/test_gpu_full_size.py::test_full_size_bench_workload" \
  "tests/test_gpu_full_size.py::test_full_size_dataflow_config4_shape" \
  > gpurun_out/r04/pytest1.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r04/pytest1.log; exit 1; }
tail -3 gpurun_out/r04/pytest1.log
echo all-done
