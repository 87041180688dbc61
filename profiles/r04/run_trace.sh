# Per-item traces of the dataflow sweep: product library vs the round-3 library.
set -o pipefail
mkdir -p gpurun_out/r04/trace_new gpurun_out/r04/trace_base
timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_new > gpurun_out/r04/trace_new.txt 2>&1 || exit 1
DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_base > gpurun_out/r04/trace_base.txt 2>&1 || exit 1
grep -A3 '"F0"\|"A0"\|"A1"\|sweep_us' gpurun_out/r04/trace_new.txt | head -40
echo ---- base
grep -A3 '"F0"\|"A0"\|"A1"\|sweep_us' gpurun_out/r04/trace_base.txt | head -40
