# PMC + SQ profiles of config 5's ends: N = 1 (dataflow, default) and N = 8 (dataflow, 8-wave
# tiles); per-item traces of the headline shape with 8- and 12-wave tiles
set -o pipefail
mkdir -p gpurun_out/r04/trace_w
timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_w > gpurun_out/r04/trace_w/w8.txt 2>&1 || exit 1
DG_SWEEP_WAVES=12 timeout -k 10 120 python profiles/r03/sweep_trace.py --out gpurun_out/r04/trace_w > gpurun_out/r04/trace_w/w12.txt 2>&1 || exit 1
grep -A3 '"F0"\|"A0"\|"A1"\|sweep_us' gpurun_out/r04/trace_w/w8.txt gpurun_out/r04/trace_w/w12.txt | grep -v p10 | head -60
bash profiles/r04/collect.sh N1 k_sweep_rp --N 1 || exit 1
DG_SWEEP_WAVES=8 bash profiles/r04/collect.sh N8 k_sweep_rp --N 8 || exit 1
echo all-done
