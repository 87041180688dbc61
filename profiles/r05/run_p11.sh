set -o pipefail
mkdir -p gpurun_out/r05/p11
timeout -k 10 300 python profiles/r05/probes/pflow_trace.py 1 4 > gpurun_out/r05/p11/trace_w1.json 2> gpurun_out/r05/p11/trace_w1.err || { tail gpurun_out/r05/p11/trace_w1.err; exit 1; }
cat gpurun_out/r05/p11/trace_w1.json
