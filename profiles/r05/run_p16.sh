set -o pipefail
o=gpurun_out/r05/p16; mkdir -p $o
timeout -k 10 300 python profiles/r05/probes/psweep_trace.py 2 > $o/trace_w2.json 2> $o/trace_w2.err || { tail $o/trace_w2.err; exit 1; }
echo all-done
