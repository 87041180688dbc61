# Per-item timeline of the one-launch p-estimate (probes/pflow_trace.py) at 256- and
# 512-element tiles, with the chain and the dataflow launch timed alternately; alone, and
# after the snapshot forward as the bench runs it
set -o pipefail
o=gpurun_out/r05/p11; mkdir -p $o
for tw in 1 2; do
  for f in alone fwd; do
    timeout -k 10 300 python profiles/r05/probes/pflow_trace.py $tw 4 $f > $o/trace_w${tw}_$f.json 2> $o/trace_w${tw}_$f.err || { tail $o/trace_w${tw}_$f.err; exit 1; }
  done
done
echo all-done
