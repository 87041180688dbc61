set -o pipefail
out=gpurun_out/r04/trace_n1; mkdir -p $out
for n in 1 2; do
timeout -k 10 120 python profiles/r03/sweep_trace.py --N $n --out $out > $out/N$n.txt 2>&1 || { echo "trace failed"; tail -5 $out/N$n.txt; exit 1; }
DG_SWEEP_WAVES=8 timeout -k 10 120 python profiles/r03/sweep_trace.py --N $n --out $out > $out/N${n}_w8.txt 2>&1 || { echo "trace failed"; exit 1; }
done
for f in $out/*.json; do python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1], 'untraced %.1f traced %.1f' % (d['sweep_us_untraced'], d['sweep_us_traced']), {k: (round(v['wait_mean'],2), round(v['compute_mean'],1), round(v['first_taken'],1), round(v['last_taken'],1), round(v['last_done'],1)) for k,v in d['phases'].items()})
print(' inflight', d['timeline_5us']['in_flight'])
" $f; done
