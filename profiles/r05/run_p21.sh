# Per-item trace of the whole-sweep launch (fixed tile count) at 20 steps, and kernel duration
# vs the items' span at 8, 20 and 32 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
o=gpurun_out/r05/p21; mkdir -p $o
for n in 20 8 32; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof$n -- python3 profiles/r05/probes/psweep_trace.py 2 $o/trace_raw$n.npy $n > $o/trace$n.json 2> $o/trace$n.err || { tail $o/trace$n.err; exit 1; }
python3 - $n <<'PY'
import csv, glob, json, sys, numpy as np
n = sys.argv[1]
f = glob.glob(f"gpurun_out/r05/p21/prof{n}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_psweep" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
t = json.load(open(f"gpurun_out/r05/p21/trace{n}.json"))
print("n", n, "k_psweep median %.1f last %.1f span %.1f items %d" % (np.median(d), d[-1], t["span_us"], t["items"]))
PY
done
echo all-done
