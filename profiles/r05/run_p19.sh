# k_psweep without the occupancy cap (no scratch): kernel duration vs in-kernel span, W1 and W2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
o=gpurun_out/r05/p19; mkdir -p $o
for tw in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof$tw -- python3 profiles/r05/probes/psweep_trace.py $tw $o/trace_raw$tw.npy > $o/trace$tw.json 2> $o/trace$tw.err || { tail $o/trace$tw.err; exit 1; }
python3 - $tw <<'PY'
import csv, glob, json, sys, numpy as np
tw = sys.argv[1]
f = glob.glob(f"gpurun_out/r05/p19/prof{tw}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_psweep" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
t = json.load(open(f"gpurun_out/r05/p19/trace{tw}.json"))
print("tw", tw, "k_psweep median", np.median(d), "last", d[-1], "scratch", rows[-1]["Scratch_Size"], "span", t["span_us"], "in flight", t["mean_in_flight"])
PY
done
echo all-done
