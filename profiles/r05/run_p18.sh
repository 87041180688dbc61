# k_psweep: kernel duration (rocprof) against its in-kernel span (trace), same process
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
o=gpurun_out/r05/p18; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -- python3 profiles/r05/probes/psweep_trace.py 2 $o/trace_raw.npy > $o/trace.json 2> $o/trace.err || { tail $o/trace.err; exit 1; }
python3 - <<'PY'
import csv, glob, json, numpy as np
f = glob.glob("gpurun_out/r05/p18/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_psweep" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("k_psweep calls", len(d), "median", np.median(d), "last", d[-1], "scratch", rows[-1]["Scratch_Size"], "vgpr", rows[-1]["VGPR_Count"])
t = json.load(open("gpurun_out/r05/p18/trace.json"))
print("span", t["span_us"], "first deq", t["blocks"][0]["deq_first_us"], "mean in flight", t["mean_in_flight"])
PY
echo all-done
