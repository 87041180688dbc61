# k_psweep: kernel duration vs in-kernel span at 8, 12, 20 and 32 steps (W2, default build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
o=gpurun_out/r05/p20; mkdir -p $o
for n in 8 20 32; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof$n -- python3 profiles/r05/probes/psweep_trace.py 2 $o/trace_raw$n.npy $n > $o/trace$n.json 2> $o/trace$n.err || { tail $o/trace$n.err; exit 1; }
python3 - $n <<'PY'
import csv, glob, json, sys, numpy as np
n = sys.argv[1]
f = glob.glob(f"gpurun_out/r05/p20/prof{n}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_psweep" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3 for i in range(len(rows) - 1)]
t = json.load(open(f"gpurun_out/r05/p20/trace{n}.json"))
print("n", n, "k_psweep median %.1f last %.1f span %.1f  gap between launches median %.1f" % (np.median(d), d[-1], t["span_us"], np.median(gaps)))
PY
done
echo all-done
