# k_adjp_flow's duration under rocprof in the probe (forward + estimate loop) and in the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
o=gpurun_out/r05/p12; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/probe -- python3 profiles/r05/probes/pflow_trace.py 1 4 fwd > $o/probe.json 2> $o/probe.err || { tail $o/probe.err; exit 1; }
DG_P_FLOW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-margin --indicator p > $o/bench.log 2>&1 || { tail $o/bench.log; exit 1; }
python3 - <<'PY'
import csv, glob, numpy as np
for tag in ("probe", "bench"):
  f = glob.glob(f"gpurun_out/r05/p12/{tag}/**/*kernel_trace.csv", recursive=True)[0]
  rows = list(csv.DictReader(open(f)))
  for k in ("k_adjp_flow", "k_adj_ph", "k_step"):
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if k in r['Kernel_Name']]
    if d:
      print(tag, k, len(d), np.round(np.percentile(d, [0, 10, 50, 90, 100]), 1))
PY
echo all-done
