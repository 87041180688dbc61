#!/bin/bash
# rocprof kernel stats of bench.py --config 3 (narrow-cone adjoint tiles + the wide pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/c3prof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 bench.py --config 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
STATS=$(find $OUT/prof -name '*kernel_stats.csv' -print -quit); cp "$STATS" $OUT/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c3prof/kernel_stats.csv")))
for r in rows[:12]:
    print(r["Name"][:90], r["Calls"], f'{float(r["AverageNs"])/1e3:.1f} us', f'{float(r["Percentage"]):.1f}%')
PY
