# Snapshot forward on pair tiles + terminal prolong fused: parity (new tests + dwr + parity
# forward tests), then the p-estimate profile (kernel stats, PMC, SQ) and two bench lines
set -o pipefail
out=gpurun_out/r05/p4; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwr.py tests/test_gpu_parity.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit 1
bash profiles/r05/collect.sh p k_adj_ph --indicator p || exit 1
bash profiles/r05/ab_env.sh $out/ab "--indicator p" "DG_P_HORNER=1" "DG_P_HORNER=2" || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r05/p/kernel_stats.csv')))
for r in rows[:8]:
  print('%-60s %6s %8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY

bash profiles/r05/collect_c3.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r05/config3/pmc.json')); print({k: (v.get('hbm_bytes_per_launch'), v.get('avg_us')) for k, v in d['kernels'].items()})"
echo all-done
