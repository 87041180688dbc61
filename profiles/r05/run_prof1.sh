# Round-5 profiles: the headline (driver command's config) and the p-estimate (--indicator p)
set -o pipefail
bash profiles/r05/collect.sh headline k_sweep_rp || exit 1
bash profiles/r05/collect.sh p k_adj_ph --indicator p || exit 1
for t in headline p; do python3 -c "
import json; d=json.load(open('gpurun_out/r05/$t/sq_summary.json')); t=json.load(open('gpurun_out/r05/$t/pmc_traffic.json'))
print('$t', d['kernel'], 'wait %.3f valu %.3f' % (d['wait_any_frac_of_wave_cycles'], d['valu_active_frac_of_wave_cycles']), 'traffic', t['adj_bytes_per_launch'])"; done
echo all-done
