# SQ occupancy / issue counters of the direct-to-LDS Horner estimate at 256- and 512-element tiles
set -o pipefail
export DG_P_HORNER=3
bash profiles/r05/collect.sh p_gl_w1 k_adj_ph --indicator p || exit 1
DG_P_TILE_WIDTH=2 DG_P_STEPS_PER_LAUNCH=4 bash profiles/r05/collect.sh p_gl_w2 k_adj_ph --indicator p || exit 1
for t in p_gl_w1 p_gl_w2; do python3 -c "
import json; d=json.load(open('gpurun_out/r05/$t/sq_summary.json')); print('$t', d['kernel'][0][:40], {k: round(v,1) for k,v in d['per_wave'].items()}, d['wait_any_frac_of_wave_cycles'], d['valu_active_frac_of_wave_cycles'], d['per_launch']['SQ_WAVE_CYCLES']/d['per_launch']['GRBM_GUI_ACTIVE'])"; done
echo all-done
