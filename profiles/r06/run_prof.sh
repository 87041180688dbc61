# Round 6: refreshed profiles of the bench lines (headline dataflow sweep, p sweep, N = 1)
set -o pipefail
bash profiles/r06/collect.sh headline k_sweep_rp && \
bash profiles/r06/collect.sh p k_psweep --indicator p && \
bash profiles/r06/collect.sh N1 k_sweep_rp --N 1 && echo all-done
