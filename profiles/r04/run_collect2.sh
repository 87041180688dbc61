set -o pipefail
bash profiles/r04/collect.sh headline k_sweep_rp || exit 1
bash profiles/r04/collect.sh p k_adj_p --indicator p || exit 1
echo all-done
