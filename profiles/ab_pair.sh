# A/B of the in-tree library against an experiment build (lib/exp), alternating processes.
#   bash profiles/ab_pair.sh [extra ab_variants.py arguments]
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 120 python profiles/ab_variants.py --rounds 7 "$@" > gpurun_out/ab_base_$i.json &&
timeout -k 10 120 python profiles/ab_variants.py --rounds 7 "$@" --lib adjoint-ode-adaptivity_amd/lib/exp/libdgadv.so > gpurun_out/ab_exp_$i.json || exit 1
done
