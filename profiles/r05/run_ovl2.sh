# Overlapped waves at low order: N = 1 (Np = 2) and N = 2 (Np = 3), tile widths, A/B on one box
set -o pipefail
out=gpurun_out/r05/ovl2; mkdir -p $out
bash profiles/r05/ab_env.sh $out/n1 "--N 1" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1 DG_SWEEP_WAVES=16" "DG_SWEEP_EXCHANGE=1 DG_SWEEP_WAVES=12" || exit 1
bash profiles/r05/ab_env.sh $out/n2 "--N 2" "DG_SWEEP_EXCHANGE=0" "DG_SWEEP_EXCHANGE=1" "DG_SWEEP_EXCHANGE=1 DG_SWEEP_WAVES=16" || exit 1
echo all-done
