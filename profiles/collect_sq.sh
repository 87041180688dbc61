# SQ/GRBM counter passes for the step kernels (one pass per counter group; no tracing).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sq_a_$TAG" -- python3 "$GRAFT_REPO_ROOT/profiles/ab_variants.py" --variants 1:4 --rounds 1 --nsteps 20 > gpurun_out/sq_a_$TAG.log 2>&1 || { echo "pass A failed"; tail -20 gpurun_out/sq_a_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sq_b_$TAG" -- python3 "$GRAFT_REPO_ROOT/profiles/ab_variants.py" --variants 1:4 --rounds 1 --nsteps 20 > gpurun_out/sq_b_$TAG.log 2>&1 || { echo "pass B failed"; tail -20 gpurun_out/sq_b_$TAG.log; exit 1; }
echo done
