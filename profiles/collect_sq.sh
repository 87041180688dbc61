# SQ/GRBM counter passes for one step kernel (one pass per counter group; no tracing).
#   bash profiles/collect_sq.sh <tag> [fwd_nosnap|fwd|adj]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r1}; WHAT=${2:-fwd_nosnap}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || true
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
         "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $G --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sq_${TAG}_$i" -- python3 "$GRAFT_REPO_ROOT/profiles/kernel_driver.py" --what $WHAT > gpurun_out/sq_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_${TAG}_$i.log; }
done
echo done
