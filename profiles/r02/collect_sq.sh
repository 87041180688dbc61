# SQ/GRBM counter passes for one step kernel (one pass per counter group; no tracing).
#   bash profiles/r02/collect_sq.sh <tag> <fwd|fwd_nosnap|adj> [kernel_driver args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-x}; WHAT=${2:-fwd}; shift 2
OUT="$GRAFT_REPO_ROOT/gpurun_out/sq"; mkdir -p "$OUT"
[ -f "$OUT/counters_avail.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 || true
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
         "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d "$OUT/${TAG}_$i" -- python3 "$GRAFT_REPO_ROOT/profiles/kernel_driver.py" --what $WHAT "$@" > "$OUT/${TAG}_$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/${TAG}_$i.log"; }
done
python3 profiles/sq_summary.py "$OUT" "$TAG" > "$OUT/${TAG}_summary.txt" 2>&1; cat "$OUT/${TAG}_summary.txt"
