set -o pipefail
cd "$GRAFT_REPO_ROOT"
for k in 2097152 4194304; do
  bash profiles/r02/ab_env.sh fxK$k "" "DG_REC_FWD_STEPS_PER_LAUNCH=10" -- --K $k || exit 1
done
bash profiles/r02/ab_env.sh fxC4 "" "DG_REC_FWD_STEPS_PER_LAUNCH=10" -- --K 65536 --ics 1024 || exit 1
