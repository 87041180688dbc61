set -o pipefail
cd "$GRAFT_REPO_ROOT"
for n in 1 2 6; do
  bash profiles/r02/ab_env.sh f20N$n "" "DG_REC_FWD_STEPS_PER_LAUNCH=10" -- --N $n || exit 1
done
