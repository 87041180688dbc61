set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/f2
timeout -k 10 120 ./profiles/probes/fp64_mix > gpurun_out/f2/fp64_mix.jsonl && cat gpurun_out/f2/fp64_mix.jsonl
