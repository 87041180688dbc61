# Round 4: full-size p-estimate parity, then the headline and p-estimate profiles.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_dwr.py::test_full_size_p_estimate" > gpurun_out/r04/p_full.log 2>&1 || { echo "p test failed"; tail -30 gpurun_out/r04/p_full.log; exit 1; }
tail -1 gpurun_out/r04/p_full.log
bash profiles/r04/collect.sh headline k_sweep_rp || exit 1
bash profiles/r04/collect.sh p k_adj_p --indicator p || exit 1
echo all-done
