# jump-record sweeps: parity tests (incl. ensemble + full size), then record shapes at N=4
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/rec; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rec.py tests/test_gpu_eta_modes.py tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -v --timeout 300 --timeout-method thread > gpurun_out/rec/pytest2.log 2>&1
rc=$?; tail -2 gpurun_out/rec/pytest2.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/rec/pytest2.log | head -30; exit $rc; }
bash profiles/r02/tune_rec.sh "4" "2:8 4:8 4:4 2:4 2:8"
