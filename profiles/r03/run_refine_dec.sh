#!/bin/bash
# The dataflow cleanup (4/8-wave groups only, argmax slots sized by waves) and the multi-rank
# refine decision's device half, then bench --gpus 2 (two ranks on one GPU over gloo).
set -o pipefail
mkdir -p gpurun_out/refdec
true &&
timeout -k 10 200 python -u bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 > gpurun_out/refdec/bench2.log 2>&1
rc=$?
tail -5 gpurun_out/refdec/pytest.log; tail -2 gpurun_out/refdec/bench2.log
exit $rc
