# config 4 shape on one GPU (1024 trajectories x 65,536 elements): record vs snapshot sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c4; export TMPDIR=/tmp
for r in jumps snapshots; do
  timeout -k 10 300 python bench.py --K 65536 --ics 1024 --steps 10 --warmup 3 --no-cpu-baseline --record $r > gpurun_out/c4/bench_$r.json 2> gpurun_out/c4/err || { tail -5 gpurun_out/c4/err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4/bench_$r.json')); print('$r', '%.4g' % d['value'], 'ms', '%.3f' % d['ms_per_step'], 'adj', '%.1f' % d['roofline']['launch_us'], '%.3f' % d['roofline']['frac'], 'fwd', '%.1f' % d['roofline_fwd']['launch_us'], '%.3f' % d['roofline_fwd']['frac'], d['launch_steps'])"
done
