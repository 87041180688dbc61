set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c4; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --K 65536 --ics 1024 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c4/bench_config4_$r.json 2> gpurun_out/c4/err_$r || { tail -5 gpurun_out/c4/err_$r; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('config4', '%.4g'%d['value'], 'adj %.0f fwd %.0f'%(d['roofline']['launch_us'], d['roofline_fwd']['launch_us']), d['launch_steps_fwd'])" gpurun_out/c4/bench_config4_$r.json
done
