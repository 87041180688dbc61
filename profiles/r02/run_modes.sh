# The three bench modes on one box at the end of round 2: config 2 (record sweep, default),
# config 2 with snapshots, config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/modes; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/err1 || { tail -5 $OUT/err1; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --record snapshots --no-cpu-baseline > $OUT/bench_snapshots.json 2> $OUT/err2 || { tail -5 $OUT/err2; exit 1; }
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline > $OUT/bench_config3.json 2> $OUT/err3 || { tail -5 $OUT/err3; exit 1; }
for f in default snapshots config3; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], '%.4g'%d['value'], r.get('kernel','')[:40], 'launch %.1f'%r['launch_us'], 'frac %.3f'%r['frac'])" $OUT/bench_$f.json $f; done
