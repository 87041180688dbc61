# Round 6: config-3 forward tile width A/B (512 = default, 768, 1024-element workgroup tiles;
# variant libraries built from patched csrc copies, DG_LIB_PATH)
set -o pipefail
out=gpurun_out/r06/c3w; mkdir -p $out
L=adjoint-ode-adaptivity_amd/lib
for i in 1 2; do
  for v in base w3 w4; do
    if [ $v = base ]; then lib=$L/libdgadv.so; else lib=$L/libdgadv_$v.so; fi
    DG_LIB_PATH=$lib timeout -k 10 300 python3 -u bench.py --config 3 --no-cpu-baseline > $out/c3_${v}_$i.json 2> $out/c3_${v}_$i.err || { tail $out/c3_${v}_$i.err; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06/c3w/*.json")):
  d = json.loads(open(f).read().strip().splitlines()[-1])
  print(f, "%.4g" % d["value"], "adj %.1f" % d["roofline"]["launch_us"], "fwd %.1f" % d["roofline_fwd"]["launch_us"])
PY
echo all-done
