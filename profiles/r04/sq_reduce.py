"""Mean SQ/GRBM counters per dispatch of one kernel (matched by substring) over the SQ passes
of profiles/r04/collect.sh, and the derived figures the bench line reads: issued fp64 flops
per launch (64 lanes x (2 FMA + ADD + MUL) wave instructions), wait and VALU-active shares of
the wave cycles, VALU instructions per wave.

  python profiles/r04/sq_reduce.py OUTDIR KERNEL_SUBSTRING   -> OUTDIR/sq_summary.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
  out, ksub = sys.argv[1], sys.argv[2]
  agg = collections.defaultdict(list)
  names = set()
  for f in glob.glob(os.path.join(out, "sq*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
      if ksub in r["Kernel_Name"]:
        names.add(r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:120])
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
  res = {c: sum(v) / len(v) for c, v in agg.items()}
  w = res.get("SQ_WAVES", 1.0)
  per_wave = {c: res[c] / w for c in res
              if c.startswith(("SQ_INSTS", "SQ_WAIT", "SQ_ACTIVE")) or c in ("SQ_WAVE_CYCLES",
                                                                              "SQ_BUSY_CYCLES")}
  fl = 64.0 * (2 * res.get("SQ_INSTS_VALU_FMA_F64", 0) + res.get("SQ_INSTS_VALU_ADD_F64", 0) +
               res.get("SQ_INSTS_VALU_MUL_F64", 0))
  summary = {"kernel": sorted(names), "per_launch": res, "per_wave": per_wave,
             "fp64_flops_issued_per_launch": fl,
             "wait_any_frac_of_wave_cycles":
                 res.get("SQ_WAIT_ANY", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1),
             "valu_active_frac_of_wave_cycles":
                 res.get("SQ_ACTIVE_INST_VALU", 0) / max(res.get("SQ_WAVE_CYCLES", 1), 1),
             "note": "SQ_WAVE_CYCLES counts quad-cycles on gfx950 (MI355X_MICROARCH.md); the "
                     "fractions are of the waves' own cycles"}
  json.dump(summary, open(os.path.join(out, "sq_summary.json"), "w"), indent=1)
  print(json.dumps(summary, indent=1))


if __name__ == "__main__":
  main()
