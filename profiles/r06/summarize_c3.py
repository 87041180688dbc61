"""Per-kernel HBM traffic, issued fp64 operations and wait / VALU-active fractions of the
config-3 kernels (both exchanges: k_step_nl / k_adj_nl / k_adj_nl_wide and the overlapped-wave
k_step_nlw / k_adj_nlw / k_adj_nlw_wide) from rocprofv3 CSVs (profiles/r06/collect_c3.sh) ->
one JSON the bench's config-3 line reads (profiles/r06/config3/pmc.json).

FETCH_SIZE / WRITE_SIZE in KiB (FETCH_SIZE doubled: gfx950 counts half of a 16-B/lane stream,
MI355X_MICROARCH.md); SQ_INSTS_VALU_{FMA,ADD,MUL}_F64 count wave instructions, so issued fp64
flops = 64 lanes x (2 FMA + ADD + MUL) per launch (every lane of a wave counted: ghost and halo
lanes included).  SQ_WAIT_ANY and SQ_ACTIVE_INST_VALU over SQ_WAVE_CYCLES: the fraction of the
waves' cycles spent waiting / issuing VALU (all three count quad-cycles on gfx950)."""
import argparse
import collections
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from summarize import short  # noqa: E402


def per_kernel(path, name):
  agg = collections.defaultdict(list)
  if not path or not os.path.exists(path):
    return agg
  for r in csv.DictReader(open(path)):
    if r["Counter_Name"] == name:
      agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
  return agg


def mean(v):
  return sum(v) / len(v) if v else 0.0


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--stats", required=True)
  p.add_argument("--fetch")
  p.add_argument("--write")
  p.add_argument("--sq")
  p.add_argument("--wait")
  p.add_argument("--out", required=True)
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--K", type=int, default=1 << 22)
  a = p.parse_args()
  out = {"N": a.N, "K": a.K, "kernels": {}, "source": os.path.relpath(a.out)}
  stats = {short(r["Name"]): r for r in csv.DictReader(open(a.stats))}
  fetch, write = per_kernel(a.fetch, "FETCH_SIZE"), per_kernel(a.write, "WRITE_SIZE")
  fma, add, mul = (per_kernel(a.sq, c) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64",
                                                  "SQ_INSTS_VALU_MUL_F64"))
  wait, cyc, valu = (per_kernel(a.wait, c) for c in ("SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
                                                      "SQ_ACTIVE_INST_VALU"))
  ivalu, isalu, ilds, waves = (per_kernel(a.wait, c) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU",
                                                               "SQ_INSTS_LDS", "SQ_WAVES"))
  for k in stats:
    if not re.match(r"k_(step|adj)_nl", k):
      continue
    d = {"avg_us": float(stats[k]["AverageNs"]) / 1e3, "calls": int(stats[k]["Calls"])}
    if fetch.get(k) and write.get(k):
      d["hbm_bytes_per_launch"] = 1024.0 * (2.0 * mean(fetch[k]) + mean(write[k]))
    if fma.get(k):
      d["fp64_flops_issued_per_launch"] = 64.0 * (2 * mean(fma[k]) + mean(add.get(k, [])) +
                                                  mean(mul.get(k, [])))
    if cyc.get(k) and mean(cyc[k]) > 0:
      d["wait_any_frac"] = mean(wait.get(k, [])) / mean(cyc[k])
      d["valu_active_frac"] = mean(valu.get(k, [])) / mean(cyc[k])
    if ivalu.get(k) and waves.get(k) and mean(waves[k]) > 0:
      # VALU / SALU / LDS instructions per wave, and all of a launch's VALU instructions
      w = mean(waves[k])
      d["valu_insts_per_wave"] = mean(ivalu[k]) / w
      d["salu_insts_per_wave"] = mean(isalu.get(k, [])) / w
      d["lds_insts_per_wave"] = mean(ilds.get(k, [])) / w
      d["valu_insts_per_launch"] = mean(ivalu[k])
    out["kernels"][k] = d
  json.dump(out, open(a.out, "w"), indent=1)
  print(json.dumps(out, indent=1))


if __name__ == "__main__":
  main()
