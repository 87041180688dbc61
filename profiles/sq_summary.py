"""Per-kernel means of SQ/GRBM counter passes (profiles/r02/collect_sq.sh output).

  python profiles/sq_summary.py <dir> <tag>
Prints, per kernel, the mean counter value per dispatch and derived figures: cycles per wave
(SQ_WAVE_CYCLES counts quad-cycles on gfx950, MI355X_MICROARCH.md), the VALU-active and
wait shares, and the effective clock GRBM_GUI_ACTIVE / 8 XCDs / dispatch time."""
import collections
import csv
import glob
import os
import sys


def main():
  d, tag = sys.argv[1], sys.argv[2]
  vals = collections.defaultdict(lambda: collections.defaultdict(list))
  for path in glob.glob(os.path.join(d, f"{tag}_*", "**", "*counter_collection.csv"),
                        recursive=True):
    for r in csv.DictReader(open(path)):
      k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
      vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
  for k, cs in vals.items():
    if not any(s in k for s in ("k_step", "k_adj", "k_wstep")):
      continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c in sorted(m):
      print(f"  {c:28s} {m[c]:.4g}")
    if "SQ_WAVES" in m and "SQ_WAVE_CYCLES" in m:
      print(f"  wave-cycles per wave (x4)    {4 * m['SQ_WAVE_CYCLES'] / m['SQ_WAVES']:.1f}")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
      if c in m and "SQ_WAVE_CYCLES" in m:
        print(f"  {c} / WAVE_CYCLES        {m[c] / m['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
      print(f"  VALU insts per wave          {m['SQ_INSTS_VALU'] / m['SQ_WAVES']:.1f}")


if __name__ == "__main__":
  main()
