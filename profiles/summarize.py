"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE / WRITE_SIZE passes) into
one JSON per round, and derive the per-launch HBM traffic of the hot kernels.

  python profiles/summarize.py --stats <kernel_stats.csv> --fetch <counter_collection.csv>
         --write <counter_collection.csv> --out profiles/rNN/summary.json [--traffic-json profiles/pmc_traffic.json]

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reads exactly half of the bytes of a 16-B/lane coalesced stream, so the read
side is doubled; WRITE_SIZE is exact for 16-B/lane stores.
"""
import argparse
import collections
import csv
import json
import re


def short(name):
  name = name.replace("(anonymous namespace)::", "").replace("void ", "")
  m = re.match(r"([A-Za-z_:0-9]+)(<[^(]*>)?", name)
  return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def counters(path, counter):
  agg = collections.defaultdict(list)
  for r in csv.DictReader(open(path)):
    if r["Counter_Name"] == counter:
      agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
  return agg


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--stats", required=True)
  p.add_argument("--fetch")
  p.add_argument("--write")
  p.add_argument("--out", required=True)
  p.add_argument("--traffic-json")
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--K", type=int, default=1 << 20)
  p.add_argument("--steps-per-launch", type=int, default=4)
  p.add_argument("--batch", type=int, default=1)
  p.add_argument("--record", default="jumps", choices=("jumps", "snapshots"))
  p.add_argument("--indicator", default="jump", choices=("jump", "p"))
  p.add_argument("--tile-width", type=int, default=None)
  a = p.parse_args()
  out = collections.OrderedDict()
  for r in csv.DictReader(open(a.stats)):
    out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                             "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
                             "pct": float(r["Percentage"])}
  for path, cnt, scale in ((a.fetch, "FETCH_SIZE", 2.0), (a.write, "WRITE_SIZE", 1.0)):
    if not path:
      continue
    for k, v in counters(path, cnt).items():
      d = out.setdefault(k, {})
      d[cnt + "_KiB_avg"] = sum(v) / len(v)
      d[cnt.split("_")[0].lower() + "_bytes_corrected"] = scale * 1024.0 * sum(v) / len(v)
      d[cnt.split("_")[0].lower() + "_dispatches"] = len(v)
  json.dump(out, open(a.out, "w"), indent=1)
  print(json.dumps(out, indent=1))
  if a.traffic_json:
    def hbm(key):
      d = out.get(key, {})
      if "fetch_bytes_corrected" in d and "write_bytes_corrected" in d:
        return d["fetch_bytes_corrected"] + d["write_bytes_corrected"]
      return None
    def sweep_mean(prefix):
      # a sweep's launches may run several instantiations (e.g. 8 + 8 + 4 steps): the
      # dispatch-weighted mean per launch over all of them, as bench.py averages its bytes
      keys = [k for k in out if k.startswith(prefix) and hbm(k) is not None]
      n = sum(out[k].get("fetch_dispatches", 0) for k in keys)
      if not keys or n == 0:
        return keys, None
      return keys, sum(hbm(k) * out[k]["fetch_dispatches"] for k in keys) / n

    adj, adj_b = sweep_mean("k_adj_p" if a.indicator == "p" else "k_adj")
    p_flow = p_sweep = False
    if a.indicator == "p":
      pf, pf_b = sweep_mean("k_adjp_flow")
      if pf:  # the p-estimate as one dataflow launch
        adj, adj_b, p_flow = pf, pf_b, True
      ps, ps_b = sweep_mean("k_psweep")
      if ps:  # the whole p sweep as one dataflow launch: both directions' traffic
        adj, adj_b, fwd, fwd_b, p_flow, p_sweep = ps, ps_b, [], None, True, True
    fwd, fwd_b = sweep_mean("k_step")
    dataflow = False
    sw, sw_b = sweep_mean("k_sweep_rp")
    if sw:  # the dataflow sweep: one launch per sweep carries both directions' traffic
      adj, adj_b, fwd, fwd_b, dataflow = sw, sw_b, [], None, True
    tr = {"N": a.N, "K": a.K, "batch": a.batch, "steps_per_launch": a.steps_per_launch,
          "record": a.record, "indicator": a.indicator, "dataflow": dataflow, "p_flow": p_flow,
          "p_sweep": p_sweep,
          "tile_width": a.tile_width, "source": a.out,
          "adj_kernel": adj, "adj_bytes_per_launch": adj_b,
          "fwd_kernel": fwd, "fwd_bytes_per_launch": fwd_b,
          "note": "FETCH_SIZE x2 (gfx950 16-B/lane half count) + WRITE_SIZE, KiB->bytes; "
                  "dispatch-weighted mean over the sweep's kernel instantiations"}
    json.dump(tr, open(a.traffic_json, "w"), indent=1)


if __name__ == "__main__":
  main()
