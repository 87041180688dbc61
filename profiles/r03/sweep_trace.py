"""Timeline of the dataflow sweep's work items (dg_plan_sweep_trace): per item the wall-clock
times it was taken, its producers were done and it was published.  Prints per phase (forward
blocks, adjoint blocks) the span, the mean wait for producers and the mean compute time, and
the number of items in flight over time; saves the raw trace.

  python profiles/r03/sweep_trace.py [--N 4] [--K 1048576] [--nsteps 20] [--out DIR]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--K", type=int, default=1 << 20)
  p.add_argument("--nsteps", type=int, default=20)
  p.add_argument("--fwd-steps", type=int, default=0)
  p.add_argument("--reps", type=int, default=30)
  p.add_argument("--out", default="gpurun_out/r03/trace")
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  mesh = pkg.BaseGalerkin1D(n=a.N, k=a.K)
  op = pkg.operators.DGAdvection1D(mesh)
  if a.fwd_steps:
    op.tune(rec_fwd_steps_per_launch=a.fwd_steps)
  on, msf, msa, items, waves, T = op.query_sweep(a.nsteps, tile=True)
  assert on, "the plan does not run the dataflow sweep"
  dt = mesh.cfl_dt()
  u0 = op.new_field()
  op.init_sine([1.0], [1.0], [0.0], out=u0)
  rec, w = op.new_jumps(a.nsteps), op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
  sw = lambda: op.sweep_rec(u0, rec, w, 0.0, dt, a.nsteps, eta=eta, eta_assign=True, eta_abs=True)  # noqa
  st = torch.cuda.current_stream()
  for _ in range(a.reps):
    sw()
  ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
  ev[0].record(st)
  for _ in range(a.reps):
    sw()
  ev[1].record(st)
  torch.cuda.synchronize()
  t_plain = ev[0].elapsed_time(ev[1]) * 1e3 / a.reps
  tr = torch.zeros(4 * items, dtype=torch.int64, device=op.device)
  op.sweep_trace(tr)
  for _ in range(3):
    sw()
  torch.cuda.synchronize()
  op.sweep_trace(None)
  assert op.sweep_status() == 0
  t = tr.cpu().numpy().reshape(items, 4)
  t0 = t[:, 0].min()
  deq, ready, done = [(t[:, k] - t0) / 100.0 for k in range(3)]  # us (100 MHz)
  xcc = (t[:, 3] >> 32).astype(int)
  nTF = (items - (a.nsteps // msa) * 0) and None
  nbF, nbA = a.nsteps // msf, a.nsteps // msa
  # item counts per phase (T: elements per tile, the plan's shape)
  nTF = -(-op.ktot // (T - 2 * ((msf * 5 + 2) & ~1)))
  nTA = -(-op.ktot // (T - 2 * ((msa * 5 + 1) & ~1)))
  phases = [(f"F{b}", b * nTF, (b + 1) * nTF) for b in range(nbF)]
  phases += [(f"A{b}", nbF * nTF + b * nTA, nbF * nTF + (b + 1) * nTA) for b in range(nbA)]
  summ = {"N": a.N, "K": a.K, "nsteps": a.nsteps, "blocks": [msf, msa], "items": int(items),
          "tile_elements": int(T), "waves": int(waves),
          "sweep_us_untraced": t_plain, "sweep_us_traced": float(done.max()),
          "xcc_items": np.bincount(xcc, minlength=8).tolist(), "phases": {}}
  for name, lo, hi in phases:
    summ["phases"][name] = {
        "items": hi - lo, "first_taken": float(deq[lo:hi].min()), "last_taken": float(deq[lo:hi].max()),
        "first_done": float(done[lo:hi].min()), "last_done": float(done[lo:hi].max()),
        "wait_mean": float((ready[lo:hi] - deq[lo:hi]).mean()),
        "wait_max": float((ready[lo:hi] - deq[lo:hi]).max()),
        "wait_gt_1us": int(((ready[lo:hi] - deq[lo:hi]) > 1.0).sum()),
        "compute_mean": float((done[lo:hi] - ready[lo:hi]).mean()),
        "compute_p10_p90": [float(np.percentile(done[lo:hi] - ready[lo:hi], q)) for q in (10, 90)]}
  grid = np.arange(0, done.max() + 5, 5.0)
  inflight = [int(((deq <= g) & (done > g)).sum()) for g in grid]
  waiting = [int(((deq <= g) & (ready > g)).sum()) for g in grid]
  summ["timeline_5us"] = {"t": grid.tolist(), "in_flight": inflight, "waiting": waiting}
  os.makedirs(a.out, exist_ok=True)
  np.save(os.path.join(a.out, f"trace_N{a.N}_f{msf}_w{waves}.npy"), t)
  with open(os.path.join(a.out, f"trace_N{a.N}_f{msf}_w{waves}.json"), "w") as f:
    json.dump(summ, f, indent=1)
  print(json.dumps({k: v for k, v in summ.items() if k != "timeline_5us"}, indent=1))
  print("in flight every 20 us:", inflight[::4])
  print("waiting   every 20 us:", waiting[::4])


if __name__ == "__main__":
  main()
