"""Launch time of one fused forward launch (4 steps, no snapshots) at K = 256*n*TE elements,
i.e. exactly n tiles per CU, n = 1..12: where the time per round jumps shows how many
workgroups per CU are really co-resident.

  python profiles/occupancy_probe.py [--N 4] [--ms 4]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--ms", type=int, default=4)
  p.add_argument("--reps", type=int, default=20)
  p.add_argument("--what", default="fwd")
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  TE = 256 - 2 * a.ms * 5
  out = {}
  for n in list(range(1, 13)) + [16, 24]:
    K = 256 * n * TE
    mesh = pkg.BaseGalerkin1D(n=a.N, k=K)
    op = pkg.operators.DGAdvection1D(mesh).tune(steps_per_launch=a.ms)
    dt = mesh.cfl_dt()
    snaps = op.new_field(a.ms + 1)
    op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
    op.forward(snaps[0], 0.0, dt, a.ms, snaps)
    u = op.new_field()
    eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
    st = torch.cuda.current_stream()
    ts = []
    for r in range(a.reps + 2):
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      if a.what == "adj":
        u.copy_(snaps[a.ms])
      e0.record(st)
      if a.what == "fwd":
        op.forward(u, 0.0, dt, a.ms)
      elif a.what == "fwdsnap":  # one launch writing ms snapshots, no copies in the bracket
        op.forward(snaps[0], 0.0, dt, a.ms, snaps)
      else:
        op.adjoint(u, snaps, 0.0, dt, a.ms, eta=eta)
      e1.record(st)
      torch.cuda.synchronize()
      if r >= 2:
        ts.append(e0.elapsed_time(e1) * 1e3)
    out[n] = {"K": K, "us": float(np.median(ts)), "us_per_tile_round": float(np.median(ts)) / n}
    print(n, out[n], flush=True)
    del snaps, u, eta, op, mesh
  print(json.dumps(out))


if __name__ == "__main__":
  main()
