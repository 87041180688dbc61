"""In-process A/B of the step-kernel shapes (cdna_hip_programming.md §5.4 rule 24):
interleaved rounds, median per-launch time of the forward and adjoint kernels.

  python profiles/ab_variants.py [--N 4] [--K 1048576] [--nsteps 20] [--rounds 5]
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
  p.add_argument("--K", type=int, default=1 << 20)
  p.add_argument("--nsteps", type=int, default=20)
  p.add_argument("--rounds", type=int, default=5)
  p.add_argument("--variants", default="1:4:1,1:4:0,2:4:1,2:4:0,1:2:1,2:2:1")
  p.add_argument("--lib", default=None, help="load this libdgadv.so instead (experiment builds)")
  p.add_argument("--flux", default="linear", choices=("linear", "burgers"))
  p.add_argument("--limiter", default="0", choices=("0", "N", "1"))
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  if a.lib:
    pkg._lib.LIB_PATH = os.path.abspath(a.lib)
  mesh = pkg.BaseGalerkin1D(n=a.N, k=a.K)
  op = pkg.operators.DGAdvection1D(mesh, flux=a.flux,
                                   limiter={"0": False, "N": "N", "1": "1"}[a.limiter])
  dt = mesh.cfl_dt()
  snaps = op.new_field(a.nsteps + 1)
  op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
  w = op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
  variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
  res = {v: {"fwd": [], "adj": [], "fwd_nosnap": []} for v in variants}
  u2 = op.new_field()
  st = torch.cuda.current_stream()
  for r in range(a.rounds + 1):
    for v in variants:
      op.tune(tile_width=v[0], steps_per_launch=v[1], xcd_order=(v[2] if len(v) > 2 else 1),
              lane_elements=(v[3] if len(v) > 3 else 0))
      e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
      e[0].record(st)
      op.forward(snaps[0], 0.0, dt, a.nsteps, snaps)
      e[1].record(st)
      w.copy_(snaps[a.nsteps])
      op.adjoint(w, snaps, 0.0, dt, a.nsteps, eta=eta)
      e[2].record(st)
      u2.copy_(snaps[0])
      e[3].record(st)
      op.forward(u2, 0.0, dt, a.nsteps)  # final state only: no snapshot stores
      e.append(torch.cuda.Event(enable_timing=True))
      e[4].record(st)
      torch.cuda.synchronize()
      if r > 0:  # round 0 is warm-up
        res[v]["fwd"].append(e[0].elapsed_time(e[1]) * 1e3 / a.nsteps)
        res[v]["adj"].append(e[1].elapsed_time(e[2]) * 1e3 / a.nsteps)
        res[v]["fwd_nosnap"].append(e[3].elapsed_time(e[4]) * 1e3 / a.nsteps)
  Np = a.N + 1
  fb, ab = 16.0 * Np * a.K, 24.0 * Np * a.K + 16.0 * a.K
  out = {}
  for v in variants:
    f, d = float(np.median(res[v]["fwd"])), float(np.median(res[v]["adj"]))
    out[f"width={v[0]} steps/launch={v[1]} xcd={v[2] if len(v) > 2 else 1} "
        f"lane_elems={v[3] if len(v) > 3 else 0}"] = {"fwd_us": f, "fwd_GBs": fb / f / 1e3, "adj_us": d,
                                         "adj_GBs": ab / d / 1e3,
                                         "fwd_nosnap_us": float(np.median(res[v]["fwd_nosnap"])),
                                         "fwd_min_us": float(np.min(res[v]["fwd"])),
                                         "adj_min_us": float(np.min(res[v]["adj"]))}
  print(json.dumps({"N": a.N, "K": a.K, "nsteps": a.nsteps, "results": out}, indent=1))


if __name__ == "__main__":
  main()
