"""In-process A/B of the jump-record sweep shapes (pair tiles): interleaved rounds of one
forward_rec + adjoint_rec sweep per variant, HIP-event time per sweep direction (median).
A variant is "fwd_steps:adj_steps[:tile_width]" (tile width 2 by default: 1024-element tiles).
Also checks that every variant's w and eta are bit-identical to the first variant with the
same steps per launch (the tile shape never changes the arithmetic).

  python profiles/r03/ab_rec.py [--N 4] [--K 1048576] [--nsteps 20] [--rounds 7]
      [--variants 20:10,10:10:1,...]
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
  p.add_argument("--batch", type=int, default=1)
  p.add_argument("--nsteps", type=int, default=20)
  p.add_argument("--rounds", type=int, default=7)
  p.add_argument("--variants", default="20:10,10:10,20:20")
  p.add_argument("--lib", default=None, help="load this libdgadv.so instead (experiment builds)")
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  if a.lib:
    pkg._lib.LIB_PATH = os.path.abspath(a.lib)
  mesh = pkg.BaseGalerkin1D(n=a.N, k=a.K)
  op = pkg.operators.DGAdvection1D(mesh, batch=a.batch)
  dt = mesh.cfl_dt()
  u0 = op.new_field()
  # sine + seeded noise: resolved jumps, so eta is not rounding noise
  gen = torch.Generator(device=op.device).manual_seed(3)
  op.init_sine([1.0] * a.batch, [1.0] * a.batch, [0.0] * a.batch, out=u0)
  u0 += 0.01 * torch.randn(u0.shape, generator=gen, dtype=torch.float64, device=op.device)
  jumps = op.new_jumps(a.nsteps)
  w = op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
  variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
  res = {v: {"fwd": [], "adj": []} for v in variants}
  ref = {}
  same = {}
  st = torch.cuda.current_stream()
  for r in range(a.rounds + 1):
    for v in variants:
      op.tune(rec_tile_width=(v[2] if len(v) > 2 else 2), rec_steps_per_launch=v[1],
              rec_fwd_steps_per_launch=v[0])
      e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
      e[0].record(st)
      op.forward_rec(u0, 0.0, dt, a.nsteps, jumps, out=w)
      e[1].record(st)
      op.adjoint_rec(w, jumps, 0.0, dt, a.nsteps, eta=eta, eta_assign=True, eta_abs=True)
      e[2].record(st)
      torch.cuda.synchronize()
      if r == 0:
        key = (v[0], v[1])
        if key not in ref:
          ref[key] = (w.clone(), eta.clone())
        else:
          same[v] = bool(torch.equal(ref[key][0], w) and torch.equal(ref[key][1], eta))
      else:
        res[v]["fwd"].append(e[0].elapsed_time(e[1]) * 1e3)
        res[v]["adj"].append(e[1].elapsed_time(e[2]) * 1e3)
  out = {}
  dof = 2.0 * op.Np * op.ktot * a.nsteps
  for v in variants:
    f, d = float(np.median(res[v]["fwd"])), float(np.median(res[v]["adj"]))
    out[":".join(map(str, v))] = {"fwd_us": round(f, 2), "adj_us": round(d, 2),
                                  "sweep_us": round(f + d, 2),
                                  "dof_updates_per_s": dof / (f + d) * 1e6,
                                  "bit_identical_to_first_same_steps": same.get(v, True)}
  print(json.dumps({"N": a.N, "K": a.K, "batch": a.batch, "nsteps": a.nsteps, "lib": a.lib,
                    "variant": "fwd_steps:adj_steps[:tile_width]", "results": out},
                   indent=1))


if __name__ == "__main__":
  main()
