"""Minimal driver for counter collection on one step kernel (no timing, no checks):

  python profiles/kernel_driver.py --what fwd_nosnap|fwd|adj|fwd_rec|adj_rec [--N 4] [--K 1048576] [--reps 3]
                                   [--physics linear|burgers_limited] [--nonuniform]

Runs `reps` sweeps of --nsteps steps of the chosen kernel after one warm-up sweep.
--physics burgers_limited is BASELINE config 3 (Burgers flux + SlopeLimitN per stage);
--nonuniform splits one element first, as the config-3 refine loop does, so the kernels run
their non-uniform-mesh specialisation."""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--what", default="fwd_nosnap")
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--K", type=int, default=1 << 20)
  p.add_argument("--nsteps", type=int, default=20)
  p.add_argument("--reps", type=int, default=3)
  p.add_argument("--steps-per-launch", type=int, default=None)
  p.add_argument("--physics", default="linear", choices=("linear", "burgers_limited"))
  p.add_argument("--nonuniform", action="store_true")
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  v_x = np.linspace(0.0, 1.0, a.K + 1)
  if a.nonuniform:
    v_x = np.insert(v_x, a.K // 3 + 1, 0.5 * (v_x[a.K // 3] + v_x[a.K // 3 + 1]))[:-1]
    v_x = v_x / v_x[-1]
  mesh = pkg.BaseGalerkin1D(n=a.N, v_x=v_x)
  kw = {} if a.physics == "linear" else dict(flux="burgers", limiter=True)
  op = pkg.operators.DGAdvection1D(mesh, **kw)
  if a.steps_per_launch is not None:
    op.tune(steps_per_launch=a.steps_per_launch)
  elif a.physics == "linear":
    op.tune(steps_per_launch=4)
  dt = mesh.cfl_dt()
  snaps = op.new_field(a.nsteps + 1)
  op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
  # limited plans: the forward's decision record, read back by the adjoint (as AdaptiveSweep)
  rec = (torch.zeros(a.nsteps * op.ktot, dtype=torch.int16, device=op.device)
         if op.limiter else None)
  op.forward(snaps[0], 0.0, dt, a.nsteps, snaps, decisions=rec)
  w = op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
  u = op.new_field()
  jumps = None
  if a.what.endswith("_rec"):  # the jump-record sweeps (their own default shape)
    jumps = op.new_jumps(a.nsteps)
    op.forward_rec(snaps[0], 0.0, dt, a.nsteps, jumps, out=u)
  for _ in range(a.reps + 1):
    if a.what == "fwd_rec":
      op.forward_rec(snaps[0], 0.0, dt, a.nsteps, jumps, out=u)
    elif a.what == "adj_rec":
      w.copy_(u)
      op.adjoint_rec(w, jumps, 0.0, dt, a.nsteps, eta=eta)
    elif a.what == "fwd_nosnap":
      u.copy_(snaps[0])
      op.forward(u, 0.0, dt, a.nsteps)
    elif a.what == "fwd":
      op.forward(snaps[0], 0.0, dt, a.nsteps, snaps, decisions=rec)
    else:
      w.copy_(snaps[a.nsteps])
      op.adjoint(w, snaps, 0.0, dt, a.nsteps, eta=eta, decisions=rec)
  torch.cuda.synchronize()
  print("ok", a.what, a.physics, "uniform" if op.uniform else "nonuniform")


if __name__ == "__main__":
  main()
