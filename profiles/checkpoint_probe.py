"""Cost of the checkpointed adjoint (checkpoint.CheckpointedSweep) against full snapshot
storage, for one config-2 trajectory (N=4, K=2^20) and long sweeps, timed with HIP events.

  python profiles/checkpoint_probe.py [--K 1048576] [--steps 64 256] [--every 0 4 8 16]

every = 0 is the full-storage sweep (nsteps + 1 fields).  Reported per case: device fields
held, sweep time (forward + adjoint), DOF-updates/s counted as the full-storage sweep
counts them (2 Np K nsteps: the recomputed forward steps are overhead, not work)."""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
  st = torch.cuda.current_stream()
  fn()
  torch.cuda.synchronize()
  ts = []
  for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    fn()
    e1.record(st)
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e-3)
  return float(np.median(ts))


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--K", type=int, default=1 << 20)
  p.add_argument("--steps", type=int, nargs="+", default=[64, 256])
  p.add_argument("--every", type=int, nargs="+", default=[0, 4, 8, 16])
  p.add_argument("--reps", type=int, default=5)
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  N = 4
  mesh = pkg.BaseGalerkin1D(n=N, k=a.K)
  op = pkg.operators.DGAdvection1D(mesh)
  h = 1.0 / a.K
  dt = 0.5 * 0.75 / (2 * np.pi) * h * (mesh.r_gl[1] - mesh.r_gl[0]) / 2  # One_code.mlx:111
  u0 = op.init_sine(np.ones(1), np.ones(1), np.zeros(1))
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
  w = op.new_field()
  for nsteps in a.steps:
    units = 2.0 * op.Np * a.K * nsteps
    for every in a.every:
      if every == 0:
        snaps = op.new_field(nsteps + 1)
        u = u0.clone()

        def run():
          u.copy_(u0)
          op.forward(u, 0.0, dt, nsteps, snaps)
          w.copy_(u)
          op.adjoint(w, snaps, 0.0, dt, nsteps, eta=eta)
        fields = nsteps + 1
      else:
        sweep = pkg.checkpoint.CheckpointedSweep(op, nsteps, every)
        u = u0.clone()

        def run():
          u.copy_(u0)
          sweep.forward(u, 0.0, dt)
          w.copy_(u)
          sweep.adjoint(w, eta=eta)
        fields = sweep.fields
      t = timed(run, a.reps)
      print(json.dumps({"K": a.K, "N": N, "nsteps": nsteps, "every": every or None,
                        "fields": fields, "field_MB": op.field_numel * 8 / 1e6,
                        "sweep_s": t, "dof_updates_per_s": units / t}), flush=True)
      del run
      if every == 0:
        del snaps
      else:
        del sweep
      torch.cuda.empty_cache()


if __name__ == "__main__":
  main()
