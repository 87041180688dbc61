"""Throughput of the FD ensemble sweep (fd_ensemble.FDEnsemble.sweep, one dg_fd_adapt_sweep
launch): forward Euler on the coarse grid, the adjoint recursion on the ref_factor-refined
grid and the windowed DWR sums, for n_ics members, timed with HIP events.

  python profiles/fd_probe.py [--ics 1048576] [--steps 64] [--rf 4] [--reps 5]

Unit: member fine-steps per second (one fine adjoint step with its residual, per member).
Algorithmic bytes per member: U written once and read back (8 B per coarse node each way),
err_steps written once (8 B per coarse step); the kernel is bound by the fp64 sin/cos and
the correctly rounded division of np.interp, not by HBM."""
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
  p.add_argument("--ics", type=int, default=1 << 20)
  p.add_argument("--steps", type=int, default=64)
  p.add_argument("--rf", type=int, default=4)
  p.add_argument("--reps", type=int, default=5)
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  rng = np.random.default_rng(0)
  u0 = rng.uniform(0.2, 2.8, a.ics)
  times = np.linspace(0.0, 2.0, a.steps + 1)
  ens = pkg.fd_ensemble.FDEnsemble(times, u0, ref_factor=a.rf)
  ens.sweep()  # warm-up
  torch.cuda.synchronize()
  st = torch.cuda.current_stream()
  ts = []
  for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    ens.sweep()
    e1.record(st)
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e-3)
  t = float(np.median(ts))
  units = a.ics * a.steps * a.rf
  hbm = a.ics * (16.0 * (a.steps + 1) + 8.0 * a.steps)
  print(json.dumps({"ics": a.ics, "coarse_steps": a.steps, "ref_factor": a.rf, "sweep_s": t,
                    "member_fine_steps_per_s": units / t, "algorithmic_GBs": hbm / t / 1e9}))


if __name__ == "__main__":
  main()
