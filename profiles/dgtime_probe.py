"""Throughput of the batched DG-in-time marches (dgtime.DGTimeEnsemble): one forward and
one adjoint march of n_ics ensemble members over n_slabs slabs, timed with HIP events.

  python profiles/dgtime_probe.py [--N 1] [--ics 1048576] [--slabs 64] [--reps 5]

Unit: member-slab updates per second (one Newton-converged forward slab, or one adjoint
slab solve with its indicator, for one member)."""
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
  p.add_argument("--N", type=int, default=1)
  p.add_argument("--ics", type=int, default=1 << 20)
  p.add_argument("--slabs", type=int, default=64)
  p.add_argument("--reps", type=int, default=5)
  a = p.parse_args()
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  rng = np.random.default_rng(0)
  y0 = rng.uniform(0.2, 2.8, a.ics)
  times = np.linspace(0.0, 2.0, a.slabs + 1)
  ens = pkg.dgtime.DGTimeEnsemble(a.N, times, y0)
  Y, its, td = ens.march()  # warm-up
  ens.adjoint(Y, td)
  torch.cuda.synchronize()
  st = torch.cuda.current_stream()
  tf, ta = [], []
  for _ in range(a.reps):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record(st)
    Y, its, td = ens.march()
    e[1].record(st)
    ens.adjoint(Y, td)
    e[2].record(st)
    torch.cuda.synchronize()
    tf.append(e[0].elapsed_time(e[1]) * 1e-3)
    ta.append(e[1].elapsed_time(e[2]) * 1e-3)
  units = a.ics * a.slabs
  print(json.dumps({"N": a.N, "ics": a.ics, "slabs": a.slabs,
                    "newton_iters_max": int(its.max().item()),
                    "newton_iters_mean": float(its.float().mean().item()),
                    "fwd_s": float(np.median(tf)), "adj_s": float(np.median(ta)),
                    "fwd_member_slabs_per_s": units / float(np.median(tf)),
                    "adj_member_slabs_per_s": units / float(np.median(ta))}))


if __name__ == "__main__":
  main()
