"""How many of the config-3 adjoint's narrow-cone tiles (236 outputs, 10-element halo) hold
a troubled cell, per step, in the bench's refine loop (bench.py --config 3 workload)."""
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
N, K, nsteps = 4, 1 << 22, 20
mesh = pkg.BaseGalerkin1D(n=N, k=K, domain=[0.0, 1.0])
run = pkg.adaptive.AdaptiveSweep(mesh, nsteps, 8, flux="burgers", limiter=True)
for it in range(3):
  run.iterate()
run.forward()
torch.cuda.synchronize()
k = run.op.ktot
codes = run.decisions().cpu().numpy().reshape(nsteps, k)
te = 236
nt = -(-k // te)
for n in range(0, nsteps, 4):
  nz = np.nonzero(codes[n])[0]
  tiles = set()
  for e in nz:
    for t in ((e + 10) // te, (e - 10) // te, e // te):
      if 0 <= t < nt and t * te - 10 <= e < t * te + te + 10:
        tiles.add(t)
  print(f"step {n}: troubled cells {len(nz)}, troubled tiles {len(tiles)} of {nt}",
        "cells at", nz[:8], flush=True)
