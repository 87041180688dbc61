"""Diagnostic: how the config-2 bench step evolves from a cold start.

Runs the bench step (forward sweep + adjoint sweep + argmax) --steps times with no warm-up,
recording HIP-event times of every step, then idles --idle seconds and runs --after more
steps, and prints one JSON line with the per-step series (forward sweep, adjoint sweep,
whole step, in microseconds) and the host time since the first launch.

  python profiles/ramp_probe.py [--steps 400] [--idle 1.0] [--after 60]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--steps", type=int, default=400)
  p.add_argument("--idle", type=float, default=1.0)
  p.add_argument("--after", type=int, default=60)
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--K", type=int, default=1 << 20)
  p.add_argument("--nsteps", type=int, default=20)
  a = p.parse_args()
  import torch
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  ens = pkg.ensemble
  dev = torch.device("cuda", 0)
  mesh = pkg.BaseGalerkin1D(n=a.N, k=a.K, domain=[0.0, 1.0])
  sweep = ens.EnsembleSweep(mesh, [0], a.nsteps, mesh.cfl_dt(),
                            params=(np.array([1.0]), np.array([1.0]), np.array([0.0])))
  st = torch.cuda.current_stream(dev)
  torch.cuda.synchronize()

  def run(n):
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n)]
    t_host = []
    t0 = time.perf_counter()
    for s in range(n):
      evs[s][0].record(st)
      sweep.forward()
      evs[s][1].record(st)
      sweep.eta.zero_()
      evs[s][2].record(st)
      sweep.run_adjoint()
      evs[s][3].record(st)
      sweep.op.argmax_async(sweep.eta)
      t_host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    fwd = [e[0].elapsed_time(e[1]) * 1e3 for e in evs]
    adj = [e[2].elapsed_time(e[3]) * 1e3 for e in evs]
    step = [evs[i][0].elapsed_time(evs[i + 1][0]) * 1e3 for i in range(n - 1)]
    return {"fwd_us": fwd, "adj_us": adj, "step_us": step, "host_s": t_host}

  cold = run(a.steps)
  time.sleep(a.idle)
  after = run(a.after)
  out = {"N": a.N, "K": a.K, "nsteps": a.nsteps, "cold": cold, "idle_s": a.idle, "after_idle": after}
  for name, r in (("cold", cold), ("after_idle", after)):
    f, d = np.array(r["fwd_us"]), np.array(r["adj_us"])
    print(f"[{name}] fwd sweep us: first5 {np.round(f[:5], 1).tolist()} "
          f"med {np.median(f):.1f} last {f[-1]:.1f}; adj: first5 {np.round(d[:5], 1).tolist()} "
          f"med {np.median(d):.1f} last {d[-1]:.1f}", file=sys.stderr)
    if len(f) >= 50:
      blocks = [float(np.mean(f[i:i + 10] + d[i:i + 10])) for i in range(0, len(f), 10)]
      print(f"[{name}] fwd+adj mean per 10-step block: {np.round(blocks, 1).tolist()}",
            file=sys.stderr)
  print(json.dumps(out))


if __name__ == "__main__":
  main()
