"""CPU timings of the config-1 case and of the FD oracle ("also time the FD
oracle's functions for config 1").  Test infrastructure: the oracle is the checker, and
this only reports how long its pieces take on the host, one thread.

  python profiles/cpu_config1.py  ->  one JSON line

Config 1: K = 64, N = 4, forward Euler (u += dt rhs), 50 steps; its discrete adjoint by the
reverse sweep and by the monolithic (J_F^T - I) v = -K solve of Main_finite_difference.py:73.
FD oracle: Main_finite_difference.py's loop (du/dt = sin u, J = int u^2, ref_factor 4),
12 iterations from 2 steps (the golden run's configuration).
"""
import json
import os
import sys
import time

import numpy as np
from threadpoolctl import threadpool_limits

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import adjoint as oadj  # noqa: E402
from oracle import advec as oadv  # noqa: E402
from oracle import fd as ofd  # noqa: E402
from oracle import setup1d  # noqa: E402


def best_of(fn, reps=5):
  ts = []
  for _ in range(reps):
    t0 = time.perf_counter()
    fn()
    ts.append(time.perf_counter() - t0)
  return min(ts)


def main():
  out = {}
  with threadpool_limits(1):
    S = setup1d.uniform_setup(4, 64, metric="element")
    a = 2 * np.pi
    dt = 0.1 * oadv.bench_dt(S)
    u0 = np.sin(2 * np.pi * S["x"])
    nsteps = 50
    snaps, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, a, S, scheme="euler")
    g = snaps[-1].copy()
    out["config1_forward_euler_s"] = best_of(
        lambda: oadv.forward_sweep(u0, 0.0, dt, nsteps, a, S, scheme="euler"))
    out["config1_adjoint_reverse_sweep_s"] = best_of(
        lambda: oadj.adjoint_sweep(g, snaps, times, dt, a, S, scheme="euler"))
    out["config1_adjoint_monolithic_s"] = best_of(
        lambda: oadj.monolithic_adjoint(snaps, dt, a, S, 0.0, g, scheme="euler"), reps=1)
    out["config1_dof_updates"] = 2 * 5 * 64 * nsteps
    out["fd_adapt_12_iterations_s"] = best_of(
        lambda: ofd.adapt_loop(np.linspace(0.0, 2.0, 3), 1.0, 4, 12), reps=3)
  out["threads"] = 1
  print(json.dumps(out))


if __name__ == "__main__":
  main()
