"""BASELINE config 1 at its own size on the GPU: K = 64, N = 4, forward Euler (the
Main_finite_difference.py:131-132 update), 50 steps, forward + adjoint with the reference's
quadratic functional pattern (getK = 2 u dt, Main_finite_difference.py:225-227), against the
oracle's reverse sweep; and the adjoint against the monolithic (J_F^T - I) v = -K solve of
Main_finite_difference.py:73 at a reduced step count (the dense system has (nsteps+1) * 320
unknowns).  VERDICT r02 item 5d.  Needs an MI355X.

dt is a tenth of the LSERK4 bench step: forward Euler with the central flux is unstable
(SURVEY §7), and at the full CFL step 50 steps would amplify the high modes' rounding by ~1e7,
so the two implementations' last-bit differences would exceed the 1e-10 bar by themselves.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu

RTOL = 1e-10
A = 2 * np.pi


def rel_err(x, ref):
  return float(np.max(np.abs(np.asarray(x) - ref)) / np.max(np.abs(ref)))


def host(t):
  return t.detach().cpu().numpy()


def run(pkg, gpu, nsteps):
  import torch
  N, K = 4, 64
  S = setup1d.uniform_setup(N, K, metric="element")
  op = pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=N, k=K), time_scheme="euler")
  dt = 0.1 * oadv.bench_dt(S)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.05 * np.random.default_rng(1).standard_normal(S["x"].shape)
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(torch.tensor(setup1d.to_elem_major(u0), device=gpu))
  op.forward(snaps[0], 0.0, dt, nsteps, snaps)
  g = 2 * dt * snaps[nsteps].clone()  # J = dt sum_n |u^n|^2: terminal 2 dt u^N, source 2 dt u^n
  w = g.clone()
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, 0.0, dt, nsteps, src_coef=2 * dt, eta=eta)
  torch.cuda.synchronize()
  gs = [setup1d.from_elem_major(host(snaps[n]), N + 1) for n in range(nsteps + 1)]
  return S, dt, u0, gs, setup1d.from_elem_major(host(g), N + 1), \
      setup1d.from_elem_major(host(w), N + 1), host(eta)


def test_config1_forward_and_adjoint(pkg, gpu):
  S, dt, u0, gs, g, w0, eta = run(pkg, gpu, 50)
  ref, times = oadv.forward_sweep(u0, 0.0, dt, 50, A, S, scheme="euler")
  assert rel_err(gs[-1], ref[-1]) <= RTOL
  w_ref, eta_ref, _ = oadj.adjoint_sweep(g, gs, times, dt, A, S, src_coef=2 * dt,
                                         scheme="euler")
  assert rel_err(w0, w_ref) <= RTOL
  assert rel_err(eta, eta_ref) <= RTOL


def test_config1_adjoint_is_the_monolithic_solve(pkg, gpu):
  nsteps = 5
  S, dt, _, gs, g, w0, _ = run(pkg, gpu, nsteps)
  v = oadj.monolithic_adjoint(gs, dt, A, S, 2 * dt, g, scheme="euler")
  assert rel_err(w0, v[0]) <= RTOL
