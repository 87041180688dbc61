"""Checkpointed sweeps on the GPU (checkpoint.CheckpointedSweep) against the full-storage
sweep of the same plan, and through it against the oracle.  Needs an MI355X.

Tolerances: the checkpointed forward state, dJ/du^0 and the DWR indicator within
RTOL = 1e-12 of the full-storage sweep (they differ only where a segment boundary moves
a launch boundary or the node-0 source), and the indicator within 1e-10 of the oracle
(north_star); argmax indices exact.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu

A = 2 * np.pi


def rel_err(x, ref):
  x, ref = np.asarray(x), np.asarray(ref)
  return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-300))


def host(t):
  return t.detach().cpu().numpy()


def setup(pkg, N, K, **kw):
  _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  S = setup1d.startup1d(N, v_x, metric="element")
  return S, pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), **kw)


def both_sweeps(pkg, op, u0, w0, t0, dt, nsteps, every, src):
  import torch
  u = u0.clone()
  snaps = op.new_field(nsteps + 1)
  op.forward(u, t0, dt, nsteps, snaps)
  w, eta = w0.clone(), torch.zeros(op.ktot, dtype=torch.float64, device=u0.device)
  op.adjoint(w, snaps, t0, dt, nsteps, src_coef=src, eta=eta)
  sweep = pkg.checkpoint.CheckpointedSweep(op, nsteps, every)
  uc = u0.clone()
  sweep.forward(uc, t0, dt)
  wc, etac = w0.clone(), torch.zeros_like(eta)
  sweep.adjoint(wc, src_coef=src, eta=etac)
  torch.cuda.synchronize()
  return (u, w, eta, snaps), (uc, wc, etac, sweep)


@pytest.mark.parametrize("nsteps,every", [(13, None), (13, 1), (16, 4), (16, 8), (21, 5),
                                          (9, 100)])
def test_linear_checkpointed_equals_full_storage(pkg, gpu, nsteps, every):
  import torch
  S, op = setup(pkg, 4, 900)
  dt = oadv.bench_dt(S)
  x = torch.tensor(setup1d.to_elem_major(S["x"]), device=gpu)
  u0 = torch.sin(2 * np.pi * x) + 0.2 * torch.cos(10 * np.pi * x)
  w0 = torch.cos(4 * np.pi * x)
  (u, w, eta, snaps), (uc, wc, etac, sweep) = both_sweeps(pkg, op, u0, w0, 0.01, dt, nsteps,
                                                          every, 0.3)
  assert rel_err(host(uc), host(u)) <= 1e-12
  assert rel_err(host(wc), host(w)) <= 1e-12
  assert rel_err(host(etac), host(eta)) <= 1e-12
  for c, (s, _) in enumerate(sweep.segments):
    assert rel_err(host(sweep.checkpoints[c]), host(snaps[s])) <= 1e-12
  assert op.argmax(etac) == op.argmax(eta)
  assert sweep.fields < nsteps + 1 or every in (1, 100)


def test_linear_checkpointed_indicator_matches_oracle(pkg, gpu):
  import torch
  N, K, nsteps = 3, 400, 12
  S, op = setup(pkg, N, K)
  dt = oadv.bench_dt(S)
  # a rough state, so that the jump residual is O(1) and not a cancellation-limited
  # difference (for smooth states the parity tests feed the oracle the GPU's snapshots)
  rng = np.random.default_rng(11)
  u0 = rng.standard_normal(S["x"].shape)
  g = rng.standard_normal(S["x"].shape)
  sweep = pkg.checkpoint.CheckpointedSweep(op, nsteps, 4)
  u = torch.tensor(setup1d.to_elem_major(u0), device=gpu)
  sweep.forward(u, 0.0, dt)
  w = torch.tensor(setup1d.to_elem_major(g), device=gpu)
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  sweep.adjoint(w, src_coef=0.5, eta=eta)
  # the oracle's adjoint over the oracle's own forward states
  ref, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  w_ref, eta_ref, _ = oadj.adjoint_sweep(g, ref, times, dt, A, S, src_coef=0.5)
  assert rel_err(setup1d.from_elem_major(host(u), N + 1), ref[-1]) <= 1e-10
  assert rel_err(setup1d.from_elem_major(host(w), N + 1), w_ref) <= 1e-10
  assert rel_err(host(eta), eta_ref) <= 1e-10
  assert op.argmax(eta) == int(np.argmax(np.abs(eta_ref)))


@pytest.mark.parametrize("flux,limiter", [("burgers", True), ("linear", True),
                                          ("burgers", "1")])
def test_config3_checkpointed_equals_full_storage(pkg, gpu, flux, limiter):
  import torch
  S, op = setup(pkg, 4, 700, flux=flux, limiter=limiter)
  dt = 0.5 * oadv.bench_dt(S)
  x = torch.tensor(setup1d.to_elem_major(S["x"]), device=gpu)
  u0 = torch.sin(2 * np.pi * x) + 0.8 * (x > 0.5)
  w0 = u0.clone()
  (u, w, eta, _), (uc, wc, etac, _) = both_sweeps(pkg, op, u0, w0, 0.0, dt, 11, 3, 0.2)
  assert rel_err(host(uc), host(u)) <= 1e-12
  assert rel_err(host(wc), host(w)) <= 1e-12
  assert rel_err(host(etac), host(eta)) <= 1e-12
  assert op.argmax(etac) == op.argmax(eta)
