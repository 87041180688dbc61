"""Host logic of the checkpointed sweep (checkpoint.CheckpointedSweep), no GPU.

A stand-in operator with the library's calling contract (include/dg_advec.h:
dg_lserk4_fwd snapshot/alias rules, dg_lserk4_adj source and indicator order, time levels
by repeated addition) runs a small time-dependent linear map on CPU tensors.  The
checkpointed composition must then reproduce the full-storage sweep bit for bit: same
states, same w, same eta, for every segment length.
"""
import numpy as np
import pytest
import torch

from conftest import load_pkg

ck = load_pkg().checkpoint


class LinearStandIn:
  """u^{n+1} = A u^n + sin(t_n) b;  eta += dt * w^{n+1} * (u^{n+1})^2 (an elementwise
  'residual'); w^n = A^T w^{n+1}; source w^{n+1} += src u^{n+1} for n+1 < N and
  w^0 += src u^0 — the dg_lserk4_adj order."""

  def __init__(self, F=7, seed=0):
    g = torch.Generator().manual_seed(seed)
    self.A = torch.randn(F, F, generator=g, dtype=torch.float64) / F
    self.b = torch.randn(F, generator=g, dtype=torch.float64)
    self.F = F
    self.calls = []

  def new_field(self, count=None):
    shape = (self.F,) if count is None else (count, self.F)
    return torch.empty(shape, dtype=torch.float64)

  def forward(self, u, t0, dt, nsteps, snapshots=None):
    self.calls.append(("fwd", t0, nsteps))
    tn = ck.step_times(t0, dt, nsteps)
    alias = snapshots is not None and snapshots[0].data_ptr() == u.data_ptr()
    x = u.clone()
    if snapshots is not None and not alias:
      snapshots[0].copy_(x)
    for n in range(nsteps):
      x = self.A @ x + np.sin(tn[n]) * self.b
      if snapshots is not None:
        snapshots[n + 1].copy_(x)
    if not alias:
      u.copy_(x)
    return u

  def adjoint(self, w, snapshots, t0, dt, nsteps, src_coef=0.0, eta=None):
    self.calls.append(("adj", t0, nsteps))
    assert snapshots.shape[0] == nsteps + 1
    for n in range(nsteps - 1, -1, -1):
      if n + 1 < nsteps:
        w += src_coef * snapshots[n + 1]
      if eta is not None:
        eta += dt * w * snapshots[n + 1] ** 2
      w.copy_(self.A.T @ w)
    w += src_coef * snapshots[0]
    return w, eta


def full_sweep(op, u0, w0, t0, dt, nsteps, src):
  u = u0.clone()
  snaps = op.new_field(nsteps + 1)
  op.forward(u, t0, dt, nsteps, snaps)
  w, eta = w0.clone(), torch.zeros(op.F, dtype=torch.float64)
  op.adjoint(w, snaps, t0, dt, nsteps, src_coef=src, eta=eta)
  return u, w, eta


@pytest.mark.parametrize("nsteps", [1, 5, 12, 13])
@pytest.mark.parametrize("every", [None, 1, 2, 4, 5, 100])
def test_checkpointed_sweep_reproduces_full_storage(nsteps, every):
  op = LinearStandIn()
  g = torch.Generator().manual_seed(nsteps)
  u0 = torch.randn(op.F, generator=g, dtype=torch.float64)
  w0 = torch.randn(op.F, generator=g, dtype=torch.float64)
  t0, dt, src = 0.1, 0.037, 0.7
  u_ref, w_ref, eta_ref = full_sweep(op, u0, w0, t0, dt, nsteps, src)

  sweep = ck.CheckpointedSweep(op, nsteps, every)
  u = u0.clone()
  sweep.forward(u, t0, dt)
  w, eta = w0.clone(), torch.zeros(op.F, dtype=torch.float64)
  sweep.adjoint(w, src_coef=src, eta=eta)
  assert torch.equal(u, u_ref)
  assert torch.equal(w, w_ref)
  assert torch.equal(eta, eta_ref)
  # a second adjoint (the last segment is no longer resident) gives the same again
  w2, eta2 = w0.clone(), torch.zeros(op.F, dtype=torch.float64)
  sweep.adjoint(w2, src_coef=src, eta=eta2)
  assert torch.equal(w2, w_ref) and torch.equal(eta2, eta_ref)


def test_segments_times_and_recompute_count():
  op = LinearStandIn()
  sweep = ck.CheckpointedSweep(op, 10, 4)
  assert sweep.segments == [(0, 4), (4, 8), (8, 10)]
  assert sweep.fields == 3 + 5 == ck.CheckpointedSweep.fields_needed(10, 4)
  u = torch.ones(op.F, dtype=torch.float64)
  op.calls.clear()
  sweep.forward(u, 0.5, 0.1)
  sweep.adjoint(torch.ones(op.F, dtype=torch.float64))
  t = ck.step_times(0.5, 0.1, 10)
  # the forward's segments, then backwards: last segment resident, the others recomputed
  assert op.calls == [("fwd", t[0], 4), ("fwd", t[4], 4), ("fwd", t[8], 2),
                      ("adj", t[8], 2), ("fwd", t[4], 4), ("adj", t[4], 4),
                      ("fwd", t[0], 4), ("adj", t[0], 4)]


def test_default_segment_minimises_memory():
  for n in (16, 100, 1000):
    sweep = ck.CheckpointedSweep(LinearStandIn(F=2), n)
    assert sweep.fields <= 2 * int(np.ceil(np.sqrt(n))) + 1 < n + 1


def test_adjoint_needs_forward():
  sweep = ck.CheckpointedSweep(LinearStandIn(), 4, 2)
  with pytest.raises(RuntimeError):
    sweep.adjoint(torch.zeros(7, dtype=torch.float64))
  with pytest.raises(ValueError):
    ck.CheckpointedSweep(LinearStandIn(), 0)


def test_adjoint_refuses_w_in_the_scratch():
  op = LinearStandIn()
  sweep = ck.CheckpointedSweep(op, 4, 2)
  sweep.forward(torch.ones(op.F, dtype=torch.float64), 0.0, 0.1)
  with pytest.raises(ValueError):
    sweep.adjoint(sweep.scratch[2])
