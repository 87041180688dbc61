"""Discrete adjoint and dual-weighted residual of the DG advection step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference has no advection adjoint (adjoint_sens.m is empty,
err_contribution.m is symbolic).  The build defines it with the reference's own
patterns and this module restates that definition independently of the kernels:

* discrete adjoint = exact transpose of the fully discrete forward map, the
  ``(J_F^T - I) v = -K`` system of python/Main_finite_difference.py:54-76 solved
  backwards step by step (``adjoint_sweep``) or monolithically (``monolithic_adjoint``);
* the transposed spatial operator is assembled here by scatter-adding through the
  MATLAB connectivity maps (vmapM/vmapP, BuildMaps1D.m) — a different formulation from
  the kernel's per-element face exchange;
* indicator = adjoint-weighted residual ``err = res * v`` of
  python/Main_finite_difference.py:79-94, with res the interelement-jump residual
  LIFT*(Fscale.*du) of AdvecRHS1D.m:19 at t_{n+1}, paired with v^{n+1} and summed over
  nodes of each element and over steps (dt-weighted): eta_k.
"""
import numpy as np

from .advec import INFLOW_A, INFLOW_ZERO, face_jumps, inflow_value, lift_residual, step
from .setup1d import RK4A, RK4B


def advec_linear(u, a, S):
  """The linear part L u of AdvecRHS1D (inflow value 0)."""
  du = face_jumps(u, 0.0, a, S)
  return -a * S["rx"] * (S["Dr"] @ u) + S["LIFT"] @ (S["Fscale"] * du)


def advec_linear_T(w, a, S):
  """L^T w by scatter-add through vmapM/vmapP (independent of the kernel's formulation)."""
  Np, K = S["Np"], S["K"]
  nxf = S["nx"].ravel(order="F")
  c = a * nxf / 2  # (a*nx - (1-alpha)|a nx|)/2 with alpha = 1
  z = (S["Fscale"] * (S["LIFT"].T @ w)).ravel(order="F")  # 2K face weights
  coef = c * z
  coef[S["mapO"]] = 0.0  # du(mapO) = 0
  out = (S["Dr"].T @ (-a * S["rx"] * w)).ravel(order="F")
  vmapM, vmapP = S["vmapM"], S["vmapP"]
  np.add.at(out, vmapM, coef)
  interior = np.ones(2 * K, dtype=bool)
  interior[S["mapI"]] = False  # du(mapI) = c*(u(vmapI) - uin): no neighbour term
  interior[S["mapO"]] = False
  np.add.at(out, vmapP[interior], -coef[interior])
  return out.reshape(Np, K, order="F")


def adjoint_step(w_next, dt, a, S, scheme="lserk4"):
  """Reverse of one forward step: for s = last..0: lr += B_s lu; lu += dt L^T lr; lr = A_s lr."""
  if scheme == "lserk4":
    A, B = RK4A, RK4B
  else:
    A, B = np.array([0.0]), np.array([1.0])
  lu = w_next.copy()
  lr = np.zeros_like(lu)
  for s in reversed(range(len(A))):
    lr = lr + B[s] * lu
    lu = lu + dt * advec_linear_T(lr, a, S)
    lr = A[s] * lr
  return lu


def adjoint_sweep(wT, snaps, times, dt, a, S, inflow=INFLOW_A, src_coef=0.0, scheme="lserk4",
                  with_eta=True):
  """Backward sweep n = nsteps-1..0 (see include/dg_advec.h dg_lserk4_adj):
     w^{n+1} += src*u^{n+1} (not at n+1 = nsteps); eta += dt*sum_i w^{n+1} R(u^{n+1}, t_{n+1});
     w^n = S^T w^{n+1};  finally w^0 += src*u^0.
  Returns (w^0, eta (K,), list of adjoint states w^0..w^N)."""
  nsteps = len(snaps) - 1
  K = S["K"]
  eta = np.zeros(K)
  w = wT.copy()
  states = [None] * (nsteps + 1)
  for n in range(nsteps - 1, -1, -1):
    if n != nsteps - 1:
      w = w + src_coef * snaps[n + 1]
    states[n + 1] = w
    if with_eta:
      R = lift_residual(snaps[n + 1], times[n + 1], a, S, inflow)
      eta = eta + dt * np.sum(w * R, axis=0)
    w = adjoint_step(w, dt, a, S, scheme)
  w = w + src_coef * snaps[0]
  states[0] = w
  return w, eta, states


def functional(snaps, dt, src_coef, g):
  """J(u) = <g, u^N> + (src/2) * sum_{n=0}^{N-1} |u^n|^2 — the functional whose gradient the
  sweep returns (terminal weight g; left-endpoint source, cf. getK of
  python/Main_finite_difference.py:225-227)."""
  J = float(np.sum(g * snaps[-1]))
  for u in snaps[:-1]:
    J += 0.5 * src_coef * float(np.sum(u * u))
  return J


def dense_operator(fn, shape):
  """Assemble the matrix of a linear map on (Np, K) fields (element-major ordering)."""
  Np, K = shape
  n = Np * K
  M = np.zeros((n, n))
  for j in range(n):
    e = np.zeros(n)
    e[j] = 1.0
    M[:, j] = fn(e.reshape(Np, K, order="F")).ravel(order="F")
  return M


def step_matrix(dt, a, S, scheme="lserk4"):
  """The homogeneous part of one forward step (inflow forcing removed) as a dense matrix."""
  Np, K = S["Np"], S["K"]

  def lin_step(u):
    return step(u, 0.0, dt, a, S, INFLOW_ZERO, scheme)  # inflow forcing removed

  return dense_operator(lin_step, (Np, K))


def monolithic_adjoint(snaps, dt, a, S, src_coef, g, scheme="lserk4"):
  """Solve (J_F^T - I) v = -K for all time levels at once (python/Main_finite_difference.py:73)
  with J_F the block-subdiagonal Jacobian of the step map and K = dJ/dU."""
  nsteps = len(snaps) - 1
  Np, K = S["Np"], S["K"]
  n = Np * K
  Sm = step_matrix(dt, a, S, scheme)
  JF = np.zeros(((nsteps + 1) * n, (nsteps + 1) * n))
  for m in range(1, nsteps + 1):
    JF[m * n:(m + 1) * n, (m - 1) * n:m * n] = Sm
  Kvec = np.zeros((nsteps + 1) * n)
  for m in range(nsteps):
    Kvec[m * n:(m + 1) * n] = src_coef * snaps[m].ravel(order="F")
  Kvec[nsteps * n:] += g.ravel(order="F")
  v = np.linalg.solve(JF.T - np.eye(JF.shape[0]), -Kvec)
  return [v[m * n:(m + 1) * n].reshape(Np, K, order="F") for m in range(nsteps + 1)]


def sum_rows(x):
  """Fixed-order row sum (ascending row index) — dg_sum_rows."""
  x = np.asarray(x)
  acc = x[0].copy()
  for r in range(1, x.shape[0]):
    acc = acc + x[r]
  return acc


def ensemble_indicator(rows):
  """The ensemble refine indicator: the mean over ICs of each IC's |eta| (the reference's
  errorIndicator returns jnp.abs(err) per IC, python/Main_width_ref.py:139; the mean over
  ICs is :479, the refine index its argmax + 1, :491), summed in IC order."""
  rows = np.asarray(rows)
  return sum_rows(np.abs(rows)) / float(rows.shape[0])


def argmax(x, use_abs=False):
  """numpy.argmax semantics (first index on ties, NaN is maximal) — dg_argmax."""
  x = np.asarray(x)
  return int(np.argmax(np.abs(x) if use_abs else x))
