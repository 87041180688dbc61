"""Nonlinear (Burgers-type) flux with SlopeLimitN after every LSERK4 stage: BASELINE
config 3 / SURVEY §8(f)1, restated on the CPU with its tangent and discrete adjoint.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference never runs a nonlinear DG problem: SURVEY §8d leaves the flux
build-defined ("e.g. Burgers u^2/2 with the same central-flux structure").  The build
defines it as

* flux f(u) = a*u^2/2 collocated at the nodes, and AdvecRHS1D's central-flux structure
  (utils/AdvecRHS1D.m:9-19, alpha = 1) applied to f instead of a*u:
      rhsu = -rx.*(Dr*f) + LIFT*(Fscale.*du),   du = nx.*(f(u^-) - f(u^+))/2,
  inflow f(uin) at x = 0 with the same uin(t) variants, du = 0 at the outflow face.
  For the linear flux f = a*u this is exactly AdvecRHS1D.
* the LSERK4 stage loop of utils/One_code.mlx:120-137 with ``u = SlopeLimitN(u)``
  (utils/SlopeLimitN.m:1-33) after every stage's update.

Adjoint (build-defined): the exact transpose of the tangent of one limited step with the
limiter's discrete decisions (troubled-cell set, SlopeLimitN.m:23, and the active
minmod argument, minmod.m:10, first index on ties) frozen at the forward state — the
derivative of the step wherever those decisions are locally constant.  This module
forms the tangent (``step_jvp``) by forward differentiation of each stage, and the
transpose by assembling the step Jacobian from column-coloured tangents
(``step_vjp``): a formulation independent of the kernels' hand-transposed stages.

Indicator: eta_k += dt * sum_i w^{n+1}_{k,i} R_i(u^{n+1}, t_{n+1}) with R the
interelement-jump residual LIFT*(Fscale.*du) of the nonlinear RHS (the linear path's
definition, oracle/adjoint.py, with f in place of a*u).
"""
import numpy as np

from .advec import INFLOW_A, face_jumps, inflow_value
from .limiter import _row_dot, cell_average, minmod, slope_limit_1, slope_limit_n
from .setup1d import RK4A, RK4B, RK4C

FLUX_LINEAR = "linear"
FLUX_BURGERS = "burgers"


def flux(u, kind):
  """Nodal flux divided by a: u (linear) or u^2/2 (Burgers)."""
  return 0.5 * u * u if kind == FLUX_BURGERS else u


def flux_jumps(u, uin, a, S, kind):
  """du of the central flux on f: face_jumps applied to f(u) with inflow f(uin)
  (AdvecRHS1D.m:9-16 with a*u -> a*f(u))."""
  return face_jumps(flux(u, kind), flux(uin, kind), a, S)


def rhs(u, t, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A):
  """rhsu = -a*rx.*(Dr*f) + LIFT*(Fscale.*du)  (AdvecRHS1D.m:19 with u -> f(u))."""
  f = flux(u, kind)
  du = flux_jumps(u, inflow_value(a, t, inflow), a, S, kind)
  return -a * S["rx"] * (S["Dr"] @ f) + S["LIFT"] @ (S["Fscale"] * du), du


def jump_residual(u, t, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A):
  """The interelement-jump residual LIFT*(Fscale.*du) of the nonlinear RHS."""
  du = flux_jumps(u, inflow_value(a, t, inflow), a, S, kind)
  return S["LIFT"] @ (S["Fscale"] * du)


def rhs_tangent(u, du, a, S, kind=FLUX_BURGERS):
  """d rhs = L (f'(u) du): the homogeneous operator on the flux perturbation."""
  df = u * du if kind == FLUX_BURGERS else du
  dfj = face_jumps(df, 0.0, a, S)
  return -a * S["rx"] * (S["Dr"] @ df) + S["LIFT"] @ (S["Fscale"] * dfj)


# ---------------------------------------------------------------------------
# Limited LSERK4 step
# ---------------------------------------------------------------------------
def _limit(v, S, limit):
  """The stage limiter: limit True / "N" = SlopeLimitN (troubled cells only), "1" =
  SlopeLimit1 (utils/SlopeLimit1.m: every cell).  Returns (u, limited cell indices)."""
  if limit == "1":
    return slope_limit_1(v, S), np.arange(v.shape[1])
  return slope_limit_n(v, S, return_ids=True)


def limited_step(u, time, dt, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A, limit=True,
                 return_ids=False):
  """One LSERK4 step (One_code.mlx:120-137) with u = SlopeLimitN(u) (limit True or "N") or
  u = SlopeLimit1(u) (limit "1") after every stage.
  return_ids: also the list of the 5 limited-cell index arrays."""
  resu = np.zeros_like(u)
  ids_all = []
  for s in range(5):
    rhsu, _ = rhs(u, time + RK4C[s] * dt, a, S, kind, inflow)
    resu = RK4A[s] * resu + dt * rhsu
    v = u + RK4B[s] * resu
    if limit:
      u, ids = _limit(v, S, limit)
      ids_all.append(ids)
    else:
      u = v
  return (u, ids_all) if return_ids else u


def forward_sweep(u0, t0, dt, nsteps, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A, limit=True):
  """nsteps limited steps from t0 (time = time + dt, One_code.mlx:139): snapshots, times."""
  snaps, times = [u0.copy()], [t0]
  u, time = u0.copy(), t0
  for _ in range(nsteps):
    u = limited_step(u, time, dt, a, S, kind, inflow, limit)
    time = time + dt
    snaps.append(u)
    times.append(time)
  return snaps, times


# ---------------------------------------------------------------------------
# Tangent (frozen limiter decisions)
# ---------------------------------------------------------------------------
def _neighbours(v):
  K = v.shape[0]
  return np.concatenate(([v[0]], v[:K - 1])), np.concatenate((v[1:], [v[K - 1]]))  # :18


def slope_limit_n_jvp(v, dv, S, limit=True):
  """(SlopeLimitN(v), its derivative applied to dv) with the troubled-cell set and the
  active minmod argument frozen at v (first index on ties, as minmod's min).  limit "1":
  the same for SlopeLimit1 (every cell limited)."""
  y, ids = _limit(v, S, limit)
  dy = dv.copy()
  if ids.size == 0:
    return y, dy
  avg, uh0 = cell_average(v, S)
  davg, duh0 = cell_average(dv, S)
  vm, vp = _neighbours(avg)
  dvm, dvp = _neighbours(davg)
  V, Np = S["V"], S["Np"]
  xl = S["x"][:, ids]
  h = xl[Np - 1, :] - xl[0, :]  # SlopeLimitLin.m:10
  x0 = xl[0, :] + h / 2  # :11
  uh1 = _row_dot(S["invV"][1, :], v[:, ids])
  ul = V[:, 0:1] * uh0[None, ids] + V[:, 1:2] * uh1[None, :]
  args = np.vstack(((2.0 / h) * _row_dot(S["Dr"][0, :], ul),
                    (vp[ids] - avg[ids]) / h, (avg[ids] - vm[ids]) / h))  # :16-18
  duh1 = _row_dot(S["invV"][1, :], dv[:, ids])
  dul = V[:, 0:1] * duh0[None, ids] + V[:, 1:2] * duh1[None, :]
  dargs = np.vstack(((2.0 / h) * _row_dot(S["Dr"][0, :], dul),
                     (dvp[ids] - davg[ids]) / h, (davg[ids] - dvm[ids]) / h))
  s = np.sum(np.sign(args), 0) / 3.0
  active = np.abs(s) == 1  # minmod.m:9
  branch = np.argmin(np.abs(args), axis=0)
  dm = np.where(active, dargs[branch, np.arange(ids.size)], 0.0)
  m = minmod(args)
  assert np.array_equal(y[:, ids], avg[None, ids] + (xl - x0[None, :]) * m[None, :])
  dy[:, ids] = davg[None, ids] + (xl - x0[None, :]) * dm[None, :]
  return y, dy


def step_jvp(u, du, time, dt, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A, limit=True):
  """(step(u), d step(u)[du]) of ``limited_step``."""
  resu = np.zeros_like(u)
  dres = np.zeros_like(u)
  for s in range(5):
    rhsu, _ = rhs(u, time + RK4C[s] * dt, a, S, kind, inflow)
    drhs = rhs_tangent(u, du, a, S, kind)
    resu = RK4A[s] * resu + dt * rhsu
    dres = RK4A[s] * dres + dt * drhs
    v = u + RK4B[s] * resu
    dv = du + RK4B[s] * dres
    if limit:
      u, du = slope_limit_n_jvp(v, dv, S, limit)
    else:
      u, du = v, dv
  return u, du


def step_vjp(u, w, time, dt, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A, limit=True):
  """J^T w for the step Jacobian J = d step(u)/du, assembled from coloured tangents.

  One stage couples elements k-2..k+2 (face fluxes, then the limiter's neighbour
  averages), so a step couples k-10..k+10 (k-5..k+5 unlimited): seeding every P-th
  element (P = 2*reach + 1) with one node's unit vector gives columns with disjoint row
  supports, and (J^T w)[j] = sum over j's support of (J e_j) * w."""
  Np, K = u.shape
  reach = 10 if limit else 5
  P = min(2 * reach + 1, K)
  out = np.zeros_like(u)
  for c in range(P):
    cols = np.arange(c, K, P)
    for p in range(Np):
      seed = np.zeros_like(u)
      seed[p, cols] = 1.0
      _, d = step_jvp(u, seed, time, dt, a, S, kind, inflow, limit)
      prod = np.sum(d * w, axis=0)  # per element
      for k in cols:
        lo, hi = max(0, k - reach), min(K, k + reach + 1)
        out[p, k] = np.sum(prod[lo:hi])
  return out


def step_matrix(u, time, dt, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A, limit=True):
  """Dense step Jacobian (element-major ordering) for tiny meshes."""
  Np, K = u.shape
  n = Np * K
  M = np.zeros((n, n))
  for j in range(n):
    e = np.zeros(n)
    e[j] = 1.0
    _, d = step_jvp(u, e.reshape(K, Np).T, time, dt, a, S, kind, inflow, limit)
    M[:, j] = d.T.ravel()
  return M


def adjoint_sweep(wT, snaps, times, dt, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A,
                  limit=True, src_coef=0.0, with_eta=True):
  """Backward sweep n = nsteps-1..0 (include/dg_advec.h dg_lserk4_adj):
     w^{n+1} += src*u^{n+1} (not at n+1 = nsteps); eta += dt*sum_i w^{n+1} R(u^{n+1}, t_{n+1});
     w^n = J_n^T w^{n+1} with J_n linearised at u^n;  finally w^0 += src*u^0.
  Returns (w^0, eta (K,), list of adjoint states w^0..w^N)."""
  nsteps = len(snaps) - 1
  eta = np.zeros(S["K"])
  w = wT.copy()
  states = [None] * (nsteps + 1)
  for n in range(nsteps - 1, -1, -1):
    if n != nsteps - 1:
      w = w + src_coef * snaps[n + 1]
    states[n + 1] = w
    if with_eta:
      R = jump_residual(snaps[n + 1], times[n + 1], a, S, kind, inflow)
      eta = eta + dt * np.sum(w * R, axis=0)
    w = step_vjp(snaps[n], w, times[n], dt, a, S, kind, inflow, limit)
  w = w + src_coef * snaps[0]
  states[0] = w
  return w, eta, states


def limiter_stage_ids(u0, t0, dt, nsteps, a, S, kind=FLUX_BURGERS, inflow=INFLOW_A):
  """Troubled-cell counts per stage of a limited sweep (diagnostics for the tests)."""
  counts = []
  u, time = u0.copy(), t0
  for _ in range(nsteps):
    u, ids = limited_step(u, time, dt, a, S, kind, inflow, True, return_ids=True)
    counts.append([int(i.size) for i in ids])
    time = time + dt
  return counts
