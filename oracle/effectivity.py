"""Effectivity of the DG-advection dual-weighted-residual indicator.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): a CPU study, never on the product path.

The reference prints, next to its DWR sum, the functional differences it estimates
(matlab/MAIN.m:55-76: J(u_H) - J(u_h) and J(u_H) - J(u) against sum(err_con1)).  This module
asks the same of the advection indicator the kernels compute, on a problem with a known exact
solution (u0 a bump inside (0, 1), zero inflow: u(x, t) = u0(x - a t)), for a
mesh-independent LINEAR functional, a smooth window average of the final state:

  J(u) = int_0^1 psi(x) u(x, T) dx,  J_h(u_h) = g . u_h^N,  g_k = (h_k/2) int phi_i psi

(g, exact by Gauss quadrature, is the adjoint's terminal weight: dg_lserk4_adj takes any
terminal weight; the bench uses J = |u^N|^2/2).  A linear J makes the DWR identity exact (a
quadratic one such as 1/2 int u^2 is conserved by the central-flux scheme, so its error is
second order in the state error and no first-order estimate can track it).

Two indicators:
* "jump" -- the kernels' indicator (dg_lserk4_adj, include/dg_advec.h): eta_k = sum_n dt
  w^{n+1}_k . R(u^{n+1})_k with R = LIFT (Fscale .* du) the interelement-jump part of
  AdvecRHS1D (utils/AdvecRHS1D.m:19), paired with the same-order discrete adjoint.
* "p" -- the p-prolonged residual variant of SURVEY 8(a) row 8 (the pattern of
  matlab/MAIN.m:33-34, which marches the adjoint at order Ns+1, and of errEst,
  python/Main_finite_difference.py:79-94, res[n] = u_f[n] - Phi(u_f[n-1])): prolong the
  order-N states to order N+1 (interpolation, exact for the polynomials), take the one-step
  residual of the order-(N+1) scheme R^n = P u^{n+1} - S_{N+1}(P u^n), and pair it with the
  order-(N+1) discrete adjoint: eta_k = -sum_n w_{N+1}^{n+1} . R^n on element k.  For the
  linear scheme e^{n+1} = S e^n - R^n (e = u_{N+1} - P u_h, e^0 = 0), so sum_k eta_k =
  g . e^N = J_{N+1}(u_{N+1}) - J_{N+1}(P u_h) exactly (J linear).

The per-element yardstick for ranking: the gain |J(u_split_k) - J(u_h)| of refining element
k alone (the greedy refinement the loop performs), every split run with one common dt.
"""
import numpy as np

from .adjoint import adjoint_step
from .advec import INFLOW_ZERO, forward_sweep, lift_residual, step
from .setup1d import jacobi_gq, startup1d, vandermonde1d


def window(x, c=0.62, w=0.08):
  """psi: a smooth bump of half-width w around c (the functional's weight)."""
  z = (x - c) / w
  return np.where(np.abs(z) < 1, np.cos(0.5 * np.pi * z) ** 4, 0.0)


def weight(S, psi=window, nq=12):
  """g_k,i = (h_k/2) int_{-1}^{1} l_i(r) psi(x_k(r)) dr by nq-point Gauss quadrature."""
  rq, wq = jacobi_gq(0, 0, nq - 1)
  Lq = vandermonde1d(S["N"], rq) @ S["invV"]  # l_i(r_q), (nq, Np)
  VX = S["VX"]
  h = np.diff(VX)
  xq = VX[:-1][None, :] + (0.5 * (rq + 1))[:, None] * h[None, :]  # (nq, K)
  return (h / 2.0)[None, :] * (Lq.T @ (wq[:, None] * psi(xq)))


def functional(u, S, g=None):
  """J_h(u) = g . u: the window average of the DG polynomial (quadrature-exact)."""
  g = weight(S) if g is None else g
  return float(np.sum(g * u))


def exact_functional(u0_fn, shift, psi=window):
  """int psi(x) u0(x - shift) dx by Gauss quadrature on 400 panels."""
  r, w = jacobi_gq(0, 0, 20)
  edges = np.linspace(0.0, 1.0, 401)
  tot = 0.0
  for a, b in zip(edges[:-1], edges[1:]):
    x = a + (r + 1) * (b - a) / 2
    tot += np.sum(w * psi(x) * u0_fn(x - shift)) * (b - a) / 2
  return tot


def prolong_matrix(S_lo, S_hi):
  """Interpolation of order-N element polynomials to the order-(N+1) LGL nodes."""
  return vandermonde1d(S_lo["N"], S_hi["r"]) @ S_lo["invV"]


def adjoint_weights(snaps, g, dt, a, S):
  """Discrete adjoint states w^0..w^N of the step map (terminal weight g, no source)."""
  nsteps = len(snaps) - 1
  ws = [None] * (nsteps + 1)
  w = g.copy()
  ws[nsteps] = w
  for n in range(nsteps - 1, -1, -1):
    w = adjoint_step(w, dt, a, S)
    ws[n] = w
  return ws


def jump_indicator(snaps, times, dt, a, S, inflow=INFLOW_ZERO):
  """The kernels' indicator for the functional J_h (terminal weight gradient(u^N))."""
  ws = adjoint_weights(snaps, weight(S), dt, a, S)
  eta = np.zeros(S["K"])
  for n in range(len(snaps) - 1):
    R = lift_residual(snaps[n + 1], times[n + 1], a, S, inflow)
    eta += dt * np.sum(ws[n + 1] * R, axis=0)
  return eta


def p_estimate(snaps, times, dt, a, S, S_hi, g_hi, inflow=INFLOW_ZERO):
  """The p-prolonged residual estimate for the terminal weight g_hi (order N+1): the CPU
  statement of dg_lserk4_adj_p (include/dg_advec.h).  Per step n (MAIN.m:32-34 marches the
  adjoint at order Ns+1; adj_march.m:117 pairs it with the residual; errEst's
  res[n] = u_f[n] - Phi(u_f[n-1]), Main_finite_difference.py:79-94):
    R^n = P u^{n+1} - S_{N+1}(P u^n, t_n),   eta_k -= w^{n+1}_k . R^n_k.
  Returns (eta, w^0) with w^0 the order-(N+1) adjoint at t_0."""
  P = prolong_matrix(S, S_hi)
  ps = [P @ u for u in snaps]
  ws = adjoint_weights(ps, g_hi, dt, a, S_hi)  # the linear adjoint needs no states
  eta = np.zeros(S["K"])
  for n in range(len(snaps) - 1):
    R = ps[n + 1] - step(ps[n], times[n], dt, a, S_hi, inflow)
    eta -= np.sum(ws[n + 1] * R, axis=0)
  return eta, ws[0]


def p_indicator(snaps, times, dt, a, S, S_hi, inflow=INFLOW_ZERO):
  """The p-prolonged residual variant (order N+1 residual and adjoint) for the window
  functional, and the order-(N+1) solution's functional for reference.
  Returns (eta, J_{N+1}(u_{N+1}))."""
  P = prolong_matrix(S, S_hi)
  hi_snaps, _ = forward_sweep(P @ snaps[0], times[0], dt, len(snaps) - 1, a, S_hi, inflow)
  eta, _ = p_estimate(snaps, times, dt, a, S, S_hi, weight(S_hi), inflow)
  return eta, functional(hi_snaps[-1], S_hi)


def split_mesh(VX, k):
  """Split element k at its midpoint (MAIN.m:137-141 / Main_finite_difference.py:336-341)."""
  return np.insert(VX, k + 1, 0.5 * (VX[k] + VX[k + 1]))


def study(N, K, T, u0_fn, a=2 * np.pi, cfl=0.75, gains=True):
  """Effectivities of both indicators and their agreement with the per-element refinement
  gains on a uniform K-element mesh.  One dt for every solve (the CFL step of the finest mesh
  involved: the order-(N+1) nodes of a split element), nsteps = ceil(T/dt)."""
  VX = np.linspace(0.0, 1.0, K + 1)
  S = startup1d(N, VX, metric="element")
  S_hi = startup1d(N + 1, VX, metric="element")
  S_fine = startup1d(N, np.linspace(0.0, 1.0, 2 * K + 1), metric="element")
  r = S_hi["r"]
  gap = min(np.min(np.diff(r)), np.min(np.diff(S["r"])))
  dt = 0.5 * cfl / a * (0.5 / K) * gap / 2  # split element: h/2; LGL gap in reference units
  nsteps = int(np.ceil(T / dt))
  dt = T / nsteps

  def solve(Sx):
    u0 = u0_fn(Sx["x"])
    snaps, times = forward_sweep(u0, 0.0, dt, nsteps, a, Sx, INFLOW_ZERO)
    return snaps, times

  snaps, times = solve(S)
  J_h = functional(snaps[-1], S)
  J_exact = exact_functional(u0_fn, a * T)
  J_fine = functional(solve(S_fine)[0][-1], S_fine)
  eta_j = jump_indicator(snaps, times, dt, a, S)
  eta_p, J_hi = p_indicator(snaps, times, dt, a, S, S_hi)
  out = dict(N=N, K=K, T=T, dt=dt, nsteps=nsteps, J_h=J_h, J_exact=J_exact, J_h2=J_fine,
             J_p1=J_hi,
             err_exact=J_exact - J_h, err_h2=J_fine - J_h, err_p1=J_hi - J_h,
             sum_eta_jump=float(eta_j.sum()), sum_eta_p=float(eta_p.sum()))
  for k in ("exact", "h2", "p1"):
    e = out["err_" + k]
    out["effectivity_jump_vs_" + k] = out["sum_eta_jump"] / e if e != 0 else None
    out["effectivity_p_vs_" + k] = out["sum_eta_p"] / e if e != 0 else None
  out["eta_jump"] = eta_j
  out["eta_p"] = eta_p
  if gains:
    g = np.zeros(K)
    for k in range(K):
      Sk = startup1d(N, split_mesh(VX, k), metric="element")
      g[k] = abs(functional(solve(Sk)[0][-1], Sk) - J_h)
    out["gain"] = g
    for name, eta in (("jump", eta_j), ("p", eta_p)):
      out["spearman_" + name] = spearman(np.abs(eta), g)
      out["argmax_" + name] = int(np.argmax(np.abs(eta)))
      out["top5_overlap_" + name] = len(set(np.argsort(-np.abs(eta))[:5])
                                        & set(np.argsort(-g)[:5]))
    out["argmax_gain"] = int(np.argmax(g))
  return out


def spearman(x, y):
  """Spearman rank correlation (average ranks on ties)."""
  def ranks(v):
    order = np.argsort(v, kind="mergesort")
    rk = np.empty(len(v))
    rk[order] = np.arange(len(v), dtype=float)
    for val in np.unique(v):  # average ties
      m = v == val
      if m.sum() > 1:
        rk[m] = rk[m].mean()
    return rk
  rx, ry = ranks(np.asarray(x)), ranks(np.asarray(y))
  rx -= rx.mean()
  ry -= ry.mean()
  den = np.sqrt(np.sum(rx * rx) * np.sum(ry * ry))
  return float(np.sum(rx * ry) / den) if den > 0 else 0.0
