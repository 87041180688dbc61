"""DG-in-time forward march, adjoint march and DWR indicator for the scalar ODE
du/dt = sin(u): the nonlinear branches of matlab/dg_march.m, matlab/adj_march.m and
matlab/fem_setup.m, driven as in matlab/MAIN.m.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restated line by line; MATLAB/Octave
is not available, and the reference records no outputs of these routines, so the
restatement is pinned by identities (complex-step Jacobian check of matlab/test_jacobian.m,
convergence to the exact solution) — "parity unpinned" by reference-produced values.

Two behaviours of the reference are kept as written:
* polyfit/polyval in the monomial basis evaluate the slab polynomial (dg_march.m:49-51,
  adj_march.m:75-79);
* adj_march.m:73 sets hk = x(1) - x(end) < 0, so its quadrature points
  r_interp = t_a + (1+r) hk/2 (adj_march.m:78) lie in [t_a - h, t_a], before the slab, and
  the mass terms carry the negative hk.
"""
import math

import numpy as np

from . import setup1d


def fem_setup(n, tspan, n_gq):
  """matlab/fem_setup.m:1-43 for one element (K = 1) on tspan, order n, n_gq+1 Gauss points.
  Returns the globals the marches read: x, V, Dr, Np, r (Gauss points), w, Phi."""
  S = setup1d.startup1d(n, np.asarray(tspan, dtype=float), metric="matlab")
  r, w = setup1d.jacobi_gq(0, 0, n_gq)  # fem_setup.m:27 (overwrites r)
  Np = n + 1
  invVT = np.linalg.inv(S["V"].T)
  Phi = np.zeros((r.size, Np))
  for k in range(r.size):  # :31-38
    for i in range(Np):
      p = [invVT[i, nn] * setup1d.jacobi_p(np.array([r[k]]), 0, 0, nn)[0] for nn in range(Np)]
      Phi[k, i] = np.sum(p)
  return dict(x=S["x"][:, 0].copy(), V=S["V"], Dr=S["Dr"], Np=Np, r=r, w=w, Phi=Phi)


def _newton_parts(st, U, uR_prev):
  """R(U), dR/dU of dg_march.m:47-63 for the slab set up in st."""
  x, V, Dr, Np, r, w, Phi = (st[k] for k in ("x", "V", "Dr", "Np", "r", "w", "Phi"))
  N = Np - 1
  hk = x[-1] - x[0]  # dg_march.m:33
  pu = np.polyfit(x, U, N)  # :49
  x_interp = x[0] + (1 + r) * hk / 2  # :50
  ur = np.polyval(pu, x_interp)  # :51
  wfu = w * np.sin(ur)  # :53
  wdf = np.diag(w * np.cos(ur))  # :54
  M_tilde = hk / 2 * (Phi.T @ wfu)  # :55
  dMtdU = hk / 2 * (Phi.T @ wdf @ Phi)  # :56
  S = np.linalg.solve(V @ V.T, Dr)  # :57
  B = np.zeros((Np, Np))
  B[-1, -1] = -1.0  # :58
  F = np.zeros(Np, dtype=np.result_type(U, float))
  F[0] = uR_prev  # :59
  A = S.T + B  # :61
  return A @ U + M_tilde + F, A + dMtdU  # :64, :62


def dg_march(N, times, y0, tol=1e-7, maxit=500):
  """matlab/dg_march.m:36-77 (nonlinear branch), uniform order N on every slab.
  Returns (t, y, iterations): node times and nodal values per slab."""
  Ks = len(times) - 1
  t, y, its = [], [], []
  uR_prev = float(y0)
  for k in range(Ks):
    st = fem_setup(N, times[k:k + 2], 30 * N)  # :38
    U_old = uR_prev * np.ones(N + 1)  # :46
    it, err = 0, 1.0
    U_next = U_old
    while it <= maxit and err > tol:  # :53
      R, J = _newton_parts(st, U_old, uR_prev)
      delta = np.linalg.solve(J, R)  # :65
      U_next = U_old - delta  # :66
      err = float(np.linalg.norm(U_old - U_next))  # :67
      U_old = U_next
      it += 1
    uR_prev = U_next[-1]  # :75
    y.append(U_next)
    t.append(st["x"])
    its.append(it)
  return t, y, its


def adj_march(Na, times, y1, t1, y0=1.0):
  """matlab/adj_march.m:61-119 (nonlinear branch; J = integral of u, F = M_k*1 at :96).
  Na is the adjoint order (MAIN.m:34 calls it with Ns+1); y1/t1 the forward march.
  Returns (t, v, err)."""
  Ks = len(times) - 1
  t, v, err = [None] * Ks, [None] * Ks, np.zeros(Ks)
  vL_prev = 0.0
  for k in range(Ks - 1, -1, -1):
    U_k = y1[k]
    tk = t1[k]
    st = fem_setup(Na, [tk[0], tk[-1]], 2 * Na)  # :71
    x, V, Dr, Np, r, w, Phi = (st[kk] for kk in ("x", "V", "Dr", "Np", "r", "w", "Phi"))
    hk = x[0] - x[-1]  # :73 (negative)
    pu = np.polyfit(tk, U_k, Na - 1)  # :76
    uh_k = np.polyval(pu, x)  # :78
    r_interp = tk[0] + (1 + r) * hk / 2  # :79
    ur_k = np.polyval(pu, r_interp)  # :80
    w_tilde = np.diag(w * np.cos(ur_k))  # :82
    M_v = hk / 2 * (Phi.T @ w_tilde @ Phi)  # :83
    M_k = hk / 2 * np.linalg.inv(V @ V.T)  # :84
    S = np.linalg.inv(V @ V.T) @ Dr  # :85
    B = np.zeros((Np, Np))
    B[0, 0] = -1.0  # :86
    A = -S.T + B - M_v  # :87
    F = M_k @ np.ones(Np)  # :96
    F[-1] = F[-1] - vL_prev
    v_k = np.linalg.solve(A, F)  # :98
    v[k] = v_k
    vL_prev = v_k[0]  # :100
    t[k] = x
    wfu = w * np.sin(ur_k)  # :104
    M_tilde = hk / 2 * (Phi.T @ wfu)  # :105
    S = np.linalg.solve(V @ V.T, Dr)  # :106
    B = np.zeros((Np, Np))
    B[-1, -1] = -1.0  # :107
    F = np.zeros(Np)
    F[0] = y0 if k == 0 else y1[k - 1][-1]  # :108-113
    A = -S.T - B  # :115
    err[k] = v_k @ (-A @ uh_k - M_tilde + F)  # :117
  return t, v, err


def refine(times, err):
  """matlab/MAIN.m:137-141: split the slab with the largest |err| (first index on ties:
  MATLAB's find would return every tie)."""
  ref_i = int(np.argmax(np.abs(err)))
  times = np.asarray(times, dtype=float)
  out = np.zeros(times.size + 1)
  out[:ref_i + 1] = times[:ref_i + 1]
  out[ref_i + 2:] = times[ref_i + 1:]
  out[ref_i + 1] = np.mean(times[[ref_i, ref_i + 1]])
  return out, ref_i


def exact(t, y0=1.0):
  """du/dt = sin(u), u(0) = y0: u = 2 atan(tan(y0/2) e^t) (MAIN.m:13-15 dsolve)."""
  return 2 * np.arctan(math.tan(y0 / 2) * np.exp(np.asarray(t, dtype=float)))
