"""Batched DG-in-time adaptivity for ensembles of the scalar ODE du/dt = sin(u):
the matlab/MAIN.m loop (dg_march -> adj_march -> refine the slab with the largest
|err|) with every ensemble member (initial value y0) advanced by the HIP kernels of
csrc/dg_time.hip, one lane per member.

Host side (numpy) builds the reference-element operators fem_setup.m builds per slab —
they depend only on the order and the Gauss rule, so they are computed once:
  forward, order N:   S = (V V')\\Dr, Phi (nodal basis at the 30N+1 Gauss points), w
  adjoint, order N+1: S_a = inv(V V')*Dr, M_a = inv(V V'), Phi_a (2(N+1)+1 Gauss points),
                      Pext (order-N basis where adj_march.m:79 evaluates u_h),
                      Ifa  (order-N basis at the adjoint nodes, adj_march.m:78)
The device work per iteration is one forward and one adjoint launch; the per-member
indicators are summed over the ensemble in fixed order (dg_sum_rows) and the split
follows MAIN.m:137-141 with the first index on ties.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .galerkin import BaseGalerkin1D


def _ref(n):
  """Reference-element pieces of order n (LGL nodes, V, Dr) via BaseGalerkin1D's
  StartUp1D restatement (a 2-element mesh: the reference element does not depend on it)."""
  g = BaseGalerkin1D(n=n, k=2)
  return g, g.r_gl, g.v, g.d_r


def basis_at(n, xi):
  """Nodal (LGL, order n) basis functions evaluated at reference points xi: the Phi of
  fem_setup.m:30-38 (Phi = P(xi)^T inv(V))."""
  g, r, V, _ = _ref(n)
  P = g.vandermonde1D(n, np.asarray(xi, dtype=np.float64))
  return P @ np.linalg.inv(V)


def forward_ops(n):
  g, r, V, Dr = _ref(n)
  rq, wq = g.jacobiGQ(0, 0, 30 * n)  # dg_march.m:38 -> fem_setup(Ns, 1, tk, 30 Ns)
  S = np.linalg.solve(V @ V.T, Dr)  # dg_march.m:57
  return dict(n=n, S=S, Phi=basis_at(n, rq), wq=wq, rq=rq)


def adjoint_ops(n_fwd):
  na = n_fwd + 1
  g, r, V, Dr = _ref(na)
  rq, wq = g.jacobiGQ(0, 0, 2 * na)  # adj_march.m:71 -> fem_setup(Ns, 1, tspan, 2 Ns)
  Minv = np.linalg.inv(V @ V.T)
  return dict(n=na, Sa=Minv @ Dr, Ma=Minv, Phia=basis_at(na, rq), wq=wq,
              # adj_march.m:73,79: hk = x(1) - x(end) < 0, so r_interp = t_a + (1+r) hk/2
              # sits at reference coordinate -2 - r of the forward slab
              Pext=basis_at(n_fwd, -2.0 - rq),
              Ifa=basis_at(n_fwd, r))


def refine(times, err_total):
  """MAIN.m:137-141 (first index on ties)."""
  ref_i = int(np.argmax(np.abs(err_total)))
  times = np.asarray(times, dtype=np.float64)
  out = np.empty(times.size + 1)
  out[:ref_i + 1] = times[:ref_i + 1]
  out[ref_i + 2:] = times[ref_i + 1:]
  out[ref_i + 1] = np.mean(times[[ref_i, ref_i + 1]])
  return out, ref_i


class DGTimeEnsemble:
  """MAIN.m's DG-in-time adaptivity for an ensemble of initial values on one slab mesh."""

  def __init__(self, n, times, y0, device=None, tol=1e-7, maxit=500):
    if not torch.cuda.is_available():
      raise _lib.DGLibraryError("DGTimeEnsemble needs a ROCm GPU (torch.cuda is unavailable)")
    self.n = int(n)
    self.dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    self.times = np.asarray(times, dtype=np.float64).copy()
    self.y0 = torch.as_tensor(np.asarray(y0, dtype=np.float64), device=self.dev).contiguous()
    self.n_ics = int(self.y0.numel())
    self.tol, self.maxit = float(tol), int(maxit)
    self._lib = _lib.load()
    f, a = forward_ops(self.n), adjoint_ops(self.n)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64,  # noqa: E731
                                  device=self.dev)
    self.f = {k: t(v) for k, v in f.items() if isinstance(v, np.ndarray)}
    self.a = {k: t(v) for k, v in a.items() if isinstance(v, np.ndarray)}
    self.nq_f, self.nq_a = f["wq"].size, a["wq"].size
    self.history = []

  @property
  def n_slabs(self):
    return self.times.size - 1

  def _s(self):
    return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

  @staticmethod
  def _p(x):
    return ctypes.c_void_p(x.data_ptr())

  def march(self, times_dev=None):
    """Forward march (dg_march.m): Y [n_slabs, n+1, n_ics], Newton iterations."""
    Ks, Np = self.n_slabs, self.n + 1
    td = torch.as_tensor(self.times, device=self.dev) if times_dev is None else times_dev
    Y = torch.empty((Ks, Np, self.n_ics), dtype=torch.float64, device=self.dev)
    its = torch.empty((Ks, self.n_ics), dtype=torch.int32, device=self.dev)
    rc = self._lib.dg_time_march(Np, self.nq_f, self._p(self.f["S"]), self._p(self.f["Phi"]),
                                 self._p(self.f["wq"]), Ks, self._p(td), self.n_ics,
                                 self._p(self.y0), self.tol, self.maxit, self._p(Y),
                                 self._p(its), self._s())
    _lib.check(rc, "dg_time_march")
    return Y, its, td

  def adjoint(self, Y, times_dev):
    """Adjoint march + DWR indicator (adj_march.m): V [n_slabs, n+2, n_ics], err [n_ics, n_slabs]."""
    Ks, Npf = self.n_slabs, self.n + 1
    V = torch.empty((Ks, Npf + 1, self.n_ics), dtype=torch.float64, device=self.dev)
    err = torch.empty((self.n_ics, Ks), dtype=torch.float64, device=self.dev)
    a = self.a
    rc = self._lib.dg_time_adjoint(Npf, self.nq_a, self._p(a["Sa"]), self._p(a["Ma"]),
                                   self._p(a["Phia"]), self._p(a["Pext"]), self._p(a["Ifa"]),
                                   self._p(a["wq"]), Ks, self._p(times_dev), self.n_ics,
                                   self._p(self.y0), self._p(Y), self._p(V), self._p(err),
                                   self._s())
    _lib.check(rc, "dg_time_adjoint")
    return V, err

  def indicator(self, err):
    """Per-slab indicator: sum over the ensemble, in member order (dg_sum_rows), of each
    member's |err| -- MAIN.m:137 refines by |err| of its one trajectory, and the ensemble
    path takes that magnitude per member before combining (Main_width_ref.py:139,479 and
    FDEnsemble do the same), so opposite-signed members never cancel."""
    from .operators import sum_rows
    return sum_rows(err.abs().contiguous(), self.n_ics)

  def adapt(self):
    """One MAIN.m iteration: march, adjoint, indicator, split.  Returns the refined slab."""
    Y, its, td = self.march()
    V, err = self.adjoint(Y, td)
    total = self.indicator(err).cpu().numpy()
    self.times, ref_i = refine(self.times, total)
    self.history.append(dict(ref_i=ref_i, err=total, iters=int(its.max().item())))
    return ref_i
