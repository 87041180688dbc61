"""The finite-difference DWR adapt loop of python/Main_finite_difference.py for ensembles of
du/dt = sin(u) (J = int u^2, ref_factor-refined adjoint), one ensemble member per lane on the
device (csrc/dg_fd.hip).

Per iteration: ``forwardSolve`` (:34-51), ``adjSolve`` (:54-76, the bidiagonal
(J_F^T - I) v = -K solved as its backward recursion), ``errEst`` (:79-94), the windowed
|err| sums (:270-277) — all per member on the device — then the member sum in fixed order
(dg_sum_rows) and the reference's split ``ref_idx = argmax + 1`` (:336-341) on the host.
With one member and u0 = 1 this is the reference's own __main__ loop, pinned by
tests/golden/fd_adapt_golden.json.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def refine_all(dt_n, ref_factor):
  """Main_finite_difference.py:16-21."""
  n_steps = len(dt_n) * ref_factor
  dt_fine = np.zeros(n_steps)
  for f in range(ref_factor):
    dt_fine[f:n_steps - ref_factor + f + 1:ref_factor] = dt_n / ref_factor
  return dt_fine, n_steps


def interp_codes(t_coarse, t_fine):
  """Where np.interp(t_fine, t_coarse, .) takes each value from (compiled_base.c arr_interp):
  code j >= 0 interpolates in interval j, code -(j+1) returns node j exactly."""
  j = np.searchsorted(t_coarse, t_fine, side="right") - 1
  j = np.clip(j, 0, t_coarse.size - 1)
  exact = (j == t_coarse.size - 1) | (t_coarse[j] == t_fine)
  return np.where(exact, -(j + 1), j).astype(np.int32)


def split_step(times, err_steps):
  """Main_finite_difference.py:336-341: ref_idx = argmax + 1, insert the midpoint."""
  n_steps = len(times) - 1
  times_new = np.zeros(n_steps + 2)
  ref_idx = int(np.argmax(err_steps) + 1)
  times_new[0:ref_idx] = times[0:ref_idx]
  times_new[ref_idx + 1:] = times[ref_idx:]
  times_new[ref_idx] = np.mean(times[ref_idx - 1:ref_idx + 1])
  return times_new, ref_idx


class FDEnsemble:
  """Main_finite_difference.py's adapt loop for an ensemble of initial values."""

  def __init__(self, times, u0, ref_factor=4, device=None):
    if not torch.cuda.is_available():
      raise _lib.DGLibraryError("FDEnsemble needs a ROCm GPU (torch.cuda is unavailable)")
    self.dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    self.times = np.asarray(times, dtype=np.float64).copy()
    self.rf = int(ref_factor)
    self.u0 = torch.as_tensor(np.asarray(u0, dtype=np.float64).ravel(), device=self.dev)
    self.n_ics = int(self.u0.numel())
    self._lib = _lib.load()
    self.history = []

  def sweep(self, with_v=False):
    """One forward + adjoint + indicator sweep on the current grid for every member.
    Returns U [n+1, n_ics], V [n*rf+1, n_ics] (or None), err_steps [n_ics, n]."""
    dt_n = np.diff(self.times, 1)
    n = dt_n.size
    dt_fine, nf = refine_all(dt_n, self.rf)
    t_coarse = np.concatenate(([0], np.cumsum(dt_n)), axis=None)  # interpU (:27-28)
    t_fine = np.concatenate(([0], np.cumsum(dt_fine)), axis=None)
    t = lambda x, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(x), dtype=dt,  # noqa: E731
                                                    device=self.dev)
    dtd, tcd, tfd = t(dt_n), t(t_coarse), t(t_fine)
    codes = t(interp_codes(t_coarse, t_fine), torch.int32)
    U = torch.empty((n + 1, self.n_ics), dtype=torch.float64, device=self.dev)
    V = torch.empty((nf + 1, self.n_ics), dtype=torch.float64, device=self.dev) if with_v else None
    err = torch.empty((self.n_ics, n), dtype=torch.float64, device=self.dev)
    p = lambda x: ctypes.c_void_p(x.data_ptr()) if x is not None else None  # noqa: E731
    rc = self._lib.dg_fd_adapt_sweep(n, self.rf, p(dtd), p(tcd), p(tfd), p(codes), p(self.u0),
                                     self.n_ics, p(U), p(V), p(err),
                                     ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
    _lib.check(rc, "dg_fd_adapt_sweep")
    return U, V, err

  def adapt(self):
    """One iteration of the __main__ loop (:263-343): sweep, member sum, split."""
    from .operators import sum_rows
    U, _, err = self.sweep()
    total = sum_rows(err.contiguous(), self.n_ics).cpu().numpy()
    self.times, ref_idx = split_step(self.times, total)
    self.history.append(dict(ref_idx=ref_idx, err_steps=total))
    return ref_idx
