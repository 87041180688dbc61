"""Restatement of the finite-difference DWR adapt loop.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Follows
python/Main_finite_difference.py line by line; pinned to the reference's own outputs
in tests/golden/fd_adapt_golden.json (bit-exact refine indices, <=1e-12 floats).
"""
import numpy as np


def refine_all(dt_n, ref_factor):
  """Main_finite_difference.py:16-21."""
  n_steps = len(dt_n) * ref_factor
  dt_fine = np.zeros(n_steps)
  for f in range(ref_factor):
    dt_fine[f:n_steps - ref_factor + f + 1:ref_factor] = dt_n / ref_factor
  return dt_fine, n_steps


def interp_u(dt_n, u, ref_factor):
  """Main_finite_difference.py:24-31 (its ref_factor module global made explicit)."""
  dt_fine, _ = refine_all(dt_n, ref_factor)
  t_coarse = np.concatenate(([0], np.cumsum(dt_n)), axis=None)
  t_fine = np.concatenate(([0], np.cumsum(dt_fine)), axis=None)
  return np.interp(t_fine, t_coarse, u)


def forward_solve(update, dt_n, u0):
  """Main_finite_difference.py:34-51."""
  u = np.zeros(len(dt_n) + 1)
  u[0] = u0
  for n in range(1, len(dt_n) + 1):
    u[n] = update(u, dt_n, n)
  return u


def adj_solve(get_k, get_jf, dt_n, u, ref_factor):
  """Main_finite_difference.py:54-76: dense (J_F^T - I) v = -K on the refined grid."""
  dt_fine, _ = refine_all(dt_n, ref_factor)
  u_fine = interp_u(dt_n, u, ref_factor)
  jf = get_jf(u_fine, dt_fine)
  k = get_k(dt_fine, u_fine)
  return np.linalg.solve(jf.T - np.eye(jf.shape[0]), -k)


def err_est(update, u, v, dt_n, ref_factor):
  """Main_finite_difference.py:79-94: res[n] = u_f[n] - Phi(u_f[n-1]); err = res*v."""
  dt_fine, n_steps = refine_all(dt_n, ref_factor)
  u_fine = interp_u(dt_n, u, ref_factor)
  res = np.zeros_like(u_fine)
  for n in np.arange(n_steps) + 1:
    res[n] = u_fine[n] - update(u_fine, dt_fine, n)
  return res * v


def window_errors(err_fine, ref_factor):
  """Main_finite_difference.py:270-277: abs()[2:], windows of ref_factor-1 at stride
  ref_factor, summed (skips the first fine step of every coarse step)."""
  e = np.abs(err_fine)[2:]
  n_rows = (e.size - (ref_factor - 1)) // ref_factor + 1
  return np.array([np.sum(e[r * ref_factor:r * ref_factor + ref_factor - 1])
                   for r in range(n_rows)])


def split_step(times, err_steps):
  """Main_finite_difference.py:336-341: argmax+1, insert the midpoint."""
  n_steps = len(times) - 1
  times_new = np.zeros(n_steps + 2)
  ref_idx = int(np.argmax(err_steps) + 1)
  times_new[0:ref_idx] = times[0:ref_idx]
  times_new[ref_idx + 1:] = times[ref_idx:]
  times_new[ref_idx] = np.mean(times[ref_idx - 1:ref_idx + 1])
  return times_new, ref_idx


# The golden run's configuration (Main_finite_difference.py:131-140, 225-227).
def sin_update(u, dt_n, n):
  return u[n - 1] + np.sin(u[n - 1]) * dt_n[n - 1]


def sin_jf(u, dt_n):
  return np.diag(1 + np.cos(u[:-1]) * dt_n, -1)


def u2_k(dt_n, u, v0=0):
  return np.concatenate((2 * u[:-1] * dt_n, v0), axis=None)


def adapt_loop(times, u0, ref_factor, iterations, update=sin_update, get_jf=sin_jf, get_k=u2_k,
               tol=1e-5):
  """The __main__ loop of Main_finite_difference.py:263-343 without plotting."""
  out = []
  err = 1.0
  for _ in range(iterations):
    if err <= tol:
      break
    dt_n = np.diff(times, 1)
    u = forward_solve(update, dt_n, u0)
    v = adj_solve(get_k, get_jf, dt_n, u, ref_factor)
    raw = err_est(update, u, v, dt_n, ref_factor)
    err_steps = window_errors(raw, ref_factor)
    new_times, ref_idx = split_step(times, err_steps)
    out.append(dict(times=times, u=u, v=v, err_fine=raw, err_steps=err_steps, ref_idx=ref_idx))
    times = new_times
    err = np.sum(err_steps)
  return out
