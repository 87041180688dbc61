"""Restatement of the minmod slope limiters.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  The reference never executes
these routines and records no outputs for them ("parity unpinned" by the reference);
the oracle is pinned by a minmod truth table and limiter identities in the tests.

Summation order: the small matrix-vector products the limiter needs (cell average,
linear mode, slope) are written as explicit left-to-right sums with no fused
multiply-add, and the HIP kernel (k_limit) evaluates them in the same order with FP
contraction off, so the troubled-cell set ``ids`` (SlopeLimitN.m:23, an integer
decision against eps0 = 1e-8) is bit-exact between the two.
"""
import numpy as np


def minmod(v):
  """utils/minmod.m:6-12 — v is (m, n); returns (n,)."""
  v = np.asarray(v, dtype=float)
  m = v.shape[0]
  mfunc = np.zeros(v.shape[1])
  s = np.sum(np.sign(v), 0) / m
  ids = np.nonzero(np.abs(s) == 1)[0]
  if ids.size:
    mfunc[ids] = s[ids] * np.min(np.abs(v[:, ids]), axis=0)
  return mfunc


def minmod_b(v, M, h):
  """utils/minmodB.m:6-11 — TVB-modified minmod."""
  v = np.asarray(v, dtype=float)
  mfunc = v[0, :].copy()
  ids = np.nonzero(np.abs(mfunc) > M * np.asarray(h) ** 2)[0]
  if ids.size:
    mfunc[ids] = minmod(v[:, ids])
  return mfunc


def _row_dot(row, u):
  """sum_j row[j]*u[j,:] left to right, unfused."""
  acc = row[0] * u[0, :]
  for j in range(1, u.shape[0]):
    acc = acc + row[j] * u[j, :]
  return acc


def cell_average(u, S):
  """SlopeLimitN.m:9 — uh = invV*u; uh(2:Np,:)=0; uavg = V*uh; v = uavg(1,:)."""
  uh0 = _row_dot(S["invV"][0, :], u)
  return S["V"][0, 0] * uh0, uh0


def slope_limit_lin(ul, xl, vm1, v0, vp1, S, M=None):
  """utils/SlopeLimitLin.m:10-18; with M (> 0) its minmod is minmodB(., M, h), the TVB variant
  (utils/minmodB.m:6-11, which the reference defines but none of its limiters calls)."""
  Np = S["Np"]
  h = xl[Np - 1, :] - xl[0, :]  # :10
  x0 = xl[0, :] + h / 2  # :11
  ux0 = (2.0 / h) * _row_dot(S["Dr"][0, :], ul)  # :16 (row 1 of (2./hN).*(Dr*ul))
  args = np.vstack((ux0, (vp1 - v0) / h, (v0 - vm1) / h))
  m = minmod_b(args, M, h) if M else minmod(args)  # :18
  return v0[None, :] + (xl - x0[None, :]) * m[None, :]


def slope_limit_n(u, S, return_ids=False, M=None):
  """utils/SlopeLimitN.m:1-33 for one trajectory (u is (Np, K)); M: the TVB constant of the
  SlopeLimitLin it calls (slope_limit_lin)."""
  K = u.shape[1]
  v, uh0 = cell_average(u, S)  # :9
  ulimit = u.copy()
  eps0 = 1.0e-8  # :12
  ue1, ue2 = u[0, :], u[-1, :]  # :15
  vk = v
  vkm1 = np.concatenate(([v[0]], v[:K - 1]))  # :18
  vkp1 = np.concatenate((v[1:], [v[K - 1]]))
  ve1 = vk - minmod(np.vstack((vk - ue1, vk - vkm1, vkp1 - vk)))  # :21
  ve2 = vk + minmod(np.vstack((ue2 - vk, vk - vkm1, vkp1 - vk)))  # :22
  ids = np.nonzero((np.abs(ve1 - ue1) > eps0) | (np.abs(ve2 - ue2) > eps0))[0]  # :23
  if ids.size:  # :26-31
    uid = u[:, ids]
    uh1 = _row_dot(S["invV"][1, :], uid)
    V = S["V"]
    ul = V[:, 0:1] * uh0[None, ids] + V[:, 1:2] * uh1[None, :]  # :28 (uhl(3:Np,:)=0)
    ulimit[:, ids] = slope_limit_lin(ul, S["x"][:, ids], vkm1[ids], vk[ids], vkp1[ids], S, M)
  if return_ids:
    return ulimit, ids
  return ulimit


def slope_limit_1(u, S, M=None):
  """utils/SlopeLimit1.m:6-22 — Pi^1 limiter applied to every cell (M: as slope_limit_n)."""
  K = u.shape[1]
  v, uh0 = cell_average(u, S)
  uh1 = _row_dot(S["invV"][1, :], u)
  V = S["V"]
  ul = V[:, 0:1] * uh0[None, :] + V[:, 1:2] * uh1[None, :]
  vkm1 = np.concatenate(([v[0]], v[:K - 1]))
  vkp1 = np.concatenate((v[1:], [v[K - 1]]))
  return slope_limit_lin(ul, S["x"], vkm1, v, vkp1, S, M)
