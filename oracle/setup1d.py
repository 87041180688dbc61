"""Restatement of the Hesthaven–Warburton 1D nodal-DG setup used by the reference.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Arrays keep MATLAB's
orientation: nodal fields are (Np, K) (column k = element k), so MATLAB linear
indexing ``u(vmapM)`` is ``u.ravel(order='F')[vmapM]``.  Index maps are 0-based
here; ``startup1d(...)['matlab']`` holds the 1-based copies for golden checks.
"""
import math

import numpy as np
import scipy.sparse as sp

NODETOL = 1e-10  # utils/StartUp1D.m:5

# utils/Globals1D.m:20-34 — low-storage RK coefficients.
RK4A = np.array([0.0,
                 -567301805773.0 / 1357537059087.0,
                 -2404267990393.0 / 2016746695238.0,
                 -3550918686646.0 / 2091501179385.0,
                 -1275806237668.0 / 842570457699.0])
RK4B = np.array([1432997174477.0 / 9575080441755.0,
                 5161836677717.0 / 13612068292357.0,
                 1720146321549.0 / 2090206949498.0,
                 3134564353537.0 / 4481467310338.0,
                 2277821191437.0 / 14882151754819.0])
RK4C = np.array([0.0,
                 1432997174477.0 / 9575080441755.0,
                 2526269341429.0 / 6820363962896.0,
                 2006345519317.0 / 3224310063776.0,
                 2802321613138.0 / 2924317926251.0])


def jacobi_gq(alpha, beta, N):
  """utils/JacobiGQ.m:8-22 — Gauss quadrature by the symmetric Jacobi-matrix eig."""
  if N == 0:  # :8
    return np.array([-(alpha - beta) / (alpha + beta + 2)]), np.array([2.0])
  n = np.arange(N + 1, dtype=float)
  h1 = 2 * n + alpha + beta  # :12
  with np.errstate(divide="ignore", invalid="ignore"):
    diag = -0.5 * (alpha ** 2 - beta ** 2) / (h1 + 2) / h1  # :13
  m = np.arange(1, N + 1, dtype=float)
  off = 2.0 / (h1[:N] + 2) * np.sqrt(m * (m + alpha + beta) * (m + alpha) * (m + beta)
                                      / (h1[:N] + 1) / (h1[:N] + 3))  # :14-15
  J = np.diag(diag) + np.diag(off, 1)
  if alpha + beta < 10 * np.finfo(float).eps:  # :16
    J[0, 0] = 0.0
  J = J + J.T  # :17
  x, V = np.linalg.eigh(J)  # :20 (ascending, as MATLAB eig of a symmetric matrix)
  w = V[0, :] ** 2 * 2 ** (alpha + beta + 1) / (alpha + beta + 1) * math.gamma(alpha + 1) * \
      math.gamma(beta + 1) / math.gamma(alpha + beta + 1)  # :21-22
  return x, w


def jacobi_gl(alpha, beta, N):
  """utils/JacobiGL.m:8-12 — Gauss–Lobatto nodes."""
  if N == 1:
    return np.array([-1.0, 1.0])
  xint, _ = jacobi_gq(alpha + 1, beta + 1, N - 2)
  return np.concatenate(([-1.0], xint, [1.0]))


def jacobi_p(x, alpha, beta, N):
  """utils/JacobiP.m:9-36 — orthonormal Jacobi polynomial of order N at x."""
  xp = np.asarray(x, dtype=float).ravel()
  PL = np.zeros((N + 1, xp.size))
  gamma0 = 2 ** (alpha + beta + 1) / (alpha + beta + 1) * math.gamma(alpha + 1) * \
      math.gamma(beta + 1) / math.gamma(alpha + beta + 1)  # :15-16
  PL[0, :] = 1.0 / math.sqrt(gamma0)
  if N == 0:
    return PL[0, :].copy()
  gamma1 = (alpha + 1) * (beta + 1) / (alpha + beta + 3) * gamma0  # :19
  PL[1, :] = ((alpha + beta + 2) * xp / 2 + (alpha - beta) / 2) / math.sqrt(gamma1)
  if N == 1:
    return PL[1, :].copy()
  aold = 2 / (2 + alpha + beta) * math.sqrt((alpha + 1) * (beta + 1) / (alpha + beta + 3))
  for i in range(1, N):  # :27-34
    h1 = 2 * i + alpha + beta
    anew = 2 / (h1 + 2) * math.sqrt((i + 1) * (i + 1 + alpha + beta) * (i + 1 + alpha) *
                                    (i + 1 + beta) / (h1 + 1) / (h1 + 3))
    bnew = -(alpha ** 2 - beta ** 2) / h1 / (h1 + 2)
    PL[i + 1, :] = 1 / anew * (-aold * PL[i - 1, :] + (xp - bnew) * PL[i, :])
    aold = anew
  return PL[N, :].copy()


def grad_jacobi_p(r, alpha, beta, N):
  """utils/GradJacobiP.m:7-12."""
  r = np.asarray(r, dtype=float).ravel()
  if N == 0:
    return np.zeros(r.size)
  return math.sqrt(N * (N + alpha + beta + 1)) * jacobi_p(r, alpha + 1, beta + 1, N - 1)


def vandermonde1d(N, r):
  """utils/Vandermonde1D.m:6-9."""
  V = np.zeros((len(r), N + 1))
  for j in range(N + 1):
    V[:, j] = jacobi_p(r, 0, 0, j)
  return V


def grad_vandermonde1d(N, r):
  """utils/GradVandermonde1D.m:6-11."""
  DVr = np.zeros((len(r), N + 1))
  for i in range(N + 1):
    DVr[:, i] = grad_jacobi_p(r, 0, 0, i)
  return DVr


def dmatrix1d(N, r, V):
  """utils/Dmatrix1D.m:7-8 — Dr = Vr / V."""
  Vr = grad_vandermonde1d(N, r)
  return np.linalg.solve(V.T, Vr.T).T


def lift1d(Np, Nfaces, Nfp, V):
  """utils/Lift1D.m:7-13 — LIFT = V (V^T E)."""
  E = np.zeros((Np, Nfaces * Nfp))
  E[0, 0] = 1.0
  E[Np - 1, 1] = 1.0
  return V @ (V.T @ E)


def mesh_gen1d(xmin, xmax, K):
  """utils/MeshGen1D.m:4-14 (EToV 0-based)."""
  Nv = K + 1
  VX = np.array([(xmax - xmin) * (i - 1) / (Nv - 1) + xmin for i in range(1, Nv + 1)])
  EToV = np.stack((np.arange(K), np.arange(1, K + 1)), axis=1)
  return Nv, VX, K, EToV


def connect1d(EToV):
  """utils/Connect1D.m:7-40 — face-to-face connectivity via the sparse FToV product."""
  Nfaces = 2
  K = EToV.shape[0]
  TotalFaces = Nfaces * K
  Nv = K + 1
  vn = [0, 1]  # :12 local face -> local vertex
  rows = np.arange(TotalFaces)  # sk = k*Nfaces + face (:16-22)
  cols = EToV[:, vn].ravel()
  SpFToV = sp.csr_matrix((np.ones(TotalFaces), (rows, cols)), shape=(TotalFaces, Nv))
  SpFToF = (SpFToV @ SpFToV.T - sp.identity(TotalFaces)).tocoo()
  sel = SpFToF.data == 1
  faces1, faces2 = SpFToF.row[sel], SpFToF.col[sel]
  element1, face1 = faces1 // Nfaces, faces1 % Nfaces
  element2, face2 = faces2 // Nfaces, faces2 % Nfaces
  EToE = np.repeat(np.arange(K)[:, None], Nfaces, axis=1)
  EToF = np.repeat(np.arange(Nfaces)[None, :], K, axis=0)
  EToE[element1, face1] = element2
  EToF[element1, face1] = face2
  return EToE, EToF


def build_maps1d(S):
  """utils/BuildMaps1D.m:10-43 (vectorised; same node-distance test D < NODETOL)."""
  K, Np, Fmask, x = S["K"], S["Np"], S["Fmask"], S["x"]
  Nfaces = 2
  nodeids = np.arange(K * Np).reshape(K, Np).T  # MATLAB reshape(1:K*Np, Np, K), 0-based
  vmapM = np.zeros((Nfaces, K), dtype=np.int64)  # (Nfp=1, Nfaces, K) squeezed
  for f in range(Nfaces):
    vmapM[f, :] = nodeids[Fmask[f], :]
  k2 = S["EToE"]  # (K, Nfaces)
  f2 = S["EToF"]
  vidM = vmapM  # (Nfaces, K)
  vidP = vmapM[f2.T, k2.T]
  xf = x.ravel(order="F")
  D = (xf[vidM] - xf[vidP]) ** 2
  vmapP = np.where(D < NODETOL, vidP, 0)
  vmapP = vmapP.ravel(order="F")
  vmapM = vmapM.ravel(order="F")
  mapB = np.nonzero(vmapP == vmapM)[0]
  vmapB = vmapM[mapB]
  return vmapM, vmapP, vmapB, mapB


def startup1d(N, VX, metric="matlab"):
  """utils/StartUp1D.m:5-39 for the mesh VX (length K+1).  Returns a dict of the
  MATLAB globals (0-based maps) plus 'matlab' with 1-based copies.

  metric="matlab": J = Dr*x, rx = 1./J, Fscale = 1./J(Fmask,:) node by node, exactly as
  GeometricFactors1D.m:6 / StartUp1D.m:33 (used for the One_code.mlx goldens).  On fine
  meshes that nodal J carries rounding noise of relative size ~eps*|x|/h (about 1e-10 at
  K = 2^20) although the elements are affine.
  metric="element": the per-element constant the HIP plan uses (dg_plan_create):
  rx = Fscale = 2/h_k with h_k = VX(k+1)-VX(k), or 2/mean(h) when the mesh is uniform to
  1e-12 (the same test as the plan).  GPU parity tests compare against this mode."""
  K = len(VX) - 1
  EToV = np.stack((np.arange(K), np.arange(1, K + 1)), axis=1)
  Np = N + 1
  r = jacobi_gl(0, 0, N)  # :9
  V = vandermonde1d(N, r)  # :12
  invV = np.linalg.inv(V)
  Dr = dmatrix1d(N, r, V)  # :13
  LIFT = lift1d(Np, 2, 1, V)  # :16
  va, vb = EToV[:, 0], EToV[:, 1]  # :19
  x = np.ones((N + 1, 1)) * VX[va][None, :] + (0.5 * (r + 1))[:, None] * (VX[vb] - VX[va])[None, :]
  J = Dr @ x  # GeometricFactors1D.m:6
  if metric == "element":
    h = np.diff(np.asarray(VX, dtype=float))
    hmean = np.cumsum(h)[-1] / K  # sequential sum, as the plan
    if (h.max() - h.min()) <= 1e-12 * hmean:
      s_el = np.full(K, 2.0 / hmean)
    else:
      s_el = 2.0 / h
    J = np.ones((Np, 1)) * (1.0 / s_el)[None, :]
  rx = 1.0 / J
  if metric == "element":
    rx = np.ones((Np, 1)) * s_el[None, :]
  fmask1 = np.nonzero(np.abs(r + 1) < NODETOL)[0]  # :26-28
  fmask2 = np.nonzero(np.abs(r - 1) < NODETOL)[0]
  Fmask = np.concatenate((fmask1, fmask2))
  Fx = x[Fmask, :]
  nx = np.vstack((-np.ones(K), np.ones(K)))  # Normals1D.m:10
  Fscale = 1.0 / J[Fmask, :]  # :33
  if metric == "element":
    Fscale = np.ones((2, 1)) * s_el[None, :]
  S = dict(N=N, K=K, Np=Np, Nfp=1, Nfaces=2, VX=np.asarray(VX, float), EToV=EToV, r=r, V=V,
           invV=invV, Dr=Dr, LIFT=LIFT, x=x, J=J, rx=rx, Fmask=Fmask, Fx=Fx, nx=nx,
           Fscale=Fscale)
  S["EToE"], S["EToF"] = connect1d(EToV)  # :36
  S["vmapM"], S["vmapP"], S["vmapB"], S["mapB"] = build_maps1d(S)  # :39
  S["mapI"], S["mapO"], S["vmapI"], S["vmapO"] = 0, K * 2 - 1, 0, K * Np - 1  # BuildMaps1D.m:43
  S["matlab"] = dict(Fmask=Fmask + 1, EToE=S["EToE"] + 1, EToF=S["EToF"] + 1,
                     vmapM=S["vmapM"] + 1, vmapP=S["vmapP"] + 1, vmapB=S["vmapB"] + 1,
                     mapB=S["mapB"] + 1, mapI=1, mapO=2 * K, vmapI=1, vmapO=K * Np)
  return S


def uniform_setup(N, K, xmin=0.0, xmax=1.0, metric="matlab"):
  """MeshGen1D + StartUp1D (the One_code.mlx:33-102 sequence)."""
  _, VX, _, _ = mesh_gen1d(xmin, xmax, K)
  return startup1d(N, VX, metric)


def to_elem_major(u):
  """(Np, K) MATLAB field -> flat element-major vector u[k*Np+i] (product layout)."""
  return np.ascontiguousarray(u.T).ravel()


def from_elem_major(v, Np):
  return np.asarray(v).reshape(-1, Np).T.copy()
