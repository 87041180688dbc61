"""Host-side nodal-DG setup with the attribute surface of the reference's BaseGalerkin1D.

The reference class (python/galerkin.py:14-263) is an uncalled, jax-only and broken
port of utils/StartUp1D.m (SURVEY §8c lists its defects).  This class keeps its
configuration attributes (``n, k, domain, n_gq, node_tol, n_fp, n_faces``,
galerkin.py:18-24) and the attribute names it sets (galerkin.py:199-263), computed in
numpy on the host with the MATLAB semantics of utils/*.m.  These are the constants
the HIP plan is built from (``DGAdvection1D``); nothing here runs per time step.

Corrections relative to galerkin.py (each noted where it applies): ``lift`` is built
with all of Lift1D's arguments (:211 vs :114); ``d_r`` uses order n (:208);
``r_x``/``j_mat`` are not swapped (:220); the Jacobi recurrence writes row i+1
(:84); eigenvalues are sorted (:42); ``v_map_o`` is the last node (:194).
"""
import math

import numpy as np


def _gamma(z):
  return math.gamma(z)


class BaseGalerkin1D:
  """Reference-element operators, mesh, metric and connectivity of a 1D nodal-DG mesh.

  Fields are (n_p, k) arrays in MATLAB orientation; the device layout is their
  column-major flattening (element-major), see ``to_device_layout``.
  """
  n: int = 1
  k: int = 2
  domain = np.array([0.0, 1.0])
  n_gq: int = 2
  node_tol: float = 1e-10
  n_fp = 1
  n_faces = 2

  def __init__(self, n=None, k=None, domain=None, v_x=None, n_gq=None):
    if n is not None:
      self.n = int(n)
    if n_gq is not None:
      self.n_gq = int(n_gq)
    if v_x is not None:
      self.v_x = np.asarray(v_x, dtype=np.float64).copy()
      self.k = len(self.v_x) - 1
      self.domain = np.array([self.v_x[0], self.v_x[-1]])
    else:
      if k is not None:
        self.k = int(k)
      if domain is not None:
        self.domain = np.asarray(domain, dtype=np.float64)
      nv = self.k + 1
      # MeshGen1D.m:7-9: VX(i) = (xmax-xmin)*(i-1)/(Nv-1) + xmin
      i = np.arange(1, nv + 1, dtype=np.float64)
      self.v_x = (self.domain[1] - self.domain[0]) * (i - 1) / (nv - 1) + self.domain[0]
    if self.n < 1:
      raise ValueError("polynomial order n must be >= 1")
    if self.k < 2:
      raise ValueError("need at least 2 elements")
    self.e_to_v = np.stack((np.arange(self.k), np.arange(1, self.k + 1)), axis=1)
    self.startUp1D()
    # galerkin.py:252-263: Gauss quadrature nodes/weights and the nodal basis there.
    self.r_gl = self.r
    self.r, self.w = self.jacobiGQ(0, 0, self.n_gq)
    self.n_r = self.r.shape[0]
    self.phi = self.vandermonde1D(self.n, self.r) @ self.inv_v  # phi[q, i] = l_i(r_q)

  # --- L0: reference element (utils/Jacobi*.m, Vandermonde1D.m, Dmatrix1D.m, Lift1D.m) ---
  def jacobiGQ(self, a, b, n):
    """JacobiGQ.m:8-22."""
    if n == 0:
      return np.array([-(a - b) / (a + b + 2)]), np.array([2.0])
    h1 = 2.0 * np.arange(n + 1) + a + b
    with np.errstate(divide="ignore", invalid="ignore"):
      main = -0.5 * (a * a - b * b) / (h1 + 2) / h1
    j = np.arange(1, n + 1, dtype=np.float64)
    sub = 2.0 / (h1[:-1] + 2) * np.sqrt(j * (j + a + b) * (j + a) * (j + b) /
                                        (h1[:-1] + 1) / (h1[:-1] + 3))
    jmat = np.diag(main) + np.diag(sub, 1)
    if a + b < 10 * np.finfo(np.float64).eps:
      jmat[0, 0] = 0.0
    jmat = jmat + jmat.T
    d, v = np.linalg.eigh(jmat)  # sorted ascending
    w = v[0, :] ** 2 * 2 ** (a + b + 1) / (a + b + 1) * _gamma(a + 1) * _gamma(b + 1) / \
        _gamma(a + b + 1)
    return d, w

  def jacobiGL(self, a, b, n):
    """JacobiGL.m:8-12."""
    if n == 1:
      return np.array([-1.0, 1.0])
    x_int, _ = self.jacobiGQ(a + 1, b + 1, n - 2)
    return np.concatenate(([-1.0], x_int, [1.0]))

  def jacobiP(self, x, a, b, n):
    """JacobiP.m:9-36 (orthonormal)."""
    xp = np.asarray(x, dtype=np.float64).ravel()
    g0 = 2 ** (a + b + 1) / (a + b + 1) * _gamma(a + 1) * _gamma(b + 1) / _gamma(a + b + 1)
    p_prev = np.full(xp.shape, 1.0 / math.sqrt(g0))
    if n == 0:
      return p_prev
    g1 = (a + 1) * (b + 1) / (a + b + 3) * g0
    p = ((a + b + 2) * xp / 2 + (a - b) / 2) / math.sqrt(g1)
    if n == 1:
      return p
    a_old = 2 / (2 + a + b) * math.sqrt((a + 1) * (b + 1) / (a + b + 3))
    for i in range(1, n):
      h1 = 2 * i + a + b
      a_new = 2 / (h1 + 2) * math.sqrt((i + 1) * (i + 1 + a + b) * (i + 1 + a) * (i + 1 + b) /
                                       (h1 + 1) / (h1 + 3))
      b_new = -(a * a - b * b) / h1 / (h1 + 2)
      p_prev, p = p, 1 / a_new * (-a_old * p_prev + (xp - b_new) * p)
      a_old = a_new
    return p

  def vandermonde1D(self, n, r):
    return np.stack([self.jacobiP(r, 0, 0, j) for j in range(n + 1)], axis=1)

  def gradJacobiP(self, r, a, b, n):
    if n == 0:
      return np.zeros(np.asarray(r).size)
    return math.sqrt(n * (n + a + b + 1)) * self.jacobiP(r, a + 1, b + 1, n - 1)

  def gradVandermonde1D(self, n, r):
    return np.stack([self.gradJacobiP(r, 0, 0, j) for j in range(n + 1)], axis=1)

  def dMatrix1D(self, n, r, v):
    """Dmatrix1D.m:7-8: Dr = Vr / V."""
    return np.linalg.solve(v.T, self.gradVandermonde1D(n, r).T).T

  def lift1D(self, n_p, n_faces, n_fp, v):
    """Lift1D.m:7-13."""
    e_mat = np.zeros((n_p, n_faces * n_fp))
    e_mat[0, 0] = 1.0
    e_mat[n_p - 1, 1] = 1.0
    return v @ (v.T @ e_mat)

  # --- L1: mesh, metric, connectivity (StartUp1D.m, GeometricFactors1D.m, Normals1D.m,
  #     Connect1D.m, BuildMaps1D.m) ---
  def geometricFactors1D(self, x, d_r):
    j_mat = d_r @ x
    return 1.0 / j_mat, j_mat  # (r_x, j_mat): galerkin.py:220 had them swapped

  def normals1D(self):
    return np.stack((-np.ones(self.k), np.ones(self.k)))

  def connect1D(self, e_to_v):
    """Connect1D.m: for a 1D chain, face 0 of element k meets face 1 of k-1 and vice versa;
    boundary faces point to themselves."""
    k = e_to_v.shape[0]
    e_to_e = np.stack((np.arange(k) - 1, np.arange(k) + 1), axis=1)
    e_to_f = np.stack((np.ones(k, dtype=np.int64), np.zeros(k, dtype=np.int64)), axis=1)
    e_to_e[0, 0], e_to_f[0, 0] = 0, 0
    e_to_e[k - 1, 1], e_to_f[k - 1, 1] = k - 1, 1
    return e_to_e, e_to_f

  def buildMaps1D(self):
    """BuildMaps1D.m:10-43 (0-based)."""
    k, n_p = self.k, self.n_p
    node_ids = np.arange(k * n_p).reshape(k, n_p).T
    v_map_m = np.stack([node_ids[self.f_mask[f], :] for f in range(self.n_faces)])  # (2, k)
    v_id_p = v_map_m[self.e_to_f.T, self.e_to_e.T]
    xf = self.x.ravel(order="F")
    d = (xf[v_map_m] - xf[v_id_p]) ** 2
    v_map_p = np.where(d < self.node_tol, v_id_p, 0).ravel(order="F")
    v_map_m = v_map_m.ravel(order="F")
    map_b = np.nonzero(v_map_p == v_map_m)[0]
    v_map_b = v_map_m[map_b]
    self.map_i = 0
    self.map_o = k * self.n_faces - 1
    self.v_map_i = 0
    self.v_map_o = k * n_p - 1
    return v_map_m, v_map_p, v_map_b, map_b

  def startUp1D(self):
    """StartUp1D.m:5-39."""
    self.n_p = self.n + 1
    self.r = self.jacobiGL(0, 0, self.n)
    self.v = self.vandermonde1D(self.n, self.r)
    self.inv_v = np.linalg.inv(self.v)
    self.d_r = self.dMatrix1D(self.n, self.r, self.v)
    self.lift = self.lift1D(self.n_p, self.n_faces, self.n_fp, self.v)
    v_a, v_b = self.e_to_v[:, 0], self.e_to_v[:, 1]
    self.x = np.ones((self.n_p, 1)) * self.v_x[v_a][None, :] + \
        (0.5 * (self.r + 1))[:, None] * (self.v_x[v_b] - self.v_x[v_a])[None, :]
    self.r_x, self.j_mat = self.geometricFactors1D(self.x, self.d_r)
    self.f_mask = np.concatenate((np.nonzero(np.abs(self.r + 1) < self.node_tol)[0],
                                  np.nonzero(np.abs(self.r - 1) < self.node_tol)[0]))
    self.f_x = self.x[self.f_mask, :]
    self.n_x = self.normals1D()
    self.f_scale = 1.0 / self.j_mat[self.f_mask, :]
    self.e_to_e, self.e_to_f = self.connect1D(self.e_to_v)
    self.v_map_m, self.v_map_p, self.v_map_b, self.map_b = self.buildMaps1D()

  # --- helpers ---
  def cfl_dt(self, cfl=0.75):
    """Step size of One_code.mlx:111-112: 0.5*CFL/(2*pi)*min|x_1 - x_2|."""
    return 0.5 * (cfl / (2 * np.pi) * np.min(np.abs(self.x[0, :] - self.x[1, :])))

  def to_device_layout(self, u):
    """(n_p, k) field -> flat element-major vector (the device layout)."""
    return np.ascontiguousarray(np.asarray(u).T).ravel()

  def from_device_layout(self, v):
    return np.asarray(v).reshape(-1, self.n_p).T.copy()


def prolongation(lo, hi):
  """P (hi.n_p x lo.n_p): the order-lo.n element polynomial through its nodal values,
  evaluated at the order-hi.n LGL nodes (u_hi = P u_lo; Vandermonde1D.m at the new nodes
  times invV).  The p-enrichment of the DWR estimate (MAIN.m:32-34 marches the adjoint one
  order up; dg_lserk4_adj_p)."""
  return lo.vandermonde1D(lo.n, hi.r_gl) @ lo.inv_v


def split_interval(nodes, idx):
  """Insert the midpoint of interval ``idx`` (0-based) into a sorted node vector —
  the refinement of python/Main_finite_difference.py:336-341 (ref_idx = idx + 1) and
  matlab/MAIN.m:137-141 (1-based slab ref_i = idx + 1)."""
  nodes = np.asarray(nodes, dtype=np.float64)
  ref_idx = int(idx) + 1
  out = np.zeros(nodes.size + 1)
  out[0:ref_idx] = nodes[0:ref_idx]
  out[ref_idx + 1:] = nodes[ref_idx:]
  out[ref_idx] = np.mean(nodes[ref_idx - 1:ref_idx + 1])
  return out
