"""ctypes wrapper of oracle/c/advec_oracle.c -- TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

A compiled (gcc -O3, OpenMP) restatement of :func:`oracle.advec.forward_sweep`,
:func:`oracle.adjoint.adjoint_sweep` (source 0) and :func:`oracle.effectivity.p_estimate`
(inflow ``INFLOW_A``) for bench.py's CPU baseline: the same algorithm as the numpy oracle,
written the way a CPU port would run it (element loops, all host cores).  tests/test_oracle_cport.py checks it against the numpy
oracle.  :func:`build` compiles it into ``oracle/liboracle_advec.so`` (git-ignored; it travels
to the GPU box with the tree like the product library).
"""
import ctypes
import os
import subprocess

import numpy as np

from .setup1d import RK4A, RK4B, RK4C

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "c", "advec_oracle.c")
LIB = os.path.join(HERE, "liboracle_advec.so")
# portable code (no -march=native: the library is built here and run on the GPU box's host)
CFLAGS = ["-O3", "-fopenmp", "-fPIC", "-shared", "-std=c99"]

_lib = None


def build(force=False):
  """gcc the C restatement into LIB (if missing or older than its source)."""
  if (not force and os.path.exists(LIB)
      and os.path.getmtime(LIB) >= os.path.getmtime(SRC)):
    return LIB
  tmp = LIB + ".tmp"
  subprocess.run(["gcc", *CFLAGS, "-o", tmp, SRC, "-lm"], check=True)
  os.replace(tmp, LIB)
  return LIB


def load():
  global _lib
  if _lib is None:
    if not os.path.exists(LIB):
      raise FileNotFoundError(f"{LIB} not built (oracle.cport.build())")
    lib = ctypes.CDLL(LIB)
    dp, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_double
    lib.oc_forward_sweep.restype = i32
    lib.oc_forward_sweep.argtypes = [i32, i64, dp, dp, dp, dp, dp, f64, f64, f64, i32, dp, dp]
    lib.oc_adjoint_sweep.restype = i32
    lib.oc_adjoint_sweep.argtypes = [i32, i64, dp, dp, dp, dp, dp, f64, f64, i32, dp, dp, dp,
                                     dp, dp]
    lib.oc_p_estimate.restype = i32
    lib.oc_p_estimate.argtypes = [i32, i32, i64, dp, dp, dp, dp, dp, dp, f64, f64, i32, dp, dp,
                                  dp, dp, dp]
    lib.oc_set_threads.restype = None
    lib.oc_set_threads.argtypes = [i32]
    _lib = lib
  return _lib


def _p(x):
  return x.ctypes.data_as(ctypes.c_void_p)


class Mesh:
  """The operator arrays of an oracle setup (metric="element": rx and Fscale constant per
  element) in the C port's layout."""

  def __init__(self, S, a):
    self.Np, self.K, self.a = S["Np"], S["K"], float(a)
    rx, fs = S["rx"], S["Fscale"]
    if not (np.all(rx == rx[0:1, :]) and fs.shape == (2, self.K)):
      raise ValueError("the C port takes one metric per element (setup metric='element')")
    self.dr = np.ascontiguousarray(S["Dr"], dtype=np.float64)
    self.lift = np.ascontiguousarray(S["LIFT"], dtype=np.float64)
    self.rx = np.ascontiguousarray(rx[0], dtype=np.float64)
    self.fsl = np.ascontiguousarray(fs[0], dtype=np.float64)
    self.fsr = np.ascontiguousarray(fs[1], dtype=np.float64)
    self.rk = np.ascontiguousarray(np.concatenate((RK4A, RK4B, RK4C)), dtype=np.float64)

  def args(self):
    return (self.Np, self.K, _p(self.dr), _p(self.lift), _p(self.rx), _p(self.fsl),
            _p(self.fsr), self.a)


def forward_sweep(u0, t0, dt, nsteps, mesh, threads=1):
  """u0: element-major (K Np,).  Returns (snaps (nsteps+1, K Np), times)."""
  lib = load()
  lib.oc_set_threads(int(threads))
  n = mesh.Np * mesh.K
  snaps = np.empty((nsteps + 1, n))
  snaps[0] = u0
  rc = lib.oc_forward_sweep(*mesh.args(), float(t0), float(dt), int(nsteps), _p(mesh.rk),
                            _p(snaps))
  if rc:
    raise RuntimeError(f"oc_forward_sweep failed ({rc})")
  times = [float(t0)]
  for _ in range(nsteps):
    times.append(times[-1] + dt)  # time = time + dt (One_code.mlx:139)
  return snaps, times


def adjoint_sweep(wT, snaps, times, dt, mesh, threads=1):
  """wT: element-major terminal weight.  Returns (w^0, eta (K,))."""
  lib = load()
  lib.oc_set_threads(int(threads))
  w = np.array(wT, dtype=np.float64, copy=True)
  eta = np.empty(mesh.K)
  tt = np.ascontiguousarray(times, dtype=np.float64)
  sn = np.ascontiguousarray(snaps)
  rc = lib.oc_adjoint_sweep(*mesh.args(), float(dt), int(len(snaps) - 1), _p(mesh.rk), _p(tt),
                            _p(sn), _p(w), _p(eta))
  if rc:
    raise RuntimeError(f"oc_adjoint_sweep failed ({rc})")
  return w, eta


def p_estimate(snaps, times, dt, mesh_hi, P, g_hi, npl, threads=1):
  """oracle/effectivity.py p_estimate (inflow INFLOW_A) on element-major fields: snaps
  (nsteps+1, K npl) at order N, g_hi the order-(N+1) terminal weight, P (nph, npl), mesh_hi
  the order-(N+1) setup's Mesh.  Returns (eta (K,), w^0 at order N+1)."""
  lib = load()
  lib.oc_set_threads(int(threads))
  w = np.array(g_hi, dtype=np.float64, copy=True)
  eta = np.empty(mesh_hi.K)
  tt = np.ascontiguousarray(times, dtype=np.float64)
  sn = np.ascontiguousarray(snaps)
  Pc = np.ascontiguousarray(P, dtype=np.float64)
  rc = lib.oc_p_estimate(int(npl), mesh_hi.Np, mesh_hi.K, _p(mesh_hi.dr), _p(mesh_hi.lift),
                         _p(mesh_hi.rx), _p(mesh_hi.fsl), _p(mesh_hi.fsr), _p(Pc), mesh_hi.a,
                         float(dt), int(len(snaps) - 1), _p(mesh_hi.rk), _p(tt), _p(sn), _p(w),
                         _p(eta))
  if rc:
    raise RuntimeError(f"oc_p_estimate failed ({rc})")
  return eta, w
