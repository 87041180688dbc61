"""Restatement of AdvecRHS1D and the LSERK4 Advec1D loop.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Fields are MATLAB-oriented
(Np, K) arrays; ``S`` is the dict returned by :func:`oracle.setup1d.startup1d`.
Vectorised the way MATLAB runs it (whole-array passes, ``Dr @ u``): this is also the
CPU baseline timed by bench.py.
"""
import math

import numpy as np

from .setup1d import RK4A, RK4B, RK4C

INFLOW_A = "a"    # uin = -sin(a*t)    utils/AdvecRHS1D.m:14
INFLOW_A2 = "a2"  # uin = -sin(a*a*t)  utils/One_code.mlx:129 (the executed copy)
INFLOW_ZERO = "zero"  # uin = 0: the homogeneous (linear) part, used by the adjoint identities


def inflow_value(a, t, inflow):
  if inflow == INFLOW_ZERO:
    return 0.0
  return -math.sin(a * a * t) if inflow == INFLOW_A2 else -math.sin(a * t)


def face_jumps(u, uin, a, S):
  """du of AdvecRHS1D.m:9-16 (central flux, alpha = 1) for a given inflow value.
  Returns du as (2, K) (row 0 = left face, row 1 = right face)."""
  alpha = 1.0
  uf = u.ravel(order="F")
  nxf = S["nx"].ravel(order="F")
  vmapM, vmapP = S["vmapM"], S["vmapP"]
  du = (uf[vmapM] - uf[vmapP]) * (a * nxf - (1 - alpha) * np.abs(a * nxf)) / 2  # :11
  mapI, mapO, vmapI = S["mapI"], S["mapO"], S["vmapI"]
  du[mapI] = (uf[vmapI] - uin) * (a * nxf[mapI] - (1 - alpha) * abs(a * nxf[mapI])) / 2  # :15
  du[mapO] = 0.0  # :16
  return du.reshape(2, S["K"], order="F")


def advec_rhs_uin(u, uin, a, S):
  """rhsu = -a*rx.*(Dr*u) + LIFT*(Fscale.*du)  (AdvecRHS1D.m:19) for a given inflow value."""
  du = face_jumps(u, uin, a, S)
  rhsu = -a * S["rx"] * (S["Dr"] @ u) + S["LIFT"] @ (S["Fscale"] * du)
  return rhsu, du


def advec_rhs1d(u, t, a, S, inflow=INFLOW_A):
  """utils/AdvecRHS1D.m:1-20 (inflow=INFLOW_A) / One_code.mlx:124-134 (INFLOW_A2)."""
  return advec_rhs_uin(u, inflow_value(a, t, inflow), a, S)


def lift_residual(u, t, a, S, inflow=INFLOW_A):
  """The interelement-jump (strong-form) residual LIFT*(Fscale.*du) of AdvecRHS1D.m:19."""
  du = face_jumps(u, inflow_value(a, t, inflow), a, S)
  return S["LIFT"] @ (S["Fscale"] * du)


def cfl_dt(S, final_time, cfl=0.75):
  """One_code.mlx:111-113: dt = 0.5*CFL/(2*pi)*min|x1-x2|; Nsteps = ceil(T/dt); dt = T/Nsteps."""
  x = S["x"]
  xmin = np.min(np.abs(x[0, :] - x[1, :]))
  dt = cfl / (2 * np.pi) * xmin
  dt = 0.5 * dt
  nsteps = int(math.ceil(final_time / dt))
  return final_time / nsteps, nsteps


def bench_dt(S, cfl=0.75):
  """Step size of the benchmark sweeps: the One_code.mlx:111-112 formula without the
  FinalTime rounding (fixed nsteps from t = 0)."""
  x = S["x"]
  return 0.5 * (cfl / (2 * np.pi) * np.min(np.abs(x[0, :] - x[1, :])))


def lserk4_step(u, time, dt, a, S, inflow=INFLOW_A, return_stages=False):
  """One step of the One_code.mlx:120-137 stage loop (resu is step-local: rk4a(1) = 0)."""
  resu = np.zeros_like(u)
  du = rhsu = None
  for s in range(5):
    timelocal = time + RK4C[s] * dt  # :121
    rhsu, du = advec_rhs1d(u, timelocal, a, S, inflow)  # :124-134
    resu = RK4A[s] * resu + dt * rhsu  # :135
    u = u + RK4B[s] * resu  # :136
  if return_stages:
    return u, du, rhsu, resu
  return u


def euler_step(u, time, dt, a, S, inflow=INFLOW_A):
  """Forward Euler u += dt*rhs (config 1; the update of Main_finite_difference.py:131-132)."""
  rhsu, _ = advec_rhs1d(u, time, a, S, inflow)
  return u + dt * rhsu


def step(u, time, dt, a, S, inflow=INFLOW_A, scheme="lserk4"):
  if scheme == "lserk4":
    return lserk4_step(u, time, dt, a, S, inflow)
  return euler_step(u, time, dt, a, S, inflow)


def forward_sweep(u0, t0, dt, nsteps, a, S, inflow=INFLOW_A, scheme="lserk4"):
  """nsteps steps from t0 with time = time + dt (One_code.mlx:139); returns the list of
  the nsteps+1 states (the snapshots) and the time levels."""
  snaps = [u0.copy()]
  times = [t0]
  u, time = u0.copy(), t0
  for _ in range(nsteps):
    u = step(u, time, dt, a, S, inflow, scheme)
    time = time + dt
    snaps.append(u)
    times.append(time)
  return snaps, times


def advec1d(u, final_time, a, S, inflow=INFLOW_A2):
  """The Advec1D loop of One_code.mlx:106-140.  Returns u and the last-stage du, rhsu,
  resu (the variables displayed at :151-154) plus dt and Nsteps."""
  dt, nsteps = cfl_dt(S, final_time)
  time = 0.0
  resu = np.zeros_like(u)
  du = rhsu = None
  for _ in range(nsteps):
    for s in range(5):
      timelocal = time + RK4C[s] * dt
      rhsu, du = advec_rhs1d(u, timelocal, a, S, inflow)
      resu = RK4A[s] * resu + dt * rhsu
      u = u + RK4B[s] * resu
    time = time + dt
  return dict(u=u, du=du, rhsu=rhsu, resu=resu, dt=dt, nsteps=nsteps)
