"""The adapt-loop callback API of the reference (python/factory.py:18-630), for the
finite-difference scalar ODEs and for the GPU DG advection path.

Reference surface mirrored here (names, argument meaning and order):

* ``Problem`` (factory.py:18-26), ``Funs`` (:29-35), ``AdaptFuns`` (:38-46),
  ``AdaptState`` (:49-71), ``FunFactory`` (:74) with ``getFunctions`` (:79) and
  ``getAdaptFunctions`` (:269).
* ``forwardSolve(funs, dt_n, u0)``, ``adjointSolve(funs, dt_n, u)``,
  ``errorEstimate(funs, dt_n, u, v)``, ``refineAll(dt_n)``, ``interpU(dt_fine, dt_n, u)``,
  ``adapt(state, u0, plot)``.

Differences, each deliberate:

* factory.py:359 calls ``getJF(dt_fine, u_fine)`` although ``getJF(u, dt_n)`` (:114) — the
  arguments are swapped there; here they are passed in the declared order, which is what
  Main_finite_difference.py:69 does (its outputs are the golden reference).
* ``plot`` / ``animate`` (matplotlib/cv2 presentation) are out of scope and are no-ops.
* The neural-network (``is_net``) branch is out of scope and raises.

The DG path (``DGProblem`` / ``DGFunFactory``) keeps the same shape for spatial
adaptivity: the refined grid is the mesh ``v_x`` instead of ``times``, the forward and
adjoint sweeps run on the GPU through :class:`~.operators.DGAdvection1D`, the error
estimate is the per-element dual-weighted residual, and ``adapt`` splits the argmax
element (matlab/MAIN.m:137-141; Main_finite_difference.py:336-341).
"""
import math
from typing import Callable, NamedTuple, Union

import numpy as np

from .galerkin import BaseGalerkin1D, split_interval


class Problem(NamedTuple):
  case: str
  is_net: bool
  linear_ode: bool
  linear_out_functional: bool
  ode: str
  out_functional: str
  ref_factor: Union[float, int]
  t_span: np.ndarray


class Funs(NamedTuple):
  exactAdj: Callable
  exactFwd: Callable
  fwdUpdate: Callable
  getF: Callable
  getJF: Callable
  getK: Callable


class AdaptFuns(NamedTuple):
  adapt: Callable
  adjointSolve: Callable
  animate: Callable
  errorEstimate: Callable
  forwardSolve: Callable
  interpU: Callable
  plot: Callable
  refineAll: Callable


class AdaptState:
  """factory.py:49-71."""

  def __init__(self, problem, times):
    self.it = 0
    self.problem = problem
    self.times = times
    self.times_new = times
    self.err_steps = None
    self.u = None
    self.v = None
    self.bar_ylim = None

  def iterate(self, err_steps, times, times_new, u, v):
    self.it += 1
    self.err_steps = err_steps
    self.times = times
    self.times_new = times_new
    self.u = u
    self.v = v


def _integral(fn, a, b):
  import scipy.integrate as integrate
  return integrate.quad(fn, a, b)[0]


def window_errors(err_fine, ref_factor):
  """|err|[2:], windows of ref_factor-1 at stride ref_factor, summed
  (Main_finite_difference.py:270-277; factory.py:317-326)."""
  e = np.abs(np.asarray(err_fine))[2:]
  rows = (e.size - (ref_factor - 1)) // ref_factor + 1
  return np.array([e[r * ref_factor:r * ref_factor + ref_factor - 1].sum() for r in range(rows)])


class FunFactory:
  """Callback factory of factory.py:74-630 for the finite-difference scalar ODEs."""

  def __init__(self, problem: Problem):
    self.problem = problem

  def getFunctions(self) -> Funs:
    problem = self.problem
    if problem.is_net:
      raise NotImplementedError("the ResNet-ODE (is_net) branch is out of scope (SURVEY §2)")
    t_end = float(problem.t_span[-1])
    if problem.ode == "du/dt=u":  # factory.py:84-99

      def fwdUpdate(dt_n, u, n):
        return (1 + dt_n[n - 1]) * u[n - 1]

      def getF(u, dt_n):
        return np.concatenate((u[0], (1 + dt_n) * u[:-1]), axis=None)

      def getJF(u, dt_n):
        return np.diag(1 + dt_n, -1)

      def exactFwd(t, u0=1.0):
        return u0 * np.exp(t)

    elif problem.ode == "du/dt=sin(u)":  # factory.py:101-117

      def fwdUpdate(dt_n, u, n):
        return u[n - 1] + np.sin(u[n - 1]) * dt_n[n - 1]

      def getF(u, dt_n):
        return np.concatenate((u[0], u[:-1] + np.sin(u[:-1]) * dt_n), axis=None)

      def getJF(u, dt_n):
        return np.diag(1 + np.cos(u[:-1]) * dt_n, -1)

      def exactFwd(t, u0=1.0):
        return 2 * np.arctan2(np.sin(u0 / 2) * np.exp(t), np.cos(u0 / 2))

    else:
      raise ValueError(f"unknown ode {problem.ode!r}")

    f = problem.out_functional
    if f == "J=int(u)":

      def getK(dt_n, u=None, v0=0):
        return np.concatenate((dt_n, v0), axis=None)

    elif f == "J=u_N":

      def getK(dt_n, u=None, v0=0):
        k = np.zeros_like(dt_n)
        k[-1] = 1
        return np.concatenate((k, v0), axis=None)

    elif f == "J=int(u^2)":

      def getK(dt_n, u, v0=0):
        return np.concatenate((2 * u[:-1] * dt_n, v0), axis=None)

    else:
      raise ValueError(f"unknown functional {f!r}")

    def exactAdj(t, u):
      """Continuous adjoint by quadrature (Main_finite_difference.py:157-240 forms)."""
      t = np.asarray(t, dtype=float)
      u = np.asarray(u, dtype=float)
      a = np.zeros_like(u)
      u_interp = lambda x: np.interp(x, t, u)  # noqa: E731
      fp = (lambda y: 1.0) if problem.ode == "du/dt=u" else (lambda y: np.cos(u_interp(y)))
      for i in range(len(u) - 1):
        decay = math.exp(-_integral(fp, t_end, t[i]))
        if f == "J=u_N":
          a[i] = decay
        elif f == "J=int(u)":
          a[i] = decay * _integral(lambda z: -math.exp(_integral(fp, t_end, z)), t_end, t[i])
        else:
          a[i] = decay * _integral(lambda z: math.exp(_integral(fp, t_end, z)) * u_interp(z) * -2,
                                   t_end, t[i])
      return a

    return Funs(exactAdj, exactFwd, fwdUpdate, getF, getJF, getK)

  def getAdaptFunctions(self) -> AdaptFuns:
    problem = self.problem
    rf = int(problem.ref_factor)

    def refineAll(dt_n):  # factory.py:273-279
      n_steps = len(dt_n) * rf
      dt_fine = np.zeros(n_steps)
      for f in range(rf):
        dt_fine[f:n_steps - rf + f + 1:rf] = dt_n / rf
      return dt_fine, n_steps

    def interpU(dt_fine, dt_n, u):  # factory.py:281-286
      t_coarse = np.concatenate(([0], np.cumsum(dt_n)), axis=None)
      t_fine = np.concatenate(([0], np.cumsum(dt_fine)), axis=None)
      return np.interp(t_fine, t_coarse, u)

    def forwardSolve(funs, dt_n, u0=None):  # factory.py:380-397
      def solve(u0):
        u_vec = np.zeros(len(dt_n) + 1)
        u_vec[0] = u0
        for n in range(1, len(dt_n) + 1):
          u_vec[n] = funs.fwdUpdate(dt_n, u_vec, n)
        return u_vec
      return solve if u0 is None else solve(u0)

    def adjointSolve(funs, dt_n, u):  # factory.py:346-363, J_F in declared argument order
      dt_fine, _ = refineAll(dt_n)
      u_fine = interpU(dt_fine, dt_n, u)
      jf = funs.getJF(u_fine, dt_fine)
      k = funs.getK(dt_fine, u_fine)
      return np.linalg.solve(jf.T - np.eye(jf.shape[0]), -k)

    def errorEstimate(funs, dt_n, u, v):  # factory.py:365-378
      dt_fine, n_steps = refineAll(dt_n)
      u_fine = interpU(dt_fine, dt_n, u)
      res = np.zeros_like(u_fine)
      for n in np.arange(n_steps) + 1:
        res[n] = u_fine[n] - funs.fwdUpdate(dt_fine, u_fine, n)
      return res * v

    def adapt(state, u0, plot=False):  # factory.py:305-344
      funs = FunFactory(state.problem).getFunctions()
      times = state.times_new
      dt_n = np.diff(times, 1)
      u = forwardSolve(funs, dt_n, u0)
      v = adjointSolve(funs, dt_n, u)
      err_steps = window_errors(errorEstimate(funs, dt_n, u, v), rf)
      ref_idx = int(np.argmax(err_steps))
      times_new = split_interval(times, ref_idx)
      state.iterate(err_steps, times, times_new, u, v)
      return state

    def plot(*_args, **_kw):  # presentation: out of scope
      return None

    def animate(*_args, **_kw):
      return None

    return AdaptFuns(adapt, adjointSolve, animate, errorEstimate, forwardSolve, interpU, plot,
                     refineAll)


# ---------------------------------------------------------------------------
# DG advection: spatial adaptivity driven by the GPU sweeps.
# ---------------------------------------------------------------------------
class DGProblem(NamedTuple):
  """Configuration of the DG adapt loop (the advection analogue of ``Problem``)."""
  case: str = "dg_advection"
  N: int = 4
  a: float = 2 * np.pi
  inflow: str = "a"              # "a": -sin(a t) (AdvecRHS1D.m:14), "a2": -sin(a^2 t)
  time_scheme: str = "lserk4"
  t0: float = 0.0
  nsteps: int = 20               # fixed step count per sweep
  cfl: float = 0.75              # dt = 0.5*cfl/(2 pi) * min|x1 - x2| (One_code.mlx:111-112)
  src_coef: float = 0.0          # J = <g, u^N> + src/2 sum_n |u^n|^2 ; g = u^N (J=|u^N|^2/2)


class DGAdaptState(AdaptState):
  """AdaptState over the mesh: ``times``/``times_new`` hold the vertex vectors."""

  @property
  def v_x(self):
    return self.times

  @property
  def v_x_new(self):
    return self.times_new


class DGFunFactory:
  """``getAdaptFunctions`` for the DG advection path (GPU)."""

  def __init__(self, problem: DGProblem):
    self.problem = problem

  def getAdaptFunctions(self) -> AdaptFuns:
    import torch

    from .operators import DGAdvection1D
    pb = self.problem

    def make(v_x):
      mesh = BaseGalerkin1D(n=pb.N, v_x=v_x)
      op = DGAdvection1D(mesh, a=pb.a, inflow=pb.inflow, time_scheme=pb.time_scheme)
      return mesh, op, mesh.cfl_dt(pb.cfl)

    def forwardSolve(op, dt, u0):
      """u0: CUDA tensor in device layout -> snapshots (nsteps+1, field)."""
      snaps = op.new_field(pb.nsteps + 1)
      snaps[0].copy_(u0)
      op.forward(snaps[0], pb.t0, dt, pb.nsteps, snaps)
      return snaps

    def adjointSolve(op, dt, snaps):
      """Terminal w^N = u^N (J = |u^N|^2/2); returns (dJ/du^0, eta)."""
      w = snaps[pb.nsteps].clone()
      eta = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
      op.adjoint(w, snaps, pb.t0, dt, pb.nsteps, src_coef=pb.src_coef, eta=eta)
      return w, eta

    def errorEstimate(op, dt, snaps, w_eta):
      return w_eta[1]

    def adapt(state, u0_fn, plot=False):
      """One spatial adapt iteration: solve on state.times_new (the mesh), estimate,
      split the element with the largest |eta| (first index on ties)."""
      v_x = np.asarray(state.times_new, dtype=np.float64)
      mesh, op, dt = make(v_x)
      u0 = torch.tensor(mesh.to_device_layout(u0_fn(mesh.x)), dtype=torch.float64,
                        device=op.device)
      snaps = forwardSolve(op, dt, u0)
      w_eta = adjointSolve(op, dt, snaps)
      eta = errorEstimate(op, dt, snaps, w_eta)
      idx = op.argmax(eta, use_abs=True)
      v_x_new = split_interval(v_x, idx)
      state.iterate(eta.abs().cpu().numpy(), v_x, v_x_new, snaps[pb.nsteps].cpu().numpy(),
                    w_eta[0].cpu().numpy())
      state.ref_idx = idx
      op.close()
      return state

    def refineAll(v_x):
      """Split every element once (uniform h-refinement of the mesh)."""
      v_x = np.asarray(v_x, dtype=np.float64)
      mids = 0.5 * (v_x[:-1] + v_x[1:])
      out = np.empty(2 * len(v_x) - 1)
      out[0::2] = v_x
      out[1::2] = mids
      return out, len(out) - 1

    def interpU(*_args, **_kw):
      raise NotImplementedError("state transfer between meshes is not needed: each adapt "
                                "iteration re-solves from the initial condition")

    def plot(*_args, **_kw):
      return None

    def animate(*_args, **_kw):
      return None

    return AdaptFuns(adapt, adjointSolve, animate, errorEstimate, forwardSolve, interpU, plot,
                     refineAll)
