"""Device-resident spatial adapt loop: BASELINE config 3 ("nonlinear advection with
SlopeLimitN, fwd + adj + err_contribution refine loop").

One iteration is the reference's adapt step (python/Main_finite_difference.py:263-343;
matlab/MAIN.m:29-141) on the DG mesh, with every array kept in HBM:

  u^0 = IC on the current mesh  ->  forward sweep (snapshots)  ->  adjoint sweep in place on
  u^N (J = |u^N|^2/2) accumulating the dual-weighted residual eta  ->  argmax |eta|  ->
  split that element on the device (dg_plan_refine)

The only host traffic per iteration is the refine index and the split element's width
(the next step size follows the CFL rule of utils/One_code.mlx:111-112 on the refined
mesh).  Buffers are sized once for ``max_refinements`` splits.
"""
import numpy as np
import torch

from .operators import DGAdvection1D


def check_indicator(value_at_refine_index, idx):
  """Failure detection for the adapt loop: the refine index comes from an
  argmax that ranks NaN and +-inf first, so the indicator is finite everywhere exactly
  when it is finite there.  A non-finite indicator (a blown-up sweep, e.g. a time step
  above the CFL limit) raises instead of refining element ``idx``."""
  if not np.isfinite(value_at_refine_index):
    raise FloatingPointError(f"non-finite DWR indicator ({value_at_refine_index}) at element "
                             f"{idx}: the forward or adjoint sweep diverged")


class AdaptiveSweep:
  """Fixed-step forward + adjoint sweeps and device refinement on one trajectory.

  Args:
    mesh: initial :class:`~.galerkin.BaseGalerkin1D`.
    nsteps: time steps per sweep (each direction).
    max_refinements: how many splits the buffers are sized for.
    flux, limiter, a, inflow: the plan's physics (config 3: "burgers", True).
    ic: (amplitude, frequency, phase) of u0 = A sin(2 pi m x + phi).
  """

  def __init__(self, mesh, nsteps, max_refinements, a=2 * np.pi, inflow="a", flux="burgers",
               limiter=True, cfl=0.75, ic=(1.0, 1.0, 0.0), t0=0.0):
    self.nsteps = int(nsteps)
    self.cfl = float(cfl)
    self.t0 = float(t0)
    self.ic = tuple(float(v) for v in ic)
    self.op = DGAdvection1D(mesh, a=a, inflow=inflow, flux=flux, limiter=limiter)
    k_cap = mesh.k + int(max_refinements)
    self.op.reserve(k_cap)
    dev = self.op.device
    self._snaps = torch.empty((self.nsteps + 1) * k_cap * mesh.n_p, dtype=torch.float64,
                              device=dev)
    self._eta = torch.zeros(k_cap, dtype=torch.float64, device=dev)
    # the forward sweep's limiter decisions, read back by the adjoint (dg_lserk4_fwd_ex)
    self._codes = (torch.zeros(self.nsteps * k_cap, dtype=torch.int16, device=dev)
                   if self.op.limiter else None)
    self.idx = torch.zeros(1, dtype=torch.int64, device=dev)
    self.h_split = torch.zeros(1, dtype=torch.float64, device=dev)
    # min |x_1 - x_2| over elements = h_min * (r_1 - r_0) / 2 (LGL nodes are affine images)
    self._half_gap = 0.5 * float(mesh.r_gl[1] - mesh.r_gl[0])
    self.h_min = float(np.min(np.diff(mesh.v_x)))
    self._length = float(np.max(np.abs(mesh.v_x)))
    self.history = []

  @property
  def K(self):
    return self.op.K

  @property
  def dt(self):
    """One_code.mlx:111-112: 0.5 * CFL/(2 pi) * min|x_1 - x_2| on the current mesh."""
    return 0.5 * (self.cfl / (2 * np.pi) * (self.h_min * self._half_gap))

  def snapshots(self):
    n = self.op.field_numel
    return self._snaps[:(self.nsteps + 1) * n].view(self.nsteps + 1, n)

  def eta(self):
    return self._eta[:self.op.ktot]

  def init_state(self):
    """u^0 = the IC on the current mesh (snapshot 0).  (eta needs no reset: the adjoint's
    first launch assigns it, DG_ADJ_ETA_ASSIGN.)"""
    amp, freq, phase = self.ic
    self.op.init_sine([amp], [freq], [phase], out=self.snapshots()[0])

  def decisions(self):
    return None if self._codes is None else self._codes[:self.nsteps * self.op.ktot]

  def forward(self, dt=None, init=True):
    """init_state() (unless init=False: the caller did it) then the forward sweep."""
    snaps = self.snapshots()
    if init:
      self.init_state()
    self.op.forward(snaps[0], self.t0, self.dt if dt is None else dt, self.nsteps, snaps,
                    decisions=self.decisions())
    return snaps

  def adjoint(self, dt=None):
    """The adjoint sweep writing eta (assigned by its first launch), with the forward's
    recorded limiter decisions."""
    snaps = self.snapshots()
    eta = self.eta()
    # J = |u^N|^2 / 2: the terminal adjoint is u^N itself; the sweep runs in place on it.
    self.op.adjoint(snaps[self.nsteps], snaps, self.t0, self.dt if dt is None else dt,
                    self.nsteps, eta=eta, eta_assign=True, decisions=self.decisions())
    return eta

  def refine(self):
    """argmax |eta| and the device split; returns the DOF-updates of the iteration's sweeps
    (2 Np K nsteps on the mesh they ran on).  Asynchronous: call ``sync`` before the next
    iteration needs the step size."""
    dofs = 2 * self.op.Np * self.op.ktot * self.nsteps
    self.op.argmax_async(self.eta(), use_abs=True, out=self.idx)
    # argmax puts NaN (and |inf|) first, so eta at the refine index is finite iff all are
    self._eta_at = self._eta.index_select(0, self.idx)
    self.op.refine(self.idx, self.h_split)
    return dofs

  def sync(self):
    """Bring the refine index and the split width to the host; update h_min."""
    idx = int(self.idx.item())
    check_indicator(float(self._eta_at.item()), idx)
    h_new = 0.5 * float(self.h_split.item())
    if not h_new > 64 * np.finfo(np.float64).eps * self._length:
      raise FloatingPointError(f"refining element {idx} left elements of width {h_new:g}: "
                               "the split has reached fp64 resolution of the coordinates")
    self.h_min = min(self.h_min, h_new)
    self.history.append(idx)
    return idx

  def iterate(self):
    dt = self.dt
    self.forward(dt)
    self.adjoint(dt)
    dofs = self.refine()
    return dofs, self.sync()
