"""GPU DG advection operator: the Python face of the HIP plan (include/dg_advec.h).

``DGAdvection1D`` replaces the MATLAB global-state calls of the reference hot path:

=================================  ===============================================
reference                           here
=================================  ===============================================
``AdvecRHS1D(u, t, a)``             ``op.rhs(u, t)``          (utils/AdvecRHS1D.m:1)
LSERK4 loop, One_code.mlx:106-140   ``op.forward(u, t0, dt, nsteps, snapshots)``
``adj_march`` / adjSolve role       ``op.adjoint(w, snapshots, t0, dt, nsteps, ...)``
``err_contribution`` / errEst role  the ``eta`` output of ``op.adjoint``
``SlopeLimitN(u)``                  ``op.slope_limit(u)``      (utils/SlopeLimitN.m:1)
``argmax(err)`` (:337)              ``op.argmax(eta, use_abs=True)``
split of :336-341 / MAIN.m:137-141  ``op.refine(idx)`` (on the device)
=================================  ===============================================

``flux="burgers"`` and/or ``limiter=True`` select the config-3 physics (BASELINE.json
configs[2]): the build-defined flux a*u^2/2 with AdvecRHS1D's central-flux structure and
SlopeLimitN after every LSERK4 stage (see include/dg_advec.h ``dg_plan_set_physics``).

Tensors are torch CUDA float64 tensors in the device layout (element-major,
``u[(b*K + k)*Np + i]``); any shape with that many contiguous elements is accepted.
Work is enqueued on torch's current stream.  There is no CPU path: a CPU tensor or a
missing library raises.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .galerkin import BaseGalerkin1D, prolongation

INFLOW = {"a": _lib.DG_INFLOW_SIN_AT, "a2": _lib.DG_INFLOW_SIN_A2T, "zero": _lib.DG_INFLOW_ZERO}
SCHEME = {"lserk4": _lib.DG_TIME_LSERK4, "euler": _lib.DG_TIME_EULER}
FLUX = {"linear": _lib.DG_FLUX_LINEAR, "burgers": _lib.DG_FLUX_BURGERS}
LIMITER = {False: _lib.DG_LIMIT_NONE, True: _lib.DG_LIMIT_EACH_STAGE,
           "N": _lib.DG_LIMIT_EACH_STAGE, "1": _lib.DG_LIMIT_PI1_EACH_STAGE}


def _stream(device):
  return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class DGAdvection1D:
  """A plan for ``batch`` trajectories of 1D linear advection on one nodal-DG mesh.

  Args:
    mesh: a :class:`BaseGalerkin1D` (its ``r_gl``, ``v``, ``inv_v``, ``d_r``, ``lift``,
      ``v_x`` are handed to the plan), or an int polynomial order together with ``v_x``.
    a: advection speed (One_code.mlx:116 uses 2*pi).
    batch: independent trajectories (ensemble ICs) sharing the mesh.
    inflow: "a" (uin = -sin(a t), AdvecRHS1D.m:14), "a2" (-sin(a^2 t), One_code.mlx:129) or
      "zero" (uin = 0, the homogeneous problem).
    time_scheme: "lserk4" (Globals1D.m:19-34) or "euler".
    flux: "linear" (a*u, AdvecRHS1D) or "burgers" (a*u^2/2, build-defined, config 3).
    limiter: after every LSERK4 stage apply SlopeLimitN (True or "N", utils/SlopeLimitN.m)
      or SlopeLimit1 ("1", utils/SlopeLimit1.m: every cell limited); False: none.
  """

  def __init__(self, mesh, a=2 * np.pi, batch=1, inflow="a", time_scheme="lserk4",
               v_x=None, device=None, flux="linear", limiter=False):
    if not isinstance(mesh, BaseGalerkin1D):
      mesh = BaseGalerkin1D(n=int(mesh), v_x=v_x)
    if not torch.cuda.is_available():
      raise _lib.DGLibraryError("DGAdvection1D needs a ROCm GPU (torch.cuda is unavailable)")
    self.mesh = mesh
    self.a = float(a)
    self.batch = int(batch)
    self.inflow = inflow
    self.time_scheme = time_scheme
    self.N = mesh.n
    self.Np = mesh.n_p
    self.K = mesh.k
    self.ktot = self.K * self.batch
    self.field_numel = self.ktot * self.Np
    self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    lib = _lib.load()
    keep = [_lib.dbl_array(x) for x in (mesh.r_gl, mesh.v, mesh.inv_v, mesh.d_r, mesh.lift,
                                        mesh.v_x)]
    handle = ctypes.c_void_p()
    with torch.cuda.device(self.device):
      rc = lib.dg_plan_create(self.N, self.K, self.batch, *[p for _, p in keep], self.a,
                              INFLOW[inflow], SCHEME[time_scheme], ctypes.byref(handle))
    _lib.check(rc, "dg_plan_create")
    self._plan = handle
    self._lib = lib
    self.flux = flux
    if limiter not in LIMITER:
      raise ValueError(f"limiter must be one of {sorted(LIMITER, key=str)}, got {limiter!r}")
    self.limiter = bool(limiter)
    self.limiter_kind = {0: None, 1: "N", 2: "1"}[LIMITER[limiter]]
    if flux != "linear" or limiter:
      _lib.check(lib.dg_plan_set_physics(handle, FLUX[flux], LIMITER[limiter]),
                 "dg_plan_set_physics")
    self._query()
    self._idx = torch.zeros(1, dtype=torch.int64, device=self.device)

  def _query(self):
    q = (ctypes.c_int64 * 8)()
    _lib.check(self._lib.dg_plan_query(self._plan, q), "dg_plan_query")
    self.K = int(q[2])
    self.ktot = self.K * self.batch
    self.field_numel = self.ktot * self.Np
    self.uniform = bool(q[4])
    self.stages = int(q[5])
    self.tile_width = int(q[6])
    self.steps_per_launch = int(q[7])
    r = (ctypes.c_int64 * 4)()
    _lib.check(self._lib.dg_plan_query_rec(self._plan, r), "dg_plan_query_rec")
    self.rec_tile_width = int(r[0])  # the jump-record sweeps' shape
    self.rec_steps_per_launch = int(r[1])
    self.rec_lane_elements = int(r[2])
    self.rec_fwd_steps_per_launch = int(r[3])
    f = (ctypes.c_int64 * 2)()
    _lib.check(self._lib.dg_plan_query_rec_fwd(self._plan, f), "dg_plan_query_rec_fwd")
    self.rec_fwd_tile_width = int(f[0])
    n = (ctypes.c_int64 * 3)()
    _lib.check(self._lib.dg_plan_query_nl(self._plan, n), "dg_plan_query_nl")
    # the config-3 kernels: exchange (0 workgroup tiles, 1 overlapped waves), forward steps
    # per launch with / without snapshots
    self.nl_exchange = int(n[0])
    self.nl_steps_per_launch = (int(n[1]), int(n[2]))

  # --- lifetime ---
  def close(self):
    if getattr(self, "_plan", None):
      self._lib.dg_plan_destroy(self._plan)
      self._plan = None

  def __del__(self):
    try:
      self.close()
    except Exception:  # interpreter shutdown
      pass

  def __enter__(self):
    return self

  def __exit__(self, *exc):
    self.close()

  def tune(self, tile_width=None, steps_per_launch=None, xcd_order=None, lane_elements=None,
           rec_tile_width=None, rec_steps_per_launch=None, rec_lane_elements=None,
           rec_fwd_steps_per_launch=None, rec_fwd_tile_width=None, rec_sweep=None,
           sweep_waves=None, sweep_lane_elements=None, sweep_take=None, sweep_exchange=None,
           snap_pairs=None, nl_exchange=None):
    """Shape of the fused step kernels: tiles of 256*``tile_width`` elements (1 or 2; one
    element per lane), ``steps_per_launch`` (1, 2, 4, or 8 on 512-element tiles) time steps
    fused per launch, and
    ``xcd_order`` gives each XCD a contiguous range of tiles.  Tile width and order do not
    change the arithmetic; steps per launch changes it at rounding level (the state stays
    in even/odd coordinates between fused steps).  ``rec_tile_width`` (1, 2) and
    ``rec_steps_per_launch`` shape the jump-record sweeps (``forward_rec``/``adjoint_rec``);
    ``rec_lane_elements`` = 2 runs them with two consecutive elements per lane (tiles of
    512*``rec_tile_width`` elements, bit-identical at equal steps per launch);
    ``rec_fwd_steps_per_launch`` gives the forward its own steps per launch (setting
    ``rec_steps_per_launch`` applies to both directions and clears it);
    ``rec_fwd_tile_width`` likewise gives the forward its own tile width (0: the adjoint's;
    setting ``rec_tile_width`` applies to both).  ``rec_sweep`` (1, default / 0): ``sweep_rec``
    runs both directions as one dataflow launch where the shape allows, or as the two launch
    chains (bit-identical).  ``sweep_waves`` (0 / 4 / 8 / 12 / 16): the dataflow launch's
    workgroup waves, tiles of 128 * waves elements in both directions (0: as the record tile
    width; bit-identical at any value); ``sweep_lane_elements`` (2, or 4 at N <= 2): consecutive
    elements per lane of its tiles; ``sweep_take`` (0 / 1): its work items from one take
    counter or by workgroup id (bit-identical); ``sweep_exchange`` (0 / 1): its tiles exchange
    faces through LDS with a barrier per Horner level, or on overlapped waves by DPP with one
    LDS exchange and barrier per step (tiles of waves * 116 + 12 elements; bit-identical);
    ``snap_pairs`` (0 / 1): ``forward`` with snapshots on the stage-loop kernels or on
    Horner-form pair tiles (512 * ``tile_width`` elements, ``steps_per_launch`` steps per
    launch; equal to rounding).  ``nl_exchange`` (0 / 1): the config-3 kernels (``flux`` /
    ``limiter``) on workgroup tiles exchanging through LDS with a barrier per exchange, or on
    overlapped waves exchanging by DPP with no barrier inside a step (bit-identical)."""
    for key, val in ((_lib.DG_TUNE_REC_TILE_WIDTH, rec_tile_width),
                     (_lib.DG_TUNE_REC_SWEEP, rec_sweep),
                     (_lib.DG_TUNE_REC_STEPS_PER_LAUNCH, rec_steps_per_launch),
                     (_lib.DG_TUNE_REC_LANE_ELEMENTS, rec_lane_elements),
                     (_lib.DG_TUNE_REC_FWD_STEPS_PER_LAUNCH, rec_fwd_steps_per_launch),
                     (_lib.DG_TUNE_REC_FWD_TILE_WIDTH, rec_fwd_tile_width),
                     (_lib.DG_TUNE_SWEEP_WAVES, sweep_waves),
                     (_lib.DG_TUNE_SWEEP_LANE_ELEMENTS, sweep_lane_elements),
                     (_lib.DG_TUNE_SWEEP_TAKE, sweep_take),
                     (_lib.DG_TUNE_SWEEP_EXCHANGE, sweep_exchange),
                     (_lib.DG_TUNE_SNAP_PAIRS, snap_pairs),
                     (_lib.DG_TUNE_NL_EXCHANGE, nl_exchange)):
      if val is not None:
        _lib.check(self._lib.dg_plan_tune(self._plan, key, int(val)), "dg_plan_tune")
    if xcd_order is not None:
      _lib.check(self._lib.dg_plan_tune(self._plan, _lib.DG_TUNE_XCD_ORDER, int(xcd_order)),
                 "dg_plan_tune")
    if lane_elements is not None:  # forward steps on one-wave tiles (0 = workgroup tiles)
      _lib.check(self._lib.dg_plan_tune(self._plan, _lib.DG_TUNE_LANE_ELEMENTS,
                                        int(lane_elements)), "dg_plan_tune")
    if tile_width is not None:
      _lib.check(self._lib.dg_plan_tune(self._plan, _lib.DG_TUNE_TILE_WIDTH,
                                        int(tile_width)), "dg_plan_tune")
    if steps_per_launch is not None:
      _lib.check(self._lib.dg_plan_tune(self._plan, _lib.DG_TUNE_STEPS_PER_LAUNCH,
                                        int(steps_per_launch)), "dg_plan_tune")
    self._query()
    return self

  # --- mesh refinement on the device ---
  def reserve(self, k_capacity):
    """Size the plan's device buffers for meshes of up to ``k_capacity`` elements."""
    _lib.check(self._lib.dg_plan_reserve(self._plan, int(k_capacity)), "dg_plan_reserve")
    return self

  def refine(self, idx, h_split=None):
    """Split element ``idx`` (a 1-element CUDA int64 tensor, e.g. ``argmax_async``'s
    output) at its midpoint on the device (Main_finite_difference.py:336-341,
    MAIN.m:137-141).  K grows by one; fields of the old size must be re-initialised.
    ``h_split`` (1-element CUDA float64, optional) receives the split element's width."""
    if not isinstance(idx, torch.Tensor) or not idx.is_cuda or idx.dtype != torch.int64:
      raise TypeError("idx must be a CUDA int64 tensor")
    hp = None
    if h_split is not None:
      if not h_split.is_cuda or h_split.dtype != torch.float64:
        raise TypeError("h_split must be a CUDA float64 tensor")
      hp = ctypes.c_void_p(h_split.data_ptr())
    rc = self._lib.dg_plan_refine(self._plan, ctypes.c_void_p(idx.data_ptr()), hp,
                                  _stream(self.device))
    _lib.check(rc, "dg_plan_refine")
    self._query()
    return self.K

  def v_x(self):
    """The plan's current vertex coordinates (host copy; synchronises)."""
    out = np.empty(self.K + 1)
    rc = self._lib.dg_plan_get_mesh(self._plan, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    _lib.check(rc, "dg_plan_get_mesh")
    return out

  # --- checks ---
  def _field(self, t, name, numel=None, dtype=torch.float64):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
      raise TypeError(f"{name} must be a CUDA tensor (no CPU path)")
    if t.dtype != dtype:
      raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
      raise ValueError(f"{name} must be contiguous")
    want = self.field_numel if numel is None else numel
    if t.numel() != want:
      raise ValueError(f"{name} has {t.numel()} elements, expected {want}")
    return ctypes.c_void_p(t.data_ptr())

  def new_field(self, count=None):
    shape = (self.field_numel,) if count is None else (count, self.field_numel)
    return torch.empty(shape, dtype=torch.float64, device=self.device)

  # --- kernels ---
  def rhs(self, u, t, out=None):
    """AdvecRHS1D(u, t, a) (utils/AdvecRHS1D.m:1-20)."""
    out = torch.empty_like(u) if out is None else out
    rc = self._lib.dg_advec_rhs(self._plan, self._field(u, "u"), self._field(out, "out"),
                                float(t), _stream(self.device))
    _lib.check(rc, "dg_advec_rhs")
    return out

  def _decisions(self, decisions, nsteps):
    if decisions is None:
      return None
    if (not isinstance(decisions, torch.Tensor) or not decisions.is_cuda
        or decisions.dtype != torch.int16 or not decisions.is_contiguous()):
      raise TypeError("decisions must be a contiguous CUDA int16 tensor (uint16 bits)")
    if decisions.numel() < nsteps * self.ktot:
      raise ValueError(f"decisions holds {decisions.numel()} words, need {nsteps * self.ktot}")
    return ctypes.c_void_p(decisions.data_ptr())

  def forward(self, u, t0, dt, nsteps, snapshots=None, decisions=None):
    """nsteps fused steps in place on u (One_code.mlx:119-140); optional snapshots
    ((nsteps+1) * field) receive u^0..u^nsteps.  ``decisions`` (CUDA int16, nsteps*batch*K;
    plans with a per-stage limiter) records the limiter's per-stage decisions for
    ``adjoint`` (dg_lserk4_fwd_ex)."""
    snap_p = None
    if snapshots is not None:
      snap_p = self._field(snapshots, "snapshots", (nsteps + 1) * self.field_numel)
    rc = self._lib.dg_lserk4_fwd_ex(self._plan, self._field(u, "u"), float(t0), float(dt),
                                    int(nsteps), snap_p, self._decisions(decisions, nsteps),
                                    _stream(self.device))
    _lib.check(rc, "dg_lserk4_fwd_ex")
    return u

  def adjoint(self, w, snapshots, t0, dt, nsteps, src_coef=0.0, eta=None, eta_assign=False,
              eta_abs=False, decisions=None):
    """Discrete adjoint sweep in place on w (terminal dJ/du^N in, dJ/du^0 out) and the
    dual-weighted residual accumulated into eta (batch*K, caller-zeroed).

    ``eta_assign``: eta is assigned instead of accumulated (no zero fill needed);
    ``eta_abs``: eta ends as |eta| (Main_width_ref.py:139 ``jnp.abs(err)``).  Both are
    folded into the sweep's first / last launch (dg_lserk4_adj_ex).  ``decisions``: the
    record ``forward`` wrote for these snapshots (limited plans): the frozen limiter
    decisions are read instead of re-tested (bit-identical results, less work)."""
    eta_p = None if eta is None else self._field(eta, "eta", self.ktot)
    flags = (_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) | (_lib.DG_ADJ_ETA_ABS if eta_abs else 0)
    rc = self._lib.dg_lserk4_adj_ex(self._plan, self._field(w, "w"),
                                    self._field(snapshots, "snapshots",
                                                (nsteps + 1) * self.field_numel),
                                    float(t0), float(dt), int(nsteps), float(src_coef), eta_p,
                                    int(flags), self._decisions(decisions, nsteps),
                                    _stream(self.device))
    _lib.check(rc, "dg_lserk4_adj_ex")
    return w, eta

  # --- snapshot-free sweep pair (linear LSERK4 plans, terminal functionals) ---
  @property
  def jump_ld(self):
    """Row length of the jump record: batch*K rounded up to even (16-byte aligned rows)."""
    return (self.ktot + 1) & ~1

  def new_jumps(self, nsteps):
    """A jump record for an ``nsteps`` sweep: (nsteps, jump_ld) float64; row n-1, entry e is
    u^n's left-face jump u_0 - uL of element e (include/dg_advec.h)."""
    return torch.empty((int(nsteps), self.jump_ld), dtype=torch.float64, device=self.device)

  def _jumps(self, jumps, nsteps):
    return self._field(jumps, "jumps", int(nsteps) * self.jump_ld)

  def forward_rec(self, u0, t0, dt, nsteps, jumps, out=None):
    """``nsteps`` LSERK4 steps from u0 into ``out`` (default: in place on u0), recording
    per element and step the left-face jump of each state u^1..u^nsteps instead of the states
    (dg_lserk4_fwd_rec: 8 bytes per element-step for 8*Np).  With
    ``adjoint_rec`` this is the snapshot sweep pair with src_coef = 0, bit for bit."""
    out = u0 if out is None else out
    rc = self._lib.dg_lserk4_fwd_rec(self._plan, self._field(u0, "u0"), self._field(out, "out"),
                                     float(t0), float(dt), int(nsteps),
                                     self._jumps(jumps, nsteps), _stream(self.device))
    _lib.check(rc, "dg_lserk4_fwd_rec")
    return out

  def adjoint_rec(self, w, jumps, t0, dt, nsteps, eta=None, eta_assign=False, eta_abs=False):
    """``adjoint`` (src_coef = 0) from the record ``forward_rec`` wrote for this sweep."""
    eta_p = None if eta is None else self._field(eta, "eta", self.ktot)
    flags = (_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) | (_lib.DG_ADJ_ETA_ABS if eta_abs else 0)
    rc = self._lib.dg_lserk4_adj_rec(self._plan, self._field(w, "w"), self._jumps(jumps, nsteps),
                                     float(t0), float(dt), int(nsteps), eta_p, int(flags),
                                     _stream(self.device))
    _lib.check(rc, "dg_lserk4_adj_rec")
    return w, eta

  def sweep_rec(self, u0, jumps, w, t0, dt, nsteps, uN=None, eta=None, eta_assign=False,
                eta_abs=False, terminal_state=True):
    """``forward_rec`` + ``adjoint_rec`` in one call (dg_lserk4_sweep_rec): u0 -> u^nsteps
    (into ``uN`` if given), then the adjoint into ``w`` (w^0 on exit) from the terminal weight
    u^nsteps (``terminal_state``: J = |u^N|^2/2, w's content ignored) or from w itself.  Where
    the record shape allows, both directions run as one dataflow launch (``query_sweep``);
    the results are bit-identical to the two calls either way."""
    eta_p = None if eta is None else self._field(eta, "eta", self.ktot)
    un_p = None if uN is None else self._field(uN, "uN")
    flags = ((_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) |
             (_lib.DG_ADJ_ETA_ABS if eta_abs else 0) |
             (_lib.DG_SWEEP_TERMINAL_STATE if terminal_state else 0))
    rc = self._lib.dg_lserk4_sweep_rec(self._plan, self._field(u0, "u0"), un_p,
                                       self._field(w, "w"), self._jumps(jumps, nsteps),
                                       float(t0), float(dt), int(nsteps), eta_p, int(flags),
                                       _stream(self.device))
    _lib.check(rc, "dg_lserk4_sweep_rec")
    return w, eta

  def sweep_refine(self, u0, jumps, w, t0, dt, nsteps, eta, idx, value=None, nonfinite=None,
                   uN=None, eta_assign=True, eta_abs=True, terminal_state=True):
    """``sweep_rec`` + the refine decision ``argmax_ex(eta, use_abs=True)`` in one call
    (dg_lserk4_sweep_refine): in the dataflow launch the last adjoint tiles reduce the argmax
    themselves.  ``idx`` / ``nonfinite`` (CUDA int64, 1) and ``value`` (CUDA float64, 1) as
    for ``argmax_ex``."""
    def p1(t, dtype, name):
      if t is None:
        return None
      if isinstance(t, int):  # a device address (host_alias of pinned host memory)
        return ctypes.c_void_p(t)
      if not t.is_cuda or t.dtype != dtype or t.numel() < 1:
        raise TypeError(f"{name} must be a CUDA {dtype} tensor or a device address")
      return ctypes.c_void_p(t.data_ptr())
    flags = ((_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) |
             (_lib.DG_ADJ_ETA_ABS if eta_abs else 0) |
             (_lib.DG_SWEEP_TERMINAL_STATE if terminal_state else 0))
    un_p = None if uN is None else self._field(uN, "uN")
    rc = self._lib.dg_lserk4_sweep_refine(
        self._plan, self._field(u0, "u0"), un_p, self._field(w, "w"), self._jumps(jumps, nsteps),
        float(t0), float(dt), int(nsteps), self._field(eta, "eta", self.ktot), int(flags),
        p1(idx, torch.int64, "idx"), p1(value, torch.float64, "value"),
        p1(nonfinite, torch.int64, "nonfinite"), _stream(self.device))
    _lib.check(rc, "dg_lserk4_sweep_refine")
    return idx

  def query_sweep(self, nsteps, tile=False):
    """(dataflow, forward steps per block, adjoint steps per block, work items) of
    ``sweep_rec`` for an ``nsteps`` sweep; dataflow False: the two launch chains run.
    ``tile``: also (workgroup waves, elements per tile)."""
    q = (ctypes.c_int64 * 6)()
    _lib.check(self._lib.dg_plan_query_sweep_ex(self._plan, int(nsteps), q),
               "dg_plan_query_sweep_ex")
    out = (bool(q[0]), int(q[1]), int(q[2]), int(q[3]))
    return out + (int(q[4]), int(q[5])) if tile else out

  def query_sweep_kernel(self, nsteps):
    """The dataflow launch's kernel for an ``nsteps`` sweep, as a profile must match it:
    dict(Np, uniform, waves, msf, msa, lane_elements, exchange, waves_per_simd, name) with
    name the rocprof kernel name prefix ``k_sweep_rp<Np, uniform, waves, msf, msa, E, X>``;
    None when ``sweep_rec`` runs the two launch chains."""
    q = (ctypes.c_int64 * 8)()
    _lib.check(self._lib.dg_plan_query_sweep_kernel(self._plan, int(nsteps), q),
               "dg_plan_query_sweep_kernel")
    if q[0] == 0:
      return None
    keys = ("Np", "uniform", "waves", "msf", "msa", "lane_elements", "exchange",
            "waves_per_simd")
    d = {k: int(v) for k, v in zip(keys, q)}
    d["name"] = (f"k_sweep_rp<{d['Np']}, {'true' if d['uniform'] else 'false'}, {d['waves']}, "
                 f"{d['msf']}, {d['msa']}, {d['lane_elements']}, {d['exchange']}>")
    return d

  def sweep_trace(self, trace):
    """Profiling: record per work item of every later dataflow sweep {taken, producers done,
    published (wall clock, 100 MHz), XCC id << 32 | workgroup} into ``trace`` (CUDA int64,
    4 * ``query_sweep(nsteps)[3]`` entries for the jump sweep; the p launches write 8 per
    item: size it with ``DWREstimate.trace_words``); None turns it off."""
    ptr = None
    if trace is not None:
      if not trace.is_cuda or trace.dtype != torch.int64 or not trace.is_contiguous():
        raise TypeError("trace must be a contiguous CUDA int64 tensor")
      ptr = ctypes.c_void_p(trace.data_ptr())
    _lib.check(self._lib.dg_plan_sweep_trace(self._plan, ptr), "dg_plan_sweep_trace")
    self._trace = trace

  def sweep_status(self):
    """0, or 1 if a dataflow sweep since the last call gave up waiting for a producer (its
    outputs are garbage); synchronises the device stream."""
    st = ctypes.c_int(0)
    _lib.check(self._lib.dg_sweep_status(self._plan, ctypes.byref(st), _stream(self.device)),
               "dg_sweep_status")
    return int(st.value)

  def set_tvb(self, M):
    """The TVB constant of ``slope_limit`` / ``slope_limit_1`` (utils/minmodB.m: the element's
    own slope is kept unless |ux| > M h^2); 0 restores the plain minmod (dg_plan_set_tvb)."""
    _lib.check(self._lib.dg_plan_set_tvb(self._plan, float(M)), "dg_plan_set_tvb")
    self.tvb_M = float(M)
    return self

  def slope_limit(self, u, out=None, ids=None):
    """SlopeLimitN(u) (utils/SlopeLimitN.m:1-33); ids (int32, batch*K) marks limited cells."""
    out = torch.empty_like(u) if out is None else out
    ids_p = None if ids is None else self._field(ids, "ids", self.ktot, torch.int32)
    rc = self._lib.dg_slope_limit_n(self._plan, self._field(u, "u"), self._field(out, "out"),
                                    ids_p, _stream(self.device))
    _lib.check(rc, "dg_slope_limit_n")
    return out

  def slope_limit_1(self, u, out=None):
    """SlopeLimit1(u) (utils/SlopeLimit1.m:1-23): the Pi^1 limiter on every element."""
    out = torch.empty_like(u) if out is None else out
    rc = self._lib.dg_slope_limit_1(self._plan, self._field(u, "u"), self._field(out, "out"),
                                    _stream(self.device))
    _lib.check(rc, "dg_slope_limit_1")
    return out

  def argmax_async(self, x, use_abs=True, out=None):
    """Device-side argmax (numpy semantics) into a 1-element int64 tensor."""
    out = self._idx if out is None else out
    n = x.numel()
    if not x.is_cuda or x.dtype != torch.float64 or not x.is_contiguous():
      raise TypeError("x must be a contiguous CUDA float64 tensor")
    rc = self._lib.dg_argmax(self._plan, ctypes.c_void_p(x.data_ptr()), n, int(use_abs),
                             ctypes.c_void_p(out.data_ptr()), _stream(self.device))
    _lib.check(rc, "dg_argmax")
    return out

  def argmax(self, x, use_abs=True):
    return int(self.argmax_async(x, use_abs).item())

  def argmax_ex(self, x, idx, value=None, nonfinite=None, use_abs=True):
    """argmax into ``idx`` (1-element CUDA int64) plus, on the device, the winning value into
    ``value`` (1-element CUDA float64) and +1 into ``nonfinite`` (1-element CUDA int64) when
    that value is not finite (dg_argmax_ex; no host sync)."""
    n = x.numel()
    if not x.is_cuda or x.dtype != torch.float64 or not x.is_contiguous():
      raise TypeError("x must be a contiguous CUDA float64 tensor")
    for t, name, dt_ in ((idx, "idx", torch.int64), (value, "value", torch.float64),
                         (nonfinite, "nonfinite", torch.int64)):
      if t is not None and (not t.is_cuda or t.dtype != dt_ or t.numel() < 1):
        raise TypeError(f"{name} must be a CUDA {dt_} tensor")
    ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rc = self._lib.dg_argmax_ex(self._plan, ctypes.c_void_p(x.data_ptr()), n, int(use_abs),
                                ptr(idx), ptr(value), ptr(nonfinite), _stream(self.device))
    _lib.check(rc, "dg_argmax_ex")
    return idx

  def slice_candidate(self, x, n, divisor, offset, cand):
    """This rank's refine candidate from its received slices x (rows, ld) CUDA float64:
    cand (CUDA int64[2]) = (bits of |m[i]|, i + offset), m = the rows' ascending sum over the
    first n columns / divisor, i = argmax |m| (dg_slice_candidate; no host sync)."""
    if not x.is_cuda or x.dtype != torch.float64 or x.dim() != 2 or not x.is_contiguous():
      raise TypeError("x must be a contiguous 2-D CUDA float64 tensor")
    if not cand.is_cuda or cand.dtype != torch.int64 or cand.numel() < 2:
      raise TypeError("cand must be a CUDA int64 tensor of 2 elements")
    rows, ld = x.shape
    rc = self._lib.dg_slice_candidate(self._plan, ctypes.c_void_p(x.data_ptr()), int(rows),
                                      int(n), int(ld), float(divisor), int(offset),
                                      ctypes.c_void_p(cand.data_ptr()), _stream(self.device))
    _lib.check(rc, "dg_slice_candidate")
    return cand

  def init_sine(self, amp, freq, phase, out=None):
    """u_b(x) = amp[b] sin(2 pi freq[b] x + phase[b]) on the device (ensemble ICs)."""
    out = self.new_field() if out is None else out
    vals = [torch.as_tensor(np.asarray(v, dtype=np.float64), device=self.device)
            for v in (amp, freq, phase)]
    for v in vals:
      if v.numel() != self.batch:
        raise ValueError("amp/freq/phase need one value per trajectory")
    rc = self._lib.dg_init_sine(self._plan, *[ctypes.c_void_p(v.data_ptr()) for v in vals],
                                self._field(out, "u"), _stream(self.device))
    _lib.check(rc, "dg_init_sine")
    return out


class DWREstimate:
  """The p-enriched dual-weighted-residual ERROR ESTIMATE of a linear LSERK4 plan (SURVEY
  8(a) row 8; include/dg_advec.h ``dg_lserk4_adj_p``).

  The reference estimates the error of its order-Ns solution with an adjoint marched one
  order up (matlab/MAIN.m:32-34, adj_march.m:103-117: err(k) = v_k'(-A uh_k - M~ + F)) and
  documents its FD variant as "the Adjoint-Weighted Residual as an error estimate"
  (python/Main_finite_difference.py:79-94).  Here: P u_h prolongs the order-N snapshots to
  order N+1, R^n = P u^{n+1} - S_{N+1}(P u^n) is the enriched scheme's one-step residual and
  eta_k = -sum_n w^{n+1}_k . R^n_k with w the order-(N+1) discrete adjoint, so that
  sum_k eta_k = J_{N+1}(u_{N+1}) - J_{N+1}(P u_h) for a linear functional (the DWR identity).

  ``hi`` is the order-(N+1) plan on the lo plan's current mesh (its ``forward`` marches
  u_{N+1} for the identity); ``P`` the prolongation (galerkin.prolongation)."""

  def __init__(self, lo, tile_width=None, steps_per_launch=None):
    if lo.flux != "linear" or lo.limiter or lo.time_scheme != "lserk4":
      raise ValueError("the p-estimate is the linear LSERK4 sweep's")
    if lo.N > 7:
      raise ValueError("the p-estimate supports N <= 7 (the enriched plan needs N+1 <= 8)")
    self.lo = lo
    v_x = lo.v_x()  # the lo plan's current (possibly device-refined) mesh
    mesh_lo = BaseGalerkin1D(n=lo.N, v_x=v_x)
    self.mesh_hi = BaseGalerkin1D(n=lo.N + 1, v_x=v_x)
    self.hi = DGAdvection1D(self.mesh_hi, a=lo.a, batch=lo.batch, inflow=lo.inflow,
                            device=lo.device.index)
    self.P = prolongation(mesh_lo, self.mesh_hi)
    self._P, self._P_ptr = _lib.dbl_array(self.P)
    self.tune(tile_width, steps_per_launch)

  def tune(self, tile_width=None, steps_per_launch=None, flow=None, sweep=None):
    """Tiles of 256*``tile_width`` elements (1, 2) and ``steps_per_launch`` (1, 2, 4; 8 on
    512-element tiles) reverse steps per launch of dg_lserk4_adj_p; ``flow`` (0 / 1): one
    launch per block, or the whole estimate as one dataflow launch where the steps split
    into 2 or more blocks of 4 (or 8 on 512-element tiles) steps (bit-identical); ``sweep``
    (0 / 1): ``sweep`` as the chains or as one dataflow launch (bit-identical)."""
    lib, plan = self.lo._lib, self.lo._plan
    if sweep is not None:
      _lib.check(lib.dg_plan_tune(plan, _lib.DG_TUNE_P_SWEEP, int(sweep)), "dg_plan_tune")
    if flow is not None:
      _lib.check(lib.dg_plan_tune(plan, _lib.DG_TUNE_P_FLOW, int(flow)), "dg_plan_tune")
    if tile_width is not None:
      _lib.check(lib.dg_plan_tune(plan, _lib.DG_TUNE_P_TILE_WIDTH, int(tile_width)), "dg_plan_tune")
    if steps_per_launch is not None:
      _lib.check(lib.dg_plan_tune(plan, _lib.DG_TUNE_P_STEPS_PER_LAUNCH, int(steps_per_launch)),
                 "dg_plan_tune")
    q = (ctypes.c_int64 * 2)()
    _lib.check(lib.dg_plan_query_p(plan, q), "dg_plan_query_p")
    self.tile_width, self.steps_per_launch = int(q[0]), int(q[1])
    return self

  def query_flow(self, nsteps):
    """True if ``estimate`` over ``nsteps`` steps runs as one dataflow launch."""
    out = ctypes.c_int32()
    _lib.check(self.lo._lib.dg_plan_query_p_flow(self.lo._plan, int(nsteps), ctypes.byref(out)),
               "dg_plan_query_p_flow")
    return bool(out.value)

  def query_sweep(self, nsteps):
    """True if ``sweep`` over ``nsteps`` steps runs forward and estimate as one dataflow
    launch (dg_lserk4_sweep_p)."""
    out = ctypes.c_int32()
    _lib.check(self.lo._lib.dg_plan_query_p_sweep(self.lo._plan, int(nsteps), ctypes.byref(out)),
               "dg_plan_query_p_sweep")
    return bool(out.value)

  def trace_words(self, nsteps):
    """uint64 words a per-item trace (``DGAdvection1D.sweep_trace`` on the lo plan) needs for
    this estimate's dataflow launches over ``nsteps``: 8 per work item of ``estimate``'s or
    ``sweep``'s launch, whichever is larger (dg_plan_query_p_trace); 0 if neither is one."""
    q = (ctypes.c_int64 * 3)()
    _lib.check(self.lo._lib.dg_plan_query_p_trace(self.lo._plan, int(nsteps), q),
               "dg_plan_query_p_trace")
    return int(q[2]) * max(int(q[0]), int(q[1]))

  def sweep(self, snapshots, w, t0, dt, nsteps, eta=None, eta_assign=True, eta_abs=True,
            idx=None, value=None, nonfinite=None):
    """The whole p sweep (dg_lserk4_sweep_p): the order-N forward from ``snapshots[0]`` (u^0)
    into ``snapshots[1..nsteps]``, then the estimate with the terminal weight P u^nsteps into
    ``w`` (order N+1, swept back to t_0) and ``eta``; with ``idx`` also the refine decision
    (as ``estimate_refine``).  One dataflow launch where ``query_sweep`` says so, else the
    launch chains; bit-identical to ``lo.forward`` at 4 steps per launch + ``estimate``."""
    def p1(t, dtype, name):
      if t is None:
        return None
      if isinstance(t, int):  # a device address (host_alias of pinned host memory)
        return ctypes.c_void_p(t)
      if not t.is_cuda or t.dtype != dtype or t.numel() < 1:
        raise TypeError(f"{name} must be a CUDA {dtype} tensor or a device address")
      return ctypes.c_void_p(t.data_ptr())
    eta_p = None if eta is None else self.lo._field(eta, "eta", self.lo.ktot)
    flags = ((_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) |
             (_lib.DG_ADJ_ETA_ABS if eta_abs else 0))
    rc = self.lo._lib.dg_lserk4_sweep_p(
        self.lo._plan, self.hi._plan, self._P_ptr,
        self.lo._field(snapshots, "snapshots", (nsteps + 1) * self.lo.field_numel),
        self.hi._field(w, "w"), float(t0), float(dt), int(nsteps), eta_p, int(flags),
        p1(idx, torch.int64, "idx"), p1(value, torch.float64, "value"),
        p1(nonfinite, torch.int64, "nonfinite"), _stream(self.lo.device))
    _lib.check(rc, "dg_lserk4_sweep_p")
    return w, eta

  def new_field(self, count=None):
    return self.hi.new_field(count)

  def prolong(self, u, out=None):
    """P u: an order-N field (lo plan) to the order-(N+1) nodes (hi plan), on the device."""
    out = self.hi.new_field() if out is None else out
    rc = self.lo._lib.dg_prolong(self.lo._plan, self.hi._plan, self._P_ptr,
                                 self.lo._field(u, "u"), self.hi._field(out, "out"),
                                 _stream(self.lo.device))
    _lib.check(rc, "dg_prolong")
    return out

  def estimate(self, w, snapshots, t0, dt, nsteps, eta=None, eta_assign=False, eta_abs=False,
               terminal_prolong=False):
    """The estimate over the sweep the lo plan's ``forward`` wrote into ``snapshots``
    ((nsteps+1) order-N fields): ``w`` (an order-(N+1) field, dJ_{N+1}/du at t_N) is swept
    back in place to t_0 and eta (batch*K) receives -sum_n w^{n+1} . R^n per element
    (``eta_assign``: assign instead of accumulate; ``eta_abs``: store |eta|).
    ``terminal_prolong``: the terminal weight is P u^nsteps (J = |P u^N|^2 / 2), formed by the
    first launch from the snapshot (w's input is not read; equal bit for bit to ``prolong``
    into w first)."""
    eta_p = None if eta is None else self.lo._field(eta, "eta", self.lo.ktot)
    flags = ((_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) |
             (_lib.DG_ADJ_ETA_ABS if eta_abs else 0) |
             (_lib.DG_ADJ_P_TERMINAL_PROLONG if terminal_prolong else 0))
    rc = self.lo._lib.dg_lserk4_adj_p(
        self.lo._plan, self.hi._plan, self._P_ptr, self.hi._field(w, "w"),
        self.lo._field(snapshots, "snapshots", (nsteps + 1) * self.lo.field_numel),
        float(t0), float(dt), int(nsteps), eta_p, int(flags), _stream(self.lo.device))
    _lib.check(rc, "dg_lserk4_adj_p")
    return w, eta

  def estimate_refine(self, w, snapshots, t0, dt, nsteps, eta, idx, value=None, nonfinite=None,
                      eta_assign=True, eta_abs=True, terminal_prolong=False):
    """``estimate`` + the refine decision ``argmax_ex(eta, use_abs=True)`` in one call
    (dg_lserk4_adj_p_refine): in the dataflow launch the last block's tiles reduce the argmax
    themselves.  ``idx`` / ``nonfinite`` (CUDA int64, 1) and ``value`` (CUDA float64, 1) as
    for ``argmax_ex``."""
    def p1(t, dtype, name):
      if t is None:
        return None
      if isinstance(t, int):  # a device address (host_alias of pinned host memory)
        return ctypes.c_void_p(t)
      if not t.is_cuda or t.dtype != dtype or t.numel() < 1:
        raise TypeError(f"{name} must be a CUDA {dtype} tensor or a device address")
      return ctypes.c_void_p(t.data_ptr())
    flags = ((_lib.DG_ADJ_ETA_ASSIGN if eta_assign else 0) |
             (_lib.DG_ADJ_ETA_ABS if eta_abs else 0) |
             (_lib.DG_ADJ_P_TERMINAL_PROLONG if terminal_prolong else 0))
    rc = self.lo._lib.dg_lserk4_adj_p_refine(
        self.lo._plan, self.hi._plan, self._P_ptr, self.hi._field(w, "w"),
        self.lo._field(snapshots, "snapshots", (nsteps + 1) * self.lo.field_numel),
        float(t0), float(dt), int(nsteps), self.lo._field(eta, "eta", self.lo.ktot), int(flags),
        p1(idx, torch.int64, "idx"), p1(value, torch.float64, "value"),
        p1(nonfinite, torch.int64, "nonfinite"), _stream(self.lo.device))
    _lib.check(rc, "dg_lserk4_adj_p_refine")
    return idx

  def close(self):
    self.hi.close()


def host_alias(t):
  """The device address of a pinned (page-locked, mapped) host tensor's storage, for kernels
  that write small results straight to the host (dg_host_alias); None if it is not mapped."""
  if t.is_cuda or not t.is_pinned():
    return None
  lib = _lib.load()
  d = ctypes.c_void_p()
  if lib.dg_host_alias(ctypes.c_void_p(t.data_ptr()), ctypes.byref(d)) != _lib.DG_OK:
    return None
  return int(d.value) if d.value else None


def stream_copy(src, dst):
  """dst = src with the library's 16-byte-per-lane copy kernel (dg_stream_copy): the
  achievable-HBM-bandwidth ceiling the bench reports."""
  lib = _lib.load()
  for t in (src, dst):
    if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
      raise TypeError("stream_copy needs contiguous CUDA float64 tensors")
  if src.numel() != dst.numel():
    raise ValueError("src and dst differ in size")
  rc = lib.dg_stream_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                          src.numel(), _stream(src.device))
  _lib.check(rc, "dg_stream_copy")
  return dst


def sum_rows(x, rows, out=None):
  """out[k] = sum_r x[r, k] in ascending r (dg_sum_rows)."""
  lib = _lib.load()
  if not x.is_cuda or x.dtype != torch.float64 or not x.is_contiguous():
    raise TypeError("x must be a contiguous CUDA float64 tensor")
  n = x.numel() // rows
  out = torch.empty(n, dtype=torch.float64, device=x.device) if out is None else out
  rc = lib.dg_sum_rows(ctypes.c_void_p(x.data_ptr()), int(rows), int(n),
                       ctypes.c_void_p(out.data_ptr()), _stream(x.device))
  _lib.check(rc, "dg_sum_rows")
  return out


def candidates_argmax(cands, idx, value=None, nonfinite=None):
  """The refine decision from the ranks' candidates (CUDA int64 (W, 2), rank order) into idx
  (and value / +1 nonfinite) on the device (dg_candidates_argmax)."""
  lib = _lib.load()
  if not cands.is_cuda or cands.dtype != torch.int64 or not cands.is_contiguous():
    raise TypeError("cands must be a contiguous CUDA int64 tensor")
  ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
  rc = lib.dg_candidates_argmax(ctypes.c_void_p(cands.data_ptr()), cands.numel() // 2, ptr(idx),
                                ptr(value), ptr(nonfinite), _stream(cands.device))
  _lib.check(rc, "dg_candidates_argmax")
  return idx
