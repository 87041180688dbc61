"""Ensembles of independent initial conditions, sharded one process per GPU.

The reference's only data-parallel axis is the ensemble of initial conditions
(``vmap`` over ICs, python/Main_width_ref.py:466-478), reduced by a mean over ICs and
an argmax (:479, :491).  Here each rank owns a contiguous block of ICs, runs the
forward + adjoint sweeps for all of them as one batched plan (no data-path
communication), takes each IC's indicator magnitude |eta_ic| (the reference's
errorIndicator returns ``jnp.abs(err)`` per IC, :139, before the mean over ICs, :479),
reduces them to one K-vector in fixed order, and the
ranks sum those partial sums in rank order with a reduce-scatter built from one
all-to-all (each rank owns a 1/W slice and adds the W partials of it in rank order)
and one all-gather of the summed slices (RCCL over xGMI on GPUs).  The mean indicator
and the refine index are bit-identical on all ranks and independent of the
collectives' internal order, which an RCCL all-reduce would not pin down.
"""
import numpy as np
import torch
import torch.distributed as dist

from .operators import DGAdvection1D, DWREstimate, candidates_argmax, sum_rows


def ic_params(indices, seed_base=0):
  """Synthetic IC family of SURVEY §8d: u0_j(x) = A_j sin(2 pi m_j x + phi_j) with
  rng = default_rng(seed_base + j), A ~ U[0.5, 1.5], m ~ U{1..8}, phi ~ U[0, 2 pi)."""
  amp, freq, phase = [], [], []
  for j in indices:
    rng = np.random.default_rng(seed_base + int(j))
    amp.append(rng.uniform(0.5, 1.5))
    freq.append(float(rng.integers(1, 9)))
    phase.append(rng.uniform(0.0, 2 * np.pi))
  return np.array(amp), np.array(freq), np.array(phase)


def shard(n_total, rank, world):
  """Contiguous block of IC indices owned by ``rank`` (sizes differ by at most one)."""
  base, extra = divmod(n_total, world)
  start = rank * base + min(rank, extra)
  return range(start, start + base + (1 if rank < extra else 0))


class EnsembleSweep:
  """One forward + adjoint sweep over this rank's ICs, producing the rank's partial
  indicator sum sum_ic |eta_ic| (K values).  J = 1/2 |u(T)|^2 per IC (terminal adjoint
  w^N = u^N).  Each IC's row is stored as |eta_ic| by the last adjoint launch
  (DG_ADJ_ETA_ABS), as python/Main_width_ref.py:139 returns jnp.abs(err) per IC, so
  opposite-signed indicators of different ICs never cancel in the mean.

  All work is enqueued on torch's current stream; ``run`` does not synchronise.
  """

  RECORDS = ("jumps", "snapshots")
  INDICATORS = ("jump", "p")

  def __init__(self, mesh, ic_indices, nsteps, dt, a=2 * np.pi, inflow="a", seed_base=0,
               params=None, record="jumps", indicator="jump"):
    self.ic_indices = list(ic_indices)
    self.batch = len(self.ic_indices)
    if self.batch < 1:
      raise ValueError("a rank needs at least one IC")
    if record not in self.RECORDS:
      raise ValueError(f"record must be one of {self.RECORDS}, got {record!r}")
    if indicator not in self.INDICATORS:
      raise ValueError(f"indicator must be one of {self.INDICATORS}, got {indicator!r}")
    if indicator == "p" and record != "snapshots":
      raise ValueError("the p-enriched estimate recomputes each step from the order-N "
                       "snapshots: record='snapshots'")
    self.record = record
    self.indicator = indicator
    self.est = None
    self.nsteps, self.dt = int(nsteps), float(dt)
    self.op = DGAdvection1D(mesh, a=a, batch=self.batch, inflow=inflow)
    amp, freq, phase = params if params is not None else ic_params(self.ic_indices, seed_base)
    if record == "jumps":
      # The snapshot-free pair (dg_lserk4_fwd_rec / dg_lserk4_adj_rec): the forward keeps
      # per element and step only the left-face jump the indicator needs (8 B instead of
      # 8 Np B; the right face's is the next element's).  At equal steps per launch w, eta and the refine decision are bit-identical
      # to the snapshot pair's; at the record pair's own (longer) launches the states differ
      # in the last bits and eta by the indicator's conditioning (~1e-9 relative on smooth
      # solutions, DESIGN.md §5 "The indicator's conditioning").
      self.u0 = self.op.new_field()
      self.op.init_sine(amp, freq, phase, out=self.u0)
      self.jumps = self.op.new_jumps(self.nsteps)
      # J = |u^N|^2 / 2: the forward writes u^N into w, the adjoint's terminal value
      self.w = self.op.new_field()
      self.snaps = None
    else:
      self.snaps = self.op.new_field(self.nsteps + 1)
      # u^0 lives in snapshot 0; the forward sweep with u aliasing it leaves it untouched.
      self.op.init_sine(amp, freq, phase, out=self.snaps[0])
      self.u0 = self.snaps[0]
      if indicator == "p":
        # The p-enriched DWR estimate (dg_lserk4_adj_p): the adjoint runs
        # at order N+1 from w = P u^N (J = |P u^N|^2 / 2 on the enriched nodes).
        self.est = DWREstimate(self.op)
        self.w = self.est.new_field()
        if self.op.N >= 3:
          # a separate ``forward`` (the bench's pflow path with the whole-sweep launch tuned
          # off) keeps every state in launches of the stage-loop step, 8 steps per launch on
          # 512-element tiles (88 us per launch, profiles/r05/p; the Horner-form pair step with
          # register snapshot stores, snap_pairs=1, took 108 us); ``sweep`` / ``sweep_refine``
          # run the forward at 4 steps per launch whatever this says (dg_lserk4_sweep_p)
          self.op.tune(tile_width=2, steps_per_launch=8)
      else:
        # J = |u^N|^2 / 2: the terminal adjoint is u^N itself, so the adjoint sweep runs in
        # place on snapshot N (the library allows that alias) and leaves dJ/du^0 there.
        self.w = self.snaps[self.nsteps]
    # per-IC |eta| rows; the adjoint's first launch assigns them (DG_ADJ_ETA_ASSIGN), so
    # they need no zero fill
    self.eta = torch.zeros(self.op.ktot, dtype=torch.float64, device=self.op.device)
    self.partial = torch.zeros(self.op.K, dtype=torch.float64, device=self.op.device)
    self._graphs = None

  @property
  def dof_updates(self):
    """DOF-updates of one sweep: nsteps forward + nsteps adjoint steps of every DOF."""
    return 2 * self.op.Np * self.op.ktot * self.nsteps

  def forward(self):
    if self.record == "jumps":
      self.op.forward_rec(self.u0, 0.0, self.dt, self.nsteps, self.jumps, out=self.w)
    else:
      self.op.forward(self.snaps[0], 0.0, self.dt, self.nsteps, self.snaps)

  def adjoint(self):
    self.terminal()
    self.run_adjoint()

  def terminal(self):
    """Nothing: the jump and snapshot modes' forward leaves u^N where the adjoint starts, and
    the p-estimate's first adjoint launch forms its terminal weight w = P u^N from snapshot N
    itself (DG_ADJ_P_TERMINAL_PROLONG, equal to dg_prolong into w first)."""

  def run_adjoint(self):
    """The adjoint kernels: w^N -> w^0 in place and eta = |DWR| per IC row (assigned, not
    accumulated: no zero fill needed)."""
    if self.est is not None:
      self.est.estimate(self.w, self.snaps, 0.0, self.dt, self.nsteps, eta=self.eta,
                        eta_assign=True, eta_abs=True, terminal_prolong=True)
    elif self.record == "jumps":
      self.op.adjoint_rec(self.w, self.jumps, 0.0, self.dt, self.nsteps, eta=self.eta,
                          eta_assign=True, eta_abs=True)
    else:
      self.op.adjoint(self.w, self.snaps, 0.0, self.dt, self.nsteps, eta=self.eta,
                      eta_assign=True, eta_abs=True)

  @property
  def dataflow(self):
    """True when ``sweep`` runs forward + adjoint as ONE dataflow launch
    (dg_lserk4_sweep_rec, jump record, the plan's shape allowing it)."""
    return self.record == "jumps" and self.op.query_sweep(self.nsteps)[0]

  def sweep(self):
    """Forward + adjoint + |eta|.  Jump record: one dg_lserk4_sweep_rec call -- a single
    dataflow launch where the record shape allows (csrc/dg_sweep.hip), else the two launch
    chains; bit-identical either way (J = |u^N|^2/2: the terminal weight is u^N, w ends as
    w^0).  Snapshots: ``forward`` then ``adjoint``."""
    if self.record == "jumps":
      self.op.sweep_rec(self.u0, self.jumps, self.w, 0.0, self.dt, self.nsteps, eta=self.eta,
                        eta_assign=True, eta_abs=True, terminal_state=True)
    elif self.est is not None:
      # the p-estimate's whole sweep (dg_lserk4_sweep_p): one dataflow launch where the shape
      # allows (p_sweep), else the chains with the forward at the launch's 4-step blocks --
      # the same bits either way, whatever nsteps
      self.est.sweep(self.snaps, self.w, 0.0, self.dt, self.nsteps, eta=self.eta,
                     eta_assign=True, eta_abs=True)
    else:
      self.forward()
      self.adjoint()

  def sweep_refine(self, reducer, idx=None, value=None):
    """``sweep`` plus the refine decision into ``reducer`` (index, value, non-finite count:
    the DeviceReducer state) in ONE dg_lserk4_sweep_refine call -- for a single trajectory on
    a single rank, whose indicator is the whole mean (Main_width_ref.py:479 with one IC); the
    dataflow launch reduces the argmax in its last tiles (the p-estimate: the snapshot forward,
    then dg_lserk4_adj_p_refine).  ``idx`` / ``value``: other
    destinations for the index and value (e.g. ``operators.host_alias`` addresses of pinned
    host memory: the decision lands on the host with no copy launch)."""
    if self.batch != 1 or (self.record != "jumps" and self.est is None):
      raise ValueError("sweep_refine: one trajectory with the jump record or the p-estimate")
    idx = reducer.idx if idx is None else idx
    value = reducer.value if value is None else value
    if self.est is not None:
      # forward + estimate + refine decision (dg_lserk4_sweep_p): one dataflow launch where
      # the shape allows, else the chains at the same 4-step forward blocks
      self.est.sweep(self.snaps, self.w, 0.0, self.dt, self.nsteps, eta=self.eta,
                     eta_assign=True, eta_abs=True, idx=idx, value=value,
                     nonfinite=reducer.nonfinite)
      return
    self.op.sweep_refine(self.u0, self.jumps, self.w, 0.0, self.dt, self.nsteps, self.eta,
                         idx, value, reducer.nonfinite)

  def estimate_refine(self, idx, value, nonfinite):
    """The p-estimate's adjoint (``run_adjoint``) + the refine decision in one call."""
    self.est.estimate_refine(self.w, self.snaps, 0.0, self.dt, self.nsteps, self.eta, idx,
                             value, nonfinite, eta_assign=True, eta_abs=True,
                             terminal_prolong=True)

  @property
  def p_dataflow(self):
    """True when the p-estimate runs as ONE dataflow launch (dg_lserk4_adj_p, DG_TUNE_P_FLOW)."""
    return self.est is not None and self.est.query_flow(self.nsteps)

  @property
  def p_sweep(self):
    """True when the p-estimate's forward and estimate run as ONE dataflow launch
    (dg_lserk4_sweep_p: the forward's 4-step blocks are the estimate's)."""
    return self.est is not None and self.est.query_sweep(self.nsteps)

  def capture(self):
    """Capture the sweep as HIP graphs (replayed by sweep_graph, or forward_graph /
    adjoint_graph for the two halves of the snapshot pair): the per-launch host work
    (operator constants, inflow values) is baked in once and the kernels run back to back."""
    dev = self.op.device
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):  # warm-up outside capture (allocates the sweep scratch)
      self.sweep()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    if self.dataflow or self.p_sweep:
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g):
        self.sweep()
      self._graphs = (g,)
      return self
    gf, ga = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf):
      self.forward()
    with torch.cuda.graph(ga):
      self.adjoint()
    self._graphs = (gf, ga)
    return self

  def sweep_graph(self):
    if len(self._graphs) == 1:
      self._graphs[0].replay()
    else:
      self._graphs[0].replay()
      self._graphs[1].replay()

  def forward_graph(self):
    self._graphs[0].replay()

  def adjoint_graph(self):
    self._graphs[1].replay()

  def reduce(self):
    if self.batch == 1:  # one IC: the partial sum is eta itself
      return self.eta
    sum_rows(self.eta, self.batch, out=self.partial)
    return self.partial

  def run(self):
    self.sweep()
    return self.reduce()

  def per_ic(self):
    """This rank's per-IC indicator magnitudes |eta_ic|, (batch, K) — a view of eta (IC b
    is row b), the rows Main_width_ref.py:139 returns."""
    return self.eta.view(self.batch, self.op.K)


class DeviceReducer:
  """Fixed-order sum and numpy-semantics argmax through the HIP library.

  ``state`` (device int64[3]) holds the last refine index, the indicator value there (as
  float64 bits: ``value``) and a running count of argmax calls whose winner was not finite
  (``nonfinite``; argmax ranks NaN and +-inf first, so that is "some indicator entry was not
  finite"), all written by dg_argmax_ex without a host sync."""

  def __init__(self, op):
    self.op = op
    self.state = torch.zeros(3, dtype=torch.int64, device=op.device)
    self.idx = self.state[0:1]
    self.value = self.state[1:2].view(torch.float64)
    self.nonfinite = self.state[2:3]

  def sum_rows(self, stacked):
    return sum_rows(stacked.contiguous(), stacked.shape[0])

  def argmax(self, x):
    return self.op.argmax_ex(x.contiguous(), self.idx, self.value, self.nonfinite, use_abs=True)

  def candidate(self, slices, n, divisor, offset):
    """This rank's refine candidate as a device int64[2] (the bits of |m[i]| and i + offset,
    m = the slices' rank-order sum over the first n columns / divisor, i = argmax |m|):
    dg_slice_candidate, two launches, state untouched."""
    c = torch.empty(2, dtype=torch.int64, device=self.op.device)
    return self.op.slice_candidate(slices.contiguous(), n, divisor, offset, c)

  def finish(self, cands):
    """The refine decision from the ranks' candidates (W, 2) int64 in rank order: the argmax
    of the values under numpy's order (ties to the lowest rank, which owns the lowest
    indices) into the state (dg_candidates_argmax), then its index."""
    return candidates_argmax(cands.contiguous(), self.idx, self.value, self.nonfinite)


def _exchange(coll, send, group, n_out=None):
  """out = coll(out, send) over the process group.  RCCL ("nccl") moves device tensors over
  xGMI directly; the gloo backend (several ranks on one GPU in tests) takes the exchange
  through host copies, since gloo's all-to-all handles CPU tensors only."""
  staged = send.is_cuda and dist.get_backend(group) == "gloo"
  src = send.cpu() if staged else send
  out = src.new_empty(src.numel() if n_out is None else n_out)
  coll(out, src, group=group)
  return out.to(send.device) if staged else out


def gather_indicator(partial, n_total, reducer, group=None):
  """Sum the per-rank partial indicators over the ranks in rank order, take the mean over
  all ICs and the argmax of its magnitude (python/Main_width_ref.py:479,491).
  Returns (mean indicator, index tensor).  Works for any world size (1 = no collective).

  The exchange is a rank-ordered reduce-scatter built from one all-to-all (rank j
  receives every rank's partial for its slice j of the K values and sums them in rank
  order) followed by an all-gather of the summed slices: 2 (W-1)/W K doubles in and out per
  rank, like a ring all-reduce, instead of the (W-1) K of gathering every partial.  The
  result is bit-identical on every rank and equal to summing the W partials in rank order."""
  if dist.is_available() and dist.is_initialized():
    world = dist.get_world_size(group)
  else:
    world = 1
  if world > 1:
    K = partial.numel()
    chunk = -(-K // world)
    send = partial.new_zeros(world * chunk)
    send[:K] = partial.reshape(-1)
    recv = _exchange(dist.all_to_all_single, send, group)  # recv row r: rank r's slice
    mine = reducer.sum_rows(recv.view(world, chunk))  # rank order
    full = _exchange(dist.all_gather_into_tensor, mine.contiguous(), group, world * chunk)
    total = full[:K]
  else:
    # one slice: its sum is itself
    total = partial
  # dividing by 1 is exact (bit-identical shortcut).  The divisor is a 0-dim tensor on the
  # indicator's device: with a Python float PyTorch's CUDA division multiplies by the
  # reciprocal (a * (1/b), one ulp off a / b for b = 3, 6, 12, ...), while dg_slice_candidate
  # (refine_decision at W > 1) divides; a tensor divisor keeps true division on both paths.
  if n_total != 1:
    mean = torch.div(total, torch.tensor(float(n_total), dtype=total.dtype, device=total.device))
  else:
    mean = total
  return mean, reducer.argmax(mean)


def refine_decision(partial, n_total, reducer, group=None):
  """The refine decision of ``gather_indicator`` (argmax of the mean indicator's magnitude,
  python/Main_width_ref.py:491) without materialising the mean on every rank: after the
  rank-ordered all-to-all each rank takes the argmax of its summed slice's mean, and the W
  (value, index) candidates are all-gathered -- 16 B per rank instead of the (W-1)/W K doubles
  of gathering the summed slices.  The winner is the argmax over the candidates under
  numpy's order: a tie goes to the lowest rank, which owns the lowest indices, and a NaN
  anywhere wins as it would in the full vector, so index and value are those of
  ``gather_indicator`` bit for bit (the slices hold the same doubles).  One rank: exactly
  ``gather_indicator``.  Returns the index tensor (the reducer's state holds index, value and
  the non-finite count)."""
  if dist.is_available() and dist.is_initialized():
    world, rank = dist.get_world_size(group), dist.get_rank(group)
  else:
    world, rank = 1, 0
  if world == 1:
    return gather_indicator(partial, n_total, reducer, group)[1]
  K = partial.numel()
  chunk = -(-K // world)
  if K == world * chunk and partial.is_contiguous():
    send = partial.reshape(-1)  # no padding needed: no copy
  else:
    send = partial.new_zeros(world * chunk)
    send[:K] = partial.reshape(-1)
  recv = _exchange(dist.all_to_all_single, send, group)
  lo = rank * chunk
  n = max(0, min(chunk, K - lo))
  if n > 0:  # the rank-order sum of the received slices, its mean and argmax in one pass
    cand = reducer.candidate(recv.view(world, chunk), n, float(n_total), lo)
  else:  # a rank past the end of K: the weakest candidate
    cand = torch.tensor([np.array([-np.inf]).view(np.int64)[0], np.iinfo(np.int64).max],
                        dtype=torch.int64, device=partial.device)
  allc = _exchange(dist.all_gather_into_tensor, cand, group, 2 * world).view(world, 2)
  return reducer.finish(allc)


_KEEP = {}


def _keep_index(n_total, world, per, device):
  """Rows of the padded all-gather that hold real ICs (cached per shape and device)."""
  key = (n_total, world, per, str(device))
  if key not in _KEEP:
    keep = [r * per + i for r in range(world) for i in range(len(shard(n_total, r, world)))]
    _KEEP[key] = torch.tensor(keep, device=device)
  return _KEEP[key]


def gather_per_ic(rows, n_total, group=None):
  """All-gather every rank's per-IC indicator rows (``rows``: (batch_r, K), the ICs
  ``shard(n_total, rank, W)``) into the (n_total, K) array of all ICs in IC order, on every
  rank — the per-IC training-data gather of north_star (Main_width_ref.py:466-478 computes
  one indicator row per IC; models.py trains on them).

  Shards differ by at most one IC, so each rank pads its block to ceil(n_total/W) rows and
  one all_gather_into_tensor (RCCL over xGMI on GPUs) moves W * ceil(n_total/W) * K doubles
  (512 MiB at config 4); the pad rows are dropped.  Pure data movement: the result is
  bit-identical to the rows."""
  if dist.is_available() and dist.is_initialized():
    world, rank = dist.get_world_size(group), dist.get_rank(group)
  else:
    world, rank = 1, 0
  rows = rows.reshape(len(shard(n_total, rank, world)), -1)
  if world == 1:
    return rows
  K = rows.shape[1]
  per = -(-n_total // world)
  send = rows.new_zeros(per, K)
  send[: rows.shape[0]] = rows
  full = _exchange(dist.all_gather_into_tensor, send.reshape(-1), group,
                   world * per * K).view(world * per, K)
  if n_total % world == 0:  # no pad rows: the gathered block is the answer
    return full
  return full.index_select(0, _keep_index(n_total, world, per, full.device))
