"""Ensembles of independent initial conditions, sharded one process per GPU.

The reference's only data-parallel axis is the ensemble of initial conditions
(``vmap`` over ICs, python/Main_width_ref.py:466-478), reduced by a mean over ICs and
an argmax (:479, :491).  Here each rank owns a contiguous block of ICs, runs the
forward + adjoint sweeps for all of them as one batched plan (no data-path
communication), reduces its per-IC indicators to one K-vector in fixed order, and the
ranks sum those partial sums in rank order with a reduce-scatter built from one
all-to-all (each rank owns a 1/W slice and adds the W partials of it in rank order)
and one all-gather of the summed slices (RCCL over xGMI on GPUs).  The mean indicator
and the refine index are bit-identical on all ranks and independent of the
collectives' internal order, which an RCCL all-reduce would not pin down.
"""
import numpy as np
import torch
import torch.distributed as dist

from .operators import DGAdvection1D, sum_rows


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
  indicator sum (K values).  J = 1/2 |u(T)|^2 per IC (terminal adjoint w^N = u^N).

  All work is enqueued on torch's current stream; ``run`` does not synchronise.
  """

  def __init__(self, mesh, ic_indices, nsteps, dt, a=2 * np.pi, inflow="a", seed_base=0,
               params=None):
    self.ic_indices = list(ic_indices)
    self.batch = len(self.ic_indices)
    if self.batch < 1:
      raise ValueError("a rank needs at least one IC")
    self.nsteps, self.dt = int(nsteps), float(dt)
    self.op = DGAdvection1D(mesh, a=a, batch=self.batch, inflow=inflow)
    amp, freq, phase = params if params is not None else ic_params(self.ic_indices, seed_base)
    self.snaps = self.op.new_field(self.nsteps + 1)
    # u^0 lives in snapshot 0; the forward sweep with u aliasing it leaves it untouched.
    self.op.init_sine(amp, freq, phase, out=self.snaps[0])
    # J = |u^N|^2 / 2: the terminal adjoint is u^N itself, so the adjoint sweep runs in
    # place on snapshot N (the library allows that alias) and leaves dJ/du^0 there.
    self.w = self.snaps[self.nsteps]
    self.eta = torch.zeros(self.op.ktot, dtype=torch.float64, device=self.op.device)
    self.partial = torch.zeros(self.op.K, dtype=torch.float64, device=self.op.device)
    self._graphs = None

  @property
  def dof_updates(self):
    """DOF-updates of one sweep: nsteps forward + nsteps adjoint steps of every DOF."""
    return 2 * self.op.Np * self.op.ktot * self.nsteps

  def forward(self):
    self.op.forward(self.snaps[0], 0.0, self.dt, self.nsteps, self.snaps)

  def adjoint(self):
    self.eta.zero_()
    self.run_adjoint()

  def run_adjoint(self):
    """The adjoint kernels alone (eta already zeroed by the caller)."""
    self.op.adjoint(self.w, self.snaps, 0.0, self.dt, self.nsteps, eta=self.eta)

  def capture(self):
    """Capture the forward and adjoint sweeps as two HIP graphs (replayed by
    forward_graph / adjoint_graph): the per-launch host work (operator constants, inflow
    values) is baked in once and the kernels run back to back."""
    dev = self.op.device
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):  # warm-up outside capture
      self.forward()
      self.adjoint()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    gf, ga = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf):
      self.forward()
    with torch.cuda.graph(ga):
      self.adjoint()
    self._graphs = (gf, ga)
    return self

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
    self.forward()
    self.adjoint()
    return self.reduce()

  def per_ic(self):
    """This rank's per-IC indicators, (batch, K) — a view of eta (IC b is row b)."""
    return self.eta.view(self.batch, self.op.K)


class DeviceReducer:
  """Fixed-order sum and numpy-semantics argmax through the HIP library."""

  def __init__(self, op):
    self.op = op

  def sum_rows(self, stacked):
    return sum_rows(stacked.contiguous(), stacked.shape[0])

  def argmax(self, x):
    return self.op.argmax_async(x.contiguous(), use_abs=True)


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
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)  # recv row r: rank r's slice
    mine = reducer.sum_rows(recv.view(world, chunk))  # rank order
    full = torch.empty_like(send)
    dist.all_gather_into_tensor(full, mine.contiguous(), group=group)
    total = full[:K]
  else:
    # one slice: its sum is itself
    total = partial
  # dividing by 1 is exact (bit-identical shortcut)
  mean = total / float(n_total) if n_total != 1 else total
  return mean, reducer.argmax(mean)


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
  full = rows.new_empty(world * per, K)
  dist.all_gather_into_tensor(full, send, group=group)
  keep = [r * per + i for r in range(world) for i in range(len(shard(n_total, r, world)))]
  return full[torch.tensor(keep, device=full.device)]
