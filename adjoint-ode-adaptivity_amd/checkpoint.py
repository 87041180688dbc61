"""Checkpointed forward + adjoint sweeps: the adjoint of a sweep whose snapshots do not fit.

The full-storage sweep (``DGAdvection1D.forward`` with ``snapshots``, then ``.adjoint``)
keeps every state u^0..u^N for the reverse pass (SURVEY §7 "Snapshot memory for the
adjoint": one N=4 field is 168 MB at K = 2^22, so storing every step of a long sweep is
impossible).  ``CheckpointedSweep`` keeps u at the start of every segment of ``every``
steps and, going backwards, re-runs each segment's forward steps into a scratch of
``every + 1`` fields before running that segment's adjoint:

* memory: ceil(N / every) checkpoints + (every + 1) scratch fields instead of N + 1
  (every ~ sqrt(N) minimises it: 2 sqrt(N) + 1 fields);
* work: one extra forward pass over all segments but the last (the forward sweep leaves
  the last segment's states in the scratch, so its adjoint starts at once).

The composition is exact, not an approximation of the full-storage sweep:
  - the time levels are formed by repeated addition from t0, as the library forms them
    (``tn[n+1] = tn[n] + dt``, dg_lserk4_fwd / One_code.mlx:139), so each segment sees the
    same t_n as the uninterrupted sweep;
  - the recomputed states equal the checkpointed forward's own states bit for bit (same
    calls, same launch shapes);
  - dg_lserk4_adj over [s, e] adds the functional source at u^s..u^{e-1} and the
    indicator contributions of steps s..e-1, so the segments partition the sweep's source
    (left-endpoint rule, Main_finite_difference.py:225-227) and its DWR sum.
Against the full-storage sweep the results agree to rounding (the per-launch step
grouping and where the node-0 source is added can differ at segment boundaries);
``tests/test_gpu_checkpoint.py`` bounds the difference.

Everything runs on the device through the existing entry points (dg_lserk4_fwd /
dg_lserk4_adj); there is no host round trip inside either sweep.
"""
import math

import torch


def step_times(t0, dt, n):
  """t_0..t_n by repeated addition (the library's time levels, dg_advec.hip tn[])."""
  t = [float(t0)]
  for _ in range(n):
    t.append(t[-1] + float(dt))
  return t


class CheckpointedSweep:
  """Forward sweep of ``nsteps`` steps that keeps every ``every``-th state, and the adjoint
  sweep (+ DWR indicator) that recomputes the states in between.

  Args:
    op: a :class:`~operators.DGAdvection1D` (linear or config-3 physics).
    nsteps: steps per sweep.
    every: segment length (default ceil(sqrt(nsteps))).
  """

  def __init__(self, op, nsteps, every=None):
    if nsteps < 1:
      raise ValueError("nsteps must be >= 1")
    every = int(math.ceil(math.sqrt(nsteps))) if every is None else int(every)
    if every < 1:
      raise ValueError("every must be >= 1")
    self.op = op
    self.nsteps = int(nsteps)
    self.every = min(every, self.nsteps)
    self.segments = [(s, min(s + self.every, self.nsteps))
                     for s in range(0, self.nsteps, self.every)]
    self.checkpoints = op.new_field(len(self.segments))
    self.scratch = op.new_field(self.every + 1)
    self._times = None
    self._dt = None
    self._last_resident = False

  @property
  def fields(self):
    """Device fields held (checkpoints + scratch), against nsteps + 1 for full storage."""
    return len(self.segments) + self.every + 1

  def forward(self, u, t0, dt):
    """nsteps steps in place on u; checkpoints[c] receives u at the start of segment c."""
    self._times = step_times(t0, dt, self.nsteps)
    self._dt = float(dt)
    for c, (s, e) in enumerate(self.segments):
      self.checkpoints[c].copy_(u)
      self.op.forward(u, self._times[s], self._dt, e - s, self.scratch[: e - s + 1])
    self._last_resident = True
    return u

  def adjoint(self, w, src_coef=0.0, eta=None):
    """The adjoint sweep of the last ``forward`` in place on w (dJ/du^N in, dJ/du^0 out),
    with the DWR indicator accumulated into eta — what ``op.adjoint`` computes over the
    full snapshot array.  w must not alias the scratch."""
    if self._times is None:
      raise RuntimeError("adjoint() needs a preceding forward()")
    lo, hi = self.scratch.data_ptr(), self.scratch.data_ptr() + self.scratch.nbytes
    if lo <= w.data_ptr() < hi:
      raise ValueError("w must not alias the scratch (copy the terminal state first)")
    for c in range(len(self.segments) - 1, -1, -1):
      s, e = self.segments[c]
      snaps = self.scratch[: e - s + 1]
      if not (c == len(self.segments) - 1 and self._last_resident):
        # re-run the segment from its checkpoint; u aliases snapshot 0 (left as u^s)
        snaps[0].copy_(self.checkpoints[c])
        self.op.forward(snaps[0], self._times[s], self._dt, e - s, snaps)
      self.op.adjoint(w, snaps, self._times[s], self._dt, e - s, src_coef=src_coef, eta=eta)
    self._last_resident = False  # the scratch now holds segment 0
    return w, eta

  @staticmethod
  def fields_needed(nsteps, every):
    """Fields a CheckpointedSweep(nsteps, every) holds: ceil(nsteps/every) + every + 1."""
    every = min(int(every), int(nsteps))
    return -(-int(nsteps) // every) + every + 1
