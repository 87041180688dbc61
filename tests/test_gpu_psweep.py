"""The p-estimate's whole sweep -- order-N snapshot forward + estimate -- as ONE dataflow
launch (dg_lserk4_sweep_p, csrc/dg_dwr.hip k_psweep) against the launch chains it replaces:
``lo.forward`` at 4 steps per launch (k_step) + ``estimate`` with the terminal weight P u^N.

The dataflow launch runs the same tile bodies (step_tile, adjph_tile) on the same 4-step
blocks, so every snapshot, w^0 and eta must agree BIT FOR BIT (the chain is pinned to the CPU
oracle by test_gpu_dwr.py).  Covered: orders N = 2..7, 256- and 512-element tiles, trajectory
edges inside tiles, a non-uniform mesh, eta modes, the fused refine decision, repeated
launches (take-counter epochs), the fallbacks and the watchdog."""
import numpy as np
import pytest

from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu

A = 2.0 * np.pi


def dev(x, device):
  import torch
  return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=device)


def host(t):
  return t.detach().cpu().numpy()


def setup(pkg, gpu, N, K, batch=1, v_x=None, seed=0, tw=2):
  ops = pkg.operators
  if v_x is None:
    v_x = np.linspace(0.0, 1.0, K + 1)
  S = setup1d.startup1d(N, v_x, metric="element")
  op = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), a=A, batch=batch)
  op.tune(lane_elements=0, steps_per_launch=4)  # the forward chain on workgroup tiles, 4 steps
  est = ops.DWREstimate(op, tile_width=tw, steps_per_launch=4)
  dt = oadv.bench_dt(S)
  rng = np.random.default_rng(seed)
  u0 = dev(np.concatenate([setup1d.to_elem_major(np.sin(2 * np.pi * (b + 1) * S["x"]) +
                                                 0.1 * rng.standard_normal(S["x"].shape))
                           for b in range(batch)]), gpu)
  return op, est, u0, dt


def chain(op, est, u0, dt, nsteps, eta_init=None, assign=True, absval=True):
  import torch
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(u0)
  op.forward(snaps[0], 0.0, dt, nsteps, snaps)
  w = est.new_field()
  eta = (torch.zeros(op.ktot, dtype=torch.float64, device=u0.device) if eta_init is None
         else eta_init.clone())
  est.estimate(w, snaps, 0.0, dt, nsteps, eta=eta, eta_assign=assign, eta_abs=absval,
               terminal_prolong=True)
  torch.cuda.synchronize()
  return host(snaps), host(w), host(eta)


def fused(op, est, u0, dt, nsteps, eta_init=None, assign=True, absval=True, idx=None):
  import torch
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(u0)
  w = torch.full((est.hi.field_numel,), float("nan"), dtype=torch.float64, device=u0.device)
  eta = (torch.zeros(op.ktot, dtype=torch.float64, device=u0.device) if eta_init is None
         else eta_init.clone())
  est.sweep(snaps, w, 0.0, dt, nsteps, eta=eta, eta_assign=assign, eta_abs=absval,
            idx=None if idx is None else idx[0:1],
            value=None if idx is None else idx[1:2].view(torch.float64),
            nonfinite=None if idx is None else idx[2:3])
  torch.cuda.synchronize()
  return host(snaps), host(w), host(eta)


def assert_same(a, b, what):
  for x, y, name in zip(a, b, ("snapshots", "w", "eta")):
    assert np.array_equal(x, y), (what, name, float(np.nanmax(np.abs(x - y))))


@pytest.mark.parametrize("N,K,batch,tw,nsteps", [
    (4, 3000, 1, 2, 20),    # config 2's shape
    (4, 2500, 1, 1, 12),    # 256-element tiles
    (3, 2000, 2, 2, 16),    # trajectory edges inside tiles
    (2, 900, 1, 2, 8),
    (5, 1200, 1, 2, 32),    # the longest fused sweep (8 blocks)
    (6, 700, 2, 1, 8),
    (7, 500, 1, 2, 12),
    (4, 60, 1, 2, 8),       # the whole mesh inside one (edge) tile
    (4, 777, 1, 2, 8),      # K Np odd: every other snapshot starts 8 bytes off 16-byte alignment
    (3, 1001, 3, 1, 12),
])
def test_psweep_equals_chains(pkg, gpu, N, K, batch, tw, nsteps):
  op, est, u0, dt = setup(pkg, gpu, N, K, batch, seed=N + K, tw=tw)
  assert est.query_sweep(nsteps)
  ref = chain(op, est, u0, dt, nsteps)
  got = fused(op, est, u0, dt, nsteps)
  assert np.isfinite(ref[2]).all() and np.abs(ref[2]).max() > 0
  assert_same(got, ref, "psweep vs chains")
  assert op.sweep_status() == 0


def test_psweep_eta_modes_and_non_uniform_mesh(pkg, gpu):
  rng = np.random.default_rng(4)
  v_x = np.concatenate(([0.0], np.cumsum(rng.uniform(0.3, 1.7, 1500))))
  op, est, u0, dt = setup(pkg, gpu, 4, 1500, 1, v_x=v_x / v_x[-1], seed=4)
  assert not op.uniform and est.query_sweep(12)
  base = dev(rng.standard_normal(op.ktot), gpu)
  for kw in (dict(), dict(eta_init=base, assign=False, absval=False),
             dict(eta_init=base, assign=False, absval=True), dict(assign=True, absval=False)):
    assert_same(fused(op, est, u0, dt, 12, **kw), chain(op, est, u0, dt, 12, **kw), kw)
  assert op.sweep_status() == 0


def test_psweep_refine_and_repeats(pkg, gpu):
  """The fused refine decision equals numpy's argmax of |eta| (value and non-finite count
  too), over repeated launches and alternating sweep lengths on one plan."""
  import torch
  op, est, u0, dt = setup(pkg, gpu, 4, 40000, 1, seed=5)
  refs = {n: chain(op, est, u0, dt, n) for n in (20, 12)}
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  for rep in range(3):
    for n in (20, 12):
      res = fused(op, est, u0, dt, n, idx=got)
      assert_same(res, refs[n], (rep, n))
      e = np.abs(refs[n][2])
      g = host(got)
      assert int(g[0]) == int(np.argmax(e)), (rep, n)
      assert host(got[1:2].view(torch.float64))[0] == e.max()
      assert int(g[2]) == 0
  assert op.sweep_status() == 0


def test_psweep_fallbacks(pkg, gpu):
  """Shapes the dataflow launch does not take run the chains (same bits): 6 steps (not 4-step
  blocks), 36 steps (> 32), one block, the wave-tile forward (lane_elements 4), the sweep or
  the estimate's dataflow launch off."""
  op, est, u0, dt = setup(pkg, gpu, 3, 1000, 1, seed=7)
  for n in (6, 36, 4):
    assert not est.query_sweep(n)
    assert_same(fused(op, est, u0, dt, n), chain(op, est, u0, dt, n), n)
  op.tune(lane_elements=4)
  assert not est.query_sweep(8)
  assert_same(fused(op, est, u0, dt, 8), chain(op, est, u0, dt, 8), "wave tiles")
  op.tune(lane_elements=0)
  est.tune(sweep=0)
  assert not est.query_sweep(8)
  assert_same(fused(op, est, u0, dt, 8), chain(op, est, u0, dt, 8), "sweep off")
  est.tune(sweep=1, flow=0)
  assert not est.query_sweep(8)
  assert_same(fused(op, est, u0, dt, 8), chain(op, est, u0, dt, 8), "flow off")


def test_psweep_watchdog_gives_up_loudly(pkg, gpu):
  """Forced give-ups (DG_TUNE_SWEEP_SPIN_LIMIT = 1 on the lo plan): NaN in the outputs and the
  fused refine value, the non-finite count raised, the next call raises until sweep_status()
  clears the flag, and a normal launch after that gives the chains' bits again."""
  import torch
  _lib = pkg._lib
  op, est, u0, dt = setup(pkg, gpu, 4, 1 << 18, 1, seed=8)
  ref = chain(op, est, u0, dt, 20)
  _lib.check(op._lib.dg_plan_tune(op._plan, _lib.DG_TUNE_SWEEP_SPIN_LIMIT, 1), "dg_plan_tune")
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  res = fused(op, est, u0, dt, 20, idx=got)
  assert np.isnan(host(got[1:2].view(torch.float64))[0])
  assert int(host(got)[2]) == 1
  assert np.isnan(res[2]).any()
  with pytest.raises(_lib.DGLibraryError, match="gave up"):
    fused(op, est, u0, dt, 20, idx=got)
  assert op.sweep_status() == 1
  assert op.sweep_status() == 0
  _lib.check(op._lib.dg_plan_tune(op._plan, _lib.DG_TUNE_SWEEP_SPIN_LIMIT, 0), "dg_plan_tune")
  assert_same(fused(op, est, u0, dt, 20), ref, "after the watchdog fired")


@pytest.mark.slow
def test_psweep_full_size(pkg, gpu):
  """Config 2's size (N = 4, K = 2^20, 20 steps): bit for bit against the chains."""
  op, est, u0, dt = setup(pkg, gpu, 4, 1 << 20, 1, seed=21)
  assert_same(fused(op, est, u0, dt, 20), chain(op, est, u0, dt, 20), "full size")
  assert op.sweep_status() == 0


def test_psweep_fallback_ignores_the_plans_steps_per_launch(pkg, gpu):
  """The chains dg_lserk4_sweep_p falls back to run the forward at the dataflow launch's 4-step
  blocks whatever the lo plan's steps per launch: a sweep whose nsteps does not
  fit the launch (36 > 32 steps, 6 = not 4-step blocks) and one that does give the bits of the
  4-step chain even with the plan tuned to 8 (or 2) steps per launch."""
  op, est, u0, dt = setup(pkg, gpu, 4, 1200, 1, seed=9)
  refs = {n: chain(op, est, u0, dt, n) for n in (36, 6, 12)}  # chain: op at 4 steps per launch
  for spl in (8, 2):
    op.tune(tile_width=2, steps_per_launch=spl)
    for n, fits in ((36, False), (6, False), (12, True)):
      assert est.query_sweep(n) == fits
      assert_same(fused(op, est, u0, dt, n), refs[n], (spl, n))
  op.tune(steps_per_launch=4)


def test_p_trace_buffer_is_sized_by_the_query(pkg, gpu):
  """dg_plan_query_p_trace gives the p launches' trace size (8 words per work item; ADVICE
  r05): a trace of exactly that many words, followed by a canary, is filled by the estimate's
  and the sweep's dataflow launches and the canary is untouched."""
  import torch
  op, est, u0, dt = setup(pkg, gpu, 4, 5000, 1, seed=10)
  nsteps = 20
  assert est.query_flow(nsteps) and est.query_sweep(nsteps)
  words = est.trace_words(nsteps)
  tiles = -(-op.ktot // (256 * 2 - 40))  # the 4-step blocks' 512-element tiles
  assert words == 8 * 2 * (nsteps // 4) * tiles  # the sweep's launch: forward + estimate items
  canary = 1 << 62
  buf = torch.full((words + 64,), canary, dtype=torch.int64, device=gpu)
  op.sweep_trace(buf[:words])
  try:
    fused(op, est, u0, dt, nsteps)
    chain(op, est, u0, dt, nsteps)  # the estimate's own dataflow launch
  finally:
    op.sweep_trace(None)
  torch.cuda.synchronize()
  tr = host(buf)
  assert (tr[words:] == canary).all()
  # every item recorded (the sweep's launch fills all): words 0..5 of each 8-word record
  assert (tr[:words].reshape(-1, 8)[:, :6] != canary).all()
