"""The p-enriched estimate as ONE dataflow launch (dg_lserk4_adj_p with DG_TUNE_P_FLOW = 1,
csrc/dg_dwr.hip k_adjp_flow) against the launch-per-block chain (DG_TUNE_P_FLOW = 0).

The two run the same tile arithmetic (adjph_tile) on the same blocks of reverse steps, and the
dataflow launch adds the blocks' indicator partials in launch order, so w^0 and eta must agree
BIT FOR BIT; the chain itself is pinned to the CPU oracle (oracle/effectivity.py p_estimate)
by test_gpu_dwr.py.  Covered here: the launch shapes (256-element tiles x 4 steps, 512 x 4,
512 x 8), orders N = 1..7, trajectory edges inside tiles, non-uniform meshes, the eta modes
(accumulate / assign / abs / none), the terminal weight formed in the kernel, the fused refine
decision (dg_lserk4_adj_p_refine == dg_argmax_ex of |eta|), repeated launches and alternating
shapes on one plan (take-counter epochs), the fallbacks, and the watchdog."""
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


def setup(pkg, gpu, N, K, batch=1, v_x=None, seed=0, nsteps=20):
  ops = pkg.operators
  if v_x is None:
    v_x = np.linspace(0.0, 1.0, K + 1)
  S = setup1d.startup1d(N, v_x, metric="element")
  op = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), a=A, batch=batch)
  est = ops.DWREstimate(op)
  dt = oadv.bench_dt(S)
  rng = np.random.default_rng(seed)
  x = np.concatenate([setup1d.to_elem_major(np.sin(2 * np.pi * (b + 1) * S["x"]) +
                                            0.1 * rng.standard_normal(S["x"].shape))
                      for b in range(batch)])
  snaps = op.new_field(nsteps + 1)
  op.forward(dev(x, gpu), 0.0, dt, nsteps, snaps)
  w0 = dev(rng.standard_normal(batch * K * (N + 2)), gpu)
  return op, est, snaps, w0, dt


def run(est, snaps, w0, dt, nsteps, flow, eta_init=None, term=False, assign=True, absval=True,
        with_eta=True):
  import torch
  est.tune(flow=flow)
  assert est.query_flow(nsteps) == bool(flow)
  w = w0.clone()
  eta = None
  if with_eta:
    eta = (torch.zeros(est.lo.ktot, dtype=torch.float64, device=w.device) if eta_init is None
           else eta_init.clone())
  est.estimate(w, snaps[:nsteps + 1], 0.0, dt, nsteps, eta=eta, eta_assign=assign,
               eta_abs=absval, terminal_prolong=term)
  torch.cuda.synchronize()
  return host(w), (host(eta) if with_eta else None)


def assert_same(a, b, what):
  for x, y, name in zip(a, b, ("w", "eta")):
    if x is None:
      continue
    assert np.array_equal(x, y, equal_nan=False), (what, name, float(np.max(np.abs(x - y))))


@pytest.mark.parametrize("N,K,batch,tw,spl,nsteps", [
    (4, 3000, 1, 1, 4, 20),    # config 2's shape (256-element tiles, 4 steps per block)
    (4, 2000, 2, 2, 4, 12),    # 512-element tiles, trajectory edges inside tiles
    (3, 1500, 1, 2, 8, 16),    # 512-element tiles, 8 steps per block
    (2, 700, 3, 1, 4, 8),
    (1, 900, 1, 1, 4, 40),     # the longest sweep (10 blocks)
    (5, 800, 1, 2, 4, 8),
    (6, 600, 1, 1, 4, 8),      # Np = 7, 8: no occupancy cap
    (7, 500, 2, 2, 8, 16),
    (4, 40, 1, 1, 4, 8),       # the whole mesh inside one (edge) tile
    (4, 777, 1, 2, 4, 12),     # K Np odd: snapshots off 16-byte alignment (direct-to-LDS loads)
    (2, 1001, 1, 1, 4, 8),
])
def test_flow_equals_chain(pkg, gpu, N, K, batch, tw, spl, nsteps):
  op, est, snaps, w0, dt = setup(pkg, gpu, N, K, batch, seed=N + K, nsteps=nsteps)
  est.tune(tile_width=tw, steps_per_launch=spl)
  ref = run(est, snaps, w0, dt, nsteps, 0)
  got = run(est, snaps, w0, dt, nsteps, 1)
  assert np.isfinite(ref[1]).all() and np.abs(ref[1]).max() > 0
  assert_same(got, ref, "flow vs chain")
  assert op.sweep_status() == 0


def test_flow_eta_modes_and_terminal_weight(pkg, gpu):
  """Accumulate into an existing eta, assign without abs, no indicator at all, and the
  terminal weight P u^N formed by the first block (w's input unread)."""
  import torch
  op, est, snaps, w0, dt = setup(pkg, gpu, 4, 2500, 2, seed=3, nsteps=12)
  base = dev(np.random.default_rng(9).standard_normal(op.ktot), gpu)
  for kw in (dict(eta_init=base, assign=False, absval=False),
             dict(eta_init=base, assign=False, absval=True),
             dict(assign=True, absval=False),
             dict(with_eta=False),
             dict(term=True)):
    ref = run(est, snaps, w0, dt, 12, 0, **kw)
    got = run(est, snaps, w0, dt, 12, 1, **kw)
    assert_same(got, ref, kw)
  # the terminal weight: w's input is not read (NaN in, finite out)
  wn = torch.full_like(w0, float("nan"))
  got = run(est, snaps, wn, dt, 12, 1, term=True)
  ref = run(est, snaps, w0, dt, 12, 0, term=True)
  assert_same(got, ref, "terminal weight with NaN input")
  assert op.sweep_status() == 0


def test_flow_non_uniform_mesh(pkg, gpu):
  rng = np.random.default_rng(4)
  v_x = np.concatenate(([0.0], np.cumsum(rng.uniform(0.3, 1.7, 1800))))
  op, est, snaps, w0, dt = setup(pkg, gpu, 3, 1800, 1, v_x=v_x / v_x[-1], seed=4, nsteps=8)
  assert not op.uniform
  assert_same(run(est, snaps, w0, dt, 8, 1), run(est, snaps, w0, dt, 8, 0), "non-uniform")


@pytest.mark.parametrize("tw,spl", [(1, 4), (2, 8)])
def test_flow_refine_fused_equals_argmax(pkg, gpu, tw, spl):
  """dg_lserk4_adj_p_refine: the last block's tiles reduce (|eta|, element) to the winner in
  the launch; equal to the chain's separate dg_argmax_ex, value and non-finite count too."""
  import torch
  op, est, snaps, w0, dt = setup(pkg, gpu, 4, 30000, 1, seed=5, nsteps=16)
  est.tune(tile_width=tw, steps_per_launch=spl)
  res = {}
  for flow in (0, 1):
    est.tune(flow=flow)
    assert est.query_flow(16) == bool(flow)
    w = w0.clone()
    eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
    got = torch.zeros(3, dtype=torch.int64, device=gpu)
    est.estimate_refine(w, snaps, 0.0, dt, 16, eta, got[0:1], got[1:2].view(torch.float64),
                        got[2:3])
    torch.cuda.synchronize()
    res[flow] = (host(w), host(eta), host(got))
    e = np.abs(host(eta))
    assert int(res[flow][2][0]) == int(np.argmax(e))
    assert host(got[1:2].view(torch.float64))[0] == e.max()
    assert int(res[flow][2][2]) == 0
  assert_same(res[1][:2], res[0][:2], "refine")
  assert res[1][2].tolist() == res[0][2].tolist()
  assert op.sweep_status() == 0


def test_flow_repeats_and_alternating_shapes(pkg, gpu):
  """Take-counter epochs across repeated launches, and shapes alternating on one plan (8 and
  4 steps per block, 12, 16 and 24 steps; each change re-zeroes the control words): every launch
  gives the chain's bits, and the fused refine stays aligned with dg_argmax_ex."""
  import torch
  op, est, snaps, w0, dt = setup(pkg, gpu, 4, 20000, 1, seed=6, nsteps=24)
  est.tune(tile_width=2)
  refs = {}
  shapes = {8: (24, 16), 4: (16, 12)}
  for spl, ns in shapes.items():
    for n in ns:
      est.tune(steps_per_launch=spl)
      refs[spl, n] = run(est, snaps, w0, dt, n, 0)
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  for rep in range(3):
    for spl, ns in shapes.items():
      for n in ns:
        est.tune(steps_per_launch=spl)
        assert_same(run(est, snaps, w0, dt, n, 1), refs[spl, n], (rep, spl, n))
        w = w0.clone()
        eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
        est.estimate_refine(w, snaps[:n + 1], 0.0, dt, n, eta, got[0:1],
                            got[1:2].view(torch.float64))
        torch.cuda.synchronize()
        assert int(host(got)[0]) == int(np.argmax(np.abs(refs[spl, n][1]))), (rep, spl, n)
  assert op.sweep_status() == 0


def test_flow_fallbacks(pkg, gpu):
  """Where the shape does not split into >= 2 blocks of the plan's steps per launch (or the
  plan asks for it), the chain runs: query_flow says so and the results are the chain's."""
  op, est, snaps, w0, dt = setup(pkg, gpu, 3, 1200, 1, seed=7, nsteps=20)
  est.tune(tile_width=1, steps_per_launch=4, flow=1)
  assert est.query_flow(20) and est.query_flow(8)
  assert not est.query_flow(4)    # one block
  assert not est.query_flow(6)    # not a multiple of 4
  assert not est.query_flow(44)   # more than 40 steps
  est.tune(steps_per_launch=2)
  assert not est.query_flow(8)    # 2-step blocks: the chain only
  est.tune(steps_per_launch=4)
  for n in (4, 6):
    assert_same(run_any(est, snaps, w0, dt, n, 1), run_any(est, snaps, w0, dt, n, 0), n)


def run_any(est, snaps, w0, dt, nsteps, flow):
  import torch
  est.tune(flow=flow)
  w = w0.clone()
  eta = torch.zeros(est.lo.ktot, dtype=torch.float64, device=w.device)
  est.estimate(w, snaps[:nsteps + 1], 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True)
  torch.cuda.synchronize()
  return host(w), host(eta)


def test_flow_watchdog_gives_up_loudly(pkg, gpu):
  """A work item that gives up waiting (forced: DG_TUNE_SWEEP_SPIN_LIMIT = 1 on the lo plan)
  poisons what it publishes: eta holds NaN and the fused refine value is NaN with the
  non-finite count raised; the next call raises until sweep_status() clears the flag; a
  normal launch after that gives the chain's bits again."""
  import torch
  _lib = pkg._lib
  op, est, snaps, w0, dt = setup(pkg, gpu, 4, 1 << 18, 1, seed=8, nsteps=20)
  ref = run(est, snaps, w0, dt, 20, 0)
  _lib.check(op._lib.dg_plan_tune(op._plan, _lib.DG_TUNE_SWEEP_SPIN_LIMIT, 1), "dg_plan_tune")
  est.tune(flow=1)
  w = w0.clone()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=gpu)
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  est.estimate_refine(w, snaps, 0.0, dt, 20, eta, got[0:1], got[1:2].view(torch.float64),
                      got[2:3])
  torch.cuda.synchronize()
  assert np.isnan(host(got[1:2].view(torch.float64))[0])
  assert int(host(got)[2]) == 1
  assert np.isnan(host(eta)).any()
  with pytest.raises(_lib.DGLibraryError, match="gave up"):
    est.estimate_refine(w, snaps, 0.0, dt, 20, eta, got[0:1])
  assert op.sweep_status() == 1
  assert op.sweep_status() == 0
  _lib.check(op._lib.dg_plan_tune(op._plan, _lib.DG_TUNE_SWEEP_SPIN_LIMIT, 0), "dg_plan_tune")
  assert_same(run(est, snaps, w0, dt, 20, 1), ref, "after the watchdog fired")


@pytest.mark.slow
def test_flow_full_size(pkg, gpu):
  """Config 2's size (N = 4, K = 2^20, 20 steps, terminal weight P u^N as the bench runs it):
  the dataflow launch equals the chain bit for bit, and the fused refine index is numpy's
  argmax of |eta|."""
  import torch
  op, est, snaps, w0, dt = setup(pkg, gpu, 4, 1 << 20, 1, seed=21, nsteps=20)
  ref = run(est, snaps, w0, dt, 20, 0, term=True)
  got = run(est, snaps, w0, dt, 20, 1, term=True)
  assert_same(got, ref, "full size")
  w = w0.clone()
  eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
  idx = torch.zeros(1, dtype=torch.int64, device=gpu)
  est.estimate_refine(w, snaps, 0.0, dt, 20, eta, idx, terminal_prolong=True)
  torch.cuda.synchronize()
  assert int(host(idx)[0]) == int(np.argmax(np.abs(ref[1])))
  assert op.sweep_status() == 0
