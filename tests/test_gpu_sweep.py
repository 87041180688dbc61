"""The dataflow sweep (dg_lserk4_sweep_rec, csrc/dg_sweep.hip): forward and adjoint record
sweeps as ONE launch whose work items are the tiles of every block of steps.

Bars:
  * bit-identical to the launch-per-block pair (dg_lserk4_fwd_rec + dg_lserk4_adj_rec, the
    same tile arithmetic and steps per block) in u^N, the record, w^0 and eta -- for every Np
    the pair tiles run at 1024 elements, 10- and 20-step forward blocks, 1 to 4 adjoint
    blocks, batches with trajectory edges inside tiles, both inflow variants, a refined mesh,
    every indicator mode and a caller-supplied terminal weight;
  * repeated launches (the kernel re-arms its own queue and epochs) and HIP-graph replays give
    the same bits; a launch beside a concurrent bandwidth-heavy kernel (uneven load on the
    hand-offs, cdna_hip_programming.md §6 Guideline 16 pitfall 3) too;
  * no launch gives up waiting for a producer (dg_sweep_status);
  * shapes the dataflow launch does not cover fall back to the two launch chains (query).
The oracle comparison of this path at full size (the bench's timed launch, K = 2^20 at N = 4
and 6, and config 4's batched shape) is tests/test_gpu_full_size.py::test_full_size_dataflow_*;
the watchdog's give-up path is test_watchdog_gives_up_loudly below.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def host(t):
  return t.detach().cpu().numpy()


def noisy_sine(op, seed, batch):
  import torch
  rng = np.random.default_rng(seed)
  u0 = op.new_field()
  op.init_sine(rng.uniform(0.5, 1.5, batch), rng.integers(1, 5, batch).astype(float),
               rng.uniform(0, 6, batch), out=u0)
  gen = torch.Generator(device=u0.device).manual_seed(seed)
  u0 += 0.1 * torch.randn(u0.shape, dtype=u0.dtype, device=u0.device, generator=gen)
  return u0


def run_sweep(op, u0, dt, nsteps, dataflow, eta_assign=True, eta_abs=False, eta_init=None,
              with_eta=True, terminal=None):
  """One sweep_rec call; returns (uN, rec, w, eta) as host arrays."""
  import torch
  op.tune(rec_sweep=1 if dataflow else 0)
  rec = op.new_jumps(nsteps)
  rec.fill_(float("nan"))
  uN = op.new_field()
  w = op.new_field() if terminal is None else terminal.clone()
  eta = None
  if with_eta:
    eta = (torch.full((op.ktot,), float("nan"), dtype=torch.float64, device=op.device)
           if eta_init is None else eta_init.clone())
  op.sweep_rec(u0, rec, w, 0.0, dt, nsteps, uN=uN, eta=eta, eta_assign=eta_assign,
               eta_abs=eta_abs, terminal_state=terminal is None)
  torch.cuda.synchronize()
  out = (host(uN), host(rec), host(w), None if eta is None else host(eta))
  if dataflow:
    assert op.sweep_status() == 0, "a work item gave up waiting for a producer"
  return out


def assert_same(a, b, what):
  for name, x, y in zip(("u^N", "record", "w^0", "eta"), a, b):
    if x is None and y is None:
      continue
    np.testing.assert_array_equal(x, y, err_msg=f"{what}: {name}")


@pytest.mark.parametrize("N,K,batch,fsteps,nsteps,inflow,refined,width", [
    (4, 5000, 1, 20, 20, "a", False, 2),      # the bench's shape: forward 20, adjoint 10 + 10
    (4, 5000, 1, 10, 20, "a", False, 2),      # forward 10 + 10
    (4, 3000, 3, 20, 40, "a2", False, 2),     # trajectory edges inside tiles, 2 + 4 blocks
    (4, 2500, 2, 10, 30, "a", False, 2),      # 3 + 3 blocks
    (1, 4000, 1, 20, 20, "a", False, 2),
    (2, 1500, 2, 10, 10, "a", False, 2),      # one block each way
    (3, 2000, 1, 20, 20, "zero", False, 2),
    (5, 2000, 2, 20, 20, "a", False, 2),
    (6, 1200, 1, 10, 20, "a", False, 2),
    (7, 1100, 1, 20, 20, "a", False, 2),
    (4, 3000, 2, 20, 20, "a", True, 2),       # refined (non-uniform metric)
    (4, 700, 1, 20, 20, "a", False, 2),       # fewer elements than one tile's output
    (8, 3000, 2, 10, 20, "a", False, 1),      # Np = 9 on 512-element tiles (4-wave workgroups)
    (4, 2000, 1, 5, 20, "a2", True, 1),       # 512-element tiles, 4 + 2 blocks, refined
])
def test_dataflow_equals_launch_chains(pkg, gpu, N, K, batch, fsteps, nsteps, inflow, refined,
                                       width):
  v_x = np.linspace(0.0, 1.0, K + 1)
  if refined:
    for k in (3, 900, 901, K - 1):
      v_x = np.insert(v_x, k + 1, 0.5 * (v_x[k] + v_x[k + 1]))
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch, inflow=inflow)
  assert op.uniform != refined
  op.tune(rec_tile_width=width, rec_steps_per_launch=10, rec_fwd_steps_per_launch=fsteps)
  on, msf, msa, items = op.query_sweep(nsteps)
  assert on and (msf, msa) == (fsteps, 10) and items > 0
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 11 + N, batch)
  for assign, absval in ((True, False), (True, True)):
    ref = run_sweep(op, u0, dt, nsteps, False, assign, absval)
    got = run_sweep(op, u0, dt, nsteps, True, assign, absval)
    assert_same(got, ref, f"N={N} K={K} batch={batch} {fsteps}/{nsteps} assign={assign} abs={absval}")
  assert np.isfinite(ref[3]).all() and np.abs(ref[3]).max() > 0


def test_dataflow_indicator_modes_and_terminal_weight(pkg, gpu):
  """eta accumulated onto caller values, no eta, a caller terminal weight (in place over 2
  blocks, through a copy with one block)."""
  import torch
  N, K, nsteps = 4, 2600, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh, batch=2)
  op.tune(rec_tile_width=2, rec_steps_per_launch=10, rec_fwd_steps_per_launch=20)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 3, 2)
  init = torch.linspace(-1.0, 1.0, op.ktot, dtype=torch.float64, device=gpu)
  for kw in (dict(eta_assign=False, eta_init=init), dict(eta_assign=False, eta_abs=True,
                                                         eta_init=init),
             dict(with_eta=False)):
    ref = run_sweep(op, u0, dt, nsteps, False, **kw)
    got = run_sweep(op, u0, dt, nsteps, True, **kw)
    assert_same(got, ref, str({k: v for k, v in kw.items() if k != "eta_init"}))
  g = noisy_sine(op, 9, 2)  # an arbitrary terminal weight dJ/du^N
  for n in (20, 10):
    ref = run_sweep(op, u0, dt, n, False, terminal=g)
    got = run_sweep(op, u0, dt, n, True, terminal=g)
    assert_same(got, ref, f"terminal weight, nsteps={n}")


def test_dataflow_repeats_graphs_and_uneven_load(pkg, gpu):
  """Back-to-back launches (self re-armed queue, epochs), HIP-graph replays and launches
  racing a bandwidth-heavy copy on another stream all give the same bits."""
  import torch
  N, K, nsteps = 4, 60000, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  op.tune(rec_tile_width=2, rec_steps_per_launch=10, rec_fwd_steps_per_launch=20, rec_sweep=1)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 21, 1)
  ref = run_sweep(op, u0, dt, nsteps, False)
  rec, uN, w = op.new_jumps(nsteps), op.new_field(), op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=gpu)

  def sweep():
    op.sweep_rec(u0, rec, w, 0.0, dt, nsteps, uN=uN, eta=eta, eta_assign=True)

  def check(what):
    torch.cuda.synchronize()
    assert_same((host(uN), host(rec), host(w), host(eta)), ref, what)

  for i in range(5):
    sweep()
  check("5 back-to-back launches")
  # HIP graph (the first call above allocated the scratch outside capture)
  side = torch.cuda.Stream()
  side.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(side):
    sweep()
  torch.cuda.current_stream().wait_stream(side)
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    sweep()
  for i in range(3):
    w.zero_()
    eta.zero_()
    g.replay()
  check("graph replays")
  # uneven load: a 1 GiB stream copy on another stream while the sweeps run
  big = torch.empty(1 << 27, dtype=torch.float64, device=gpu)
  dst = torch.empty_like(big)
  copy_stream = torch.cuda.Stream()
  for i in range(3):
    with torch.cuda.stream(copy_stream):
      pkg.operators.stream_copy(big, dst)
    sweep()
    check(f"beside a concurrent copy ({i})")
  assert op.sweep_status() == 0


def test_dataflow_fallbacks(pkg, gpu):
  """Shapes the dataflow launch does not cover run the launch chains with the same results:
  nsteps not a multiple of the blocks, more than 40 steps, 512-element tiles, the switch off."""
  mesh = pkg.BaseGalerkin1D(n=4, k=1500)
  op = pkg.operators.DGAdvection1D(mesh)
  op.tune(rec_tile_width=2, rec_steps_per_launch=10, rec_fwd_steps_per_launch=20)
  assert op.query_sweep(20)[0]
  assert not op.query_sweep(15)[0]
  assert not op.query_sweep(60)[0]
  assert not op.query_sweep(0)[0]
  op.tune(rec_sweep=0)
  assert not op.query_sweep(20)[0]
  op.tune(rec_sweep=1, rec_tile_width=1, rec_steps_per_launch=10)
  assert op.query_sweep(20)[0]  # 512-element tiles, 10-step blocks
  op.tune(rec_fwd_steps_per_launch=20)
  assert op.query_sweep(20)[:3] == (True, 10, 10)  # 512-element tiles cap the blocks at 10
  op.tune(rec_tile_width=2, rec_fwd_tile_width=1)
  assert not op.query_sweep(20)[0]  # one tile width for both directions
  op.tune(rec_tile_width=2, rec_steps_per_launch=10, rec_fwd_steps_per_launch=20)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 4, 1)
  for n in (15, 7):
    ref = run_sweep(op, u0, dt, n, False)
    got = run_sweep(op, u0, dt, n, True)  # the fallback inside sweep_rec
    assert_same(got, ref, f"fallback nsteps={n}")


@pytest.mark.parametrize("N,K,fsteps,asteps,nsteps,width", [
    (4, 1 << 16, 20, 10, 20, 2),   # the bench's shape
    (4, 9000, 10, 5, 20, 2),
    (3, 3000, 5, 5, 10, 2),
    (6, 2048, 20, 10, 40, 2),
    (5, 20000, 10, 10, 20, 1),     # 512-element tiles: the reduction over 4 waves
])
def test_sweep_refine_equals_sweep_then_argmax(pkg, gpu, N, K, fsteps, asteps, nsteps, width):
  """dg_lserk4_sweep_refine (the argmax reduced by the dataflow launch's last tiles) gives the
  index, value and non-finite count of sweep_rec + dg_argmax_ex(|eta|), and the same w, eta;
  the launch-chain fallback too."""
  import torch
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  op.tune(rec_tile_width=width, rec_steps_per_launch=asteps, rec_fwd_steps_per_launch=fsteps)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 40 + N, 1)
  for dataflow in (True, False):
    op.tune(rec_sweep=1 if dataflow else 0)
    assert op.query_sweep(nsteps)[0] == dataflow
    rec, w = op.new_jumps(nsteps), op.new_field()
    eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
    ref = torch.zeros(3, dtype=torch.int64, device=gpu)
    op.sweep_rec(u0, rec, w, 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True)
    op.argmax_ex(eta, ref[0:1], ref[1:2].view(torch.float64), ref[2:3], use_abs=True)
    eta_ref, w_ref = eta.clone(), w.clone()
    got = torch.zeros(3, dtype=torch.int64, device=gpu)
    for rep in range(3):  # repeated launches (the arrival counter grows by the tiles each time)
      eta.fill_(float("nan"))
      op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, got[0:1], got[1:2].view(torch.float64),
                      got[2:3])
      torch.cuda.synchronize()
      np.testing.assert_array_equal(host(eta), host(eta_ref))
      np.testing.assert_array_equal(host(w), host(w_ref))
      assert host(got)[:2].tolist() == host(ref)[:2].tolist(), (dataflow, rep)
      assert int(host(got)[0]) == int(np.argmax(np.abs(host(eta_ref))))
    assert int(host(got)[2]) == 0 and op.sweep_status() == 0


def test_sweep_refine_ties_and_nonfinite(pkg, gpu):
  """numpy.argmax rules in the fused reduction: an exact tie across tiles goes to the lower
  index; a NaN indicator wins (first NaN) and bumps the non-finite count."""
  import torch
  N, K, nsteps = 4, 8192, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh, inflow="zero")
  op.tune(rec_tile_width=2, rec_steps_per_launch=10, rec_fwd_steps_per_launch=20, rec_sweep=1)
  assert op.query_sweep(nsteps)[0]
  dt = mesh.cfl_dt()
  # two identical bumps far apart (translation-invariant interior): their indicator patterns
  # are equal bit for bit, so the maximum is an exact tie between two tiles
  x = np.arange(K * (N + 1)) // (N + 1)
  bump = lambda c: np.exp(-((x - c) / 6.0) ** 2)  # noqa: E731
  u0h = bump(2000) + bump(6000)
  u0 = torch.tensor(u0h, dtype=torch.float64, device=gpu)
  rec, w = op.new_jumps(nsteps), op.new_field()
  eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, got[0:1], got[1:2].view(torch.float64), got[2:3])
  torch.cuda.synchronize()
  e = host(eta)
  i = int(host(got)[0])
  assert i == int(np.argmax(e)) and e[i] == e.max()
  twin = np.flatnonzero(e == e.max())
  assert len(twin) >= 2 and i == twin[0] and twin[-1] >= 4000, twin  # the tie spans tiles
  u0[5 * (N + 1) + 2] = float("nan")  # element 5 and its downwind cone turn NaN
  op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, got[0:1], got[1:2].view(torch.float64), got[2:3])
  torch.cuda.synchronize()
  e = host(eta)
  assert int(host(got)[0]) == int(np.flatnonzero(np.isnan(e))[0])
  assert np.isnan(host(got[1:2].view(torch.float64))[0]) and int(host(got)[2]) == 1


def test_sweep_refine_into_pinned_host_memory(pkg, gpu):
  """The refine decision written by the launch straight into pinned host memory (its
  dg_host_alias device address: the bench's path, no copy launch) equals the device one."""
  import torch
  mesh = pkg.BaseGalerkin1D(n=4, k=30000)
  op = pkg.operators.DGAdvection1D(mesh)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 77, 1)
  rec, w = op.new_jumps(20), op.new_field()
  eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
  dev = torch.zeros(3, dtype=torch.int64, device=gpu)
  op.sweep_refine(u0, rec, w, 0.0, dt, 20, eta, dev[0:1], dev[1:2].view(torch.float64), dev[2:3])
  host_buf = torch.full((2,), -7, dtype=torch.int64).pin_memory()
  alias = pkg.operators.host_alias(host_buf)
  assert alias is not None
  assert pkg.operators.host_alias(torch.zeros(2, dtype=torch.int64)) is None  # not pinned
  nf = torch.zeros(1, dtype=torch.int64, device=gpu)
  for _ in range(2):
    host_buf.fill_(-7)
    op.sweep_refine(u0, rec, w, 0.0, dt, 20, eta, alias, alias + 8, nf)
    torch.cuda.synchronize()
    assert host_buf.tolist() == host(dev)[:2].tolist()
  assert int(nf.item()) == 0


def test_watchdog_gives_up_loudly(pkg, gpu):
  """A work item that gives up waiting for its producers (here forced: the test-only tune key
  DG_TUNE_SWEEP_SPIN_LIMIT = 1 on a multi-block sweep) poisons what it publishes: the fused
  refine value is NaN and the non-finite count fires, eta holds NaN, the plan's next sweep
  call raises until sweep_status() reports and clears the flag, and a normal launch after
  that gives the launch chains' bits again."""
  import torch
  N, K, nsteps = 4, 1 << 18, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  assert op.query_sweep(nsteps)[:3] == (True, 20, 10)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 5, 1)
  ref = run_sweep(op, u0, dt, nsteps, False)
  op.tune(rec_sweep=1)
  _lib = pkg._lib
  _lib.check(op._lib.dg_plan_tune(op._plan, _lib.DG_TUNE_SWEEP_SPIN_LIMIT, 1), "dg_plan_tune")
  rec, w = op.new_jumps(nsteps), op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=gpu)
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, got[0:1], got[1:2].view(torch.float64),
                  got[2:3])
  torch.cuda.synchronize()
  assert np.isnan(host(got[1:2].view(torch.float64))[0]), "the fused value must be NaN"
  assert int(host(got)[2]) == 1
  assert np.isnan(host(eta)).any()
  with pytest.raises(pkg._lib.DGLibraryError, match="gave up"):
    op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, got[0:1], got[1:2].view(torch.float64),
                    got[2:3])
  assert op.sweep_status() == 1
  assert op.sweep_status() == 0  # cleared
  _lib.check(op._lib.dg_plan_tune(op._plan, _lib.DG_TUNE_SWEEP_SPIN_LIMIT, 0), "dg_plan_tune")
  assert_same(run_sweep(op, u0, dt, nsteps, True), ref, "after the watchdog fired")


def test_grown_scratch_keeps_captured_graph_valid(pkg, gpu):
  """A graph captured around sweep_rec keeps the scratch addresses in its kernel arguments;
  a later call that needs more scratch (sweep_refine's argmax slots, a longer sweep) must not
  free them: the replay still gives the same bits."""
  import torch
  N, K, nsteps = 4, 30000, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 8, 1)
  ref = run_sweep(op, u0, dt, nsteps, False)
  op.tune(rec_sweep=1)
  rec, uN, w = op.new_jumps(nsteps), op.new_field(), op.new_field()
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=gpu)

  def sweep():
    op.sweep_rec(u0, rec, w, 0.0, dt, nsteps, uN=uN, eta=eta, eta_assign=True)

  sweep()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    sweep()
  # grow the scratch: a 40-step sweep, then the fused refine decision
  run_sweep(op, u0, dt, 40, True)
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  rec40, w40 = op.new_jumps(40), op.new_field()
  e40 = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
  op.sweep_refine(u0, rec40, w40, 0.0, dt, 40, e40, got[0:1])
  torch.cuda.synchronize()
  for _ in range(2):
    w.zero_()
    eta.zero_()
    uN.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert_same((host(uN), host(rec), host(w), host(eta)), ref, "graph replay after growth")
  assert op.sweep_status() == 0


def test_alternating_shapes_keep_refine_aligned(pkg, gpu):
  """Launch shapes alternating on one plan (adjoint blocks of 10 and 5 steps: different
  adjoint tile counts) re-zero the control words on every change, so the fused refine's
  arrival counter and the take counter stay aligned: each decision equals dg_argmax_ex."""
  import torch
  N, K, nsteps = 4, 50000, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 12, 1)
  rec, w = op.new_jumps(nsteps), op.new_field()
  eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
  got = torch.zeros(3, dtype=torch.int64, device=gpu)
  ref = torch.zeros(3, dtype=torch.int64, device=gpu)
  for rep in range(3):
    for asteps in (10, 5):
      op.tune(rec_steps_per_launch=asteps, rec_fwd_steps_per_launch=20, rec_sweep=1)
      assert op.query_sweep(nsteps)[:3] == (True, 20, asteps)
      op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, got[0:1],
                      got[1:2].view(torch.float64), got[2:3])
      op.argmax_ex(eta, ref[0:1], ref[1:2].view(torch.float64), ref[2:3], use_abs=True)
      torch.cuda.synchronize()
      assert host(got)[:2].tolist() == host(ref)[:2].tolist(), (rep, asteps)
  assert op.sweep_status() == 0


@pytest.mark.parametrize("N,K,batch,waves,fsteps,nsteps", [
    (4, 9000, 1, 12, 20, 20),   # 1536-element tiles
    (4, 7000, 2, 16, 20, 20),   # 2048-element tiles, trajectory edges inside tiles
    (1, 9000, 1, 16, 10, 20),
    (8, 6000, 1, 12, 20, 20),   # Np = 9: the launch chains run 1024 forward / 512 adjoint tiles
    (6, 5000, 1, 12, 10, 40),
])
def test_wide_dataflow_tiles_equal_launch_chains(pkg, gpu, N, K, batch, waves, fsteps, nsteps):
  """DG_TUNE_SWEEP_WAVES = 12 / 16: the dataflow launch on tiles of 1536 / 2048 elements in both
  directions (also where the launch chains' forward and adjoint widths differ, Np = 9) gives
  the launch chains' bits: every element's arithmetic is the same on any tile."""
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch)
  op.tune(rec_steps_per_launch=10, rec_fwd_steps_per_launch=fsteps)
  if N == 8:
    op.tune(rec_tile_width=1, rec_fwd_tile_width=2)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 60 + N, batch)
  ref = run_sweep(op, u0, dt, nsteps, False)
  op.tune(sweep_waves=waves, rec_sweep=1)
  on, f, a, items, w, T = op.query_sweep(nsteps, tile=True)
  assert on and (f, a, w, T) == (fsteps, 10, waves, 128 * waves)
  got = run_sweep(op, u0, dt, nsteps, True)
  assert_same(got, ref, f"{waves} waves, N={N}")


@pytest.mark.parametrize("N,K,batch,waves,fsteps,nsteps,inflow", [
    (1, 9000, 1, 8, 20, 20, "a"),    # 2048-element tiles
    (1, 3001, 3, 8, 10, 20, "a2"),   # trajectory edges inside tiles, odd element count
    (2, 7000, 1, 4, 20, 40, "a"),    # 1024-element tiles on 4 waves
    (2, 2500, 2, 8, 10, 30, "zero"),
])
def test_four_elements_per_lane_equal_launch_chains(pkg, gpu, N, K, batch, waves, fsteps, nsteps,
                                                    inflow):
  """DG_TUNE_SWEEP_LANE_ELEMENTS = 4 (Np <= 3): the dataflow launch with four consecutive
  elements per lane (two 16-byte record accesses per lane and step) gives the launch chains'
  bits."""
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch, inflow=inflow)
  op.tune(rec_steps_per_launch=10, rec_fwd_steps_per_launch=fsteps)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 70 + N, batch)
  ref = run_sweep(op, u0, dt, nsteps, False)
  op.tune(sweep_waves=waves, sweep_lane_elements=4, rec_sweep=1)
  on, f, a, items, w, T = op.query_sweep(nsteps, tile=True)
  assert on and (f, a, w, T) == (fsteps, 10, waves, 256 * waves)
  got = run_sweep(op, u0, dt, nsteps, True)
  assert_same(got, ref, f"4 elements per lane, N={N}, {waves} waves")
  # and the fused refine decision on these tiles
  import torch
  rec, w_ = op.new_jumps(nsteps), op.new_field()
  eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
  res = torch.zeros(3, dtype=torch.int64, device=gpu)
  if batch == 1:
    op.sweep_refine(u0, rec, w_, 0.0, dt, nsteps, eta, res[0:1], res[1:2].view(torch.float64),
                    res[2:3])
    torch.cuda.synchronize()
    e = np.abs(host(eta))
    assert int(host(res)[0]) == int(np.argmax(e)) and op.sweep_status() == 0


@pytest.mark.parametrize("N,K,batch,waves,fsteps,nsteps,inflow,refined", [
    (4, 9000, 1, 12, 20, 20, "a", False),    # the headline shape: 1404-element tiles
    (4, 7000, 3, 12, 20, 40, "a2", False),   # trajectory edges inside tiles, 2 + 4 blocks
    (4, 5000, 2, 8, 10, 20, "a", True),      # 940-element tiles, refined (non-uniform metric)
    (1, 9000, 1, 8, 20, 20, "a", False),     # Np = 2 at 8 waves per SIMD
    (1, 3001, 3, 16, 10, 20, "zero", False),  # 1868-element tiles, odd element count
    (2, 6000, 1, 12, 20, 20, "a", False),
    (3, 2000, 2, 16, 10, 30, "a", False),
    (5, 4000, 1, 12, 20, 20, "a2", False),
    (6, 5000, 1, 12, 10, 40, "a", False),
    (7, 3000, 2, 8, 20, 20, "a", True),
    (8, 6000, 1, 8, 20, 20, "a", False),     # Np = 9 (operator blocks re-read from kernargs)
    (4, 700, 1, 12, 20, 20, "a", False),     # fewer elements than one tile's output
])
def test_overlapped_waves_equal_launch_chains(pkg, gpu, N, K, batch, waves, fsteps, nsteps,
                                              inflow, refined):
  """DG_TUNE_SWEEP_EXCHANGE = 1 (dg_ovl_tiles.h): faces within a wave by DPP, ghosts refreshed
  through LDS once per step.  Every element's arithmetic is the pair tiles' on the same doubles,
  so u^N, the record, w^0 and eta equal the launch chains' bit for bit; the fused refine
  decision equals numpy's argmax of |eta|."""
  import torch
  v_x = np.linspace(0.0, 1.0, K + 1)
  if refined:
    for k in (3, 900, 901, K - 1):
      v_x = np.insert(v_x, k + 1, 0.5 * (v_x[k] + v_x[k + 1]))
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch, inflow=inflow)
  op.tune(rec_steps_per_launch=10, rec_fwd_steps_per_launch=fsteps)
  if N == 8:
    op.tune(rec_tile_width=1, rec_fwd_tile_width=2)
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 80 + N, batch)
  ref = run_sweep(op, u0, dt, nsteps, False)
  op.tune(sweep_waves=waves, sweep_exchange=1, rec_sweep=1)
  on, f, a, items, w, T = op.query_sweep(nsteps, tile=True)
  assert on and (f, a, w, T) == (fsteps, 10, waves, 116 * waves + 12)
  for rep in range(2):
    got = run_sweep(op, u0, dt, nsteps, True)
    assert_same(got, ref, f"overlapped waves, N={N}, {waves} waves, rep {rep}")
  if batch == 1:
    rec, w_ = op.new_jumps(nsteps), op.new_field()
    eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
    res = torch.zeros(3, dtype=torch.int64, device=gpu)
    op.sweep_refine(u0, rec, w_, 0.0, dt, nsteps, eta, res[0:1], res[1:2].view(torch.float64),
                    res[2:3])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(np.abs(host(eta)), np.abs(ref[3]))
    e = np.abs(host(eta))
    assert int(host(res)[0]) == int(np.argmax(e)) and op.sweep_status() == 0


def test_refine_loop_reuses_the_sweep_scratch(pkg, gpu):
  """An adapt loop on the public API (sweep_refine, then refine the winner, within the plan's
  reserved capacity) must not grow device memory: the dataflow scratch is sized for the
  capacity, so the refines reuse one region (each refine used to retire the old
  region and allocate a slightly larger one, tens of MB per iteration at this size)."""
  import torch
  N, K, nsteps, iters = 4, 60000, 20, 8
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  op.reserve(K + 2 * iters)
  dt = mesh.cfl_dt()
  field_bytes = 8 * (N + 1) * (K + iters)
  free = []
  for it in range(iters):
    u0 = noisy_sine(op, 90 + it, 1)
    rec, w = op.new_jumps(nsteps), op.new_field()
    eta = torch.empty(op.ktot, dtype=torch.float64, device=gpu)
    res = torch.zeros(3, dtype=torch.int64, device=gpu)
    assert op.query_sweep(nsteps)[0]
    op.sweep_refine(u0, rec, w, 0.0, dt, nsteps, eta, res[0:1], res[1:2].view(torch.float64),
                    res[2:3])
    torch.cuda.synchronize()
    assert int(host(res)[0]) == int(np.argmax(np.abs(host(eta))))
    op.refine(res[0:1])
    torch.cuda.synchronize()
    del u0, rec, w, eta
    torch.cuda.empty_cache()
    free.append(torch.cuda.mem_get_info(gpu)[0])
  assert op.sweep_status() == 0
  # after the first iteration (which allocates the scratch) free memory stays flat
  assert free[0] - free[-1] < field_bytes, (free, field_bytes)
