"""Config-3 path on the GPU (Burgers-type flux, SlopeLimitN after every LSERK4 stage,
frozen-decision adjoint, device-side refinement) vs the CPU oracle (oracle/burgers.py),
through the C ABI.  Needs an MI355X.

Tolerances: fp64 fields and indicators within RTOL = 1e-10 of max|oracle| (north_star);
the device split of the mesh is bit-exact against the host split_interval.  As for the
linear path, the adjoint/indicator oracle is fed the GPU's own forward snapshots.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import burgers as ob
from oracle import setup1d

pytestmark = pytest.mark.gpu

RTOL = 1e-10
A = 2 * np.pi
PHYSICS = [("burgers", True), ("burgers", False), ("linear", True), ("burgers", "1")]


def rel_err(x, ref):
  x, ref = np.asarray(x), np.asarray(ref)
  return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-300))


def dev(x, device):
  import torch
  return torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=device)


def host(t):
  return t.detach().cpu().numpy()


def setup(pkg, N, K, v_x=None, **kw):
  if v_x is None:
    _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  S = setup1d.startup1d(N, v_x, metric="element")
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  return S, mesh, pkg.operators.DGAdvection1D(mesh, **kw)


def ic(S, rng, jump=0.8):
  x = S["x"]
  return np.sin(2 * np.pi * x) + jump * (x > 0.5) + 0.05 * rng.standard_normal(x.shape)


def refined_vx(K, rng):
  _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  for _ in range(7):
    v_x = np.insert(v_x, (j := int(rng.integers(0, len(v_x) - 1))) + 1,
                    0.5 * (v_x[j] + v_x[j + 1]))
  return v_x


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("N", [1, 2, 4, 8])
@pytest.mark.parametrize("inflow", ["a", "a2"])
def test_burgers_rhs(pkg, gpu, N, inflow):
  rng = np.random.default_rng(N)
  S, mesh, op = setup(pkg, N, 333, flux="burgers", inflow=inflow)
  u = rng.standard_normal((N + 1, 333))
  ref, _ = ob.rhs(u, 0.37, A, S, ob.FLUX_BURGERS, inflow)
  got = host(op.rhs(dev(setup1d.to_elem_major(u), gpu), 0.37))
  assert rel_err(setup1d.from_elem_major(got, N + 1), ref) <= RTOL


def test_burgers_rhs_nonuniform(pkg, gpu):
  rng = np.random.default_rng(3)
  v_x = refined_vx(200, rng)
  S, mesh, op = setup(pkg, 3, None, v_x=v_x, flux="burgers")
  assert not op.uniform
  u = rng.standard_normal((4, len(v_x) - 1))
  ref, _ = ob.rhs(u, 0.1, A, S)
  got = host(op.rhs(dev(setup1d.to_elem_major(u), gpu), 0.1))
  assert rel_err(setup1d.from_elem_major(got, 4), ref) <= RTOL


@pytest.mark.parametrize("flux,limit", PHYSICS)
@pytest.mark.parametrize("N,K,uniform", [(4, 300, True), (2, 257, True), (7, 150, True),
                                         (3, 240, False)])
def test_limited_forward_sweep(pkg, gpu, flux, limit, N, K, uniform):
  rng = np.random.default_rng(N * 1000 + K)
  v_x = None if uniform else refined_vx(K, rng)
  S, mesh, op = setup(pkg, N, K, v_x=v_x, flux=flux, limiter=limit)
  u0 = ic(S, rng)
  dt = oadv.bench_dt(S)
  nsteps = 5  # snapshots: 1 step per launch by default; ping-pong: 2 + 2 + 1
  ref, _ = ob.forward_sweep(u0, 0.02, dt, nsteps, A, S, flux, limit=limit)
  if limit:
    counts = ob.limiter_stage_ids(u0, 0.02, dt, 1, A, S, flux)
    assert min(counts[0]) > 0  # the limiter is active
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.02, dt, nsteps, snaps)
  for n in range(nsteps + 1):
    assert rel_err(setup1d.from_elem_major(host(snaps[n]), N + 1), ref[n]) <= RTOL, n
  np.testing.assert_array_equal(host(u), host(snaps[nsteps]))
  # ping-pong path (no snapshots: 2 + 2 + 1 steps per launch; the snapshot path ran 1 per
  # launch, so the two may differ in the last bit where the compiler contracted differently)
  u2 = dev(setup1d.to_elem_major(u0), gpu)
  op.forward(u2, 0.02, dt, nsteps)
  assert rel_err(host(u2), host(snaps[nsteps])) <= 1e-12
  op.tune(steps_per_launch=1)
  u3 = dev(setup1d.to_elem_major(u0), gpu)
  op.forward(u3, 0.02, dt, nsteps)
  assert rel_err(host(u3), host(u2)) <= 1e-12
  op.tune(steps_per_launch=2)  # 2-step launches writing snapshots (2 + 2 + 1)
  snaps2 = op.new_field(nsteps + 1)
  u4 = dev(setup1d.to_elem_major(u0), gpu)
  op.forward(u4, 0.02, dt, nsteps, snaps2)
  for n in range(nsteps + 1):
    assert rel_err(host(snaps2[n]), host(snaps[n])) <= 1e-12, n


@pytest.mark.parametrize("flux,limit", PHYSICS)
@pytest.mark.parametrize("N,K,uniform", [(3, 70, True), (4, 45, False)])
def test_adjoint_sweep_and_indicator(pkg, gpu, flux, limit, N, K, uniform):
  import torch
  rng = np.random.default_rng(K + N)
  v_x = None if uniform else refined_vx(K, rng)
  S, mesh, op = setup(pkg, N, K, v_x=v_x, flux=flux, limiter=limit)
  K = S["K"]
  u0 = ic(S, rng)
  dt = oadv.bench_dt(S)
  nsteps, src = 3, 0.6
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.01, dt, nsteps, snaps)
  times = [0.01]
  for _ in range(nsteps):
    times.append(times[-1] + dt)
  gsnaps = [setup1d.from_elem_major(host(snaps[n]), N + 1) for n in range(nsteps + 1)]
  g = rng.standard_normal(u0.shape)
  w_ref, eta_ref, _ = ob.adjoint_sweep(g, gsnaps, times, dt, A, S, flux, limit=limit,
                                       src_coef=src)
  w = dev(setup1d.to_elem_major(g), gpu)
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, 0.01, dt, nsteps, src_coef=src, eta=eta)
  assert rel_err(setup1d.from_elem_major(host(w), N + 1), w_ref) <= RTOL
  assert rel_err(host(eta), eta_ref) <= RTOL


@pytest.mark.parametrize("limit", [False, True, "1"])
def test_gradient_matches_finite_difference(pkg, gpu, limit):
  """dJ/du0 through 4 limited Burgers steps vs a central difference of J on the GPU
  (matlab/test_jacobian.m:38-55 method).  With the limiter the step is only piecewise
  smooth: its troubled-cell test compares against eps0 = 1e-8 (SlopeLimitN.m:23), so the
  difference step must stay far below that for no decision to flip (h = 1e-10, and a
  looser tolerance for the rounding of the difference quotient)."""
  import torch
  rng = np.random.default_rng(11)
  S, mesh, op = setup(pkg, 4, 400, flux="burgers", limiter=limit)
  u0 = dev(setup1d.to_elem_major(ic(S, rng)), gpu)
  d = dev(rng.standard_normal(5 * 400), gpu)
  g = dev(rng.standard_normal(5 * 400), gpu)
  dt = oadv.bench_dt(S)
  nsteps, src = 4, 0.3

  def J(x):
    snaps = op.new_field(nsteps + 1)
    op.forward(x.clone(), 0.0, dt, nsteps, snaps)
    val = float(torch.dot(g, snaps[nsteps]))
    for n in range(nsteps):
      val += 0.5 * src * float(torch.dot(snaps[n], snaps[n]))
    return val, snaps

  _, snaps = J(u0)
  w = g.clone()
  op.adjoint(w, snaps, 0.0, dt, nsteps, src_coef=src)
  h, tol = (1e-10, 1e-5) if limit else (1e-6, 1e-7)
  # Difference the fields before the dot products: J(u+hd) - J(u-hd) formed from two
  # rounded J values would carry ~eps*|J|/h of noise (1e-5 relative at h = 1e-10).
  _, sp = J(u0 + h * d)
  _, sm = J(u0 - h * d)
  fd = float(torch.dot(g, sp[nsteps] - sm[nsteps]))
  for n in range(nsteps):
    fd += 0.5 * src * float(torch.dot(sp[n] - sm[n], sp[n] + sm[n]))
  fd /= 2 * h
  ad = float(torch.dot(w, d))
  assert abs(fd - ad) <= tol * abs(ad)


def test_adjoint_in_place_on_terminal_snapshot(pkg, gpu):
  import torch
  rng = np.random.default_rng(12)
  S, mesh, op = setup(pkg, 4, 500, flux="burgers", limiter=True)
  u0 = dev(setup1d.to_elem_major(ic(S, rng)), gpu)
  dt = oadv.bench_dt(S)
  for nsteps in (1, 4):
    snaps = op.new_field(nsteps + 1)
    op.forward(u0.clone(), 0.0, dt, nsteps, snaps)
    w = snaps[nsteps].clone()
    e1 = torch.zeros(500, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.0, dt, nsteps, eta=e1)
    e2 = torch.zeros(500, dtype=torch.float64, device=gpu)
    op.adjoint(snaps[nsteps], snaps, 0.0, dt, nsteps, eta=e2)
    np.testing.assert_array_equal(host(snaps[nsteps]), host(w))
    np.testing.assert_array_equal(host(e1), host(e2))


# ---------------------------------------------------------------------------
def test_device_refine_is_the_host_split(pkg, gpu):
  """dg_plan_refine == split_interval (Main_finite_difference.py:336-341) bit-exactly, and
  the refined plan computes exactly what a plan created on the split mesh computes."""
  import torch
  rng = np.random.default_rng(13)
  K0 = 300
  S, mesh, op = setup(pkg, 4, K0, flux="burgers", limiter=True)
  op.reserve(K0 + 8)
  v_host = mesh.v_x.copy()
  hs = torch.zeros(1, dtype=torch.float64, device=gpu)
  for j in (0, 17, K0 - 1, 150, 151, 3):
    idx = torch.tensor([j], dtype=torch.int64, device=gpu)
    h_expect = v_host[j + 1] - v_host[j]
    op.refine(idx, hs)
    v_host = pkg.split_interval(v_host, j)
    np.testing.assert_array_equal(op.v_x(), v_host)
    assert float(hs.item()) == h_expect
  assert op.K == K0 + 6 and not op.uniform
  with pytest.raises(pkg._lib.DGLibraryError):
    for _ in range(3):
      op.refine(torch.tensor([0], dtype=torch.int64, device=gpu))
  # same results as a fresh plan on the refined mesh
  fresh = pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=4, v_x=op.v_x()), flux="burgers",
                                      limiter=True)
  S2 = setup1d.startup1d(4, fresh.mesh.v_x, metric="element")
  u0 = dev(setup1d.to_elem_major(ic(S2, rng)), gpu)
  dt = oadv.bench_dt(S2)
  a_, b_ = u0.clone(), u0.clone()
  op.forward(a_, 0.0, dt, 3)
  fresh.forward(b_, 0.0, dt, 3)
  np.testing.assert_array_equal(host(a_), host(b_))


def test_refine_loop_with_device_argmax(pkg, gpu):
  """Adapt loop on the device: init IC, limited fwd + adj, argmax |eta|, refine — the
  refine indices agree with the oracle's argmax on the same snapshots whenever its top-2
  gap exceeds the parity tolerance."""
  import torch
  N, K0, nsteps = 3, 120, 4
  S, mesh, op = setup(pkg, N, K0, flux="burgers", limiter=True)
  op.reserve(K0 + 5)
  for _ in range(4):
    v_x = op.v_x()
    S = setup1d.startup1d(N, v_x, metric="element")
    dt = oadv.bench_dt(S)
    snaps = op.new_field(nsteps + 1)
    op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
    np.testing.assert_allclose(setup1d.from_elem_major(host(snaps[0]), N + 1),
                               np.sin(2 * np.pi * S["x"]), atol=1e-13)
    op.forward(snaps[0], 0.0, dt, nsteps, snaps)
    w = snaps[nsteps].clone()
    eta = torch.zeros(op.K, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.0, dt, nsteps, eta=eta)
    idx = op.argmax_async(eta, use_abs=True)
    gs = [setup1d.from_elem_major(host(snaps[n]), N + 1) for n in range(nsteps + 1)]
    times = [0.0]
    for _n in range(nsteps):
      times.append(times[-1] + dt)
    _, eta_ref, _ = ob.adjoint_sweep(gs[-1], gs, times, dt, A, S, limit=True)
    assert rel_err(host(eta), eta_ref) <= RTOL
    top = np.sort(np.abs(eta_ref))[::-1]
    j = int(idx.item())
    if top[0] - top[1] > 1e-8 * top[0]:
      assert j == int(np.argmax(np.abs(eta_ref)))
    k_before = op.K
    op.refine(idx)
    assert op.K == k_before + 1
    np.testing.assert_array_equal(op.v_x(), pkg.split_interval(v_x, j))


@pytest.mark.slow
def test_full_size_config3(pkg, gpu):
  """BASELINE config 3 size (N=4, K=4,194,304, Burgers + limiter): 2 limited steps vs
  the oracle, and the size-independent gradient identity of one adjoint step (central
  difference of <g, S(u)>).  The directions are smooth: a random perturbation of size h
  would itself trip SlopeLimitN's 1e-8 troubled-cell test in every cell."""
  import torch
  N, K, nsteps = 4, 1 << 22, 2
  S, mesh, op = setup(pkg, N, K, flux="burgers", limiter=True)
  x = S["x"]
  u0 = np.sin(2 * np.pi * x) + 0.5 * (x > 0.5)
  dt = oadv.bench_dt(S)
  ref, _ = ob.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.0, dt, nsteps, snaps)
  assert rel_err(setup1d.from_elem_major(host(u), N + 1), ref[-1]) <= RTOL
  del ref
  g = dev(setup1d.to_elem_major(np.sin(5 * np.pi * x)), gpu)
  d = dev(setup1d.to_elem_major(np.cos(3 * np.pi * x) + 0.3 * np.sin(7 * np.pi * x)), gpu)
  w = g.clone()
  op.adjoint(w, snaps[:2].contiguous(), 0.0, dt, 1)
  # <g, S(u + h d) - S(u - h d)> / 2h, differencing the fields before the dot product: a
  # difference of two 2e7-term dot products would carry their rounding (~1e-9) / 2h.
  h = 1e-6
  yp, ym = snaps[0] + h * d, snaps[0] - h * d
  op.forward(yp, 0.0, dt, 1)
  op.forward(ym, 0.0, dt, 1)
  fd = float(torch.dot(g, yp - ym)) / (2 * h)
  ad = float(torch.dot(w, d))
  assert abs(fd - ad) <= 1e-5 * abs(ad)


def test_adaptive_sweep_driver(pkg, gpu):
  """adaptive.AdaptiveSweep (the config-3 bench loop): its step size follows the CFL rule
  on the refined mesh and its refine sequence equals the host-split loop's."""
  import torch
  N, K0, nsteps = 4, 200, 3
  mesh = pkg.BaseGalerkin1D(n=N, k=K0)
  run = pkg.adaptive.AdaptiveSweep(mesh, nsteps, 6)
  v_x = mesh.v_x.copy()
  for _ in range(5):
    ref_mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
    assert abs(run.dt - ref_mesh.cfl_dt()) <= 1e-12 * ref_mesh.cfl_dt()
    dt = run.dt
    _, j = run.iterate()
    # host-side replay of the same iteration on a fresh plan
    op = pkg.operators.DGAdvection1D(ref_mesh, flux="burgers", limiter=True)
    snaps = op.new_field(nsteps + 1)
    op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
    op.forward(snaps[0], 0.0, dt, nsteps, snaps)
    eta = torch.zeros(op.K, dtype=torch.float64, device=gpu)
    op.adjoint(snaps[nsteps], snaps, 0.0, dt, nsteps, eta=eta)
    assert j == op.argmax(eta, use_abs=True)
    v_x = pkg.split_interval(v_x, j)
    np.testing.assert_array_equal(run.op.v_x(), v_x)
  assert run.K == K0 + 5


def test_diverged_sweep_is_refused(pkg, gpu):
  """A time step far above the CFL limit blows the unlimited sweep up; the adapt loop
  raises instead of refining on a NaN indicator."""
  mesh = pkg.BaseGalerkin1D(n=4, k=64, domain=[0.0, 1.0])
  run = pkg.adaptive.AdaptiveSweep(mesh, 300, 2, flux="linear", limiter=False, cfl=60.0)
  with pytest.raises(FloatingPointError):
    run.iterate()


def window_setup(N, v_x, k0, k1, s_glob):
  """The oracle's setup on elements [k0, k1) of a uniform mesh, with the plan's global
  metric 2/mean(h) (the window's own mean differs in the last bit).

  The window's coordinates start at 0 (v_x[k0] subtracted; exact on mesh_gen1d's dyadic
  vertices).  SlopeLimitLin.m:10-11 forms h = x_N - x_0 and x - x0 from nodal coordinates,
  which at x ~ 0.5 and h = 2^-22 carry relative rounding of eps*|x|/h ~ 2e-10; the kernels use
  h*r/2 (exact).  Only differences of x enter the limiter, so the shift changes nothing but
  that rounding: measured on this test's jump window, the unshifted oracle's one-step forward
  differs from the GPU's by 1.7e-11 and its adjoint by 2.7e-10 of max|w|, the shifted one by
  1.8e-15 and 1.4e-14."""
  S = setup1d.startup1d(N, v_x[k0:k1 + 1] - v_x[k0], metric="element")
  S["rx"][:] = s_glob
  S["Fscale"][:] = s_glob
  S["J"][:] = 1.0 / s_glob
  return S


@pytest.mark.slow
def test_full_size_config3_adjoint_and_indicator(pkg, gpu):
  """BASELINE config 3 size (N=4, K=4,194,304, Burgers + SlopeLimitN per stage, 2 steps):
  the GPU's adjoint w^0 and indicator eta against oracle/burgers.py's adjoint sweep on the
  GPU's own snapshots.  The oracle's coloured-Jacobian transpose costs
  ~100 tangent sweeps per step, so it runs on windows of the full mesh: w^0 and eta of an
  element depend only on the snapshots and w^N within the adjoint's cone (10 elements per
  limited step and side), so on a window's interior -- 30 elements in from a cut -- the
  windowed oracle is the full-size oracle.  Windows: the inflow boundary, the jump at x = 0.5
  (troubled cells), a random interior stretch and the outflow boundary."""
  import torch
  N, K, nsteps, margin = 4, 1 << 22, 2, 30
  _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  op = pkg.operators.DGAdvection1D(mesh, flux="burgers", limiter=True)
  assert op.uniform
  h = np.diff(v_x)
  s_glob = 2.0 / (np.cumsum(h)[-1] / K)
  rng = np.random.default_rng(42)
  snaps = op.new_field(nsteps + 1)
  # u0 = sin(2 pi x) + 0.8 (x > 0.5) + seeded per-node noise, built on the device from the
  # node coordinates.  The noise makes the interelement jumps O(0.01) everywhere: a smooth
  # IC's jumps at h = 2^-22 are below fp64 resolution, its indicator rounding noise (the
  # first version of this test saw |eta| ~ 1e-16 in the interior window).
  r = torch.tensor(setup1d.jacobi_gl(0, 0, N), dtype=torch.float64, device=gpu)
  vxd = torch.tensor(v_x, dtype=torch.float64, device=gpu)
  xd = vxd[:-1, None] + 0.5 * (r[None, :] + 1.0) * (vxd[1:] - vxd[:-1])[:, None]  # (K, Np)
  gen = torch.Generator(device=gpu).manual_seed(7)
  noise = torch.randn(xd.shape, generator=gen, dtype=torch.float64, device=gpu)
  snaps[0].copy_((torch.sin(2 * np.pi * xd) + 0.8 * (xd > 0.5) + 0.01 * noise).reshape(-1))
  dt = mesh.cfl_dt()
  op.forward(snaps[0], 0.0, dt, nsteps, snaps)
  wT = (torch.cos(3 * np.pi * xd) + 0.2 * torch.sin(11 * np.pi * xd)).reshape(-1)
  w = wT.clone()
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, 0.0, dt, nsteps, eta=eta)
  torch.cuda.synchronize()
  times = [0.0]
  for _ in range(nsteps):
    times.append(times[-1] + dt)
  k_jump = int(np.searchsorted(v_x, 0.5)) - 200
  k_rand = int(rng.integers(1000, K - 2000))
  Np = N + 1
  for k0, k1 in ((0, 400), (k_jump, k_jump + 400), (k_rand, k_rand + 400), (K - 400, K)):
    S = window_setup(N, v_x, k0, k1, s_glob)
    sl = slice(k0 * Np, k1 * Np)
    gs = [setup1d.from_elem_major(host(snaps[n][sl]), Np) for n in range(nsteps + 1)]
    gw = setup1d.from_elem_major(host(wT[sl]), Np)
    w_ref, eta_ref, _ = ob.adjoint_sweep(gw, gs, times, dt, A, S, limit=True)
    lo = 0 if k0 == 0 else margin  # a real boundary needs no margin
    hi = (k1 - k0) if k1 == K else (k1 - k0) - margin
    got_w = setup1d.from_elem_major(host(w[sl]), Np)[:, lo:hi]
    assert rel_err(got_w, w_ref[:, lo:hi]) <= RTOL, (k0, rel_err(got_w, w_ref[:, lo:hi]))
    got_eta = host(eta[k0:k1])[lo:hi]
    assert rel_err(got_eta, eta_ref[lo:hi]) <= RTOL, (k0, rel_err(got_eta, eta_ref[lo:hi]))
  # the jump window holds troubled cells (the frozen-decision transpose is exercised)
  u_mid = setup1d.from_elem_major(host(snaps[1][k_jump * Np:(k_jump + 400) * Np]), Np)
  _, ids = ob.limited_step(u_mid, times[1], dt, A, window_setup(N, v_x, k_jump, k_jump + 400,
                                                                  s_glob), return_ids=True)
  assert sum(i.size for i in ids) > 0


def _device_ic(pkg, run, gpu, seed=7):
  """u0 = sin(2 pi x) + 0.8 (x > 0.5) + seeded per-node noise on the run's current mesh,
  built on the device from the node coordinates (the noise keeps every interelement jump
  O(0.01): a smooth IC's jumps at h = 2^-22 are below fp64 resolution)."""
  import torch
  N = run.op.N
  r = torch.tensor(setup1d.jacobi_gl(0, 0, N), dtype=torch.float64, device=gpu)
  vx = torch.tensor(run.op.v_x(), dtype=torch.float64, device=gpu)
  xd = vx[:-1, None] + 0.5 * (r[None, :] + 1.0) * (vx[1:] - vx[:-1])[:, None]
  gen = torch.Generator(device=gpu).manual_seed(seed)
  noise = torch.randn(xd.shape, generator=gen, dtype=torch.float64, device=gpu)
  return (torch.sin(2 * np.pi * xd) + 0.8 * (xd > 0.5) + 0.01 * noise).reshape(-1)


@pytest.mark.slow
@pytest.mark.parametrize("exchange", [1, 0])
def test_full_size_config3_bench_path(pkg, gpu, exchange):
  """The timed config-3 instantiation against the oracle: BASELINE config
  3's N = 4, K = 2^22 through adaptive.AdaptiveSweep -- the bench's own calls, forward with the
  decision record and the adjoint in place on u^N reading it -- after device refinements (two
  adapt iterations, then splits placed inside the checked windows), so the plan is non-uniform
  and the UNI = false kernels run; 20 + 20 steps; a jump IC, so troubled cells exist every step
  and the adjoint's wide-cone pass runs beside the narrow-cone tiles / windows (the decision
  record is checked to hold troubled cells).  Both exchanges (DG_TUNE_NL_EXCHANGE).

  The oracle (oracle/burgers.py) runs on windows of the refined mesh: an output depends only on
  its cone -- 10 elements per limited step and side for the forward, and for w^0 / eta 10 per
  reverse step on the GPU's own snapshots -- so 220 elements in from a cut the windowed oracle
  is the full-size oracle after 20 steps.  Windows: the inflow boundary, the jump at x = 0.5
  (troubled cells, refined elements), a random interior stretch with refined elements, the
  outflow boundary, and the GPU's top-2 |eta| elements.  Forward states: every snapshot within
  1e-10 of max|oracle|; w^0 and eta likewise.  The refine index: the device argmax is numpy's
  argmax of the GPU's |eta|, and when its margin over the runner-up clears the parity
  tolerance, the oracle ranks the two the same way."""
  import torch
  N, K0, nsteps, margin, width = 4, 1 << 22, 20, 220, 800
  Np = N + 1
  mesh = pkg.BaseGalerkin1D(n=N, k=K0, domain=[0.0, 1.0])
  run = pkg.adaptive.AdaptiveSweep(mesh, nsteps, 16, flux="burgers", limiter=True)
  run.op.tune(nl_exchange=exchange)
  for _ in range(2):  # the bench's iterations (sin IC): argmax |eta| and the device split
    run.iterate()
  rng = np.random.default_rng(2026)
  k_jump = int(np.searchsorted(run.op.v_x(), 0.5))
  k_rand = int(rng.integers(20000, K0 - 20000))
  for j in (k_jump - 120, k_jump + 90, k_rand + 300, k_rand + 301, k_rand + 500):
    run.op.refine(torch.tensor([j], dtype=torch.int64, device=gpu))
  run.h_min = float(np.min(np.diff(run.op.v_x())))  # the CFL step on the refined mesh
  assert not run.op.uniform
  v_x = run.op.v_x()
  K = run.K
  snaps = run.snapshots()
  snaps[0].copy_(_device_ic(pkg, run, gpu))
  dt = run.dt
  run.forward(dt, init=False)
  uN = snaps[nsteps].clone()  # the terminal weight: the adjoint runs in place on u^N
  run.adjoint(dt)
  eta = run.eta()
  idx = run.op.argmax(eta, use_abs=True)
  torch.cuda.synchronize()
  dec = run.decisions()
  assert int(torch.count_nonzero(dec)) > 0  # troubled cells: the wide pass ran
  top = torch.topk(eta.abs(), 2)
  i1, i2 = (int(i) for i in top.indices)
  assert idx == i1 == int(np.argmax(np.abs(host(eta))))
  times = [0.0]
  for _ in range(nsteps):
    times.append(times[-1] + dt)
  k_jump = int(np.searchsorted(v_x, 0.5))
  windows = [(0, width), (k_jump - width // 2, k_jump + width // 2),
             (k_rand, k_rand + width), (K - width, K)]
  for c in (i1, i2):
    k0 = min(max(c - width // 2, 0), K - width)
    windows.append((k0, k0 + width))
  h = np.diff(v_x)
  refined = np.flatnonzero(h < h.max() * 0.75)
  eta_ref_at = {}
  for k0, k1 in windows:
    S = setup1d.startup1d(N, v_x[k0:k1 + 1] - v_x[k0], metric="element")
    sl = slice(k0 * Np, k1 * Np)
    lo = 0 if k0 == 0 else margin  # a real boundary needs no margin
    hi = (k1 - k0) if k1 == K else (k1 - k0) - margin
    gs = [setup1d.from_elem_major(host(snaps[n][sl]), Np) for n in range(nsteps)]
    gs.append(setup1d.from_elem_major(host(uN[sl]), Np))
    ref, _ = ob.forward_sweep(gs[0], 0.0, dt, nsteps, A, S)
    for n in range(1, nsteps + 1):
      err = rel_err(gs[n][:, lo:hi], ref[n][:, lo:hi])
      assert err <= RTOL, (k0, n, err)
    w_ref, eta_ref, _ = ob.adjoint_sweep(gs[-1], gs, times, dt, A, S, limit=True)
    got_w = setup1d.from_elem_major(host(snaps[nsteps][sl]), Np)[:, lo:hi]
    assert rel_err(got_w, w_ref[:, lo:hi]) <= RTOL, (k0, rel_err(got_w, w_ref[:, lo:hi]))
    got_eta = host(eta[k0:k1])[lo:hi]
    assert rel_err(got_eta, eta_ref[lo:hi]) <= RTOL, (k0, rel_err(got_eta, eta_ref[lo:hi]))
    for c in (i1, i2):
      if k0 + lo <= c < k0 + hi:
        eta_ref_at[c] = abs(float(eta_ref[c - k0]))
  # refined elements were inside checked windows
  inside = [k for k in refined for k0, k1 in windows[1:3] if k0 + margin <= k < k1 - margin]
  assert len(inside) >= 3, inside
  # the refine decision: the oracle's |eta| at the GPU's top two, ranked the same way when the
  # GPU's margin clears the tolerance (1e-10 of the top value, twice: both values may move)
  assert i1 in eta_ref_at and i2 in eta_ref_at
  v1, v2 = float(top.values[0]), float(top.values[1])
  if v1 - v2 > 2 * RTOL * v1:
    assert eta_ref_at[i1] > eta_ref_at[i2]
  run.refine()
  assert run.sync() == i1
  np.testing.assert_array_equal(run.op.v_x(), pkg.split_interval(v_x, i1))
