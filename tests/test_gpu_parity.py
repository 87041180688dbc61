"""HIP path vs the CPU oracle, through the C ABI (ctypes).  Needs an MI355X.

Inputs are identical on both sides: the oracle runs with the plan's per-element metric
(oracle.setup1d.startup1d(metric="element")), and the adjoint/indicator oracle is fed
the GPU's own forward snapshots (the jump residual of a smooth solution is a
cancellation-limited difference, so it is compared on the same states; the forward
states themselves are compared separately).

Tolerances (north_star: fp64 state and indicator within 1e-10 relative; integer
outputs bit-exact):
  * fp64 fields: max|gpu - oracle| <= RTOL * max|oracle|, RTOL = 1e-10;
  * limiter troubled-cell ids, argmax indices, ensemble row sums: exact.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import limiter as olim
from oracle import setup1d

pytestmark = pytest.mark.gpu

RTOL = 1e-10
A = 2 * np.pi


def rel_err(x, ref):
  x, ref = np.asarray(x), np.asarray(ref)
  return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-300))


def mesh_pair(pkg, N, K, v_x=None, xmin=0.0, xmax=1.0):
  if v_x is None:
    _, v_x, _, _ = setup1d.mesh_gen1d(xmin, xmax, K)
  S = setup1d.startup1d(N, v_x, metric="element")  # the plan's per-element rx = 2/h
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  return S, mesh


def dev(x, device):
  import torch
  return torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=device)


def host(t):
  return t.detach().cpu().numpy()


def make_op(pkg, mesh, **kw):
  return pkg.operators.DGAdvection1D(mesh, **kw)


def random_field(rng, Np, K):
  return rng.standard_normal((Np, K))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("inflow", ["a", "a2"])
def test_rhs_matches_AdvecRHS1D(pkg, gpu, N, inflow):
  rng = np.random.default_rng(N)
  S, mesh = mesh_pair(pkg, N, 37)
  u = random_field(rng, N + 1, 37)
  op = make_op(pkg, mesh, inflow=inflow)
  got = host(op.rhs(dev(setup1d.to_elem_major(u), gpu), 0.37))
  ref, _ = oadv.advec_rhs1d(u, 0.37, A, S, inflow)
  assert rel_err(setup1d.from_elem_major(got, N + 1), ref) <= RTOL


def test_rhs_nonuniform_mesh(pkg, gpu):
  rng = np.random.default_rng(7)
  v_x = np.concatenate(([0.0], np.cumsum(rng.uniform(0.5, 1.5, 60))))
  v_x = v_x / v_x[-1]
  S, mesh = mesh_pair(pkg, 4, 60, v_x=v_x)
  op = make_op(pkg, mesh)
  assert not op.uniform
  u = random_field(rng, 5, 60)
  got = host(op.rhs(dev(setup1d.to_elem_major(u), gpu), 0.1))
  ref, _ = oadv.advec_rhs1d(u, 0.1, A, S)
  assert rel_err(setup1d.from_elem_major(got, 5), ref) <= RTOL


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("N,K", [(1, 300), (2, 513), (4, 1000), (4, 246), (6, 250), (8, 777)])
def test_forward_sweep_matches_lserk4_loop(pkg, gpu, N, K):
  import torch
  S, mesh = mesh_pair(pkg, N, K)
  u0 = np.sin(2 * np.pi * S["x"])
  dt = oadv.bench_dt(S)
  nsteps = 7
  ref, _ = oadv.forward_sweep(u0, 0.05, dt, nsteps, A, S)
  op = make_op(pkg, mesh)
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.05, dt, nsteps, snaps)
  torch.cuda.synchronize()
  for n in range(nsteps + 1):
    assert rel_err(setup1d.from_elem_major(host(snaps[n]), N + 1), ref[n]) <= RTOL, n
  assert rel_err(setup1d.from_elem_major(host(u), N + 1), ref[-1]) <= RTOL


@pytest.mark.parametrize("nsteps", [1, 2, 5, 6])
def test_forward_without_snapshots_pingpong(pkg, gpu, nsteps):
  S, mesh = mesh_pair(pkg, 4, 500)
  u0 = np.cos(3 * np.pi * S["x"])
  dt = oadv.bench_dt(S)
  ref, _ = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  op = make_op(pkg, mesh)
  u = dev(setup1d.to_elem_major(u0), gpu)
  op.forward(u, 0.0, dt, nsteps)
  assert rel_err(setup1d.from_elem_major(host(u), 5), ref[-1]) <= RTOL


def test_forward_nonuniform_and_euler(pkg, gpu):
  rng = np.random.default_rng(3)
  v_x = np.concatenate(([0.0], np.cumsum(rng.uniform(0.3, 1.7, 400))))
  v_x = v_x / v_x[-1]
  S, mesh = mesh_pair(pkg, 3, 400, v_x=v_x)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
  dt = 0.2 * oadv.bench_dt(S)
  for scheme in ("lserk4", "euler"):
    ref, _ = oadv.forward_sweep(u0, 0.0, dt, 4, A, S, scheme=scheme)
    op = make_op(pkg, mesh, time_scheme=scheme)
    u = dev(setup1d.to_elem_major(u0), gpu)
    op.forward(u, 0.0, dt, 4)
    assert rel_err(setup1d.from_elem_major(host(u), 4), ref[-1]) <= RTOL, scheme


def test_golden_run_one_code_mlx(pkg, gpu):
  """The executed reference run (One_code.mlx:106-140: N=2, K=20, T=2, uin=-sin(a^2 t)),
  1341 steps on the GPU vs the oracle that reproduces the MATLAB outputs."""
  S, mesh = mesh_pair(pkg, 2, 20)
  u0 = np.sin(2 * np.pi * S["x"])
  ref = oadv.advec1d(u0.copy(), 2.0, A, S, inflow="a2")
  op = make_op(pkg, mesh, inflow="a2")
  u = dev(setup1d.to_elem_major(u0), gpu)
  op.forward(u, 0.0, ref["dt"], ref["nsteps"])
  assert rel_err(setup1d.from_elem_major(host(u), 3), ref["u"]) <= RTOL


def test_ensemble_batch_matches_single_trajectories(pkg, gpu):
  """batch trajectories in one plan == each trajectory alone (per-trajectory inflow/outflow)."""
  import torch
  S, mesh = mesh_pair(pkg, 4, 130)
  rng = np.random.default_rng(11)
  B = 3
  u0s = [np.sin(2 * np.pi * rng.integers(1, 5) * S["x"] + rng.uniform(0, 6)) for _ in range(B)]
  dt = oadv.bench_dt(S)
  opb = make_op(pkg, mesh, batch=B)
  ub = dev(np.concatenate([setup1d.to_elem_major(u) for u in u0s]), gpu)
  opb.forward(ub, 0.0, dt, 6)
  op1 = make_op(pkg, mesh)
  for b in range(B):
    u1 = dev(setup1d.to_elem_major(u0s[b]), gpu)
    op1.forward(u1, 0.0, dt, 6)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(ub)[b * 650:(b + 1) * 650], host(u1))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("scheme", ["lserk4", "euler"])
@pytest.mark.parametrize("N,K", [(4, 50), (2, 300), (7, 260)])
def test_adjoint_sweep_and_indicator(pkg, gpu, scheme, N, K):
  rng = np.random.default_rng(N * 100 + K)
  S, mesh = mesh_pair(pkg, N, K)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.3 * np.cos(6 * np.pi * S["x"])
  dt = oadv.bench_dt(S) * (1.0 if scheme == "lserk4" else 0.1)
  nsteps, src = 6, 0.7
  snaps, times = oadv.forward_sweep(u0, 0.02, dt, nsteps, A, S, scheme=scheme)
  g = rng.standard_normal(u0.shape)
  op = make_op(pkg, mesh, time_scheme=scheme)
  u = dev(setup1d.to_elem_major(u0), gpu)
  snap_d = op.new_field(nsteps + 1)
  op.forward(u, 0.02, dt, nsteps, snap_d)
  gsnaps = [setup1d.from_elem_major(host(snap_d[n]), N + 1) for n in range(nsteps + 1)]
  for n in range(nsteps + 1):
    assert rel_err(gsnaps[n], snaps[n]) <= RTOL
  w_ref, eta_ref, _ = oadj.adjoint_sweep(g, gsnaps, times, dt, A, S, src_coef=src, scheme=scheme)
  w = dev(setup1d.to_elem_major(g), gpu)
  import torch
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snap_d, 0.02, dt, nsteps, src_coef=src, eta=eta)
  assert rel_err(setup1d.from_elem_major(host(w), N + 1), w_ref) <= RTOL
  assert rel_err(host(eta), eta_ref) <= RTOL


def test_adjoint_is_exact_transpose(pkg, gpu):
  """<S u - S 0, w> == <u, S^T w> for one GPU step (dot-product test)."""
  import torch
  rng = np.random.default_rng(5)
  S, mesh = mesh_pair(pkg, 4, 700)
  op = make_op(pkg, mesh)
  dt = oadv.bench_dt(S)
  u = dev(rng.standard_normal(5 * 700), gpu)
  z = torch.zeros_like(u)
  su, s0 = u.clone(), z.clone()
  snaps = op.new_field(2)
  op.forward(su, 0.3, dt, 1, snaps)
  op.forward(s0, 0.3, dt, 1)
  w = dev(rng.standard_normal(5 * 700), gpu)
  wt = w.clone()
  op.adjoint(wt, snaps, 0.3, dt, 1)
  lhs = float(torch.dot(su - s0, w))
  rhs = float(torch.dot(u, wt))
  assert abs(lhs - rhs) <= 1e-12 * abs(lhs)


def test_adjoint_gradient_matches_finite_difference(pkg, gpu):
  """dJ/du0 from the sweep vs a central difference of J (J is quadratic, so exact up to
  rounding): the complex-step / FD method of matlab/test_jacobian.m:38-55."""
  import torch
  rng = np.random.default_rng(9)
  N, K, nsteps, src = 3, 90, 5, 0.4
  S, mesh = mesh_pair(pkg, N, K)
  op = make_op(pkg, mesh)
  dt = oadv.bench_dt(S)
  g = dev(rng.standard_normal((N + 1) * K), gpu)
  u0 = dev(rng.standard_normal((N + 1) * K), gpu)
  d = dev(rng.standard_normal((N + 1) * K), gpu)

  def J(u_init):
    snaps = op.new_field(nsteps + 1)
    op.forward(u_init.clone(), 0.0, dt, nsteps, snaps)
    val = float(torch.dot(g, snaps[nsteps]))
    for n in range(nsteps):
      val += 0.5 * src * float(torch.dot(snaps[n], snaps[n]))
    return val, snaps

  _, snaps = J(u0)
  w = g.clone()
  op.adjoint(w, snaps, 0.0, dt, nsteps, src_coef=src)
  h = 1e-3
  fd = (J(u0 + h * d)[0] - J(u0 - h * d)[0]) / (2 * h)
  ad = float(torch.dot(w, d))
  assert abs(fd - ad) <= 1e-9 * abs(ad)


# ---------------------------------------------------------------------------
def _limiter_input(rng, S):
  x = S["x"]
  u = np.sin(2 * np.pi * x) + (x > 0.5) * 1.0 + 0.02 * rng.standard_normal(x.shape)
  u[:, ::7] = u[:, ::7].mean(axis=0)  # some exactly-constant cells
  return u


@pytest.mark.parametrize("N", [1, 2, 4, 8])
def test_slope_limiter_matches_SlopeLimitN(pkg, gpu, N):
  import torch
  rng = np.random.default_rng(N)
  K = 517
  S, mesh = mesh_pair(pkg, N, K)
  u = _limiter_input(rng, S)
  ref, ids_ref = olim.slope_limit_n(u, S, return_ids=True)
  op = make_op(pkg, mesh)
  ids = torch.zeros(K, dtype=torch.int32, device=gpu)
  got = host(op.slope_limit(dev(setup1d.to_elem_major(u), gpu), ids=ids))
  np.testing.assert_array_equal(np.nonzero(host(ids))[0], ids_ref)
  assert 0 < ids_ref.size < K
  np.testing.assert_allclose(setup1d.from_elem_major(got, N + 1), ref, rtol=0, atol=1e-13)


@pytest.mark.parametrize("N", [1, 2, 4, 8])
def test_slope_limiter_matches_SlopeLimit1(pkg, gpu, N):
  """dg_slope_limit_1 vs utils/SlopeLimit1.m (every cell limited), same summation order."""
  rng = np.random.default_rng(100 + N)
  K = 517
  S, mesh = mesh_pair(pkg, N, K)
  u = _limiter_input(rng, S)
  ref = olim.slope_limit_1(u, S)
  op = make_op(pkg, mesh)
  got = host(op.slope_limit_1(dev(setup1d.to_elem_major(u), gpu)))
  np.testing.assert_allclose(setup1d.from_elem_major(got, N + 1), ref, rtol=0, atol=1e-13)


@pytest.mark.parametrize("N,M", [(1, 3e6), (2, 1e6), (4, 3e6), (8, 1e7)])
def test_slope_limiter_tvb_matches_minmodB(pkg, gpu, N, M):
  """dg_plan_set_tvb(M): SlopeLimitLin's minmod becomes utils/minmodB.m (the element's own
  slope kept where |ux| <= M h^2) in dg_slope_limit_n and dg_slope_limit_1, against the oracle
  with the same M; M chosen so that both branches occur (h = 1/517: M h^2 ~ 4..40 against
  slopes ~ 2 pi .. 50); M = 0 restores the plain limiter bit for bit."""
  import torch
  rng = np.random.default_rng(200 + N)
  K = 517
  S, mesh = mesh_pair(pkg, N, K)
  u = _limiter_input(rng, S)
  op = make_op(pkg, mesh)
  ud = dev(setup1d.to_elem_major(u), gpu)
  plain_n, plain_1 = host(op.slope_limit(ud)), host(op.slope_limit_1(ud))
  op.set_tvb(M)
  ref_n, ids_ref = olim.slope_limit_n(u, S, return_ids=True, M=M)
  ref_1 = olim.slope_limit_1(u, S, M=M)
  ids = torch.zeros(K, dtype=torch.int32, device=gpu)
  got_n = host(op.slope_limit(ud, ids=ids))
  got_1 = host(op.slope_limit_1(ud))
  np.testing.assert_array_equal(np.nonzero(host(ids))[0], ids_ref)
  np.testing.assert_allclose(setup1d.from_elem_major(got_n, N + 1), ref_n, rtol=0, atol=1e-13)
  np.testing.assert_allclose(setup1d.from_elem_major(got_1, N + 1), ref_1, rtol=0, atol=1e-13)
  kept = np.any(np.abs(setup1d.from_elem_major(got_1 - plain_1, N + 1)) > 1e-12, axis=0)
  assert 0 < kept.sum() < K, kept.sum()  # TVB kept some slopes, minmod limited others
  op.set_tvb(0.0)
  np.testing.assert_array_equal(host(op.slope_limit(ud)), plain_n)
  np.testing.assert_array_equal(host(op.slope_limit_1(ud)), plain_1)


# ---------------------------------------------------------------------------
def test_argmax_numpy_semantics(pkg, gpu):
  S, mesh = mesh_pair(pkg, 2, 4000)
  op = make_op(pkg, mesh)
  rng = np.random.default_rng(1)
  cases = []
  x = rng.standard_normal(12000)
  cases.append(x)
  y = x.copy()
  y[[17, 9000, 11999]] = 50.0  # ties: first index wins
  cases.append(y)
  z = x.copy()
  z[[3000, 4000]] = np.nan  # NaN is the maximum, first NaN wins
  cases.append(z)
  cases.append(-np.abs(x))
  cases.append(np.zeros(5))
  cases.append(np.array([-np.inf, -np.inf, -np.inf]))
  for c in cases:
    for use_abs in (False, True):
      assert op.argmax(dev(c, gpu), use_abs=use_abs) == oadj.argmax(c, use_abs), (c[:4], use_abs)


def test_sum_rows_fixed_order(pkg, gpu):
  rng = np.random.default_rng(2)
  x = rng.standard_normal((7, 3001)) * 10.0 ** rng.integers(-8, 8, (7, 3001))
  got = host(pkg.operators.sum_rows(dev(x.ravel(), gpu), 7))
  np.testing.assert_array_equal(got, oadj.sum_rows(x))


def test_init_sine(pkg, gpu):
  S, mesh = mesh_pair(pkg, 4, 333)
  op = make_op(pkg, mesh, batch=2)
  got = host(op.init_sine([0.7, 1.3], [3.0, 5.0], [0.1, 2.0]))
  for b, (A_, m, ph) in enumerate([(0.7, 3.0, 0.1), (1.3, 5.0, 2.0)]):
    ref = A_ * np.sin(2 * np.pi * m * S["x"] + ph)
    np.testing.assert_allclose(setup1d.from_elem_major(got[b * 5 * 333:(b + 1) * 5 * 333], 5),
                               ref, atol=1e-13)


# ---------------------------------------------------------------------------
@pytest.mark.slow
def test_full_size_config2_forward_adjoint(pkg, gpu):
  """BASELINE config 2 size (N=4, K=1,048,576): 2 fused steps vs the oracle, plus the
  size-independent transpose identity of the adjoint at full size."""
  import torch
  N, K, nsteps = 4, 1 << 20, 2
  S, mesh = mesh_pair(pkg, N, K)
  u0 = np.sin(2 * np.pi * S["x"])
  dt = oadv.bench_dt(S)
  ref, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  op = make_op(pkg, mesh)
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.0, dt, nsteps, snaps)
  assert rel_err(setup1d.from_elem_major(host(u), N + 1), ref[-1]) <= RTOL
  rng = np.random.default_rng(0)
  g = rng.standard_normal(u0.shape)
  gsnaps = [setup1d.from_elem_major(host(snaps[n]), N + 1) for n in range(nsteps + 1)]
  w_ref, eta_ref, _ = oadj.adjoint_sweep(g, gsnaps, times, dt, A, S)
  w = dev(setup1d.to_elem_major(g), gpu)
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, 0.0, dt, nsteps, eta=eta)
  assert rel_err(setup1d.from_elem_major(host(w), N + 1), w_ref) <= RTOL
  assert rel_err(host(eta), eta_ref) <= RTOL
  assert op.argmax(eta) == int(np.argmax(np.abs(host(eta))))


@pytest.mark.parametrize("N,K", [(4, 3000), (2, 20000), (8, 1111), (1, 777)])
def test_kernel_variants_bit_identical(pkg, gpu, N, K):
  """Every step-kernel shape (elements per lane x steps per launch) gives the same answer."""
  import torch
  S, mesh = mesh_pair(pkg, N, K)
  u0 = dev(setup1d.to_elem_major(np.sin(2 * np.pi * S["x"]) + 0.1 * np.cos(40 * S["x"])), gpu)
  dt = oadv.bench_dt(S)
  outs = []
  nsteps = 7  # exercises the greedy 4 + 2 + 1 chunking
  shapes = ((1, 1, 1, 0), (2, 1, 0, 0), (1, 2, 1, 0), (1, 4, 1, 0), (2, 4, 0, 0), (1, 4, 0, 0),
            (2, 2, 1, 0), (1, 4, 1, 4), (1, 4, 1, 2), (1, 2, 1, 4), (2, 8, 1, 0), (2, 8, 1, 4),
            (2, 8, 1, 8), (2, 8, 1, 2))
  for width, ms, xcd, lanes in shapes:
    if lanes and N == 8:
      lanes = 0  # wave tiles cover Np <= 8
    op = make_op(pkg, mesh).tune(tile_width=width, steps_per_launch=ms, xcd_order=xcd,
                                 lane_elements=lanes)
    snaps = op.new_field(nsteps + 1)
    op.forward(u0.clone(), 0.0, dt, nsteps, snaps)
    w = snaps[nsteps].clone()
    eta = torch.zeros(K, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.0, dt, nsteps, src_coef=0.3, eta=eta)
    u_plain = u0.clone()
    op.forward(u_plain, 0.0, dt, nsteps)
    outs.append((host(snaps), host(w), host(eta), host(u_plain)))
  # Elements per lane does not change the arithmetic: bit-identical.  Fusing steps keeps
  # the state in even/odd coordinates between steps (one rounding round-trip fewer per
  # step), so different steps-per-launch agree to rounding.
  for a_, b_ in zip(outs[0], outs[1]):
    np.testing.assert_array_equal(a_, b_)
  # same steps per launch, other lane packing / tile order / wave tiles
  # (8-step launches on wave tiles: 4 and 8 elements per lane; with 2 elements per lane the
  # plan caps the launch at 4 steps, so shape 13 equals shape 3's 4-step sweep)
  for i, j in ((3, 4), (3, 5), (3, 7), (3, 8), (2, 9), (10, 11), (10, 12), (3, 13)):
    for a_, b_ in zip(outs[i], outs[j]):
      np.testing.assert_array_equal(a_, b_)
  # States agree to 1e-12; the indicator (a cancellation-limited jump residual) to RTOL.
  for o in outs[2:]:
    for a_, b_, tol in zip(outs[0], o, (1e-12, 1e-12, RTOL, 1e-12)):
      assert rel_err(b_, a_) <= tol


@pytest.mark.parametrize("nsteps", [3, 8, 13])
def test_adjoint_in_place_on_terminal_snapshot(pkg, gpu, nsteps):
  """w aliasing snapshot N (J = |u^N|^2/2) gives the same gradient and indicator as a
  separate w buffer, for single- and multi-launch sweeps."""
  import torch
  S, mesh = mesh_pair(pkg, 4, 900)
  op = make_op(pkg, mesh)
  dt = oadv.bench_dt(S)
  u0 = dev(setup1d.to_elem_major(np.sin(2 * np.pi * S["x"]) + 0.2 * np.cos(14 * S["x"])), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u0.clone(), 0.0, dt, nsteps, snaps)
  w_sep = snaps[nsteps].clone()
  eta_sep = torch.zeros(900, dtype=torch.float64, device=gpu)
  op.adjoint(w_sep, snaps, 0.0, dt, nsteps, eta=eta_sep)
  eta_al = torch.zeros(900, dtype=torch.float64, device=gpu)
  op.adjoint(snaps[nsteps], snaps, 0.0, dt, nsteps, eta=eta_al)
  np.testing.assert_array_equal(host(snaps[nsteps]), host(w_sep))
  np.testing.assert_array_equal(host(eta_al), host(eta_sep))


@pytest.mark.parametrize("record", ["jumps", "snapshots"])
def test_ensemble_sweep_graph_matches_eager(pkg, gpu, record):
  """The HIP-graph replay of the sweeps (bench --graph) reproduces the eager sweeps (the jump
  record's 20-step sweep is one dataflow launch)."""
  import torch
  ens = pkg.ensemble
  mesh = pkg.BaseGalerkin1D(n=4, k=2000)
  dt = mesh.cfl_dt()
  a = ens.EnsembleSweep(mesh, [0, 1, 2], 20, dt, record=record)
  b = ens.EnsembleSweep(mesh, [0, 1, 2], 20, dt, record=record).capture()
  assert b.dataflow == (record == "jumps")
  pa = a.run().clone()
  b.sweep_graph()
  pb = b.reduce().clone()
  torch.cuda.synchronize()
  np.testing.assert_array_equal(host(pa), host(pb))
  np.testing.assert_array_equal(host(a.w), host(b.w))


def test_dg_adapt_loop_refines_the_oracle_argmax(pkg, gpu):
  """The DG adapt loop (factory.DGFunFactory): GPU sweeps + indicator + argmax split,
  against the oracle indicator computed from the same snapshots; the refine index must
  agree whenever the oracle's top-2 gap exceeds the parity tolerance."""
  import torch
  fac = pkg.factory
  problem = fac.DGProblem(N=3, nsteps=12)
  afuns = fac.DGFunFactory(problem).getAdaptFunctions()
  v_x = np.linspace(0.0, 1.0, 41)
  state = fac.DGAdaptState(problem, v_x)
  u0_fn = lambda x: np.sin(2 * np.pi * x) + 0.5 * np.exp(-200 * (x - 0.3) ** 2)  # noqa: E731
  seen = []
  for _ in range(4):
    v_x_now = np.asarray(state.times_new)
    state = afuns.adapt(state, u0_fn)
    # oracle on the same mesh (GPU forward snapshots as inputs)
    S = setup1d.startup1d(3, v_x_now, metric="element")
    mesh = pkg.BaseGalerkin1D(n=3, v_x=v_x_now)
    op = make_op(pkg, mesh)
    dt = mesh.cfl_dt()
    snaps = op.new_field(problem.nsteps + 1)
    snaps[0].copy_(dev(mesh.to_device_layout(u0_fn(mesh.x)), gpu))
    op.forward(snaps[0], 0.0, dt, problem.nsteps, snaps)
    gs = [setup1d.from_elem_major(host(snaps[n]), 4) for n in range(problem.nsteps + 1)]
    times = [0.0]
    for _n in range(problem.nsteps):
      times.append(times[-1] + dt)
    _, eta_ref, _ = oadj.adjoint_sweep(gs[-1], gs, times, dt, A, S)
    assert rel_err(state.err_steps, np.abs(eta_ref)) <= RTOL
    top = np.sort(np.abs(eta_ref))[::-1]
    if top[0] - top[1] > 1e-8 * top[0]:
      assert state.ref_idx == int(np.argmax(np.abs(eta_ref)))
    assert len(state.times_new) == len(v_x_now) + 1
    seen.append(state.ref_idx)
  assert len(state.times_new) == 45  # four splits of a 40-element mesh


def test_ensemble_per_ic_rows_and_gather(pkg, gpu):
  """per_ic() rows are each IC's own indicator; their fixed-order sum is reduce(); the
  single-process per-IC gather returns them unchanged."""
  import torch
  K, ics = 200, [3, 4, 5]
  mesh = pkg.BaseGalerkin1D(n=4, k=K)
  S = setup1d.uniform_setup(4, K, metric="element")
  dt = oadv.bench_dt(S)
  sweep = pkg.ensemble.EnsembleSweep(mesh, ics, 8, dt)
  partial = sweep.run().clone()
  rows = sweep.per_ic()
  assert rows.shape == (3, K)
  torch.testing.assert_close(pkg.operators.sum_rows(rows.contiguous(), 3), partial, rtol=0,
                             atol=0)
  for b, j in enumerate(ics):
    one = pkg.ensemble.EnsembleSweep(mesh, [j], 8, dt)
    one.run()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(rows[b]), host(one.eta))
  assert torch.equal(pkg.ensemble.gather_per_ic(rows, 3), rows)


@pytest.mark.parametrize("N,K,tw,ms,nsteps,refined", [
    (4, 3000, 2, 8, 20, False),   # the p-estimate bench's forward shape: 8 + 8 + 4 launches
    (4, 1000, 1, 4, 7, False),    # 512-element tiles, 4 + 2 + 1
    (1, 2000, 2, 8, 9, False),
    (2, 777, 1, 2, 5, True),
    (6, 1500, 2, 4, 6, True),
    (8, 900, 2, 8, 8, False),
    (3, 100, 2, 8, 3, False),     # fewer elements than one tile's output
])
def test_snapshot_forward_on_pair_tiles(pkg, gpu, N, K, tw, ms, nsteps, refined):
  """DG_TUNE_SNAP_PAIRS = 1: the snapshot forward as the Horner-form step on pair tiles
  (k_step_rps), every snapshot and u^N against the oracle's LSERK4 loop at 1e-10."""
  import torch
  rng = np.random.default_rng(N + 7)
  v_x = None
  if refined:
    v_x = np.concatenate(([0.0], np.cumsum(rng.uniform(0.5, 1.5, K))))
    v_x = v_x / v_x[-1]
  S, mesh = mesh_pair(pkg, N, K, v_x=v_x)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
  dt = oadv.bench_dt(S)
  ref, _ = oadv.forward_sweep(u0, 0.05, dt, nsteps, A, S)
  op = make_op(pkg, mesh)
  op.tune(tile_width=tw, steps_per_launch=ms, snap_pairs=1)
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.05, dt, nsteps, snaps)
  torch.cuda.synchronize()
  for n in range(nsteps + 1):
    assert rel_err(setup1d.from_elem_major(host(snaps[n]), N + 1), ref[n]) <= RTOL, n
  assert rel_err(setup1d.from_elem_major(host(u), N + 1), ref[-1]) <= RTOL


def test_snapshot_forward_pairs_batch_edges(pkg, gpu):
  """Pair-tile snapshots of a batch (trajectory edges inside tiles, odd Np * ktot so the
  snapshot stride is not 16-byte aligned) equal the stage-loop kernels' to rounding."""
  import torch
  N, K, batch, nsteps = 4, 1001, 3, 10
  S, mesh = mesh_pair(pkg, N, K)
  op = make_op(pkg, mesh, batch=batch, inflow="a2")
  rng = np.random.default_rng(5)
  u0 = dev(rng.standard_normal(batch * K * (N + 1)), gpu)
  dt = oadv.bench_dt(S)
  out = []
  for pairs in (0, 1):
    op.tune(tile_width=2, steps_per_launch=8 if pairs else 4, snap_pairs=pairs)
    snaps = op.new_field(nsteps + 1)
    u = u0.clone()
    op.forward(u, 0.0, dt, nsteps, snaps)
    torch.cuda.synchronize()
    out.append(host(snaps))
  assert np.all(np.isfinite(out[1]))
  for n in range(nsteps + 1):
    assert rel_err(out[1][n], out[0][n]) <= 1e-12, n
