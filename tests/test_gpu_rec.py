"""The snapshot-free sweep pair (dg_lserk4_fwd_rec / dg_lserk4_adj_rec, include/dg_advec.h).

For linear advection the adjoint step S^T does not depend on the state and the indicator
needs of each u^n only its two interelement jumps per element (R = LIFT*(Fscale.*du),
utils/AdvecRHS1D.m:19); a face's jump is shared by its two elements, so the forward records
one number per element and step in place of the snapshots: the left-face jump du0 = u_0 - uL
(element e's right-face du1 is -du0 of element e+1, or 0 at a trajectory's last element).
Bars:
  * the record equals the jumps of the snapshot sweep's states, bit for bit (same doubles,
    same subtractions), and agrees with the oracle's AdvecRHS1D face jumps (face_jumps,
    which carry the (a nx)/2 factors) to rounding;
  * with one element per lane (the stage-loop record kernels of dg_advec.hip) final state,
    w^0 and eta equal the snapshot sweep pair's (src_coef = 0) bit for bit, for every tile
    shape, steps per launch, batch (trajectory edges inside tiles), inflow variant and a
    refined (non-uniform) mesh;
  * the pair-tile kernels (dg_rec.hip, the default) evaluate each LSERK4 step as its stability
    polynomial in Horner form (round 3): equal to the stage loop to rounding, so against the
    snapshot pair they are held to HORNER_RTOL of max|.| on ICs with resolved jumps (a smooth
    IC's jumps are below fp64 resolution at fine meshes and its indicator is rounding noise),
    and bit for bit across their own tile shapes.
"""
import numpy as np
import pytest

from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu


HORNER_RTOL = 1e-11  # Horner vs stage loop: ~2e-16 per step; the parity bar is 1e-10


def host(t):
  return t.detach().cpu().numpy()


def close(a, b, rtol=HORNER_RTOL, what=""):
  a, b = np.asarray(a), np.asarray(b)
  np.testing.assert_allclose(a, b, rtol=0, atol=rtol * max(np.abs(b).max(), 1e-300), err_msg=what)


def noisy_sine(op, seed, batch):
  """Sine ICs plus seeded per-node noise of 0.1: O(0.1) interelement jumps, a well-conditioned
  indicator."""
  import torch
  rng = np.random.default_rng(seed)
  u0 = op.new_field()
  op.init_sine(rng.uniform(0.5, 1.5, batch), rng.integers(1, 5, batch).astype(float),
               rng.uniform(0, 6, batch), out=u0)
  gen = torch.Generator(device=u0.device).manual_seed(seed)
  u0 += 0.1 * torch.randn(u0.shape, dtype=u0.dtype, device=u0.device, generator=gen)
  return u0


def raw_jumps(u_em, K, batch, Np, uin):
  """The left-face jump du0 = u_0 - (left neighbour's u_N, or the inflow value) per element
  of an element-major field, (batch*K,)."""
  u = u_em.reshape(batch, K, Np)
  left = np.concatenate([np.full((batch, 1), uin), u[:, :-1, Np - 1]], axis=1)
  return (u[:, :, 0] - left).reshape(batch * K)


def sweep_pair(pkg, op, u0, dt, nsteps, t0=0.0):
  """The snapshot pair and the record pair from the same u0; returns both results."""
  import torch
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(u0)
  op.forward(snaps[0], t0, dt, nsteps, snaps)
  w_s = snaps[nsteps].clone()
  eta_s = torch.zeros(op.ktot, dtype=torch.float64, device=op.device)
  op.adjoint(w_s, snaps, t0, dt, nsteps, eta=eta_s)
  rec = op.new_jumps(nsteps)
  uN = op.new_field()
  op.forward_rec(u0, t0, dt, nsteps, rec, out=uN)
  w_r = uN.clone()
  eta_r = torch.full((op.ktot,), float("nan"), dtype=torch.float64, device=op.device)
  op.adjoint_rec(w_r, rec, t0, dt, nsteps, eta=eta_r, eta_assign=True)
  torch.cuda.synchronize()
  return snaps, w_s, eta_s, rec, uN, w_r, eta_r


@pytest.mark.parametrize("N,K,batch,tw,rtw,spl,nsteps,inflow", [
    (4, 1000, 1, 1, 1, 4, 9, "a"),
    (4, 700, 3, 1, 2, 4, 8, "a2"),
    (4, 600, 2, 2, 2, 8, 17, "a"),
    (4, 2600, 2, 2, 2, 8, 20, "a"),
    (5, 1800, 1, 1, 2, 4, 9, "a"),
    (3, 513, 1, 2, 2, 4, 6, "a"),
    (2, 900, 2, 1, 1, 2, 5, "a2"),
    (1, 300, 1, 1, 2, 1, 3, "a"),
    (6, 260, 1, 1, 1, 4, 4, "a"),
    (8, 400, 1, 2, 2, 2, 7, "a"),
    (4, 77, 1, 1, 1, 4, 2, "a"),     # one launch, fewer steps than steps_per_launch
])
@pytest.mark.parametrize("lane_elements", [1, 2])
def test_record_pair_equals_snapshot_pair(pkg, gpu, N, K, batch, tw, rtw, spl, nsteps, inflow,
                                          lane_elements):
  """At equal steps per launch (which sets where the state leaves even/odd coordinates);
  tile widths never change the arithmetic.  One element per lane: bit for bit; pair tiles
  (Horner form): to HORNER_RTOL."""
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch, inflow=inflow)
  op.tune(tile_width=tw, steps_per_launch=spl, lane_elements=0, rec_tile_width=rtw,
          rec_steps_per_launch=spl, rec_lane_elements=lane_elements)
  assert op.rec_steps_per_launch == op.steps_per_launch
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, N * 100 + K, batch)
  u0_copy = u0.clone()
  snaps, w_s, eta_s, rec, uN, w_r, eta_r = sweep_pair(pkg, op, u0, dt, nsteps, t0=0.01)
  np.testing.assert_array_equal(host(u0), host(u0_copy))  # u0 untouched
  exact = lane_elements == 1
  same = np.testing.assert_array_equal if exact else (lambda a, b, err_msg="": close(a, b, what=err_msg))
  same(host(uN), host(snaps[nsteps]), err_msg="u^N")
  # the record: u^n's jumps at t_n, n = 1..nsteps (absolute error against max|u|: jumps are
  # differences of O(1) values)
  t = [0.01]
  for _ in range(nsteps):
    t.append(t[-1] + dt)
  R = host(rec)
  umax = np.abs(host(u0)).max()
  for n in range(1, nsteps + 1):
    uin = oadv.inflow_value(op.a, t[n], inflow)
    ref = raw_jumps(host(snaps[n]), K, batch, N + 1, uin)
    if exact:
      np.testing.assert_array_equal(R[n - 1, :K * batch], ref, err_msg=f"record {n - 1}")
    else:
      np.testing.assert_allclose(R[n - 1, :K * batch], ref, rtol=0, atol=HORNER_RTOL * umax,
                                 err_msg=f"record {n - 1}")
  same(host(w_r), host(w_s), err_msg="w^0")
  same(host(eta_r), host(eta_s), err_msg="eta")
  assert np.abs(host(eta_s)).max() > 0


def test_record_is_the_oracle_face_jumps(pkg, gpu):
  """The recorded raw jumps are AdvecRHS1D's du (utils/AdvecRHS1D.m:9-16, oracle face_jumps)
  up to its (a nx)/2 factors: du_left = -(a/2) du0, du_right = (a/2) du1."""
  N, K, nsteps = 4, 200, 4
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  S = setup1d.startup1d(N, np.linspace(0.0, 1.0, K + 1))
  dt = mesh.cfl_dt()
  u0 = op.new_field()
  op.init_sine([1.0], [1.0], [0.0], out=u0)
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(u0)
  op.forward(snaps[0], 0.0, dt, nsteps, snaps)
  rec = op.new_jumps(nsteps)
  op.forward_rec(u0, 0.0, dt, nsteps, rec, out=op.new_field())
  R = host(rec)
  t = 0.0
  for n in range(1, nsteps + 1):
    t += dt
    u = setup1d.from_elem_major(host(snaps[n]), N + 1)
    du = oadv.face_jumps(u, oadv.inflow_value(op.a, t, "a"), op.a, S)
    du0 = R[n - 1, :K]
    du1 = np.append(-R[n - 1, 1:K], 0.0)  # the right neighbour's left jump; outflow: 0
    np.testing.assert_allclose(du[0], -0.5 * op.a * du0, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(du[1], 0.5 * op.a * du1, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("lane_elements", [1, 2])
def test_record_pair_on_a_refined_mesh(pkg, gpu, lane_elements):
  """Non-uniform metric (the refine loop's meshes): bit-identical to the snapshots with one
  element per lane, to HORNER_RTOL on pair tiles (their non-uniform Horner levels)."""
  N, K, nsteps = 4, 500, 8
  v_x = np.linspace(0.0, 1.0, K + 1)
  for k in (3, 170, 171, 499):
    v_x = np.insert(v_x, k + 1, 0.5 * (v_x[k] + v_x[k + 1]))
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  op = pkg.operators.DGAdvection1D(mesh, batch=2)
  op.tune(rec_tile_width=1, rec_steps_per_launch=op.steps_per_launch,
          rec_lane_elements=lane_elements)
  assert not op.uniform
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, 5, 2)
  snaps, w_s, eta_s, rec, uN, w_r, eta_r = sweep_pair(pkg, op, u0, dt, nsteps)
  same = (np.testing.assert_array_equal if lane_elements == 1
          else (lambda a, b, err_msg="": close(a, b, what=err_msg)))
  same(host(uN), host(snaps[nsteps]), err_msg="u^N")
  same(host(w_r), host(w_s), err_msg="w^0")
  same(host(eta_r), host(eta_s), err_msg="eta")


def test_record_in_place_and_flags(pkg, gpu):
  """forward_rec in place on u0 (one launch and several), adjoint_rec's |eta| flag, the
  empty sweep."""
  import torch
  N, K = 4, 300
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  dt = mesh.cfl_dt()
  for nsteps in (1, 3, 10):
    u0 = op.new_field()
    op.init_sine([1.0], [1.0], [0.0], out=u0)
    ref = op.new_field()
    rec_a, rec_b = op.new_jumps(nsteps), op.new_jumps(nsteps)
    op.forward_rec(u0, 0.0, dt, nsteps, rec_a, out=ref)
    op.forward_rec(u0, 0.0, dt, nsteps, rec_b)  # in place
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(u0), host(ref))
    np.testing.assert_array_equal(host(rec_a), host(rec_b))
    w1, w2 = ref.clone(), ref.clone()
    e1 = torch.zeros(K, dtype=torch.float64, device=gpu)
    e2 = torch.zeros(K, dtype=torch.float64, device=gpu)
    op.adjoint_rec(w1, rec_a, 0.0, dt, nsteps, eta=e1)
    op.adjoint_rec(w2, rec_a, 0.0, dt, nsteps, eta=e2, eta_assign=True, eta_abs=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(w1), host(w2))
    np.testing.assert_array_equal(np.abs(host(e1)), host(e2))
  u0 = op.new_field()
  op.init_sine([1.0], [1.0], [0.0], out=u0)
  out = op.new_field()
  op.forward_rec(u0, 0.0, dt, 0, op.new_jumps(0), out=out)
  eta = torch.full((K,), 3.0, dtype=torch.float64, device=gpu)
  op.adjoint_rec(out, op.new_jumps(0), 0.0, dt, 0, eta=eta, eta_assign=True)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(host(out), host(u0))
  assert not host(eta).any()


def test_record_rejects_what_it_cannot_do(pkg, gpu):
  import torch
  mesh = pkg.BaseGalerkin1D(n=4, k=100)
  op = pkg.operators.DGAdvection1D(mesh, flux="burgers", limiter=True)
  u = op.new_field()
  with pytest.raises(pkg._lib.DGLibraryError):
    op.forward_rec(u, 0.0, 1e-4, 2, op.new_jumps(2))
  lin = pkg.operators.DGAdvection1D(mesh)
  u = lin.new_field()
  lin.init_sine([1.0], [1.0], [0.0], out=u)
  buf = torch.empty(2 * 100 + 1, dtype=torch.float64, device=gpu)
  with pytest.raises(pkg._lib.DGLibraryError):  # 8-byte aligned only
    lin.forward_rec(u, 0.0, 1e-4, 2, buf[1:])
  with pytest.raises(ValueError):
    lin.forward_rec(u, 0.0, 1e-4, 3, lin.new_jumps(2))


def rec_sweep(op, u0, dt, nsteps, t0=0.0):
  """The record pair from u0 with the plan's current record shape."""
  import torch
  rec = op.new_jumps(nsteps)
  uN = op.new_field()
  op.forward_rec(u0, t0, dt, nsteps, rec, out=uN)
  w = uN.clone()
  eta = torch.full((op.ktot,), float("nan"), dtype=torch.float64, device=op.device)
  op.adjoint_rec(w, rec, t0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True)
  torch.cuda.synchronize()
  return host(rec)[:, :op.ktot], host(uN), host(w), host(eta)  # (the pad entry is unwritten)


@pytest.mark.parametrize("N,K,batch,rtw,spl,nsteps,inflow,refined", [
    (4, 3000, 1, 2, 8, 20, "a", False),
    (4, 2100, 3, 1, 8, 17, "a2", False),   # trajectory edges inside 512-element tiles
    (4, 900, 2, 2, 4, 9, "a", True),
    (4, 5000, 1, 1, 4, 6, "a", False),
    (1, 1500, 2, 2, 8, 11, "a", False),
    (2, 1100, 1, 1, 2, 5, "a2", True),
    (3, 640, 2, 2, 8, 8, "a", False),
    (5, 1030, 1, 2, 1, 3, "a", False),
    (6, 700, 1, 1, 8, 16, "a", True),
    (7, 800, 2, 2, 4, 4, "a", False),
    (4, 50, 1, 2, 8, 3, "a", False),       # one edge tile holds the whole mesh
])
def test_pair_tiles_equal_one_element_per_lane(pkg, gpu, N, K, batch, rtw, spl, nsteps, inflow,
                                               refined):
  """The record sweeps on pair tiles (two consecutive elements per lane, Horner-form steps,
  dg_rec.hip) against the one-element-per-lane stage-loop record kernels at the same steps
  per launch: record, final state, w^0 and |eta| to HORNER_RTOL (resolved jumps)."""
  v_x = np.linspace(0.0, 1.0, K + 1)
  if refined:
    for k in (2, K // 3, K // 3 + 1, K - 1):
      v_x = np.insert(v_x, k + 1, 0.5 * (v_x[k] + v_x[k + 1]))
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch, inflow=inflow)
  assert op.uniform != refined
  dt = mesh.cfl_dt()
  u0 = noisy_sine(op, N * 1000 + K, batch)
  op.tune(rec_tile_width=2, rec_steps_per_launch=spl, rec_lane_elements=1)
  assert (op.rec_steps_per_launch, op.rec_lane_elements) == (spl, 1)
  ref = rec_sweep(op, u0, dt, nsteps, t0=0.02)
  op.tune(rec_tile_width=rtw, rec_steps_per_launch=spl, rec_lane_elements=2)
  assert (op.rec_tile_width, op.rec_steps_per_launch, op.rec_lane_elements) == (rtw, spl, 2)
  got = rec_sweep(op, u0, dt, nsteps, t0=0.02)
  umax = float(np.abs(host(u0)).max())
  np.testing.assert_allclose(got[0], ref[0], rtol=0, atol=HORNER_RTOL * umax, err_msg="record")
  for name, a, b in zip(("u^N", "w^0", "|eta|"), got[1:], ref[1:]):
    close(a, b, what=name)
  assert np.abs(ref[3]).max() > 0


@pytest.mark.parametrize("N,K,batch,rtw,spl,nsteps", [
    (4, 4000, 1, 1, 10, 20),   # 10 + 10
    (4, 3000, 2, 2, 20, 20),   # one launch of 20 steps on 1024-element tiles
    (4, 2500, 1, 2, 16, 23),   # 16 + 4 + 2 + 1
    (1, 2000, 2, 1, 5, 17),    # 5 + 5 + 5 + 2
    (7, 1500, 1, 2, 10, 13),   # 10 + 2 + 1
    (4, 90, 1, 2, 20, 20),     # the whole mesh inside one edge tile
])
def test_pair_tiles_long_launches(pkg, gpu, N, K, batch, rtw, spl, nsteps):
  """Pair tiles with 5, 10, 16 or 20 steps per launch (no one-element-per-lane counterpart):
  against the snapshot sweep pair.  The states leave even/odd coordinates at other steps, so
  u^N and w^0 agree to rounding (1e-12 relative), the record to 1e-12 of max|u|, and eta to
  its conditioning (the jumps of a smooth solution are ~1e-7 of u: 1e-7 relative)."""
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh, batch=batch)
  dt = mesh.cfl_dt()
  u0 = op.new_field()
  rng = np.random.default_rng(N * 7 + K)
  op.init_sine(rng.uniform(0.5, 1.5, batch), rng.integers(1, 5, batch).astype(float),
               rng.uniform(0, 6, batch), out=u0)
  snaps, w_s, eta_s, _, _, _, _ = sweep_pair(pkg, op, u0, dt, nsteps)
  op.tune(rec_tile_width=rtw, rec_steps_per_launch=spl, rec_lane_elements=2)
  assert (op.rec_tile_width, op.rec_steps_per_launch, op.rec_lane_elements) == (rtw, spl, 2)
  rec, uN, w, eta = rec_sweep(op, u0, dt, nsteps)
  scale = np.abs(host(u0)).max()
  np.testing.assert_allclose(uN, host(snaps[nsteps]), rtol=0, atol=1e-12 * scale)
  np.testing.assert_allclose(w, host(w_s), rtol=0, atol=1e-12 * np.abs(host(w_s)).max())
  for n in range(1, nsteps + 1):
    uin = oadv.inflow_value(op.a, n * dt, "a")  # t_n by repeated addition: equal to rounding
    ref = raw_jumps(host(snaps[n]), K, batch, N + 1, uin)
    np.testing.assert_allclose(rec[n - 1, :K * batch], ref, rtol=0, atol=1e-12 * scale,
                               err_msg=f"record {n - 1}")
  e_ref = np.abs(host(eta_s))
  np.testing.assert_allclose(eta, e_ref, rtol=0, atol=1e-7 * e_ref.max())


def test_long_launch_shapes_are_checked(pkg, gpu):
  """Width-1 pair tiles cap 16 / 20 steps at 8 / 10; the one-element-per-lane kernels take the
  largest power of two <= the setting (<= 8); other values are refused."""
  mesh = pkg.BaseGalerkin1D(n=4, k=500)
  op = pkg.operators.DGAdvection1D(mesh)
  op.tune(rec_tile_width=1, rec_lane_elements=2, rec_steps_per_launch=20)
  assert op.rec_steps_per_launch == 10
  op.tune(rec_steps_per_launch=16)
  assert op.rec_steps_per_launch == 8
  op.tune(rec_tile_width=2, rec_lane_elements=1, rec_steps_per_launch=10)
  assert op.rec_steps_per_launch == 8
  op.tune(rec_steps_per_launch=5)
  assert op.rec_steps_per_launch == 4
  for bad in (3, 6, 12, 32):
    with pytest.raises(pkg._lib.DGLibraryError):
      op.tune(rec_steps_per_launch=bad)


def test_forward_own_steps_per_launch(pkg, gpu):
  """The forward record sweep's own steps per launch (DG_TUNE_REC_FWD_STEPS_PER_LAUNCH; a
  default plan of up to 3*2^20 elements runs one 20-step forward launch and 10 + 10 adjoint
  launches, a larger one 10 + 10 both ways): setting the
  common value applies to both directions and clears the forward's; the default sweep agrees
  with both directions at 10 steps to rounding (the state leaves even/odd coordinates at other
  steps): u^N, w^0 and the record to 1e-12, eta to its conditioning."""
  import torch
  N, K, nsteps = 4, 3000, 20
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  assert (op.rec_steps_per_launch, op.rec_fwd_steps_per_launch) == (10, 20)
  dt = mesh.cfl_dt()
  u0 = op.new_field()
  op.init_sine([1.0], [1.0], [0.0], out=u0)
  gen = torch.Generator(device=u0.device).manual_seed(3)
  u0 += 0.1 * torch.randn(u0.shape, dtype=u0.dtype, device=u0.device, generator=gen)  # resolved jumps
  got = rec_sweep(op, u0, dt, nsteps)
  op.tune(rec_steps_per_launch=10)
  assert (op.rec_steps_per_launch, op.rec_fwd_steps_per_launch) == (10, 10)
  ref = rec_sweep(op, u0, dt, nsteps)
  scale = float(np.abs(host(u0)).max())
  for name, a, b in zip(("record", "u^N", "w^0"), got[:3], ref[:3]):
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-12 * max(scale, np.abs(b).max()), err_msg=name)
  np.testing.assert_allclose(got[3], ref[3], rtol=0, atol=1e-10 * np.abs(ref[3]).max())
  op.tune(rec_fwd_steps_per_launch=5)
  assert (op.rec_steps_per_launch, op.rec_fwd_steps_per_launch) == (10, 5)
  with pytest.raises(pkg._lib.DGLibraryError):
    op.tune(rec_fwd_steps_per_launch=3)
  op.tune(rec_tile_width=1, rec_fwd_steps_per_launch=20)
  assert op.rec_fwd_steps_per_launch == 10  # 20-step launches need 1024-element tiles
  # the default is by size: one 20-step forward launch up to 3*2^20 elements per plan
  big = pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=4, k=1 << 20), batch=4)
  assert (big.rec_steps_per_launch, big.rec_fwd_steps_per_launch) == (10, 10)
  del big
  mid = pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=4, k=1 << 20), batch=3)
  assert mid.rec_fwd_steps_per_launch == 20


def test_adjoint_rec_needs_the_record_even_without_eta(pkg, gpu):
  """The record kernels read the record on every reverse step, so a null record is an
  argument error whenever there is a step to run, also with eta = NULL; with
  the record and eta = NULL, w is the eta run's w bit for bit."""
  import ctypes

  import torch
  mesh = pkg.BaseGalerkin1D(n=4, k=300)
  op = pkg.operators.DGAdvection1D(mesh)
  dt = mesh.cfl_dt()
  u0 = torch.sin(torch.linspace(0, 6.0, op.field_numel, dtype=torch.float64, device=gpu))
  rec = op.new_jumps(5)
  uN = op.new_field()
  op.forward_rec(u0, 0.0, dt, 5, rec, out=uN)
  w = uN.clone()
  rc = op._lib.dg_lserk4_adj_rec(op._plan, ctypes.c_void_p(w.data_ptr()), None, 0.0, dt, 5,
                                 None, 0, None)
  assert rc == pkg._lib.DG_ERR_ARG and b"null" in op._lib.dg_last_error()
  assert torch.equal(w, uN)  # refused before any launch
  w_noeta, w_eta = uN.clone(), uN.clone()
  op.adjoint_rec(w_noeta, rec, 0.0, dt, 5)
  eta = torch.zeros(op.ktot, dtype=torch.float64, device=gpu)
  op.adjoint_rec(w_eta, rec, 0.0, dt, 5, eta=eta)
  torch.cuda.synchronize()
  assert torch.equal(w_noeta, w_eta)
  # nsteps = 0: nothing to read, a null record is fine
  assert op._lib.dg_lserk4_adj_rec(op._plan, ctypes.c_void_p(w.data_ptr()), None, 0.0, dt, 0,
                                   None, 0, None) == 0


def test_env_override_is_the_tune_key(pkg, gpu, monkeypatch):
  """DG_REC_STEPS_PER_LAUNCH sets the record steps per launch of both directions, as
  dg_plan_tune(DG_TUNE_REC_STEPS_PER_LAUNCH) does (the env override used to leave
  the forward on its size-based 20-step default)."""
  mesh = pkg.BaseGalerkin1D(n=4, k=2000)
  tuned = pkg.operators.DGAdvection1D(mesh).tune(rec_steps_per_launch=8)
  monkeypatch.setenv("DG_REC_STEPS_PER_LAUNCH", "8")
  env = pkg.operators.DGAdvection1D(mesh)
  assert (env.rec_steps_per_launch, env.rec_fwd_steps_per_launch) == \
      (tuned.rec_steps_per_launch, tuned.rec_fwd_steps_per_launch) == (8, 8)
  monkeypatch.setenv("DG_REC_FWD_STEPS_PER_LAUNCH", "20")  # the forward's own override wins
  both = pkg.operators.DGAdvection1D(mesh)
  assert (both.rec_steps_per_launch, both.rec_fwd_steps_per_launch) == (8, 20)


def test_forward_own_tile_width(pkg, gpu):
  """The forward record sweep's own tile width (DG_TUNE_REC_FWD_TILE_WIDTH): the tile shape
  never changes the arithmetic, so at equal steps per launch everything is bit-identical to
  both directions on one width.  Np = 9's default is 1024-element tiles forward (one 20-step
  launch) and 512-element tiles for the adjoint (10 steps); setting rec_tile_width applies to
  both directions again."""
  import torch
  mesh = pkg.BaseGalerkin1D(n=8, k=3000)
  op = pkg.operators.DGAdvection1D(mesh, batch=2)
  assert (op.rec_fwd_tile_width, op.rec_fwd_steps_per_launch) == (2, 20)
  assert (op.rec_tile_width, op.rec_steps_per_launch, op.rec_lane_elements) == (1, 10, 2)
  dt = mesh.cfl_dt()
  u0 = op.new_field()
  op.init_sine([1.0, 0.8], [2.0, 3.0], [0.0, 0.5], out=u0)
  gen = torch.Generator(device=gpu).manual_seed(11)
  u0 += 0.1 * torch.randn(u0.shape, dtype=u0.dtype, device=u0.device, generator=gen)
  nsteps = 20
  op.tune(rec_fwd_steps_per_launch=10)
  mixed = rec_sweep(op, u0, dt, nsteps)
  op.tune(rec_tile_width=2, rec_steps_per_launch=10)
  assert (op.rec_fwd_tile_width, op.rec_tile_width) == (2, 2)
  same = rec_sweep(op, u0, dt, nsteps)
  for name, a, b in zip(("record", "u^N", "w^0", "eta"), mixed, same):
    np.testing.assert_array_equal(a, b, err_msg=name)
  op.tune(rec_fwd_tile_width=1)
  assert (op.rec_fwd_tile_width, op.rec_tile_width) == (1, 2)
  narrow = rec_sweep(op, u0, dt, nsteps)
  for name, a, b in zip(("record", "u^N", "w^0", "eta"), narrow, same):
    np.testing.assert_array_equal(a, b, err_msg=name)
  with pytest.raises(pkg._lib.DGLibraryError):
    op.tune(rec_fwd_tile_width=3)
