"""The config-3 oracle (oracle/burgers.py: Burgers-type flux, SlopeLimitN after every
LSERK4 stage, its frozen-decision tangent and adjoint) — CPU.

The reference never runs this path (SlopeLimitN has no recorded outputs and
the nonlinear flux is build-defined), so it is pinned by identities: the linear flux
reduces to AdvecRHS1D, the tangent matches central differences of the limited step, the
coloured-Jacobian adjoint equals the dense transpose, and the adjoint sweep's gradient
matches a finite difference of the functional (matlab/test_jacobian.m:38-55 method).
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import burgers as ob
from oracle import limiter as olim
from oracle import setup1d

A = 2 * np.pi


def _state(S, rng, jump=0.8):
  x = S["x"]
  return np.sin(2 * np.pi * x) + jump * (x > 0.5) + 0.05 * rng.standard_normal(x.shape)


def test_linear_flux_is_AdvecRHS1D():
  rng = np.random.default_rng(0)
  S = setup1d.uniform_setup(4, 9)
  u = rng.standard_normal((5, 9))
  for inflow in (oadv.INFLOW_A, oadv.INFLOW_A2):
    got, _ = ob.rhs(u, 0.3, A, S, ob.FLUX_LINEAR, inflow)
    ref, _ = oadv.advec_rhs1d(u, 0.3, A, S, inflow)
    np.testing.assert_array_equal(got, ref)
  np.testing.assert_array_equal(ob.jump_residual(u, 0.3, A, S, ob.FLUX_LINEAR),
                                oadv.lift_residual(u, 0.3, A, S))


def test_burgers_rhs_is_conservative_and_consistent():
  """Constant states have zero RHS when they match the inflow; the element-sum of the
  mass-weighted RHS telescopes to the boundary fluxes (central flux is conservative):
  the inflow face carries the central flux (f(uin) + f(u_0))/2, the outflow face f(u_N)."""
  S = setup1d.uniform_setup(3, 10)
  t = 0.05
  uin = oadv.inflow_value(A, t, oadv.INFLOW_A)
  r, _ = ob.rhs(np.full((4, 10), uin), t, A, S)
  np.testing.assert_allclose(r, 0.0, atol=1e-12)
  rng = np.random.default_rng(1)
  u = rng.standard_normal((4, 10))
  r, _ = ob.rhs(u, t, A, S)
  M = np.linalg.inv(S["V"] @ S["V"].T)  # reference mass matrix
  total = np.sum((M @ r) / S["rx"][0][None, :])  # sum_k int_k du/dt
  f_in = A * 0.5 * (0.5 * uin ** 2 + 0.5 * u[0, 0] ** 2)
  f_out = A * 0.5 * u[-1, -1] ** 2
  np.testing.assert_allclose(total, f_in - f_out, rtol=1e-10)


@pytest.mark.parametrize("kind", [ob.FLUX_BURGERS, ob.FLUX_LINEAR])
@pytest.mark.parametrize("limit", [False, True, "1"])
def test_step_tangent_matches_central_difference(kind, limit):
  rng = np.random.default_rng(2)
  S = setup1d.uniform_setup(3, 12, metric="element")
  u = _state(S, rng)
  dt = oadv.bench_dt(S)
  _, ids = ob.limited_step(u, 0.1, dt, A, S, kind, limit=True, return_ids=True)
  assert min(len(i) for i in ids) > 0  # the limiter is active on this state
  d = rng.standard_normal(u.shape)
  _, jv = ob.step_jvp(u, d, 0.1, dt, A, S, kind, limit=limit)
  h = 1e-6
  fd = (ob.limited_step(u + h * d, 0.1, dt, A, S, kind, limit=limit)
        - ob.limited_step(u - h * d, 0.1, dt, A, S, kind, limit=limit)) / (2 * h)
  assert np.max(np.abs(jv - fd)) <= 1e-8 * np.max(np.abs(jv))


@pytest.mark.parametrize("kind,limit", [(ob.FLUX_BURGERS, True), (ob.FLUX_BURGERS, False),
                                        (ob.FLUX_LINEAR, True), (ob.FLUX_BURGERS, "1")])
def test_coloured_adjoint_equals_dense_transpose(kind, limit):
  rng = np.random.default_rng(3)
  S = setup1d.uniform_setup(2, 25, metric="element")  # K > 21: real colouring
  u = _state(S, rng)
  dt = oadv.bench_dt(S)
  M = ob.step_matrix(u, 0.2, dt, A, S, kind, limit=limit)
  w = rng.standard_normal(u.shape)
  got = ob.step_vjp(u, w, 0.2, dt, A, S, kind, limit=limit)
  ref = (M.T @ w.T.ravel()).reshape(25, 3).T
  np.testing.assert_allclose(got, ref, atol=1e-13 * np.abs(ref).max())
  # and <J d, w> = <d, J^T w>
  d = rng.standard_normal(u.shape)
  _, jd = ob.step_jvp(u, d, 0.2, dt, A, S, kind, limit=limit)
  assert abs(np.sum(jd * w) - np.sum(d * got)) <= 1e-12 * abs(np.sum(jd * w))


def test_linear_unlimited_adjoint_is_the_linear_adjoint():
  rng = np.random.default_rng(4)
  S = setup1d.uniform_setup(3, 8)
  u = rng.standard_normal((4, 8))
  w = rng.standard_normal((4, 8))
  dt = oadv.bench_dt(S)
  got = ob.step_vjp(u, w, 0.0, dt, A, S, ob.FLUX_LINEAR, limit=False)
  np.testing.assert_allclose(got, oadj.adjoint_step(w, dt, A, S), atol=1e-13)


@pytest.mark.parametrize("limit", [False, True, "1"])
def test_adjoint_sweep_gradient_matches_finite_difference(limit):
  """dJ/du0 for J = <g, u^N> + src/2 sum |u^n|^2 through 3 limited Burgers steps."""
  rng = np.random.default_rng(5)
  S = setup1d.uniform_setup(3, 14, metric="element")
  u0 = _state(S, rng)
  dt = oadv.bench_dt(S)
  g = rng.standard_normal(u0.shape)
  d = rng.standard_normal(u0.shape)
  nsteps, src = 3, 0.4

  def J(u):
    snaps, _ = ob.forward_sweep(u, 0.0, dt, nsteps, A, S, limit=limit)
    return oadj.functional(snaps, dt, src, g), snaps

  _, snaps = J(u0)
  times = [0.0]
  for _ in range(nsteps):
    times.append(times[-1] + dt)
  w0, eta, _ = ob.adjoint_sweep(g, snaps, times, dt, A, S, limit=limit, src_coef=src)
  h = 1e-6
  fd = (J(u0 + h * d)[0] - J(u0 - h * d)[0]) / (2 * h)
  assert abs(fd - np.sum(w0 * d)) <= 1e-7 * abs(fd)
  assert eta.shape == (14,) and np.all(np.isfinite(eta))


def test_limited_step_limits_every_stage():
  """With the limiter on, the state after each step is a fixed point of SlopeLimitN in
  the cells it flagged at the last stage (they are linear with a minmod slope)."""
  rng = np.random.default_rng(6)
  S = setup1d.uniform_setup(4, 30)
  u = _state(S, rng, jump=1.0)
  dt = oadv.bench_dt(S)
  y, ids = ob.limited_step(u, 0.0, dt, A, S, return_ids=True)
  modes = S["invV"] @ y[:, ids[-1]]
  np.testing.assert_allclose(modes[2:], 0.0, atol=1e-12)
  v_before, _ = olim.cell_average(u, S)
  v_after, _ = olim.cell_average(y, S)
  assert np.all(np.isfinite(v_after)) and np.max(np.abs(v_after - v_before)) < 1.0
