"""Identities that pin the parts of the oracle the reference records no outputs for
(the advection adjoint, the indicator, the limiter) — CPU."""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import limiter as olim
from oracle import setup1d

A = 2 * np.pi


@pytest.mark.parametrize("N,K", [(1, 5), (2, 7), (4, 6), (7, 4)])
def test_transposed_operator_dot_product(N, K):
  """<L u, w> = <u, L^T w> with L^T assembled by scatter through vmapM/vmapP."""
  rng = np.random.default_rng(N + K)
  S = setup1d.uniform_setup(N, K)
  for _ in range(3):
    u = rng.standard_normal((N + 1, K))
    w = rng.standard_normal((N + 1, K))
    lhs = np.sum(oadj.advec_linear(u, A, S) * w)
    rhs = np.sum(u * oadj.advec_linear_T(w, A, S))
    assert abs(lhs - rhs) <= 1e-12 * max(abs(lhs), 1.0)


def test_transposed_operator_matches_dense_transpose():
  S = setup1d.uniform_setup(3, 5)
  L = oadj.dense_operator(lambda u: oadj.advec_linear(u, A, S), (4, 5))
  LT = oadj.dense_operator(lambda w: oadj.advec_linear_T(w, A, S), (4, 5))
  np.testing.assert_allclose(LT, L.T, atol=1e-12 * np.abs(L).max())


def test_linear_part_plus_inflow_is_AdvecRHS1D():
  rng = np.random.default_rng(1)
  S = setup1d.uniform_setup(4, 9)
  u = rng.standard_normal((5, 9))
  rhs, _ = oadv.advec_rhs1d(u, 0.3, A, S)
  forcing, _ = oadv.advec_rhs1d(np.zeros_like(u), 0.3, A, S)
  np.testing.assert_allclose(rhs, oadj.advec_linear(u, A, S) + forcing, atol=1e-12)


@pytest.mark.parametrize("scheme", ["lserk4", "euler"])
def test_reverse_sweep_equals_monolithic_adjoint(scheme):
  """The backward sweep solves (J_F^T - I) v = -K of Main_finite_difference.py:73
  (config 1 plumbing: small DG problem, forward Euler and LSERK4)."""
  rng = np.random.default_rng(2)
  S = setup1d.uniform_setup(1, 4)
  dt = oadv.bench_dt(S) * (1.0 if scheme == "lserk4" else 0.2)
  u0 = rng.standard_normal((2, 4))
  snaps, times = oadv.forward_sweep(u0, 0.1, dt, 5, A, S, scheme=scheme)
  g = rng.standard_normal(u0.shape)
  src = 0.8
  w0, _, states = oadj.adjoint_sweep(g, snaps, times, dt, A, S, src_coef=src, scheme=scheme,
                                     with_eta=False)
  mono = oadj.monolithic_adjoint(snaps, dt, A, S, src, g, scheme=scheme)
  for n in range(len(snaps)):
    np.testing.assert_allclose(states[n], mono[n], atol=1e-11 * np.abs(mono[0]).max())


def test_adjoint_gradient_by_complex_step():
  """dJ/du0 from the sweep against the complex-step derivative (matlab/test_jacobian.m:38-55
  method): J is quadratic in u0, so Im J(u0 + i h d)/h is exact to rounding."""
  rng = np.random.default_rng(3)
  S = setup1d.uniform_setup(2, 6)
  dt = oadv.bench_dt(S)
  u0 = rng.standard_normal((3, 6))
  g = rng.standard_normal((3, 6))
  d = rng.standard_normal((3, 6))
  src, nsteps = 0.5, 4
  snaps, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S, inflow=oadv.INFLOW_ZERO)
  w0, _, _ = oadj.adjoint_sweep(g, snaps, times, dt, A, S, inflow=oadv.INFLOW_ZERO,
                                src_coef=src, with_eta=False)
  h = 1e-20
  Sm = oadj.step_matrix(dt, A, S)
  uc = (u0 + 1j * h * d).ravel(order="F")
  J = np.sum(g.ravel(order="F") * (np.linalg.matrix_power(Sm, nsteps) @ uc))
  for n in range(nsteps):
    un = np.linalg.matrix_power(Sm, n) @ uc
    J = J + 0.5 * src * np.sum(un * un)
  cs = J.imag / h
  assert abs(cs - np.sum(w0 * d)) <= 1e-10 * abs(cs)


def test_indicator_is_dt_weighted_adjoint_times_lift_residual():
  rng = np.random.default_rng(4)
  S = setup1d.uniform_setup(3, 8)
  dt = oadv.bench_dt(S)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
  snaps, times = oadv.forward_sweep(u0, 0.0, dt, 3, A, S)
  g = rng.standard_normal(u0.shape)
  _, eta, states = oadj.adjoint_sweep(g, snaps, times, dt, A, S)
  ref = np.zeros(8)
  for n in range(3):
    ref += dt * np.sum(states[n + 1] * oadv.lift_residual(snaps[n + 1], times[n + 1], A, S), 0)
  np.testing.assert_allclose(eta, ref, rtol=1e-14, atol=1e-300)


def test_indicator_vanishes_for_continuous_state():
  """The interelement-jump residual is zero for a state continuous across faces that also
  satisfies the inflow condition, and the outflow face never contributes."""
  S = setup1d.uniform_setup(2, 6)
  t = 0.05
  uin = oadv.inflow_value(A, t, oadv.INFLOW_A)
  u = np.full((3, 6), uin)  # constant = inflow value: no jumps anywhere
  R = oadv.lift_residual(u, t, A, S)
  np.testing.assert_allclose(R, 0.0, atol=1e-13)


# --- limiter ---------------------------------------------------------------
def test_minmod_truth_table():
  v = np.array([[1.0, -1.0, 1.0, 0.0, 2.0, -3.0],
                [2.0, -2.0, -1.0, 1.0, 0.5, -1.0],
                [3.0, -0.5, 1.0, 1.0, 1.0, -2.0]])
  np.testing.assert_array_equal(olim.minmod(v), [1.0, -0.5, 0.0, 0.0, 0.5, -1.0])


def test_minmod_b_keeps_small_slopes():
  v = np.array([[0.01, 5.0], [1.0, 1.0], [-1.0, 2.0]])
  # |v1| <= M h^2 keeps v1 (TVB); otherwise plain minmod
  np.testing.assert_array_equal(olim.minmod_b(v, 100.0, np.array([0.1, 0.1])), [0.01, 1.0])


def test_limiter_leaves_linear_data_alone():
  """Interior cells of globally linear data are untouched.  The two end cells are
  flagged: SlopeLimitN.m:18 replicates the end averages, so their one-sided difference
  is 0 and minmod flattens them (reference semantics)."""
  S = setup1d.uniform_setup(4, 12)
  u = 0.3 + 2.0 * S["x"]
  out, ids = olim.slope_limit_n(u, S, return_ids=True)
  np.testing.assert_array_equal(ids, [0, 11])
  np.testing.assert_array_equal(out[:, 1:11], u[:, 1:11])
  v, _ = olim.cell_average(u, S)
  np.testing.assert_allclose(out[:, [0, 11]], np.ones((5, 1)) * v[[0, 11]], atol=1e-14)


def test_limiter_flags_discontinuity_and_preserves_means():
  S = setup1d.uniform_setup(3, 40)
  u = np.where(S["x"] > 0.5, 1.0, 0.0) + np.sin(6 * S["x"])
  out, ids = olim.slope_limit_n(u, S, return_ids=True)
  assert 0 < ids.size < 40
  assert 19 in ids or 20 in ids  # the cell at the jump
  v_in, _ = olim.cell_average(u, S)
  v_out, _ = olim.cell_average(out, S)
  np.testing.assert_allclose(v_out, v_in, atol=1e-13)  # limiting is conservative
  # limited cells are linear: the modes above 1 vanish
  modes = S["invV"] @ out[:, ids]
  np.testing.assert_allclose(modes[2:], 0.0, atol=1e-12)


def test_slope_limit_1_is_linear_everywhere():
  S = setup1d.uniform_setup(3, 10)
  u = np.sin(2 * np.pi * S["x"])
  out = olim.slope_limit_1(u, S)
  np.testing.assert_allclose((S["invV"] @ out)[2:], 0.0, atol=1e-12)


def test_sum_rows_and_argmax_semantics():
  x = np.array([[1.0, 2.0], [3.0, -4.0], [0.5, 0.25]])
  np.testing.assert_array_equal(oadj.sum_rows(x), [4.5, -1.75])
  assert oadj.argmax([1.0, 3.0, 3.0]) == 1
  assert oadj.argmax([1.0, np.nan, 5.0, np.nan]) == 1
  assert oadj.argmax([1.0, -5.0, 4.0], use_abs=True) == 1


def test_tvb_slope_limiter_reduces_to_minmod_and_keeps_small_slopes():
  """oracle slope_limit_n / slope_limit_1 with the TVB constant (utils/minmodB.m:6-11): M = 0
  is the plain minmod; a huge M keeps every cell's own linear slope (SlopeLimitLin then only
  projects to the linear part); intermediate M switches per cell on |ux| > M h^2."""
  from oracle import limiter as olim
  from oracle import setup1d
  rng = np.random.default_rng(5)
  S = setup1d.uniform_setup(3, 200, metric="element")
  x = S["x"]
  u = np.sin(2 * np.pi * x) + (x > 0.5) + 0.02 * rng.standard_normal(x.shape)
  np.testing.assert_array_equal(olim.slope_limit_1(u, S, M=0.0), olim.slope_limit_1(u, S))
  big = olim.slope_limit_1(u, S, M=1e30)
  # the Pi^1 projection of u: cell average + linear mode, i.e. SlopeLimitLin with m = ux
  v, uh0 = olim.cell_average(u, S)
  uh1 = olim._row_dot(S["invV"][1, :], u)
  V = S["V"]
  ul = V[:, 0:1] * uh0[None, :] + V[:, 1:2] * uh1[None, :]
  np.testing.assert_allclose(big, ul, atol=1e-12)
  h = x[-1, :] - x[0, :]
  mid = olim.slope_limit_1(u, S, M=1e5)
  plain = olim.slope_limit_1(u, S)
  differs = np.any(np.abs(mid - plain) > 1e-12, axis=0)
  assert 0 < differs.sum() < u.shape[1]
