"""Effectivity of the DG-advection DWR indicator on the CPU oracle (VERDICT r01 item 7;
the reference's printout of J(u_H) - J(u_h) next to sum(err), matlab/MAIN.m:55-76).

Problem: a bump transported by a = 2 pi with zero inflow (exact solution u0(x - a t)), the
linear window functional J(u) = int psi u(x, T) (oracle/effectivity.py).  Pinned facts:
* the p-prolonged residual variant (order N+1 residual x order N+1 adjoint) sums to
  J_{N+1}(u_{N+1}) - J_h(u_h) exactly (the DWR identity of a linear scheme and functional);
* the kernels' jump indicator does NOT estimate the error (its sum is off by 1-2 orders of
  magnitude and of either sign), but it ranks elements by the gain of refining them at
  least as well as the p-variant (Spearman >= 0.85 here): it is a refinement indicator,
  not an error estimator -- DESIGN.md §6 records the numbers (profiles/r02/effectivity.json).
* the jump indicator here is the one the kernels compute (oracle/adjoint.py's sweep with the
  window weight as terminal adjoint), so the GPU parity tests of eta carry over.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import effectivity as ef


def bump(x):
  return np.exp(-300.0 * (x - 0.3) ** 2)


@pytest.fixture(scope="module")
def case():
  return ef.study(2, 16, 0.05, bump)


def test_p_variant_is_exact_for_the_enriched_error(case):
  assert abs(case["effectivity_p_vs_p1"] - 1.0) <= 1e-9
  # and it sees a fair part of the true error (p-enrichment misses the rest)
  assert 0.5 <= case["effectivity_p_vs_exact"] <= 1.0


def test_jump_indicator_ranks_but_does_not_estimate(case):
  assert case["spearman_jump"] >= 0.85
  assert case["spearman_jump"] >= case["spearman_p"] - 0.05
  assert case["top5_overlap_jump"] >= 4
  assert abs(case["effectivity_jump_vs_exact"]) > 3.0  # not an estimate of the error


def test_jump_indicator_is_the_kernels_sweep(case):
  """ef.jump_indicator == oracle.adjoint.adjoint_sweep (the GPU's parity reference) with the
  window weight as terminal adjoint."""
  from oracle import setup1d
  from oracle.advec import INFLOW_ZERO, forward_sweep
  S = setup1d.startup1d(2, np.linspace(0.0, 1.0, 17), metric="element")
  snaps, times = forward_sweep(bump(S["x"]), 0.0, case["dt"], 20, 2 * np.pi, S, INFLOW_ZERO)
  g = ef.weight(S)
  _, eta, _ = oadj.adjoint_sweep(g, snaps, times, case["dt"], 2 * np.pi, S, inflow=INFLOW_ZERO)
  np.testing.assert_allclose(ef.jump_indicator(snaps, times, case["dt"], 2 * np.pi, S), eta,
                             rtol=1e-13, atol=1e-18)


def test_window_functional_is_quadrature_exact():
  from oracle import setup1d
  S = setup1d.startup1d(3, np.linspace(0.0, 1.0, 33), metric="element")
  u = np.ones((4, 32))  # u = 1: J = int psi = 0.06 (psi is C^3 at its edges: 1e-9 here)
  assert abs(ef.functional(u, S) - ef.exact_functional(lambda x: np.ones_like(x), 0.0)) < 1e-9
