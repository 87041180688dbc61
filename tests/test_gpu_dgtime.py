"""Batched DG-in-time marches on the GPU (csrc/dg_time.hip via dgtime.DGTimeEnsemble)
against the oracle restatement of matlab/dg_march.m / adj_march.m / MAIN.m, one ensemble
member per lane.  Needs an MI355X.

Tolerances: nodal values, adjoints and indicators within 1e-10 of max|oracle| (the
Newton iteration stops on ||U_old - U_next|| <= 1e-7 as dg_march.m:53, so equal iteration
counts are required too); the MAIN.m refine sequence is bit-exact."""
import numpy as np
import pytest

from oracle import dgtime as odt

pytestmark = pytest.mark.gpu
RTOL = 1e-10


def rel(x, ref):
  return float(np.max(np.abs(np.asarray(x) - np.asarray(ref))) / max(np.max(np.abs(ref)), 1e-300))


@pytest.mark.parametrize("N", [1, 2, 3])
def test_march_and_adjoint_match_oracle(pkg, gpu, N):
  rng = np.random.default_rng(N)
  times = np.sort(np.concatenate(([0.0, 2.0], rng.uniform(0.1, 1.9, 4))))
  y0 = np.array([1.0, 0.3, -0.7, 2.5, 0.05])
  ens = pkg.dgtime.DGTimeEnsemble(N, times, y0)
  Y, its, td = ens.march()
  V, err = ens.adjoint(Y, td)
  Y, its, V, err = (t.cpu().numpy() for t in (Y, its, V, err))
  for j, y in enumerate(y0):
    t, yo, ito = odt.dg_march(N, times, y)
    ta, vo, erro = odt.adj_march(N + 1, times, yo, t, y0=y)
    assert list(its[:, j]) == ito
    assert rel(Y[:, :, j], np.array(yo)) <= RTOL
    assert rel(V[:, :, j], np.array(vo)) <= RTOL
    assert rel(err[j], erro) <= RTOL


def test_main_adapt_loop_refine_sequence(pkg, gpu):
  """MAIN.m's loop (n = 1, y0 = 1): the device march/adjoint/indicator reproduce the
  oracle's refine sequence over 10 iterations."""
  times = np.linspace(0.0, 2.0, 3)
  ens = pkg.dgtime.DGTimeEnsemble(1, times, [1.0])
  t_or = times.copy()
  for _ in range(10):
    ri = ens.adapt()
    t, y, _ = odt.dg_march(1, t_or, 1.0)
    _, _, err = odt.adj_march(2, t_or, y, t)
    assert rel(ens.history[-1]["err"], np.abs(err)) <= RTOL  # |err| (MAIN.m:137's abs)
    t_or, ri_or = odt.refine(t_or, err)
    assert ri == ri_or
    np.testing.assert_array_equal(ens.times, t_or)


def test_ensemble_indicator_is_the_member_sum(pkg, gpu):
  rng = np.random.default_rng(7)
  y0 = rng.uniform(0.2, 2.8, 1000)
  times = np.linspace(0.0, 2.0, 9)
  ens = pkg.dgtime.DGTimeEnsemble(2, times, y0)
  Y, its, td = ens.march()
  _, err = ens.adjoint(Y, td)
  tot = ens.indicator(err).cpu().numpy()
  e = err.cpu().numpy()
  acc = np.abs(e[0])
  for r in range(1, e.shape[0]):
    acc = acc + np.abs(e[r])  # member magnitudes, summed in member order
  np.testing.assert_array_equal(tot, acc)
  for j in (0, 333, 999):  # spot-check members against the oracle
    t, yo, _ = odt.dg_march(2, times, y0[j])
    _, _, erro = odt.adj_march(3, times, yo, t, y0=y0[j])
    assert rel(e[j], erro) <= RTOL
