"""The DG-in-time oracle (oracle/dgtime.py: matlab/dg_march.m, adj_march.m, fem_setup.m,
MAIN.m) — CPU.  The reference records no outputs of these routines, so the restatement is
pinned by the reference's own verification method (the complex-step Jacobian test of
matlab/test_jacobian.m:11-55), by convergence to the exact solution of du/dt = sin(u), and
by the host operators the GPU path uses agreeing with fem_setup's."""
import importlib

import numpy as np
import pytest

from oracle import dgtime as odt


@pytest.mark.parametrize("N", [1, 2, 3])
def test_newton_jacobian_complex_step(N):
  """matlab/test_jacobian.m: || Im R(U + i h d)/h - dRdU d || / || dRdU d || at h = 1e-20."""
  rng = np.random.default_rng(N)
  st = odt.fem_setup(N, [0.0, 1.0], 4 * N)
  for _ in range(10):
    U = rng.random(N + 1)
    d = rng.random(N + 1)
    d /= np.linalg.norm(d)
    _, J = odt._newton_parts(st, U, 1.0)
    h = 1e-20
    Rc, _ = odt._newton_parts(st, U + 1j * h * d, 1.0)
    jd = J @ d
    assert np.linalg.norm(Rc.imag / h - jd) <= 1e-12 * np.linalg.norm(jd)


def test_forward_march_converges_to_exact_solution():
  errs = []
  for Ks in (2, 4, 8, 16):
    times = np.linspace(0.0, 2.0, Ks + 1)
    t, y, its = odt.dg_march(1, times, 1.0)
    assert max(its) <= 10
    errs.append(abs(y[-1][-1] - odt.exact(2.0)))  # end-of-slab value (superconvergent)
  rates = np.log2(np.array(errs[:-1]) / np.array(errs[1:]))
  assert np.all(rates > 2.5), rates  # order 2N+1 = 3 at the slab ends for N = 1


def test_adjoint_march_and_refine_loop():
  times = np.linspace(0.0, 2.0, 3)
  seq = []
  for _ in range(6):
    t, y, _ = odt.dg_march(1, times, 1.0)
    ta, v, err = odt.adj_march(2, times, y, t)
    assert err.shape == (times.size - 1,) and np.all(np.isfinite(err))
    assert all(vk.shape == (3,) for vk in v)
    times, ri = odt.refine(times, err)
    seq.append(ri)
  assert times.size == 9 and np.all(np.diff(times) > 0)
  assert seq[0] == 0  # the first slab carries the larger indicator (MAIN.m initial split)


@pytest.mark.parametrize("N", [1, 2, 4])
def test_host_operators_match_fem_setup(N):
  """The reference-element operators dgtime.py hands the kernels equal fem_setup.m's."""
  dgt = importlib.import_module("adjoint-ode-adaptivity_amd.dgtime")
  f = dgt.forward_ops(N)
  st = odt.fem_setup(N, [0.3, 0.7], 30 * N)
  np.testing.assert_allclose(f["Phi"], st["Phi"], atol=1e-12)
  np.testing.assert_allclose(f["wq"], st["w"], atol=1e-14)
  np.testing.assert_allclose(f["S"], np.linalg.solve(st["V"] @ st["V"].T, st["Dr"]), atol=1e-12)
  a = dgt.adjoint_ops(N)
  sa = odt.fem_setup(N + 1, [0.3, 0.7], 2 * (N + 1))
  np.testing.assert_allclose(a["Phia"], sa["Phi"], atol=1e-12)
  np.testing.assert_allclose(a["Ma"], np.linalg.inv(sa["V"] @ sa["V"].T), atol=1e-12)
  # Pext / Ifa evaluate the forward polynomial like polyfit/polyval on the slab
  rng = np.random.default_rng(N)
  U = rng.standard_normal(N + 1)
  tf = odt.fem_setup(N, [0.3, 0.7], 2)["x"]
  pu = np.polyfit(tf, U, N)
  hk = sa["x"][0] - sa["x"][-1]
  np.testing.assert_allclose(a["Pext"] @ U, np.polyval(pu, tf[0] + (1 + sa["r"]) * hk / 2),
                             atol=1e-10)
  np.testing.assert_allclose(a["Ifa"] @ U, np.polyval(pu, sa["x"]), atol=1e-12)
