"""The oracle against the reference's own recorded outputs (CPU).

* utils/One_code.mlx cached MATLAB R2020b outputs (tests/golden/one_code_mlx_golden.json):
  operators, mesh, maps and the final-stage du/rhsu/resu of the executed N=2, K=20,
  T=2 LSERK4 run — 4-decimal display, so |oracle - golden| <= 5e-5.
* python/Main_finite_difference.py adapt loop run by the reference's own functions
  (tests/golden/fd_adapt_golden.json): refine indices bit-exact, floats <= 1e-12.
"""
import json
import os

import numpy as np
import pytest

from oracle import advec as oadv
from oracle import fd as ofd
from oracle import setup1d

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def mlx():
  with open(os.path.join(GOLDEN, "one_code_mlx_golden.json")) as f:
    g = json.load(f)
  by = {}
  for e in g["entries"]:
    by.setdefault(e["name"], []).append(e)
  return g, by


@pytest.fixture(scope="module")
def golden_run():
  S = setup1d.uniform_setup(2, 20, 0.0, 1.0)  # MATLAB metric (GeometricFactors1D.m)
  u0 = np.sin(2 * np.pi * S["x"])  # One_code.mlx:103
  out = oadv.advec1d(u0.copy(), 2.0, 2 * np.pi, S, inflow=oadv.INFLOW_A2)
  return S, u0, out


def _cmp(entry, arr, atol):
  rows = np.array(entry["rows"], dtype=float)
  arr = np.atleast_2d(np.asarray(arr, dtype=float))
  np.testing.assert_allclose(arr[:rows.shape[0], :rows.shape[1]], rows, rtol=0, atol=atol,
                             err_msg=f"{entry['name']} (line {entry['line']})")


def test_reference_element_operators(mlx, golden_run):
  g, by = mlx
  S, _, _ = golden_run
  atol = g["display_atol"]
  _cmp(by["r"][0], S["r"][:, None], atol)
  _cmp(by["V"][0], S["V"], atol)
  _cmp(by["Dr"][0], S["Dr"], atol)
  _cmp(by["Dr"][1], S["Dr"], atol)
  _cmp(by["LIFT"][0], S["LIFT"], atol)
  _cmp(by["rk4a"][0], setup1d.RK4A[None, :], atol)


def test_mesh_metric_and_maps(mlx, golden_run):
  g, by = mlx
  S, u0, _ = golden_run
  atol = g["display_atol"]
  _cmp(by["x"][1], S["x"], atol)
  _cmp(by["Fx"][0], S["Fx"], atol)
  _cmp(by["nx"][0], S["nx"], atol)
  _cmp(by["Fscale"][0], S["Fscale"], atol)
  _cmp(by["rx"][0], S["rx"], atol)
  _cmp(by["u"][0], u0, atol)
  m = S["matlab"]
  _cmp(by["Fmask"][0], m["Fmask"][None, :], 0)
  _cmp(by["EToE"][0], m["EToE"], 0)
  _cmp(by["EToF"][0], m["EToF"], 0)
  _cmp(by["vmapM"][0], m["vmapM"][:, None], 0)
  _cmp(by["vmapP"][0], m["vmapP"][:, None], 0)
  _cmp(by["vmapB"][0], m["vmapB"][:, None], 0)
  _cmp(by["mapB"][0], m["mapB"][:, None], 0)
  assert by["mapI"][0]["rows"][0][0] == m["mapI"]
  assert by["mapO"][0]["rows"][0][0] == m["mapO"]
  ans = by["ans"]
  _cmp(ans[0], m["vmapM"][None, :], 0)  # vmapM' (:145)
  _cmp(ans[1], m["vmapP"][None, :], 0)  # vmapP' (:146)


def test_lserk4_golden_run(mlx, golden_run):
  """The only reference-produced numbers on the RHS+LSERK4 path (One_code.mlx:151-154)."""
  g, by = mlx
  _, _, out = golden_run
  atol = g["display_atol"]
  assert out["nsteps"] == 1341
  np.testing.assert_allclose(out["dt"], 1.4914243102162564e-3, rtol=1e-15)
  _cmp(by["du"][0], out["du"], atol)
  _cmp(by["rhsu"][0], out["rhsu"], atol)
  _cmp(by["resu"][0], out["resu"], atol)
  assert abs(by["ans"][2]["rows"][0][0] - out["du"].ravel(order="F")[2]) <= atol  # du(3)


def test_inflow_variant_of_AdvecRHS1D_does_not_match_golden(mlx, golden_run):
  """utils/AdvecRHS1D.m:14 (uin = -sin(a t)) is NOT what the executed live script ran
  (One_code.mlx:129, -sin(a^2 t)): the flag matters."""
  _, by = mlx
  S, u0, _ = golden_run
  out = oadv.advec1d(u0.copy(), 2.0, 2 * np.pi, S, inflow=oadv.INFLOW_A)
  rows = np.array(by["rhsu"][0]["rows"])
  assert np.max(np.abs(out["rhsu"] - rows)) > 1.0


@pytest.fixture(scope="module")
def fd_golden():
  with open(os.path.join(GOLDEN, "fd_adapt_golden.json")) as f:
    return json.load(f)


def test_fd_adapt_loop_matches_reference_functions(fd_golden):
  cfg = fd_golden["config"]
  iters = fd_golden["iterations"]
  times = np.linspace(cfg["t_span"][0], cfg["t_span"][1], cfg["n_steps0"] + 1)
  out = ofd.adapt_loop(times, cfg["u0"], cfg["ref_factor"], len(iters))
  assert [o["ref_idx"] for o in out] == [it["ref_idx"] for it in iters]
  for o, it in zip(out, iters):
    np.testing.assert_array_equal(o["times"], np.array(it["times"]))
    for key in ("u", "v", "err_fine", "err_steps"):
      np.testing.assert_allclose(o[key], np.array(it[key]), rtol=1e-12, atol=1e-15)


def test_fd_golden_first_iterations_survey_values(fd_golden):
  it0, it1 = fd_golden["iterations"][:2]
  np.testing.assert_allclose(it0["u"], [1, 1.8414709848078965, 2.80506170934973], rtol=1e-15)
  np.testing.assert_allclose(it0["err_steps"], [0.4363759560670887, 0.1258225898236005],
                             rtol=1e-14)
  assert [it["ref_idx"] for it in fd_golden["iterations"][:12]] == \
      [1, 1, 4, 4, 1, 3, 6, 8, 10, 1, 11, 6]
