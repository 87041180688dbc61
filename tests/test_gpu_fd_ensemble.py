"""The finite-difference DWR adapt loop for ODE ensembles on the GPU (csrc/dg_fd.hip via
fd_ensemble.FDEnsemble).  Needs an MI355X.

Pinned by the reference itself: with one member and u0 = 1 the device loop must reproduce
tests/golden/fd_adapt_golden.json — the outputs of python/Main_finite_difference.py's own
functions (tests/golden/make_fd_golden.py) — refine indices bit-exact, floats to 1e-12.
Ensembles are checked member by member against the oracle (oracle/fd.py)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import fd as ofd

pytestmark = pytest.mark.gpu


def rel(x, ref):
  return float(np.max(np.abs(np.asarray(x) - np.asarray(ref))) / max(np.max(np.abs(ref)), 1e-300))


def test_reproduces_the_reference_golden_run(pkg, gpu):
  with open(os.path.join(GOLDEN, "fd_adapt_golden.json")) as f:
    g = json.load(f)
  cfg = g["config"]
  times = np.linspace(0.0, 2.0, cfg["n_steps0"] + 1)
  ens = pkg.fd_ensemble.FDEnsemble(times, [cfg["u0"]], ref_factor=cfg["ref_factor"])
  for it in g["iterations"]:
    np.testing.assert_array_equal(ens.times, np.array(it["times"]))
    U, V, err = ens.sweep(with_v=True)
    assert rel(U[:, 0].cpu().numpy(), it["u"]) <= 1e-12
    assert rel(V[:, 0].cpu().numpy(), it["v"]) <= 1e-12
    assert rel(err[0].cpu().numpy(), it["err_steps"]) <= 1e-12
    assert ens.adapt() == it["ref_idx"]


def test_ensemble_members_match_the_oracle(pkg, gpu):
  rng = np.random.default_rng(3)
  u0 = rng.uniform(-2.5, 2.5, 4097)
  times = np.sort(np.concatenate(([0.0, 2.0], rng.uniform(0.05, 1.95, 9))))
  rf = 4
  ens = pkg.fd_ensemble.FDEnsemble(times, u0, ref_factor=rf)
  U, V, err = (t.cpu().numpy() for t in ens.sweep(with_v=True))
  dt_n = np.diff(times)
  for j in (0, 1, 1000, 4096):
    u = ofd.forward_solve(ofd.sin_update, dt_n, u0[j])
    v = ofd.adj_solve(ofd.u2_k, ofd.sin_jf, dt_n, u, rf)
    steps = ofd.window_errors(ofd.err_est(ofd.sin_update, u, v, dt_n, rf), rf)
    assert rel(U[:, j], u) <= 1e-12
    assert rel(V[:, j], v) <= 1e-12
    assert rel(err[j], steps) <= 1e-12
  # the ensemble indicator is the fixed-order member sum
  ens.adapt()
  acc = err[0].copy()
  for r in range(1, err.shape[0]):
    acc = acc + err[r]
  np.testing.assert_array_equal(ens.history[-1]["err_steps"], acc)
