"""The GPU pinned DIRECTLY to the reference's recorded numbers.

* One_code.mlx's executed run (N=2, K=20, T=2, uin = -sin(a^2 t), 1341 steps) records the
  last stage's du (2x20), rhsu (3x20) and resu (3x20) after the final step
  (utils/One_code.mlx:151-154, cached MATLAB R2020b values in
  tests/golden/one_code_mlx_golden.json, displayed to 4 decimals).  The GPU runs 1340 steps
  with dg_lserk4_fwd, then replays step 1341 stage by stage with dg_advec_rhs (the kernel's
  AdvecRHS1D) and the low-storage update of One_code.mlx:135-136, and the recorded arrays are
  compared at the display tolerance 5e-5.  du is the face-jump array One_code.mlx:126-131
  forms from the stage's input state, gathered here from the GPU's state.
* A constructed exact tie: two bit-identical bumps on a uniform mesh, far from the inflow, so
  the indicator is bit-identical at the two copies; the refine index must be the first copy's
  (numpy argmax / dg_argmax: first index on ties), on the GPU and in the oracle.
"""
import json
import os

import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
A = 2 * np.pi


def _golden():
  with open(os.path.join(GOLDEN, "one_code_mlx_golden.json")) as f:
    g = json.load(f)
  by = {}
  for e in g["entries"]:
    by.setdefault(e["name"], []).append(np.array(e["rows"], dtype=float))
  return g["display_atol"], by


def host(t):
  return t.detach().cpu().numpy()


def test_last_stage_du_rhsu_resu_match_the_matlab_record(pkg, gpu):
  import torch
  atol, by = _golden()
  N, K = 2, 20
  S = setup1d.uniform_setup(N, K, 0.0, 1.0)  # MATLAB mesh; x for the IC
  mesh = pkg.BaseGalerkin1D(n=N, v_x=np.linspace(0.0, 1.0, K + 1))
  op = pkg.operators.DGAdvection1D(mesh, a=A, inflow="a2")
  dt, nsteps = oadv.cfl_dt(S, 2.0)  # One_code.mlx:111-113
  assert nsteps == 1341
  u0 = np.sin(2 * np.pi * S["x"])  # One_code.mlx:103
  u = torch.tensor(setup1d.to_elem_major(u0), device=gpu)
  op.forward(u, 0.0, dt, nsteps - 1)  # steps 1..1340 on the fused kernels
  t = 0.0
  for _ in range(nsteps - 1):  # the library's time levels: time = time + dt (:139)
    t = t + dt
  rk4a = [0.0, -567301805773.0 / 1357537059087.0, -2404267990393.0 / 2016746695238.0,
          -3550918686646.0 / 2091501179385.0, -1275806237668.0 / 842570457699.0]
  rk4b = [1432997174477.0 / 9575080441755.0, 5161836677717.0 / 13612068292357.0,
          1720146321549.0 / 2090206949498.0, 3134564353537.0 / 4481467310338.0,
          2277821191437.0 / 14882151754819.0]
  rk4c = [0.0, 1432997174477.0 / 9575080441755.0, 2526269341429.0 / 6820363962896.0,
          2006345519317.0 / 3224310063776.0, 2802321613138.0 / 2924317926251.0]
  np.testing.assert_allclose(rk4a, by["rk4a"][0][0], atol=atol)  # the recorded coefficients
  resu = torch.zeros_like(u)
  rhsu = torch.empty_like(u)
  for s in range(5):  # step 1341, stage by stage (One_code.mlx:120-137)
    stage_in = u.clone()
    op.rhs(u, t + rk4c[s] * dt, out=rhsu)  # AdvecRHS1D on the GPU
    resu = rk4a[s] * resu + dt * rhsu
    u = u + rk4b[s] * resu
  torch.cuda.synchronize()
  v = setup1d.from_elem_major(host(stage_in), N + 1)  # the last stage's input state
  uin = -np.sin(A * A * (t + rk4c[4] * dt))
  du = np.empty((2, K))
  du[0, :] = (v[0, :] - np.concatenate([[uin], v[-1, :-1]])) * (-A) / 2.0  # :126, :129
  du[1, :-1] = (v[-1, :-1] - v[0, 1:]) * A / 2.0
  du[1, -1] = 0.0  # :131 du(mapO) = 0
  np.testing.assert_allclose(du, by["du"][0], rtol=0, atol=atol)
  np.testing.assert_allclose(setup1d.from_elem_major(host(rhsu), N + 1), by["rhsu"][0],
                             rtol=0, atol=atol)
  np.testing.assert_allclose(setup1d.from_elem_major(host(resu), N + 1), by["resu"][0],
                             rtol=0, atol=atol)
  # the replayed step agrees with the fused kernel's own step 1341
  u_full = torch.tensor(setup1d.to_elem_major(u0), device=gpu)
  op.forward(u_full, 0.0, dt, nsteps)
  torch.cuda.synchronize()
  ref = host(u_full)
  assert np.max(np.abs(host(u) - ref)) <= 1e-12 * np.max(np.abs(ref))


def test_exact_tie_refines_the_first_copy(pkg, gpu):
  import torch
  N, K, nsteps = 4, 4096, 12
  Np = N + 1
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  S = setup1d.uniform_setup(N, K, metric="element")
  op = pkg.operators.DGAdvection1D(mesh)
  dt = mesh.cfl_dt()
  rng = np.random.default_rng(4)
  bump = rng.standard_normal((40, Np)) * np.hanning(40)[:, None]  # 40 elements, nodal
  k1, k2 = 1500, 2900  # > 5*nsteps elements from the inflow and from each other
  u0 = np.zeros((K, Np))
  u0[k1:k1 + 40] = bump
  u0[k2:k2 + 40] = bump  # the same bits
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(torch.tensor(u0.ravel(), device=gpu))
  op.forward(snaps[0], 0.0, dt, nsteps, snaps)
  eta = torch.full((K,), float("nan"), dtype=torch.float64, device=gpu)
  op.adjoint(snaps[nsteps], snaps, 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True)
  idx = op.argmax(eta, use_abs=True)
  e = host(eta)
  np.testing.assert_array_equal(e[k1 - 30:k1 + 70], e[k2 - 30:k2 + 70])  # an exact tie
  j = int(np.argmax(e[k1 - 30:k1 + 70]))
  assert idx == k1 - 30 + j == int(np.argmax(e))
  # the oracle on the same forward states: the same element up to its own rounding (numpy's
  # BLAS may order a column's sums by position, so its copies tie to ~1e-16, not always
  # bit for bit: then either copy is its answer)
  snaps2 = op.new_field(nsteps + 1)
  snaps2[0].copy_(torch.tensor(u0.ravel(), device=gpu))
  op.forward(snaps2[0], 0.0, dt, nsteps, snaps2)
  gs = [setup1d.from_elem_major(host(snaps2[n]), Np) for n in range(nsteps + 1)]
  times = [0.0]
  for _ in range(nsteps):
    times.append(times[-1] + dt)
  _, eta_ref, _ = oadj.adjoint_sweep(gs[-1], gs, times, dt, A, S)
  assert oadj.argmax(eta_ref, use_abs=True) in (idx, idx + (k2 - k1))
  np.testing.assert_allclose(e, np.abs(eta_ref), rtol=0, atol=1e-10 * np.max(e))
