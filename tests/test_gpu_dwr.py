"""The p-enriched DWR error estimate on the GPU (dg_prolong / dg_lserk4_adj_p, SURVEY 8(a)
row 8) against its CPU statement ``oracle.effectivity.p_estimate`` and against the DWR
identity.  Needs an MI355X.

Reference pattern: matlab/MAIN.m:32-34 (adjoint marched at order Ns+1), adj_march.m:103-117
(err(k) = v_k'(-A uh_k - M~ + F)), python/Main_finite_difference.py:79-94 (errEst: the
adjoint-weighted one-step residual of the interpolated state, "the Adjoint-Weighted Residual
as an error estimate") and MAIN.m:55-76 (the effectivity printout).  The reference records no
advection outputs: parity is pinned by the oracle restatement plus the identity
sum_k eta_k = J_{N+1}(u_{N+1}) - J_{N+1}(P u_h), which holds exactly for the linear scheme and
a linear functional.

Inputs are identical on both sides: the oracle is fed the GPU's own order-N snapshots (the
residual is a difference of nearby states; the forward states are compared elsewhere,
tests/test_gpu_parity.py).  Tolerances (north_star: fp64 indicator within 1e-10 relative):
  eta, w^0:        max|gpu - oracle| <= 1e-10 * max|oracle|
  DWR identity:    |sum eta - (J_{N+1}(u_{N+1}) - J_{N+1}(P u_h))| <= 1e-9 * |J diff|
                   (both sides are GPU results; the difference itself is a cancellation of
                   two O(1) functionals, hence the looser bar)
"""
import json
import os

import numpy as np
import pytest

from oracle import advec as oadv
from oracle import effectivity as ef
from oracle import setup1d

pytestmark = pytest.mark.gpu

RTOL = 1e-10
A = 2 * np.pi
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel_err(x, ref):
  x, ref = np.asarray(x), np.asarray(ref)
  return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-300))


def dev(x, device):
  import torch
  return torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=device)


def host(t):
  return t.detach().cpu().numpy()


def times_of(t0, dt, nsteps):
  t = [t0]
  for _ in range(nsteps):
    t.append(t[-1] + dt)  # time = time + dt, One_code.mlx:139
  return t


def run_case(pkg, gpu, N, K, nsteps, inflow="a", v_x=None, batch=1, tile_width=None, spl=None,
             seed=0, t0=0.0, flags=()):
  """GPU forward (order N, snapshots) + GPU estimate; the oracle on the GPU's snapshots."""
  import torch
  ops = pkg.operators
  if v_x is None:
    v_x = np.linspace(0.0, 1.0, K + 1)
  S = setup1d.startup1d(N, v_x, metric="element")
  S_hi = setup1d.startup1d(N + 1, v_x, metric="element")
  rng = np.random.default_rng(seed)
  op = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), a=A, batch=batch, inflow=inflow)
  est = ops.DWREstimate(op, tile_width=tile_width, steps_per_launch=spl)
  dt = oadv.bench_dt(S)
  u0s = [np.sin(2 * np.pi * (b + 1) * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
         for b in range(batch)]
  ghs = [rng.standard_normal((N + 2, K)) for _ in range(batch)]
  u = dev(np.concatenate([setup1d.to_elem_major(x) for x in u0s]), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, t0, dt, nsteps, snaps)
  w = dev(np.concatenate([setup1d.to_elem_major(g) for g in ghs]), gpu)
  eta = torch.full((batch * K,), 7.0 if "assign" in flags else 0.0, dtype=torch.float64,
                   device=gpu)
  est.estimate(w, snaps, t0, dt, nsteps, eta=eta, eta_assign="assign" in flags,
               eta_abs="abs" in flags)
  torch.cuda.synchronize()
  times = times_of(t0, dt, nsteps)
  fl, fh = K * (N + 1), K * (N + 2)
  out = []
  for b in range(batch):
    gs = [setup1d.from_elem_major(host(snaps[n][b * fl:(b + 1) * fl]), N + 1)
          for n in range(nsteps + 1)]
    eta_ref, w0_ref = ef.p_estimate(gs, times, dt, A, S, S_hi, ghs[b], inflow)
    if "abs" in flags:
      eta_ref = np.abs(eta_ref)
    out.append((host(eta[b * K:(b + 1) * K]), eta_ref,
                setup1d.from_elem_major(host(w[b * fh:(b + 1) * fh]), N + 2), w0_ref))
  return out, est


def check(out):
  for b, (eta, eta_ref, w0, w0_ref) in enumerate(out):
    assert rel_err(eta, eta_ref) <= RTOL, (b, rel_err(eta, eta_ref))
    assert rel_err(w0, w0_ref) <= RTOL, (b, rel_err(w0, w0_ref))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 6, 7])
def test_estimate_matches_oracle(pkg, gpu, N):
  out, _ = run_case(pkg, gpu, N, 300, 7, seed=N)
  check(out)


@pytest.mark.parametrize("N,K,nsteps,batch", [(4, 1000, 8, 1), (3, 700, 12, 2), (2, 300, 20, 1)])
def test_estimate_dataflow_matches_oracle(pkg, gpu, N, K, nsteps, batch):
  """The default shape runs the estimate as ONE dataflow launch (k_adjp_flow) when the steps
  split into >= 2 blocks of 4: against the oracle directly (test_gpu_pflow.py: bit for bit
  against the launch chain)."""
  out, est = run_case(pkg, gpu, N, K, nsteps, batch=batch, seed=N + 40)
  assert est.query_flow(nsteps)
  check(out)


@pytest.mark.parametrize("inflow", ["a", "a2", "zero"])
def test_estimate_inflow_variants(pkg, gpu, inflow):
  out, _ = run_case(pkg, gpu, 4, 777, 5, inflow=inflow, t0=0.013)
  check(out)


def test_estimate_refined_mesh(pkg, gpu):
  rng = np.random.default_rng(11)
  v_x = np.concatenate(([0.0], np.cumsum(rng.uniform(0.3, 1.7, 400))))
  out, est = run_case(pkg, gpu, 3, 400, 6, v_x=v_x / v_x[-1], seed=3)
  assert not est.lo.uniform and not est.hi.uniform
  check(out)


def test_estimate_batch_with_trajectory_edges_inside_tiles(pkg, gpu):
  out, _ = run_case(pkg, gpu, 2, 333, 6, batch=3, seed=5)
  check(out)


def test_estimate_one_tile(pkg, gpu):
  out, _ = run_case(pkg, gpu, 4, 20, 9, seed=6)  # the whole mesh inside one (edge) tile
  check(out)


@pytest.mark.parametrize("tw,spl", [(1, 1), (1, 2), (1, 4), (2, 2), (2, 4), (2, 8)])
def test_estimate_launch_shapes(pkg, gpu, tw, spl):
  out, est = run_case(pkg, gpu, 4, 1000, 9, tile_width=tw, spl=spl, seed=7)
  assert (est.tile_width, est.steps_per_launch) == (tw, spl)
  check(out)


@pytest.mark.parametrize("flags", [("assign",), ("abs",), ("assign", "abs")])
def test_estimate_eta_flags(pkg, gpu, flags):
  out, _ = run_case(pkg, gpu, 4, 500, 6, seed=8, flags=flags)
  check(out)


def test_prolong_is_the_interpolation(pkg, gpu):
  ops = pkg.operators
  N, K = 3, 257
  v_x = np.linspace(0.0, 1.0, K + 1)
  S, S_hi = setup1d.startup1d(N, v_x, "element"), setup1d.startup1d(N + 1, v_x, "element")
  est = ops.DWREstimate(ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), a=A))
  u = np.random.default_rng(1).standard_normal((N + 1, K))
  got = setup1d.from_elem_major(host(est.prolong(dev(setup1d.to_elem_major(u), gpu))), N + 2)
  assert rel_err(got, ef.prolong_matrix(S, S_hi) @ u) <= 1e-14
  # a polynomial of degree N is reproduced exactly at the new nodes
  assert rel_err(setup1d.from_elem_major(host(est.prolong(dev(setup1d.to_elem_major(
      S["x"] ** 3), gpu))), N + 2), S_hi["x"] ** 3) <= 1e-13


def test_empty_sweep_assign_zeroes_eta(pkg, gpu):
  import torch
  ops = pkg.operators
  op = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=2, k=50), a=A)
  est = ops.DWREstimate(op)
  snaps = op.new_field(1).normal_()
  w = est.new_field().normal_()
  w_before = w.clone()
  eta = torch.ones(50, dtype=torch.float64, device=gpu)
  est.estimate(w, snaps, 0.0, 1e-3, 0, eta=eta, eta_assign=True)
  torch.cuda.synchronize()
  assert torch.equal(w, w_before) and not eta.any()


def test_mismatched_plans_are_refused(pkg, gpu):
  import ctypes
  ops = pkg.operators
  lib = pkg._lib
  lo = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=2, k=40), a=A)
  wrong = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=3, k=41), a=A)  # order N+1, other mesh
  P, Pp = lib.dbl_array(np.eye(4, 3))
  snaps = lo.new_field(2)
  w = wrong.new_field()
  rc = lo._lib.dg_lserk4_adj_p(lo._plan, wrong._plan, Pp, ctypes.c_void_p(w.data_ptr()),
                               ctypes.c_void_p(snaps.data_ptr()), 0.0, 1e-3, 1, None, 0, None)
  assert rc == lib.DG_ERR_ARG and b"K or batch" in lo._lib.dg_last_error()
  with pytest.raises(ValueError):
    ops.DWREstimate(ops.DGAdvection1D(pkg.BaseGalerkin1D(n=8, k=40), a=A))
  with pytest.raises(ValueError):
    ops.DWREstimate(ops.DGAdvection1D(pkg.BaseGalerkin1D(n=2, k=40), a=A, flux="burgers"))


# ---------------------------------------------------------------------------
# The estimate on the effectivity problem: a bump carried by a = 2 pi with
# zero inflow (exact solution u0(x - a t)), J(u) = int psi u(x, T), psi a cos^4 window.
def bump(x):
  return np.exp(-300.0 * (x - 0.3) ** 2)


def gpu_study(pkg, gpu, N, K, T=0.05, gains=True):
  """oracle.effectivity.study with every solve on the GPU (same dt rule, same functional):
  the jump indicator (dg_lserk4_adj), the p-estimate (dg_lserk4_adj_p), J_{N+1}(u_{N+1}) by the
  order-(N+1) plan's forward from P u^0, and the split-one-element gains."""
  import torch
  ops = pkg.operators
  VX = np.linspace(0.0, 1.0, K + 1)
  S = setup1d.startup1d(N, VX, metric="element")
  S_hi = setup1d.startup1d(N + 1, VX, metric="element")
  gap = min(np.min(np.diff(S_hi["r"])), np.min(np.diff(S["r"])))
  dt = 0.5 * 0.75 / A * (0.5 / K) * gap / 2  # the oracle study's rule (split element, N+1)
  nsteps = int(np.ceil(T / dt))
  dt = T / nsteps

  def solve(vx):
    Sx = setup1d.startup1d(N, vx, metric="element")
    opx = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=vx), a=A, inflow="zero")
    snaps = opx.new_field(nsteps + 1)
    opx.forward(dev(setup1d.to_elem_major(bump(Sx["x"])), gpu), 0.0, dt, nsteps, snaps)
    g = dev(setup1d.to_elem_major(ef.weight(Sx)), gpu)
    return opx, snaps, g, float(torch.dot(g, snaps[nsteps]))

  op, snaps, g_lo, J_h = solve(VX)
  eta_j = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(g_lo.clone(), snaps, 0.0, dt, nsteps, eta=eta_j)
  est = ops.DWREstimate(op)
  g_hi = dev(setup1d.to_elem_major(ef.weight(S_hi)), gpu)
  eta_p = torch.zeros(K, dtype=torch.float64, device=gpu)
  est.estimate(g_hi.clone(), snaps, 0.0, dt, nsteps, eta=eta_p)
  u_hi = est.prolong(snaps[0])
  est.hi.forward(u_hi, 0.0, dt, nsteps)
  J_p1 = float(torch.dot(g_hi, u_hi))
  J_Puh = float(torch.dot(g_hi, est.prolong(snaps[nsteps])))
  out = dict(N=N, K=K, nsteps=nsteps, dt=dt, J_h=J_h, J_p1=J_p1, J_Puh=J_Puh,
             err_p1=J_p1 - J_h, sum_eta_jump=float(eta_j.sum()), sum_eta_p=float(eta_p.sum()),
             eta_jump=host(eta_j), eta_p=host(eta_p), snaps=snaps)
  out["effectivity_p_vs_p1"] = out["sum_eta_p"] / out["err_p1"]
  if gains:
    gain = np.array([abs(solve(ef.split_mesh(VX, k))[3] - J_h) for k in range(K)])
    out["gain"] = gain
    for name in ("jump", "p"):
      eta = out["eta_" + name]
      out["spearman_" + name] = ef.spearman(np.abs(eta), gain)
      out["argmax_" + name] = int(np.argmax(np.abs(eta)))
    out["argmax_gain"] = int(np.argmax(gain))
  return out


@pytest.mark.parametrize("N,K", [(2, 16), (4, 16)])
def test_dwr_identity_on_the_gpu(pkg, gpu, N, K):
  """sum_k eta_p = J_{N+1}(u_{N+1}) - J_{N+1}(P u_h), every term computed on the GPU."""
  o = gpu_study(pkg, gpu, N, K, gains=False)
  diff = o["J_p1"] - o["J_Puh"]
  assert abs(o["sum_eta_p"] - diff) <= 1e-9 * abs(diff), (o["sum_eta_p"], diff)
  # J_{N+1}(P u_h) is J_h(u_h) (the window integral of the same polynomial) to quadrature
  # rounding, so the estimate is the reference's effectivity quantity J(u_H) - J(u_h)
  assert abs(o["J_Puh"] - o["J_h"]) <= 1e-12 * abs(o["J_h"])


@pytest.mark.parametrize("N,K", [(1, 16), (2, 16), (2, 32), (4, 16)])
def test_effectivity_table_on_the_gpu(pkg, gpu, N, K):
  """DESIGN.md §6c's CPU table (profiles/r02/effectivity.json, oracle/effectivity.study)
  reproduced with GPU solves: the p-estimate's effectivity against the enriched error, the
  indicator sums, the Spearman rank agreement with the split-one-element gains and the
  argmax of each indicator."""
  with open(os.path.join(ROOT, "profiles", "r02", "effectivity.json")) as f:
    rows = {(r["N"], r["K"]): r for r in json.load(f)["rows"]}
  ref = rows[(N, K)]
  o = gpu_study(pkg, gpu, N, K)
  print(f"[effectivity gpu] N={N} K={K}: sum eta_p / (J_p1 - J_h) = "
        f"{o['effectivity_p_vs_p1']:.12f}; sum eta_jump {o['sum_eta_jump']:.4e} (cpu "
        f"{ref['sum_eta_jump']:.4e}); Spearman jump {o['spearman_jump']:.3f} p "
        f"{o['spearman_p']:.3f}; argmax jump/p/gain {o['argmax_jump']}/{o['argmax_p']}/"
        f"{o['argmax_gain']}")
  assert abs(o["effectivity_p_vs_p1"] - 1.0) <= 1e-8
  assert o["nsteps"] == ref["nsteps"]
  for key in ("sum_eta_jump", "sum_eta_p", "err_p1"):
    assert abs(o[key] - ref[key]) <= 1e-8 * abs(ref[key]), key
  # the gains of elements the bump never reaches are rounding noise whose order may differ
  # between the GPU's and the CPU's arithmetic: the rank correlation agrees to that noise
  for key in ("spearman_jump", "spearman_p"):
    assert abs(o[key] - ref[key]) <= 0.02, key
  for key in ("argmax_jump", "argmax_p", "argmax_gain"):
    assert o[key] == ref[key], key


@pytest.mark.slow
def test_full_size_p_estimate(pkg, gpu):
  """The p sweep at config 2's size (N = 4, K = 2^20) through the path the
  bench times: ONE dataflow launch of the order-N snapshot forward, the estimate with the
  terminal weight P u^N and the refine decision (dg_lserk4_sweep_p, 8 steps = 2 + 2 blocks),
  against oracle.effectivity.p_estimate on the launch's own snapshots -- the whole mesh --
  for eta and w^0 at 1e-10 of max|oracle|, and the fused refine index against numpy's
  argmax of the oracle's |eta|.  The terminal weight handed to the oracle is dg_prolong of
  snapshot N (bit-identical to the in-launch one: test_terminal_prolong_equals_prolong_first).
  The IC is a sine plus per-node noise so the residual is resolved."""
  import torch
  ops = pkg.operators
  N, K, nsteps = 4, 1 << 20, 8
  v_x = np.linspace(0.0, 1.0, K + 1)
  S = setup1d.startup1d(N, v_x, metric="element")
  S_hi = setup1d.startup1d(N + 1, v_x, metric="element")
  op = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), a=A)
  est = ops.DWREstimate(op)
  assert (est.tile_width, est.steps_per_launch) == (2, 4)  # the default launch shape (round 5)
  assert est.query_sweep(nsteps)
  dt = oadv.bench_dt(S)
  rng = np.random.default_rng(21)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
  snaps = op.new_field(nsteps + 1)
  snaps[0].copy_(dev(setup1d.to_elem_major(u0), gpu))
  w = est.new_field()
  eta = torch.empty(K, dtype=torch.float64, device=gpu)
  res = torch.zeros(3, dtype=torch.int64, device=gpu)
  est.sweep(snaps, w, 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=False, idx=res[0:1],
            value=res[1:2].view(torch.float64), nonfinite=res[2:3])
  g = setup1d.from_elem_major(host(est.prolong(snaps[nsteps])), N + 2)
  torch.cuda.synchronize()
  gs = [setup1d.from_elem_major(host(snaps[n]), N + 1) for n in range(nsteps + 1)]
  eta_ref, w0_ref = ef.p_estimate(gs, times_of(0.0, dt, nsteps), dt, A, S, S_hi, g, "a")
  out = [(host(eta), eta_ref, setup1d.from_elem_major(host(w), N + 2), w0_ref)]
  check(out)
  a = np.sort(np.abs(eta_ref))
  assert a[-1] - a[-2] > 1e3 * RTOL * a[-1]
  assert int(host(res)[0]) == int(np.argmax(np.abs(eta_ref))) and int(host(res)[2]) == 0
  assert op.sweep_status() == 0


@pytest.mark.slow
def test_full_size_p_estimate_chain(pkg, gpu):
  """The estimate alone at config 2's size through the launch chain (4 steps: one block):
  dg_lserk4_adj_p from a seeded order-(N+1) terminal weight against the oracle, as round 4."""
  out, est = run_case(pkg, gpu, 4, 1 << 20, 4, seed=21)
  assert (est.tile_width, est.steps_per_launch) == (2, 4)  # the default launch shape (round 5)
  check(out)
  eta, eta_ref = out[0][0], out[0][1]
  a = np.sort(np.abs(eta_ref))
  assert a[-1] - a[-2] > 1e3 * RTOL * a[-1]
  assert int(np.argmax(np.abs(eta))) == int(np.argmax(np.abs(eta_ref)))


@pytest.mark.parametrize("N,tw,spl", [(4, None, None), (2, 2, 4), (3, 1, 2)])
def test_terminal_prolong_equals_prolong_first(pkg, gpu, N, tw, spl):
  """DG_ADJ_P_TERMINAL_PROLONG (the bench's J = |P u^N|^2 / 2): the first launch forms
  w = P u^N from the snapshot; w^0 and eta equal dg_prolong into w + the estimate bit for bit,
  also on a batch with trajectory edges inside tiles."""
  import torch
  ops = pkg.operators
  K, nsteps, batch = 700, 9, 2
  v_x = np.linspace(0.0, 1.0, K + 1)
  S = setup1d.startup1d(N, v_x, metric="element")
  op = ops.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x), a=A, batch=batch)
  est = ops.DWREstimate(op, tile_width=tw, steps_per_launch=spl)
  dt = oadv.bench_dt(S)
  rng = np.random.default_rng(N)
  u = dev(rng.standard_normal(batch * K * (N + 1)), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.0, dt, nsteps, snaps)
  w_ref = est.new_field()
  est.prolong(snaps[nsteps], out=w_ref)
  eta_ref = torch.empty(batch * K, dtype=torch.float64, device=gpu)
  est.estimate(w_ref, snaps, 0.0, dt, nsteps, eta=eta_ref, eta_assign=True, eta_abs=True)
  w = torch.full_like(w_ref, float("nan"))  # not read
  eta = torch.empty_like(eta_ref)
  est.estimate(w, snaps, 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True,
               terminal_prolong=True)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(host(w), host(w_ref))
  np.testing.assert_array_equal(host(eta), host(eta_ref))
