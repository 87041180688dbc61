"""The config-3 kernels on overlapped waves (DG_TUNE_NL_EXCHANGE = 1, csrc/dg_burgers_ov.hip)
against the workgroup tiles (0, csrc/dg_burgers.hip): the same stage arithmetic (dg_nl.h) with
DPP wave shifts instead of LDS + barriers, so every output must be the SAME BITS -- forward
snapshots, the limiter's decision record, the adjoint w^0 and the indicator eta -- for every
physics, on uniform and refined meshes, for one and several trajectories, with troubled cells
(the jump IC) so the adjoint's wide-cone windows run.  The oracle parity of the config-3 path is
tests/test_gpu_nonlinear.py's (both exchanges); this file pins that switching the exchange
changes nothing.  Needs an MI355X.
"""
import numpy as np
import pytest

from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu

PHYSICS = [("burgers", True), ("burgers", False), ("linear", True), ("burgers", "1")]


def host(t):
  return t.detach().cpu().numpy()


def refined_vx(K, rng, splits=9):
  _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  for _ in range(splits):
    j = int(rng.integers(0, len(v_x) - 1))
    v_x = np.insert(v_x, j + 1, 0.5 * (v_x[j] + v_x[j + 1]))
  return v_x


def make_ic(x, rng, jump=0.8):
  return np.sin(2 * np.pi * x) + jump * (x > 0.5) + 0.05 * rng.standard_normal(x.shape)


def run_both(pkg, gpu, N, v_x, flux, limit, batch, nsteps, src=0.4, with_decisions=True):
  """Forward (snapshots + decisions) and adjoint (w, eta) under both exchanges."""
  import torch
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  S = setup1d.startup1d(N, v_x, metric="element")
  K = S["K"]
  rng = np.random.default_rng(N * 7 + K + batch)
  u0 = np.concatenate([setup1d.to_elem_major(make_ic(S["x"], rng)) for _ in range(batch)])
  g = rng.standard_normal(u0.shape)
  dt = oadv.bench_dt(S)
  out = {}
  for ex in (0, 1):
    op = pkg.operators.DGAdvection1D(mesh, batch=batch, flux=flux, limiter=limit)
    op.tune(nl_exchange=ex)
    snaps = op.new_field(nsteps + 1)
    u = torch.tensor(u0, device=gpu)
    dec = (torch.zeros(nsteps * op.ktot, dtype=torch.int16, device=gpu)
           if (limit and with_decisions) else None)
    op.forward(u, 0.01, dt, nsteps, snaps, decisions=dec)
    w = torch.tensor(g, device=gpu)
    eta = torch.zeros(op.ktot, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.01, dt, nsteps, src_coef=src, eta=eta, decisions=dec)
    torch.cuda.synchronize()
    out[ex] = (host(snaps), None if dec is None else host(dec), host(w), host(eta), op.uniform)
  return out


def assert_same(out):
  (s0, d0, w0, e0, u0), (s1, d1, w1, e1, u1) = out[0], out[1]
  assert u0 == u1
  np.testing.assert_array_equal(s1, s0)
  if d0 is not None:
    np.testing.assert_array_equal(d1, d0)
  np.testing.assert_array_equal(w1, w0)
  np.testing.assert_array_equal(e1, e0)


@pytest.mark.parametrize("flux,limit", PHYSICS)
@pytest.mark.parametrize("N,K,uniform,batch", [(4, 700, True, 1), (4, 611, False, 1),
                                               (1, 333, True, 2), (2, 500, False, 1),
                                               (6, 257, True, 1), (8, 190, False, 2),
                                               (3, 45, True, 1)])
def test_exchange_is_bit_identical(pkg, gpu, flux, limit, N, K, uniform, batch):
  rng = np.random.default_rng(K)
  v_x = setup1d.mesh_gen1d(0.0, 1.0, K)[1] if uniform else refined_vx(K, rng)
  out = run_both(pkg, gpu, N, v_x, flux, limit, batch, nsteps=4)
  assert out[0][4] == uniform
  if limit:
    assert np.count_nonzero(out[0][1]) > 0  # troubled cells: the wide-cone windows ran
  assert_same(out)


def test_exchange_without_decision_record(pkg, gpu):
  """A limited adjoint without the decision record runs the workgroup tiles under either
  setting (the narrow cone needs the record); the forward still runs on overlapped waves."""
  rng = np.random.default_rng(5)
  out = run_both(pkg, gpu, 4, refined_vx(400, rng), "burgers", True, 1, nsteps=3,
                 with_decisions=False)
  assert_same(out)


@pytest.mark.slow
def test_exchange_bit_identical_at_config3_size(pkg, gpu):
  """BASELINE config 3 size through adaptive.AdaptiveSweep (the bench's calls: forward with
  the decision record, adjoint in place on u^N with eta assigned), N = 4, K = 2^22 + refined
  elements, 20 + 20 steps, a jump IC (troubled cells every step): both exchanges give the same
  bits for every snapshot, the record, w^0, eta and the refine index."""
  import torch
  N, K, nsteps = 4, 1 << 22, 20
  res = {}
  for ex in (0, 1):
    mesh = pkg.BaseGalerkin1D(n=N, k=K, domain=[0.0, 1.0])
    run = pkg.adaptive.AdaptiveSweep(mesh, nsteps, 8, flux="burgers", limiter=True)
    run.op.tune(nl_exchange=ex)
    for j in (K // 3, K // 3 + 1, 5, K - 2):  # non-uniform: the UNI = false kernels
      run.op.refine(torch.tensor([j], dtype=torch.int64, device=gpu))
    run.h_min = float(np.min(np.diff(run.op.v_x())))  # the CFL step on the refined mesh
    assert not run.op.uniform
    snaps = run.snapshots()
    r = torch.tensor(setup1d.jacobi_gl(0, 0, N), dtype=torch.float64, device=gpu)
    vx = torch.tensor(run.op.v_x(), dtype=torch.float64, device=gpu)
    xd = vx[:-1, None] + 0.5 * (r[None, :] + 1.0) * (vx[1:] - vx[:-1])[:, None]
    gen = torch.Generator(device=gpu).manual_seed(3)
    noise = torch.randn(xd.shape, generator=gen, dtype=torch.float64, device=gpu)
    snaps[0].copy_((torch.sin(2 * np.pi * xd) + 0.8 * (xd > 0.5) + 0.01 * noise).reshape(-1))
    dt = run.dt
    run.forward(dt, init=False)
    run.adjoint(dt)
    idx = run.op.argmax(run.eta(), use_abs=True)
    torch.cuda.synchronize()
    dec = run.decisions()
    res[ex] = dict(snaps=snaps.clone(), dec=dec.clone(), eta=run.eta().clone(), idx=idx)
    del run, snaps
    torch.cuda.empty_cache()
  a, b = res[0], res[1]
  assert int(torch.count_nonzero(a["dec"])) > 0
  assert torch.equal(a["dec"], b["dec"])
  assert torch.equal(a["snaps"], b["snaps"])
  assert torch.equal(a["eta"], b["eta"])
  assert a["idx"] == b["idx"]
