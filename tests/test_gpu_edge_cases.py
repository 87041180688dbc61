"""Edge cases of the HIP path vs the oracle, through the C ABI.  Needs an MI355X.

Tiny meshes (K smaller than one tile's halo, down to a single element), batches of tiny
trajectories (one tile holding many trajectory ends), sweeps split over every launch
shape (8 steps per launch down to 1), and the empty sweep.  Tolerance as in
test_gpu_parity.py: fp64 within 1e-10 of max|oracle|.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import burgers as ob
from oracle import setup1d

pytestmark = pytest.mark.gpu

RTOL = 1e-10
A = 2 * np.pi


def rel_err(x, ref):
  x, ref = np.asarray(x), np.asarray(ref)
  return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-300))


def dev(x, device):
  import torch
  return torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=device)


def host(t):
  return t.detach().cpu().numpy()


@pytest.mark.parametrize("physics", ["linear", "burgers+limiter"])
@pytest.mark.parametrize("N", [1, 4])
@pytest.mark.parametrize("K,batch", [(2, 1), (2, 7), (3, 5), (21, 3), (40, 2)])
def test_tiny_meshes_and_batches(pkg, gpu, physics, N, K, batch):
  import torch
  rng = np.random.default_rng(1000 * N + 10 * K + batch)
  _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  S = setup1d.startup1d(N, v_x, metric="element")
  mesh = pkg.BaseGalerkin1D(n=N, v_x=v_x)
  nonlin = physics != "linear"
  kw = dict(flux="burgers", limiter=True) if nonlin else {}
  op = pkg.operators.DGAdvection1D(mesh, batch=batch, **kw)
  Np = N + 1
  u0s = [np.sin(2 * np.pi * (b + 1) * S["x"]) + 0.2 * rng.standard_normal(S["x"].shape)
         for b in range(batch)]
  gs = [rng.standard_normal(S["x"].shape) for _ in range(batch)]
  dt = 0.5 * oadv.bench_dt(S)
  nsteps, t0, src = 9, 0.03, 0.4
  u = dev(np.concatenate([setup1d.to_elem_major(x) for x in u0s]), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, t0, dt, nsteps, snaps)
  w = dev(np.concatenate([setup1d.to_elem_major(x) for x in gs]), gpu)
  eta = torch.zeros(batch * K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, t0, dt, nsteps, src_coef=src, eta=eta)
  field = K * Np
  for b in range(batch):
    sl = slice(b * field, (b + 1) * field)
    if nonlin:
      ref, times = ob.forward_sweep(u0s[b], t0, dt, nsteps, A, S)
    else:
      ref, times = oadv.forward_sweep(u0s[b], t0, dt, nsteps, A, S)
    gsn = [setup1d.from_elem_major(host(snaps[n])[sl], Np) for n in range(nsteps + 1)]
    for n in range(nsteps + 1):
      assert rel_err(gsn[n], ref[n]) <= RTOL, (b, n)
    if nonlin:
      w_ref, eta_ref, _ = ob.adjoint_sweep(gs[b], gsn, times, dt, A, S, src_coef=src)
    else:
      w_ref, eta_ref, _ = oadj.adjoint_sweep(gs[b], gsn, times, dt, A, S, src_coef=src)
    assert rel_err(setup1d.from_elem_major(host(w)[sl], Np), w_ref) <= RTOL, b
    assert rel_err(host(eta)[b * K:(b + 1) * K], eta_ref) <= RTOL, b


@pytest.mark.parametrize("steps_per_launch", [1, 2, 4, 8])
def test_every_launch_shape_gives_the_same_sweep(pkg, gpu, steps_per_launch):
  """A 13-step sweep chunked into launches of 8/4/2/1 fused steps (tile width 2 where the
  8-step shape needs it) equals the oracle; the adjoint likewise."""
  import torch
  N, K = 4, 3001
  _, v_x, _, _ = setup1d.mesh_gen1d(0.0, 1.0, K)
  S = setup1d.startup1d(N, v_x, metric="element")
  op = pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=N, v_x=v_x))
  op.tune(tile_width=2 if steps_per_launch == 8 else 1, steps_per_launch=steps_per_launch)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * np.cos(14 * np.pi * S["x"])
  dt, nsteps = oadv.bench_dt(S), 13
  ref, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  u = dev(setup1d.to_elem_major(u0), gpu)
  snaps = op.new_field(nsteps + 1)
  op.forward(u, 0.0, dt, nsteps, snaps)
  gsn = [setup1d.from_elem_major(host(snaps[n]), N + 1) for n in range(nsteps + 1)]
  for n in range(nsteps + 1):
    assert rel_err(gsn[n], ref[n]) <= RTOL, n
  g = np.cos(2 * np.pi * S["x"])
  w_ref, eta_ref, _ = oadj.adjoint_sweep(g, gsn, times, dt, A, S)
  w = dev(setup1d.to_elem_major(g), gpu)
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, 0.0, dt, nsteps, eta=eta)
  assert rel_err(setup1d.from_elem_major(host(w), N + 1), w_ref) <= RTOL
  assert rel_err(host(eta), eta_ref) <= RTOL


def test_single_element_mesh_is_refused(pkg, gpu):
  """K = 1 is outside the plan's contract (K >= 2): a clean DG_ERR_ARG, not a launch."""
  import ctypes
  lib = pkg._lib.load()
  bufs = [pkg._lib.dbl_array(np.zeros(16))[1] for _ in range(6)]
  out = ctypes.c_void_p()
  rc = lib.dg_plan_create(2, 1, 1, *bufs, 1.0, 0, 0, ctypes.byref(out))
  assert rc == pkg._lib.DG_ERR_ARG
  assert b"K >= 2" in lib.dg_last_error()


def test_empty_sweep_is_identity(pkg, gpu):
  """nsteps = 0: the forward leaves u (and snapshot 0 = u^0) and the adjoint leaves w."""
  import torch
  N, K = 3, 77
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  op = pkg.operators.DGAdvection1D(mesh)
  rng = np.random.default_rng(4)
  u0 = dev(rng.standard_normal(K * (N + 1)), gpu)
  u = u0.clone()
  snaps = op.new_field(1)
  op.forward(u, 0.0, 1e-3, 0, snaps)
  assert torch.equal(u, u0)
  assert torch.equal(snaps[0], u0)
  w0 = dev(rng.standard_normal(K * (N + 1)), gpu)
  w = w0.clone()
  eta = torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w, snaps, 0.0, 1e-3, 0, eta=eta)
  assert torch.equal(w, w0)
  assert not torch.any(eta)
