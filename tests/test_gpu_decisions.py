"""The limiter's decision record (dg_lserk4_fwd_ex / dg_lserk4_adj_ex, config 3): the forward
records per element and step the 5 stages' decisions (troubled or not, SlopeLimitN.m:21-23,
and the active minmod argument, minmod.m:9-11); the adjoint reads them back instead of
re-testing every cell and skips the limiter work in stages where a tile has no troubled
cell.  Bars: the troubled bits equal the oracle's limited-cell sets stage by stage (exact);
the adjoint with the record is bit-identical to the adjoint without it."""
import numpy as np
import pytest

from oracle import advec as oadv
from oracle import burgers as ob
from oracle import setup1d

from test_gpu_nonlinear import A, dev, host, ic, refined_vx, setup

pytestmark = pytest.mark.gpu


def troubled_sets(code, K):
  """Per stage, the element indices whose record says troubled."""
  return [np.nonzero((code >> (3 * s)) & 4)[0] for s in range(5)]


@pytest.mark.parametrize("limit", [True, "1"])
@pytest.mark.parametrize("N,K,uniform", [(4, 300, True), (3, 240, False), (2, 1000, True)])
def test_record_matches_the_oracle_and_adjoint_is_unchanged(pkg, gpu, limit, N, K, uniform):
  import torch
  rng = np.random.default_rng(N * 7 + K)
  v_x = None if uniform else refined_vx(K, rng)
  S, mesh, op = setup(pkg, N, K, v_x=v_x, flux="burgers", limiter=limit)
  K = S["K"]
  u0 = ic(S, rng)
  dt = oadv.bench_dt(S)
  nsteps = 4
  snaps = op.new_field(nsteps + 1)
  rec = torch.full((nsteps * K,), -1, dtype=torch.int16, device=gpu)
  op.forward(dev(setup1d.to_elem_major(u0), gpu), 0.02, dt, nsteps, snaps, decisions=rec)
  codes = host(rec).astype(np.int64) & 0xFFFF
  times = [0.02]
  for _ in range(nsteps):
    times.append(times[-1] + dt)
  n_troubled = 0
  for n in range(nsteps):  # each step from the GPU's own state: the oracle's limited sets
    un = setup1d.from_elem_major(host(snaps[n]), N + 1)
    _, ids = ob.limited_step(un, times[n], dt, A, S, ob.FLUX_BURGERS, limit=limit,
                             return_ids=True)
    got = troubled_sets(codes[n * K:(n + 1) * K], K)
    for s in range(5):
      np.testing.assert_array_equal(got[s], np.sort(ids[s]), err_msg=f"step {n} stage {s}")
      n_troubled += len(ids[s])
  assert n_troubled > 0
  if limit == "1":
    assert all(len(troubled_sets(codes[:K], K)[s]) == K for s in range(5))
  # the adjoint with and without the record
  g = snaps[nsteps].clone()
  outs = []
  for d in (None, rec):
    w = g.clone()
    eta = torch.zeros(K, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.02, dt, nsteps, src_coef=0.4, eta=eta, decisions=d)
    outs.append((host(w), host(eta)))
  np.testing.assert_array_equal(outs[0][0], outs[1][0])
  np.testing.assert_array_equal(outs[0][1], outs[1][1])


def test_record_skips_quiet_tiles_exactly(pkg, gpu):
  """A large smooth run where almost every tile has no troubled cell (the config-3 bench
  regime): the record-driven adjoint still equals the re-testing adjoint bit for bit."""
  import torch
  N, K, nsteps = 4, 20000, 3
  S, mesh, op = setup(pkg, N, K, flux="burgers", limiter=True)
  dt = oadv.bench_dt(S)
  snaps = op.new_field(nsteps + 1)
  op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
  rec = torch.zeros(nsteps * K, dtype=torch.int16, device=gpu)
  op.forward(snaps[0], 0.0, dt, nsteps, snaps, decisions=rec)
  frac = float((host(rec) != 0).mean())
  assert 0 < frac < 0.01
  res = []
  for d in (None, rec):
    w = snaps[nsteps].clone()
    eta = torch.zeros(K, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.0, dt, nsteps, eta=eta, decisions=d)
    res.append((host(w), host(eta)))
  np.testing.assert_array_equal(res[0][0], res[1][0])
  np.testing.assert_array_equal(res[0][1], res[1][1])


def test_record_is_validated(pkg, gpu):
  import torch
  S, mesh, op = setup(pkg, 2, 50, flux="burgers", limiter=True)
  snaps = op.new_field(3)
  with pytest.raises(ValueError):
    op.forward(snaps[0], 0.0, 1e-4, 2, snaps,
               decisions=torch.zeros(50, dtype=torch.int16, device=gpu))
  with pytest.raises(TypeError):
    op.forward(snaps[0], 0.0, 1e-4, 2, snaps,
               decisions=torch.zeros(100, dtype=torch.int32, device=gpu))


@pytest.mark.parametrize("limit,N,K,uniform", [
    ("1", 2, 150000, True),     # every cell troubled: every tile on the wide cone
    (True, 4, 200000, False),   # a jump every 400 elements: wide and narrow tiles side by side
])
def test_troubled_tiles_on_the_wide_cone(pkg, gpu, limit, N, K, uniform):
  """The record-driven adjoint lays its tiles out for the narrow cone (no troubled cell) and
  lists the others for k_adj_nl_wide, which recomputes them as half tiles on the wide cone
  (grid-stride over the list, the list reset by its last workgroup for the next step).  With
  more listed tiles than the wide launch has workgroups, over several steps, the result
  equals the re-testing adjoint bit for bit."""
  import torch
  rng = np.random.default_rng(K)
  v_x = None if uniform else refined_vx(K, rng)
  S, mesh, op = setup(pkg, N, K, v_x=v_x, flux="burgers", limiter=limit)
  K = S["K"]
  dt = oadv.bench_dt(S)
  nsteps = 3
  x = S["x"]
  u0 = np.sin(2 * np.pi * x) + np.floor(x * (K / 400.0)) % 2
  snaps = op.new_field(nsteps + 1)
  rec = torch.zeros(nsteps * K, dtype=torch.int16, device=gpu)
  op.forward(dev(setup1d.to_elem_major(u0), gpu), 0.0, dt, nsteps, snaps, decisions=rec)
  te = 236  # k_adj_nl's narrow-cone tile outputs
  codes = host(rec).reshape(nsteps, K)
  for n in range(nsteps):
    tiles = np.zeros(-(-K // te), dtype=bool)
    lo = np.maximum(np.arange(len(tiles)) * te - 10, 0)
    for t in range(len(tiles)):
      tiles[t] = codes[n, lo[t]:t * te + te + 10].any()
    assert tiles.sum() > 256  # more (tile, half) items than 2 x CUs
    if limit is True:
      assert not tiles.all()
  res = []
  for d in (None, rec):
    w = snaps[nsteps].clone()
    eta = torch.zeros(K, dtype=torch.float64, device=gpu)
    op.adjoint(w, snaps, 0.0, dt, nsteps, src_coef=0.3, eta=eta, decisions=d)
    res.append((host(w), host(eta)))
  np.testing.assert_array_equal(res[0][0], res[1][0])
  np.testing.assert_array_equal(res[0][1], res[1][1])
