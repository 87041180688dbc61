"""Round-2 ABI additions, through ctypes on the GPU: the adjoint's indicator write flags
(dg_lserk4_adj_ex), the ensemble's per-IC magnitudes, dg_argmax_ex's device-side value and
non-finite count, and the dg_stream_copy bandwidth kernel.

Bars: the flags change no arithmetic, so flagged and unflagged sweeps agree bit for bit
(|x| of the same bits); argmax indices exact; the copy exact.
"""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import setup1d

pytestmark = pytest.mark.gpu


def host(t):
  return t.detach().cpu().numpy()


@pytest.mark.parametrize("physics", ["linear", "burgers_limited"])
def test_adjoint_eta_flags_are_bit_identical(pkg, gpu, physics):
  import torch
  N, K, nsteps = 4, 333, 7
  mesh = pkg.BaseGalerkin1D(n=N, k=K)
  kw = {} if physics == "linear" else dict(flux="burgers", limiter=True)
  op = pkg.operators.DGAdvection1D(mesh, **kw)
  dt = mesh.cfl_dt() * (1.0 if physics == "linear" else 0.5)
  snaps = op.new_field(nsteps + 1)
  op.init_sine([0.9], [2.0], [0.3], out=snaps[0])
  op.forward(snaps[0], 0.0, dt, nsteps, snaps)
  g = snaps[nsteps].clone()
  w0, eta0 = g.clone(), torch.zeros(K, dtype=torch.float64, device=gpu)
  op.adjoint(w0, snaps, 0.0, dt, nsteps, src_coef=0.3, eta=eta0)
  w1 = g.clone()
  eta1 = torch.full((K,), float("nan"), dtype=torch.float64, device=gpu)  # assign overwrites
  op.adjoint(w1, snaps, 0.0, dt, nsteps, src_coef=0.3, eta=eta1, eta_assign=True, eta_abs=True)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(host(w1), host(w0))
  np.testing.assert_array_equal(host(eta1), np.abs(host(eta0)))
  assert (host(eta0) < 0).any() and (host(eta0) > 0).any()  # both signs occur


def test_eta_assign_with_zero_steps_zeroes(pkg, gpu):
  import torch
  mesh = pkg.BaseGalerkin1D(n=3, k=64)
  op = pkg.operators.DGAdvection1D(mesh)
  snaps = op.new_field(1)
  op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
  eta = torch.full((64,), 7.0, dtype=torch.float64, device=gpu)
  op.adjoint(snaps[0].clone(), snaps, 0.0, 1e-3, 0, eta=eta, eta_assign=True)
  torch.cuda.synchronize()
  assert not host(eta).any()


@pytest.mark.parametrize("record", ["jumps", "snapshots"])
def test_ensemble_rows_are_per_ic_magnitudes(pkg, gpu, record):
  """EnsembleSweep rows = |signed eta| of each IC run alone (Main_width_ref.py:139), their
  rank partial = the IC-order sum of the magnitudes, and the refine index = argmax of the
  oracle's ensemble_indicator of the signed rows -- with either indicator record."""
  import torch
  K, ics, nsteps = 256, [1, 2, 5, 6], 8
  mesh = pkg.BaseGalerkin1D(n=4, k=K)
  dt = mesh.cfl_dt()
  sweep = pkg.ensemble.EnsembleSweep(mesh, ics, nsteps, dt, record=record)
  partial = sweep.run().clone()
  rows = host(sweep.per_ic())
  signed = []
  for j in ics:
    op = pkg.operators.DGAdvection1D(mesh)
    eta = torch.zeros(K, dtype=torch.float64, device=gpu)
    if record == "jumps":
      u0, w, rec = op.new_field(), op.new_field(), op.new_jumps(nsteps)
      op.init_sine(*pkg.ensemble.ic_params([j]), out=u0)
      op.forward_rec(u0, 0.0, dt, nsteps, rec, out=w)
      op.adjoint_rec(w, rec, 0.0, dt, nsteps, eta=eta)
    else:
      snaps = op.new_field(nsteps + 1)
      op.init_sine(*pkg.ensemble.ic_params([j]), out=snaps[0])
      op.forward(snaps[0], 0.0, dt, nsteps, snaps)
      op.adjoint(snaps[nsteps], snaps, 0.0, dt, nsteps, eta=eta)
    torch.cuda.synchronize()
    signed.append(host(eta))
  signed = np.array(signed)
  np.testing.assert_array_equal(rows, np.abs(signed))
  np.testing.assert_array_equal(host(partial), oadj.sum_rows(np.abs(signed)))
  mean, idx = pkg.ensemble.gather_indicator(partial, len(ics),
                                            pkg.ensemble.DeviceReducer(sweep.op))
  np.testing.assert_allclose(host(mean), oadj.ensemble_indicator(signed), rtol=1e-15)
  assert int(idx[0]) == oadj.argmax(oadj.ensemble_indicator(signed), use_abs=True)


def test_argmax_ex_value_and_nonfinite_count(pkg, gpu):
  import torch
  mesh = pkg.BaseGalerkin1D(n=2, k=5000)
  op = pkg.operators.DGAdvection1D(mesh)
  rng = np.random.default_rng(3)
  x = rng.standard_normal(5000)
  x[[17, 4000]] = -9.5  # tie in |x|: first index wins
  xd = torch.tensor(x, device=gpu)
  idx = torch.zeros(1, dtype=torch.int64, device=gpu)
  val = torch.zeros(1, dtype=torch.float64, device=gpu)
  bad = torch.zeros(1, dtype=torch.int64, device=gpu)
  op.argmax_ex(xd, idx, val, bad)
  torch.cuda.synchronize()
  assert int(idx) == 17 == oadj.argmax(x, use_abs=True)
  assert float(val) == 9.5 and int(bad) == 0
  op.argmax_ex(xd, idx, val, bad, use_abs=False)
  assert int(idx) == int(np.argmax(x)) and float(val) == x.max()
  for poison in (np.nan, np.inf, -np.inf):
    y = x.copy()
    y[2222] = poison
    op.argmax_ex(torch.tensor(y, device=gpu), idx, val, bad)
    torch.cuda.synchronize()
    assert int(idx) == 2222
  assert int(bad) == 3  # counted once per call that saw a non-finite winner


@pytest.mark.parametrize("n", [1, 2, 1001, (1 << 22) + 3])
def test_stream_copy_is_exact(pkg, gpu, n):
  import torch
  src = torch.randn(n, dtype=torch.float64, device=gpu)
  dst = torch.zeros_like(src)
  pkg.operators.stream_copy(src, dst)
  torch.cuda.synchronize()
  assert torch.equal(src, dst)


def test_stream_copy_rejects_misaligned(pkg, gpu):
  import torch
  src = torch.randn(101, dtype=torch.float64, device=gpu)
  dst = torch.zeros(101, dtype=torch.float64, device=gpu)
  with pytest.raises(pkg._lib.DGLibraryError, match="aligned"):
    pkg.operators.stream_copy(src[1:], dst[1:])


@pytest.mark.parametrize("kind,n_total", [("rand", 3), ("tie", 4), ("nan", 3), ("signed", 1)])
def test_device_reducer_candidates_pick_the_full_argmax(pkg, gpu, kind, n_total):
  """DeviceReducer.candidate / finish (dg_slice_candidate, dg_candidates_argmax), the device
  half of ensemble.refine_decision: each of W ranks sums the W rows it received for its slice
  in rank order, divides by the IC count and takes its argmax candidate; the candidates,
  reduced in rank order, give the index and value of numpy's argmax of |mean| over the whole
  vector bit for bit (the collectives around them are covered on CPU by
  tests/test_dist_gloo.py).  K not a multiple of W: the last slice is short."""
  import torch
  K, W = 10007, 4
  mesh = pkg.BaseGalerkin1D(n=2, k=K)
  red = pkg.ensemble.DeviceReducer(pkg.operators.DGAdvection1D(mesh))
  rng = np.random.default_rng(11)
  parts = rng.standard_normal((W, K)) * 10.0 ** rng.integers(-3, 3, (W, K))
  if kind != "signed":
    parts = np.abs(parts)
  if kind == "tie":
    parts[:, [9000, 2600, 2500]] = [[7e6], [1e6], [5e5], [5e5]]  # equal maximal sums in slices 3, 1, 0
  elif kind == "nan":
    parts[2, 8000] = np.nan
    parts[:, 100] = 1e6
  total = oadj.sum_rows(parts)
  mean = total / n_total if n_total != 1 else total
  chunk = -(-K // W)
  padded = np.zeros((W, W * chunk))
  padded[:, :K] = parts
  cands = []
  for r in range(W):
    recv = torch.tensor(np.ascontiguousarray(padded[:, r * chunk:(r + 1) * chunk]), device=gpu)
    n = min(chunk, K - r * chunk)
    cands.append(red.candidate(recv, n, float(n_total), r * chunk))
  out = red.finish(torch.stack(cands))
  torch.cuda.synchronize()
  want = oadj.argmax(mean, use_abs=True)
  assert int(out[0]) == int(red.idx[0]) == want
  np.testing.assert_array_equal(host(red.value), np.abs(mean[want:want + 1]))
  assert int(red.nonfinite[0]) == (1 if kind == "nan" else 0)
  if kind == "tie":
    assert want == 2500


@pytest.mark.parametrize("use_abs", [0, 1])
def test_argmax_winner_past_the_first_grid_stride_pass(pkg, gpu, use_abs):
  """k_argmax_partial's threads each see several elements (grid-stride loop): winners placed
  in the last pass, among all-negative values (use_abs = 0: no |.| to lift them above the
  start value), with a -inf and a tie, are found with numpy's index and value.  Guards the
  loop form ROCm 7.2 miscompiled in k_slice_partial (profiles/probes/argmax_phi_copy.hip)."""
  import torch
  n = 300007  # ~ 293 partial blocks of 256 threads: 4 passes per thread
  mesh = pkg.BaseGalerkin1D(n=2, k=n)
  op = pkg.operators.DGAdvection1D(mesh)
  rng = np.random.default_rng(3)
  x = -1.0 - rng.random(n)  # all negative
  if not use_abs:
    x[17] = -np.inf  # the weakest value there is: it must still lose to every other
  for where in (n - 1, n - 300, 250000, 1024 * 7 + 5):
    y = x.copy()
    y[where] = -50.0 if use_abs else -0.5  # the maximum of |y| / of y
    y[where + 1 if where + 1 < n else where - 1] = y[where]  # a tie: the lower index wins
    want = int(np.argmax(np.abs(y) if use_abs else y))
    assert want <= where
    t = torch.tensor(y, device=gpu)
    idx = torch.zeros(1, dtype=torch.int64, device=gpu)
    val = torch.zeros(1, dtype=torch.float64, device=gpu)
    op.argmax_ex(t, idx, val, use_abs=bool(use_abs))
    torch.cuda.synchronize()
    assert int(idx.item()) == want, (where, int(idx.item()), want)
    ref = abs(y[want]) if use_abs else y[want]
    assert float(val.item()) == ref


@pytest.mark.parametrize("rows,divisor", [(1, 3.0), (4, 3.0), (4, 6.0), (2, 1.0)])
def test_slice_candidate_winner_past_the_first_pass(pkg, gpu, rows, divisor):
  """dg_slice_candidate (rank-order row sum, division, argmax of |m|) with the winner in the
  last grid-stride pass and divisors whose reciprocal is inexact: index and value bits of
  numpy's argmax of |sum / divisor| (true division)."""
  import torch
  n, ld = 200003, 200011
  mesh = pkg.BaseGalerkin1D(n=2, k=n)
  red = pkg.ensemble.DeviceReducer(pkg.operators.DGAdvection1D(mesh))
  rng = np.random.default_rng(rows * 7 + int(divisor))
  x = rng.random((rows, ld))
  x[:, n - 2] = 5.0  # beyond every thread's first pass
  m = oadj.sum_rows(x[:, :n]) / divisor
  want = int(np.argmax(np.abs(m)))
  assert want == n - 2
  c = red.candidate(torch.tensor(x, device=gpu), n, divisor, 100)
  torch.cuda.synchronize()
  c = host(c)
  assert int(c[1]) == want + 100
  assert c[0:1].view(np.float64)[0] == np.abs(m[want])


@pytest.mark.parametrize("n_total", [3, 6, 12])
def test_gather_indicator_divides_like_the_candidate_kernel(pkg, gpu, n_total):
  """refine_decision (dg_slice_candidate: true division on the device) and gather_indicator
  (torch division of the summed indicator) give the same index and value bit for bit on the
  GPU for IC counts whose reciprocal is inexact (a Python-float divisor would make PyTorch
  multiply by the reciprocal, one ulp away), and the mean equals numpy's total / n."""
  import torch
  K = 40009
  mesh = pkg.BaseGalerkin1D(n=2, k=K)
  red = pkg.ensemble.DeviceReducer(pkg.operators.DGAdvection1D(mesh))
  rng = np.random.default_rng(n_total)
  total = rng.random(K) * 10.0 ** rng.integers(-3, 3, K)
  t = torch.tensor(total, device=gpu)
  mean, idx = pkg.ensemble.gather_indicator(t, n_total, red)
  torch.cuda.synchronize()
  np.testing.assert_array_equal(host(mean), total / float(n_total))
  i_g, v_g = int(idx.item()), host(red.value)[0]
  c = red.candidate(t.view(1, K), K, float(n_total), 0)
  red.finish(c.view(1, 2))
  torch.cuda.synchronize()
  assert int(red.idx.item()) == i_g
  assert host(red.value)[0] == v_g
