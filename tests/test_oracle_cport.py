"""The C restatement of the oracle's config-2 sweep (oracle/c/advec_oracle.c, bench.py's CPU
baseline) against the numpy oracle it restates: snapshots, w^0 and eta on the same inputs,
serial and threaded.  The two differ only in summation order (numpy's BLAS products vs the
C loops), so the bar is rounding: 1e-12 of each field's scale."""
import numpy as np
import pytest

from oracle import adjoint as oadj
from oracle import advec as oadv
from oracle import cport
from oracle import effectivity as oef
from oracle import setup1d

A = 2.0 * np.pi


@pytest.fixture(scope="module")
def built():
  cport.build()
  return cport.load()


def close(x, y, what):
  scale = max(np.max(np.abs(y)), 1e-300)
  err = np.max(np.abs(x - y)) / scale
  assert err <= 1e-12, (what, err)


@pytest.mark.parametrize("N,K,nsteps,threads,refined", [
    (4, 300, 10, 1, False),   # config 2's order
    (4, 257, 6, 4, False),    # threaded, odd K
    (1, 200, 8, 2, False),
    (7, 90, 5, 1, False),
    (3, 150, 7, 3, True),     # non-uniform mesh: per-element metric
])
def test_cport_equals_numpy_oracle(built, N, K, nsteps, threads, refined):
  rng = np.random.default_rng(N * 100 + K)
  if refined:
    vx = np.concatenate(([0.0], np.cumsum(rng.uniform(0.3, 1.7, K))))
    S = setup1d.startup1d(N, vx / vx[-1], metric="element")
  else:
    S = setup1d.uniform_setup(N, K, metric="element")
  dt = oadv.bench_dt(S)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
  snaps, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  w0, eta, _ = oadj.adjoint_sweep(snaps[-1], snaps, times, dt, A, S)

  mesh = cport.Mesh(S, A)
  csn, ctimes = cport.forward_sweep(setup1d.to_elem_major(u0), 0.0, dt, nsteps, mesh,
                                    threads=threads)
  assert ctimes == times
  for n in range(nsteps + 1):
    close(csn[n], setup1d.to_elem_major(snaps[n]), f"u^{n}")
  cw0, ceta = cport.adjoint_sweep(csn[-1], csn, ctimes, dt, mesh, threads=threads)
  close(cw0, setup1d.to_elem_major(w0), "w^0")
  close(ceta, eta, "eta")
  assert int(np.argmax(np.abs(ceta))) == int(np.argmax(np.abs(eta)))


def test_cport_threads_agree(built):
  """Every element's arithmetic is the same whatever the thread count: bit-identical."""
  S = setup1d.uniform_setup(4, 1000, metric="element")
  dt = oadv.bench_dt(S)
  mesh = cport.Mesh(S, A)
  u0 = setup1d.to_elem_major(np.sin(2 * np.pi * S["x"]))
  outs = []
  for th in (1, 3, 8):
    sn, tm = cport.forward_sweep(u0, 0.0, dt, 6, mesh, threads=th)
    outs.append((sn,) + cport.adjoint_sweep(sn[-1], sn, tm, dt, mesh, threads=th))
  for o in outs[1:]:
    for x, y in zip(o, outs[0]):
      np.testing.assert_array_equal(x, y)


def test_cport_rejects_a_nodal_metric(built):
  S = setup1d.uniform_setup(3, 40, metric="matlab")
  if np.all(S["rx"] == S["rx"][0:1, :]):
    pytest.skip("this mesh's nodal metric happens to be constant per element")
  with pytest.raises(ValueError):
    cport.Mesh(S, A)


@pytest.mark.parametrize("N,K,nsteps,threads", [(4, 200, 8, 1), (2, 150, 6, 3), (6, 80, 4, 2)])
def test_cport_p_estimate_equals_numpy_oracle(built, N, K, nsteps, threads):
  """The p-enriched estimate (order-(N+1) adjoint from P u^N, prolonged one-step residual)
  against oracle/effectivity.py p_estimate on the same order-N snapshots."""
  rng = np.random.default_rng(7 * N + K)
  S = setup1d.uniform_setup(N, K, metric="element")
  S_hi = setup1d.uniform_setup(N + 1, K, metric="element")
  dt = oadv.bench_dt(S)
  u0 = np.sin(2 * np.pi * S["x"]) + 0.1 * rng.standard_normal(S["x"].shape)
  snaps, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, A, S)
  P = oef.prolong_matrix(S, S_hi)
  eta, w0 = oef.p_estimate(snaps, times, dt, A, S, S_hi, P @ snaps[-1], inflow=oadv.INFLOW_A)
  esn = np.stack([setup1d.to_elem_major(u) for u in snaps])
  ceta, cw0 = cport.p_estimate(esn, times, dt, cport.Mesh(S_hi, A), P,
                               setup1d.to_elem_major(P @ snaps[-1]), N + 1, threads=threads)
  close(ceta, eta, "eta")
  close(cw0, setup1d.to_elem_major(w0), "w^0")
