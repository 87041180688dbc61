"""Benchmark: DOF-updates/s of the 1D DG advection forward + adjoint sweep (BASELINE.json).

One bench step = one forward sweep of --nsteps fused LSERK4 steps (recording for the
indicator the two face jumps per element and step, or with --record snapshots the states),
one adjoint sweep of --nsteps reverse steps writing each trajectory's dual-weighted
residual magnitude |eta| (DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS: no zero fill, no extra pass),
the per-rank indicator reduction, the cross-rank rank-ordered sum (all-to-all + all-gather)
+ argmax (the refine decision, its value and a running non-finite count, all on the device),
and the refine index + value copied to the host.

Workload per rank = BASELINE config 2 (N=4, K=1,048,576, fp64, uniform mesh on [0,1],
a = 2*pi, dt from One_code.mlx:111-112).  Rank 0 runs u0 = sin(2 pi x) (the golden IC);
rank j > 0 runs IC j of the synthetic ensemble.  N GPUs = an ensemble of N
trajectories, one per GPU (weak scaling; the only exchange is the indicator sum).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--nsteps S] [--no-cpu-baseline]
  python bench.py --K 65536 --ics 1024   BASELINE config 4 (ensemble sharded over ranks,
                                         strong scaling)
  python bench.py --config 3             BASELINE config 3: Burgers-type flux + SlopeLimitN after
                                         every stage, K = 4,194,304, one refine iteration per step
                                         (fwd + adj + argmax + device split; replicas per GPU)
  python bench.py --N n                  BASELINE config 5 (polynomial-order sweep)
  python bench.py --indicator p          the p-enriched DWR error estimate (SURVEY 8(a) row 8:
                                         order-(N+1) adjoint + one-step residual of the
                                         prolonged snapshots, dg_lserk4_adj_p) instead of the
                                         jump indicator; forward with snapshots

Multi-GPU: `--gpus N` without a launcher spawns N ranks itself (one process per GPU, before
this process touches the GPU), each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1
in its environment; under torch.distributed.run (WORLD_SIZE already set) it runs as that rank.

Warm-up: at least --warmup steps, then more until the step time has converged (the GPU's
clock ramps over the first ~30-60 ms of load, profiles/r02/ramp.json); the count is reported
as `warmup_effective`.  The timed region is exactly --steps steps either way.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector spec peak (AMD data sheet; not in the guide)
# fp64 FMA probe on the box (profiles/probes/fp64_peak.hip, 8 waves/SIMD x 8 chains): the clock
# gives back ~18 % under a dense fp64 load
FP64_PROBE_TFLOPS = 64.6


EPS = float(np.finfo(np.float64).eps)


def eo_flops_per_update(Np, adjoint):
  """fp64 flops per DOF-update that the even/odd kernels execute for an interior element
  (per element-stage 4 + 5 Np + 4 NE NO forward; 6 + 5 Np + 4 NE NO reverse, plus
  the indicator's 2 Np + 2 per element-step), counted like the bytes: the algorithm, no halo."""
  NE, NO = (Np + 1) // 2, Np // 2
  if not adjoint:
    return 5.0 * (4 + 5 * Np + 4 * NE * NO) / Np
  return (5.0 * (6 + 5 * Np + 4 * NE * NO) + 2 * Np + 2) / Np


def horner_flops_per_update(Np, adjoint):
  """fp64 flops per DOF-update of the Horner-form record kernels (pair tiles, dg_rec_tiles.h;
  k_step_rp / k_adj_rp / k_sweep_rp) for an interior element of a uniform mesh, counted from
  the code (FMA = 2): per element-step the forward's five levels issue 5 (2 NE NO + Np) FMAs,
  4 Np multiplies and 21 adds, the adjoint's 5 (2 NE NO + Np) FMAs, 4 Np multiplies and 30
  adds plus the indicator's Np + 1 FMAs, a multiply and 3 adds -- at Np = 5 211 and 236 flops
  (126 and 145 instructions), against the stage loop's 265 / 287 (eo_flops_per_update).
  Checked against PMC: profiles/r03/sq/sq_summary_k_sweep_rp.json issues 10.87 GFLOP per
  20 + 20-step sweep at K = 2^20, = these counts x the tiles' halo factors (1.25 / 1.11)
  within 1.5 %."""
  NE, NO = (Np + 1) // 2, Np // 2
  if not adjoint:
    return (21.0 + 14.0 * Np + 20.0 * NE * NO) / Np
  return (36.0 + 16.0 * Np + 20.0 * NE * NO) / Np


def p_flops_per_update(Np):
  """fp64 flops per (order-N) DOF-update of k_adj_p (dg_dwr.hip) for an interior element: per
  element-step the prolongation (even/odd transform + the two blocks), the order-(N+1)
  forward step that recomputes S_{N+1}(P u^n), the residual pairing and the order-(N+1)
  reverse step -- divided by the Np order-N DOFs the step advances."""
  Nh = Np + 1
  NEl, NOl, NEh, NOh = (Np + 1) // 2, Np // 2, (Nh + 1) // 2, Nh // 2
  prolong = 4 * NOl + 2 * (NEh * NEl + NOh * NOl)
  fwd = 5.0 * (4 + 5 * Nh + 4 * NEh * NOh)
  rev = 5.0 * (6 + 5 * Nh + 4 * NEh * NOh)
  return (prolong + fwd + 3 * Nh + rev) / Np


def halo_factor(T, H):
  """Lanes issued per useful lane of a tile of T elements whose launch writes T - 2 H."""
  return T / float(T - 2 * H)
# Profiles of bench configurations (profiles/r06/collect.sh, profiles/r05/collect.sh): each
# directory holds the per-launch PMC traffic of the sweep kernel (pmc_traffic.json) and its SQ
# passes (sq_summary.json: issued fp64 instructions); a bench line uses the first whose N, K,
# shape and kernel (instantiation and occupancy target, `sweep_kernel`) match, else reports
# traffic null
PROFILE_DIRS = {
    "jumps": ([os.path.join(ROOT, "profiles", "r06", d) for d in ("headline", "N1")] +
              [os.path.join(ROOT, "profiles", "r05", d)
               for d in ("headline", "N1", "N2", "N6", "N8", "c4")]),
    "snapshots": [os.path.join(ROOT, "profiles", "r02")],
    "p": [os.path.join(ROOT, "profiles", d, "p") for d in ("r06", "r05")]}
PROFILE_TRAFFIC_FILE = {"snapshots": "pmc_traffic_snapshots.json"}  # default pmc_traffic.json


def parse(argv=None):
  p = argparse.ArgumentParser()
  p.add_argument("--gpus", type=int, default=1)
  p.add_argument("--steps", type=int, default=None,
                 help="timed steps (default 100; config 3: 10 refine iterations)")
  p.add_argument("--warmup", type=int, default=None,
                 help="untimed steps first, at least (default 10; config 3: 4); more follow "
                      "until the step time converges unless --no-converge")
  p.add_argument("--no-converge", action="store_true",
                 help="warm up exactly --warmup steps (no clock-ramp convergence)")
  p.add_argument("--converge-min-ms", type=float, default=200.0,
                 help="warm-up lasts at least this long (wall) before convergence is tested")
  p.add_argument("--N", type=int, default=4)
  p.add_argument("--config", type=int, default=2, choices=(2, 3),
                 help="2: linear advection (headline); 3: Burgers flux + limiter refine loop")
  p.add_argument("--K", type=int, default=None, help="elements (default 2^20; config 3: 2^22)")
  p.add_argument("--nsteps", type=int, default=20, help="time steps per sweep (each direction)")
  p.add_argument("--gather-ics", action="store_true",
                 help="also all-gather every IC's indicator row to every rank each step "
                      "(the per-IC training-data path; 512 MiB at config 4)")
  p.add_argument("--ics", type=int, default=0,
                 help="ensemble size over all ranks (config 4: --K 65536 --ics 1024); "
                      "default: one trajectory per rank (config 2 per GPU, weak scaling)")
  p.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                 help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo stages the "
                      "exchange through host memory: for tests with several ranks on one GPU)")
  p.add_argument("--record", default="jumps", choices=("jumps", "snapshots"),
                 help="what the forward sweep keeps for the indicator: the two face jumps per "
                      "element and step (dg_lserk4_fwd_rec, default) or full snapshots "
                      "(dg_lserk4_fwd); bit-identical at equal steps per launch, else equal to "
                      "the indicator's conditioning (~1e-9 relative on smooth solutions)")
  p.add_argument("--indicator", default="jump", choices=("jump", "p"),
                 help="jump: the lifted interelement-jump indicator paired with the order-N "
                      "adjoint (a refinement ranking, DESIGN.md 6c); p: the p-enriched DWR "
                      "error estimate (order-(N+1) adjoint x one-step residual of the prolonged "
                      "snapshots; implies --record snapshots)")
  p.add_argument("--no-cpu-baseline", action="store_true")
  p.add_argument("--no-margin", action="store_true",
                 help="skip the refine-decision margin check after the timed region (it re-runs "
                      "the sweep in another block shape: profiler passes use this so that every "
                      "dispatch they average has the timed shape)")
  p.add_argument("--cpu-steps", type=int, default=12, help="time steps of the CPU sample")
  p.add_argument("--graph", action="store_true",
                 help="replay each sweep as a captured HIP graph (measured 1-3%% slower than "
                      "eager launches on this path, profiles/r01/bench_eager_vs_graph.txt)")
  a = p.parse_args(argv)
  # Config 3 refines one element per step, so its step count is bounded by how often the
  # loop can split the same region before the element width reaches fp64 resolution.
  if a.steps is None:
    a.steps = 10 if a.config == 3 else 100
  if a.warmup is None:
    a.warmup = 4 if a.config == 3 else 10
  if a.indicator == "p":
    a.record = "snapshots"
  return a


# ---------------------------------------------------------------------------
# Multi-rank launch: one process per GPU (the reference's own multi-GPU pattern is one
# process per GPU from its launcher, python/Submit_schedule_frontera/
# Generating_argurment_files.py:23-36).  Nothing here touches the GPU.
# ---------------------------------------------------------------------------
def free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def spawn_ranks(nprocs, argv, script=None, env_extra=None, poll_s=0.2):
  """Run `script argv` as ranks 0..nprocs-1 (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set),
  rank 0's stdout passed through, the others' discarded (they print nothing), everyone's
  stderr passed through.  If a rank fails, the others are terminated (by handle).  Returns
  the first non-zero exit code, else 0."""
  script = script or os.path.abspath(__file__)
  port = free_port()
  procs = []
  for r in range(nprocs):
    env = dict(os.environ)
    env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nprocs),
                "LOCAL_WORLD_SIZE": str(nprocs), "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.update(env_extra or {})
    out = None if r == 0 else subprocess.DEVNULL
    procs.append(subprocess.Popen([sys.executable, script, *argv], env=env, stdout=out))
  rc = 0
  live = list(procs)
  while live:
    for p in list(live):
      code = p.poll()
      if code is None:
        continue
      live.remove(p)
      if code != 0 and rc == 0:
        rc = code
        for q in live:
          q.terminate()
    time.sleep(poll_s)
  for p in procs:
    p.wait()
  return rc


def stream_copy_gbs(dev, nbytes=1 << 30, reps=10):
  """Achievable HBM bandwidth on this box: the library's 16-byte-per-lane copy
  kernel (dg_stream_copy) over `nbytes` (read + write counted), median over `reps`, timed
  with HIP events on the stream it runs on."""
  import importlib

  import torch
  ops = importlib.import_module("adjoint-ode-adaptivity_amd.operators")
  src = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
  dst = torch.empty_like(src)
  st = torch.cuda.current_stream(dev)
  for _ in range(3):
    ops.stream_copy(src, dst)
  ts = []
  for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    ops.stream_copy(src, dst)
    e1.record(st)
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e-3)
  del src, dst
  return 2.0 * nbytes / float(np.median(ts)) / 1e9


BASELINE_METRIC = "DOF-updates/sec, 1D DG advection fwd+adjoint sweep, N=4, K=1e6"


def metric_name(N, K):
  """BASELINE.json's metric string for its own configuration (N = 4, K = 2^20); the same
  metric with the run's actual N and K otherwise (config 3, 4 and 5 lines)."""
  if N == 4 and K == 1 << 20:
    return BASELINE_METRIC
  return f"DOF-updates/sec, 1D DG advection fwd+adjoint sweep, N={N}, K={K}"


def cpu_baseline(N, K, nsteps, threads=1, indicator="jump", ics=1, ics_total=1):
  """The oracle (numpy restatement of utils/*.m + One_code.mlx, vectorised like MATLAB,
  `threads` BLAS/OpenMP threads) on a bounded sample of the same workload: `nsteps`
  forward + adjoint steps at the full N, K, for `ics` of the workload's `ics_total`
  trajectories (the oracle runs trajectories one after another, so its DOF-updates/s does
  not depend on how many are sampled).  SURVEY §8d asks for 1 and 8 threads; only the
  Dr/LIFT products are threaded by numpy, the elementwise passes stay serial.
  indicator "p": the oracle's p-estimate (order-(N+1) residual + adjoint) instead of the
  jump indicator."""
  from threadpoolctl import threadpool_limits

  from oracle import adjoint as oadj
  from oracle import advec as oadv
  from oracle import effectivity as oef
  from oracle import setup1d
  S = setup1d.uniform_setup(N, K, metric="element")
  S_hi = setup1d.uniform_setup(N + 1, K, metric="element") if indicator == "p" else None
  a = 2 * np.pi
  dt = oadv.bench_dt(S)
  with threadpool_limits(threads):
    t0 = time.perf_counter()
    for j in range(ics):
      u0 = np.sin(2 * np.pi * (j + 1) * S["x"])
      snaps, times = oadv.forward_sweep(u0, 0.0, dt, nsteps, a, S)
      if indicator == "p":
        P = oef.prolong_matrix(S, S_hi)
        oef.p_estimate(snaps, times, dt, a, S, S_hi, P @ snaps[-1], inflow=oadv.INFLOW_A)
      else:
        oadj.adjoint_sweep(snaps[-1], snaps, times, dt, a, S)
    el = time.perf_counter() - t0
  dofs = 2 * (N + 1) * K * nsteps * ics
  what = "p-enriched DWR estimate" if indicator == "p" else "DWR jump indicator"
  sample = (f"{nsteps} fwd + {nsteps} adj LSERK4 steps (with {what}) at N={N}, K={K}, "
            f"numpy oracle, {threads} thread(s), {el:.1f} s")
  if ics_total > 1:
    sample += (f"; {ics} of the workload's {ics_total} trajectories (the oracle's time is "
               f"linear in the trajectory count, so the rate stands for all of them)")
  return {"value": dofs / el, "unit": "DOF-updates/s", "cores": threads, "kind": "port",
          "sample": sample}


def cpu_baseline_cport(N, K, nsteps, threads, ics=1, ics_total=1, min_seconds=2.0,
                       indicator="jump"):
  """The oracle's C restatement (oracle/c/advec_oracle.c: the same LSERK4 forward + discrete
  adjoint + DWR jump indicator as the numpy oracle, element loops compiled with gcc -O3 and
  OpenMP, checked against it by tests/test_oracle_cport.py) over `nsteps` forward + adjoint
  steps at the full N, K on `threads` host threads: a CPU port as one would run it, beside
  the MATLAB-style numpy restatement.  None when its library is not built."""
  from oracle import advec as oadv
  from oracle import cport
  from oracle import setup1d
  try:
    cport.load()
  except OSError:
    return None
  S = setup1d.uniform_setup(N, K, metric="element")
  mesh = cport.Mesh(S, 2 * np.pi)
  pmode = indicator == "p"
  if pmode:  # the p-enriched estimate: order N+1 operators and the prolongation
    from oracle import effectivity as oef
    S_hi = setup1d.uniform_setup(N + 1, K, metric="element")
    mesh_hi = cport.Mesh(S_hi, 2 * np.pi)
    P = oef.prolong_matrix(S, S_hi)
  dt = oadv.bench_dt(S)
  u0 = setup1d.to_elem_major(np.sin(2 * np.pi * S["x"]))
  # untimed: one short sweep of the same kind on a small mesh (the first call of each entry
  # point costs ~0.3-0.6 s on its own: the OpenMP runtime and the library starting up)
  Kw = 256
  S_w = setup1d.uniform_setup(N, Kw, metric="element")
  m_w = cport.Mesh(S_w, 2 * np.pi)
  w_snaps, w_times = cport.forward_sweep(setup1d.to_elem_major(np.sin(S_w["x"])), 0.0, dt, 2,
                                         m_w, threads=threads)
  if pmode:
    S_wh = setup1d.uniform_setup(N + 1, Kw, metric="element")
    cport.p_estimate(w_snaps, w_times, dt, cport.Mesh(S_wh, 2 * np.pi), P,
                     np.zeros(Kw * (N + 2)), N + 1, threads=threads)
  else:
    cport.adjoint_sweep(w_snaps[-1], w_snaps, w_times, dt, m_w, threads=threads)
  # whole sweeps, at least three and until min_seconds have passed (a 16-thread sweep takes
  # ~0.3 s); the rate is the median sweep's (a first sweep can carry start-up costs)
  reps, el, laps = 0, 0.0, []
  while reps < 3 or el < min_seconds:
    t0 = time.perf_counter()
    snaps, times = cport.forward_sweep(u0, 0.0, dt, nsteps, mesh, threads=threads)
    if pmode:
      g_hi = (P @ snaps[-1].reshape(K, N + 1).T).T.ravel()  # P u^N, element-major
      cport.p_estimate(snaps, times, dt, mesh_hi, P, g_hi, N + 1, threads=threads)
    else:
      cport.adjoint_sweep(snaps[-1], snaps, times, dt, mesh, threads=threads)
    laps.append(time.perf_counter() - t0)
    el += laps[-1]
    reps += 1
    del snaps
  lap = float(np.median(laps))
  dofs = 2 * (N + 1) * K * nsteps
  what = "p-enriched DWR estimate" if pmode else "DWR jump indicator"
  sample = (f"median of {reps} sweeps of {nsteps} fwd + {nsteps} adj LSERK4 steps with {what} "
            f"at N={N}, K={K}, C port of the oracle (gcc -O3, OpenMP), {threads} thread(s), "
            f"{lap:.2f} s per sweep")
  if ics_total > 1:
    sample += (f"; 1 of the workload's {ics_total} trajectories (time is linear in the "
               f"trajectory count, so the rate stands for all of them)")
  return {"value": dofs / lap, "unit": "DOF-updates/s", "cores": threads, "kind": "port",
          "sample": sample}


def host_threads():
  """The host threads a CPU baseline may use: OMP_NUM_THREADS where set (16 on the GPU box),
  else the process's CPU affinity, at most 16."""
  env = os.environ.get("OMP_NUM_THREADS")
  if env and env.isdigit() and int(env) > 0:
    return int(env)
  try:
    n = len(os.sched_getaffinity(0))
  except (AttributeError, OSError):
    n = os.cpu_count() or 1
  return max(1, min(16, n))


def cpu_baseline_config3(N, K, nsteps):
  """The oracle's limited Burgers forward step (numpy, one thread) on a bounded sample of
  the config-3 workload.  Forward only: the oracle's adjoint is a coloured-Jacobian checker
  (~100 tangent sweeps per step), not a CPU port worth timing, so this baseline flatters
  the CPU by counting its forward rate for both directions."""
  from threadpoolctl import threadpool_limits

  from oracle import advec as oadv
  from oracle import burgers as ob
  from oracle import setup1d
  S = setup1d.uniform_setup(N, K, metric="element")
  a = 2 * np.pi
  dt = oadv.bench_dt(S)
  u0 = np.sin(2 * np.pi * S["x"])
  with threadpool_limits(1):
    t0 = time.perf_counter()
    ob.forward_sweep(u0, 0.0, dt, nsteps, a, S)
    el = time.perf_counter() - t0
  dofs = (N + 1) * K * nsteps
  return {"value": dofs / el, "unit": "DOF-updates/s", "cores": 1, "kind": "port",
          "sample": f"{nsteps} forward LSERK4 steps with SlopeLimitN per stage (Burgers flux) "
                    f"at N={N}, K={K}, numpy oracle, 1 thread, {el:.1f} s; forward rate "
                    f"stands for both directions"}


def warm_up(step, args, stream, max_steps, block=10):
  """--warmup steps, then blocks of `block` steps until (a) --converge-min-ms of wall time
  has passed and (b) the last block's device time is within 1 % of the previous block's and
  of the fastest block so far -- the GPU's clock ramps over the first tens of ms of load
  (profiles/r02/ramp.json) -- or `max_steps` is reached.  Returns (steps run, wall ms,
  last block ms per step)."""
  import torch
  t0 = time.perf_counter()
  n = 0
  for _ in range(args.warmup):
    step()
    n += 1
  if args.no_converge:
    torch.cuda.synchronize()
    return n, (time.perf_counter() - t0) * 1e3, None
  best = prev = None
  last = None
  while n + block <= max_steps:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(block):
      step()
    e1.record(stream)
    e1.synchronize()
    n += block
    last = e0.elapsed_time(e1) / block
    waited = (time.perf_counter() - t0) * 1e3 >= args.converge_min_ms
    if (waited and prev is not None and abs(last - prev) <= 0.01 * prev
        and last <= 1.01 * best):
      break
    best = last if best is None else min(best, last)
    prev = last
  return n, (time.perf_counter() - t0) * 1e3, last


def stats(xs):
  xs = np.asarray(xs, dtype=float)
  return {"first": float(xs[0]), "median": float(np.median(xs)), "last": float(xs[-1]),
          "min": float(xs.min()), "max": float(xs.max())}


def rank_device(backend, world, local, local_world, ndev):
  """This rank's GPU index and its process-group arguments (None for one rank).  RCCL (the
  torch "nccl" backend) runs one rank per GPU: the group is bound to this rank's device
  (device_id, so RCCL sets up its communicator eagerly on that GPU), and more ranks on a node
  than visible GPUs is refused here with a clear message -- RCCL itself would fail later with
  a duplicate-GPU error.  gloo (tests: several ranks sharing one GPU) maps ranks round-robin."""
  if ndev < 1:
    raise RuntimeError("bench.py needs a ROCm GPU")
  if world == 1:
    return local % ndev, None
  if backend == "nccl":
    if local_world > ndev or local >= ndev:
      raise RuntimeError(
          f"RCCL needs one GPU per rank: {local_world} ranks on this node but {ndev} GPU(s) "
          f"visible (local rank {local}); use --backend gloo to share a GPU between ranks")
    return local, {"backend": "nccl", "device_id": local}
  return local % ndev, {"backend": "gloo"}


def init_dist(args):
  import torch
  import torch.distributed as dist
  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
  idx, pg = rank_device(args.backend, world, local, local_world, torch.cuda.device_count())
  torch.cuda.set_device(idx)
  dev = torch.device("cuda", idx)
  if pg is not None:
    if "device_id" in pg:
      dist.init_process_group(pg["backend"], device_id=dev)
    else:
      dist.init_process_group(pg["backend"])
  return world, rank, dev


def ranks_agree(value, world, dev, backend):
  """All ranks' values (ints), gathered to every rank."""
  if world == 1:
    return [int(value)]
  import torch
  import torch.distributed as dist
  d = dev if backend == "nccl" else torch.device("cpu")
  mine = torch.tensor([int(value)], dtype=torch.int64, device=d)
  allv = torch.empty(world, dtype=torch.int64, device=d)
  dist.all_gather_into_tensor(allv, mine)
  return [int(v) for v in allv.cpu()]


def max_over_ranks(x, world, dev, backend):
  if world == 1:
    return float(x)
  import torch
  import torch.distributed as dist
  d = dev if backend == "nccl" else torch.device("cpu")
  t = torch.tensor([float(x)], dtype=torch.float64, device=d)
  dist.all_reduce(t, op=dist.ReduceOp.MAX)
  return float(t.item())


def sum_over_ranks(x, world, dev, backend):
  if world == 1:
    return float(x)
  import torch
  import torch.distributed as dist
  d = dev if backend == "nccl" else torch.device("cpu")
  t = torch.tensor([float(x)], dtype=torch.float64, device=d)
  dist.all_reduce(t)
  return float(t.item())


def barrier(world):
  if world > 1:
    import torch.distributed as dist
    dist.barrier()


def main_config3(args, world, rank, dev):
  """Config 3: one refine iteration per bench step on a trajectory of K elements (each
  rank an independent replica; no data-path collective)."""
  import importlib

  import torch
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  N, K, nsteps = args.N, args.K or (1 << 22), args.nsteps
  max_warm = args.warmup + 60
  mesh = pkg.BaseGalerkin1D(n=N, k=K, domain=[0.0, 1.0])
  run = pkg.adaptive.AdaptiveSweep(mesh, nsteps, max_warm + args.steps + 1,
                                   flux="burgers", limiter=True)
  stream = torch.cuda.current_stream(dev)
  warm, warm_ms, _ = warm_up(lambda: run.iterate(), args, stream, max_warm, block=4)
  torch.cuda.synchronize()
  barrier(world)
  torch.cuda.synchronize()
  evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
  total = 0
  t0 = time.perf_counter()
  for s in range(args.steps):
    dt = run.dt
    run.init_state()  # IC on the refined mesh and eta = 0, outside the kernel brackets
    evs[s][0].record(stream)
    run.forward(dt, init=False)
    evs[s][1].record(stream)
    evs[s][2].record(stream)
    run.adjoint(dt)
    evs[s][3].record(stream)
    total += run.refine()
    ref_idx = run.sync()
  torch.cuda.synchronize()
  barrier(world)
  torch.cuda.synchronize()
  elapsed = max_over_ranks(time.perf_counter() - t0, world, dev, args.backend)
  total = sum_over_ranks(total, world, dev, args.backend)
  Np = N + 1
  k_mid = K + warm + args.steps // 2
  # forward steps per launch with snapshots (dg_burgers.hip chunk_nl): 2 only when tuned to 2;
  # the exchange: workgroup tiles (k_step_nl / k_adj_nl + k_adj_nl_wide) or overlapped waves
  # (k_step_nlw / k_adj_nlw + k_adj_nlw_wide, DG_TUNE_NL_EXCHANGE)
  ms = run.op.nl_steps_per_launch[0]
  ow = run.op.nl_exchange == 1
  kf_name, ka_name = ("k_step_nlw", "k_adj_nlw") if ow else ("k_step_nl", "k_adj_nl")
  fwd_launches = (nsteps + ms - 1) // ms
  fwd_us = [e[0].elapsed_time(e[1]) * 1e3 / fwd_launches for e in evs]
  adj_us = [e[2].elapsed_time(e[3]) * 1e3 / nsteps for e in evs]
  fwd_m, adj_m = float(np.mean(fwd_us)), float(np.mean(adj_us))
  # Algorithmic bytes per launch: forward reads u^n once and writes ms snapshots; the
  # adjoint (one step per launch) reads w^{n+1} and u^n, writes w^n, updates eta.
  fwd_bytes = (8.0 + 8.0 * ms) * Np * k_mid
  adj_bytes = 24.0 * Np * k_mid + 16.0 * k_mid
  out = {
      "metric": metric_name(N, K),
      "value": total / elapsed,
      "unit": "DOF-updates/s",
      "n_gpus": world,
      "steps": args.steps,
      "warmup": args.warmup,
      "warmup_effective": warm,
      "warmup_ms": warm_ms,
      "ms_per_step": elapsed / args.steps * 1e3,
      "higher_is_better": True,
      "scaling": "weak",
      "vs_baseline": None,
      "dtype": "f64",
      "data": "synthetic (u0 = sin(2 pi x), re-initialised on the refined mesh every step)",
      "config": {"workload": (f"config 3: Burgers-type flux + SlopeLimitN after every LSERK4 "
                              f"stage, N={N}, K={K}+refinements, {nsteps}+{nsteps} steps/sweep "
                              f"+ DWR indicator + argmax + device element split per step"),
                 "N": N, "K": K, "nsteps_per_sweep": nsteps, "parallelism": f"replicas{world}"},
      "roofline": {"bound": "hbm", "achieved": adj_bytes / (adj_m * 1e-6) / 1e9,
                   "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": adj_bytes / (adj_m * 1e-6) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                   "kernel": (f"k_adj_nlw<{Np},burgers,limiter,nonuniform> (1 reverse step + "
                              f"stage recompute + DWR per launch on overlapped-wave windows, "
                              f"narrow cone; + k_adj_nlw_wide for windows with a troubled cell)"
                              if ow else
                              f"k_adj_nl<{Np},burgers,limiter,nonuniform> (1 reverse step + "
                              f"stage recompute + DWR per launch, tiles on the narrow cone; "
                              f"+ k_adj_nl_wide for tiles with a troubled cell)"),
                   "exchange": "overlapped waves (DPP)" if ow else "workgroup tiles (LDS)",
                   "launch_us": adj_m, "launch_us_stats": stats(adj_us),
                   "algorithmic_bytes": adj_bytes},
      "roofline_fwd": {"bound": "hbm", "achieved": fwd_bytes / (fwd_m * 1e-6) / 1e9,
                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": fwd_bytes / (fwd_m * 1e-6) / 1e9 / HBM_PEAK_GBS,
                       "kernel": (f"k_step_nlw<{Np},burgers,limiter,nonuniform>" if ow else
                                  f"k_step_nl<{Np},burgers,limiter,nonuniform,{ms}>"),
                       "launch_us": fwd_m, "launch_us_stats": stats(fwd_us),
                       "algorithmic_bytes": fwd_bytes},
      "refine_index": ref_idx,
      "refine_index_ranks": ranks_agree(ref_idx, world, dev, args.backend),
      "K_final": run.K,
  }
  # Counters from the committed config-3 profile (profiles/r03/collect_c3.sh: FETCH_SIZE /
  # WRITE_SIZE and SQ fp64 VALU passes of this bench), used when N and K match: HBM traffic
  # per launch, and the issued fp64 rate = the profile's issued flops per launch / this run's
  # launch time (every lane of a wave counted: halo lanes included).
  try:
    with open(os.path.join(ROOT, "profiles", "r06", "config3", "pmc.json")) as f:
      prof = json.load(f)
  except (OSError, ValueError):
    prof = None
  if prof and prof.get("N") == N and prof.get("K") == K:
    uni = "false"  # after its first split the refine loop's mesh is non-uniform
    pk = {k: v for k, v in prof["kernels"].items() if f", {uni}," in k or k.endswith(f", {uni}>")}
    ka = next((v for k, v in pk.items() if k.startswith(ka_name + "<")), None)
    kw = next((v for k, v in pk.items() if k.startswith(ka_name + "_wide<")), None)
    if ka and kw:  # one wide-cone pass per reverse step: count its bytes and flops with it
      ka = dict(ka)
      for key in ("hbm_bytes_per_launch", "fp64_flops_issued_per_launch"):
        if key in ka and key in kw:
          ka[key] += kw[key]
    kf = next((v for k, v in pk.items() if k.startswith(kf_name + "<")
               and (ow or k.endswith(f", {ms}>"))), None)
    src = prof.get("source")
    if ka and "hbm_bytes_per_launch" in ka:
      out["roofline"].update({"traffic": ka["hbm_bytes_per_launch"], "traffic_from_profile": True,
                              "traffic_source": src})
    if kf and "hbm_bytes_per_launch" in kf:
      out["roofline_fwd"].update({"traffic": kf["hbm_bytes_per_launch"],
                                  "traffic_from_profile": True})
    if ka and kf and "fp64_flops_issued_per_launch" in ka:
      at = ka["fp64_flops_issued_per_launch"] / (adj_m * 1e-6) / 1e12
      ft = kf["fp64_flops_issued_per_launch"] / (fwd_m * 1e-6) / 1e12
      out["roofline_fp64"] = {
          "bound": "fp64 vector", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
          "adj_issued": at, "adj_issued_frac": at / FP64_PEAK_TFLOPS,
          "fwd_issued": ft, "fwd_issued_frac": ft / FP64_PEAK_TFLOPS,
          "source": src,
          "what": "fp64 flops issued per launch (PMC: 64 lanes x (2 FMA + ADD + MUL) wave "
                  "instructions, halo lanes included) / this run's launch time"}
  if rank == 0 and world == 1 and not args.no_cpu_baseline:
    out["cpu_baseline"] = cpu_baseline_config3(N, K, 2)
  if rank == 0:
    print(json.dumps(out, allow_nan=False), flush=True)
  if world > 1:
    import torch.distributed as dist
    dist.destroy_process_group()


def sweep_chunks(nsteps, ms):
  """The library's greedy chunking of a sweep into launches of <= ms steps (dg_advec.hip
  chunk()): the steps of each launch."""
  chunks, left = [], nsteps
  while left > 0:
    m = ms
    while m > left:
      m //= 2
    left -= m
    chunks.append(m)
  return chunks


def launches_per_sweep(nsteps, ms):
  return len(sweep_chunks(nsteps, ms))


def refine_margin(sweep, step_fn):
  """Is this run's refine index decided by the indicator or by rounding?  The index is the
  argmax of |eta|; it is a real decision when the gap between the top two |eta| exceeds what
  rounding alone moves |eta| by.  That floor is measured, not modelled: the same sweep is run
  once more with the forward in a different block shape (same algorithm, states rounded at
  other steps -- 20-step vs 10-step forward blocks for the jump record, 4 vs 2 steps per
  launch for snapshots, for the p estimate a separate 2-step-launch forward and then the
  estimate instead of the sweep's 4-step forward blocks), and the floor is max |eta - eta_alt|.  Run after the timed region;
  the plan's shape is restored.  One trajectory per rank only (the headline); else None."""
  import torch
  if sweep.batch != 1:
    return None
  op = sweep.op
  with torch.no_grad():
    eta = sweep.eta.clone()
    a = eta.abs()
    top = torch.topk(a, 2)
    v1, v2 = float(top.values[0]), float(top.values[1])
    i1, i2 = int(top.indices[0]), int(top.indices[1])
    alt_fn = step_fn
    if sweep.record == "jumps":
      cur = op.rec_fwd_steps_per_launch
      alt = 10 if cur != 10 else 5
      op.tune(rec_fwd_steps_per_launch=alt)
      shape = (f"forward blocks of {alt} steps instead of {cur}"
               if sweep.nsteps % alt == 0 else None)
    elif sweep.est is not None:
      # the p estimate's sweep (dg_lserk4_sweep_p) runs its forward in 4-step blocks whatever
      # the plan's steps per launch: the alternate pass is a separate snapshot forward in
      # 2-step launches, then the estimate
      cur = op.steps_per_launch
      alt = 2
      op.tune(steps_per_launch=alt)
      shape = (f"a separate snapshot forward in launches of {alt} steps, then the estimate, "
               f"instead of the sweep's 4-step forward blocks")

      def alt_fn():
        sweep.forward()
        sweep.run_adjoint()
    else:
      cur = op.steps_per_launch
      alt = 2 if cur != 2 else 1
      op.tune(steps_per_launch=alt)
      shape = f"forward launches of {alt} steps instead of {cur}"
    alt_fn()
    torch.cuda.synchronize()
    eta_alt = sweep.eta.clone()
    if sweep.record == "jumps":
      op.tune(rec_fwd_steps_per_launch=cur)
    else:
      op.tune(steps_per_launch=cur)
    step_fn()
    torch.cuda.synchronize()
    floor = float((eta_alt - eta).abs().max())
    i_alt = int(eta_alt.abs().argmax())
  margin = v1 - v2
  return {"index": i1, "top1": v1, "top2": v2, "top2_index": i2, "margin": margin,
          "margin_rel": margin / v1 if v1 > 0 else 0.0,
          "rounding_floor": floor, "floor_rel": floor / v1 if v1 > 0 else 0.0,
          "floor_from": (f"max |eta - eta_alt| with the same sweep re-run with {shape} (the "
                         f"same algorithm, states rounded at other steps)"),
          "index_alt": i_alt,
          "decided": bool(margin > floor and i_alt == i1),
          "what": "refine index = argmax |eta|; decided when its margin over the runner-up "
                  "exceeds the measured rounding floor of |eta| and the re-run picks it too"}


def main(argv=None):
  args = parse(argv)
  if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
    # Self-launch: one rank per GPU, started before this process touches the GPU.
    sys.exit(spawn_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv)))
  import torch

  import importlib
  pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
  ens = pkg.ensemble

  world, rank, dev = init_dist(args)
  if args.gpus > 1 and world != args.gpus:
    raise RuntimeError(f"--gpus {args.gpus} but WORLD_SIZE = {world}")
  if args.config == 3:
    return main_config3(args, world, rank, dev)

  N, K, nsteps = args.N, args.K or (1 << 20), args.nsteps
  mesh = pkg.BaseGalerkin1D(n=N, k=K, domain=[0.0, 1.0])
  dt = mesh.cfl_dt()
  if args.ics > 0:  # config 4: the ensemble is sharded over the ranks (strong scaling)
    ics = list(ens.shard(args.ics, rank, world))
    params = ens.ic_params(ics)
    n_total = args.ics
  else:  # one trajectory per rank (weak scaling); rank 0 runs the golden IC
    ics = [rank]
    params = ((np.array([1.0]), np.array([1.0]), np.array([0.0])) if rank == 0
              else ens.ic_params([rank]))
    n_total = world
  sweep = ens.EnsembleSweep(mesh, ics, nsteps, dt, params=params, record=args.record,
                            indicator=args.indicator)
  reducer = ens.DeviceReducer(sweep.op)  # argmax + value + non-finite count on the device
  if args.graph:
    sweep.capture()  # each sweep becomes one HIP graph launch
  stream = torch.cuda.current_stream(dev)
  res_host = torch.zeros(2, dtype=torch.int64).pin_memory()  # refine index, value bits
  # The jump record's sweep as ONE dataflow launch (dg_lserk4_sweep_rec, csrc/dg_sweep.hip)
  # where the plan's shape allows: forward and adjoint are then not separately timeable.  With
  # one trajectory on one rank the indicator is the whole mean, so the refine decision is
  # reduced inside the same launch (dg_lserk4_sweep_refine).
  dataflow = sweep.dataflow
  # the p-estimate as ONE dataflow launch (dg_lserk4_adj_p, k_adjp_flow) after the snapshot
  # forward's launches; with one trajectory on one rank its last block reduces the refine
  # decision too (dg_lserk4_adj_p_refine)
  pflow = args.indicator == "p" and sweep.p_dataflow
  # ... and its forward with it: the whole p sweep as ONE dataflow launch (dg_lserk4_sweep_p)
  psweep = args.indicator == "p" and sweep.p_sweep
  fused_refine = ((dataflow or pflow) and world == 1 and sweep.batch == 1 and not args.gather_ics
                  and not args.graph)
  # The refine index (the mesh split's input) and the indicator there go to the host in one
  # async copy into pinned memory, read after the timed region has synced.  (The copy on a
  # side stream, with the next step waiting for it before rewriting the state, measured
  # ~30 us slower per step: the cross-stream event round trip, profiles/r03/sweep/ab5.)
  def copy_result():
    res_host.copy_(reducer.state[0:2], non_blocking=True)

  # The fused refine decision writes index and value straight into the pinned result buffer
  # (its device alias): no copy launch per step.
  res_alias = pkg.operators.host_alias(res_host) if fused_refine else None

  def one_step(ev=None):
    if ev:
      ev[0].record(stream)
    if fused_refine and psweep:  # forward + estimate + refine decision: one launch
      if res_alias is not None:
        sweep.sweep_refine(reducer, idx=res_alias, value=res_alias + 8)
      else:
        sweep.sweep_refine(reducer)
      if ev:
        ev[2].record(stream)
      if res_alias is None:
        copy_result()
      return
    if fused_refine and pflow:
      sweep.forward()
      if ev:
        ev[1].record(stream)
        ev[3].record(stream)
      if res_alias is not None:
        sweep.estimate_refine(res_alias, res_alias + 8, reducer.nonfinite)
      else:
        sweep.estimate_refine(reducer.idx, reducer.value, reducer.nonfinite)
      if ev:
        ev[2].record(stream)
      if res_alias is None:
        copy_result()
      return
    if fused_refine:
      if res_alias is not None:
        sweep.sweep_refine(reducer, idx=res_alias, value=res_alias + 8)
      else:
        sweep.sweep_refine(reducer)
      if ev:
        ev[2].record(stream)
      if res_alias is None:
        copy_result()
      return
    if dataflow or psweep:
      sweep.sweep_graph() if args.graph else sweep.sweep()
      if ev:
        ev[2].record(stream)
      partial = sweep.reduce()
      ens.refine_decision(partial, n_total, reducer)
      if args.gather_ics:
        ens.gather_per_ic(sweep.per_ic(), n_total)
      copy_result()
      return
    sweep.forward_graph() if args.graph else sweep.forward()
    if ev:
      ev[1].record(stream)
    if not args.graph:
      sweep.terminal()  # nothing (kept for the launch count; see EnsembleSweep.terminal)
    if ev:
      ev[3].record(stream)
    sweep.adjoint_graph() if args.graph else sweep.run_adjoint()
    if ev:
      ev[2].record(stream)
    partial = sweep.reduce()
    ens.refine_decision(partial, n_total, reducer)
    if args.gather_ics:
      ens.gather_per_ic(sweep.per_ic(), n_total)
    # The refine index (the mesh split's input) and the indicator there go to the host in
    # one async copy into pinned memory, read after the timed region has synced.
    copy_result()

  warm, warm_ms, warm_last = warm_up(one_step, args, stream, max_steps=args.warmup + 600)
  torch.cuda.synchronize()
  reducer.nonfinite.zero_()  # count non-finite indicators over the timed steps only
  barrier(world)
  torch.cuda.synchronize()

  evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
  ev_end = torch.cuda.Event(enable_timing=True)
  t0 = time.perf_counter()
  for s in range(args.steps):
    one_step(evs[s])
  ev_end.record(stream)
  host_issue = time.perf_counter() - t0  # host time to enqueue the steps (launch-bound check)
  torch.cuda.synchronize()
  barrier(world)
  torch.cuda.synchronize()
  elapsed = time.perf_counter() - t0
  elapsed = max_over_ranks(elapsed, world, dev, args.backend)

  ref_idx = int(res_host[0])
  ref_val = float(res_host[1:2].view(torch.float64)[0])
  nonfinite = int(reducer.nonfinite.item())
  if nonfinite:
    pkg.adaptive.check_indicator(float("nan"), ref_idx)  # raises FloatingPointError
  pkg.adaptive.check_indicator(ref_val, ref_idx)

  Np, ktot = N + 1, K * sweep.batch
  pmode = args.indicator == "p"
  if args.record == "jumps":
    ms, tw = sweep.op.rec_steps_per_launch, sweep.op.rec_tile_width
    fms = sweep.op.rec_fwd_steps_per_launch  # the forward's own (one 20-step launch)
  else:
    fms = sweep.op.steps_per_launch
    ms, tw = ((sweep.est.steps_per_launch, sweep.est.tile_width) if pmode
              else (fms, sweep.op.tile_width))
  chunks, fchunks = sweep_chunks(nsteps, ms), sweep_chunks(nsteps, fms)
  if psweep:  # the forward runs in the estimate's 4-step blocks inside the one launch
    fms, fchunks = ms, list(chunks)
  if dataflow or psweep:  # one launch per sweep: its time, reported in the adjoint's slot
    fwd_us = [float("nan") for e in evs]
    adj_us = [e[0].elapsed_time(e[2]) * 1e3 for e in evs]
  else:
    fwd_us = [e[0].elapsed_time(e[1]) * 1e3 / len(fchunks) for e in evs]
    # the p-estimate's one dataflow launch: its whole time (its blocks are not separate)
    adj_us = [e[3].elapsed_time(e[2]) * 1e3 / (1 if pflow else len(chunks)) for e in evs]
  step_ms = [evs[i][0].elapsed_time(evs[i + 1][0] if i + 1 < len(evs) else ev_end)
             for i in range(len(evs))]
  fwd_launch_us, adj_launch_us = float(np.mean(fwd_us)), float(np.mean(adj_us))
  # Algorithmic bytes of a launch of m fused steps:
  #   snapshots: forward reads u^n once and writes the m snapshots u^{n+1..n+m}: (8 + 8 m) B
  #     per DOF; the adjoint reads w^{n+m} and the m snapshots and writes w^n: (16 + 8 m) B
  #     per DOF, plus the indicator read-modify-write, 16 B per element;
  #   jumps: forward reads u^n, writes u^{n+m} and m left-face jumps: 16 B per DOF + 8 m B per
  #     element; the adjoint reads w^{n+m} and m jump rows, writes w^n, updates eta:
  #     16 B per DOF + (8 m + 16) B per element.
  # A sweep's launches may differ in m (e.g. 8 + 8 + 4 at 20 steps); the per-launch figures
  # are the sweep's averages: achieved = sweep bytes / sweep time.
  #   p-estimate (k_adj_p): reads w^{n+m} and writes w^n at order N+1 (16 (Np + 1) B per
  #     element), reads the m + 1 order-N snapshots u^n..u^{n+m} (8 (m + 1) Np B), updates eta.
  #   dataflow: the one launch moves the sum of its blocks' bytes (the forward blocks' and the
  #     adjoint blocks' figures above; a block's partial indicator row is written and read
  #     once, as the launches' read-modify-write of eta).
  if dataflow:
    fwd_bytes = float(np.sum([(16.0 * Np + 8.0 * m) * ktot for m in fchunks]))
    adj_bytes = fwd_bytes + float(np.sum([(16.0 * Np + 8.0 * m + 16.0) * ktot for m in chunks]))
  elif args.record == "jumps":
    fwd_bytes = float(np.mean([(16.0 * Np + 8.0 * m) * ktot for m in fchunks]))
    adj_bytes = float(np.mean([(16.0 * Np + 8.0 * m + 16.0) * ktot for m in chunks]))
  elif pmode:
    agg = np.sum if psweep else np.mean
    fwd_bytes = float(agg([(8.0 + 8.0 * m) * Np * ktot for m in fchunks]))
    adj_bytes = float((np.sum if pflow else np.mean)(
        [(16.0 * (Np + 1) + 8.0 * (m + 1) * Np + 16.0) * ktot for m in chunks]))
    if psweep:  # the one launch moves both directions' bytes
      adj_bytes += fwd_bytes
  else:
    fwd_bytes = float(np.mean([(8.0 + 8.0 * m) * Np * ktot for m in fchunks]))
    adj_bytes = float(np.mean([(16.0 + 8.0 * m) * Np * ktot + 16.0 * ktot for m in chunks]))
  rec_tag = ",jumps" if args.record == "jumps" else ""
  pairs = args.record == "jumps" and getattr(sweep.op, "rec_lane_elements", 1) == 2
  kadj, kstep = ("k_adj_rp", "k_step_rp") if pairs else ("k_adj", "k_step")
  if pmode:
    kadj = "k_psweep" if psweep else "k_adjp_flow" if pflow else "k_adj_p"
  if dataflow:
    kadj = "k_sweep_rp"
  tile_tag = tile_tag_fwd = f"{tw},2 elements/lane" if pairs else f"{tw}"
  # Issued vs useful lanes: each tile recomputes a halo of H elements per side (the
  # dependency cone of its fused steps) and writes T - 2H, weighted by steps.
  if pairs:
    # pair tiles: 512 elements per tile width (the dataflow launch: 128 per workgroup wave);
    # halos rounded up to even (aligned record pairs, dg_rec.hip RpHalo), the forward's one
    # wider for the final jumps
    T_pair = sweep.op.query_sweep(nsteps, tile=True)[5] if dataflow else 512 * tw
    sweep_waves = sweep.op.query_sweep(nsteps, tile=True)[4] if dataflow else None
    T_of = lambda m, fwd: T_pair  # noqa: E731
    h_fwd = lambda m: (5 * m + 2) & ~1  # noqa: E731
    h_adj = lambda m: (5 * m + 1) & ~1  # noqa: E731
  elif args.record == "jumps":
    T_of = lambda m, fwd: 256 * tw  # noqa: E731
    h_fwd = lambda m: 5 * m + 1  # noqa: E731  (the final state's jumps need one more)
    h_adj = lambda m: 5 * m  # noqa: E731
  else:
    # the snapshot forward runs on 256-element one-wave tiles (4 elements per lane) at N <= 2
    # by default (dg_plan_create), else on workgroup tiles of 256 * tile width
    T_fwd = 256 * tw if psweep else 256 if N <= 2 else 256 * sweep.op.tile_width
    T_of = lambda m, fwd: T_fwd if fwd else 256 * tw  # noqa: E731
    h_fwd = h_adj = lambda m: 5 * m  # noqa: E731
  halo_adj = float(np.average([halo_factor(T_of(m, False), h_adj(m)) for m in chunks],
                              weights=chunks))
  halo_fwd = float(np.average([halo_factor(T_of(m, True), h_fwd(m)) for m in fchunks],
                              weights=fchunks))
  adj_gbs = adj_bytes / (adj_launch_us * 1e-6) / 1e9
  fwd_gbs = fwd_bytes / (fwd_launch_us * 1e-6) / 1e9
  traffic = traffic_src = None
  prof_key = "p" if pmode else args.record
  # a dataflow profile counts only for the same kernel: its template instantiation (Np, mesh,
  # waves, blocks, lane elements, face exchange) and its occupancy target, which is an
  # attribute outside the name (round 4's Np = 2 line read a profile of the 6-waves-per-SIMD
  # build of the same name); a profile without that record matches nothing
  ksig = sweep.op.query_sweep_kernel(nsteps) if pairs and dataflow else None
  same_kernel = lambda tr: ksig is None or (  # noqa: E731
      tr.get("sweep_kernel") == ksig
      and any(str(n).startswith(ksig["name"]) for n in (tr.get("adj_kernel") or [])))
  prof_dir = None  # the matching profile directory (its SQ summary is read below)
  for d in PROFILE_DIRS[prof_key]:
    try:
      with open(os.path.join(d, PROFILE_TRAFFIC_FILE.get(prof_key, "pmc_traffic.json"))) as f:
        tr = json.load(f)
    except (OSError, ValueError):
      continue
    if (tr.get("N") == N and tr.get("K") == K and tr.get("batch") == sweep.batch
        and tr.get("steps_per_launch") == ms and bool(tr.get("dataflow")) == dataflow
        and bool(tr.get("p_flow")) == pflow and bool(tr.get("p_sweep")) == psweep
        and (not pmode or tr.get("tile_width", tw) == tw)
        and tr.get("record", "snapshots") == args.record
        and tr.get("indicator", "jump") == args.indicator
        and same_kernel(tr)):
      traffic = tr.get("adj_bytes_per_launch")
      traffic_src = os.path.relpath(d, ROOT)
      prof_dir = d
      break

  # Jump record: the same launches priced with the snapshot sweep's algorithmic bytes (what
  # the snapshot algorithm moves for the same steps) -- an effective rate, not HBM traffic.
  effective = None
  if args.record == "jumps":
    agg = np.sum if dataflow else np.mean
    snap_fwd = float(agg([(8.0 + 8.0 * m) * Np * ktot for m in fchunks]))
    snap_adj = float(agg([(16.0 + 8.0 * m) * Np * ktot + 16.0 * ktot for m in chunks]))
    if dataflow:
      snap_adj += snap_fwd
    eff_adj = snap_adj / (adj_launch_us * 1e-6) / 1e9
    eff_fwd = snap_fwd / (fwd_launch_us * 1e-6) / 1e9
    effective = {"what": "NOT moved bandwidth: the launch times priced with the bytes the "
                         "snapshot sweep would move for the same steps (what storing 8 B per "
                         "element-step instead of a snapshot saves); moved bytes are "
                         "roofline_hbm's algorithmic_bytes and traffic",
                 "adj_GBs_equiv": eff_adj, "adj_frac_equiv": eff_adj / HBM_PEAK_GBS,
                 "fwd_GBs_equiv": eff_fwd, "fwd_frac_equiv": eff_fwd / HBM_PEAK_GBS}
  total_dofs = sum_over_ranks(sweep.dof_updates, world, dev, args.backend) * args.steps
  value = total_dofs / elapsed
  # The single-step algorithm moves 16 B (fwd) + 24 B + 16/Np B (adj) per pair of
  # DOF-updates, so its HBM roofline is 8 TB/s / that per-update average.
  single_step_bytes = (16.0 + 24.0 + 16.0 / Np) / 2.0
  single_step_roofline = HBM_PEAK_GBS * 1e9 / single_step_bytes * world
  copy_gbs = stream_copy_gbs(dev) if rank == 0 else None
  import torch.distributed as dist
  dist_world = dist.get_world_size() if dist.is_initialized() else 1
  idx_ranks = ranks_agree(ref_idx, world, dev, args.backend)
  # DOF-updates per launch (sweep average; the p-estimate's dataflow launch: all its blocks)
  upl = Np * ktot * (float(np.sum(chunks)) if pflow else float(np.mean(chunks)))
  fupl = Np * ktot * float(np.mean(fchunks))
  horner = args.record == "jumps" and (pairs or dataflow)  # dg_rec_tiles.h's Horner-form steps
  if pmode:
    adj_fpu = p_flops_per_update(Np)
  else:
    adj_fpu = horner_flops_per_update(Np, True) if horner else eo_flops_per_update(Np, True)
  fwd_fpu = horner_flops_per_update(Np, False) if horner else eo_flops_per_update(Np, False)
  adj_tf = adj_fpu * upl / (adj_launch_us * 1e-6) / 1e12
  fwd_tf = fwd_fpu * fupl / (fwd_launch_us * 1e-6) / 1e12
  if dataflow or psweep:
    # the one launch executes both directions' flops; its issued lanes weight each
    # direction's halo factor by its share of them
    f_fl, a_fl = fwd_fpu * Np * ktot * nsteps, adj_fpu * Np * ktot * nsteps
    adj_tf = (f_fl + a_fl) / (adj_launch_us * 1e-6) / 1e12
    halo_adj = (f_fl * halo_fwd + a_fl * halo_adj) / (f_fl + a_fl)
  decision = refine_margin(sweep, one_step) if world == 1 and not args.no_margin else None
  out = {
      "metric": metric_name(N, K),
      "value": value,
      "unit": "DOF-updates/s",
      "n_gpus": world,
      "steps": args.steps,
      "warmup": args.warmup,
      "warmup_effective": warm,
      "warmup_ms": warm_ms,
      "warmup_last_step_ms": warm_last,
      "ms_per_step": elapsed / args.steps * 1e3,
      "higher_is_better": True,
      "scaling": "strong" if args.ics > 0 else "weak",
      "vs_baseline": None,
      "dtype": "f64",
      "data": "synthetic (u0 = sin(2 pi x) on rank 0, SURVEY 8d sine-family ICs on other ranks)",
      "config": {"workload": (f"config {'4' if args.ics > 0 else '2'}: 1D DG advection N={N} "
                              f"K={K} x {n_total} trajectories, LSERK4 fwd+adj {nsteps}+{nsteps} "
                              f"steps/sweep + DWR indicator + refine argmax; indicator "
                              f"record: {args.record}"),
                 "N": N, "K": K, "nsteps_per_sweep": nsteps, "trajectories": n_total,
                 "trajectories_per_gpu": sweep.batch, "parallelism": f"ensemble-dp{world}",
                 "per_ic_gather": bool(args.gather_ics), "record": args.record},
      "roofline": {"bound": "hbm", "achieved": adj_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": adj_gbs / HBM_PEAK_GBS, "traffic": traffic,
                   "kernel": f"{kadj}<{Np},uniform,{tile_tag},{ms}{rec_tag}> ({ms} reverse steps + DWR per launch)",
                   "launch_us": adj_launch_us, "launch_us_stats": stats(adj_us),
                   "algorithmic_bytes": adj_bytes, "traffic_source": traffic_src,
                   "traffic_from_profile": traffic is not None,
                   "note": ("p-estimate: per reverse step the order-(N+1) forward step from the "
                            "prolonged snapshot and the order-(N+1) reverse step (roofline_fp64)"
                            if pmode else None if args.record != "jumps" else
                            "jump record: 8 B per element-step instead of an 8 Np B snapshot, so "
                            "the launches are bound by fp64 issue and the per-stage barrier "
                            "chain, not HBM (roofline_fp64); the snapshot sweep's k_adj reaches "
                            "0.62 of HBM (--record snapshots, DESIGN.md section 7)")},
      "roofline_fwd": {"bound": "hbm", "achieved": fwd_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": fwd_gbs / HBM_PEAK_GBS,
                       "kernel": f"{kstep}<{Np},uniform,{tile_tag_fwd},{fms}{rec_tag}> ({fms} steps per launch)",
                       "launch_us": fwd_launch_us, "launch_us_stats": stats(fwd_us),
                       "algorithmic_bytes": fwd_bytes},
      "snapshot_bytes_equivalent": effective,
      # The compute roof of the same launches: the even/odd algorithm's fp64 flops (interior
      # elements) / launch time, against the spec and the on-box FMA probe; issued_frac
      # counts the halo lanes each tile also computes (the work the lanes actually issue).
      "roofline_fp64": {
          "bound": "fp64 vector", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
          "probe_ceiling": FP64_PROBE_TFLOPS,
          "adj_achieved": adj_tf, "adj_frac": adj_tf / FP64_PEAK_TFLOPS,
          "fwd_achieved": fwd_tf, "fwd_frac": fwd_tf / FP64_PEAK_TFLOPS,
          "adj_halo_factor": halo_adj, "fwd_halo_factor": halo_fwd,
          "adj_issued_frac": adj_tf * halo_adj / FP64_PEAK_TFLOPS,
          "fwd_issued_frac": fwd_tf * halo_fwd / FP64_PEAK_TFLOPS,
          "flop_per_update": {"fwd": fwd_fpu, "adj": adj_fpu},
          "what": "algorithmic fp64 flops of the interior elements per launch / launch time; "
                  "*_issued_frac multiplies by the tile's issued/useful lanes (halo)"},
      "step_ms_stats": stats(step_ms),
      "single_step_roofline": {"value": single_step_roofline, "unit": "DOF-updates/s",
                               "bytes_per_update": single_step_bytes,
                               "frac": value / single_step_roofline},
      "stream_copy": {"achievable_GBs": copy_gbs, "unit": "GB/s",
                      "what": "dg_stream_copy (16 B per lane, 4 in flight) of 1 GiB, read + "
                              "write, rank 0",
                      "adj_frac_of_achievable": adj_gbs / copy_gbs if copy_gbs else None,
                      "fwd_frac_of_achievable": fwd_gbs / copy_gbs if copy_gbs else None},
      "steps_per_launch": ms,
      "tile_width": tw,
      "launch_steps": chunks,
      "launch_steps_fwd": fchunks,
      "indicator": args.indicator,
      "refine_index": ref_idx,
      "refine_value": ref_val,
      "refine_index_ranks": idx_ranks,
      "refine_decision": decision,
      "nonfinite_indicator_steps": nonfinite,
      "dist_world_size": dist_world,
      "collective_backend": (None if world == 1 else
                             "rccl (torch nccl backend)" if args.backend == "nccl" else "gloo"),
      "host_issue_ms_per_step": host_issue / args.steps * 1e3,
      "library": {"path": os.path.relpath(pkg._lib.LIB_PATH, ROOT),
                  "override": bool(os.environ.get("DG_LIB_PATH"))},
  }
  if pmode:
    try:  # issued fp64 of k_adj_p from the SQ passes of the same bench (profiles/r04/p/)
      with open(os.path.join(prof_dir, "sq_summary.json")) as fh:
        sq = json.load(fh)
      if traffic is not None:
        f = out["roofline_fp64"]
        fl = sq["fp64_flops_issued_per_launch"]
        f["pmc_issued_per_launch"] = fl
        f["pmc_issued_frac"] = fl / (adj_launch_us * 1e-6) / 1e12 / FP64_PEAK_TFLOPS
        f["pmc_issued_over_useful"] = fl / (((fwd_fpu + adj_fpu) * Np * ktot * nsteps) if psweep
                                            else adj_fpu * upl)
        f["pmc_wait_any_frac"] = sq.get("wait_any_frac_of_wave_cycles")
        f["pmc_source"] = os.path.relpath(os.path.join(prof_dir, "sq_summary.json"), ROOT)
    except (OSError, ValueError, KeyError, TypeError):
      pass
  if psweep:
    r = out["roofline"]
    r["kernel"] = (f"k_psweep<{Np - 1}+1,uniform,{256 * tw} elements,{ms} steps per block> "
                   f"(ONE dataflow launch per sweep: {len(fchunks)} forward blocks + "
                   f"{len(chunks)} estimate blocks of {ms} steps + DWR"
                   f"{' + refine decision' if fused_refine else ''})")
    r["note"] = ("the p sweep as one dataflow launch (dg_lserk4_sweep_p): the order-N snapshot "
                 "forward's and the estimate's blocks are the work items; algorithmic bytes = "
                 "both directions' blocks; per reverse step the order-(N+1) forward step from "
                 "the prolonged snapshot and the order-(N+1) reverse step (roofline_fp64)")
    out["roofline_fwd"] = None
    f = out["roofline_fp64"]
    for k in ("fwd_achieved", "fwd_frac", "fwd_issued_frac"):
      f[k] = None
    f["what"] = ("algorithmic fp64 flops of both directions (interior elements) per launch / "
                 "launch time; adj_issued_frac weights each direction's halo by its flops")
    out["stream_copy"]["fwd_frac_of_achievable"] = None
    out["p_dataflow"] = {"launches_per_sweep": 1, "blocks_fwd": fchunks, "blocks": chunks,
                         "refine_in_launch": fused_refine,
                         "refine_to_host": ("written by the launch into pinned memory "
                                            "(dg_host_alias)" if res_alias is not None
                                            else "async copy"),
                         "work_items": 2 * len(chunks) * -(-ktot // (256 * tw - 10 * ms)),
                         "status": sweep.op.sweep_status()}
    if out["p_dataflow"]["status"]:
      raise RuntimeError("a p-sweep work item gave up waiting for a producer")
  elif pflow:
    r = out["roofline"]
    r["kernel"] = (f"k_adjp_flow<{Np - 1}+1,uniform,{256 * tw} elements,{ms} steps per block> "
                   f"(ONE dataflow launch per estimate: {len(chunks)} blocks of {ms} reverse "
                   f"steps + DWR{' + refine decision' if fused_refine else ''})")
    r["note"] = ("p-estimate as one dataflow launch (dg_lserk4_adj_p, DG_TUNE_P_FLOW): the blocks' "
                 "tiles are the work items; per reverse step the order-(N+1) forward step from "
                 "the prolonged snapshot and the order-(N+1) reverse step (roofline_fp64); "
                 "algorithmic bytes = the blocks' sum")
    out["p_dataflow"] = {"launches_per_estimate": 1, "blocks": chunks,
                         "refine_in_launch": fused_refine,
                         "refine_to_host": ("written by the launch into pinned memory "
                                            "(dg_host_alias)" if res_alias is not None
                                            else "async copy"),
                         "work_items": len(chunks) * -(-ktot // (256 * tw - 10 * ms)),
                         "status": sweep.op.sweep_status()}
    if out["p_dataflow"]["status"]:
      raise RuntimeError("a p-estimate work item gave up waiting for a producer")
  if dataflow:
    r = out["roofline"]
    r["kernel"] = (f"k_sweep_rp<{Np},uniform,{T_pair} elements,fwd {'+'.join(map(str, fchunks))},"
                   f"adj {'+'.join(map(str, chunks))},jumps> (ONE dataflow launch per sweep: "
                   f"{nsteps} forward + {nsteps} reverse steps + DWR)")
    r["note"] = ("dataflow sweep (dg_lserk4_sweep_rec): the forward and adjoint blocks' tiles are "
                 "the work items of one launch; algorithmic bytes = the blocks' sum (8 B record "
                 "per element-step), so the launch is bound by fp64 issue and each level's "
                 "barrier chain, not HBM (roofline_fp64)")
    out["roofline_fwd"] = None
    f = out["roofline_fp64"]
    for k in ("fwd_achieved", "fwd_frac", "fwd_issued_frac"):
      f[k] = None
    f["what"] = ("algorithmic fp64 flops of both directions (interior elements) per launch / "
                 "launch time (adj_*: the one dataflow launch); adj_issued_frac weights each "
                 "direction's issued/useful lanes (halo) by its flops")
    out["stream_copy"]["fwd_frac_of_achievable"] = None
    if out.get("snapshot_bytes_equivalent"):
      out["snapshot_bytes_equivalent"].update({"fwd_GBs_equiv": None, "fwd_frac_equiv": None})
    # the PMC-measured issued fp64 flops of the same launch (SQ passes of this bench,
    # profiles/r04/collect.sh), from the profile whose traffic matched
    try:
      with open(os.path.join(prof_dir, "sq_summary.json")) as fh:
        sq = json.load(fh)
      if ksig is None or any(str(n).startswith(ksig["name"]) for n in (sq.get("kernel") or [])):
        fl = sq["fp64_flops_issued_per_launch"]
        f["pmc_issued_per_launch"] = fl
        f["pmc_issued_frac"] = fl / (adj_launch_us * 1e-6) / 1e12 / FP64_PEAK_TFLOPS
        f["pmc_issued_over_useful"] = fl / ((fwd_fpu + adj_fpu) * Np * ktot * nsteps)
        f["pmc_wait_any_frac"] = sq.get("wait_any_frac_of_wave_cycles")
        f["pmc_source"] = os.path.relpath(os.path.join(prof_dir, "sq_summary.json"), ROOT)
    except (OSError, ValueError, KeyError, TypeError):
      pass
    # The launch's binding roof is fp64 issue (8 B per element-step of record: HBM is far
    # from bound): `roofline` carries it, the HBM view sits beside it.
    hbm = out.pop("roofline")
    out["roofline"] = {
        "bound": "fp64 vector", "achieved": f["adj_achieved"], "peak": FP64_PEAK_TFLOPS,
        "unit": "TFLOP/s", "frac": f["adj_achieved"] / FP64_PEAK_TFLOPS,
        "issued_frac": f["adj_issued_frac"], "pmc_issued_frac": f.get("pmc_issued_frac"),
        "traffic": hbm["traffic"], "traffic_unit": "HBM bytes per launch (PMC FETCH+WRITE)",
        "hbm_frac": hbm["frac"], "kernel": hbm["kernel"], "launch_us": hbm["launch_us"],
        "launch_us_stats": hbm["launch_us_stats"],
        "what": ("useful fp64 flops of both directions' interior elements per launch / launch "
                 "time (achieved, frac); issued_frac adds the halo lanes, pmc_issued_frac is "
                 "the PMC count; the HBM view (algorithmic bytes, traffic) is roofline_hbm")}
    out["roofline_hbm"] = hbm
    out["dataflow"] = {"launches_per_sweep": 1, "blocks_fwd": fchunks, "blocks_adj": chunks,
                       "refine_in_launch": fused_refine,
                       "refine_to_host": "written by the launch into pinned memory (dg_host_alias)"
                                         if res_alias is not None else "async copy",
                       "work_items": sweep.op.query_sweep(nsteps)[3],
                       "kernel": ksig,
                       "status": sweep.op.sweep_status()}
    if out["dataflow"]["status"]:
      raise RuntimeError("a dataflow work item gave up waiting for a producer")
  if len(set(idx_ranks)) != 1:
    raise RuntimeError(f"refine index differs across ranks: {idx_ranks}")
  if rank == 0 and world == 1 and not args.no_cpu_baseline:
    cs = args.cpu_steps if not pmode else max(2, args.cpu_steps // 2)
    kw = dict(indicator=args.indicator, ics=min(2, n_total), ics_total=n_total)
    numpy_1t = cpu_baseline(N, K, cs, **kw)
    cport = None
    if pmode or args.record == "jumps":
      # the oracle's C port on the host's cores (the workload's own 20 + 20 steps), and on
      # one core; the numpy restatement (MATLAB-style whole-array passes) beside them
      th = host_threads()
      ckw = dict(ics_total=n_total, indicator=args.indicator)
      cport = cpu_baseline_cport(N, K, nsteps, th, **ckw)
      if cport is not None and args.ics == 0:
        out["cpu_baseline_1t"] = cpu_baseline_cport(N, K, nsteps, 1, **ckw)
    if cport is not None:
      out["cpu_baseline"] = cport
      out["cpu_baseline_numpy"] = numpy_1t
    else:
      out["cpu_baseline"] = numpy_1t
  if rank == 0:
    print(json.dumps(out, allow_nan=False), flush=True)
  if world > 1:
    import torch.distributed as dist
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
