"""Per-item timeline of the one-launch p-estimate (k_adjp_flow) at config 2's size: for each
block, the time an item waits for its producers (ready - dequeued), its body (published -
ready), how long before its dequeue its producers had published (slack; negative = it really
waited), the take counter's latency (dequeued - started) and the publish wait (the
write-through stores' drain before the flag).  Also the chain's per-launch time for comparison.  GPU box, repo root."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import importlib
pkg = importlib.import_module("adjoint-ode-adaptivity_amd")

N, K, nsteps = 4, 1 << 20, 20
tw = int(sys.argv[1]) if len(sys.argv) > 1 else 1
spl = int(sys.argv[2]) if len(sys.argv) > 2 else 4
mesh = pkg.BaseGalerkin1D(n=N, k=K)
op = pkg.operators.DGAdvection1D(mesh)
est = pkg.operators.DWREstimate(op, tile_width=tw, steps_per_launch=spl)
dt = mesh.cfl_dt()
snaps = op.new_field(nsteps + 1)
op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
op.forward(snaps[0], 0.0, dt, nsteps, snaps)
w = est.new_field()
eta = torch.zeros(op.ktot, dtype=torch.float64, device="cuda")
TE = 256 * tw - 10 * spl
nT = -(-op.ktot // TE)
nb = nsteps // spl
items = nb * nT
trace = torch.zeros(8 * items, dtype=torch.int64, device="cuda")


WITH_FWD = len(sys.argv) > 3 and sys.argv[3] == "fwd"  # the bench's order: forward, estimate


def run(flow, reps=50, warm=20):
  est.tune(flow=flow)
  evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]
  for _ in range(warm):
    if WITH_FWD:
      op.forward(snaps[0], 0.0, dt, nsteps, snaps)
    est.estimate(w, snaps, 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True,
                 terminal_prolong=True)
  torch.cuda.synchronize()
  for r in range(reps):
    if WITH_FWD:
      op.forward(snaps[0], 0.0, dt, nsteps, snaps)
    evs[r][0].record()
    est.estimate(w, snaps, 0.0, dt, nsteps, eta=eta, eta_assign=True, eta_abs=True,
                 terminal_prolong=True)
    evs[r][1].record()
  torch.cuda.synchronize()
  return float(np.median([e[0].elapsed_time(e[1]) for e in evs])) * 1e3


run(0, reps=1, warm=400)  # clocks up
chain, flow = [], []
for _ in range(3):  # alternating
  chain.append(run(0))
  flow.append(run(1))
chain_us, flow_us = float(np.median(chain)), float(np.median(flow))
op.sweep_trace(trace)
run(1, reps=1, warm=1)
op.sweep_trace(None)
t = trace.view(items, 8).cpu().numpy().astype(np.int64)
start, deq, ready, bdone, pub = t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 4]
t0 = start.min()
out_take = (deq - start) / 100.0
out_pubwait = (pub - bdone) / 100.0
out = {"tw": tw, "spl": spl, "with_forward": WITH_FWD, "items": items, "nT": nT, "nb": nb,
       "chain_us": chain_us, "flow_us": flow_us,
       "span_us": float((pub.max() - t0) / 100.0), "blocks": []}
for b in range(nb):
  sl = slice(b * nT, (b + 1) * nT)
  wait = (ready[sl] - deq[sl]) / 100.0
  body = (bdone[sl] - ready[sl]) / 100.0
  rec = {"b": b, "deq_first_us": float((deq[sl].min() - t0) / 100.0),
         "pub_last_us": float((pub[sl].max() - t0) / 100.0),
         "wait_us_mean": float(wait.mean()), "wait_us_p90": float(np.percentile(wait, 90)),
         "body_us_mean": float(body.mean()), "body_us_p10": float(np.percentile(body, 10)),
         "body_us_p90": float(np.percentile(body, 90)),
         "take_us_mean": float(out_take[sl].mean()), "take_us_p90": float(np.percentile(out_take[sl], 90)),
         "publish_us_mean": float(out_pubwait[sl].mean())}
  if b > 0:
    j = np.arange(nT)
    prod = np.maximum.reduce([pub[(b - 1) * nT + np.clip(j + d, 0, nT - 1)] for d in (-1, 0, 1)])
    slack = (deq[sl] - prod) / 100.0
    rec["slack_us_min"] = float(slack.min())
    rec["slack_us_p10"] = float(np.percentile(slack, 10))
    rec["frac_waited"] = float((slack < 0).mean())
  out["blocks"].append(rec)
# concurrency: items in flight over time
ev_t = np.concatenate([start, pub])
ev_d = np.concatenate([np.ones(items), -np.ones(items)])
o = np.argsort(ev_t, kind="stable")
conc = np.cumsum(ev_d[o])
out["max_in_flight"] = int(conc.max())
out["mean_in_flight"] = float(np.sum(conc[:-1] * np.diff(ev_t[o])) / (ev_t[o][-1] - ev_t[o][0]))
print(json.dumps(out, indent=1))
