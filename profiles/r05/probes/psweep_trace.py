"""Per-item timeline of the whole p sweep as one dataflow launch (k_psweep) at config 2's
size: per block (forward blocks first, then the estimate's), the take latency, the producer
poll, the body, the publish drain, and the slack of the producers (how long before an item's
dequeue they had published).  GPU box, repo root."""
import importlib
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
N, K = 4, 1 << 20
tw = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
mesh = pkg.BaseGalerkin1D(n=N, k=K)
op = pkg.operators.DGAdvection1D(mesh)
est = pkg.operators.DWREstimate(op, tile_width=tw, steps_per_launch=4)
dt = mesh.cfl_dt()
snaps = op.new_field(n + 1)
op.init_sine([1.0], [1.0], [0.0], out=snaps[0])
w = est.new_field()
eta = torch.zeros(op.ktot, dtype=torch.float64, device="cuda")
TE = 256 * tw - 2 * 5 * 4  # 4-step blocks: a halo of 20 elements per side
nT = -(-op.ktot // TE)
nb = n // 4
items = 2 * nb * nT
trace = torch.zeros(8 * items, dtype=torch.int64, device="cuda")
assert est.query_sweep(n)
for _ in range(300):
  est.sweep(snaps, w, 0.0, dt, n, eta=eta)
torch.cuda.synchronize()
op.sweep_trace(trace)
est.sweep(snaps, w, 0.0, dt, n, eta=eta)
torch.cuda.synchronize()
op.sweep_trace(None)
t = trace.view(items, 8).cpu().numpy().astype(np.int64)
if len(sys.argv) > 2:
  np.save(sys.argv[2], t)  # the raw per-item words
start, deq, ready, bdone, pub = (t[:, i] for i in range(5))
t0 = start.min()
out = {"tw": tw, "items": items, "nT": nT, "span_us": float((pub.max() - t0) / 100.0), "blocks": []}
for b in range(2 * nb):
  sl = slice(b * nT, (b + 1) * nT)
  rec = {"blk": ("F%d" % b) if b < nb else ("A%d" % (b - nb)),
         "deq_first_us": float((deq[sl].min() - t0) / 100.0),
         "pub_last_us": float((pub[sl].max() - t0) / 100.0),
         "take_us": float(((deq - start)[sl]).mean() / 100.0),
         "wait_us": float(((ready - deq)[sl]).mean() / 100.0),
         "body_us": float(((bdone - ready)[sl]).mean() / 100.0),
         "publish_us": float(((pub - bdone)[sl]).mean() / 100.0)}
  if b > 0:
    j = np.arange(nT)
    prod = np.maximum.reduce([pub[(b - 1) * nT + np.clip(j + d, 0, nT - 1)] for d in (-1, 0, 1)])
    slack = (deq[sl] - prod) / 100.0
    rec["slack_us_min"] = float(slack.min())
    rec["frac_waited"] = float((slack < 0).mean())
  out["blocks"].append(rec)
ev_t = np.concatenate([start, pub])
ev_d = np.concatenate([np.ones(items), -np.ones(items)])
o = np.argsort(ev_t, kind="stable")
conc = np.cumsum(ev_d[o])
out["mean_in_flight"] = float(np.sum(conc[:-1] * np.diff(ev_t[o])) / (ev_t[o][-1] - ev_t[o][0]))
print(json.dumps(out, indent=1))
