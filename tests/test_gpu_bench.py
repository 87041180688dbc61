"""bench.py end to end on the GPU, small sizes: the single-rank JSON line, and the
self-launched multi-rank path (`--gpus 2`) with the product's HIP reducer (DeviceReducer:
dg_sum_rows + dg_argmax_ex) on every rank.  One GPU box has one GPU, so the two ranks share
it and exchange through gloo (RCCL refuses two ranks on one device); the driver's 8-GPU run
uses RCCL."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(args, timeout=240, env_extra=None):
  env = dict(os.environ)
  env.update(env_extra or {})
  r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                     capture_output=True, text=True, timeout=timeout, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
  assert len(lines) == 1, r.stdout
  return json.loads(lines[0])


@pytest.mark.parametrize("dataflow", [True, False])
def test_bench_single_rank_line(gpu, dataflow):
  """The default line (the sweep as one dataflow launch, k_sweep_rp) and the launch-chain
  line (DG_REC_SWEEP=0: k_step_rp + k_adj_rp, timed per direction)."""
  out = _run(["--K", "65536", "--steps", "3", "--warmup", "2", "--no-converge",
              "--no-cpu-baseline"], env_extra={"DG_REC_SWEEP": "1" if dataflow else "0"})
  assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup_effective"] == 2
  assert out["unit"] == "DOF-updates/s" and out["value"] > 0
  # the dataflow sweep's binding roof is fp64 issue, the chains' HBM
  assert out["roofline"]["bound"] == ("fp64 vector" if dataflow else "hbm")
  assert 0 < out["roofline"]["frac"] < 1
  if dataflow:
    assert out["roofline_hbm"]["bound"] == "hbm" and 0 < out["roofline_hbm"]["frac"] < 1
    assert out["roofline"]["frac"] == out["roofline_fp64"]["adj_frac"]
  assert "roofline_effective" not in out
  assert out["nonfinite_indicator_steps"] == 0
  assert out["stream_copy"]["achievable_GBs"] > 1000
  assert out["refine_index_ranks"] == [out["refine_index"]]
  assert "flops" not in out and out["dist_world_size"] == 1 and out["collective_backend"] is None
  fp = out["roofline_fp64"]
  keys = ("adj_frac", "fwd_frac", "adj_issued_frac", "fwd_issued_frac")
  if dataflow:
    assert out["roofline"]["kernel"].startswith("k_sweep_rp<5")
    assert out["dataflow"]["status"] == 0 and out["dataflow"]["launches_per_sweep"] == 1
    assert out["roofline_fwd"] is None and fp["fwd_frac"] is None
    keys = ("adj_frac", "adj_issued_frac")
  else:
    assert "dataflow" not in out and out["roofline"]["kernel"].startswith("k_adj_rp<5")
  for key in keys:
    assert 0 < fp[key] <= 1, key
  assert fp["adj_issued_frac"] >= fp["adj_frac"] and fp["fwd_halo_factor"] > 1
  assert out["indicator"] == "jump"
  d = out["refine_decision"]
  assert d["index"] == out["refine_index"] and d["top1"] >= d["top2"] >= 0
  assert d["rounding_floor"] >= 0 and isinstance(d["decided"], bool)
  assert d["decided"] == (d["margin"] > d["rounding_floor"] and d["index_alt"] == d["index"])
  assert out["library"]["path"].endswith("libdgadv.so") and not out["library"]["override"]


def test_bench_p_estimate_line(gpu):
  """--indicator p: the forward keeps snapshots and the estimate runs at order N+1 with the
  prolonged one-step residual -- by default both as ONE dataflow launch (k_psweep, with the
  refine decision); its line carries the same roofline blocks and a CPU baseline of the
  oracle's p-estimate.  (The jump line run first carries the compiled oracle port's.)"""
  out = _run(["--K", "65536", "--steps", "3", "--warmup", "2", "--no-converge",
              "--cpu-steps", "2"])
  assert out["indicator"] == "jump"
  # the jump line's CPU baseline: the oracle's C port on the host threads and on one, the
  # numpy oracle beside them (round 6)
  cb, c1, cn = out["cpu_baseline"], out["cpu_baseline_1t"], out["cpu_baseline_numpy"]
  assert "C port" in cb["sample"] and cb["kind"] == "port" and cb["cores"] >= 1
  assert c1["cores"] == 1 and "C port" in c1["sample"] and "numpy" in cn["sample"]
  assert cb["value"] > 0 and c1["value"] > 0 and cn["value"] > 0
  out = _run(["--K", "65536", "--steps", "3", "--warmup", "2", "--no-converge",
              "--indicator", "p", "--cpu-steps", "2"])
  assert out["indicator"] == "p" and out["config"]["record"] == "snapshots"
  assert out["roofline"]["kernel"].startswith("k_psweep<4+1")
  assert out["p_dataflow"]["launches_per_sweep"] == 1 and out["p_dataflow"]["status"] == 0
  assert out["p_dataflow"]["refine_in_launch"]
  assert 0 < out["roofline"]["frac"] < 1
  assert out["nonfinite_indicator_steps"] == 0
  assert out["cpu_baseline"]["value"] > 0 and "p-enriched" in out["cpu_baseline"]["sample"]


@pytest.mark.parametrize("extra", [[], ["--ics", "6"], ["--indicator", "p"]])
def test_bench_self_launches_two_ranks(gpu, extra):
  out = _run(["--gpus", "2", "--backend", "gloo", "--K", "65536", "--steps", "2",
              "--warmup", "1", "--no-converge", "--no-cpu-baseline", *extra])
  assert out["n_gpus"] == 2 and out["dist_world_size"] == 2
  assert out["collective_backend"] == "gloo"  # never reported as RCCL when gloo ran
  ranks = out["refine_index_ranks"]
  assert len(ranks) == 2 and ranks[0] == ranks[1] == out["refine_index"]
  if extra and extra[0] == "--indicator":  # the p sweep's one launch per rank, no fused refine
    assert out["indicator"] == "p" and out["p_dataflow"]["launches_per_sweep"] == 1
    assert not out["p_dataflow"]["refine_in_launch"] and out["p_dataflow"]["status"] == 0
  elif extra:
    assert out["scaling"] == "strong" and out["config"]["trajectories"] == 6
    assert out["config"]["trajectories_per_gpu"] == 3
