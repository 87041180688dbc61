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


def _run(args, timeout=240):
  env = dict(os.environ)
  r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                     capture_output=True, text=True, timeout=timeout, env=env)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
  assert len(lines) == 1, r.stdout
  return json.loads(lines[0])


def test_bench_single_rank_line(gpu):
  out = _run(["--K", "65536", "--steps", "3", "--warmup", "2", "--no-converge",
              "--no-cpu-baseline"])
  assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup_effective"] == 2
  assert out["unit"] == "DOF-updates/s" and out["value"] > 0
  assert out["roofline"]["bound"] == "hbm" and 0 < out["roofline"]["frac"] < 1
  assert out["nonfinite_indicator_steps"] == 0
  assert out["stream_copy"]["achievable_GBs"] > 1000
  assert out["refine_index_ranks"] == [out["refine_index"]]


@pytest.mark.parametrize("extra", [[], ["--ics", "6"]])
def test_bench_self_launches_two_ranks(gpu, extra):
  out = _run(["--gpus", "2", "--backend", "gloo", "--K", "65536", "--steps", "2",
              "--warmup", "1", "--no-converge", "--no-cpu-baseline", *extra])
  assert out["n_gpus"] == 2 and out["rccl_world_size"] == 2
  ranks = out["refine_index_ranks"]
  assert len(ranks) == 2 and ranks[0] == ranks[1] == out["refine_index"]
  if extra:
    assert out["scaling"] == "strong" and out["config"]["trajectories"] == 6
    assert out["config"]["trajectories_per_gpu"] == 3
