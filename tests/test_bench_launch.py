"""bench.py's self-launch (`--gpus N` without torch.distributed.run): N ranks, one process
each, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1 in their environment, rank 0's one
JSON line passed through, a failing rank ending the job with its exit code.  CPU only: the
ranks here run a gloo stand-in for the bench body (the GPU body is covered by
tests/test_gpu_bench.py); bench's own argument parsing and the spawn are the product code."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

CHILD = r'''
import json, os, sys
import torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
assert int(os.environ["LOCAL_RANK"]) == rank
dist.init_process_group("gloo")
mine = torch.tensor([100 + 7 * (rank % 1)], dtype=torch.int64)  # same "refine index" on all
allv = torch.empty(world, dtype=torch.int64)
dist.all_gather_into_tensor(allv, mine)
fail_rank = int(sys.argv[1]) if len(sys.argv) > 1 else -1
if rank == fail_rank:
    sys.exit(3)
if rank == 0:
    print(json.dumps({"n_gpus": dist.get_world_size(), "refine_index_ranks": allv.tolist()}))
dist.destroy_process_group()
'''


def _bench():
  sys.path.insert(0, ROOT)
  import importlib
  return importlib.import_module("bench")


@pytest.mark.parametrize("world", [2, 4])
def test_spawn_ranks_one_json_line(tmp_path, world):
  child = tmp_path / "child.py"
  child.write_text(CHILD)
  code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
          f"sys.exit(bench.spawn_ranks({world}, [], script={str(child)!r}))")
  r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
  assert r.returncode == 0, r.stderr
  # (gloo itself prints "[Gloo] Rank 0 is connected ..." lines; RCCL prints none)
  lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
  assert len(lines) == 1
  out = json.loads(lines[0])
  assert out["n_gpus"] == world
  assert len(set(out["refine_index_ranks"])) == 1 and len(out["refine_index_ranks"]) == world


def test_spawn_ranks_propagates_a_failure(tmp_path):
  child = tmp_path / "child.py"
  child.write_text(CHILD)
  code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
          f"sys.exit(bench.spawn_ranks(2, ['1'], script={str(child)!r}))")
  r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
  assert r.returncode == 3


def test_bench_arguments():
  b = _bench()
  a = b.parse(["--gpus", "8", "--steps", "20", "--warmup", "5"])
  assert (a.gpus, a.steps, a.warmup, a.config, a.backend) == (8, 20, 5, 2, "nccl")
  assert b.parse(["--config", "3"]).steps == 10
  assert b.launches_per_sweep(20, 4) == 5 and b.launches_per_sweep(7, 4) == 3


def test_bench_accounting_helpers():
  """The bench's launch chunking mirrors the library's halving (dg_advec.hip chunk_rec: a
  20-step sweep at 10 per launch is 10 + 10, at 20 one launch, 17 at 10 is 10 + 5 + 2) and
  the even/odd flop counts behind roofline_fp64 (53 forward, 57.4 adjoint flop
  per DOF-update at N = 4; per element-stage 4 + 5 Np + 4 NE NO and 6 + 5 Np + 4 NE NO)."""
  sys.path.insert(0, ROOT)
  import bench
  assert bench.sweep_chunks(20, 10) == [10, 10]
  assert bench.sweep_chunks(20, 20) == [20]
  assert bench.sweep_chunks(17, 10) == [10, 5, 2]
  assert bench.sweep_chunks(20, 8) == [8, 8, 4]
  assert bench.sweep_chunks(23, 16) == [16, 4, 2, 1]
  assert bench.eo_flops_per_update(5, False) == 53.0
  assert abs(bench.eo_flops_per_update(5, True) - 57.4) < 1e-12
  for Np in range(2, 10):  # fewer flops than SURVEY 8d's dense count 5 (2 Np + 11)
    assert bench.eo_flops_per_update(Np, False) < 5 * (2 * Np + 11)


def test_rank_device_binds_rccl_to_one_gpu_per_rank():
  """init_dist's plan: RCCL ranks get their own GPU and the process group
  is bound to it (device_id); more ranks than GPUs is refused with a clear message, not left
  to RCCL; gloo shares GPUs round-robin (the one-GPU-box tests); one rank needs no group."""
  b = _bench()
  assert b.rank_device("nccl", 8, 3, 8, 8) == (3, {"backend": "nccl", "device_id": 3})
  with pytest.raises(RuntimeError, match="one GPU per rank"):
    b.rank_device("nccl", 2, 1, 2, 1)
  assert b.rank_device("gloo", 2, 1, 2, 1) == (0, {"backend": "gloo"})
  assert b.rank_device("nccl", 1, 0, 1, 1) == (0, None)
  with pytest.raises(RuntimeError, match="needs a ROCm GPU"):
    b.rank_device("nccl", 1, 0, 1, 0)


def test_bench_p_indicator_accounting():
  """--indicator p implies the snapshot forward; k_adj_p's flop count (prolongation +
  order-(N+1) forward step + residual pairing + order-(N+1) reverse step per element-step)
  exceeds the jump adjoint's, and the halo factor is T / (T - 2H)."""
  b = _bench()
  a = b.parse(["--indicator", "p"])
  assert a.record == "snapshots" and a.indicator == "p"
  for Np in range(2, 9):
    assert b.p_flops_per_update(Np) > b.eo_flops_per_update(Np + 1, True)
  assert b.halo_factor(1024, 50) == 1024 / 924.0
