"""One p one-launch sweep (tests/test_gpu_psweep.py's first case) with the HIP runtime's error
log on: diagnosing DG_P_SWEEP_W=3."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import importlib  # noqa: E402
pkg = importlib.import_module("adjoint-ode-adaptivity_amd")
import test_gpu_psweep as t  # noqa: E402

gpu = torch.device("cuda:0")
op, est, u0, dt = t.setup(pkg, gpu, 4, 3000)
a = t.chain(op, est, u0, dt, 20)
print("chain ok", flush=True)
b = t.fused(op, est, u0, dt, 20)
print("fused ok", flush=True)
t.assert_same(b, a, "W env " + os.environ.get("DG_P_SWEEP_W", "-"))
print("same", flush=True)
