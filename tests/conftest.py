import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs the HIP kernels)")
  config.addinivalue_line("markers", "slow: long-running test")


def load_pkg():
  return importlib.import_module("adjoint-ode-adaptivity_amd")


@pytest.fixture(scope="session")
def pkg():
  return load_pkg()


@pytest.fixture(scope="session")
def gpu():
  import torch
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  return torch.device("cuda", 0)
