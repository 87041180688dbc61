"""The C-ABI library loads and exports every entry point include/dg_advec.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dg_advec.h")


def declared_functions():
  src = open(HEADER).read()
  src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
  return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(dg_\w+)\s*\(", src,
                               flags=re.M)))


def test_header_declares_the_contract():
  names = declared_functions()
  for required in ("dg_plan_create", "dg_plan_destroy", "dg_advec_rhs", "dg_lserk4_fwd",
                   "dg_lserk4_adj", "dg_slope_limit_n", "dg_argmax", "dg_last_error"):
    assert required in names


def test_library_exports_every_declared_symbol(pkg):
  lib = pkg._lib.load()
  raw = ctypes.CDLL(pkg._lib.LIB_PATH)
  missing = [n for n in declared_functions() if not hasattr(raw, n)]
  assert not missing, missing
  assert set(pkg._lib.SIGNATURES) == set(declared_functions())
  assert lib.dg_version().decode().startswith("dg_advec")


def test_library_is_built_for_gfx950(pkg):
  data = open(pkg._lib.LIB_PATH, "rb").read()
  assert b"gfx950" in data


def test_argument_errors_cross_the_abi_as_codes(pkg):
  lib = pkg._lib.load()
  out = ctypes.c_void_p()
  import numpy as np
  bufs = [pkg._lib.dbl_array(np.zeros(4))[1] for _ in range(6)]
  rc = lib.dg_plan_create(0, 10, 1, *bufs, 1.0, 0, 0, ctypes.byref(out))  # N = 0: invalid
  assert rc == pkg._lib.DG_ERR_ARG
  assert b"N must be" in lib.dg_last_error()
  assert lib.dg_plan_destroy(None) == 0
  assert lib.dg_advec_rhs(None, None, None, 0.0, None) == pkg._lib.DG_ERR_ARG


def test_missing_library_fails_loudly(pkg, monkeypatch, tmp_path):
  monkeypatch.setattr(pkg._lib, "_lib", None)
  monkeypatch.setattr(pkg._lib, "LIB_PATH", str(tmp_path / "nope.so"))
  with pytest.raises(pkg._lib.DGLibraryError):
    pkg._lib.load()


def test_operator_refuses_cpu(pkg):
  import torch
  if torch.cuda.is_available():
    pytest.skip("GPU present")
  with pytest.raises(pkg._lib.DGLibraryError):
    pkg.operators.DGAdvection1D(pkg.BaseGalerkin1D(n=2, k=8))


def header_enums():
  """name -> value of every `DG_NAME = value` enumerator in include/dg_advec.h."""
  src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
  out = {}
  for body in re.findall(r"enum\s*\{(.*?)\}", src, flags=re.S):
    for name, val in re.findall(r"\b(DG_[A-Z0-9_]+)\s*=\s*(-?\d+)", body):
      out[name] = int(val)
  return out


def test_python_constants_match_the_header(pkg):
  """The ctypes layer's constants are the header's enumerators (a new tuning key or flag
  added on one side only would pass the wrong integer across the ABI)."""
  enums = header_enums()
  assert len(enums) >= 20
  for name, val in enums.items():
    assert hasattr(pkg._lib, name), f"_lib lacks {name}"
    assert getattr(pkg._lib, name) == val, name


def test_tuning_a_null_plan_is_an_argument_error(pkg):
  lib = pkg._lib.load()
  for key in (pkg._lib.DG_TUNE_REC_LANE_ELEMENTS, pkg._lib.DG_TUNE_REC_STEPS_PER_LAUNCH):
    assert lib.dg_plan_tune(None, key, 2) == pkg._lib.DG_ERR_ARG
  out = (ctypes.c_int64 * 4)()
  assert lib.dg_plan_query_rec(None, out) == pkg._lib.DG_ERR_ARG
