"""ctypes binding of the HIP C ABI (include/dg_advec.h).

There is no CPU fallback: if ``lib/libdgadv.so`` is missing or fails to load, every
entry point raises :class:`DGLibraryError`.  Build it with ``__graft_entry__.build()``
(or ``python -m`` the package's ``build_ext``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DG_LIB_PATH: an experiment variant built by build_ext --out (A/B runs only); default: the
# in-tree product library.
LIB_PATH = os.environ.get("DG_LIB_PATH") or os.path.join(_HERE, "lib", "libdgadv.so")
HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "include", "dg_advec.h"))

# Enumerations of include/dg_advec.h
DG_OK, DG_ERR_ARG, DG_ERR_HIP, DG_ERR_NOMEM = 0, -1, -2, -3
DG_INFLOW_SIN_AT, DG_INFLOW_SIN_A2T, DG_INFLOW_ZERO = 0, 1, 2
DG_TIME_LSERK4, DG_TIME_EULER = 0, 1
DG_TUNE_TILE_WIDTH, DG_TUNE_STEPS_PER_LAUNCH, DG_TUNE_XCD_ORDER = 1, 2, 3
DG_TUNE_LANE_ELEMENTS = 4
DG_TUNE_REC_TILE_WIDTH, DG_TUNE_REC_STEPS_PER_LAUNCH = 5, 6
DG_TUNE_REC_LANE_ELEMENTS, DG_TUNE_REC_FWD_STEPS_PER_LAUNCH = 7, 8
DG_TUNE_P_TILE_WIDTH, DG_TUNE_P_STEPS_PER_LAUNCH = 9, 10
DG_TUNE_REC_FWD_TILE_WIDTH = 11
DG_TUNE_REC_SWEEP = 12
DG_TUNE_SWEEP_SPIN_LIMIT = 13
DG_TUNE_SWEEP_WAVES = 14
DG_TUNE_SWEEP_LANE_ELEMENTS = 15
DG_TUNE_SWEEP_TAKE = 16
DG_TUNE_SWEEP_EXCHANGE = 17
DG_TUNE_SNAP_PAIRS = 18
DG_TUNE_P_FLOW = 19
DG_TUNE_P_SWEEP = 20
DG_TUNE_NL_EXCHANGE = 21
DG_FLUX_LINEAR, DG_FLUX_BURGERS = 0, 1
DG_LIMIT_NONE, DG_LIMIT_EACH_STAGE, DG_LIMIT_PI1_EACH_STAGE = 0, 1, 2
DG_ADJ_ETA_ASSIGN, DG_ADJ_ETA_ABS = 1, 2
DG_ADJ_P_TERMINAL_PROLONG = 8
DG_SWEEP_TERMINAL_STATE = 4

_c_dbl_p = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int

# name -> (restype, argtypes); device pointers are passed as c_void_p integers.
SIGNATURES = {
    "dg_last_error": (ctypes.c_char_p, []),
    "dg_version": (ctypes.c_char_p, []),
    "dg_plan_create": (_i32, [_i32, _i64, _i64, _c_dbl_p, _c_dbl_p, _c_dbl_p, _c_dbl_p, _c_dbl_p,
                              _c_dbl_p, ctypes.c_double, _i32, _i32, ctypes.POINTER(_vp)]),
    "dg_plan_destroy": (_i32, [_vp]),
    "dg_plan_query": (_i32, [_vp, ctypes.POINTER(_i64)]),
    "dg_plan_tune": (_i32, [_vp, _i32, _i64]),
    "dg_plan_set_physics": (_i32, [_vp, _i32, _i32]),
    "dg_plan_set_tvb": (_i32, [_vp, ctypes.c_double]),
    "dg_plan_reserve": (_i32, [_vp, _i64]),
    "dg_plan_refine": (_i32, [_vp, _vp, _vp, _vp]),
    "dg_plan_get_mesh": (_i32, [_vp, _c_dbl_p]),
    "dg_advec_rhs": (_i32, [_vp, _vp, _vp, ctypes.c_double, _vp]),
    "dg_lserk4_fwd": (_i32, [_vp, _vp, ctypes.c_double, ctypes.c_double, _i32, _vp, _vp]),
    "dg_lserk4_adj": (_i32, [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _i32,
                             ctypes.c_double, _vp, _vp]),
    "dg_lserk4_adj_ex": (_i32, [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _i32,
                                ctypes.c_double, _vp, _i32, _vp, _vp]),
    "dg_lserk4_fwd_ex": (_i32, [_vp, _vp, ctypes.c_double, ctypes.c_double, _i32, _vp, _vp,
                                _vp]),
    "dg_plan_query_rec": (_i32, [_vp, _vp]),
    "dg_plan_query_rec_fwd": (_i32, [_vp, _vp]),
    "dg_plan_query_nl": (_i32, [_vp, _vp]),
    "dg_lserk4_fwd_rec": (_i32, [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _i32, _vp,
                                 _vp]),
    "dg_lserk4_adj_rec": (_i32, [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _i32, _vp,
                                 _i32, _vp]),
    "dg_lserk4_sweep_rec": (_i32, [_vp, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                   _i32, _vp, _i32, _vp]),
    "dg_lserk4_sweep_refine": (_i32, [_vp, _vp, _vp, _vp, _vp, ctypes.c_double,
                                      ctypes.c_double, _i32, _vp, _i32, _vp, _vp, _vp, _vp]),
    "dg_plan_query_sweep": (_i32, [_vp, _i32, _vp]),
    "dg_plan_query_sweep_ex": (_i32, [_vp, _i32, _vp]),
    "dg_plan_query_sweep_kernel": (_i32, [_vp, _i32, _vp]),
    "dg_sweep_status": (_i32, [_vp, ctypes.POINTER(_i32), _vp]),
    "dg_plan_sweep_trace": (_i32, [_vp, _vp]),
    "dg_plan_query_p": (_i32, [_vp, _vp]),
    "dg_prolong": (_i32, [_vp, _vp, _c_dbl_p, _vp, _vp, _vp]),
    "dg_lserk4_adj_p": (_i32, [_vp, _vp, _c_dbl_p, _vp, _vp, ctypes.c_double, ctypes.c_double,
                               _i32, _vp, _i32, _vp]),
    "dg_lserk4_adj_p_refine": (_i32, [_vp, _vp, _c_dbl_p, _vp, _vp, ctypes.c_double,
                                      ctypes.c_double, _i32, _vp, _i32, _vp, _vp, _vp, _vp]),
    "dg_plan_query_p_flow": (_i32, [_vp, _i32, ctypes.POINTER(_i32)]),
    "dg_plan_query_p_sweep": (_i32, [_vp, _i32, ctypes.POINTER(_i32)]),
    "dg_plan_query_p_trace": (_i32, [_vp, _i32, _vp]),
    "dg_lserk4_sweep_p": (_i32, [_vp, _vp, _c_dbl_p, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                 _i32, _vp, _i32, _vp, _vp, _vp, _vp]),
    "dg_slope_limit_n": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "dg_slope_limit_1": (_i32, [_vp, _vp, _vp, _vp]),
    "dg_argmax": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "dg_argmax_ex": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "dg_stream_copy": (_i32, [_vp, _vp, _i64, _vp]),
    "dg_host_alias": (_i32, [_vp, ctypes.POINTER(_vp)]),
    "dg_sum_rows": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "dg_slice_candidate": (_i32, [_vp, _vp, _i64, _i64, _i64, ctypes.c_double, _i64, _vp, _vp]),
    "dg_candidates_argmax": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "dg_init_sine": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "dg_time_march": (_i32, [_i32, _i32, _vp, _vp, _vp, _i32, _vp, _i64, _vp, ctypes.c_double,
                             _i32, _vp, _vp, _vp]),
    "dg_time_adjoint": (_i32, [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp,
                               _vp, _vp, _vp, _vp]),
    "dg_fd_adapt_sweep": (_i32, [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp]),
}


class DGLibraryError(RuntimeError):
  """The HIP extension is missing, failed to load, or a call returned an error code."""


_lib = None


def load():
  """Load the shared library once; raise loudly if it is absent (no fallback)."""
  global _lib
  if _lib is not None:
    return _lib
  if not os.path.exists(LIB_PATH):
    raise DGLibraryError(
        f"HIP extension not built: {LIB_PATH} is missing. Run `python -c \"import "
        f"__graft_entry__; __graft_entry__.build()\"` from the repository root.")
  try:
    lib = ctypes.CDLL(LIB_PATH)
  except OSError as e:
    raise DGLibraryError(f"failed to load {LIB_PATH}: {e}") from e
  for name, (res, args) in SIGNATURES.items():
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args
  _lib = lib
  return lib


def check(rc, what=""):
  if rc != DG_OK:
    msg = load().dg_last_error().decode(errors="replace")
    raise DGLibraryError(f"{what} failed with code {rc}: {msg}")


def dbl_array(values):
  """Host float64 buffer for the plan-creation arguments."""
  import numpy as np
  arr = np.ascontiguousarray(values, dtype=np.float64)
  return arr, arr.ctypes.data_as(_c_dbl_p)
