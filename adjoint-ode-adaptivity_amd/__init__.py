"""MI355X-native forward + adjoint nodal-DG advection time-stepper.

Drop-in for the hot path of wglao/Adjoint-ODE-Adaptivity (1D DG advection:
AdvecRHS1D + LSERK4 forward sweep, discrete adjoint sweep with the dual-weighted
residual indicator, SlopeLimitN, argmax refinement) behind the C ABI of
include/dg_advec.h.  The directory name contains hyphens, so import it with
``importlib.import_module("adjoint-ode-adaptivity_amd")``.

Submodules:
  galerkin   host-side setup with the BaseGalerkin1D attribute surface (numpy)
  operators  DGAdvection1D: the HIP plan and its kernels (torch CUDA tensors)
  factory    Problem / Funs / AdaptFuns / AdaptState / FunFactory adapt-loop API
  ensemble   ensembles of initial conditions sharded over ranks (rank-ordered RCCL sum)
  adaptive   device-resident spatial adapt loop (config 3: fwd + adj + refine)
  dgtime     batched DG-in-time marches + DWR for ODE ensembles (matlab/MAIN.m loop)
  fd_ensemble  the finite-difference DWR adapt loop for ODE ensembles on the device
  globals_io Save_to_1D_global_data.m-compatible operator/mesh dumps
  checkpoint CheckpointedSweep: adjoint sweeps from every m-th state (recompute in between)
  build_ext  in-tree hipcc build of lib/libdgadv.so
"""
from . import _lib, galerkin  # noqa: F401
from .galerkin import BaseGalerkin1D, split_interval  # noqa: F401

__all__ = ["BaseGalerkin1D", "split_interval", "operators", "factory", "ensemble", "adaptive", "dgtime", "fd_ensemble", "globals_io", "galerkin", "checkpoint"]


def __getattr__(name):
  # torch-dependent modules load on first use (the host setup does not need torch).
  if name in ("operators", "factory", "ensemble", "adaptive", "dgtime", "fd_ensemble", "globals_io",
              "checkpoint"):
    import importlib
    return importlib.import_module(f"{__name__}.{name}")
  if name == "DGAdvection1D":
    from .operators import DGAdvection1D
    return DGAdvection1D
  raise AttributeError(name)
