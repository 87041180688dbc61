"""Operator and mesh dumps compatible with utils/Save_to_1D_global_data.m:
the StartUp1D/Globals1D variables written one matrix per ``<name>.txt`` the way MATLAB's
``writematrix`` writes them (comma-delimited rows, up to 15 significant digits, index maps
1-based), so a MATLAB session and this package can cross-check each other's setup.

``save_global_data`` writes the files of Save_to_1D_global_data.m:1-34 for a
:class:`~.galerkin.BaseGalerkin1D`; ``load_global_data`` reads such a directory back
(either writer's), returning numpy arrays in MATLAB orientation.
"""
import os

import numpy as np

from .galerkin import BaseGalerkin1D

# Globals1D.m:19-34 (row vectors there)
RK4A = np.array([0.0, -567301805773.0 / 1357537059087.0, -2404267990393.0 / 2016746695238.0,
                 -3550918686646.0 / 2091501179385.0, -1275806237668.0 / 842570457699.0])
RK4B = np.array([1432997174477.0 / 9575080441755.0, 5161836677717.0 / 13612068292357.0,
                 1720146321549.0 / 2090206949498.0, 3134564353537.0 / 4481467310338.0,
                 2277821191437.0 / 14882151754819.0])
RK4C = np.array([0.0, 1432997174477.0 / 9575080441755.0, 2526269341429.0 / 6820363962896.0,
                 2006345519317.0 / 3224310063776.0, 2802321613138.0 / 2924317926251.0])

# Save_to_1D_global_data.m:1-34, in its order
NAMES = ("Dr", "EToE", "EToF", "Fmask", "Fscale", "Fx", "invV", "J", "K", "LIFT", "mapB", "mapI",
         "mapO", "N", "Nfaces", "Nfp", "NODETOL", "Np", "nx", "r", "rk4a", "rk4b", "rk4c", "rx",
         "V", "vmapB", "vmapI", "vmapM", "vmapO", "vmapP", "VX", "x", "dt")


def matlab_globals(g: BaseGalerkin1D, dt=None):
  """The Globals1D variables of mesh g in MATLAB orientation and 1-based indexing."""
  col = lambda a: np.asarray(a).reshape(-1, 1)  # noqa: E731
  return {
      "Dr": g.d_r, "EToE": g.e_to_e + 1, "EToF": g.e_to_f + 1,
      "Fmask": (g.f_mask + 1).reshape(1, -1),  # StartUp1D.m:28 (row)
      "Fscale": g.f_scale, "Fx": g.f_x, "invV": g.inv_v, "J": g.j_mat, "K": g.k,
      "LIFT": g.lift, "mapB": col(g.map_b + 1), "mapI": g.map_i + 1, "mapO": g.map_o + 1,
      "N": g.n, "Nfaces": g.n_faces, "Nfp": g.n_fp, "NODETOL": g.node_tol, "Np": g.n_p,
      "nx": g.n_x, "r": col(g.r_gl), "rk4a": RK4A.reshape(1, -1), "rk4b": RK4B.reshape(1, -1),
      "rk4c": RK4C.reshape(1, -1), "rx": g.r_x, "V": g.v, "vmapB": col(g.v_map_b + 1),
      "vmapI": g.v_map_i + 1, "vmapM": col(g.v_map_m + 1), "vmapO": g.v_map_o + 1,
      "vmapP": col(g.v_map_p + 1), "VX": np.asarray(g.v_x).reshape(1, -1), "x": g.x,
      "dt": g.cfl_dt() if dt is None else dt,
  }


def _fmt(v):
  if float(v).is_integer() and abs(v) < 1e15:
    return str(int(v))
  return f"{v:.15g}"


def save_global_data(g: BaseGalerkin1D, outdir, dt=None):
  """Write the Save_to_1D_global_data.m files for mesh g into outdir; returns the paths."""
  os.makedirs(outdir, exist_ok=True)
  data = matlab_globals(g, dt)
  paths = []
  for name in NAMES:
    a = np.atleast_2d(np.asarray(data[name], dtype=np.float64))
    path = os.path.join(outdir, f"{name}.txt")
    with open(path, "w") as f:
      for row in a:
        f.write(",".join(_fmt(v) for v in row) + "\n")
    paths.append(path)
  return paths


def load_global_data(indir):
  """Read every <name>.txt of Save_to_1D_global_data.m back (2-D float arrays)."""
  out = {}
  for name in NAMES:
    path = os.path.join(indir, f"{name}.txt")
    if os.path.exists(path):
      out[name] = np.atleast_2d(np.loadtxt(path, delimiter=",", ndmin=2))
  return out
