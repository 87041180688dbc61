"""Generate golden vectors for the finite-difference DWR adapt loop.

Run ONCE in the build container (the only place /root/reference exists):

    python tests/golden/make_fd_golden.py

It imports the reference module ``python/Main_finite_difference.py`` (the
functions ``refineAll``, ``interpU``, ``forwardSolve``, ``adjSolve`` and
``errEst`` at lines 16-94) with a stub for ``cv2`` (only used by the
``__main__`` video writer, lines 345-358), and replays the ``__main__`` adapt
loop (lines 263-343) headlessly with the configuration it hard-codes there:

* ODE ``du/dt = sin(u)`` forward-Euler update (lines 131-140),
* output functional ``J = int(u^2)``: ``getK = 2 u[:-1] dt`` (lines 225-227),
* ``t in [0, 2]``, 2 initial steps, ``u0 = 1``, ``ref_factor = 4``
  (lines 105-108, 247, 251), ``tol = 1e-5``, ``maxit = 100`` (lines 259-261).

The callbacks are re-declared here because they live under ``__main__`` and
cannot be imported; they are the INPUTS of the golden run, not product code.
The output ``fd_adapt_golden.json`` is pure data (inputs + reference outputs).
Nothing under tests/ imports the reference at test time.
"""
import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference/python/Main_finite_difference.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fd_adapt_golden.json")


def load_reference():
  sys.modules.setdefault("cv2", types.ModuleType("cv2"))
  spec = importlib.util.spec_from_file_location("fd_reference", REF)
  mod = importlib.util.module_from_spec(spec)
  spec.loader.exec_module(mod)
  return mod


def main(max_iterations=40):
  ref = load_reference()
  ref_factor = 4
  ref.ref_factor = ref_factor  # interpU reads this module global (line 25)

  def fwdUpdate(u, dt_n, n):  # Main_finite_difference.py:131-132
    return u[n - 1] + np.sin(u[n - 1]) * dt_n[n - 1]

  def getJF(u, dt_n):  # :138-140
    return np.diag(1 + np.cos(u[:-1]) * dt_n, -1)

  def getK(dt_n, u, v0=0):  # :225-227
    return np.concatenate((2 * u[:-1] * dt_n, v0), axis=None)

  times = np.linspace(0.0, 2.0, 3)
  u0 = 1.0
  it, maxit, err, tol = 0, 100, 1.0, 1e-5
  iterations = []
  while it <= maxit and err > tol and it < max_iterations:  # :263
    dt_n = np.diff(times, 1)
    n_steps = len(dt_n)
    u = ref.forwardSolve(fwdUpdate, dt_n, u0)
    v = ref.adjSolve(getK, getJF, dt_n, u, ref_factor)
    raw = ref.errEst(fwdUpdate, u, v, dt_n, ref_factor)
    err_abs = np.abs(raw)[2:]
    n_rows = (err_abs.size - (ref_factor - 1)) // ref_factor + 1
    s = err_abs.strides[0]
    win = np.lib.stride_tricks.as_strided(err_abs, shape=(n_rows, ref_factor - 1),
                                          strides=(ref_factor * s, s))
    err_steps = np.sum(win, 1)
    ref_idx = int(np.argmax(err_steps) + 1)  # :337
    iterations.append({
        "times": times.tolist(),
        "u": u.tolist(),
        "v": v.tolist(),
        "err_fine": raw.tolist(),
        "err_steps": err_steps.tolist(),
        "ref_idx": ref_idx,
    })
    times_new = np.zeros(n_steps + 2)  # :336-341
    times_new[0:ref_idx] = times[0:ref_idx]
    times_new[ref_idx + 1:] = times[ref_idx:]
    times_new[ref_idx] = np.mean(times[ref_idx - 1:ref_idx + 1])
    times = times_new
    err = np.sum(err_steps)
    it += 1

  data = {
      "source": "wglao/Adjoint-ODE-Adaptivity python/Main_finite_difference.py "
                "(functions :16-94, __main__ loop :263-343), replayed headless",
      "config": {"ode": "du/dt=sin(u)", "functional": "J=int(u^2)", "t_span": [0.0, 2.0],
                 "n_steps0": 2, "u0": u0, "ref_factor": ref_factor, "tol": tol, "maxit": maxit},
      "terminated_by_tol": bool(err <= tol),
      "iterations": iterations,
  }
  with open(OUT, "w") as f:
    json.dump(data, f, indent=1)
  print("wrote", OUT, "iterations:", len(iterations),
        "ref_idx:", [d["ref_idx"] for d in iterations])


if __name__ == "__main__":
  main()
