"""CPU study: effectivity and ranking quality of the DG-advection DWR indicators
(oracle/effectivity.py).  Writes profiles/r02/effectivity.json.

  python profiles/effectivity_study.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import effectivity as ef  # noqa: E402


def bump(x):
  return np.exp(-300.0 * (x - 0.3) ** 2)


def main():
  rows = []
  for N, K in [(1, 16), (1, 32), (2, 16), (2, 32), (3, 16), (4, 16), (4, 32)]:
    o = ef.study(N, K, 0.05, bump)
    keep = {k: v for k, v in o.items() if not isinstance(v, np.ndarray)}
    rows.append(keep)
    print(f"N={N} K={K}: err_exact {o['err_exact']:.3e} err_h/2 {o['err_h2']:.3e} "
          f"sum eta_jump {o['sum_eta_jump']:.3e} (eff {o['effectivity_jump_vs_exact']:.3g}) "
          f"sum eta_p {o['sum_eta_p']:.3e} (eff vs p+1 {o['effectivity_p_vs_p1']:.12f}, vs exact "
          f"{o['effectivity_p_vs_exact']:.3f}); Spearman vs gain: jump "
          f"{o['spearman_jump']:.3f} p {o['spearman_p']:.3f}; argmax jump/p/gain "
          f"{o['argmax_jump']}/{o['argmax_p']}/{o['argmax_gain']}")
  out = os.path.join(ROOT, "profiles", "r02", "effectivity.json")
  with open(out, "w") as f:
    json.dump({"problem": "u0 = exp(-300 (x-0.3)^2), a = 2 pi, zero inflow, T = 0.05, "
                          "J = int psi(x) u(x,T) dx, psi = cos^4 window at 0.62 +- 0.08; "
                          "gain_k = |J(u on the mesh with element k split) - J(u_h)|",
               "rows": rows}, f, indent=1)
  print("wrote", out)


if __name__ == "__main__":
  main()
