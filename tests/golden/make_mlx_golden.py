"""Extract the cached MATLAB outputs of the reference live script into a fixture.

Run ONCE in the build container (the only place /root/reference exists):

    python tests/golden/make_mlx_golden.py

``utils/One_code.mlx`` is a zip; ``matlab/output.xml`` holds the values MATLAB
R2020b displayed when the script was last run (N=2, K=20 on [0,1],
u0=sin(2*pi*x), a=2*pi, FinalTime=2, inflow uin=-sin(a*a*t); live-script lines
106-140).  Each displayed variable is stored with its live-script line number.
Values are shown to 4 decimals, so they pin the oracle to 5e-5 absolute.

Output: ``one_code_mlx_golden.json`` (pure data: variable name, line, shape,
values as displayed).  Truncated displays (MATLAB prints only the first rows
of tall matrices) are kept as the rows shown, flagged ``truncated``.
"""
import html
import json
import os
import re
import zipfile

MLX = "/root/reference/utils/One_code.mlx"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "one_code_mlx_golden.json")


def parse():
  with zipfile.ZipFile(MLX) as z:
    xml = z.read("matlab/output.xml").decode("utf-8")
  elems = re.findall(
      r"<element><type>(.*?)</type><outputData>(.*?)</outputData>"
      r"<lineNumbers type=\"array\">(.*?)</lineNumbers></element>", xml, re.S)
  out = []
  for kind, od, ln in elems:
    if kind not in ("matrix", "variable"):
      continue
    name = re.search(r"<name>(.*?)</name>", od).group(1)
    val = html.unescape(re.search(r"<value>(.*?)</value>", od, re.S).group(1))
    line = int(re.findall(r"<element>(\d+)</element>", ln)[0])
    rows = [[float(t) for t in r.split()] for r in val.strip().splitlines() if r.strip()]
    shape = None
    vs = re.search(r"<varSize>(.*?)</varSize>", od)
    if vs:
      shape = [int(t) for t in vs.group(1).split("×")]
    else:
      shape = [1, 1]
    truncated = len(rows) != shape[0]
    out.append({"name": name, "line": line, "shape": shape, "rows": rows,
                "truncated": truncated})
  return out


def main():
  entries = parse()
  data = {
      "source": "wglao/Adjoint-ODE-Adaptivity utils/One_code.mlx -> matlab/output.xml "
                "(MATLAB R2020b cached outputs, 4-decimal display)",
      "config": {"N": 2, "K": 20, "xmin": 0.0, "xmax": 1.0, "a": "2*pi", "FinalTime": 2.0,
                 "u0": "sin(2*pi*x)", "inflow": "-sin(a*a*t)", "CFL": 0.75, "dt_factor": 0.5},
      "display_atol": 5e-5,
      "entries": entries,
  }
  with open(OUT, "w") as f:
    json.dump(data, f, indent=1)
  print("wrote", OUT, [(e["name"], e["line"]) for e in entries])


if __name__ == "__main__":
  main()
