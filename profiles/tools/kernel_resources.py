"""Register / LDS / spill usage of the gfx950 kernels in a built object or library.

usage: python profiles/tools/kernel_resources.py <obj-or-.so> [name-regex]
Extracts the .hip_fatbin offload bundle, unbundles the gfx950 code object and prints each
kernel's VGPRs, SGPRs, spills, LDS bytes and waves per SIMD from its AMDGPU metadata notes.
"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/llvm/bin"


def code_object(path, tmp):
  fat = os.path.join(tmp, "fatbin")
  subprocess.run([f"{B}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", path, os.path.join(tmp, "junk")],
                 check=True)
  co = os.path.join(tmp, "co")
  subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                  "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
  return co


def kernels(co):
  out = subprocess.run([f"{B}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
  ks, cur = [], None
  for line in out.splitlines():
    m = re.match(r"\s*-?\s*\.(\w+):\s*(.*)", line)
    if not m:
      continue
    k, v = m.group(1), m.group(2).strip()
    if k == "args":
      continue
    if k == "name" and not v.endswith(".kd"):
      cur = {"name": v}
      ks.append(cur)
    elif cur is not None:
      cur[k] = v
  return ks


if __name__ == "__main__":
  path = sys.argv[1]
  pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
  with tempfile.TemporaryDirectory() as tmp:
    for k in kernels(code_object(path, tmp)):
      if pat and not pat.search(k["name"]):
        continue
      print(f'{k["name"]}: vgpr {k.get("vgpr_count")} agpr {k.get("agpr_count")} sgpr {k.get("sgpr_count")} '
            f'vspill {k.get("vgpr_spill_count")} sspill {k.get("sgpr_spill_count")} '
            f'lds {k.get("group_segment_fixed_size")} scratch {k.get("private_segment_fixed_size")}')
