"""Build the HIP extension in-tree: csrc/dg_advec.hip -> lib/libdgadv.so (gfx950).

hipcc cross-compiles without a GPU; the .so travels to the GPU box with the tree.
"""
import os
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(_HERE, "csrc", "dg_advec.hip")
INCLUDE = os.path.normpath(os.path.join(_HERE, "..", "include"))
OUT = os.path.join(_HERE, "lib", "libdgadv.so")
ARCH = os.environ.get("DG_OFFLOAD_ARCH", "gfx950")


def hipcc():
  for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
    if cand and os.path.exists(cand):
      return cand
  raise RuntimeError("hipcc not found (ROCm is required to build the HIP extension)")


def build(force=False, verbose=True, extra_flags=()):
  deps = [SRC, os.path.join(INCLUDE, "dg_advec.h")]
  if (not force and os.path.exists(OUT)
      and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps)):
    if verbose:
      print(f"[build_ext] up to date: {OUT}")
    return OUT
  os.makedirs(os.path.dirname(OUT), exist_ok=True)
  tmp = OUT + ".tmp"
  cmd = [hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
         "-I", INCLUDE, *extra_flags, "-o", tmp, SRC]
  if verbose:
    print("[build_ext]", " ".join(cmd))
  r = subprocess.run(cmd)
  if r.returncode != 0:
    raise RuntimeError(f"hipcc failed ({r.returncode}); {OUT} was NOT updated")
  os.replace(tmp, OUT)
  return OUT


if __name__ == "__main__":
  build(force="--force" in sys.argv)
