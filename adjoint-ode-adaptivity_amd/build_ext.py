"""Build the HIP extension in-tree: csrc/*.hip -> lib/libdgadv.so (gfx950).

Each translation unit is compiled to an object in parallel (they are template-heavy), then
linked into one shared library.  hipcc cross-compiles without a GPU; the .so travels to the
GPU box with the tree.
"""
import os
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(_HERE, "csrc", f) for f in ("dg_advec.hip", "dg_burgers.hip", "dg_wave.hip", "dg_time.hip", "dg_fd.hip",
                                                     "dg_util.hip", "dg_rec.hip", "dg_dwr.hip",
                                                     "dg_sweep.hip")]
COMMON = os.path.join(_HERE, "csrc", "dg_common.h")
HEADERS = [COMMON, os.path.join(_HERE, "csrc", "dg_rec_tiles.h")]
INCLUDE = os.path.normpath(os.path.join(_HERE, "..", "include"))
OUT = os.path.join(_HERE, "lib", "libdgadv.so")
ARCH = os.environ.get("DG_OFFLOAD_ARCH", "gfx950")


def hipcc():
  for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
    if cand and os.path.exists(cand):
      return cand
  raise RuntimeError("hipcc not found (ROCm is required to build the HIP extension)")


def build(force=False, verbose=True, extra_flags=(), out=None, srcdir=None):
  """Build lib/libdgadv.so; `out` + `extra_flags` build an experiment variant elsewhere
  (its own object directory; the product library is untouched); `srcdir`: a patched copy of
  csrc/ for such a variant (A/B runs)."""
  OUT_ = OUT if out is None else os.path.abspath(out)
  srcs, headers = SRCS, HEADERS
  if srcdir is not None:
    srcs = [os.path.join(srcdir, os.path.basename(f)) for f in SRCS]
    headers = [os.path.join(srcdir, os.path.basename(f)) for f in HEADERS]
  deps = srcs + headers + [os.path.join(INCLUDE, "dg_advec.h")]
  if (not force and os.path.exists(OUT_)
      and os.path.getmtime(OUT_) >= max(os.path.getmtime(d) for d in deps)):
    if verbose:
      print(f"[build_ext] up to date: {OUT_}")
    return OUT_
  os.makedirs(os.path.dirname(OUT_), exist_ok=True)
  objdir = os.path.join(os.path.dirname(OUT_), "obj" if out is None else
                        "obj_" + os.path.basename(OUT_).replace(".so", ""))
  os.makedirs(objdir, exist_ok=True)
  flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-I", INCLUDE, *extra_flags]
  procs, objs = [], []
  shared = max(os.path.getmtime(d) for d in deps[len(srcs):])
  for src in srcs:
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    objs.append(obj)
    if (not force and os.path.exists(obj)
        and os.path.getmtime(obj) >= max(os.path.getmtime(src), shared)):
      continue  # this translation unit is up to date
    cmd = [hipcc(), *flags, "-c", "-o", obj, src]
    if verbose:
      print("[build_ext]", " ".join(cmd))
    procs.append((subprocess.Popen(cmd), src))
  failed = [src for p, src in procs if p.wait() != 0]
  if failed:
    raise RuntimeError(f"hipcc failed on {failed}; {OUT_} was NOT updated")
  tmp = OUT_ + ".tmp"
  cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
  if verbose:
    print("[build_ext]", " ".join(cmd))
  if subprocess.run(cmd).returncode != 0:
    raise RuntimeError(f"link failed; {OUT_} was NOT updated")
  os.replace(tmp, OUT_)
  return OUT_


if __name__ == "__main__":
  import argparse
  ap = argparse.ArgumentParser()
  ap.add_argument("--force", action="store_true")
  ap.add_argument("--out", default=None, help="variant library path (experiments)")
  ap.add_argument("-D", action="append", default=[], help="extra -D defines")
  ap.add_argument("--srcdir", default=None, help="patched csrc/ copy for a variant")
  a = ap.parse_args()
  build(force=a.force, out=a.out, extra_flags=tuple("-D" + d for d in a.D), srcdir=a.srcdir)
