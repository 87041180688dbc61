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
SRCS = [os.path.join(_HERE, "csrc", f) for f in ("dg_advec.hip", "dg_burgers.hip", "dg_burgers_ov.hip", "dg_wave.hip", "dg_time.hip", "dg_fd.hip",
                                                     "dg_util.hip", "dg_rec.hip", "dg_dwr.hip",
                                                     "dg_sweep.hip", "dg_sweep_hi.hip",
                                                     "dg_sweep_ov.hip")]
INCLUDE = os.path.normpath(os.path.join(_HERE, "..", "include"))
OUT = os.path.join(_HERE, "lib", "libdgadv.so")
ARCH = os.environ.get("DG_OFFLOAD_ARCH", "gfx950")


def hipcc():
  for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
    if cand and os.path.exists(cand):
      return cand
  raise RuntimeError("hipcc not found (ROCm is required to build the HIP extension)")


def _includes(path, seen=None):
  """The quoted #include files a source pulls in (recursively, csrc/ and include/)."""
  import re
  seen = set() if seen is None else seen
  for line in open(path):
    m = re.match(r'\s*#include\s+"([^"]+)"', line)
    if not m:
      continue
    for d in (os.path.dirname(path), INCLUDE):
      f = os.path.join(d, m.group(1))
      if os.path.exists(f) and f not in seen:
        seen.add(f)
        _includes(f, seen)
        break
  return seen


_LLVM = "/opt/rocm/llvm/bin"


def device_calls(obj):
  """Kernels of an object's gfx950 code object that contain a call (s_swappc_b64).

  Every tile body reads its operator constants through the kernel's own kernarg segment
  pointer (dg_common.h kernarg_tail, dg_rec_tiles.h OpSrc); inside an outlined (called)
  function that pointer is 0 (the round-4 non-inlined variant faulted on it).
  The library therefore must contain no device calls at all: build() fails if one appears."""
  import re
  import tempfile
  with tempfile.TemporaryDirectory() as tmp:
    fat, co = os.path.join(tmp, "fat"), os.path.join(tmp, "co")
    subprocess.run([f"{_LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj,
                    os.path.join(tmp, "junk")], check=True)
    subprocess.run([f"{_LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--output={co}"], check=True)
    dis = subprocess.run([f"{_LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True,
                         text=True).stdout
  bad, cur = set(), None
  for line in dis.splitlines():
    m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
    if m:
      cur = m.group(1)
    elif "s_swappc_b64" in line:
      bad.add(cur)
  return sorted(bad)


def build(force=False, verbose=True, extra_flags=(), out=None, srcdir=None):
  """Build lib/libdgadv.so; `out` + `extra_flags` build an experiment variant elsewhere
  (its own object directory; the product library is untouched); `srcdir`: a patched copy of
  csrc/ for such a variant (A/B runs).  A translation unit is rebuilt when it or a header it
  includes changed.  Fails if any kernel calls a device function (device_calls)."""
  OUT_ = OUT if out is None else os.path.abspath(out)
  srcs = SRCS
  if srcdir is not None:
    srcs = [os.path.join(srcdir, os.path.basename(f)) for f in SRCS]
  deps = {src: [src, *_includes(src)] for src in srcs}
  newest = max(os.path.getmtime(d) for ds in deps.values() for d in ds)
  if not force and os.path.exists(OUT_) and os.path.getmtime(OUT_) >= newest:
    if verbose:
      print(f"[build_ext] up to date: {OUT_}")
    return OUT_
  os.makedirs(os.path.dirname(OUT_), exist_ok=True)
  objdir = os.path.join(os.path.dirname(OUT_), "obj" if out is None else
                        "obj_" + os.path.basename(OUT_).replace(".so", ""))
  os.makedirs(objdir, exist_ok=True)
  flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-I", INCLUDE, *extra_flags]
  procs, objs = [], []
  for src in srcs:
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    objs.append(obj)
    if (not force and os.path.exists(obj)
        and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps[src])):
      continue  # this translation unit is up to date
    cmd = [hipcc(), *flags, "-c", "-o", obj, src]
    if verbose:
      print("[build_ext]", " ".join(cmd))
    procs.append((subprocess.Popen(cmd), src, obj))
  failed = [src for p, src, _ in procs if p.wait() != 0]
  if failed:
    raise RuntimeError(f"hipcc failed on {failed}; {OUT_} was NOT updated")
  calls = {os.path.basename(src): device_calls(obj) for _, src, obj in procs}
  calls = {k: v for k, v in calls.items() if v}
  if calls:
    for _, _, obj in procs:
      os.remove(obj)
    raise RuntimeError(f"device calls (an outlined tile body?) in {calls}; {OUT_} was NOT "
                       "updated")
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
