"""build_ext's static check that no kernel calls a device function.

Every tile body reads operator constants through the kernel's kernarg segment pointer, which
is 0 inside a called function, so build() fails when a body is outlined.  Here
the check runs on two small probes compiled for gfx950 (no GPU needed): a kernel whose body
reads its kernarg tail through a __noinline__ function must be reported, the same body
force-inlined must not.  (profiles/r05/outline_check.log shows build() refusing the library
with ov_step_tile made __noinline__.)"""
import importlib
import os
import shutil
import subprocess

import pytest

PROBE = r'''
#include <hip/hip_runtime.h>
struct A { double c[4]; };
__device__ INLINE double body(int i) {
  const double* k = (const double*)__builtin_amdgcn_kernarg_segment_ptr();
  return k[(i & 3) + 1];
}
__global__ void k_probe(double* out, A a) { out[threadIdx.x] = body(threadIdx.x) + a.c[0]; }
'''


@pytest.mark.parametrize("inline,reported", [("__noinline__", True), ("__forceinline__", False)])
def test_device_call_check_flags_outlined_bodies(tmp_path, inline, reported):
  build_ext = importlib.import_module("adjoint-ode-adaptivity_amd.build_ext")
  try:
    hipcc = build_ext.hipcc()
  except RuntimeError:
    pytest.skip("hipcc not available")
  src = tmp_path / "probe.hip"
  src.write_text(PROBE.replace("INLINE", inline))
  obj = tmp_path / "probe.o"
  subprocess.run([hipcc, "-O3", f"--offload-arch={build_ext.ARCH}", "-c", "-o", str(obj),
                  str(src)], check=True)
  calls = build_ext.device_calls(str(obj))
  assert bool(calls) == reported, calls
  if reported:
    assert any("k_probe" in c for c in calls)


def test_shipped_objects_have_no_device_calls():
  """The in-tree objects build() linked contain no call (the check build() applies)."""
  build_ext = importlib.import_module("adjoint-ode-adaptivity_amd.build_ext")
  objdir = os.path.join(os.path.dirname(build_ext.OUT), "obj")
  objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in build_ext.SRCS]
  objs = [o for o in objs if os.path.exists(o)]
  if not objs or shutil.which(os.path.join(build_ext._LLVM, "llvm-objdump")) is None:
    pytest.skip("no built objects / LLVM tools")
  for o in objs:
    assert build_ext.device_calls(o) == [], o
