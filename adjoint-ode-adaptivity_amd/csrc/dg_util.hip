// dg_util.hip — measurement support of libdgadv.so: the achievable-HBM-bandwidth copy
// kernel ("the achievable figure must be measured with a stream-copy kernel").
#include "dg_common.h"

namespace {
using namespace dgk;

// 16-byte accesses per lane.  Measured on the box (profiles/probes/copy_probe.hip, 1 GiB):
// 1 per lane 6.25 TB/s, 2 5.7, 4 5.4, 8 4.0; a grid-stride persistent grid 5.1; hipMemcpy
// 4.5.  One access per lane and many small workgroups keep the most bytes in flight.
constexpr int kCopyVec = 1;

// dst = src, 16 bytes per lane per access.  Workgroup b owns the contiguous 16 KiB run
// [b*kCopyVec*kBlock, (b+1)*kCopyVec*kBlock) of double2: each of its kCopyVec wave-loads is a
// fully coalesced 1 KiB per wave, and consecutive workgroups walk consecutive memory (no
// grid-stride jumps across pages).
__global__ __launch_bounds__(kBlock) void k_stream_copy(const double2* __restrict__ src,
                                                        double2* __restrict__ dst, int64_t n2) {
  const int64_t base = int64_t(blockIdx.x) * (kCopyVec * kBlock) + threadIdx.x;
  double2 v[kCopyVec];
#pragma unroll
  for (int q = 0; q < kCopyVec; ++q) {
    const int64_t i = base + int64_t(q) * kBlock;
    if (i < n2) v[q] = src[i];
  }
#pragma unroll
  for (int q = 0; q < kCopyVec; ++q) {
    const int64_t i = base + int64_t(q) * kBlock;
    if (i < n2) dst[i] = v[q];
  }
}
}  // namespace

extern "C" int dg_stream_copy(const double* src, double* dst, int64_t n, void* stream) {
  if (!src || !dst) return fail(DG_ERR_ARG, "null argument");
  if (n < 0) return fail(DG_ERR_ARG, "n < 0");
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15)
    return fail(DG_ERR_ARG, "src and dst must be 16-byte aligned");
  if (n == 0) return DG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n2 = n / 2;
  if (n2 > 0) {
    const int64_t per = int64_t(kCopyVec) * kBlock;
    const int64_t grid = (n2 + per - 1) / per;
    if (grid > 0x7fffffff) return fail(DG_ERR_ARG, "n too large");
    hipLaunchKernelGGL(k_stream_copy, dim3(unsigned(grid)), dim3(kBlock), 0, st,
                       reinterpret_cast<const double2*>(src), reinterpret_cast<double2*>(dst), n2);
    HIP_TRY(hipGetLastError());
  }
  if (n & 1)
    HIP_TRY(hipMemcpyAsync(dst + n - 1, src + n - 1, sizeof(double), hipMemcpyDeviceToDevice, st));
  return DG_OK;
}

// The device address of page-locked host memory (hipHostGetDevicePointer): kernels can then
// write small results (the refine decision) straight to the host, with no copy launch.
extern "C" int dg_host_alias(void* host, void** device) {
  if (!host || !device) return fail(DG_ERR_ARG, "null argument");
  *device = nullptr;
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, host, 0);
  if (e != hipSuccess || !d)
    return fail(DG_ERR_ARG, std::string("not mapped page-locked host memory: ") +
                                hipGetErrorString(e));
  *device = d;
  return DG_OK;
}
