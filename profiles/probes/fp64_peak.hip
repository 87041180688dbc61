// fp64 vector FMA throughput probe (the compute ceiling of the fused DG kernels):
// every lane runs 8 independent v_fma_f64 chains; grid = 8 waves per CU.
//   hipcc -O3 --offload-arch=gfx950 -o profiles/probes/fp64_peak profiles/probes/fp64_peak.hip
//   ./profiles/probes/fp64_peak        -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int kChains = 8;

__global__ __launch_bounds__(256) void k_fma(double* out, int iters, double a, double b) {
  double acc[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc[c] = fma(acc[c], a, b);
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += acc[c];
  if (s == 12345.678) out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keep the chains live
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8, threads = 256, iters = 1 << 16;
  double* out = nullptr;
  if (hipMalloc(&out, sizeof(double) * blocks * threads) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, out, iters, 0.999999, 1e-7);
  std::vector<float> ms;
  for (int r = 0; r < 7; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, out, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t = 0.f;
    hipEventElapsedTime(&t, e0, e1);
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double flops = 2.0 * kChains * double(iters) * blocks * threads;
  std::printf("{\"probe\": \"fp64_fma\", \"cus\": %d, \"median_ms\": %.4f, \"tflops\": %.2f}\n",
              cus, ms[ms.size() / 2], flops / (ms[ms.size() / 2] * 1e-3) / 1e12);
  hipFree(out);
  return 0;
}
