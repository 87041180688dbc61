// fp64 issue-rate probe by instruction kind (what bounds the record kernels):
// 8 independent chains per lane, 8 waves per SIMD, one kind per kernel:
//   fma_s  acc = fma(acc, a, b), a and b wave-uniform (SGPR operands, the kernels' form)
//   fma_v  acc = fma(acc, x, y), x and y per-lane (VGPR operands)
//   add    acc = acc + b;  mul  acc = acc * a;  mix  3 fma : 1 add : 1 mul (the kernels' mix)
//   dep1   one dependent fma chain per lane, at 1 and at 8 waves per SIMD (issue latency)
//   hipcc -O3 --offload-arch=gfx950 -o profiles/probes/fp64_mix profiles/probes/fp64_mix.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kChains = 8;

template <int KIND>
__global__ __launch_bounds__(256) void k_dep(double* out, int iters, double a, double b) {
  double acc = threadIdx.x * 1e-3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) acc = fma(acc, a, b);
  }
  if (acc == 12345.678) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(double* out, int iters, double a, double b) {
  double acc[kChains];
  const double x = 0.999999 + threadIdx.x * 1e-12, y = 1e-7 + threadIdx.x * 1e-15;
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if constexpr (KIND == 0) acc[c] = fma(acc[c], a, b);
      if constexpr (KIND == 1) acc[c] = fma(acc[c], x, y);
      if constexpr (KIND == 2) acc[c] = acc[c] + b;
      if constexpr (KIND == 3) acc[c] = acc[c] * a;
      if constexpr (KIND == 4) {  // per 5 ops: 3 fma, 1 add, 1 mul
        acc[c] = fma(acc[c], a, b);
        acc[c] = fma(acc[c], a, b);
        acc[c] = fma(acc[c], a, b);
        acc[c] = acc[c] + b;
        acc[c] = acc[c] * a;
      }
    }
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += acc[c];
  if (s == 12345.678) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND, bool DEP = false>
void run(const char* name, int blocks, int iters, double* out, int ops_per_iter, int flops_per_op) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&] {
    if constexpr (DEP)
      hipLaunchKernelGGL(k_dep<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999999, 1e-7);
    else
      hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999999, 1e-7);
  };
  launch();
  std::vector<float> ms;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t = 0.f;
    hipEventElapsedTime(&t, e0, e1);
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double t = ms[ms.size() / 2] * 1e-3;
  const double insts = double(ops_per_iter) * kChains * iters * blocks * 256 / 64;  // wave-instr
  // (k_dep: 8 dependent fmas per iteration, ops_per_iter = 1 x kChains = 8 as well)
  std::printf("{\"probe\": \"fp64_%s\", \"median_ms\": %.4f, \"wave_instr_per_s_per_simd\": %.4g, "
              "\"tflops\": %.2f}\n", name, t * 1e3, insts / t / 1024.0,
              insts * 64 * flops_per_op / t / 1e12);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int blocks = prop.multiProcessorCount * 8, iters = 1 << 15;
  double* out = nullptr;
  if (hipMalloc(&out, sizeof(double) * blocks * 256) != hipSuccess) return 1;
  run<0>("fma_sgpr", blocks, iters, out, 1, 2);
  run<1>("fma_vgpr", blocks, iters, out, 1, 2);
  run<2>("add", blocks, iters, out, 1, 1);
  run<3>("mul", blocks, iters, out, 1, 1);
  run<4>("mix_3fma_add_mul", blocks, iters / 2, out, 5, 1);  // flops column: ops, not flops
  run<0, true>("dep1_1wave_per_simd", prop.multiProcessorCount, iters / 8, out, 1, 2);
  run<0, true>("dep1_2waves_per_simd", prop.multiProcessorCount * 2, iters / 8, out, 1, 2);
  run<0, true>("dep1_4waves_per_simd", prop.multiProcessorCount * 4, iters / 8, out, 1, 2);
  run<0, true>("dep1_8waves_per_simd", prop.multiProcessorCount * 8, iters / 8, out, 1, 2);
  hipFree(out);
  return 0;
}
