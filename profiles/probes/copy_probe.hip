// Stream-copy variants on MI355X: which 16-byte copy shape reaches the achievable HBM rate
// (MI355X_MICROARCH.md: 6.29 TB/s float4 copy).  Standalone probe, not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -o copy_probe copy_probe.hip && ./copy_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int V, int NT>
__global__ __launch_bounds__(256) void k_contig(const double2* __restrict__ s,
                                                double2* __restrict__ d, long n2) {
  const long base = long(blockIdx.x) * (V * 256) + threadIdx.x;
  double2 v[V];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const long i = base + long(q) * 256;
    if (i < n2) {
      if (NT & 1) {
        v[q].x = __builtin_nontemporal_load(&s[i].x);
        v[q].y = __builtin_nontemporal_load(&s[i].y);
      } else {
        v[q] = s[i];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const long i = base + long(q) * 256;
    if (i < n2) {
      if (NT & 2) {
        __builtin_nontemporal_store(v[q].x, &d[i].x);
        __builtin_nontemporal_store(v[q].y, &d[i].y);
      } else {
        d[i] = v[q];
      }
    }
  }
}

template <int V>
__global__ __launch_bounds__(256) void k_persist(const double2* __restrict__ s,
                                                 double2* __restrict__ d, long n2) {
  // each workgroup walks contiguous 16 KiB chunks, chunk = blockIdx.x + k*gridDim.x
  const long per = long(V) * 256;
  for (long c = blockIdx.x; c * per < n2; c += gridDim.x) {
    const long base = c * per + threadIdx.x;
    double2 v[V];
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const long i = base + long(q) * 256;
      if (i < n2) v[q] = s[i];
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const long i = base + long(q) * 256;
      if (i < n2) d[i] = v[q];
    }
  }
}

template <class F>
static double time_it(F launch, hipEvent_t a, hipEvent_t b) {
  for (int w = 0; w < 3; ++w) launch();
  std::vector<float> ts;
  for (int r = 0; r < 15; ++r) {
    hipEventRecord(a, 0);
    launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const long bytes = 1L << 30, n2 = bytes / 16;
  double2 *s, *d;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 0, bytes));
  CK(hipMemset(d, 0, bytes));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto report = [&](const char* name, double ms) {
    std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", name, ms,
                2.0 * bytes / (ms * 1e-3) / 1e9);
  };
#define CONTIG(V, NT)                                                                   \
  report("contig V=" #V " nt=" #NT, time_it([&] {                                        \
    k_contig<V, NT><<<unsigned((n2 + V * 256 - 1) / (V * 256)), 256>>>(s, d, n2);        \
  }, a, b))
  CONTIG(1, 0);
  CONTIG(2, 0);
  CONTIG(4, 0);
  CONTIG(8, 0);
  CONTIG(16, 0);
  CONTIG(4, 1);
  CONTIG(4, 2);
  CONTIG(4, 3);
  CONTIG(8, 2);
  CONTIG(8, 3);
#define PERSIST(V, G)                                                                   \
  report("persist V=" #V " grid=" #G, time_it([&] {                                      \
    k_persist<V><<<G, 256>>>(s, d, n2);                                                   \
  }, a, b))
  PERSIST(4, 2048);
  PERSIST(4, 4096);
  PERSIST(8, 2048);
  PERSIST(8, 1024);
  report("hipMemcpyD2D", time_it([&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); },
                                 a, b));
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
