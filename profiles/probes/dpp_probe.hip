// Probe: do the GFX9 DPP wave-shift controls (wave_shr:1 / wave_shl:1) work on gfx950?
// Prints the lanes whose shifted value is wrong (expect none).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const int* in, int* shr, int* shl) {
  const int v = in[threadIdx.x];
  shr[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
  shl[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x130, 0xf, 0xf, false);  // wave_shl:1
}
int main() {
  int h[64], r1[64], r2[64];
  for (int i = 0; i < 64; ++i) h[i] = 1000 + i;
  int *d, *a, *b;
  hipMalloc(&d, 256); hipMalloc(&a, 256); hipMalloc(&b, 256);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, a, b);
  hipMemcpy(r1, a, 256, hipMemcpyDeviceToHost);
  hipMemcpy(r2, b, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    const int e1 = i > 0 ? 1000 + i - 1 : -1, e2 = i < 63 ? 1000 + i + 1 : -1;
    if (r1[i] != e1 || r2[i] != e2) { ++bad; printf("lane %d: shr %d (want %d) shl %d (want %d)\n", i, r1[i], e1, r2[i], e2); }
  }
  printf("dpp wave shift probe: %d bad lanes\n", bad);
  return 0;
}
