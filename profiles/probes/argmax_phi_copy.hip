// argmax_phi_copy.hip — minimal reproducer of the wrong argmax seen in round 3
// (gpurun_out/xcost2/pytest.log: test_device_reducer_candidates_pick_the_full_argmax[rand-3]
// returned 5540 instead of 9036) and of its cause, a ROCm 7.2 gfx950 code-generation error.
//
// The loop (k_slice_partial before commit 7d0b2f9):
//   double bv = 0.0; int64_t bi = -1;
//   for (i = ...; i < n; i += stride) {
//     v = |sum_r x[r][i] / divisor|;
//     if (bi < 0 || better(v, i, bv, bi)) { bv = v; bi = i; }
//   }
// The optimised LLVM IR is correct (clang -O3 --cuda-device-only -emit-llvm): the loop-carried
// bv is `phi [v, %take], [bv, %keep]`.  The gfx950 machine code is not
// (profiles/probes/argmax_phi_copy_isa.txt, from `hipcc -O3 --offload-arch=gfx950 -S`): the
// register allocator gives v and the new bv the same VGPR pair, and the copy for the
// not-taken edge (new bv = old bv) is placed in the Flow block that joins the `better()`
// branches.  In the structurised (divergent) control flow every lane with bi >= 0 executes that
// block, whether or not its `better()` came out true; the taken block that follows only moves
// bi.  So after its first element a thread's bv never changes while bi still advances: the
// partial is the first grid-stride pass's value with a later index, and the argmax misses any
// winner past a thread's first element.  The disjunction `bi < 0 || ...` is what splits the
// taken edge into two predecessors (%bi<0 and %better-true) and produces the critical edge.
//
// The shipped kernels start every thread from the weakest candidate (-inf, INT64_MAX), so the
// condition is `better()` alone (one branch, no critical edge); both forms are run here.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/argmax_phi_copy argmax_phi_copy.hip && /tmp/argmax_phi_copy
// prints, per case, the CPU argmax and what each form returns (the flag form is expected to
// fail on winners past the first pass; the shipped form must match everywhere).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kBlock = 256;

__device__ __forceinline__ bool better(double va, int64_t ia, double vb, int64_t ib) {
  const bool na = isnan(va), nb = isnan(vb);
  if (na != nb) return na;
  if (!na && va != vb) return va > vb;
  return ia < ib;
}

__device__ __forceinline__ void block_argmax(double& v, int64_t& idx) {
  __shared__ double sv[kBlock];
  __shared__ int64_t si[kBlock];
  sv[threadIdx.x] = v;
  si[threadIdx.x] = idx;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w && better(sv[threadIdx.x + w], si[threadIdx.x + w], sv[threadIdx.x],
                                  si[threadIdx.x])) {
      sv[threadIdx.x] = sv[threadIdx.x + w];
      si[threadIdx.x] = si[threadIdx.x + w];
    }
    __syncthreads();
  }
  v = sv[0];
  idx = si[0];
}

// The round-3 form ("no candidate yet" flag).
__global__ __launch_bounds__(kBlock) void k_flag_form(const double* __restrict__ x, int64_t rows,
                                                      int64_t n, int64_t ld, double divisor,
                                                      double* __restrict__ pv,
                                                      int64_t* __restrict__ pi) {
  double bv = 0.0;
  int64_t bi = -1;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    double acc = x[i];
    for (int64_t r = 1; r < rows; ++r) acc = acc + x[r * ld + i];
    const double v = fabs(divisor != 1.0 ? acc / divisor : acc);
    if (bi < 0 || better(v, i, bv, bi)) {
      bv = v;
      bi = i;
    }
  }
  if (bi < 0) {
    bv = -INFINITY;
    bi = INT64_MAX;
  }
  block_argmax(bv, bi);
  if (threadIdx.x == 0) {
    pv[blockIdx.x] = bv;
    pi[blockIdx.x] = bi;
  }
}

// The shipped form (csrc/dg_advec.hip k_slice_partial / k_argmax_partial).
__global__ __launch_bounds__(kBlock) void k_weakest_form(const double* __restrict__ x,
                                                         int64_t rows, int64_t n, int64_t ld,
                                                         double divisor,
                                                         double* __restrict__ pv,
                                                         int64_t* __restrict__ pi) {
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    double acc = x[i];
    for (int64_t r = 1; r < rows; ++r) acc = acc + x[r * ld + i];
    const double v = fabs(acc / divisor);
    if (better(v, i, bv, bi)) {
      bv = v;
      bi = i;
    }
  }
  block_argmax(bv, bi);
  if (threadIdx.x == 0) {
    pv[blockIdx.x] = bv;
    pi[blockIdx.x] = bi;
  }
}

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      return 2;                                                                       \
    }                                                                                 \
  } while (0)

int main() {
  const int64_t rows_list[] = {1, 4};
  const int64_t n_list[] = {2501, 9000, 100003};
  const double div_list[] = {1.0, 3.0};
  int bad_flag = 0, bad_weak = 0, cases = 0;
  uint64_t s = 12345;
  auto rnd = [&s]() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return double(s >> 11) * (1.0 / 9007199254740992.0);
  };
  for (int64_t rows : rows_list)
    for (int64_t n : n_list)
      for (double div : div_list) {
        const int64_t ld = n + 3;
        std::vector<double> x(size_t(rows * ld));
        for (auto& v : x) v = rnd();
        const int64_t where = n - 7;  // past every thread's first grid-stride pass
        for (int64_t r = 0; r < rows; ++r) x[size_t(r * ld + where)] = 5.0;
        int64_t want = -1;
        double best = -1.0;
        for (int64_t i = 0; i < n; ++i) {
          double acc = x[size_t(i)];
          for (int64_t r = 1; r < rows; ++r) acc = acc + x[size_t(r * ld + i)];
          const double v = std::fabs(acc / div);
          if (v > best) {
            best = v;
            want = i;
          }
        }
        int64_t parts = (n + 4 * kBlock - 1) / (4 * kBlock);
        double *dx, *dpv;
        int64_t* dpi;
        CK(hipMalloc(&dx, sizeof(double) * x.size()));
        CK(hipMalloc(&dpv, sizeof(double) * parts));
        CK(hipMalloc(&dpi, sizeof(int64_t) * parts));
        CK(hipMemcpy(dx, x.data(), sizeof(double) * x.size(), hipMemcpyHostToDevice));
        int64_t got[2];
        for (int form = 0; form < 2; ++form) {
          if (form == 0)
            hipLaunchKernelGGL(k_flag_form, dim3(unsigned(parts)), dim3(kBlock), 0, 0, dx, rows,
                               n, ld, div, dpv, dpi);
          else
            hipLaunchKernelGGL(k_weakest_form, dim3(unsigned(parts)), dim3(kBlock), 0, 0, dx,
                               rows, n, ld, div, dpv, dpi);
          CK(hipGetLastError());
          std::vector<double> pv(static_cast<size_t>(parts));
          std::vector<int64_t> pi(static_cast<size_t>(parts));
          CK(hipMemcpy(pv.data(), dpv, sizeof(double) * parts, hipMemcpyDeviceToHost));
          CK(hipMemcpy(pi.data(), dpi, sizeof(int64_t) * parts, hipMemcpyDeviceToHost));
          double bv = -INFINITY;
          int64_t bi = INT64_MAX;
          for (int64_t p = 0; p < parts; ++p)
            if (pv[size_t(p)] > bv || (pv[size_t(p)] == bv && pi[size_t(p)] < bi)) {
              bv = pv[size_t(p)];
              bi = pi[size_t(p)];
            }
          got[form] = bi;
        }
        CK(hipFree(dx));
        CK(hipFree(dpv));
        CK(hipFree(dpi));
        ++cases;
        bad_flag += got[0] != want;
        bad_weak += got[1] != want;
        std::printf("rows %lld n %lld div %.0f: cpu %lld  flag form %lld %s  shipped form %lld %s\n",
                    (long long)rows, (long long)n, div, (long long)want, (long long)got[0],
                    got[0] == want ? "ok" : "WRONG", (long long)got[1],
                    got[1] == want ? "ok" : "WRONG");
      }
  std::printf("cases %d: flag form wrong %d, shipped form wrong %d\n", cases, bad_flag, bad_weak);
  return bad_weak ? 1 : 0;
}
