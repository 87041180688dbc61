// dg_common.h — internals shared by the HIP translation units of libdgadv.so
// (dg_advec.hip: linear-flux kernels + the C ABI; dg_burgers.hip: nonlinear flux and the
// per-stage limiter).  Not part of the ABI: include/dg_advec.h is.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <tuple>
#include <vector>
#include <type_traits>
#include <utility>
#include <vector>

#include "dg_advec.h"

namespace dgk {

constexpr int kBlock = 256;       // lanes per workgroup = elements per tile (incl. halo)
constexpr int kMaxNP = 9;         // N <= 8
constexpr int kArgmaxParts = 1024;

// Register budgets of the config-3 kernels.  The hardware admits 256-thread workgroups per CU
// up to floor(800 / (ceil(sgpr/16)*16 + 16)) (MI355X_MICROARCH.md, Residency): 8 at <= 80
// SGPRs, 7 at 82-96.  k_step_nl is capped at 80 SGPRs so 8 workgroups fit per CU (at 94-100
// SGPRs the hardware admits 6-7; the spills go to VGPR lanes, the kernel stays at <= 64
// VGPRs); k_adj_nl targets 5 waves per SIMD (<= 96 VGPRs, dg_burgers.hip).  (Caps on the
// linear kernels' SGPRs and wave priority were measured and rejected)
#define DG_NL_STEP_ATTR __attribute__((amdgpu_num_sgpr(80)))
constexpr int kNLAdjMinWaves = 5;

// Indicator write mode of the adjoint kernels (the `has_eta` argument field):
// bit 0 an indicator is wanted; bit 1 this launch assigns eta instead of adding to it (the
// sweep's first launch under DG_ADJ_ETA_ASSIGN: no zero fill); bit 2 this launch stores
// |eta| (the sweep's last launch under DG_ADJ_ETA_ABS).
constexpr int kEtaOn = 1, kEtaAssign = 2, kEtaAbs = 4;

__device__ __forceinline__ void eta_update(double* __restrict__ eta, int64_t e, double acc,
                                           int mode) {
  double v = (mode & kEtaAssign) ? acc : eta[e] + acc;
  if (mode & kEtaAbs) v = fabs(v);
  eta[e] = v;
}

// The jump record (dg_lserk4_fwd_rec / dg_lserk4_adj_rec).  The indicator needs of u^n only
// the interelement jumps (utils/AdvecRHS1D.m:9-16's du; R(u^n) = LIFT Fscale du, :19), and a
// face's jump is one number shared by its two elements: the record keeps, per step and
// element e, the LEFT-face jump j_e = u_0 - uL (uL = the inflow value at a trajectory's first
// element), one double.  Element e's right-face jump du1 = u_N - uR is -j_{e+1} exactly
// (IEEE subtraction is antisymmetric: b - a == -(a - b)), or 0 at a trajectory's last element,
// so the adjoint rebuilds du0 - du1 = j_e + j_{e+1} and du0 + du1 = j_e - j_{e+1} bit for bit.
// Row n - 1 holds u^n's jumps; rows are rec_ld(ktot) doubles apart (ktot rounded up to even,
// so the pair kernels' two-element accesses are 16-byte aligned).
__host__ __device__ constexpr int64_t rec_ld(int64_t ktot) { return (ktot + 1) & ~int64_t(1); }

// Kernel-argument layout pin for the edge tiles' lane-indexed kernarg reads.  A kernel whose
// parameters are pointers followed by ONE trailing by-value argument struct A has A at byte
// offset (#pointers)*8 of the kernarg segment: pointers are 8-byte aligned and A's alignment
// is 8, so no padding precedes it.  kernarg_tail<&kernel, A>() checks that shape on the
// kernel's own type at compile time, so a change to a parameter's type, count or to A's
// alignment breaks the build instead of reading garbage.
template <class F> struct KernargLayout;
template <class... P> struct KernargLayout<void (*)(P...)> {
  static constexpr int kParams = int(sizeof...(P));
  using Tail = std::tuple_element_t<sizeof...(P) - 1, std::tuple<P...>>;
  static constexpr int kPointers = (0 + ... + int(std::is_pointer_v<P>));
  static constexpr size_t kTailOffset = size_t(kParams - 1) * sizeof(void*);
};

template <class F, class A>
__device__ __forceinline__ const char* kernarg_tail() {
  using L = KernargLayout<F>;
  static_assert(std::is_same_v<typename L::Tail, A>, "kernel's last parameter is not A");
  static_assert(L::kPointers == L::kParams - 1, "all parameters before A must be pointers");
  static_assert(sizeof(void*) == 8 && alignof(A) == 8, "A must follow 8-byte pointers unpadded");
  static_assert(std::is_standard_layout_v<A> && std::is_trivially_copyable_v<A>,
                "offsetof needs a standard-layout argument struct");
  return (const char*)__builtin_amdgcn_kernarg_segment_ptr() + L::kTailOffset;
}

// The same tail as a constant-address-space (kernarg) pointer: loads through it are scalar
// loads, also after the pointer is laundered (dg_rec_tiles.h OpSrc).
#define DG_KAS __attribute__((address_space(4)))
template <class F, class A>
__device__ __forceinline__ const DG_KAS char* kernarg_tail_k() {
  (void)kernarg_tail<F, A>();  // the layout checks
  return (const DG_KAS char*)__builtin_amdgcn_kernarg_segment_ptr() + KernargLayout<F>::kTailOffset;
}

// The kernel-argument segment's size limit: launches that pass their constants by value
// (the dataflow sweeps' block tables) check their argument struct against it at compile time.
constexpr size_t kKernargMax = 4096;

// Sets the calling thread's dg_last_error() text and returns `code` (dg_advec.hip).
int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return ::dgk::fail(DG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
  } while (0)

// ---------------------------------------------------------------------------
// Low-storage RK coefficients, utils/Globals1D.m:19-34 (LSERK4) and forward Euler.
// ---------------------------------------------------------------------------
template <int NS> struct RK;
template <> struct RK<5> {
  __host__ __device__ static constexpr double A(int s) {
    return s == 0 ? 0.0
         : s == 1 ? -567301805773.0 / 1357537059087.0
         : s == 2 ? -2404267990393.0 / 2016746695238.0
         : s == 3 ? -3550918686646.0 / 2091501179385.0
                  : -1275806237668.0 / 842570457699.0;
  }
  __host__ __device__ static constexpr double B(int s) {
    return s == 0 ? 1432997174477.0 / 9575080441755.0
         : s == 1 ? 5161836677717.0 / 13612068292357.0
         : s == 2 ? 1720146321549.0 / 2090206949498.0
         : s == 3 ? 3134564353537.0 / 4481467310338.0
                  : 2277821191437.0 / 14882151754819.0;
  }
  __host__ __device__ static constexpr double C(int s) {
    return s == 0 ? 0.0
         : s == 1 ? 1432997174477.0 / 9575080441755.0
         : s == 2 ? 2526269341429.0 / 6820363962896.0
         : s == 3 ? 2006345519317.0 / 3224310063776.0
                  : 2802321613138.0 / 2924317926251.0;
  }
};
template <> struct RK<1> {
  __host__ __device__ static constexpr double A(int) { return 0.0; }
  __host__ __device__ static constexpr double B(int) { return 1.0; }
  __host__ __device__ static constexpr double C(int) { return 0.0; }
};

// Element operator, folded with the advection speed (host side, per plan):
//   rhs_i = s_k * ( sum_j Dm[i][j] u_j + L0[i]*(u_0 - uL) + L1[i]*(u_N - uR) )
//   Dm = -a*Dr, L0 = (-a/2)*LIFT(:,1), L1 = (a/2)*LIFT(:,2), s_k = rx = Fscale = 2/h_k.
template <int NP> struct OpArgs {
  double Dm[NP * NP];
  double L0[NP];
  double L1[NP];
};

// The same operator in even/odd node coordinates.  LGL nodes are symmetric about 0, so
// with J the node-reversal matrix J*Dr*J = -Dr and LIFT(:,2) = J*LIFT(:,1).  Per element
//   e_k = (u_k + u_{N-k})/2,  o_k = (u_k - u_{N-k})/2   (k < NO),   e_NO = u_mid (Np odd)
// and the element operator splits into an odd->even and an even->odd block:
//   rhs_e = Qeo o + le*(du0 - du1),   rhs_o = Qoe e + lo*(du0 + du1)
// which is 2*NE*NO + NP fused multiply-adds per stage instead of NP*NP + 2*NP.
// The blocks are built and checked on the host (make_eo).
template <int NP> struct EOArgs {
  static constexpr int NE = (NP + 1) / 2;
  static constexpr int NO = NP / 2;
  double Qeo[NE * NO];  // rhs_e[k] += Qeo[k*NO + j] * o[j]
  double Qoe[NO * NE];  // rhs_o[k] += Qoe[k*NE + j] * e[j]
  double le[NE];
  double lo[NO];
};

// Arguments of a launch that advances MS time steps of NS stages each.
template <int NP, int NS, int MS> struct StepArgs {
  EOArgs<NP> op;
  double sc;                // dt (non-uniform meshes multiply by scale[k]; uniform: folded in op)
  double uin[MS * NS + 1];  // inflow value at each stage time, then at t_{n0+MS}
  int64_t ktot;             // batch * K elements
  int64_t stride;           // doubles between consecutive snapshots
  int64_t n0;               // jump record: global index of the launch's first step
  int32_t K;                // elements per trajectory
  int32_t xcd;              // XCD-aware tile order (speed only)
  int32_t jend;             // jump record: the launch ends the sweep (record u^{n0+MS} too)
};

template <int NP, int MS> struct AdjArgs {
  EOArgs<NP> op;
  double sc;
  double uin_res[MS];  // inflow value at t_{n+st+1} for the residual of step st
  double src[MS];      // functional source coefficient for node n+st+1
  int64_t ktot;
  int64_t stride;      // doubles between consecutive snapshots
  int64_t n0;          // jump record: global index of the launch's first step
  int32_t K;
  int32_t has_eta;     // kEta* bits
  int32_t xcd;         // XCD-aware tile order (speed only)
};

// ---------------------------------------------------------------------------
// Tile staging helpers.  A tile is the contiguous range of doubles of kBlock
// consecutive elements starting at element e0 (which may be negative or run past
// the end: those doubles read as 0 and are never used by a valid lane).
// ---------------------------------------------------------------------------
template <int NP>
__device__ __forceinline__ int load_tile(const double* __restrict__ g, int64_t e0, int64_t nd,
                                         double* __restrict__ lds) {
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);           // 16-byte aligned start
  const int off = int(d0 - base);                  // 0 or 1
  const int nvec = (kBlock * NP + off + 1) >> 1;   // double2 count
  const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g);
  for (int v = threadIdx.x; v < nvec; v += kBlock) {
    const int64_t gd = base + 2 * int64_t(v);
    double2 val;
    if (gd >= 0 && gd + 1 < nd) {
      val = g2[gd >> 1];
    } else {
      val.x = (gd >= 0 && gd < nd) ? g[gd] : 0.0;
      val.y = (gd + 1 >= 0 && gd + 1 < nd) ? g[gd + 1] : 0.0;
    }
    *reinterpret_cast<double2*>(&lds[2 * v]) = val;
  }
  return off;
}

// ---------------------------------------------------------------------------
// Tile geometry of the fused step kernels.  A workgroup of LB = 256*W lanes owns a tile
// of T = LB consecutive elements, one element per lane, its state in VGPRs.  The
// dependency cone of one step is NS elements per side, so of MS fused steps the
// TE = T - 2*MS*NS interior elements are exact and written back.  W = 2 halves the
// redundant halo work (the kernels are fp64-VALU bound) at the same registers per lane.
// ---------------------------------------------------------------------------
template <int NP, int W> struct TileGeo {
  static constexpr int LB = kBlock * W;
  static constexpr int T = LB;
  static constexpr int kVec = (T * NP + 2 + 2 * LB - 1) / (2 * LB);  // double2 / lane
  static constexpr int kTileD = T * NP + 2;  // staging image (+2: 16-byte realignment)
  static constexpr int kFaceD = 4 * (T + 2);  // 2 double-buffered face arrays, padded by 1
  // The face arrays follow the image instead of aliasing it: the stages never wait for the
  // image's readers (snapshot stores, staging reads) and vice versa — 2 barriers fewer
  // per step in k_step and k_adj.
  static constexpr int kFB = (kTileD + 1) & ~1;
  static constexpr int kLds = kFB + kFaceD;
};

// Issue the 16-byte loads of one tile image into registers (coalesced: lane-consecutive
// double2), then commit them to LDS.  Elements outside [0, ktot) read as zero.
template <int NP, int W> struct TileRegs {
  double2 v[TileGeo<NP, W>::kVec];
  int off;
};

template <int NP, int W, bool EDGE = true>
__device__ __forceinline__ void tile_issue(const double* __restrict__ g, int64_t e0, int64_t nd,
                                           TileRegs<NP, W>& r) {
  using G = TileGeo<NP, W>;
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  r.off = int(d0 - base);
  const int nvec = (G::T * NP + r.off + 1) >> 1;
  const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g);
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = threadIdx.x + q * G::LB;
    const int64_t gd = base + 2 * int64_t(v);
    double2 val = make_double2(0.0, 0.0);
    if (v < nvec) {
      if (!EDGE || (gd >= 0 && gd + 1 < nd)) {  // interior tiles: always in range
        val = g2[gd >> 1];
      } else {
        if (gd >= 0 && gd < nd) val.x = g[gd];
        if (gd + 1 >= 0 && gd + 1 < nd) val.y = g[gd + 1];
      }
    }
    r.v[q] = val;
  }
}

template <int NP, int W>
__device__ __forceinline__ void tile_commit(const TileRegs<NP, W>& r, double* __restrict__ lds) {
  using G = TileGeo<NP, W>;
  const int nvec = (G::T * NP + r.off + 1) >> 1;
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = threadIdx.x + q * G::LB;
    if (v < nvec) *reinterpret_cast<double2*>(&lds[2 * v]) = r.v[q];
  }
}

// Store `count` doubles from lds[0..count) to g[o0..o0+count); o0 must be even.
template <int LB = kBlock>
__device__ __forceinline__ void store_run(double* __restrict__ g, int64_t o0, int64_t count,
                                          const double* __restrict__ lds) {
  double2* __restrict__ g2 = reinterpret_cast<double2*>(g);
  for (int64_t v = threadIdx.x; 2 * v < count; v += LB) {
    const double2 val = *reinterpret_cast<const double2*>(&lds[2 * v]);
    const int64_t gd = o0 + 2 * v;
    if (2 * v + 1 < count) {
      g2[gd >> 1] = val;
    } else {
      g[gd] = val.x;
    }
  }
}

// Store a full tile output (COUNT doubles, compile-time) from lds to g[o0..); o0 even.
template <int COUNT, int LB>
__device__ __forceinline__ void store_full(double* __restrict__ g, int64_t o0,
                                           const double* __restrict__ lds) {
  static_assert(COUNT % 2 == 0, "16-byte runs");
  constexpr int NV = COUNT / 2, NQ = (NV + LB - 1) / LB;
  double2* __restrict__ g2 = reinterpret_cast<double2*>(g + o0);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int v = int(threadIdx.x) + q * LB;
    if ((q + 1) * LB <= NV || v < NV) g2[v] = *reinterpret_cast<const double2*>(&lds[2 * v]);
  }
}

// A tile is an edge tile when its element range [e0, e0+T) leaves [0, ktot) or contains
// a trajectory's first or last element (uniform per workgroup).  Interior tiles -- all
// but a handful -- run a specialisation without inflow/outflow selects or bounds checks.
__device__ __forceinline__ bool edge_tile(int64_t e0, int T, int64_t ktot, int32_t K) {
  if (e0 < 0 || e0 + T > ktot) return true;
  const int64_t kl0 = int64_t(uint32_t(e0) % uint32_t(K));
  return kl0 == 0 || kl0 + T >= K;
}

// Per-element geometry: global element e = e0 + el, position kl inside its trajectory.
struct Elem {
  int64_t e;
  int32_t kl;
  bool inrange, first, last, valid;
};

template <int H, int T, bool EDGE = true>
__device__ __forceinline__ Elem elem_info(int64_t e0, int el, int64_t ktot, int32_t K) {
  Elem E;
  E.e = e0 + el;
  if constexpr (!EDGE) {
    E.kl = int32_t(uint32_t(E.e) % uint32_t(K));
    E.inrange = true;
    E.first = E.last = false;
    E.valid = el >= H && el < T - H;
    return E;
  }
  E.inrange = (E.e >= 0 && E.e < ktot);
  // ktot < 2^31 (checked at plan creation): 32-bit division.
  E.kl = E.inrange ? int32_t(uint32_t(E.e) % uint32_t(K)) : 0;
  E.first = (E.kl == 0);
  E.last = (E.kl == K - 1);
  E.valid = E.inrange && el >= H && el < T - H;
  return E;
}

// Tile of workgroup b.  The dispatcher deals workgroups round-robin over the 8 XCDs
// (b, b+8, ... share one; cdna_hip_programming.md §5.5 T1), so giving each XCD a
// contiguous range of tiles makes neighbouring tiles -- which re-read each other's halo
// lines -- run on one L2.  Bijective for any n; a speed choice only.
__device__ __forceinline__ int64_t tile_of(int64_t b, int64_t n, bool xcd) {
  if (!xcd || n < 16) return b;
  const int64_t q = n / 8, r = n % 8, x = b % 8, j = b / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}

// Boundary handling in the face exchange is done by *index* selection into LDS (one
// 32-bit v_cndmask), never by value/pointer selection: `c ? kernarg : lds[i]` lets the
// compiler fold a select of pointers into a flat load on every stage's critical path.
// Each kernel keeps its per-stage boundary constants (inflow values, a zero) in a few
// doubles at the end of its LDS array, written by edge tiles only.

// Materialise a value at this point of the program: an empty volatile asm keeps its
// order with the barrier, so work placed before a __syncthreads() is not sunk below it by
// the IR optimisers (the machine scheduler never moves code across s_barrier).
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }

// Even/odd element state helpers.
template <int NP>
__device__ __forceinline__ void to_eo(const double* u, double* ev, double* od) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    ev[k] = 0.5 * (u[k] + u[N - k]);
    od[k] = 0.5 * (u[k] - u[N - k]);
  }
  if constexpr (NE > NO) ev[NO] = u[NO];
}

template <int NP>
__device__ __forceinline__ void from_eo(const double* ev, const double* od, double* u) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    u[k] = ev[k] + od[k];
    u[N - k] = ev[k] - od[k];
  }
  if constexpr (NE > NO) u[NO] = ev[NO];
}

// Write the TE interior elements of the tile (element-major, nodal) through the LDS
// image with 16-byte stores.  Callers barrier before (face reads done) and after (when
// the image is reused).
template <int NP, int W, int H>
__device__ __forceinline__ void stage_out(double* __restrict__ lds, const double (*ev)[(NP + 1) / 2],
                                          const double (*od)[NP / 2], bool dual) {
  constexpr int T = TileGeo<NP, W>::T, EPL = 1;
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  const int lane = threadIdx.x;
#pragma unroll
  for (int m = 0; m < EPL; ++m) {
    const int el = m * T + lane;
    if (el >= H && el < T - H) {
      double* o = lds + (el - H) * NP;
      if (dual) {  // dual coordinates back to nodal: w_k = (we+wo)/2, w_{N-k} = (we-wo)/2
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          o[k] = 0.5 * (ev[m][k] + od[m][k]);
          o[N - k] = 0.5 * (ev[m][k] - od[m][k]);
        }
        if constexpr (NE > NO) o[NO] = ev[m][NO];
      } else {
        from_eo<NP>(ev[m], od[m], o);
      }
    }
  }
}

}  // namespace dgk

// ---------------------------------------------------------------------------
// Plan
// ---------------------------------------------------------------------------
struct dg_plan {
  int N = 0, NP = 0;
  int64_t K = 0, batch = 0, ktot = 0;
  int64_t K_cap = 0;  // elements per trajectory the device buffers hold (dg_plan_reserve)
  double a = 0.0;
  int inflow = 0, scheme = 0, nstages = 5;
  bool uniform = true;
  double s_uniform = 0.0;  // 2/h for uniform meshes
  double r[dgk::kMaxNP], V[dgk::kMaxNP * dgk::kMaxNP], invV[dgk::kMaxNP * dgk::kMaxNP],
      Dr[dgk::kMaxNP * dgk::kMaxNP],
      LIFT[dgk::kMaxNP * 2];
  double* d_scale = nullptr;  // K_cap: 2/h_k
  double* d_VX = nullptr;     // K_cap+1
  double* d_scratch = nullptr;   // two fields: adjoint ping-pong lands the last launch in w
  double* d_scratch2 = nullptr;
  double* d_pv = nullptr;
  int64_t* d_pi = nullptr;
  // tuning (dg_plan_tune): tile width of the step kernels (tile = 256*tile_width elements)
  int tile_width = 1;  // dg_plan_create: 2 for N <= 2 (measured per-N)
  int msteps = 4;  // time steps fused per launch (1, 2 or 4)
  // the jump-record sweeps' shape (dg_lserk4_fwd_rec / _adj_rec: no snapshot per step, so
  // long launches on wide tiles pay): tile width 1, 2 or 4, steps per launch 1..8
  // defaults measured at N = 4, K = 2^20: 1024-element pair tiles, 10 steps per
  // launch (a 20-step sweep is 10 + 10 launches)
  int rec_tile_width = 2;
  int rec_tile_width_fwd = 0;  // the forward record sweep's own tile width (0: as rec_tile_width)
  int rec_msteps = 10;
  // the forward's own record steps per launch: -1 by size (20 on 1024-element pair tiles up to
  // 3*2^20 elements, else as rec_msteps), 0 as rec_msteps, > 0 explicit
  int rec_msteps_fwd = -1;
  int rec_lane_elems = 2;  // 2: the pair tiles of dg_rec.hip, 1: dg_advec.hip k_step/k_adj
  // the p-enriched estimate's shape (dg_lserk4_adj_p, dg_dwr.hip): tile width 1 or 2 (256 or
  // 512 elements), steps per launch 1, 2, 4 or 8 (8 on 512-element tiles)
  int p_tile_width = 2;
  int p_msteps = 4;
  // 1: the estimate runs as ONE dataflow launch (k_adjp_flow) when its steps split into >= 2
  // blocks of p_msteps; 0: one launch per block (dg_plan_create sets 1)
  int p_flow = 0;
  // 1: dg_lserk4_sweep_p runs forward and estimate as ONE dataflow launch (k_psweep) where the
  // shape allows; 0: the chains (dg_plan_create sets 1)
  int p_sweep = 0;
  // the dataflow sweep (dg_lserk4_sweep_rec, dg_sweep.hip): its scratch (sync words, block
  // states, indicator partials; grown on demand) and the switch (1: one dataflow launch where
  // the shape allows it, 0: the launch-per-block pair)
  void* d_sweep = nullptr;
  int32_t* d_nl_list = nullptr;  // config-3 adjoint's troubled-tile list + per-step counts
  int64_t nl_list_tiles = 0, nl_list_steps = 0;
  size_t sweep_bytes = 0;
  size_t sweep_sync = 0;  // bytes of its control region (zeroed, then kept by epochs)
  int64_t sweep_items = -1;  // work items of the last dataflow launch on that region
  // the shape the control words were last zeroed for (items, waves, steps per block, nsteps,
  // adjoint tiles): the take counter counts launches modulo the items and the fused refine's
  // arrival counter modulo the last block's tiles, so any change of these zeroes them
  uint64_t sweep_sig = 0;
  // scratch regions a grown scratch replaced: kept until the plan is destroyed, because a HIP
  // graph captured earlier still holds their addresses in its kernel arguments
  std::vector<void*> sweep_retired;
  // watchdog: polls before a waiting work item gives up (0: the default, ~2^20; tests set 1)
  int sweep_spin_limit = 0;
  // the watchdog's host-visible flag (mapped page-locked word; the device alias is what the
  // kernel writes): set by a work item that gave up, read without a sync by the next sweep
  // call (which then fails) and cleared by dg_sweep_status
  uint32_t* h_sweep_err = nullptr;
  uint32_t* d_sweep_err = nullptr;
  int rec_sweep = 1;
  // the dataflow sweep's workgroup waves (tiles of 128 * waves elements): 0 = as the record
  // sweeps' tile width (4 * rec_tile_width), else 4, 8, 12 or 16 (12 / 16: dataflow only, both
  // directions on that tile, whatever the launch chains' widths; 16 at Np <= 5)
  int sweep_waves = 0;
  // consecutive elements per lane of the dataflow sweep's tiles: 2 (pair tiles), or 4 at
  // Np <= 3 on 4- or 8-wave workgroups (tiles of 64 * 4 * waves elements)
  int sweep_lane_elems = 2;
  // how the dataflow sweep's tiles exchange faces: 0 through LDS with a workgroup barrier per
  // Horner level (dg_rec_tiles.h), 1 overlapped waves: DPP within a wave, one LDS exchange and
  // barrier per step (dg_ovl_tiles.h)
  int sweep_exchange = 0;
  // how the config-3 kernels (nonlinear flux / per-stage limiter, dg_burgers*.hip) exchange
  // neighbour values: 0 workgroup tiles through LDS, a barrier per exchange (dg_burgers.hip);
  // 1 overlapped waves, DPP shifts, no barrier inside a step (dg_burgers_ov.hip)
  int nl_exchange = 0;
  // dg_lserk4_fwd with snapshots: 0 the stage-loop kernels (k_step / wave tiles; bit-identical
  // to the record sweeps' stage-loop kernels), 1 Horner-form pair tiles (k_step_rps, dg_rec.hip;
  // tiles of 512 * tile_width elements, msteps steps per launch)
  int snap_pairs = 0;
  uint64_t* sweep_trace = nullptr;  // dg_plan_sweep_trace: per-item timestamps (profiling)
  int cu_count = 0;  // compute units of the plan's device (the dataflow grid)
  int xcd_order = 1;  // XCD-aware tile order
  int lane_elems = 0;  // 0: workgroup tiles (one element per lane); 2 or 4: wave tiles
  // physics (dg_plan_set_physics): DG_FLUX_LINEAR / DG_FLUX_BURGERS, SlopeLimitN per stage
  int flux = 0;
  int limiter = 0;
  double tvb_M = 0.0;  // dg_plan_set_tvb: the TVB constant of dg_slope_limit_n / _1 (0: minmod)
  bool nonlinear() const { return flux != 0 || limiter != 0; }
};

namespace dgk {

// Tile width of the forward record sweep (the adjoint's is rec_tile_width).
inline int rec_fwd_width(const dg_plan* p) {
  return p->rec_tile_width_fwd ? p->rec_tile_width_fwd : p->rec_tile_width;
}

inline double inflow_value(const dg_plan* p, double t) {
  if (p->inflow == DG_INFLOW_ZERO) return 0.0;
  return (p->inflow == DG_INFLOW_SIN_A2T) ? -std::sin(p->a * p->a * t) : -std::sin(p->a * t);
}

// scale = 1 gives the plain operator (rhs); the steppers fold dt*2/h into it on uniform meshes.
template <int NP> OpArgs<NP> make_op(const dg_plan* p, double scale = 1.0) {
  OpArgs<NP> op;
  for (int i = 0; i < NP; ++i) {
    for (int j = 0; j < NP; ++j) op.Dm[i * NP + j] = scale * (-p->a * p->Dr[i * NP + j]);
    op.L0[i] = scale * ((-p->a / 2.0) * p->LIFT[i * 2 + 0]);
    op.L1[i] = scale * ((p->a / 2.0) * p->LIFT[i * 2 + 1]);
  }
  return op;
}

// Even/odd blocks of the element operator (see EOArgs).  Returns false if the operator
// is not centro-(anti)symmetric to 1e-12, i.e. the nodes are not symmetric.
// fold = true: the own-face parts of the lift term go into the volume blocks.  With
// du0 = u_0 - uL, du1 = u_N - uR and u_0 - u_N = 2 o_0, u_0 + u_N = 2 e_0:
//   le*(du0 - du1) = 2 le o_0 + le*(uR - uL),   lo*(du0 + du1) = 2 lo e_0 - lo*(uL + uR)
// so Qeo(:,0) += 2 le and Qoe(:,0) += 2 lo, and a stage needs only the neighbours' faces
// (uR - uL, uL + uR): two fp64 ops fewer per stage forward, four in the adjoint.
template <int NP> bool make_eo(const dg_plan* p, double scale, EOArgs<NP>* out, bool fold = false) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  double Dm[NP][NP], L0[NP], L1[NP], T[NP][NP] = {}, Ti[NP][NP] = {};
  for (int i = 0; i < NP; ++i) {
    for (int j = 0; j < NP; ++j) Dm[i][j] = scale * (-p->a * p->Dr[i * NP + j]);
    L0[i] = scale * ((-p->a / 2.0) * p->LIFT[i * 2 + 0]);
    L1[i] = scale * ((p->a / 2.0) * p->LIFT[i * 2 + 1]);
  }
  for (int k = 0; k < NO; ++k) {  // rows: e_0..e_{NE-1}, o_0..o_{NO-1}
    T[k][k] += 0.5; T[k][N - k] += 0.5;
    T[NE + k][k] += 0.5; T[NE + k][N - k] -= 0.5;
    Ti[k][k] += 1.0; Ti[k][NE + k] += 1.0;
    Ti[N - k][k] += 1.0; Ti[N - k][NE + k] -= 1.0;
  }
  if (NE > NO) { T[NO][NO] = 1.0; Ti[NO][NO] = 1.0; }
  double TD[NP][NP], Q[NP][NP], l0[NP], l1[NP];
  for (int i = 0; i < NP; ++i)
    for (int j = 0; j < NP; ++j) {
      double t = 0.0;
      for (int k = 0; k < NP; ++k) t += T[i][k] * Dm[k][j];
      TD[i][j] = t;
    }
  double qmax = 0.0, lmax = 0.0;
  for (int i = 0; i < NP; ++i) {
    for (int j = 0; j < NP; ++j) {
      double t = 0.0;
      for (int k = 0; k < NP; ++k) t += TD[i][k] * Ti[k][j];
      Q[i][j] = t;
      qmax = std::fmax(qmax, std::fabs(t));
    }
    double a0 = 0.0, a1 = 0.0;
    for (int k = 0; k < NP; ++k) {
      a0 += T[i][k] * L0[k];
      a1 += T[i][k] * L1[k];
    }
    l0[i] = a0;
    l1[i] = a1;
    lmax = std::fmax(lmax, std::fmax(std::fabs(a0), std::fabs(a1)));
  }
  bool ok = true;
  const double tq = 1e-12 * qmax, tl = 1e-12 * lmax;
  for (int i = 0; i < NE; ++i)
    for (int j = 0; j < NE; ++j) ok = ok && std::fabs(Q[i][j]) <= tq;           // even->even
  for (int i = 0; i < NO; ++i)
    for (int j = 0; j < NO; ++j) ok = ok && std::fabs(Q[NE + i][NE + j]) <= tq;  // odd->odd
  for (int k = 0; k < NE; ++k) ok = ok && std::fabs(l0[k] + l1[k]) <= tl;
  for (int k = 0; k < NO; ++k) ok = ok && std::fabs(l0[NE + k] - l1[NE + k]) <= tl;
  if (out) {
    for (int k = 0; k < NE; ++k)
      for (int j = 0; j < NO; ++j) out->Qeo[k * NO + j] = Q[k][NE + j];
    for (int k = 0; k < NO; ++k)
      for (int j = 0; j < NE; ++j) out->Qoe[k * NE + j] = Q[NE + k][j];
    for (int k = 0; k < NE; ++k) out->le[k] = 0.5 * (l0[k] - l1[k]);
    for (int k = 0; k < NO; ++k) out->lo[k] = 0.5 * (l0[NE + k] + l1[NE + k]);
    if (fold) {
      for (int k = 0; k < NE; ++k) out->Qeo[k * NO] += 2.0 * out->le[k];
      for (int k = 0; k < NO; ++k) out->Qoe[k * NE] += 2.0 * out->lo[k];
    }
  }
  return ok;
}

inline unsigned grid_for(int64_t n, int64_t per) { return unsigned((n + per - 1) / per); }

// Dispatch on Np (2..9) and the number of stages.
#define DG_DISPATCH_NP(NPV, CALL) \
  switch (NPV) {                  \
    case 2: { constexpr int NP = 2; CALL; } break; \
    case 3: { constexpr int NP = 3; CALL; } break; \
    case 4: { constexpr int NP = 4; CALL; } break; \
    case 5: { constexpr int NP = 5; CALL; } break; \
    case 6: { constexpr int NP = 6; CALL; } break; \
    case 7: { constexpr int NP = 7; CALL; } break; \
    case 8: { constexpr int NP = 8; CALL; } break; \
    case 9: { constexpr int NP = 9; CALL; } break; \
    default: return fail(DG_ERR_ARG, "unsupported Np"); \
  }

// Nonlinear-flux / per-stage-limiter steppers (dg_burgers.hip), dispatched from the C ABI
// when plan->nonlinear().
int nl_rhs(const dg_plan* p, const double* u, double* rhs, double t, hipStream_t st);
int nl_query(const dg_plan* p, int64_t out[3]);  // dg_plan_query_nl
int nl_fwd(dg_plan* p, double* u, double t0, double dt, int nsteps, double* snapshots,
           uint16_t* decisions, hipStream_t st);
int nl_adj(dg_plan* p, double* w, const double* snapshots, double t0, double dt, int nsteps,
           double src_coef, double* eta, int flags, const uint16_t* decisions, hipStream_t st);

// Wave-tile variants of the linear LSERK4 step kernels (dg_wave.hip), selected by
// plan->lane_elems; `times` as for the workgroup-tile launchers.
int wave_launch_step(const dg_plan* p, int ms, const double* in, double* snap, double* last,
                     const double* times, double dt, hipStream_t st);

// The dataflow sweep (dg_sweep.hip): buffers of one launch.  U[b]: forward block b's input
// (U[0] = u0, U[nbF] = u^N), W[a]: adjoint block a's input (W[0] the terminal weight,
// W[nbA] the caller's w); part: (nbA - 1) rows of ktot indicator partials; sync: the
// sweep_sync_words() control words followed by one flag per item.
struct SweepBufs {
  double* U[9];
  double* W[9];
  double* rec;
  double* eta;
  double* part;
  uint32_t* sync;
  int64_t* am_idx;  // nullable: fused refine decision (dg_argmax_ex of |eta|)
  double* am_val;
  int64_t* am_nf;
  double* am_pv;    // partial winners, one per last-block tile
  int64_t* am_pi;
  uint32_t* err_host;  // nullable: the plan's host-visible watchdog flag (d_sweep_err)
  int32_t spin_limit;  // 0: the default
};
int sweep_tile_elems(const dg_plan* p, int waves);
int sweep_waves_per_simd(const dg_plan* p, int waves);  // the kernel's occupancy target (0: none)
// work items / last-block adjoint tiles of a dataflow sweep over the plan's ktot elements, or
// over `elems` (>= 0: the scratch sizing for the reserved capacity)
int64_t sweep_items(const dg_plan* p, int waves, int msf, int msa, int nsteps, int64_t elems = -1);
int64_t sweep_tiles_adj(const dg_plan* p, int waves, int msa, int64_t elems = -1);
int sweep_launch_rec(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b, double t0,
                     double dt, int nsteps, int mode, hipStream_t st);
int sweep_sync_words();
int sweep_max_steps();
// The plan's dataflow scratch (dg_advec.hip): a control region of `sync_bytes` (zeroed where
// newly covered) followed by `data_bytes`; *data = the data region.
int sweep_scratch(dg_plan* p, size_t sync_bytes, size_t data_bytes, hipStream_t st, char** data);
// Fails if an earlier dataflow launch of the plan gave up; maps the watchdog's host flag.
int sweep_watchdog(dg_plan* p);
int sweep_err_word();

// Jump-record sweep launches on pair tiles (dg_rec.hip), selected by plan->rec_lane_elems == 2.
int pair_launch_step_rec(const dg_plan* p, int ms, const double* in, double* rec, double* last,
                         const double* times, double dt, hipStream_t st, int64_t n0, bool jend);
// The snapshot forward on pair tiles (dg_rec.hip k_step_rps): ms steps from `in`, step st's
// state into snap + st * field.
int pair_launch_step_snap(const dg_plan* p, int ms, const double* in, double* snap,
                          const double* times, double dt, hipStream_t st);
int pair_launch_adj_rec(const dg_plan* p, int ms, const double* win, double* wout,
                        const double* rec, double* eta, int em, const double* t_next, double dt,
                        hipStream_t st, int64_t n0);

}  // namespace dgk
