// dg_advec.hip — MI355X (gfx950) kernels + C ABI for the 1D nodal-DG advection
// forward/adjoint time-stepper (see include/dg_advec.h for the contract and DESIGN.md
// for the data layout and rooflines).
//
// Hot kernels
//   k_step<NP,NS,UNI>   one fused time step (all NS stages of LSERK4 / Euler) of
//                       AdvecRHS1D (utils/AdvecRHS1D.m:9-19) + the low-storage update
//                       (utils/One_code.mlx:120-137).  One element per lane, the element's
//                       Np nodal values and the step-local RK residual in VGPRs, a
//                       256-element tile with an NS-element halo on each side staged
//                       through LDS with 16-byte coalesced loads, face values exchanged
//                       through LDS once per stage (one barrier per stage).
//   k_adj<NP,NS,UNI>    one fused reverse step: exact transpose of k_step's stages, the
//                       functional source and the dual-weighted interelement-jump residual
//                       accumulated into eta (pattern: python/Main_finite_difference.py:54-94).
// Support kernels: k_rhs (AdvecRHS1D for parity), k_limit (SlopeLimitN.m), k_argmax_*
// (numpy.argmax semantics), k_sum_rows, k_init_sine, k_axpy_copy.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <utility>
#include <string>
#include <vector>

#include "dg_advec.h"

#define DG_VERSION "dg_advec 0.1.0 (gfx950)"

namespace {

constexpr int kBlock = 256;       // lanes per workgroup = elements per tile (incl. halo)
constexpr int kMaxNP = 9;         // N <= 8
constexpr int kArgmaxParts = 1024;

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return fail(DG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
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

template <int NP, int NS> struct StepArgs {
  OpArgs<NP> op;
  double sc;          // dt * s (uniform mesh) or dt (non-uniform: times scale[k])
  double uin[NS];     // inflow value at each stage time
  int64_t ktot;       // batch * K elements
  int32_t K;          // elements per trajectory
};

template <int NP> struct AdjArgs {
  OpArgs<NP> op;
  double sc;          // as StepArgs
  double uin_res;     // inflow value at t_{n+1} for the residual
  double src;         // functional source coefficient for node n+1
  int64_t ktot;
  int32_t K;
  int32_t has_eta;
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

// Store `count` doubles from lds[0..count) to g[o0..o0+count); o0 must be even.
__device__ __forceinline__ void store_run(double* __restrict__ g, int64_t o0, int64_t count,
                                          const double* __restrict__ lds) {
  double2* __restrict__ g2 = reinterpret_cast<double2*>(g);
  for (int64_t v = threadIdx.x; 2 * v < count; v += kBlock) {
    const double2 val = *reinterpret_cast<const double2*>(&lds[2 * v]);
    const int64_t gd = o0 + 2 * v;
    if (2 * v + 1 < count) {
      g2[gd >> 1] = val;
    } else {
      g[gd] = val.x;
    }
  }
}

// ---------------------------------------------------------------------------
// Forward fused step.
// ---------------------------------------------------------------------------
template <int NP, int NS, bool UNI>
__global__ __launch_bounds__(kBlock) void k_step(const double* __restrict__ uin,
                                                 double* __restrict__ uout,
                                                 double* __restrict__ uout2,
                                                 const double* __restrict__ scale,
                                                 StepArgs<NP, NS> args) {
  constexpr int H = NS;               // dependency cone grows one element per stage
  constexpr int TE = kBlock - 2 * H;  // output elements per tile (even)
  static_assert(TE % 2 == 0, "tile output must be 16-byte aligned");
  __shared__ __attribute__((aligned(16))) double tile[kBlock * NP + 2];
  __shared__ double faceL[2][kBlock];
  __shared__ double faceR[2][kBlock];

  const int lane = threadIdx.x;
  const int64_t tile_id = blockIdx.x;
  const int64_t e0 = tile_id * TE - H;
  const int64_t e = e0 + lane;
  const int64_t nd = args.ktot * NP;

  const int off = load_tile<NP>(uin, e0, nd, tile);
  __syncthreads();

  double u[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) u[i] = tile[off + lane * NP + i];

  const bool inrange = (e >= 0 && e < args.ktot);
  const int32_t kl = inrange ? int32_t(e % args.K) : 0;
  const bool first = (kl == 0);
  const bool last = (kl == args.K - 1);
  double sc = args.sc;
  if constexpr (!UNI) sc *= inrange ? scale[kl] : 0.0;

  double res[NP];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int b = s & 1;
    faceL[b][lane] = u[0];
    faceR[b][lane] = u[NP - 1];
    __syncthreads();
    double uL = (lane > 0) ? faceR[b][lane - 1] : u[0];
    const double uR = (lane < kBlock - 1) ? faceL[b][lane + 1] : u[NP - 1];
    if (first) uL = args.uin[s];
    const double du0 = u[0] - uL;
    const double du1 = last ? 0.0 : (u[NP - 1] - uR);
    double acc[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      double t = args.op.L0[i] * du0;
      t = fma(args.op.L1[i], du1, t);
#pragma unroll
      for (int j = 0; j < NP; ++j) t = fma(args.op.Dm[i * NP + j], u[j], t);
      acc[i] = t;
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (s == 0) {
        res[i] = sc * acc[i];  // rk4a(1) = 0: the residual register is step-local
      } else {
        res[i] = fma(RK<NS>::A(s), res[i], sc * acc[i]);
      }
      u[i] = fma(RK<NS>::B(s), res[i], u[i]);
    }
  }

  // Stage the TE valid elements back through LDS (all reads of `tile` happened before
  // the first stage barrier) and store them with 16-byte coalesced writes.
  if (lane >= H && lane < kBlock - H) {
#pragma unroll
    for (int i = 0; i < NP; ++i) tile[(lane - H) * NP + i] = u[i];
  }
  __syncthreads();
  const int64_t o0 = tile_id * TE * NP;
  const int64_t rem = nd - o0;
  const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;
  store_run(uout, o0, count, tile);
  if (uout2 != nullptr) store_run(uout2, o0, count, tile);
}

// ---------------------------------------------------------------------------
// Adjoint fused step: w^n = S^T (w^{n+1} + src*u^{n+1}), eta += DWR contribution.
// Reverse of stage s (forward: r = A_s r + dt L u ; u = u + B_s r):
//   lr += B_s lu ;  lu += dt L^T lr ;  lr = A_s lr
// L^T per element with q = sc*lr, g0 = L0.q, g1 = L1.q:
//   (L^T)_j = sum_i Dm[i][j] q_i + [j=0](g0 - g1_{left}) + [j=N]([!last] g1 - [!last] g0_{right})
// ---------------------------------------------------------------------------
template <int NP, int NS, bool UNI>
__global__ __launch_bounds__(kBlock) void k_adj(const double* __restrict__ win,
                                                double* __restrict__ wout,
                                                const double* __restrict__ usnap,
                                                double* __restrict__ eta,
                                                const double* __restrict__ scale,
                                                AdjArgs<NP> args) {
  constexpr int H = NS;
  constexpr int TE = kBlock - 2 * H;
  __shared__ __attribute__((aligned(16))) double tile_w[kBlock * NP + 2];
  __shared__ __attribute__((aligned(16))) double tile_u[kBlock * NP + 2];
  __shared__ double G0[2][kBlock];
  __shared__ double G1[2][kBlock];

  const int lane = threadIdx.x;
  const int64_t tile_id = blockIdx.x;
  const int64_t e0 = tile_id * TE - H;
  const int64_t e = e0 + lane;
  const int64_t nd = args.ktot * NP;

  const int offw = load_tile<NP>(win, e0, nd, tile_w);
  const int offu = load_tile<NP>(usnap, e0, nd, tile_u);
  __syncthreads();

  const bool inrange = (e >= 0 && e < args.ktot);
  const int32_t kl = inrange ? int32_t(e % args.K) : 0;
  const bool first = (kl == 0);
  const bool last = (kl == args.K - 1);
  double sc = args.sc;
  if constexpr (!UNI) sc *= inrange ? scale[kl] : 0.0;

  double lu[NP], us[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    lu[i] = tile_w[offw + lane * NP + i];
    us[i] = tile_u[offu + lane * NP + i];
  }
  // Neighbour face values of the snapshot for the jump residual.
  const double usL = (lane > 0) ? tile_u[offu + (lane - 1) * NP + (NP - 1)] : us[0];
  const double usR = (lane < kBlock - 1) ? tile_u[offu + (lane + 1) * NP] : us[NP - 1];

  // Functional source K^{n+1} = src * u^{n+1}.
  if (args.src != 0.0) {
#pragma unroll
    for (int i = 0; i < NP; ++i) lu[i] = fma(args.src, us[i], lu[i]);
  }

  // Dual-weighted interelement-jump residual at t_{n+1}:
  //   dt * sum_i w_i * s*(L0_i du0 + L1_i du1) = sc * (du0 * (L0.w) + du1 * (L1.w))
  if (args.has_eta) {
    const double du0 = us[0] - (first ? args.uin_res : usL);
    const double du1 = last ? 0.0 : (us[NP - 1] - usR);
    double gw0 = 0.0, gw1 = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      gw0 = fma(args.op.L0[i], lu[i], gw0);
      gw1 = fma(args.op.L1[i], lu[i], gw1);
    }
    const double contrib = sc * fma(du0, gw0, du1 * gw1);
    if (inrange && lane >= H && lane < kBlock - H) eta[e] += contrib;
  }

  double lr[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) lr[i] = 0.0;

#pragma unroll
  for (int ss = 0; ss < NS; ++ss) {
    const int s = NS - 1 - ss;
    const int b = ss & 1;
    double q[NP];
    double g0 = 0.0, g1 = 0.0;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      lr[i] = fma(RK<NS>::B(s), lu[i], lr[i]);
      q[i] = sc * lr[i];
      g0 = fma(args.op.L0[i], q[i], g0);
      g1 = fma(args.op.L1[i], q[i], g1);
    }
    G0[b][lane] = g0;
    G1[b][lane] = g1;
    __syncthreads();
    const double g1_left = (!first && lane > 0) ? G1[b][lane - 1] : 0.0;
    const double g0_right = (!last && lane < kBlock - 1) ? G0[b][lane + 1] : 0.0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      double t = lu[j];
#pragma unroll
      for (int i = 0; i < NP; ++i) t = fma(args.op.Dm[i * NP + j], q[i], t);
      lu[j] = t;
    }
    lu[0] += g0 - g1_left;
    lu[NP - 1] += (last ? 0.0 : g1) - g0_right;
#pragma unroll
    for (int i = 0; i < NP; ++i) lr[i] = RK<NS>::A(s) * lr[i];
  }

  if (lane >= H && lane < kBlock - H) {
#pragma unroll
    for (int i = 0; i < NP; ++i) tile_w[(lane - H) * NP + i] = lu[i];
  }
  __syncthreads();
  const int64_t o0 = tile_id * TE * NP;
  const int64_t rem = nd - o0;
  const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;
  store_run(wout, o0, count, tile_w);
}

// ---------------------------------------------------------------------------
// AdvecRHS1D (parity entry point): one element per thread, global neighbour reads.
// ---------------------------------------------------------------------------
template <int NP>
__global__ __launch_bounds__(kBlock) void k_rhs(const double* __restrict__ u,
                                                double* __restrict__ rhs,
                                                const double* __restrict__ scale, OpArgs<NP> op,
                                                double s_uni, double uin, int64_t ktot,
                                                int32_t K) {
  const int64_t e = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= ktot) return;
  const int32_t kl = int32_t(e % K);
  const bool first = (kl == 0), last = (kl == K - 1);
  double v[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) v[i] = u[e * NP + i];
  const double uL = first ? uin : u[(e - 1) * NP + NP - 1];
  const double du0 = v[0] - uL;
  const double du1 = last ? 0.0 : (v[NP - 1] - u[(e + 1) * NP]);
  const double s = scale ? scale[kl] : s_uni;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double t = op.L0[i] * du0;
    t = fma(op.L1[i], du1, t);
#pragma unroll
    for (int j = 0; j < NP; ++j) t = fma(op.Dm[i * NP + j], v[j], t);
    rhs[e * NP + i] = s * t;
  }
}

// ---------------------------------------------------------------------------
// SlopeLimitN (utils/SlopeLimitN.m:9-32) with SlopeLimitLin (SlopeLimitLin.m:10-18) and
// minmod (minmod.m:6-12).  Evaluated with FP contraction OFF and in the reference's
// left-to-right order so the troubled-cell decision `ids` is bit-exact with the oracle.
// ---------------------------------------------------------------------------
template <int NP> struct LimArgs {
  double invV0[NP];  // row 1 of invV  (cell-average mode)
  double invV1[NP];  // row 2 of invV  (linear mode)
  double V0[NP];     // column 1 of V
  double V1[NP];     // column 2 of V
  double Dr0[NP];    // row 1 of Dr
  double rp1h[NP];   // 0.5*(r_i + 1)  (StartUp1D.m:20)
  int64_t ktot;
  int32_t K;
};

__device__ __forceinline__ double msign(double x) { return (x > 0.0) ? 1.0 : ((x < 0.0) ? -1.0 : 0.0); }

__device__ __forceinline__ double minmod3(double a, double b, double c) {
#pragma clang fp contract(off)
  const double s = (msign(a) + msign(b) + msign(c)) / 3.0;
  if (fabs(s) == 1.0) {
    double m = fabs(a);
    m = fmin(m, fabs(b));
    m = fmin(m, fabs(c));
    return s * m;
  }
  return 0.0;
}

template <int NP>
__global__ __launch_bounds__(kBlock) void k_limit(const double* __restrict__ u,
                                                  double* __restrict__ ulim,
                                                  int32_t* __restrict__ ids,
                                                  const double* __restrict__ VX,
                                                  LimArgs<NP> args) {
#pragma clang fp contract(off)
  constexpr int H = 1;
  constexpr int TE = kBlock - 2 * H;
  __shared__ __attribute__((aligned(16))) double tile[kBlock * NP + 2];
  __shared__ double vavg[kBlock];
  const int lane = threadIdx.x;
  const int64_t tile_id = blockIdx.x;
  const int64_t e0 = tile_id * TE - H;
  const int64_t e = e0 + lane;
  const int64_t nd = args.ktot * NP;
  const int off = load_tile<NP>(u, e0, nd, tile);
  __syncthreads();
  double v[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) v[i] = tile[off + lane * NP + i];
  const bool inrange = (e >= 0 && e < args.ktot);
  const int32_t kl = inrange ? int32_t(e % args.K) : 0;
  const bool first = (kl == 0), last = (kl == args.K - 1);

  // Cell average: uh = invV*u; uh(2:Np)=0; v = (V*uh)(1)  (SlopeLimitN.m:9)
  double uh0 = args.invV0[0] * v[0];
#pragma unroll
  for (int j = 1; j < NP; ++j) uh0 = uh0 + args.invV0[j] * v[j];
  const double vk = args.V0[0] * uh0;
  vavg[lane] = vk;
  __syncthreads();
  // Neighbour averages, replicated at the trajectory ends (SlopeLimitN.m:18).
  const double vkm1 = (first || lane == 0) ? vk : vavg[lane - 1];
  const double vkp1 = (last || lane == kBlock - 1) ? vk : vavg[lane + 1];
  const double ue1 = v[0], ue2 = v[NP - 1];
  const double ve1 = vk - minmod3(vk - ue1, vk - vkm1, vkp1 - vk);   // :21
  const double ve2 = vk + minmod3(ue2 - vk, vk - vkm1, vkp1 - vk);   // :22
  const double eps0 = 1.0e-8;
  const bool flag = (fabs(ve1 - ue1) > eps0) || (fabs(ve2 - ue2) > eps0);  // :23

  double out[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) out[i] = v[i];
  if (flag) {
    // Piecewise-linear projection (SlopeLimitN.m:28) then SlopeLimitLin.m:10-18.
    double uh1 = args.invV1[0] * v[0];
#pragma unroll
    for (int j = 1; j < NP; ++j) uh1 = uh1 + args.invV1[j] * v[j];
    double ul[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) ul[i] = args.V0[i] * uh0 + args.V1[i] * uh1;
    const double xa = VX[kl], xb = VX[kl + 1];
    double x[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) x[i] = xa + args.rp1h[i] * (xb - xa);
    const double h = x[NP - 1] - x[0];
    const double x0 = x[0] + h / 2.0;
    double d = args.Dr0[0] * ul[0];
#pragma unroll
    for (int j = 1; j < NP; ++j) d = d + args.Dr0[j] * ul[j];
    const double ux0 = (2.0 / h) * d;
    const double m = minmod3(ux0, (vkp1 - vk) / h, (vk - vkm1) / h);
#pragma unroll
    for (int i = 0; i < NP; ++i) out[i] = vk + (x[i] - x0) * m;
  }
  if (inrange && lane >= H && lane < kBlock - H) {
    if (ids) ids[e] = flag ? 1 : 0;
  }
  __syncthreads();
  if (lane >= H && lane < kBlock - H) {
#pragma unroll
    for (int i = 0; i < NP; ++i) tile[(lane - H) * NP + i] = out[i];
  }
  __syncthreads();
  const int64_t o0 = tile_id * TE * NP;
  const int64_t rem = nd - o0;
  const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;
  store_run(ulim, o0, count, tile);
}

// ---------------------------------------------------------------------------
// argmax with numpy semantics: NaN is the maximum, ties go to the lowest index.
// (value, index) under this order is a strict total order, so the two-pass block
// reduction is independent of scheduling.
// ---------------------------------------------------------------------------
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
    if (threadIdx.x < w) {
      const double ov = sv[threadIdx.x + w];
      const int64_t oi = si[threadIdx.x + w];
      if (better(ov, oi, sv[threadIdx.x], si[threadIdx.x])) {
        sv[threadIdx.x] = ov;
        si[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  v = sv[0];
  idx = si[0];
}

__global__ __launch_bounds__(kBlock) void k_argmax_partial(const double* __restrict__ x,
                                                           int64_t n, int use_abs,
                                                           double* __restrict__ pv,
                                                           int64_t* __restrict__ pi) {
  double bv = 0.0;
  int64_t bi = -1;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    const double v = use_abs ? fabs(x[i]) : x[i];
    if (bi < 0 || better(v, i, bv, bi)) {
      bv = v;
      bi = i;
    }
  }
  if (bi < 0) {  // thread saw nothing: weakest possible candidate
    bv = -INFINITY;
    bi = INT64_MAX;
  }
  block_argmax(bv, bi);
  if (threadIdx.x == 0) {
    pv[blockIdx.x] = bv;
    pi[blockIdx.x] = bi;
  }
}

__global__ __launch_bounds__(kBlock) void k_argmax_final(const double* __restrict__ pv,
                                                         const int64_t* __restrict__ pi,
                                                         int nparts, int64_t* __restrict__ out) {
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  for (int p = threadIdx.x; p < nparts; p += kBlock) {
    if (better(pv[p], pi[p], bv, bi)) {
      bv = pv[p];
      bi = pi[p];
    }
  }
  block_argmax(bv, bi);
  if (threadIdx.x == 0) out[0] = bi;
}

__global__ __launch_bounds__(kBlock) void k_sum_rows(const double* __restrict__ x, int64_t rows,
                                                     int64_t n, double* __restrict__ out) {
  const int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= n) return;
  double acc = x[k];
  for (int64_t r = 1; r < rows; ++r) acc = acc + x[r * n + k];
  out[k] = acc;
}

template <int NP>
__global__ __launch_bounds__(kBlock) void k_init_sine(const double* __restrict__ VX,
                                                      const double* __restrict__ amp,
                                                      const double* __restrict__ freq,
                                                      const double* __restrict__ phase,
                                                      double* __restrict__ u, LimArgs<NP> args) {
  const int64_t e = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= args.ktot) return;
  const int64_t b = e / args.K;
  const int32_t kl = int32_t(e - b * args.K);
  const double xa = VX[kl], xb = VX[kl + 1];
  const double A = amp[b], m = freq[b], ph = phase[b];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const double x = xa + args.rp1h[i] * (xb - xa);
    u[e * NP + i] = A * sin(2.0 * M_PI * m * x + ph);
  }
}

__global__ __launch_bounds__(kBlock) void k_axpy_copy(const double* __restrict__ w,
                                                      const double* __restrict__ u, double c,
                                                      double* __restrict__ out, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = fma(c, u[i], w[i]);
}

}  // namespace

// ---------------------------------------------------------------------------
// Plan
// ---------------------------------------------------------------------------
struct dg_plan {
  int N = 0, NP = 0;
  int64_t K = 0, batch = 0, ktot = 0;
  double a = 0.0;
  int inflow = 0, scheme = 0, nstages = 5;
  bool uniform = true;
  double s_uniform = 0.0;  // 2/h for uniform meshes
  double r[kMaxNP], V[kMaxNP * kMaxNP], invV[kMaxNP * kMaxNP], Dr[kMaxNP * kMaxNP],
      LIFT[kMaxNP * 2];
  double* d_scale = nullptr;  // K: 2/h_k
  double* d_VX = nullptr;     // K+1
  double* d_scratch = nullptr;
  double* d_pv = nullptr;
  int64_t* d_pi = nullptr;
};

namespace {

double inflow_value(const dg_plan* p, double t) {
  return (p->inflow == DG_INFLOW_SIN_A2T) ? -std::sin(p->a * p->a * t) : -std::sin(p->a * t);
}

template <int NP> OpArgs<NP> make_op(const dg_plan* p) {
  OpArgs<NP> op;
  for (int i = 0; i < NP; ++i) {
    for (int j = 0; j < NP; ++j) op.Dm[i * NP + j] = -p->a * p->Dr[i * NP + j];
    op.L0[i] = (-p->a / 2.0) * p->LIFT[i * 2 + 0];
    op.L1[i] = (p->a / 2.0) * p->LIFT[i * 2 + 1];
  }
  return op;
}

template <int NP> LimArgs<NP> make_lim(const dg_plan* p) {
  LimArgs<NP> la;
  for (int i = 0; i < NP; ++i) {
    la.invV0[i] = p->invV[0 * NP + i];
    la.invV1[i] = p->invV[1 * NP + i];
    la.V0[i] = p->V[i * NP + 0];
    la.V1[i] = p->V[i * NP + 1];
    la.Dr0[i] = p->Dr[0 * NP + i];
    la.rp1h[i] = 0.5 * (p->r[i] + 1.0);
  }
  la.ktot = p->ktot;
  la.K = int32_t(p->K);
  return la;
}

inline unsigned grid_for(int64_t n, int64_t per) { return unsigned((n + per - 1) / per); }

template <int NP, int NS>
int launch_step_t(const dg_plan* p, const double* in, double* out, double* out2,
                  double t, double dt, hipStream_t st) {
  StepArgs<NP, NS> a;
  a.op = make_op<NP>(p);
  a.sc = p->uniform ? dt * p->s_uniform : dt;
  for (int s = 0; s < NS; ++s) a.uin[s] = inflow_value(p, t + RK<NS>::C(s) * dt);
  a.ktot = p->ktot;
  a.K = int32_t(p->K);
  const unsigned grid = grid_for(p->ktot, kBlock - 2 * NS);
  if (p->uniform)
    hipLaunchKernelGGL((k_step<NP, NS, true>), dim3(grid), dim3(kBlock), 0, st, in, out, out2,
                       p->d_scale, a);
  else
    hipLaunchKernelGGL((k_step<NP, NS, false>), dim3(grid), dim3(kBlock), 0, st, in, out, out2,
                       p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP, int NS>
int launch_adj_t(const dg_plan* p, const double* win, double* wout, const double* usnap,
                 double* eta, double t_next, double dt, double src, hipStream_t st) {
  AdjArgs<NP> a;
  a.op = make_op<NP>(p);
  a.sc = p->uniform ? dt * p->s_uniform : dt;
  a.uin_res = inflow_value(p, t_next);
  a.src = src;
  a.ktot = p->ktot;
  a.K = int32_t(p->K);
  a.has_eta = eta != nullptr;
  const unsigned grid = grid_for(p->ktot, kBlock - 2 * NS);
  if (p->uniform)
    hipLaunchKernelGGL((k_adj<NP, NS, true>), dim3(grid), dim3(kBlock), 0, st, win, wout, usnap,
                       eta, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_adj<NP, NS, false>), dim3(grid), dim3(kBlock), 0, st, win, wout,
                       usnap, eta, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

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

int launch_step(const dg_plan* p, const double* in, double* out, double* out2, double t,
                double dt, hipStream_t st) {
  int rc = DG_OK;
  if (p->nstages == 5) {
    DG_DISPATCH_NP(p->NP, rc = (launch_step_t<NP, 5>(p, in, out, out2, t, dt, st)));
  } else {
    DG_DISPATCH_NP(p->NP, rc = (launch_step_t<NP, 1>(p, in, out, out2, t, dt, st)));
  }
  return rc;
}

int launch_adj(const dg_plan* p, const double* win, double* wout, const double* usnap,
               double* eta, double t_next, double dt, double src, hipStream_t st) {
  int rc = DG_OK;
  if (p->nstages == 5) {
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_t<NP, 5>(p, win, wout, usnap, eta, t_next, dt, src, st)));
  } else {
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_t<NP, 1>(p, win, wout, usnap, eta, t_next, dt, src, st)));
  }
  return rc;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* dg_last_error(void) { return g_err.c_str(); }

const char* dg_version(void) { return DG_VERSION; }

int dg_plan_create(int N, int64_t K, int64_t batch, const double* r, const double* V,
                   const double* invV, const double* Dr, const double* LIFT, const double* VX,
                   double a, int inflow_variant, int time_scheme, dg_plan** out) {
  g_err.clear();
  if (!out) return fail(DG_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (N < 1 || N > kMaxNP - 1) return fail(DG_ERR_ARG, "N must be in 1..8");
  if (K < 2 || batch < 1) return fail(DG_ERR_ARG, "need K >= 2 and batch >= 1");
  if (K > INT32_MAX || K * batch > (int64_t(1) << 40))
    return fail(DG_ERR_ARG, "K*batch too large");
  if (!r || !V || !invV || !Dr || !LIFT || !VX) return fail(DG_ERR_ARG, "null operator pointer");
  if (inflow_variant != DG_INFLOW_SIN_AT && inflow_variant != DG_INFLOW_SIN_A2T)
    return fail(DG_ERR_ARG, "bad inflow_variant");
  if (time_scheme != DG_TIME_LSERK4 && time_scheme != DG_TIME_EULER)
    return fail(DG_ERR_ARG, "bad time_scheme");
  dg_plan* p = new (std::nothrow) dg_plan();
  if (!p) return fail(DG_ERR_NOMEM, "host allocation failed");
  p->N = N;
  p->NP = N + 1;
  p->K = K;
  p->batch = batch;
  p->ktot = K * batch;
  p->a = a;
  p->inflow = inflow_variant;
  p->scheme = time_scheme;
  p->nstages = (time_scheme == DG_TIME_LSERK4) ? 5 : 1;
  const int NP = p->NP;
  std::memcpy(p->r, r, sizeof(double) * NP);
  std::memcpy(p->V, V, sizeof(double) * NP * NP);
  std::memcpy(p->invV, invV, sizeof(double) * NP * NP);
  std::memcpy(p->Dr, Dr, sizeof(double) * NP * NP);
  std::memcpy(p->LIFT, LIFT, sizeof(double) * NP * 2);

  std::vector<double> scale(K);
  double hmin = 1e300, hmax = -1e300, hsum = 0.0;
  for (int64_t k = 0; k < K; ++k) {
    const double h = VX[k + 1] - VX[k];
    if (!(h > 0.0)) {
      delete p;
      return fail(DG_ERR_ARG, "VX must be strictly increasing");
    }
    scale[k] = 2.0 / h;
    hmin = h < hmin ? h : hmin;
    hmax = h > hmax ? h : hmax;
    hsum += h;
  }
  const double hmean = hsum / double(K);
  p->uniform = (hmax - hmin) <= 1e-12 * hmean;
  p->s_uniform = 2.0 / hmean;

  auto cleanup = [&](const std::string& m) {
    dg_plan_destroy(p);
    return fail(DG_ERR_NOMEM, m);
  };
  if (hipMalloc(&p->d_scale, sizeof(double) * K) != hipSuccess) return cleanup("hipMalloc scale");
  if (hipMalloc(&p->d_VX, sizeof(double) * (K + 1)) != hipSuccess) return cleanup("hipMalloc VX");
  if (hipMalloc(&p->d_scratch, sizeof(double) * p->ktot * NP) != hipSuccess)
    return cleanup("hipMalloc scratch");
  if (hipMalloc(&p->d_pv, sizeof(double) * kArgmaxParts) != hipSuccess) return cleanup("hipMalloc pv");
  if (hipMalloc(&p->d_pi, sizeof(int64_t) * kArgmaxParts) != hipSuccess) return cleanup("hipMalloc pi");
  if (hipMemcpy(p->d_scale, scale.data(), sizeof(double) * K, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->d_VX, VX, sizeof(double) * (K + 1), hipMemcpyHostToDevice) != hipSuccess) {
    dg_plan_destroy(p);
    return fail(DG_ERR_HIP, "hipMemcpy of mesh failed");
  }
  *out = p;
  return DG_OK;
}

int dg_plan_destroy(dg_plan* p) {
  if (!p) return DG_OK;
  if (p->d_scale) (void)hipFree(p->d_scale);
  if (p->d_VX) (void)hipFree(p->d_VX);
  if (p->d_scratch) (void)hipFree(p->d_scratch);
  if (p->d_pv) (void)hipFree(p->d_pv);
  if (p->d_pi) (void)hipFree(p->d_pi);
  delete p;
  return DG_OK;
}

int dg_plan_query(const dg_plan* p, int64_t out[6]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  out[0] = p->N;
  out[1] = p->NP;
  out[2] = p->K;
  out[3] = p->batch;
  out[4] = p->uniform ? 1 : 0;
  out[5] = p->nstages;
  return DG_OK;
}

int dg_advec_rhs(const dg_plan* p, const double* u, double* rhs, double t, void* stream) {
  if (!p || !u || !rhs) return fail(DG_ERR_ARG, "null argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const double uin = inflow_value(p, t);
  const unsigned grid = grid_for(p->ktot, kBlock);
  const double* sc = p->uniform ? nullptr : p->d_scale;
  DG_DISPATCH_NP(p->NP, hipLaunchKernelGGL((k_rhs<NP>), dim3(grid), dim3(kBlock), 0, st, u, rhs,
                                           sc, make_op<NP>(p), p->s_uniform, uin, p->ktot,
                                           int32_t(p->K)));
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_lserk4_fwd(dg_plan* p, double* u, double t0, double dt, int nsteps, double* snapshots,
                  void* stream) {
  if (!p || !u) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (nsteps == 0) return DG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t field = p->ktot * p->NP;
  double time = t0;  // time = time + dt, as One_code.mlx:139
  if (snapshots) {
    if (snapshots != u)
      HIP_TRY(hipMemcpyAsync(snapshots, u, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    for (int n = 0; n < nsteps; ++n) {
      double* out2 = (n == nsteps - 1 && snapshots != u) ? u : nullptr;
      const int rc = launch_step(p, snapshots + int64_t(n) * field,
                                 snapshots + int64_t(n + 1) * field, out2, time, dt, st);
      if (rc) return rc;
      time = time + dt;
    }
    return DG_OK;
  }
  // Ping-pong between u and the plan scratch; the last step lands in u.
  // Step n writes b then swaps, so the last write lands in u when the first source
  // is u for even nsteps and the scratch copy of u for odd nsteps.
  double* a = u;
  double* b = p->d_scratch;
  if (nsteps % 2 == 1) {
    HIP_TRY(hipMemcpyAsync(b, a, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    std::swap(a, b);  // a = scratch (holds u^0), b = u
  }
  for (int n = 0; n < nsteps; ++n) {
    const int rc = launch_step(p, a, b, nullptr, time, dt, st);
    if (rc) return rc;
    std::swap(a, b);
    time = time + dt;
  }
  return DG_OK;
}

int dg_lserk4_adj(dg_plan* p, double* w, const double* snapshots, double t0, double dt,
                  int nsteps, double src_coef, double* eta, void* stream) {
  if (!p || !w || !snapshots) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t field = p->ktot * p->NP;
  // Same time levels as the forward sweep (repeated addition).
  std::vector<double> tn(size_t(nsteps) + 1);
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  double* a = w;
  double* b = p->d_scratch;
  for (int n = nsteps - 1; n >= 0; --n) {
    const double src = (n == nsteps - 1) ? 0.0 : src_coef;
    const int rc = launch_adj(p, a, b, snapshots + int64_t(n + 1) * field, eta, tn[n + 1], dt,
                              src, st);
    if (rc) return rc;
    std::swap(a, b);
  }
  // Node-0 source and the hand-back into w.
  if (src_coef != 0.0 || a != w) {
    const double c = (nsteps > 0) ? src_coef : 0.0;
    hipLaunchKernelGGL(k_axpy_copy, dim3(grid_for(field, kBlock)), dim3(kBlock), 0, st, a,
                       snapshots, c, w, field);
    HIP_TRY(hipGetLastError());
  }
  return DG_OK;
}

int dg_slope_limit_n(dg_plan* p, const double* u, double* ulim, int32_t* ids, void* stream) {
  if (!p || !u || !ulim) return fail(DG_ERR_ARG, "null argument");
  if (u == ulim) return fail(DG_ERR_ARG, "in-place limiting is not supported (tiles overlap)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = grid_for(p->ktot, kBlock - 2);
  DG_DISPATCH_NP(p->NP, hipLaunchKernelGGL((k_limit<NP>), dim3(grid), dim3(kBlock), 0, st, u,
                                           ulim, ids, p->d_VX, make_lim<NP>(p)));
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_argmax(dg_plan* p, const double* x, int64_t n, int use_abs, int64_t* idx, void* stream) {
  if (!p || !x || !idx) return fail(DG_ERR_ARG, "null argument");
  if (n < 1 || n > p->ktot * p->NP) return fail(DG_ERR_ARG, "n out of range");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t parts = (n + 4 * kBlock - 1) / (4 * kBlock);
  if (parts > kArgmaxParts) parts = kArgmaxParts;
  hipLaunchKernelGGL(k_argmax_partial, dim3(unsigned(parts)), dim3(kBlock), 0, st, x, n, use_abs,
                     p->d_pv, p->d_pi);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_argmax_final, dim3(1), dim3(kBlock), 0, st, p->d_pv, p->d_pi, int(parts),
                     idx);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_sum_rows(const double* x, int64_t rows, int64_t n, double* out, void* stream) {
  if (!x || !out) return fail(DG_ERR_ARG, "null argument");
  if (rows < 1 || n < 1) return fail(DG_ERR_ARG, "rows and n must be >= 1");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_sum_rows, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, x, rows, n, out);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_init_sine(const dg_plan* p, const double* amp, const double* freq, const double* phase,
                 double* u, void* stream) {
  if (!p || !amp || !freq || !phase || !u) return fail(DG_ERR_ARG, "null argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = grid_for(p->ktot, kBlock);
  DG_DISPATCH_NP(p->NP, hipLaunchKernelGGL((k_init_sine<NP>), dim3(grid), dim3(kBlock), 0, st,
                                           p->d_VX, amp, freq, phase, u, make_lim<NP>(p)));
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

}  // extern "C"
