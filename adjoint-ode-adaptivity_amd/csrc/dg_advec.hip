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
#include "dg_step_tile.h"

#define DG_VERSION "dg_advec 0.1.0 (gfx950)"

namespace dgk {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace dgk

namespace {
using namespace dgk;

template <int NP, int NS, bool UNI, int W, int MS, bool REC>
__global__ __launch_bounds__(kBlock * W) void k_step(const double* __restrict__ uin,
                                                     double* __restrict__ snap,
                                                     double* __restrict__ last,
                                                     const double* __restrict__ scale,
                                                     StepArgs<NP, NS, MS> args);
template <int NP, int NS, bool UNI, int W, int MS, bool REC>
__global__ __launch_bounds__(kBlock * W) void k_adj(const double* __restrict__ win,
                                                    double* __restrict__ wout,
                                                    const double* __restrict__ snap,
                                                    double* __restrict__ eta,
                                                    const double* __restrict__ scale,
                                                    AdjArgs<NP, MS> args);

template <int NP, int NS, bool UNI, int W, int MS, bool REC>
__global__ __launch_bounds__(kBlock * W) void k_step(const double* __restrict__ uin,
                                                     double* __restrict__ snap,
                                                     double* __restrict__ last,
                                                     const double* __restrict__ scale,
                                                     StepArgs<NP, NS, MS> args) {
  using G = TileGeo<NP, W>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * NS + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = MS * NS + (REC ? 1 : 0);
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  // the edge tiles' lane-indexed inflow values, read straight from the kernel-argument
  // segment (layout pinned by kernarg_tail): read as a uniform struct member, the compiler
  // hoists these 2*MS*NS SGPRs over the whole kernel and pushes the interior path into SGPR
  // spills
  using SArgs = StepArgs<NP, NS, MS>;
  const double* kin = reinterpret_cast<const double*>(
      kernarg_tail<decltype(&k_step<NP, NS, UNI, W, MS, REC>), SArgs>() + offsetof(SArgs, uin));
  if (edge_tile(e0, G::T, args.ktot, args.K))
    step_tile<NP, NS, UNI, W, MS, REC, true>(lds, tile, uin, snap, last, scale, args, kin);
  else
    step_tile<NP, NS, UNI, W, MS, REC, false>(lds, tile, uin, snap, last, scale, args, kin);
}

// ---------------------------------------------------------------------------
// Adjoint fused kernel: MS reverse steps st = MS-1..0, each
//   w^{n+st+1} += src_st * u^{n+st+1};  eta += DWR(u^{n+st+1}, w^{n+st+1});  w^{n+st} = S^T w^{n+st+1}
// with u^{n+st+1} = snap + st*stride.  Reverse of stage s (forward: r = A_s r + dt L u ;
// u = u + B_s r):  lr += B_s lu ;  lu += dt L^T lr ;  lr = A_s lr.
// The adjoint lives in the dual even/odd coordinates (the transpose of the inverse
// transform): we_k = w_k + w_{N-k}, wo_k = w_k - w_{N-k}, we_NO = w_mid.
// Indicator: eta += dt * sum_i w_i * s*(L0_i du0 + L1_i du1), with L0.w = le.we + lo.wo and
// L1.w = -le.we + lo.wo.  The next snapshot tile is prefetched during each step's stages.
// ---------------------------------------------------------------------------
template <int NP, int NS, bool UNI, int W, int MS, bool REC, bool EDGE>
__device__ __forceinline__ void adj_tile(double* __restrict__ lds, int64_t tile,
                                         const double* __restrict__ win,
                                         double* __restrict__ wout,
                                         const double* __restrict__ snap,
                                         double* __restrict__ eta,
                                         const double* __restrict__ scale,
                                         const AdjArgs<NP, MS>& args) {
  using G = TileGeo<NP, W>;
  constexpr int T = G::T, LB = G::LB, EPL = 1;
  constexpr int H = MS * NS;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;

  constexpr int CB = G::kLds;  // lds[CB + st] = inflow value at t_{n+st+1}; lds[CB + MS] = 0
  TileRegs<NP, W> pw, pu;
  // REC: the left-face jumps of u^{n0+st+1} (record n0+st) of the lane's element and of its
  // right neighbour, two 8-byte loads per lane and step, prefetched a step ahead
  const bool jin = REC && e0 + lane >= 0 && e0 + lane < args.ktot;
  const bool jin1 = REC && e0 + lane + 1 >= 0 && e0 + lane + 1 < args.ktot;
  double jn = 0.0, jn1 = 0.0;
  tile_issue<NP, W, EDGE>(win, e0, nd, pw);
  if constexpr (REC) {
    const double* row = jump_row(const_cast<double*>(snap), args.n0 + MS - 1, args.ktot);
    if (jin) jn = row[e0 + lane];
    if (jin1) jn1 = row[e0 + lane + 1];
  } else {
    tile_issue<NP, W, EDGE>(snap + (MS - 1) * args.stride, e0, nd, pu);
  }
  tile_commit<NP, W>(pw, lds);
  if constexpr (EDGE) {
    using AArgs = AdjArgs<NP, MS>;
    const double* ka = reinterpret_cast<const double*>(  // see step_tile
        kernarg_tail<decltype(&k_adj<NP, NS, UNI, W, MS, REC>), AArgs>() +
        offsetof(AArgs, uin_res));
    if (lane < MS) lds[CB + lane] = ka[lane];
    if (lane == MS) lds[CB + MS] = 0.0;
  }
  __syncthreads();
  double we[EPL][NE], wo[EPL][NO];
#pragma unroll
  for (int m = 0; m < EPL; ++m) {
    const double* w = lds + pw.off + (m * LB + lane) * NP;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[m][k] = w[k] + w[N - k];
      wo[m][k] = w[k] - w[N - k];
    }
    if constexpr (NE > NO) we[m][NO] = w[NO];
  }

  Elem E[EPL];
  double sc[EPL];
  double eacc[EPL];
#pragma unroll
  for (int m = 0; m < EPL; ++m) {
    E[m] = elem_info<H, T, EDGE>(e0, m * LB + lane, args.ktot, args.K);
    sc[m] = args.sc;
    if constexpr (!UNI) sc[m] *= E[m].inrange ? scale[E[m].kl] : 0.0;
    eacc[m] = 0.0;
  }

#pragma unroll
  for (int st = MS - 1; st >= 0; --st) {
    if constexpr (REC) {
      // no snapshot: the record's jumps replace the staged tile's neighbour faces
      const double jc = jn, jc1 = jn1;
      if (st > 0) {
        const double* row = jump_row(const_cast<double*>(snap), args.n0 + st - 1, args.ktot);
        if (jin) jn = row[e0 + lane];
        if (jin1) jn1 = row[e0 + lane + 1];
      }
      if (args.has_eta) {
        double pe = 0.0, po = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) pe = fma(args.op.le[k], we[0][k], pe);
#pragma unroll
        for (int k = 0; k < NO; ++k) po = fma(args.op.lo[k], wo[0][k], po);
        // du0 = j_e, du1 = -j_{e+1} (0 at a trajectory's last element)
        const bool lst = EDGE && E[0].last;
        double c = fma(lst ? jc : jc + jc1, pe, (lst ? jc : jc - jc1) * po);
        if constexpr (!UNI) c *= sc[0];
        eacc[0] += c;
      }
    }
    // The w tile's readers must be done before the first snapshot overwrites the image;
    // later snapshots follow 5 stage barriers after the previous one's reads.
    if (!REC && st == MS - 1) __syncthreads();
    if constexpr (!REC) tile_commit<NP, W>(pu, lds);
    const int off = REC ? 0 : pu.off;
    if constexpr (!REC) __syncthreads();
    if (!REC && st > 0) tile_issue<NP, W, EDGE>(snap + (st - 1) * args.stride, e0, nd, pu);
#pragma unroll
    for (int m = 0; m < (REC ? 0 : EPL); ++m) {
      const int el = m * LB + lane;
      const double* us = lds + off + el * NP;
      if (args.src[st] != 0.0) {  // functional source (dual coordinates)
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          we[m][k] = fma(args.src[st], us[k] + us[N - k], we[m][k]);
          wo[m][k] = fma(args.src[st], us[k] - us[N - k], wo[m][k]);
        }
        if constexpr (NE > NO) we[m][NO] = fma(args.src[st], us[NO], we[m][NO]);
      }
      if (args.has_eta) {
        // Neighbour face values of the snapshot for the jump residual.
        // Lane 0 / lane T-1 read their own end node (in range; halo results are dropped).
        // Edge tiles: a trajectory's first element reads the inflow value, its last
        // element its own right node (du1 = 0).
        int iL = off + (el > 0 ? (el - 1) * NP + (NP - 1) : 0);
        int iR = off + (el < T - 1 ? (el + 1) * NP : el * NP + NP - 1);
        if constexpr (EDGE) {
          iL = E[m].first ? CB + st : iL;
          iR = E[m].last ? off + el * NP + NP - 1 : iR;
        }
        const double du0 = us[0] - lds[iL];
        const double du1 = us[NP - 1] - lds[iR];
        double pe = 0.0, po = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) pe = fma(args.op.le[k], we[m][k], pe);
#pragma unroll
        for (int k = 0; k < NO; ++k) po = fma(args.op.lo[k], wo[m][k], po);
        double c = fma(du0 - du1, pe, (du0 + du1) * po);
        if constexpr (!UNI) c *= sc[m];
        eacc[m] += c;
      }
    }

    double le_[EPL][NE], lo_[EPL][NO];  // the stage residual's adjoint
#pragma unroll
    for (int m = 0; m < EPL; ++m) {
#pragma unroll
      for (int k = 0; k < NE; ++k) le_[m][k] = 0.0;
#pragma unroll
      for (int k = 0; k < NO; ++k) lo_[m][k] = 0.0;
    }
#pragma unroll
    for (int ss = 0; ss < NS; ++ss) {
      const int s = NS - 1 - ss;
      // Face buffers alternate over the launch's global reverse-stage index: with the jump
      // record no barrier separates a step's last stage from the next step's first, so
      // alternating on ss alone (NS = 5: 4 -> 0) would let a fast wave overwrite faces a
      // slower neighbour wave has not read yet.
      const int f0 = G::kFB + (((MS - 1 - st) * NS + ss) & 1) * 2 * (T + 2);
      // g0 = lds[f0 ...], g1 = lds[f1 ...]
      const int f1 = f0 + (T + 2);
      double qe[EPL][NE], qo[EPL][NO];
      double g0[EPL], g1[EPL];
#pragma unroll
      for (int m = 0; m < EPL; ++m) {
        const int el = m * LB + lane;
        double gd = 0.0, gs = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          le_[m][k] = fma(RK<NS>::B(s), we[m][k], le_[m][k]);
          qe[m][k] = UNI ? le_[m][k] : sc[m] * le_[m][k];
          gd = fma(args.op.le[k], qe[m][k], gd);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          lo_[m][k] = fma(RK<NS>::B(s), wo[m][k], lo_[m][k]);
          qo[m][k] = UNI ? lo_[m][k] : sc[m] * lo_[m][k];
          gs = fma(args.op.lo[k], qo[m][k], gs);
        }
        // adjoints of the left / right neighbour face values uL, uR (folded operator:
        // dlt = uR - uL feeds the even part, sig = -(uL + uR) the odd part):
        // d/duL = -(gd + gs) = -g0, d/duR = gd - gs = -g1
        g0[m] = gd + gs;
        g1[m] = gs - gd;
        lds[f0 + el + 1] = g0[m];
        lds[f1 + el + 1] = g1[m];
        __builtin_amdgcn_sched_barrier(0);  // face writes first
        // The transposed volume term and the carry A_s*lr need no neighbour data: issued
        // before the barrier (a scheduling boundary), only the face terms follow it.
#pragma unroll
        for (int j = 0; j < NE; ++j) {
          double t = we[m][j];
#pragma unroll
          for (int k = 0; k < NO; ++k) t = fma(args.op.Qoe[k * NE + j], qo[m][k], t);
          we[m][j] = t;
        }
#pragma unroll
        for (int j = 0; j < NO; ++j) {
          double t = wo[m][j];
#pragma unroll
          for (int k = 0; k < NE; ++k) t = fma(args.op.Qeo[k * NO + j], qe[m][k], t);
          wo[m][j] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) le_[m][k] = RK<NS>::A(s) * le_[m][k];
#pragma unroll
        for (int k = 0; k < NO; ++k) lo_[m][k] = RK<NS>::A(s) * lo_[m][k];
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(we[m][k]);
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(wo[m][k]);
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < EPL; ++m) {
        const int el = m * LB + lane;
        // This element's u_0 = e_0 + o_0 is the right neighbour value uR of element k-1
        // (adjoint -g1 there), its u_N = e_0 - o_0 the left value uL of element k+1
        // (adjoint -g0 there).  Edge tiles: a trajectory's first element has uL = inflow
        // (nothing arrives from the left); its last one has uR = its own u_N (du1 = 0), so
        // its own -g1 lands on its u_N.
        const double gl = lds[EDGE && E[m].first ? CB + MS : f1 + el];
        const double gr = lds[EDGE && E[m].last ? f1 + el + 1 : f0 + el + 2];
        we[m][0] -= gl + gr;
        wo[m][0] += gr - gl;
      }
    }
  }

#pragma unroll
  for (int m = 0; m < EPL; ++m)
    if (args.has_eta && E[m].valid) eta_update(eta, E[m].e, eacc[m], args.has_eta);
  stage_out<NP, W, H>(lds, we, wo, true);  // the image's last reads are 5 barriers behind
  __syncthreads();
  const int64_t o0 = tile * TE * NP;
  if constexpr (EDGE) {
    const int64_t rem = nd - o0;
    store_run<LB>(wout, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
  } else {
    store_full<TE * NP, LB>(wout, o0, lds);
  }
}

template <int NP, int NS, bool UNI, int W, int MS, bool REC>
__global__ __launch_bounds__(kBlock * W) void k_adj(const double* __restrict__ win,
                                                    double* __restrict__ wout,
                                                    const double* __restrict__ snap,
                                                    double* __restrict__ eta,
                                                    const double* __restrict__ scale,
                                                    AdjArgs<NP, MS> args) {
  using G = TileGeo<NP, W>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  const int64_t e0 = tile * (G::T - 2 * MS * NS) - MS * NS;
  if (edge_tile(e0, G::T, args.ktot, args.K))
    adj_tile<NP, NS, UNI, W, MS, REC, true>(lds, tile, win, wout, snap, eta, scale, args);
  else
    adj_tile<NP, NS, UNI, W, MS, REC, false>(lds, tile, win, wout, snap, eta, scale, args);
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
  double tvbM;       // > 0: SlopeLimitLin's minmod is minmodB(., M, h) (dg_plan_set_tvb)
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

// The TVB-modified minmod, utils/minmodB.m:6-11: the first argument unless |a| > M h^2.
__device__ __forceinline__ double minmod3b(double a, double b, double c, double M, double h) {
#pragma clang fp contract(off)
  return (fabs(a) > M * (h * h)) ? minmod3(a, b, c) : a;
}

// PI1: SlopeLimit1 (utils/SlopeLimit1.m:6-22) — the same projection and SlopeLimitLin
// on every cell, without the troubled-cell test.
template <int NP, bool PI1>
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
  const bool flag = PI1 || (fabs(ve1 - ue1) > eps0) || (fabs(ve2 - ue2) > eps0);  // :23

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
    const double m = args.tvbM > 0.0 ? minmod3b(ux0, (vkp1 - vk) / h, (vk - vkm1) / h, args.tvbM, h)
                                     : minmod3(ux0, (vkp1 - vk) / h, (vk - vkm1) / h);
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
  // Every thread starts from the weakest candidate (-inf, INT64_MAX): every element beats it
  // under `better` (a -inf element by its lower index), so no "no candidate yet" flag is
  // needed.  The flag form (bi = -1; `if (bi < 0 || better(...))`) is what ROCm 7.2's gfx950
  // backend miscompiled in k_slice_partial: in the structurised divergent branch the copy for
  // the not-taken edge of the phi of bv was placed where the lanes of the taken edge run it
  // too, so a thread kept its first value as bv while bi advanced (DESIGN.md §5 "Support
  // kernels"; the ISA and a reproducer: profiles/probes/argmax_phi_copy.hip).  This kernel's
  // flag form happened to compile correctly; it no longer depends on that.
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    const double v = use_abs ? fabs(x[i]) : x[i];
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

// dg_argmax_ex: as k_argmax_final, and also hands back the winning value (|x| when use_abs)
// and counts a non-finite winner.  argmax ranks NaN first and +inf above every finite value,
// so the winner is non-finite exactly when some entry is NaN or +-inf (under use_abs; without
// it a -inf elsewhere is not seen).  One thread writes, in stream order: no atomics needed.
__global__ __launch_bounds__(kBlock) void k_argmax_final_ex(const double* __restrict__ pv,
                                                            const int64_t* __restrict__ pi,
                                                            int nparts, int64_t* __restrict__ out,
                                                            double* __restrict__ val,
                                                            int64_t* __restrict__ nonfinite) {
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  for (int p = threadIdx.x; p < nparts; p += kBlock) {
    if (better(pv[p], pi[p], bv, bi)) {
      bv = pv[p];
      bi = pi[p];
    }
  }
  block_argmax(bv, bi);
  if (threadIdx.x == 0) {
    out[0] = bi;
    if (val != nullptr) val[0] = bv;
    if (nonfinite != nullptr && !isfinite(bv)) nonfinite[0] += 1;
  }
}

__global__ __launch_bounds__(kBlock) void k_sum_rows(const double* __restrict__ x, int64_t rows,
                                                     int64_t n, double* __restrict__ out) {
  const int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= n) return;
  double acc = x[k];
  for (int64_t r = 1; r < rows; ++r) acc = acc + x[r * n + k];
  out[k] = acc;
}

// dg_slice_candidate: the rank's mean slice, never stored: summed and divided per element,
// in k_sum_rows' order, straight into the argmax partials.
__global__ __launch_bounds__(kBlock) void k_slice_partial(const double* __restrict__ x,
                                                          int64_t rows, int64_t n, int64_t ld,
                                                          double divisor,
                                                          double* __restrict__ pv,
                                                          int64_t* __restrict__ pi) {
  // Start from the weakest candidate (every |m| beats it), as k_argmax_partial: with a "no
  // candidate yet" flag this loop compiled to code that kept the first element's value as
  // the thread's best while still advancing its index (ROCm 7.2, gfx950: a phi copy on a
  // divergent edge, profiles/probes/argmax_phi_copy.hip), seen on the GPU as argmaxes over
  // the first grid-stride pass only.
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    double acc = x[i];
    for (int64_t r = 1; r < rows; ++r) acc = acc + x[r * ld + i];
    const double v = fabs(acc / divisor);  // (x / 1 == x exactly: no special case)
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

__global__ __launch_bounds__(kBlock) void k_slice_final(const double* __restrict__ pv,
                                                        const int64_t* __restrict__ pi,
                                                        int nparts, int64_t offset,
                                                        int64_t* __restrict__ cand) {
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  for (int p = threadIdx.x; p < nparts; p += kBlock) {
    if (better(pv[p], pi[p], bv, bi)) {
      bv = pv[p];
      bi = pi[p];
    }
  }
  block_argmax(bv, bi);
  if (threadIdx.x == 0) {
    cand[0] = __double_as_longlong(bv);
    cand[1] = bi + offset;
  }
}

// dg_candidates_argmax: one block over the w (value bits, index) pairs; a candidate's
// position is its tie-break key (ranks own ascending index ranges).
__global__ __launch_bounds__(kBlock) void k_candidates(const int64_t* __restrict__ cands,
                                                       int64_t w, int64_t* __restrict__ idx,
                                                       double* __restrict__ val,
                                                       int64_t* __restrict__ nonfinite) {
  double bv = -INFINITY;
  int64_t bp = INT64_MAX;
  for (int64_t p = threadIdx.x; p < w; p += kBlock) {
    const double v = __longlong_as_double(cands[2 * p]);
    if (better(v, p, bv, bp)) {
      bv = v;
      bp = p;
    }
  }
  block_argmax(bv, bp);
  if (threadIdx.x == 0) {
    idx[0] = cands[2 * bp + 1];
    if (val != nullptr) val[0] = bv;
    if (nonfinite != nullptr && !isfinite(bv)) nonfinite[0] += 1;
  }
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

// Device-side refinement (dg_plan_refine): split element j = idx[0] of the old K-element
// mesh at its midpoint, inserting vertex 0.5*(VX[j] + VX[j+1]) after vertex j -- the
// split of python/Main_finite_difference.py:336-341 (ref_idx = argmax + 1) and
// matlab/MAIN.m:137-141 -- and the new elements' metric 2/h exactly as dg_plan_create
// computes it.  One thread per new vertex 0..K+1 (and new element 0..K).
__global__ __launch_bounds__(kBlock) void k_refine(const double* __restrict__ vx_old,
                                                   const double* __restrict__ sc_old,
                                                   double* __restrict__ vx,
                                                   double* __restrict__ sc,
                                                   const int64_t* __restrict__ idx,
                                                   double* __restrict__ h_split, int64_t K) {
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  int64_t j = idx[0];
  j = j < 0 ? 0 : (j >= K ? K - 1 : j);
  const double mid = 0.5 * (vx_old[j] + vx_old[j + 1]);
  if (i <= K + 1) vx[i] = i <= j ? vx_old[i] : (i == j + 1 ? mid : vx_old[i - 1]);
  if (i <= K) {
    double s;
    if (i < j) s = sc_old[i];
    else if (i > j + 1) s = sc_old[i - 1];
    else if (i == j) s = 2.0 / (mid - vx_old[j]);
    else s = 2.0 / (vx_old[j + 1] - mid);
    sc[i] = s;
  }
  if (i == 0 && h_split != nullptr) h_split[0] = vx_old[j + 1] - vx_old[j];
}

__global__ __launch_bounds__(kBlock) void k_axpy_copy(const double* __restrict__ w,
                                                      const double* __restrict__ u, double c,
                                                      double* __restrict__ out, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = fma(c, u[i], w[i]);
}

}  // namespace

namespace {
using namespace dgk;

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
  la.tvbM = p->tvb_M;
  la.ktot = p->ktot;
  la.K = int32_t(p->K);
  return la;
}

// Jump-record sweeps (REC): `snap` is the record, `rec` = {n0, jend} (see jump_row).
struct RecPos {
  int64_t n0 = 0;
  bool jend = false;
};

template <int NP, int NS, int W, int MS, bool REC = false>
int launch_step_e(const dg_plan* p, const double* in, double* snap, double* last,
                  const double* times, double dt, hipStream_t st, RecPos rec = {}) {
  StepArgs<NP, NS, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;  // non-uniform meshes multiply by scale[k] in the kernel
  for (int m = 0; m < MS; ++m)
    for (int s = 0; s < NS; ++s) a.uin[m * NS + s] = inflow_value(p, times[m] + RK<NS>::C(s) * dt);
  a.uin[MS * NS] = inflow_value(p, times[MS]);  // t_{n0+MS} (the record's final exchange)
  a.ktot = p->ktot;
  a.stride = p->ktot * NP;
  a.n0 = rec.n0;
  a.K = int32_t(p->K);
  a.xcd = p->xcd_order;
  a.jend = rec.jend ? 1 : 0;
  constexpr int TE = kBlock * W - 2 * (MS * NS + (REC ? 1 : 0));
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_step<NP, NS, true, W, MS, REC>), dim3(grid), dim3(kBlock * W), 0, st,
                       in, snap, last, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_step<NP, NS, false, W, MS, REC>), dim3(grid), dim3(kBlock * W), 0, st,
                       in, snap, last, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP, int NS, int W, int MS, bool REC = false>
int launch_adj_e(const dg_plan* p, const double* win, double* wout, const double* snap,
                 double* eta, int eta_mode, const double* t_next, const double* src, double dt,
                 hipStream_t st, int64_t n0 = 0) {
  AdjArgs<NP, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;
  for (int m = 0; m < MS; ++m) {
    a.uin_res[m] = inflow_value(p, t_next[m]);
    a.src[m] = src[m];
  }
  a.ktot = p->ktot;
  a.stride = p->ktot * NP;
  a.n0 = n0;
  a.K = int32_t(p->K);
  a.has_eta = eta != nullptr ? (eta_mode | kEtaOn) : 0;
  a.xcd = p->xcd_order;
  constexpr int TE = kBlock * W - 2 * MS * NS;
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_adj<NP, NS, true, W, MS, REC>), dim3(grid), dim3(kBlock * W), 0, st,
                       win, wout, snap, eta, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_adj<NP, NS, false, W, MS, REC>), dim3(grid), dim3(kBlock * W), 0, st,
                       win, wout, snap, eta, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

// Instantiated shapes: tile width W in {1, 2} (256 or 512 elements per tile) x steps per
// launch in {1, 2, 4}, plus 8 steps per launch on 512-element tiles; 4 and 8 steps per
// launch only for Np <= 8 (at Np = 9 hipcc/ROCm 7.2 fails instruction selection for the
// 4-step shape; effective_msteps() never asks for them there).
template <int NP, int NS>
int launch_step_t(const dg_plan* p, int ms, const double* in, double* snap, double* last,
                  const double* times, double dt, hipStream_t st) {
  const bool w2 = p->tile_width == 2;
  if constexpr (NP <= 8) {
    if (ms == 8) return launch_step_e<NP, NS, 2, 8>(p, in, snap, last, times, dt, st);
    if (ms == 4 && w2) return launch_step_e<NP, NS, 2, 4>(p, in, snap, last, times, dt, st);
    if (ms == 4) return launch_step_e<NP, NS, 1, 4>(p, in, snap, last, times, dt, st);
  }
  if (ms == 2 && w2) return launch_step_e<NP, NS, 2, 2>(p, in, snap, last, times, dt, st);
  if (ms == 2) return launch_step_e<NP, NS, 1, 2>(p, in, snap, last, times, dt, st);
  if (w2) return launch_step_e<NP, NS, 2, 1>(p, in, snap, last, times, dt, st);
  return launch_step_e<NP, NS, 1, 1>(p, in, snap, last, times, dt, st);
}

template <int NP, int NS>
int launch_adj_t(const dg_plan* p, int ms, const double* win, double* wout, const double* snap,
                 double* eta, int em, const double* t_next, const double* src, double dt,
                 hipStream_t st) {
  const bool w2 = p->tile_width == 2;
  if constexpr (NP <= 8) {
    if (ms == 8)
      return launch_adj_e<NP, NS, 2, 8>(p, win, wout, snap, eta, em, t_next, src, dt, st);
    if (ms == 4 && w2)
      return launch_adj_e<NP, NS, 2, 4>(p, win, wout, snap, eta, em, t_next, src, dt, st);
    if (ms == 4)
      return launch_adj_e<NP, NS, 1, 4>(p, win, wout, snap, eta, em, t_next, src, dt, st);
  }
  if (ms == 2 && w2)
    return launch_adj_e<NP, NS, 2, 2>(p, win, wout, snap, eta, em, t_next, src, dt, st);
  if (ms == 2)
    return launch_adj_e<NP, NS, 1, 2>(p, win, wout, snap, eta, em, t_next, src, dt, st);
  if (w2) return launch_adj_e<NP, NS, 2, 1>(p, win, wout, snap, eta, em, t_next, src, dt, st);
  return launch_adj_e<NP, NS, 1, 1>(p, win, wout, snap, eta, em, t_next, src, dt, st);
}

int launch_step(const dg_plan* p, int ms, const double* in, double* snap, double* last,
                const double* times, double dt, hipStream_t st) {
  int rc = DG_OK;
  if (p->lane_elems != 0 && p->nstages == 5 && p->NP <= 8)
    return wave_launch_step(p, ms, in, snap, last, times, dt, st);
  if (p->nstages == 5) {
    DG_DISPATCH_NP(p->NP, rc = (launch_step_t<NP, 5>(p, ms, in, snap, last, times, dt, st)));
  } else {
    DG_DISPATCH_NP(p->NP, rc = (launch_step_t<NP, 1>(p, ms, in, snap, last, times, dt, st)));
  }
  return rc;
}

int launch_adj(const dg_plan* p, int ms, const double* win, double* wout, const double* snap,
               double* eta, int em, const double* t_next, const double* src, double dt,
               hipStream_t st) {
  int rc = DG_OK;
  if (p->nstages == 5) {
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_t<NP, 5>(p, ms, win, wout, snap, eta, em, t_next, src,
                                                    dt, st)));
  } else {
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_t<NP, 1>(p, ms, win, wout, snap, eta, em, t_next, src,
                                                    dt, st)));
  }
  return rc;
}

// Record sweeps run on pair tiles (dg_rec.hip), Np <= 9, unless DG_TUNE_REC_LANE_ELEMENTS = 1
// selects the one-element-per-lane record kernels below: W = 1 with 1..4 steps, W = 2 with
// 1..8; Np = 9: at most 2 steps there (1024-element one-element-per-lane tiles -- 16-wave
// workgroups, 74 KB of LDS -- measured 20 % slower).
inline bool rec_pairs(const dg_plan* p) { return p->rec_lane_elems == 2; }

// Record steps per launch: pair tiles take 1, 2, 4, 5, 8, 10, 16 or 20 (a sweep is chunked by
// halving: 20 -> 10 -> 5 -> 2 -> 1); the one-element-per-lane kernels 1, 2, 4 or 8.
inline bool rec_msteps_ok(int k) {
  return k == 1 || k == 2 || k == 4 || k == 5 || k == 8 || k == 10 || k == 16 || k == 20;
}

// The record steps per launch the plan's shape allows for a requested value m on tiles of
// width w.
inline int rec_msteps_cap(const dg_plan* p, int m, int w) {
  if (!rec_pairs(p)) {
    int q = 1;
    while (q * 2 <= m && q < 8) q *= 2;
    m = q;
  }
  if (m == 8 && w == 1 && !rec_pairs(p)) m = 4;
  if (rec_pairs(p) && w == 1 && m > 10) m = (m == 16) ? 8 : 10;
  if (!rec_pairs(p) && p->NP > 8 && m > 2) m = 2;
  return m;
}

// Adjoint (and, unless overridden, forward) record steps per launch.
inline int rec_msteps(const dg_plan* p) { return rec_msteps_cap(p, p->rec_msteps, p->rec_tile_width); }

// Forward record steps per launch.  By size (the default): one 20-step launch on 1024-element
// pair tiles while a 10-step launch would be only ~1.5-4 rounds of workgroups (up to 3*2^20
// elements: at K = 2^20 / 2^21 the forward is 5 / 2 % faster than 10 + 10), beyond that the
// adjoint's setting (at 2^22 equal, at config 4's 67 M elements 10 + 10 is 3 % faster: the
// wider halo outweighs the launch saved).  The adjoint prefers 10 + 10 at every size.
inline int rec_msteps_fwd(const dg_plan* p) {
  int m = p->rec_msteps_fwd;
  if (m < 0)
    m = (rec_pairs(p) && rec_fwd_width(p) == 2 && p->ktot <= (int64_t(3) << 20)) ? 20
                                                                             : p->rec_msteps;
  return rec_msteps_cap(p, m ? m : p->rec_msteps, rec_fwd_width(p));
}

// Jump-record launches: LSERK4 (NS = 5) on the workgroup tiles, the plan's tile width and
// steps per launch (the 8-step shape on 512-element tiles; Np = 9 at most 2 steps).
template <int NP>
int launch_step_rec_t(const dg_plan* p, int ms, const double* in, double* rec, double* last,
                      const double* times, double dt, hipStream_t st, RecPos pos) {
  if (rec_pairs(p))
    return pair_launch_step_rec(p, ms, in, rec, last, times, dt, st, pos.n0, pos.jend);
  const bool w2 = rec_fwd_width(p) == 2;
  if constexpr (NP <= 8) {
    if (ms == 8) return launch_step_e<NP, 5, 2, 8, true>(p, in, rec, last, times, dt, st, pos);
    if (ms == 4 && w2) return launch_step_e<NP, 5, 2, 4, true>(p, in, rec, last, times, dt, st, pos);
    if (ms == 4) return launch_step_e<NP, 5, 1, 4, true>(p, in, rec, last, times, dt, st, pos);
  }
  if (ms == 2 && w2) return launch_step_e<NP, 5, 2, 2, true>(p, in, rec, last, times, dt, st, pos);
  if (ms == 2) return launch_step_e<NP, 5, 1, 2, true>(p, in, rec, last, times, dt, st, pos);
  if (w2) return launch_step_e<NP, 5, 2, 1, true>(p, in, rec, last, times, dt, st, pos);
  return launch_step_e<NP, 5, 1, 1, true>(p, in, rec, last, times, dt, st, pos);
}

template <int NP>
int launch_adj_rec_t(const dg_plan* p, int ms, const double* win, double* wout, const double* rec,
                     double* eta, int em, const double* t_next, const double* src, double dt,
                     hipStream_t st, int64_t n0) {
  if (rec_pairs(p))
    return pair_launch_adj_rec(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
  const bool w2 = p->rec_tile_width == 2;
  if constexpr (NP <= 8) {
    if (ms == 8)
      return launch_adj_e<NP, 5, 2, 8, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
    if (ms == 4 && w2)
      return launch_adj_e<NP, 5, 2, 4, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
    if (ms == 4)
      return launch_adj_e<NP, 5, 1, 4, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
  }
  if (ms == 2 && w2)
    return launch_adj_e<NP, 5, 2, 2, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
  if (ms == 2)
    return launch_adj_e<NP, 5, 1, 2, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
  if (w2) return launch_adj_e<NP, 5, 2, 1, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
  return launch_adj_e<NP, 5, 1, 1, true>(p, win, wout, rec, eta, em, t_next, src, dt, st, n0);
}

// Steps per launch the plan's shape allows: 8 only with 512-element tiles (the cone is
// 8*NS elements per side) and Np <= 8; at Np = 9 at most 2 (hipcc/ROCm 7.2 fails
// instruction selection for the 4-step shape there).
inline int effective_msteps(const dg_plan* p) {
  int m = p->msteps;
  if (m == 8 && !(p->tile_width == 2 || p->lane_elems == 8)) m = 4;
  if (m == 8 && p->lane_elems == 2) m = 4;  // 128-element wave tiles: cone too wide
  if (p->NP > 8 && m > 2) m = 2;
  return m;
}

// Steps per launch of the next chunk of a jump-record sweep (halving the plan's setting).
inline int chunk_rec(const dg_plan* p, int left, bool fwd = false) {
  int m = fwd ? rec_msteps_fwd(p) : rec_msteps(p);
  while (m > left) m >>= 1;
  return m < 1 ? 1 : m;
}

// Steps per launch for the next chunk of `left` steps (greedy over {4, 2, 1}, capped by
// the plan's setting).
inline int chunk(const dg_plan* p, int left) {
  int m = effective_msteps(p);
  while (m > left) m >>= 1;
  return m < 1 ? 1 : m;
}

// The dataflow sweep's blocks for `nsteps` steps (dg_sweep.hip): true with the forward /
// adjoint steps per block when the plan runs it -- pair tiles of one width in both
// directions (1024 or 512 elements), the record shape's 5-, 10- or 20-step (1024 only)
// forward and 5- or 10-step adjoint launches as its blocks, nsteps a multiple of both and at
// most sweep_max_steps() -- else false (the launch-per-block pair runs, same results).
// With the plan's sweep_waves set (DG_TUNE_SWEEP_WAVES) the dataflow launch runs both
// directions on tiles of 128 * sweep_waves elements, whatever the launch chains' widths: 12
// and 16 waves take the 10- or 20-step forward and 10-step adjoint blocks (16 at Np <= 5).
// Unset (0), the shape follows the record sweeps' tile width, with the measured exceptions
// below (12-wave tiles at Np <= 5, 8-wave tiles at Np = 9 on uniform meshes).
bool sweep_shape(const dg_plan* p, int nsteps, int* waves, int* msf, int* msa) {
  const int f = rec_msteps_fwd(p), a = rec_msteps(p), w = p->rec_tile_width;
  const int sw = p->sweep_waves;
  int nw = sw;
  bool tiles;
  if (sw) {
    tiles = (sw == 4 || sw == 8) || ((sw == 12 || (sw == 16 && p->NP <= 5)) && f >= 10 && a == 10);
  } else if (p->NP == 9 && p->uniform) {
    // the launch chains run 1024-element forward and 512-element adjoint tiles here; the one
    // launch takes 8-wave (1024-element) tiles in both directions: 7.06-7.23e11 DOF-updates/s
    // at K = 2^20 against 6.65e11 for the chains (profiles/r04/opreload/)
    nw = 8;
    tiles = true;
  } else {
    // as the record sweeps' tile width; on the 6-wave-per-SIMD uniform bodies (Np <= 5) 12-wave
    // tiles where their shape allows (1536 elements, 2 workgroups per CU; forward halo 1.15
    // instead of 1.25, a third fewer items): +3-4 % at N = 4, +1-3 % at N = 2
    // (profiles/r04/take/, perN/, shape_ab/)
    nw = 4 * w;
    tiles = rec_fwd_width(p) == w && (w == 1 || w == 2);
    // (Np = 2 keeps 8 waves: at 8 waves per SIMD, four 8-wave groups per CU, see SweepOcc)
    if (tiles && w == 2 && p->uniform && p->NP >= 3 && p->NP <= 5 && p->sweep_lane_elems == 2 &&
        f >= 10 && a == 10)
      nw = 12;
  }
  *msf = f;
  *msa = a;
  *waves = nw;
  tiles = tiles && (p->sweep_lane_elems == 2 || (p->NP <= 3 && (nw == 4 || nw == 8)));
  if (p->sweep_exchange == 1)  // overlapped waves: pairs on 8, 12 or 16 (Np <= 5) waves, 20- or
                               // 10-step forward and 10-step adjoint blocks
    tiles = tiles && p->sweep_lane_elems == 2 &&
            (nw == 8 || nw == 12 || (nw == 16 && p->NP <= 5)) && f >= 10 && a == 10;
  const int T = sweep_tile_elems(p, nw);  // elements per tile
  return p->rec_sweep && rec_pairs(p) && tiles &&
         (f == 5 || f == 10 || (f == 20 && T >= 900)) && (a == 5 || a == 10) && nsteps > 0 &&
         nsteps % f == 0 && nsteps % a == 0 && nsteps <= sweep_max_steps();
}

// The plan's dataflow scratch: a control region of sync words and flags (zeroed once, then
// kept consistent by the kernel's epochs) followed by a data region (block states, indicator
// partials).  Grows the control region to `sync_bytes` (zeroing what it newly covers, which
// an earlier call may have used as data) and the allocation to hold `data_bytes` after it.
// *data = the data region's start.
}  // namespace

namespace dgk {
int sweep_scratch(dg_plan* p, size_t sync_bytes, size_t data_bytes, hipStream_t st, char** data) {
  const size_t sync = sync_bytes > p->sweep_sync ? sync_bytes : p->sweep_sync;
  if (!p->d_sweep || p->sweep_bytes < sync + data_bytes) {
    if (p->d_sweep) {
      // Not freed: an earlier sweep may still run on it, and a HIP graph captured earlier
      // keeps its addresses in the kernel arguments.  Retired until dg_plan_destroy.
      p->sweep_retired.push_back(p->d_sweep);
      p->d_sweep = nullptr;
      p->sweep_bytes = p->sweep_sync = 0;
      p->sweep_items = -1;
      p->sweep_sig = 0;
    }
    if (hipMalloc(&p->d_sweep, sync + data_bytes) != hipSuccess) {
      p->d_sweep = nullptr;
      return fail(DG_ERR_NOMEM, "hipMalloc of the dataflow sweep's scratch failed");
    }
    p->sweep_bytes = sync + data_bytes;
  }
  if (sync > p->sweep_sync) {
    HIP_TRY(hipMemsetAsync(static_cast<char*>(p->d_sweep) + p->sweep_sync, 0,
                           sync - p->sweep_sync, st));
    p->sweep_sync = sync;
  }
  *data = static_cast<char*>(p->d_sweep) + sync;
  return DG_OK;
}

// The dataflow launches' watchdog: fails if an earlier launch of the plan gave up (until
// dg_sweep_status clears the flag), and maps the host-visible flag on first use.
int sweep_watchdog(dg_plan* p) {
  if (p->h_sweep_err && *static_cast<volatile uint32_t*>(p->h_sweep_err) != 0u)
    return fail(DG_ERR_HIP, "a dataflow sweep of this plan gave up waiting for a producer (its "
                            "outputs were poisoned with NaN); dg_sweep_status clears the flag");
  if (!p->h_sweep_err) {  // mapped page-locked memory
    void* h = nullptr;
    HIP_TRY(hipHostMalloc(&h, 64, hipHostMallocMapped));
    p->h_sweep_err = static_cast<uint32_t*>(h);
    *p->h_sweep_err = 0u;
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, h, 0));
    p->d_sweep_err = static_cast<uint32_t*>(d);
  }
  return DG_OK;
}
}  // namespace dgk

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* dg_last_error(void) { return dgk::g_err.c_str(); }

const char* dg_version(void) { return DG_VERSION; }

int dg_plan_create(int N, int64_t K, int64_t batch, const double* r, const double* V,
                   const double* invV, const double* Dr, const double* LIFT, const double* VX,
                   double a, int inflow_variant, int time_scheme, dg_plan** out) {
  dgk::g_err.clear();
  if (!out) return fail(DG_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (N < 1 || N > kMaxNP - 1) return fail(DG_ERR_ARG, "N must be in 1..8");
  if (K < 2 || batch < 1) return fail(DG_ERR_ARG, "need K >= 2 and batch >= 1");
  if (K * batch >= (int64_t(1) << 31) - 4096)
    return fail(DG_ERR_ARG, "batch*K must stay below 2^31 elements per plan");
  if (!r || !V || !invV || !Dr || !LIFT || !VX) return fail(DG_ERR_ARG, "null operator pointer");
  if (inflow_variant != DG_INFLOW_SIN_AT && inflow_variant != DG_INFLOW_SIN_A2T &&
      inflow_variant != DG_INFLOW_ZERO)
    return fail(DG_ERR_ARG, "bad inflow_variant");
  if (time_scheme != DG_TIME_LSERK4 && time_scheme != DG_TIME_EULER)
    return fail(DG_ERR_ARG, "bad time_scheme");
  dg_plan* p = new (std::nothrow) dg_plan();
  if (!p) return fail(DG_ERR_NOMEM, "host allocation failed");
  p->N = N;
  p->NP = N + 1;
  p->K = K;
  p->batch = batch;
  p->K_cap = K;
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

  bool sym = false;
  DG_DISPATCH_NP(p->NP, sym = make_eo<NP>(p, 1.0, nullptr));
  if (!sym) {
    delete p;
    return fail(DG_ERR_ARG, "Dr/LIFT are not centro-(anti)symmetric (nodes must be symmetric)");
  }

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

  // Per-N default shape (config 5 sweeps, profiles/r01/tune/N*.json and
  // profiles/r02/tune/): 512-element tiles pay off at low order, where a lane's work per
  // stage is small; at N = 1 and 2 the forward runs on one-wave tiles of 4 elements per lane
  // (DPP face exchange, no workgroup barriers): 23.8 -> 18.9 us (N = 1) and 27.7 -> 24.8 us
  // (N = 2) per 4-step launch.  (8 steps per launch at N = 2 bench the same within noise but
  // leave a 4-step launch in a 20-step sweep.)
  p->tile_width = (N <= 2) ? 2 : 1;
  if (N <= 2) p->lane_elems = 4;
  // Record sweeps: pair tiles (2 elements per lane, dg_rec.hip) at every Np.  At Np = 9 the
  // adjoint (147 VGPRs: 3 waves per SIMD) runs 512-element tiles -- three 4-wave workgroups
  // fill a CU where one 8-wave workgroup leaves a third of the wave slots empty -- and the
  // forward (122 VGPRs) keeps 1024-element tiles and its one 20-step launch: 330 + 395 us per
  // 20-step sweep at K = 2^20 against 336 + 477 with both on 1024 (profiles/r03/perN/ab_N8.json).
  if (p->NP == 9) {
    p->rec_tile_width = 1;
    p->rec_tile_width_fwd = 2;
  }
  // The p-enriched estimate (dg_lserk4_adj_p, Horner form since round 5) as ONE dataflow
  // launch (k_adjp_flow) on 512-element tiles with 4-step blocks: 410 us per 20-step estimate
  // at N = 4, K = 2^20 against 437 for the launch chain of direct-to-LDS 256-element tiles and
  // 443 for the chain with register prefetch (profiles/r05/p13; the chain drains each launch:
  // 4,855 tiles are 3.16 rounds of the 1,536 resident workgroups).
  p->p_tile_width = 2;
  p->p_flow = 1;
  p->p_sweep = 1;
  {
    if (const char* v = std::getenv("DG_TILE_WIDTH")) {
      const int k = std::atoi(v);
      if (k == 1 || k == 2) p->tile_width = k;
    }
    if (const char* v = std::getenv("DG_LANE_ELEMENTS")) {
      const int k = std::atoi(v);
      if (k == 0 || k == 2 || k == 4 || k == 8) p->lane_elems = k;
    }
    if (const char* v = std::getenv("DG_STEPS_PER_LAUNCH")) {
      const int k = std::atoi(v);
      if (k == 1 || k == 2 || k == 4 || k == 8) p->msteps = k;
    }
    if (const char* v = std::getenv("DG_REC_TILE_WIDTH")) {
      const int k = std::atoi(v);
      if (k == 1 || k == 2) {
        p->rec_tile_width = k;
        p->rec_tile_width_fwd = 0;  // both directions, as DG_TUNE_REC_TILE_WIDTH
      }
    }
    if (const char* v = std::getenv("DG_REC_FWD_TILE_WIDTH")) {
      const int k = std::atoi(v);
      if (k == 0 || k == 1 || k == 2) p->rec_tile_width_fwd = k;
    }
    if (const char* v = std::getenv("DG_REC_STEPS_PER_LAUNCH")) {
      const int k = std::atoi(v);
      // both directions, as DG_TUNE_REC_STEPS_PER_LAUNCH (the forward's own override below)
      if (rec_msteps_ok(k)) {
        p->rec_msteps = k;
        p->rec_msteps_fwd = 0;
      }
    }
    if (const char* v = std::getenv("DG_REC_FWD_STEPS_PER_LAUNCH")) {
      const int k = std::atoi(v);
      if (rec_msteps_ok(k)) p->rec_msteps_fwd = k;
    }
    if (const char* v = std::getenv("DG_REC_LANE_ELEMENTS")) {
      const int k = std::atoi(v);
      if (k == 1 || k == 2) p->rec_lane_elems = k;
    }
    if (const char* v = std::getenv("DG_P_TILE_WIDTH")) {
      const int k = std::atoi(v);
      if (k == 1 || k == 2) p->p_tile_width = k;
    }
    if (const char* v = std::getenv("DG_P_STEPS_PER_LAUNCH")) {
      const int k = std::atoi(v);
      if (k == 1 || k == 2 || k == 4 || k == 8) p->p_msteps = k;
    }
  if (const char* v = std::getenv("DG_P_FLOW")) {
    const int k = std::atoi(v);
    if (k == 0 || k == 1) p->p_flow = k;
  }
  if (const char* v = std::getenv("DG_P_SWEEP")) {
    const int k = std::atoi(v);
    if (k == 0 || k == 1) p->p_sweep = k;
  }
  }
  if (const char* v = std::getenv("DG_REC_SWEEP")) {
    const int k = std::atoi(v);
    if (k == 0 || k == 1) p->rec_sweep = k;
  }
  if (const char* v = std::getenv("DG_SWEEP_LANE_ELEMENTS")) {
    const int k = std::atoi(v);
    if (k == 2 || (k == 4 && p->NP <= 3)) p->sweep_lane_elems = k;
  }
  if (const char* v = std::getenv("DG_SNAP_PAIRS")) {
    const int k = std::atoi(v);
    if (k == 0 || k == 1) p->snap_pairs = k;
  }
  if (const char* v = std::getenv("DG_SWEEP_EXCHANGE")) {
    const int k = std::atoi(v);
    if (k == 0 || k == 1) p->sweep_exchange = k;
  }
  if (const char* v = std::getenv("DG_NL_EXCHANGE")) {
    const int e = std::atoi(v);
    if (e == 0 || e == 1) p->nl_exchange = e;
  }
  if (const char* v = std::getenv("DG_SWEEP_WAVES")) {
    const int k = std::atoi(v);
    if (k == 0 || k == 4 || k == 8 || k == 12 || (k == 16 && p->NP <= 5)) p->sweep_waves = k;
  }

  {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      p->cu_count = cus;
    if (p->cu_count < 1) p->cu_count = 1;
  }
  auto cleanup = [&](const std::string& m) {
    dg_plan_destroy(p);
    return fail(DG_ERR_NOMEM, m);
  };
  if (hipMalloc(&p->d_scale, sizeof(double) * K) != hipSuccess) return cleanup("hipMalloc scale");
  if (hipMalloc(&p->d_VX, sizeof(double) * (K + 1)) != hipSuccess) return cleanup("hipMalloc VX");
  if (hipMalloc(&p->d_scratch, sizeof(double) * p->ktot * NP) != hipSuccess)
    return cleanup("hipMalloc scratch");
  if (hipMalloc(&p->d_scratch2, sizeof(double) * p->ktot * NP) != hipSuccess)
    return cleanup("hipMalloc scratch2");
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
  if (p->d_scratch2) (void)hipFree(p->d_scratch2);
  if (p->d_pv) (void)hipFree(p->d_pv);
  if (p->d_pi) (void)hipFree(p->d_pi);
  if (p->d_sweep || !p->sweep_retired.empty()) (void)hipDeviceSynchronize();
  if (p->d_sweep) (void)hipFree(p->d_sweep);
  for (void* q : p->sweep_retired) (void)hipFree(q);
  if (p->h_sweep_err) (void)hipHostFree(p->h_sweep_err);
  if (p->d_nl_list) (void)hipFree(p->d_nl_list);
  delete p;
  return DG_OK;
}

int dg_plan_query(const dg_plan* p, int64_t out[8]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  out[0] = p->N;
  out[1] = p->NP;
  out[2] = p->K;
  out[3] = p->batch;
  out[4] = p->uniform ? 1 : 0;
  out[5] = p->nstages;
  out[6] = p->tile_width;
  out[7] = effective_msteps(p);
  return DG_OK;
}

int dg_plan_query_rec(const dg_plan* p, int64_t out[4]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  const int m = rec_msteps(p);
  out[0] = p->rec_tile_width;
  out[1] = m;
  out[2] = rec_pairs(p) ? 2 : 1;
  out[3] = rec_msteps_fwd(p);
  return DG_OK;
}

int dg_plan_query_rec_fwd(const dg_plan* p, int64_t out[2]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  out[0] = rec_fwd_width(p);
  out[1] = rec_msteps_fwd(p);
  return DG_OK;
}

int dg_plan_query_nl(const dg_plan* p, int64_t out[3]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  return nl_query(p, out);
}

int dg_plan_query_p(const dg_plan* p, int64_t out[2]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  out[0] = p->p_tile_width;
  out[1] = (p->p_msteps == 8 && p->p_tile_width != 2) ? 4 : p->p_msteps;
  return DG_OK;
}

int dg_plan_tune(dg_plan* p, int key, int64_t value) {
  if (!p) return fail(DG_ERR_ARG, "null plan");
  switch (key) {
    case DG_TUNE_P_TILE_WIDTH:
      if (value != 1 && value != 2) return fail(DG_ERR_ARG, "p-estimate tile width must be 1 or 2");
      p->p_tile_width = int(value);
      return DG_OK;
    case DG_TUNE_P_STEPS_PER_LAUNCH:
      if (value != 1 && value != 2 && value != 4 && value != 8)
        return fail(DG_ERR_ARG, "p-estimate steps per launch must be 1, 2, 4 or 8");
      p->p_msteps = int(value);
      return DG_OK;
    case DG_TUNE_REC_TILE_WIDTH:
      if (value != 1 && value != 2)
        return fail(DG_ERR_ARG, "record tile width must be 1 or 2");
      p->rec_tile_width = int(value);
      p->rec_tile_width_fwd = 0;  // both directions
      return DG_OK;
    case DG_TUNE_REC_FWD_TILE_WIDTH:
      if (value != 0 && value != 1 && value != 2)
        return fail(DG_ERR_ARG, "forward record tile width must be 0 (as the adjoint's), 1 or 2");
      p->rec_tile_width_fwd = int(value);
      return DG_OK;
    case DG_TUNE_REC_STEPS_PER_LAUNCH:
      if (!rec_msteps_ok(int(value)))
        return fail(DG_ERR_ARG, "record steps per launch must be 1, 2, 4, 5, 8, 10, 16 or 20");
      p->rec_msteps = int(value);
      p->rec_msteps_fwd = 0;  // both directions
      return DG_OK;
    case DG_TUNE_REC_FWD_STEPS_PER_LAUNCH:
      if (!rec_msteps_ok(int(value)))
        return fail(DG_ERR_ARG, "record steps per launch must be 1, 2, 4, 5, 8, 10, 16 or 20");
      p->rec_msteps_fwd = int(value);
      return DG_OK;
    case DG_TUNE_REC_LANE_ELEMENTS:
      if (value != 1 && value != 2)
        return fail(DG_ERR_ARG, "record lane elements must be 1 or 2");
      p->rec_lane_elems = int(value);
      return DG_OK;
    case DG_TUNE_SWEEP_WAVES:
      if (!(value == 0 || value == 4 || value == 8 || value == 12 || (value == 16 && p->NP <= 5)))
        return fail(DG_ERR_ARG, "sweep waves: 0 (as the record tile width), 4, 8, 12 or 16 "
                                "(16 at Np <= 5)");
      p->sweep_waves = int(value);
      return DG_OK;
    case DG_TUNE_SWEEP_LANE_ELEMENTS:
      if (!(value == 2 || (value == 4 && p->NP <= 3)))
        return fail(DG_ERR_ARG, "sweep lane elements: 2, or 4 at Np <= 3");
      p->sweep_lane_elems = int(value);
      return DG_OK;
    case DG_TUNE_SWEEP_TAKE:
      // removed in round 5 (item = workgroup id relied on in-order dispatch per XCD): only the
      // take counter (0) remains
      if (value != 0) return fail(DG_ERR_ARG, "sweep take: only 0 (the take counter) is supported");
      return DG_OK;
    case DG_TUNE_P_SWEEP:
      if (value != 0 && value != 1)
        return fail(DG_ERR_ARG, "p sweep: 0 (the chains) or 1 (one dataflow launch)");
      p->p_sweep = int(value);
      return DG_OK;
    case DG_TUNE_P_FLOW:
      if (value != 0 && value != 1)
        return fail(DG_ERR_ARG, "p-estimate flow: 0 (one launch per block) or 1 (one dataflow launch)");
      p->p_flow = int(value);
      return DG_OK;
    case DG_TUNE_SNAP_PAIRS:
      if (value != 0 && value != 1)
        return fail(DG_ERR_ARG, "snapshot pairs: 0 (stage-loop kernels) or 1 (Horner pair tiles)");
      p->snap_pairs = int(value);
      return DG_OK;
    case DG_TUNE_SWEEP_EXCHANGE:
      if (value != 0 && value != 1)
        return fail(DG_ERR_ARG, "sweep exchange: 0 (LDS + barrier per level) or 1 (overlapped waves)");
      p->sweep_exchange = int(value);
      return DG_OK;
    case DG_TUNE_NL_EXCHANGE:
      if (value != 0 && value != 1)
        return fail(DG_ERR_ARG, "config-3 exchange: 0 (workgroup tiles, LDS) or 1 (overlapped waves)");
      p->nl_exchange = int(value);
      return DG_OK;
    case DG_TUNE_SWEEP_SPIN_LIMIT:
      if (value < 0 || value > (1 << 30)) return fail(DG_ERR_ARG, "spin limit: 0 (default) .. 2^30");
      p->sweep_spin_limit = int(value);
      return DG_OK;
    case DG_TUNE_REC_SWEEP:
      if (value != 0 && value != 1) return fail(DG_ERR_ARG, "record sweep mode must be 0 or 1");
      p->rec_sweep = int(value);
      return DG_OK;
    case DG_TUNE_TILE_WIDTH:
      if (value != 1 && value != 2) return fail(DG_ERR_ARG, "tile width must be 1 or 2");
      p->tile_width = int(value);
      return DG_OK;
    case DG_TUNE_XCD_ORDER:
      p->xcd_order = value ? 1 : 0;
      return DG_OK;
    case DG_TUNE_LANE_ELEMENTS:
      if (value != 0 && value != 2 && value != 4 && value != 8)
        return fail(DG_ERR_ARG, "lane elements must be 0, 2, 4 or 8");
      p->lane_elems = int(value);
      return DG_OK;
    case DG_TUNE_STEPS_PER_LAUNCH:
      if (value != 1 && value != 2 && value != 4 && value != 8)
        return fail(DG_ERR_ARG, "steps per launch must be 1, 2, 4 or 8");
      p->msteps = int(value);
      return DG_OK;
    default:
      return fail(DG_ERR_ARG, "unknown tuning key");
  }
}

int dg_plan_set_tvb(dg_plan* p, double M) {
  if (!p) return fail(DG_ERR_ARG, "null plan");
  if (!(M >= 0.0) || !std::isfinite(M)) return fail(DG_ERR_ARG, "TVB constant M must be >= 0");
  p->tvb_M = M;
  return DG_OK;
}

int dg_plan_set_physics(dg_plan* p, int flux, int limiter) {
  if (!p) return fail(DG_ERR_ARG, "null plan");
  if (flux != DG_FLUX_LINEAR && flux != DG_FLUX_BURGERS) return fail(DG_ERR_ARG, "bad flux");
  if (limiter != DG_LIMIT_NONE && limiter != DG_LIMIT_EACH_STAGE &&
      limiter != DG_LIMIT_PI1_EACH_STAGE)
    return fail(DG_ERR_ARG, "bad limiter");
  if ((flux != DG_FLUX_LINEAR || limiter != DG_LIMIT_NONE) && p->scheme != DG_TIME_LSERK4)
    return fail(DG_ERR_ARG, "nonlinear flux and the per-stage limiter need DG_TIME_LSERK4");
  if (limiter != DG_LIMIT_NONE) {
    // The limiter kernels use the LGL symmetry (dg_burgers.hip LimEO): row 1 of invV even,
    // row 2 odd, r odd.
    const int NP = p->NP, N = NP - 1;
    double worst = 0.0;
    for (int k = 0; k < NP; ++k) {
      worst = std::max(worst, std::fabs(p->invV[k] - p->invV[N - k]));
      worst = std::max(worst, std::fabs(p->invV[NP + k] + p->invV[NP + N - k]));
      worst = std::max(worst, std::fabs(p->r[k] + p->r[N - k]));
    }
    if (!(worst <= 1e-13))
      return fail(DG_ERR_ARG, "the limiter needs symmetric LGL nodes (asymmetry " +
                                  std::to_string(worst) + ")");
  }
  p->flux = flux;
  p->limiter = limiter;
  return DG_OK;
}

int dg_plan_reserve(dg_plan* p, int64_t K_capacity) {
  if (!p) return fail(DG_ERR_ARG, "null plan");
  if (K_capacity <= p->K_cap) return DG_OK;
  if (K_capacity * p->batch >= (int64_t(1) << 31) - 4096)
    return fail(DG_ERR_ARG, "batch*K must stay below 2^31 elements per plan");
  HIP_TRY(hipDeviceSynchronize());  // no kernel may still use the old buffers
  double *sc = nullptr, *vx = nullptr, *s1 = nullptr, *s2 = nullptr;
  const size_t nf = sizeof(double) * size_t(K_capacity * p->batch * p->NP);
  if (hipMalloc(&sc, sizeof(double) * K_capacity) != hipSuccess ||
      hipMalloc(&vx, sizeof(double) * (K_capacity + 1)) != hipSuccess ||
      hipMalloc(&s1, nf) != hipSuccess || hipMalloc(&s2, nf) != hipSuccess) {
    (void)hipFree(sc);
    (void)hipFree(vx);
    (void)hipFree(s1);
    (void)hipFree(s2);
    return fail(DG_ERR_NOMEM, "hipMalloc in dg_plan_reserve");
  }
  HIP_TRY(hipMemcpy(sc, p->d_scale, sizeof(double) * p->K, hipMemcpyDeviceToDevice));
  HIP_TRY(hipMemcpy(vx, p->d_VX, sizeof(double) * (p->K + 1), hipMemcpyDeviceToDevice));
  // A safe point (the device is idle): the dataflow scratch regions a grown scratch retired go
  // now.  Like the plan's own scratch fields below, they may be held by a HIP graph captured
  // before this call: such graphs must be re-captured after a reserve (include/dg_advec.h).
  for (void* r : p->sweep_retired) (void)hipFree(r);
  p->sweep_retired.clear();
  (void)hipFree(p->d_scale);
  (void)hipFree(p->d_VX);
  (void)hipFree(p->d_scratch);
  (void)hipFree(p->d_scratch2);
  p->d_scale = sc;
  p->d_VX = vx;
  p->d_scratch = s1;
  p->d_scratch2 = s2;
  p->K_cap = K_capacity;
  return DG_OK;
}

int dg_plan_refine(dg_plan* p, const int64_t* idx, double* h_split, void* stream) {
  if (!p || !idx) return fail(DG_ERR_ARG, "null argument");
  if (p->K + 1 > p->K_cap)
    return fail(DG_ERR_ARG, "plan capacity exhausted: call dg_plan_reserve first");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // The old mesh goes to scratch first (the split shifts it in place).
  double* vx_old = p->d_scratch;
  double* sc_old = p->d_scratch + (p->K + 1);
  HIP_TRY(hipMemcpyAsync(vx_old, p->d_VX, sizeof(double) * (p->K + 1), hipMemcpyDeviceToDevice, st));
  HIP_TRY(hipMemcpyAsync(sc_old, p->d_scale, sizeof(double) * p->K, hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(k_refine, dim3(grid_for(p->K + 2, kBlock)), dim3(kBlock), 0, st, vx_old,
                     sc_old, p->d_VX, p->d_scale, idx, h_split, p->K);
  HIP_TRY(hipGetLastError());
  p->K += 1;
  p->ktot = p->K * p->batch;
  p->uniform = false;  // every element now uses its own 2/h_k
  return DG_OK;
}

int dg_plan_get_mesh(const dg_plan* p, double* VX) {
  if (!p || !VX) return fail(DG_ERR_ARG, "null argument");
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(VX, p->d_VX, sizeof(double) * (p->K + 1), hipMemcpyDeviceToHost));
  return DG_OK;
}

int dg_advec_rhs(const dg_plan* p, const double* u, double* rhs, double t, void* stream) {
  if (!p || !u || !rhs) return fail(DG_ERR_ARG, "null argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (p->flux == DG_FLUX_BURGERS) return nl_rhs(p, u, rhs, t, st);
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
  return dg_lserk4_fwd_ex(p, u, t0, dt, nsteps, snapshots, nullptr, stream);
}

int dg_lserk4_fwd_ex(dg_plan* p, double* u, double t0, double dt, int nsteps, double* snapshots,
                     uint16_t* decisions, void* stream) {
  if (!p || !u) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t field = p->ktot * p->NP;
  if (nsteps == 0) {  // the empty sweep: snapshot 0 still receives u^0
    if (snapshots && snapshots != u)
      HIP_TRY(hipMemcpyAsync(snapshots, u, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    return DG_OK;
  }
  if (p->nonlinear())
    return nl_fwd(p, u, t0, dt, nsteps, snapshots, p->limiter ? decisions : nullptr, st);
  // Time levels by repeated addition (time = time + dt, One_code.mlx:139).
  std::vector<double> tn(size_t(nsteps) + 1);
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  if (snapshots && p->snap_pairs && p->nstages == 5) {
    // Horner-form pair tiles (k_step_rps): every state from the registers, the launch's last
    // through LDS; u receives u^N by a copy when it is not snapshot 0
    if (snapshots != u)
      HIP_TRY(hipMemcpyAsync(snapshots, u, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    for (int n = 0; n < nsteps;) {
      int m = p->msteps;
      while (m > nsteps - n) m >>= 1;
      if (const int rc = pair_launch_step_snap(p, m, snapshots + int64_t(n) * field,
                                               snapshots + int64_t(n + 1) * field, &tn[n], dt, st))
        return rc;
      n += m;
    }
    if (snapshots != u)
      HIP_TRY(hipMemcpyAsync(u, snapshots + int64_t(nsteps) * field, sizeof(double) * field,
                             hipMemcpyDeviceToDevice, st));
    return DG_OK;
  }
  if (snapshots) {
    if (snapshots != u)
      HIP_TRY(hipMemcpyAsync(snapshots, u, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    for (int n = 0; n < nsteps;) {
      const int m = chunk(p, nsteps - n);
      double* last = (n + m == nsteps && snapshots != u) ? u : nullptr;
      const int rc = launch_step(p, m, snapshots + int64_t(n) * field,
                                 snapshots + int64_t(n + 1) * field, last, &tn[n], dt, st);
      if (rc) return rc;
      n += m;
    }
    return DG_OK;
  }
  // Ping-pong between u and the plan scratch; if the launch count is odd the first launch
  // reads a scratch copy of u so that the last one lands in u.
  int launches = 0;
  for (int n = 0; n < nsteps; n += chunk(p, nsteps - n)) ++launches;
  double* a = u;
  double* b = p->d_scratch;
  if (launches % 2 == 1) {
    HIP_TRY(hipMemcpyAsync(b, a, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    std::swap(a, b);
  }
  for (int n = 0; n < nsteps;) {
    const int m = chunk(p, nsteps - n);
    const int rc = launch_step(p, m, a, nullptr, b, &tn[n], dt, st);
    if (rc) return rc;
    std::swap(a, b);
    n += m;
  }
  return DG_OK;
}

int dg_lserk4_adj(dg_plan* p, double* w, const double* snapshots, double t0, double dt,
                  int nsteps, double src_coef, double* eta, void* stream) {
  return dg_lserk4_adj_ex(p, w, snapshots, t0, dt, nsteps, src_coef, eta, 0, nullptr, stream);
}

int dg_lserk4_adj_ex(dg_plan* p, double* w, const double* snapshots, double t0, double dt,
                     int nsteps, double src_coef, double* eta, int flags,
                     const uint16_t* decisions, void* stream) {
  if (!p || !w || !snapshots) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (flags & ~(DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS)) return fail(DG_ERR_ARG, "unknown flags");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (eta != nullptr && nsteps == 0 && (flags & DG_ADJ_ETA_ASSIGN))  // nothing to assign from
    HIP_TRY(hipMemsetAsync(eta, 0, sizeof(double) * p->ktot, st));
  if (p->nonlinear())
    return nl_adj(p, w, snapshots, t0, dt, nsteps, src_coef, eta, flags,
                  p->limiter ? decisions : nullptr, st);
  const int64_t field = p->ktot * p->NP;
  // Same time levels as the forward sweep (repeated addition).
  std::vector<double> tn(size_t(nsteps) + 1), src(size_t(nsteps) + 1, src_coef);
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  src[nsteps] = 0.0;  // left-endpoint rule: no source at the terminal node
  // Launch l reads buf[l] and writes buf[l+1]: buf[0] = w, the last output = w, and the
  // intermediate states alternate between the two plan scratch fields.  (w may alias the
  // terminal snapshot: only the first launch reads snapshot nsteps.)
  int launches = 0;
  for (int n = nsteps; n > 0; n -= chunk(p, n)) ++launches;
  int l = 0;
  const double* in = w;
  for (int n = nsteps; n > 0; ++l) {  // this launch covers steps n-m .. n-1
    const int m = chunk(p, n);
    const int n0 = n - m;
    // (a single launch cannot write its own input: it goes through scratch and back)
    double* out = (l == launches - 1 && launches > 1)
                      ? w : ((l % 2 == 0) ? p->d_scratch : p->d_scratch2);
    // DG_ADJ_ETA_ASSIGN: the sweep's first launch assigns eta; DG_ADJ_ETA_ABS: its last
    // launch stores |eta|.
    const int em = ((l == 0 && (flags & DG_ADJ_ETA_ASSIGN)) ? kEtaAssign : 0) |
                   ((n0 == 0 && (flags & DG_ADJ_ETA_ABS)) ? kEtaAbs : 0);
    const int rc = launch_adj(p, m, in, out, snapshots + int64_t(n0 + 1) * field, eta, em,
                              &tn[n0 + 1], &src[n0 + 1], dt, st);
    if (rc) return rc;
    in = out;
    n = n0;
  }
  // Node-0 source K^0 = src * u^0 (and the hand-back of a single-launch sweep).
  if ((src_coef != 0.0 && nsteps > 0) || in != w) {
    hipLaunchKernelGGL(k_axpy_copy, dim3(grid_for(field, kBlock)), dim3(kBlock), 0, st, in,
                       snapshots, nsteps > 0 ? src_coef : 0.0, w, field);
    HIP_TRY(hipGetLastError());
  }
  return DG_OK;
}

int dg_lserk4_fwd_rec(dg_plan* p, const double* u0, double* uN, double t0, double dt,
                      int nsteps, double* jumps, void* stream) {
  if (!p || !u0 || !uN || (!jumps && nsteps > 0)) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (p->nonlinear() || p->nstages != 5)
    return fail(DG_ERR_ARG, "the jump record is the linear LSERK4 sweep's (use snapshots)");
  if (reinterpret_cast<uintptr_t>(jumps) % 16 != 0)
    return fail(DG_ERR_ARG, "the jump record must be 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t field = p->ktot * p->NP;
  if (nsteps == 0) {
    if (uN != u0)
      HIP_TRY(hipMemcpyAsync(uN, u0, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    return DG_OK;
  }
  std::vector<double> tn(size_t(nsteps) + 1);  // time = time + dt (One_code.mlx:139)
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  // Launch l reads in_l and writes the next state: the last launch lands in uN, the others
  // alternate between the two plan scratch fields (a launch never writes its own input, so
  // u0 == uN is allowed and u0 is otherwise left untouched).
  int launches = 0;
  for (int n = 0; n < nsteps; n += chunk_rec(p, nsteps - n, true)) ++launches;
  const double* in = u0;
  int l = 0;
  for (int n = 0; n < nsteps; ++l) {
    const int m = chunk_rec(p, nsteps - n, true);
    const bool final = (n + m == nsteps);
    double* out = (final && in != uN) ? uN : ((l % 2 == 0) ? p->d_scratch : p->d_scratch2);
    RecPos pos;
    pos.n0 = n;
    pos.jend = final;
    int rc = DG_OK;
    DG_DISPATCH_NP(p->NP, rc = launch_step_rec_t<NP>(p, m, in, jumps, out, &tn[n], dt, st, pos));
    if (rc) return rc;
    in = out;
    n += m;
  }
  if (in != uN)  // (a one-launch in-place sweep went through scratch)
    HIP_TRY(hipMemcpyAsync(uN, in, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
  return DG_OK;
}

int dg_lserk4_adj_rec(dg_plan* p, double* w, const double* jumps, double t0, double dt,
                      int nsteps, double* eta, int flags, void* stream) {
  // the record is read by every reverse step (the kernels prefetch it whether or not eta is
  // wanted), so it is required whenever there is a step to run
  if (!p || !w || (!jumps && nsteps > 0)) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (flags & ~(DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS)) return fail(DG_ERR_ARG, "unknown flags");
  if (p->nonlinear() || p->nstages != 5)
    return fail(DG_ERR_ARG, "the jump record is the linear LSERK4 sweep's (use snapshots)");
  if (reinterpret_cast<uintptr_t>(jumps) % 16 != 0)
    return fail(DG_ERR_ARG, "the jump record must be 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (eta != nullptr && nsteps == 0 && (flags & DG_ADJ_ETA_ASSIGN))
    HIP_TRY(hipMemsetAsync(eta, 0, sizeof(double) * p->ktot, st));
  const int64_t field = p->ktot * p->NP;
  std::vector<double> tn(size_t(nsteps) + 1), src(size_t(nsteps) + 1, 0.0);
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  int launches = 0;
  for (int n = nsteps; n > 0; n -= chunk_rec(p, n)) ++launches;
  int l = 0;
  const double* in = w;
  for (int n = nsteps; n > 0; ++l) {  // this launch covers steps n-m .. n-1
    const int m = chunk_rec(p, n);
    const int n0 = n - m;
    double* out = (l == launches - 1 && launches > 1)
                      ? w : ((l % 2 == 0) ? p->d_scratch : p->d_scratch2);
    const int em = ((l == 0 && (flags & DG_ADJ_ETA_ASSIGN)) ? kEtaAssign : 0) |
                   ((n0 == 0 && (flags & DG_ADJ_ETA_ABS)) ? kEtaAbs : 0);
    int rc = DG_OK;
    DG_DISPATCH_NP(p->NP, rc = launch_adj_rec_t<NP>(p, m, in, out, jumps, eta, em, &tn[n0 + 1],
                                                    &src[n0 + 1], dt, st, n0));
    if (rc) return rc;
    in = out;
    n = n0;
  }
  if (in != w)
    HIP_TRY(hipMemcpyAsync(w, in, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
  return DG_OK;
}

}  // extern "C"

namespace {
// dg_lserk4_sweep_rec, and with `idx` non-null also the refine decision dg_argmax_ex(eta,
// |.|) -- fused into the dataflow launch, or a separate reduction after the launch chains.
int sweep_rec_impl(dg_plan* p, const double* u0, double* uN, double* w, double* jumps,
                   double t0, double dt, int nsteps, double* eta, int flags, int64_t* idx,
                   double* value, int64_t* nonfinite, void* stream) {
  if (!p || !u0 || !w || (!jumps && nsteps > 0)) return fail(DG_ERR_ARG, "null argument");
  if (idx && !eta) return fail(DG_ERR_ARG, "the refine decision needs eta");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (flags & ~(DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS | DG_SWEEP_TERMINAL_STATE))
    return fail(DG_ERR_ARG, "unknown flags");
  if (p->nonlinear() || p->nstages != 5)
    return fail(DG_ERR_ARG, "the jump record is the linear LSERK4 sweep's (use snapshots)");
  if (reinterpret_cast<uintptr_t>(jumps) % 16 != 0)
    return fail(DG_ERR_ARG, "the jump record must be 16-byte aligned");
  if (uN && (uN == w || uN == u0)) return fail(DG_ERR_ARG, "uN must not alias u0 or w");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool term = (flags & DG_SWEEP_TERMINAL_STATE) != 0;
  const int aflags = flags & (DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS);
  const int64_t field = p->ktot * p->NP;
  const size_t fbytes = sizeof(double) * size_t(field);
  int waves = 0, msf = 0, msa = 0;
  if (!sweep_shape(p, nsteps, &waves, &msf, &msa)) {
    // the launch-per-block pair: forward into uN (or w when it is the terminal weight, or a
    // scratch field), then the adjoint in place on w
    double* fin = uN;
    if (!fin && term) fin = w;
    if (!fin) {
      char* data = nullptr;
      const size_t fcap = sizeof(double) * size_t(p->K_cap * p->batch) * size_t(p->NP);
      if (const int rc = sweep_scratch(p, 256, fcap, st, &data)) return rc;
      fin = reinterpret_cast<double*>(data);
    }
    if (const int rc = dg_lserk4_fwd_rec(p, u0, fin, t0, dt, nsteps, jumps, stream)) return rc;
    if (term && fin != w) HIP_TRY(hipMemcpyAsync(w, fin, fbytes, hipMemcpyDeviceToDevice, st));
    if (const int rc = dg_lserk4_adj_rec(p, w, jumps, t0, dt, nsteps, eta, aflags, stream))
      return rc;
    return idx ? dg_argmax_ex(p, eta, p->ktot, 1, idx, value, nonfinite, stream) : DG_OK;
  }
  if (const int rc = sweep_watchdog(p)) return rc;
  const int nbF = nsteps / msf, nbA = nsteps / msa;
  const int64_t items = sweep_items(p, waves, msf, msa, nsteps);
  // The scratch is sized for the plan's reserved capacity (K_cap elements per trajectory), so
  // the refines of an adapt loop within it (dg_plan_refine: ktot += batch) reuse one region
  // instead of retiring a slightly smaller one per iteration.
  const int64_t kcap = p->K_cap * p->batch;
  const int64_t items_cap = sweep_items(p, waves, msf, msa, nsteps, kcap);
  const size_t sync_bytes = (sizeof(uint32_t) * size_t(sweep_sync_words() + items_cap) + 255) &
                            ~size_t(255);
  // fields: forward block outputs U[1..nbF-1] (+ U[nbF] unless the caller keeps u^N), adjoint
  // block outputs W[1..nbA-1] (+ a copy of the caller's terminal weight when one block would
  // read and write w); partial indicator rows for nbA - 1 blocks
  const int wcopy = (!term && nbA == 1) ? 1 : 0;
  const int nfields = (nbF - 1) + (uN ? 0 : 1) + (nbA - 1) + wcopy;
  const int nparts = eta ? nbA - 1 : 0;
  const int64_t am_parts = idx ? sweep_tiles_adj(p, waves, msa) : 0;
  const int64_t am_parts_cap = idx ? sweep_tiles_adj(p, waves, msa, kcap) : 0;
  const size_t fcap = sizeof(double) * size_t(kcap) * size_t(p->NP);
  const size_t data_bytes = fcap * size_t(nfields) + sizeof(double) * size_t(kcap) * size_t(nparts) +
                            16 * size_t(am_parts_cap);
  char* data = nullptr;
  if (const int rc = sweep_scratch(p, sync_bytes, data_bytes, st, &data)) return rc;
  const uint64_t sig = uint64_t(items) * 1000003u ^ (uint64_t(waves) << 56) ^
                      (uint64_t(p->sweep_exchange) << 61) ^
                      (uint64_t(msf) << 48) ^ (uint64_t(msa) << 40) ^ (uint64_t(nsteps) << 32) ^
                      uint64_t(sweep_tiles_adj(p, waves, msa));
  if (p->sweep_items != items || p->sweep_sig != sig) {
    // the take counter numbers launches by items per launch and the fused refine's arrival
    // counter by the last block's tiles: a new shape starts both afresh
    HIP_TRY(hipMemsetAsync(p->d_sweep, 0, sync_bytes, st));
    p->sweep_items = items;
    p->sweep_sig = sig;
  }
  double* fld = reinterpret_cast<double*>(data);
  int next = 0;
  SweepBufs b{};
  b.sync = static_cast<uint32_t*>(p->d_sweep);
  b.U[0] = const_cast<double*>(u0);
  for (int k = 1; k < nbF; ++k) b.U[k] = fld + field * next++;
  b.U[nbF] = uN ? uN : fld + field * next++;
  if (term) {
    b.W[0] = b.U[nbF];
  } else if (wcopy) {
    b.W[0] = fld + field * next++;
    HIP_TRY(hipMemcpyAsync(b.W[0], w, fbytes, hipMemcpyDeviceToDevice, st));
  } else {
    b.W[0] = w;  // read by the first block, rewritten by the last (nbA >= 2: no tile overlap)
  }
  for (int k = 1; k < nbA; ++k) b.W[k] = fld + field * next++;
  b.W[nbA] = w;
  b.rec = jumps;
  b.eta = eta;
  b.part = nparts ? fld + field * next : nullptr;
  double* am = fld + field * next + p->ktot * nparts;
  b.am_idx = idx;
  b.am_val = value;
  b.am_nf = nonfinite;
  b.am_pv = idx ? am : nullptr;
  b.am_pi = idx ? reinterpret_cast<int64_t*>(am + am_parts) : nullptr;
  b.err_host = p->d_sweep_err;
  b.spin_limit = p->sweep_spin_limit;
  const int mode = eta ? (kEtaOn | ((aflags & DG_ADJ_ETA_ASSIGN) ? kEtaAssign : 0) |
                          ((aflags & DG_ADJ_ETA_ABS) ? kEtaAbs : 0))
                       : 0;
  return sweep_launch_rec(p, waves, msf, msa, b, t0, dt, nsteps, mode, st);
}
}  // namespace

extern "C" {

int dg_lserk4_sweep_rec(dg_plan* p, const double* u0, double* uN, double* w, double* jumps,
                        double t0, double dt, int nsteps, double* eta, int flags, void* stream) {
  return sweep_rec_impl(p, u0, uN, w, jumps, t0, dt, nsteps, eta, flags, nullptr, nullptr,
                        nullptr, stream);
}

int dg_lserk4_sweep_refine(dg_plan* p, const double* u0, double* uN, double* w, double* jumps,
                           double t0, double dt, int nsteps, double* eta, int flags,
                           int64_t* idx, double* value, int64_t* nonfinite_count,
                           void* stream) {
  if (!idx) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 1) return fail(DG_ERR_ARG, "the refine decision needs nsteps >= 1");
  return sweep_rec_impl(p, u0, uN, w, jumps, t0, dt, nsteps, eta, flags, idx, value,
                        nonfinite_count, stream);
}

int dg_plan_query_sweep(const dg_plan* p, int nsteps, int64_t out[4]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  int waves = 0, msf = 0, msa = 0;
  const bool on = sweep_shape(p, nsteps, &waves, &msf, &msa);
  out[0] = on ? 1 : 0;
  out[1] = msf;
  out[2] = msa;
  out[3] = on ? sweep_items(p, waves, msf, msa, nsteps) : 0;
  return DG_OK;
}

int dg_plan_sweep_trace(dg_plan* p, uint64_t* trace) {
  if (!p) return fail(DG_ERR_ARG, "null plan");
  p->sweep_trace = trace;
  return DG_OK;
}

int dg_plan_query_sweep_ex(const dg_plan* p, int nsteps, int64_t out[6]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  int waves = 0, msf = 0, msa = 0;
  const bool on = sweep_shape(p, nsteps, &waves, &msf, &msa);
  out[0] = on ? 1 : 0;
  out[1] = msf;
  out[2] = msa;
  out[3] = on ? sweep_items(p, waves, msf, msa, nsteps) : 0;
  out[4] = waves;
  out[5] = sweep_tile_elems(p, waves);
  return DG_OK;
}

int dg_plan_query_sweep_kernel(const dg_plan* p, int nsteps, int64_t out[8]) {
  if (!p || !out) return fail(DG_ERR_ARG, "null argument");
  int waves = 0, msf = 0, msa = 0;
  const bool on = sweep_shape(p, nsteps, &waves, &msf, &msa);
  for (int i = 0; i < 8; ++i) out[i] = 0;
  if (!on) return DG_OK;
  out[0] = p->NP;
  out[1] = p->uniform ? 1 : 0;
  out[2] = waves;
  out[3] = msf;
  out[4] = msa;
  out[5] = p->sweep_lane_elems;
  out[6] = p->sweep_exchange;
  out[7] = sweep_waves_per_simd(p, waves);
  return DG_OK;
}

int dg_sweep_status(dg_plan* p, int* status, void* stream) {
  if (!p || !status) return fail(DG_ERR_ARG, "null argument");
  *status = 0;
  if (!p->d_sweep) return DG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint32_t* err = static_cast<uint32_t*>(p->d_sweep) + sweep_err_word();
  uint32_t h = 0;
  HIP_TRY(hipMemcpyAsync(&h, err, sizeof(h), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (p->h_sweep_err && *static_cast<volatile uint32_t*>(p->h_sweep_err) != 0u) h = 1u;
  if (h) {
    HIP_TRY(hipMemsetAsync(err, 0, sizeof(uint32_t), st));
    HIP_TRY(hipStreamSynchronize(st));
    if (p->h_sweep_err) *static_cast<volatile uint32_t*>(p->h_sweep_err) = 0u;
  }
  *status = int(h);
  return DG_OK;
}

int dg_slope_limit_n(dg_plan* p, const double* u, double* ulim, int32_t* ids, void* stream) {
  if (!p || !u || !ulim) return fail(DG_ERR_ARG, "null argument");
  if (u == ulim) return fail(DG_ERR_ARG, "in-place limiting is not supported (tiles overlap)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = grid_for(p->ktot, kBlock - 2);
  DG_DISPATCH_NP(p->NP, hipLaunchKernelGGL((k_limit<NP, false>), dim3(grid), dim3(kBlock), 0, st,
                                           u, ulim, ids, p->d_VX, make_lim<NP>(p)));
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_slope_limit_1(dg_plan* p, const double* u, double* ulim, void* stream) {
  if (!p || !u || !ulim) return fail(DG_ERR_ARG, "null argument");
  if (u == ulim) return fail(DG_ERR_ARG, "in-place limiting is not supported (tiles overlap)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = grid_for(p->ktot, kBlock - 2);
  DG_DISPATCH_NP(p->NP, hipLaunchKernelGGL((k_limit<NP, true>), dim3(grid), dim3(kBlock), 0, st,
                                           u, ulim, nullptr, p->d_VX, make_lim<NP>(p)));
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

int dg_argmax_ex(dg_plan* p, const double* x, int64_t n, int use_abs, int64_t* idx,
                 double* value, int64_t* nonfinite_count, void* stream) {
  if (!p || !x || !idx) return fail(DG_ERR_ARG, "null argument");
  if (n < 1 || n > p->ktot * p->NP) return fail(DG_ERR_ARG, "n out of range");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t parts = (n + 4 * kBlock - 1) / (4 * kBlock);
  if (parts > kArgmaxParts) parts = kArgmaxParts;
  hipLaunchKernelGGL(k_argmax_partial, dim3(unsigned(parts)), dim3(kBlock), 0, st, x, n, use_abs,
                     p->d_pv, p->d_pi);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_argmax_final_ex, dim3(1), dim3(kBlock), 0, st, p->d_pv, p->d_pi,
                     int(parts), idx, value, nonfinite_count);
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

int dg_slice_candidate(dg_plan* p, const double* x, int64_t rows, int64_t n, int64_t ld,
                       double divisor, int64_t offset, int64_t* cand, void* stream) {
  if (!p || !x || !cand) return fail(DG_ERR_ARG, "null argument");
  if (rows < 1 || n < 1 || ld < n) return fail(DG_ERR_ARG, "rows, n >= 1 and ld >= n required");
  if (n > p->ktot * p->NP) return fail(DG_ERR_ARG, "n out of range");
  if (!(divisor > 0.0)) return fail(DG_ERR_ARG, "divisor must be positive");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t parts = (n + 4 * kBlock - 1) / (4 * kBlock);
  if (parts > kArgmaxParts) parts = kArgmaxParts;
  hipLaunchKernelGGL(k_slice_partial, dim3(unsigned(parts)), dim3(kBlock), 0, st, x, rows, n, ld,
                     divisor, p->d_pv, p->d_pi);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_slice_final, dim3(1), dim3(kBlock), 0, st, p->d_pv, p->d_pi, int(parts),
                     offset, cand);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_candidates_argmax(const int64_t* cands, int64_t w, int64_t* idx, double* value,
                         int64_t* nonfinite_count, void* stream) {
  if (!cands || !idx) return fail(DG_ERR_ARG, "null argument");
  if (w < 1) return fail(DG_ERR_ARG, "w must be >= 1");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_candidates, dim3(1), dim3(kBlock), 0, st, cands, w, idx, value,
                     nonfinite_count);
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
