// dg_dwr.hip — the p-enriched dual-weighted-residual ERROR ESTIMATE of SURVEY 8(a) row 8
// (dg_prolong / dg_lserk4_adj_p).
//
// The reference's indicator is an error estimate: matlab/MAIN.m:32-34 marches the primal at
// order Ns and the adjoint at order Ns+1, and adj_march.m:103-117 pairs that adjoint with the
// primal's residual, err(k) = v_k' (-A uh_k - M~ + F); python/Main_finite_difference.py:79-94
// ("the Adjoint-Weighted Residual as an error estimate") takes the one-step residual
// res[n] = u_f[n] - Phi(u_f[n-1]) of the interpolated (refined) state.  For the DG advection
// sweep the same construction, p-refined, is:
//   P        interpolation of the order-N element polynomials to the order-(N+1) LGL nodes
//   R^n      = P u^{n+1} - S_{N+1}(P u^n, t_n)       one-step residual of the enriched scheme
//   w^{n+1}  the order-(N+1) discrete adjoint (terminal weight g = dJ_{N+1}/du)
//   eta_k    = - sum_n  w^{n+1} . R^n   on element k
// For the linear (affine) step e^{n+1} = A e^n - R^n with e = u_{N+1} - P u_h, so
// sum_k eta_k = g . e^N = J_{N+1}(u_{N+1}) - J_{N+1}(P u_h) exactly for a linear J (the DWR
// identity; CPU statement oracle/effectivity.py p_indicator).
//
// k_adj_p fuses the whole estimate into the order-(N+1) adjoint launch.  Per reverse step it
// stages the order-N snapshot u^n (one tile, 16-byte loads, prefetched a step ahead),
// prolongs each lane's element in even/odd coordinates (P is block diagonal there: LGL nodes
// are symmetric), recomputes S_{N+1}(P u^n) with 5 forward stages on the tile (the cone is 5
// elements per side, inside the adjoint's own halo), forms R^n against P u^{n+1} kept in
// registers from the previous step, accumulates -w.R, and runs the 5 reverse stages.  No
// prolonged field is ever stored: HBM sees the order-N snapshots once, w^{n0+MS} and w^{n0}
// at order N+1, and eta.
#include "dg_dwr_tiles.h"
#include "dg_flow.h"

namespace dgk {

// Even/odd transform of an Np-node element (rows e_0..e_{NE-1}, o_0..o_{NO-1}) and its
// inverse, as make_eo builds them (dg_common.h).
inline void eo_matrices(int NP, double* T, double* Ti) {
  const int NE = (NP + 1) / 2, NO = NP / 2, N = NP - 1;
  for (int i = 0; i < NP * NP; ++i) T[i] = Ti[i] = 0.0;
  for (int k = 0; k < NO; ++k) {
    T[k * NP + k] += 0.5; T[k * NP + N - k] += 0.5;
    T[(NE + k) * NP + k] += 0.5; T[(NE + k) * NP + N - k] -= 0.5;
    Ti[k * NP + k] += 1.0; Ti[k * NP + NE + k] += 1.0;
    Ti[(N - k) * NP + k] += 1.0; Ti[(N - k) * NP + NE + k] -= 1.0;
  }
  if (NE > NO) { T[NO * NP + NO] = 1.0; Ti[NO * NP + NO] = 1.0; }
}

// P (NPH x NPL, row-major: u_hi = P u_lo) -> its even/odd blocks.  False if P does not
// commute with the node reversal to 1e-12 (nodes not symmetric).
template <int NPL> bool make_prolong_eo(const double* P, PrEO<NPL>* out) {
  constexpr int NPH = NPL + 1;
  using R = PrEO<NPL>;
  double Th[NPH * NPH], Tih[NPH * NPH], Tl[NPL * NPL], Til[NPL * NPL];
  eo_matrices(NPH, Th, Tih);
  eo_matrices(NPL, Tl, Til);
  double TP[NPH * NPL], M[NPH * NPL];
  double pmax = 0.0;
  for (int i = 0; i < NPH; ++i)
    for (int j = 0; j < NPL; ++j) {
      double t = 0.0;
      for (int k = 0; k < NPH; ++k) t += Th[i * NPH + k] * P[k * NPL + j];
      TP[i * NPL + j] = t;
      pmax = std::fmax(pmax, std::fabs(P[i * NPL + j]));
    }
  for (int i = 0; i < NPH; ++i)
    for (int j = 0; j < NPL; ++j) {
      double t = 0.0;
      for (int k = 0; k < NPL; ++k) t += TP[i * NPL + k] * Til[k * NPL + j];
      M[i * NPL + j] = t;
    }
  const double tol = 1e-12 * (pmax > 0.0 ? pmax : 1.0);
  bool ok = pmax > 0.0;
  for (int i = 0; i < NPH; ++i)
    for (int j = 0; j < NPL; ++j) {
      const bool even_row = i < R::NEH, even_col = j < R::NEL;
      if (even_row != even_col) ok = ok && std::fabs(M[i * NPL + j]) <= tol;
    }
  if (out) {
    for (int k = 0; k < R::NEH; ++k)
      for (int j = 0; j < R::NEL; ++j) out->Pe[k * R::NEL + j] = M[k * NPL + j];
    for (int k = 0; k < R::NOH; ++k)
      for (int j = 0; j < R::NOL; ++j) out->Po[k * R::NOL + j] = M[(R::NEH + k) * NPL + R::NEL + j];
  }
  return ok;
}

}  // namespace dgk

namespace {
using namespace dgk;

// Arguments of one k_adj_p launch (MS reverse steps n0+MS-1 .. n0).
template <int NPL, int MS> struct AdjPArgs {
  EOArgs<NPL + 1> op;        // the order-(N+1) operator, folded; dt*2/h folded on uniform meshes
  PrEO<NPL> pr;
  double sc;                 // dt (non-uniform meshes multiply by scale[k])
  double uin[MS * 5 + 1];    // inflow at the forward stages of steps n0..n0+MS-1, then 0
  int64_t ktot;
  int64_t stride;            // doubles between consecutive order-N snapshots
  int32_t K;
  int32_t has_eta;           // kEta* bits
  int32_t xcd;
};

template <int NPL, int W> struct PGeo {
  static constexpr int NPH = NPL + 1;
  static constexpr int LB = kBlock * W, T = LB;
  static constexpr int kImgD = T * NPH + 2;  // the image holds the w tile or a snapshot tile
  static constexpr int kFB = (kImgD + 1) & ~1;
  static constexpr int kFaceD = 4 * (T + 2);  // two double-buffered face arrays, padded by 1
  static constexpr int kLds = kFB + kFaceD;
};

template <int NPL, bool UNI, int W, int MS>
__global__ __launch_bounds__(kBlock * W) void k_adj_p(const double* __restrict__ win,
                                                      double* __restrict__ wout,
                                                      const double* __restrict__ snap,
                                                      double* __restrict__ eta,
                                                      const double* __restrict__ scale,
                                                      AdjPArgs<NPL, MS> args);

// One tile of a k_adj_p launch.  snap = u^{n0}; the launch reads u^{n0} .. u^{n0+MS}.
template <int NPL, bool UNI, int W, int MS, bool EDGE>
__device__ __forceinline__ void adjp_tile(double* __restrict__ lds, int64_t tile,
                                          const double* __restrict__ win,
                                          double* __restrict__ wout,
                                          const double* __restrict__ snap,
                                          double* __restrict__ eta,
                                          const double* __restrict__ scale,
                                          const AdjPArgs<NPL, MS>& args) {
  constexpr int NPH = NPL + 1, NS = 5;
  using G = PGeo<NPL, W>;
  constexpr int T = G::T, LB = G::LB;
  // The reverse cone is NS elements per step; the forward recompute of a step needs 5 more
  // around the output elements, which the reverse halo of the steps still to come covers
  // (H >= 5 for MS >= 1: the recompute is exact on [5, T-5) and the outputs lie in [H, T-H)).
  constexpr int H = MS * NS;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NPH>::NE, NO = EOArgs<NPH>::NO, NH = NPH - 1;
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t ndh = args.ktot * NPH, ndl = args.ktot * NPL;
  constexpr int CB = G::kLds;  // lds[CB + st*NS + s]: stage inflow; lds[CB + MS*NS] = 0

  TileRegs<NPH, W> pw;
  TileRegs<NPL, W> pa, pb;
  tile_issue<NPH, W, EDGE>(win, e0, ndh, pw);
  tile_issue<NPL, W, EDGE>(snap + MS * args.stride, e0, ndl, pa);
  tile_issue<NPL, W, EDGE>(snap + (MS - 1) * args.stride, e0, ndl, pb);
  tile_commit<NPH, W>(pw, lds);
  if constexpr (EDGE) {
    using A = AdjPArgs<NPL, MS>;  // lane-indexed kernarg read, see step_tile (dg_advec.hip)
    const double* ka = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_adj_p<NPL, UNI, W, MS>), A>() + offsetof(A, uin));
    if (lane <= MS * NS) lds[CB + lane] = ka[lane];
  }
  __syncthreads();
  double we[NE], wo[NO];  // the order-(N+1) adjoint in dual even/odd coordinates
  {
    const double* w = lds + pw.off + lane * NPH;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[k] = w[k] + w[NH - k];
      wo[k] = w[k] - w[NH - k];
    }
    if constexpr (NE > NO) we[NO] = w[NO];
  }
  const Elem E = elem_info<H, T, EDGE>(e0, lane, args.ktot, args.K);
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;
  __syncthreads();  // the w image is read
  tile_commit<NPL, W>(pa, lds);
  __syncthreads();
  double ne[NE], no[NO];  // P u^{n+1} of this lane's element
  prolong_eo<NPL>(lds + pa.off + lane * NPL, args.pr, ne, no);
  __syncthreads();
  tile_commit<NPL, W>(pb, lds);
  int off = pb.off;
  __syncthreads();
  double eacc = 0.0;

#pragma unroll 1
  for (int st = MS - 1; st >= 0; --st) {
    // ---- P u^n, and the next snapshot's loads in flight behind this step ----
    double ev[NE], od[NO], pn_e[NE], pn_o[NO];
    prolong_eo<NPL>(lds + off + lane * NPL, args.pr, ev, od);
#pragma unroll
    for (int k = 0; k < NE; ++k) pn_e[k] = ev[k];
#pragma unroll
    for (int k = 0; k < NO; ++k) pn_o[k] = od[k];
    if (st > 0) tile_issue<NPL, W, EDGE>(snap + (st - 1) * args.stride, e0, ndl, pa);

    // ---- S_{N+1}(P u^n): 5 forward stages (k_step's arithmetic at order N+1) ----
    double re[NE], ro[NO];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // face buffers alternate over the launch's global stage index (10 per step: even)
      const int fL = G::kFB + (s & 1) * 2 * (T + 2), fR = fL + (T + 2);
      const double u0 = ev[0] + od[0], uN = ev[0] - od[0];
      lds[fL + lane + 1] = u0;
      lds[fR + lane + 1] = uN;
      __builtin_amdgcn_sched_barrier(0);
      double pe[NE], po[NO];
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        double t = (UNI && s > 0) ? RK<NS>::A(s) * re[k] : args.op.Qeo[k * NO] * od[0];
#pragma unroll
        for (int j = (UNI && s > 0) ? 0 : 1; j < NO; ++j) t = fma(args.op.Qeo[k * NO + j], od[j], t);
        pe[k] = t;
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        double t = (UNI && s > 0) ? RK<NS>::A(s) * ro[k] : args.op.Qoe[k * NE] * ev[0];
#pragma unroll
        for (int j = (UNI && s > 0) ? 0 : 1; j < NE; ++j) t = fma(args.op.Qoe[k * NE + j], ev[j], t);
        po[k] = t;
      }
#pragma unroll
      for (int k = 0; k < NE; ++k) pin(pe[k]);
#pragma unroll
      for (int k = 0; k < NO; ++k) pin(po[k]);
      __syncthreads();
      // a trajectory's first element reads the inflow, its last one its own right node
      const int iL = EDGE && E.first ? CB + st * NS + s : fR + lane;
      const int iR = EDGE && E.last ? fR + lane + 1 : fL + lane + 2;
      const double uL = lds[iL], uR = lds[iR];
      const double dlt = uR - uL, sig = -(uL + uR);
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        if constexpr (UNI) {
          re[k] = fma(args.op.le[k], dlt, pe[k]);
        } else {
          const double a = sc * fma(args.op.le[k], dlt, pe[k]);
          re[k] = (s == 0) ? a : fma(RK<NS>::A(s), re[k], a);
        }
        ev[k] = fma(RK<NS>::B(s), re[k], ev[k]);
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        if constexpr (UNI) {
          ro[k] = fma(args.op.lo[k], sig, po[k]);
        } else {
          const double a = sc * fma(args.op.lo[k], sig, po[k]);
          ro[k] = (s == 0) ? a : fma(RK<NS>::A(s), ro[k], a);
        }
        od[k] = fma(RK<NS>::B(s), ro[k], od[k]);
      }
    }

    // ---- eta -= w^{n+1} . (P u^{n+1} - S_{N+1}(P u^n)) in dual x primal even/odd ----
    if (args.has_eta) {
      double c = 0.0;
#pragma unroll
      for (int k = 0; k < NE; ++k) c = fma(we[k], ne[k] - ev[k], c);
#pragma unroll
      for (int k = 0; k < NO; ++k) c = fma(wo[k], no[k] - od[k], c);
      eacc -= c;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) ne[k] = pn_e[k];
#pragma unroll
    for (int k = 0; k < NO; ++k) no[k] = pn_o[k];
    // the image's readers (prolong above) are 5 stage barriers behind
    if (st > 0) {
      tile_commit<NPL, W>(pa, lds);
      off = pa.off;
    }

    // ---- w^n = S_{N+1}^T w^{n+1}: 5 reverse stages (k_adj's arithmetic at order N+1) ----
    double le_[NE], lo_[NO];
#pragma unroll
    for (int k = 0; k < NE; ++k) le_[k] = 0.0;
#pragma unroll
    for (int k = 0; k < NO; ++k) lo_[k] = 0.0;
#pragma unroll
    for (int ss = 0; ss < NS; ++ss) {
      const int s = NS - 1 - ss;
      const int f0 = G::kFB + ((NS + ss) & 1) * 2 * (T + 2), f1 = f0 + (T + 2);
      double qe[NE], qo[NO];
      double gd = 0.0, gs = 0.0;
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        le_[k] = fma(RK<NS>::B(s), we[k], le_[k]);
        qe[k] = UNI ? le_[k] : sc * le_[k];
        gd = fma(args.op.le[k], qe[k], gd);
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        lo_[k] = fma(RK<NS>::B(s), wo[k], lo_[k]);
        qo[k] = UNI ? lo_[k] : sc * lo_[k];
        gs = fma(args.op.lo[k], qo[k], gs);
      }
      const double g0 = gd + gs, g1 = gs - gd;
      lds[f0 + lane + 1] = g0;
      lds[f1 + lane + 1] = g1;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        double t = we[j];
#pragma unroll
        for (int k = 0; k < NO; ++k) t = fma(args.op.Qoe[k * NE + j], qo[k], t);
        we[j] = t;
      }
#pragma unroll
      for (int j = 0; j < NO; ++j) {
        double t = wo[j];
#pragma unroll
        for (int k = 0; k < NE; ++k) t = fma(args.op.Qeo[k * NO + j], qe[k], t);
        wo[j] = t;
      }
#pragma unroll
      for (int k = 0; k < NE; ++k) le_[k] = RK<NS>::A(s) * le_[k];
#pragma unroll
      for (int k = 0; k < NO; ++k) lo_[k] = RK<NS>::A(s) * lo_[k];
#pragma unroll
      for (int k = 0; k < NE; ++k) pin(we[k]);
#pragma unroll
      for (int k = 0; k < NO; ++k) pin(wo[k]);
      __syncthreads();
      // nothing arrives at a trajectory's first element from the left (its uL is the
      // inflow); its last element's uR is its own u_N (du1 = 0)
      const double gl = lds[EDGE && E.first ? CB + MS * NS : f1 + lane];
      const double gr = lds[EDGE && E.last ? f1 + lane + 1 : f0 + lane + 2];
      we[0] -= gl + gr;
      wo[0] += gr - gl;
    }
  }

  if (args.has_eta && E.valid) eta_update(eta, E.e, eacc, args.has_eta);
  {
    const double(*pwe)[NE] = &we;
    const double(*pwo)[NO] = &wo;
    stage_out<NPH, W, H>(lds, pwe, pwo, true);  // the image's last reads are 5 barriers behind
  }
  __syncthreads();
  const int64_t o0 = tile * TE * NPH;
  if constexpr (EDGE) {
    const int64_t rem = ndh - o0;
    store_run<LB>(wout, o0, rem < int64_t(TE) * NPH ? rem : int64_t(TE) * NPH, lds);
  } else {
    store_full<TE * NPH, LB>(wout, o0, lds);
  }
}

template <int NPL, bool UNI, int W, int MS>
__global__ __launch_bounds__(kBlock * W) void k_adj_p(const double* __restrict__ win,
                                                      double* __restrict__ wout,
                                                      const double* __restrict__ snap,
                                                      double* __restrict__ eta,
                                                      const double* __restrict__ scale,
                                                      AdjPArgs<NPL, MS> args) {
  using G = PGeo<NPL, W>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 5 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = MS * 5;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  if (edge_tile(e0, G::T, args.ktot, args.K))
    adjp_tile<NPL, UNI, W, MS, true>(lds, tile, win, wout, snap, eta, scale, args);
  else
    adjp_tile<NPL, UNI, W, MS, false>(lds, tile, win, wout, snap, eta, scale, args);
}

// u_hi = P u_lo, one element per lane (the enriched terminal state / initial state).
template <int NPL>
__global__ __launch_bounds__(kBlock) void k_prolong(const double* __restrict__ u,
                                                    double* __restrict__ uh, PrEO<NPL> pr,
                                                    int64_t ktot) {
  constexpr int NPH = NPL + 1;
  const int64_t e = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= ktot) return;
  double ul[NPL], ev[EOArgs<NPH>::NE], od[EOArgs<NPH>::NO], out[NPH];
#pragma unroll
  for (int i = 0; i < NPL; ++i) ul[i] = u[e * NPL + i];
  prolong_eo<NPL>(ul, pr, ev, od);
  from_eo<NPH>(ev, od, out);
#pragma unroll
  for (int i = 0; i < NPH; ++i) uh[e * NPH + i] = out[i];
}

template <int NPL, int W, int MS>
int launch_adj_p_e(const dg_plan* lo, const dg_plan* hi, const PrEO<NPL>& pr, const double* win,
                   double* wout, const double* snap, double* eta, int eta_mode,
                   const double* tn, double dt, hipStream_t st) {
  AdjPArgs<NPL, MS> a;
  make_eo<NPL + 1>(hi, hi->uniform ? dt * hi->s_uniform : 1.0, &a.op, true);
  a.pr = pr;
  a.sc = dt;
  for (int m = 0; m < MS; ++m)
    for (int s = 0; s < 5; ++s) a.uin[m * 5 + s] = inflow_value(lo, tn[m] + RK<5>::C(s) * dt);
  a.uin[MS * 5] = 0.0;
  a.ktot = lo->ktot;
  a.stride = lo->ktot * NPL;
  a.K = int32_t(lo->K);
  a.has_eta = eta != nullptr ? (eta_mode | kEtaOn) : 0;
  a.xcd = lo->xcd_order;
  constexpr int TE = kBlock * W - 2 * MS * 5;
  const unsigned grid = grid_for(lo->ktot, TE);
  if (hi->uniform)
    hipLaunchKernelGGL((k_adj_p<NPL, true, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, win, wout,
                       snap, eta, hi->d_scale, a);
  else
    hipLaunchKernelGGL((k_adj_p<NPL, false, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, win, wout,
                       snap, eta, hi->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

// The Horner-form estimate (dg_dwr_tiles.h); the default since round 5 (DG_P_HORNER=0: round
// 3's stage-loop kernel k_adj_p, for A/B runs).
template <int NPL, bool UNI, int W, int MS, bool GL>
__global__ __launch_bounds__(kBlock * W) void k_adj_ph(const double* __restrict__ win,
                                                       double* __restrict__ wout,
                                                       const double* __restrict__ snap,
                                                       double* __restrict__ eta,
                                                       const double* __restrict__ scale,
                                                       AdjPHArgs<NPL, MS> args) {
  using G = PHGeo<NPL, W>;
  using A = AdjPHArgs<NPL, MS>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 5 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = MS * 5;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  const DG_KAS A* ka =
      reinterpret_cast<const DG_KAS A*>(kernarg_tail_k<decltype(&k_adj_ph<NPL, UNI, W, MS, GL>), A>());
  const double* kbnd = reinterpret_cast<const double*>(
      kernarg_tail<decltype(&k_adj_ph<NPL, UNI, W, MS, GL>), A>() + offsetof(A, bnd));
  if (edge_tile(e0, G::T, args.ktot, args.K))
    adjph_tile<NPL, UNI, W, MS, true, GL>(lds, tile, win, wout, snap, eta, scale, args, ka, kbnd,
                                          args.term != 0);
  else
    adjph_tile<NPL, UNI, W, MS, false, GL>(lds, tile, win, wout, snap, eta, scale, args, ka, kbnd,
                                           args.term != 0);
}

// The pipelined form (dg_dwr_tiles.h adjpq_tile): the forward recompute of step n-1 beside
// the reverse step n, one barrier for both per level.
// 4 waves per SIMD (<= 128 VGPRs) where the body is near it: 130 unconstrained at Np = 5
template <int NPL> constexpr int kPQWaves = NPL <= 6 ? 4 : 1;

template <int NPL, bool UNI, int W, int MS>
__global__ __launch_bounds__(kBlock * W) __attribute__((amdgpu_waves_per_eu(kPQWaves<NPL>))) void k_adj_pq(const double* __restrict__ win,
                                                       double* __restrict__ wout,
                                                       const double* __restrict__ snap,
                                                       double* __restrict__ eta,
                                                       const double* __restrict__ scale,
                                                       AdjPHArgs<NPL, MS> args) {
  using G = PQGeo<NPL, W>;
  using A = AdjPHArgs<NPL, MS>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 5 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = MS * 5;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  const DG_KAS A* ka =
      reinterpret_cast<const DG_KAS A*>(kernarg_tail_k<decltype(&k_adj_pq<NPL, UNI, W, MS>), A>());
  const double* kbnd = reinterpret_cast<const double*>(
      kernarg_tail<decltype(&k_adj_pq<NPL, UNI, W, MS>), A>() + offsetof(A, bnd));
  if (edge_tile(e0, G::T, args.ktot, args.K))
    adjpq_tile<NPL, UNI, W, MS, true>(lds, tile, win, wout, snap, eta, scale, args, ka, kbnd);
  else
    adjpq_tile<NPL, UNI, W, MS, false>(lds, tile, win, wout, snap, eta, scale, args, ka, kbnd);
}

inline int p_horner();

template <int NPL, int W, int MS>
int launch_adj_ph_e(const dg_plan* lo, const dg_plan* hi, const PrEO<NPL>& pr, const double* win,
                    double* wout, const double* snap, double* eta, int eta_mode,
                    const double* tn, double dt, hipStream_t st, bool term) {
  const dgr::RkPoly& P = dgr::rk_poly();
  if (!P.ok) return fail(DG_ERR_HIP, "LSERK4 stability polynomial: beta_0 = beta_1 = 1 expected");
  AdjPHArgs<NPL, MS> a;
  make_eo<NPL + 1>(hi, hi->uniform ? dt * hi->s_uniform : 1.0, &a.op, true);
  a.pr = pr;
  a.sc = dt;
  for (int k = 0; k < 6; ++k) a.beta[k] = P.beta[k];
  double bnd[MS * 6 + 1];
  dgr::rp_block_bnd(lo, MS, tn, dt, bnd);  // level weights of the MS steps (+ inflow values)
  for (int i = 0; i < MS * 5; ++i) a.bnd[i] = bnd[i];
  a.bnd[MS * 5] = 0.0;
  a.ktot = lo->ktot;
  a.stride = lo->ktot * NPL;
  a.K = int32_t(lo->K);
  a.has_eta = eta != nullptr ? (eta_mode | kEtaOn) : 0;
  a.xcd = lo->xcd_order;
  a.term = term ? 1 : 0;
  constexpr int TE = kBlock * W - 2 * MS * 5;
  const unsigned grid = grid_for(lo->ktot, TE);
  if (p_horner() == 2) {
    if (hi->uniform)
      hipLaunchKernelGGL((k_adj_pq<NPL, true, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, win,
                         wout, snap, eta, hi->d_scale, a);
    else
      hipLaunchKernelGGL((k_adj_pq<NPL, false, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, win,
                         wout, snap, eta, hi->d_scale, a);
  } else if (p_horner() == 3) {
    if (hi->uniform)
      hipLaunchKernelGGL((k_adj_ph<NPL, true, W, MS, true>), dim3(grid), dim3(kBlock * W), 0, st,
                         win, wout, snap, eta, hi->d_scale, a);
    else
      hipLaunchKernelGGL((k_adj_ph<NPL, false, W, MS, true>), dim3(grid), dim3(kBlock * W), 0, st,
                         win, wout, snap, eta, hi->d_scale, a);
  } else if (hi->uniform) {
    hipLaunchKernelGGL((k_adj_ph<NPL, true, W, MS, false>), dim3(grid), dim3(kBlock * W), 0, st,
                       win, wout, snap, eta, hi->d_scale, a);
  } else {
    hipLaunchKernelGGL((k_adj_ph<NPL, false, W, MS, false>), dim3(grid), dim3(kBlock * W), 0, st,
                       win, wout, snap, eta, hi->d_scale, a);
  }
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

// ---------------------------------------------------------------------------
// The estimate as ONE dataflow launch (k_adjp_flow; plan->p_flow, dg_plan_tune
// DG_TUNE_P_FLOW).  The launch-per-block chain pays each launch's fill and drain: at K = 2^20,
// Np = 5 a 4-step launch is 4,855 tiles of 17-us workgroups over 1,536 resident slots, and the
// SQ counters put the average residency at 4.3 of 6 waves per SIMD (profiles/r05/p_gl_w1).
// Here the blocks' tiles are the work items of one launch, in queue order block 0 (the last
// MS steps) tiles 0..nT-1, block 1, ...; item (b, j) waits for (b-1, j-1..j+1), whose outputs
// cover its input range (halo < TE).  The hand-off protocol, the take counter, the watchdog
// and the poisoning are the jump sweep's (dg_sweep_kernel.h, dg_flow.h): w is handed off
// write-through and loaded sc1; each block but the last writes its indicator partials to its
// own row and the last adds them in launch order (bit-identical to the chain); the fused
// refine decision (dg_lserk4_adj_p_refine) reduces the last block's tile winners.  The
// snapshots come from an earlier launch: plain loads (and direct-to-LDS, GL).
// ---------------------------------------------------------------------------
template <int NPL, int MS> struct AdjPFArgs {
  static constexpr int kMaxBlocks = dgr::kSweepMaxSteps / MS;
  EOArgs<NPL + 1> op;
  PrEO<NPL> pr;
  double sc;
  double beta[6];
  double bnd[kMaxBlocks * (MS * 5 + 1)];  // block b's level weights at b (5 MS + 1), then a 0
  const double* snap;                    // u^0 .. u^nsteps, `stride` doubles apart
  double* W[kMaxBlocks + 1];             // block b reads W[b] (W[0]: terminal weight), writes W[b+1]
  double* eta;
  double* part;                          // (nb - 1) rows of ktot: the blocks' partial indicators
  const double* scale;
  uint32_t* sync;                        // kSync* words, then one flag per item
  uint32_t* err_host;
  uint64_t* trace;                       // nullable: 8 words per item {started, dequeued,
                                         // producers done, body done, published, XCC id << 32
                                         // | workgroup id, 0, 0} (wall clock, 100 MHz)
  int64_t* am_idx;                       // nullable: the fused refine decision
  double* am_val;
  int64_t* am_nf;
  double* am_pv;                         // per last-block tile: its (|eta|, element) winner
  int64_t* am_pi;
  int64_t ktot;
  int64_t stride;
  int32_t K;
  int32_t has_eta;                       // kEta* bits of the whole sweep
  int32_t term;                          // block 0's terminal weight is P u^nsteps
  int32_t nb, nT, nsteps, spin_limit;
};

// 6 waves per SIMD (<= 80 VGPRs, as k_adj_ph<..., GL> compiles unconstrained) where the body
// fits: the item decode and the indicator sink would otherwise take it to 100 at Np = 5.
template <int NPL, bool UNI> constexpr int kPFWaves = (UNI && NPL <= 5) ? 6 : 1;

template <int NPL, bool UNI, int W, int MS>
__global__ __launch_bounds__(kBlock * W) __attribute__((amdgpu_waves_per_eu(kPFWaves<NPL, UNI>)))
void k_adjp_flow(AdjPFArgs<NPL, MS> a) {
  using G = PHGeo<NPL, W>;
  using A = AdjPFArgs<NPL, MS>;
  static_assert(sizeof(A) <= kKernargMax, "k_adjp_flow's arguments exceed the kernarg segment");
  constexpr int NPH = NPL + 1, H = MS * 5, TE = G::T - 2 * H, NW = kBlock * W / 64;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 5 + 1];
  __shared__ uint32_t s_item, s_epoch, s_last, s_bad;
  __shared__ double s_av[NW];
  __shared__ int64_t s_ai[NW];
  uint32_t* sync = a.sync;
  uint32_t* flags = sync + dgr::kSyncFlags;
  const int tid = threadIdx.x;
  const int nT = a.nT, nb = a.nb;
  const uint64_t t_start = a.trace ? uint64_t(wall_clock64()) : 0;
  if (tid == 0) {
    uint32_t it, ep;
    dgr::flow_take(sync, int64_t(nb) * nT, &it, &ep);
    s_item = it;
    s_epoch = ep;
    s_bad = 0u;
  }
  __syncthreads();
  const int64_t item = s_item;
  const uint32_t epoch = s_epoch;
  const uint64_t t_deq = a.trace ? uint64_t(wall_clock64()) : 0;
  uint64_t t_ready = 0;
  const int blk = int(item / nT), j = int(item - int64_t(blk) * nT);
  // the poll of the previous block's tiles j-1..j+1, run by the tile body once its snapshot
  // loads are in flight
  const auto wait_inputs = [&]() {
    if (blk > 0 && tid < 64) {
      const int lo = j > 0 ? j - 1 : 0, hi = j + 1 < nT ? j + 1 : nT - 1;
      const bool gave_up = dgr::sweep_wait(flags + int64_t(blk - 1) * nT + lo, hi - lo + 1,
                                           epoch, sync, a.err_host, a.spin_limit);
      if (tid == 0 && gave_up) s_bad = 1u;
    }
    // no acquire fence: every load of handed-off bytes is an sc1 load; this only keeps the
    // compiler from hoisting them above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    if (a.trace) t_ready = uint64_t(wall_clock64());
  };
  const DG_KAS A* ka =
      reinterpret_cast<const DG_KAS A*>(kernarg_tail_k<decltype(&k_adjp_flow<NPL, UNI, W, MS>), A>());
  const double* kbnd = reinterpret_cast<const double*>(
                           kernarg_tail<decltype(&k_adjp_flow<NPL, UNI, W, MS>), A>() +
                           offsetof(A, bnd)) + blk * (MS * 5 + 1);
  const int64_t ktot = a.ktot;
  const int64_t n0 = int64_t(a.nsteps) - int64_t(blk + 1) * MS;
  const bool lastb = blk == nb - 1;
  dgr::EtaSink es;
  es.eta = a.eta;
  es.part_out = (a.has_eta && !lastb) ? a.part + int64_t(blk) * ktot : nullptr;
  es.part_in = a.part;
  es.part_ld = ktot;
  es.nparts = lastb ? nb - 1 : 0;
  es.mode = a.has_eta;
  es.argmax = lastb && a.am_idx != nullptr;
  es.bv = -INFINITY;  // the weakest candidate (dg_argmax's convention)
  es.bi = INT64_MAX;
  const double* snap = a.snap + n0 * a.stride;
  const bool term = a.term != 0 && blk == 0;
  const int64_t e0 = int64_t(j) * TE - H;
  if (edge_tile(e0, G::T, ktot, a.K))
    adjph_tile<NPL, UNI, W, MS, true, true, true, A>(lds, j, a.W[blk], a.W[blk + 1], snap, a.eta,
                                                     a.scale, a, ka, kbnd, term, &es,
                                                     wait_inputs);
  else
    adjph_tile<NPL, UNI, W, MS, false, true, true, A>(lds, j, a.W[blk], a.W[blk + 1], snap,
                                                      a.eta, a.scale, a, ka, kbnd, term, &es,
                                                      wait_inputs);
  if (s_bad) {
    // the body's own write-through stores (another lane mapping) complete first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int64_t o0 = int64_t(j) * TE, ndh = ktot * NPH;
    const int64_t ne = (ktot - o0) < TE ? ktot - o0 : int64_t(TE);
    dgr::poison_run<kBlock * W>(a.W[blk + 1], o0 * NPH,
                                (ndh - o0 * NPH) < int64_t(TE) * NPH ? ndh - o0 * NPH
                                                                     : int64_t(TE) * NPH);
    if (a.has_eta) dgr::poison_run<kBlock * W>(es.part_out ? es.part_out : a.eta, o0, ne);
    es.bv = __builtin_nan("");
  }
  if (es.argmax) {  // the tile's winner, a hand-off to the last arriving tile
    dgr::wg_argmax<NW>(es.bv, es.bi, s_av, s_ai);
    if (tid == 0) {
      dgr::st8_agent(a.am_pv + j, __builtin_bit_cast(uint64_t, es.bv));
      dgr::st8_agent(a.am_pi + j, uint64_t(es.bi));
    }
  }
  // publish: every wave's write-through stores have completed, then one flag store
  const uint64_t t_body = a.trace ? uint64_t(wall_clock64()) : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) dgr::st_agent(flags + item, epoch);
  if (es.argmax)
    dgr::flow_refine_arrive<NW>(sync, nT, a.am_pv, a.am_pi, a.am_idx, a.am_val, a.am_nf, &s_last,
                                s_av, s_ai);
  if (a.trace && tid == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* tr = a.trace + 8 * item;
    tr[0] = t_start;
    tr[1] = t_deq;
    tr[2] = t_ready;
    tr[3] = t_body;
    tr[4] = uint64_t(wall_clock64());
    tr[5] = (uint64_t(xcc) << 32) | blockIdx.x;
  }
}

// Buffers of one k_adjp_flow launch (dg_lserk4_adj_p's scratch on the order-N plan).
struct PFlowBufs {
  double* W[dgr::kSweepMaxSteps + 1];
  double* part;
  uint32_t* sync;
  int64_t* am_idx;
  double* am_val;
  int64_t* am_nf;
  double* am_pv;
  int64_t* am_pi;
};

template <int NPL, int W, int MS>
int launch_adjp_flow(dg_plan* lo, const dg_plan* hi, const PrEO<NPL>& pr, const PFlowBufs& b,
                     const double* snapshots, double* eta, int mode, const double* tn, double dt,
                     int nsteps, bool term, hipStream_t st) {
  const dgr::RkPoly& P = dgr::rk_poly();
  if (!P.ok) return fail(DG_ERR_HIP, "LSERK4 stability polynomial: beta_0 = beta_1 = 1 expected");
  using A = AdjPFArgs<NPL, MS>;
  const int nb = nsteps / MS;
  if (nb < 2 || nb > A::kMaxBlocks || nb * MS != nsteps)
    return fail(DG_ERR_ARG, "p-estimate dataflow: nsteps must be 2..40/MS blocks of MS steps");
  A a;
  make_eo<NPL + 1>(hi, hi->uniform ? dt * hi->s_uniform : 1.0, &a.op, true);
  a.pr = pr;
  a.sc = dt;
  for (int k = 0; k < 6; ++k) a.beta[k] = P.beta[k];
  for (int bk = 0; bk < nb; ++bk) {  // block b covers steps n0 .. n0+MS-1, n0 = nsteps - (b+1) MS
    const int n0 = nsteps - (bk + 1) * MS;
    double bnd[MS * 6 + 1];
    dgr::rp_block_bnd(lo, MS, &tn[n0], dt, bnd);
    double* row = a.bnd + bk * (MS * 5 + 1);
    for (int i = 0; i < MS * 5; ++i) row[i] = bnd[i];
    row[MS * 5] = 0.0;
  }
  for (int bk = nb; bk < A::kMaxBlocks; ++bk)
    for (int i = 0; i <= MS * 5; ++i) a.bnd[bk * (MS * 5 + 1) + i] = 0.0;
  a.snap = snapshots;
  for (int i = 0; i <= A::kMaxBlocks; ++i) a.W[i] = i <= nb ? b.W[i] : nullptr;
  a.eta = eta;
  a.part = b.part;
  a.scale = hi->d_scale;
  a.sync = b.sync;
  a.err_host = lo->d_sweep_err;
  a.trace = lo->sweep_trace;
  a.am_idx = b.am_idx;
  a.am_val = b.am_val;
  a.am_nf = b.am_nf;
  a.am_pv = b.am_pv;
  a.am_pi = b.am_pi;
  a.ktot = lo->ktot;
  a.stride = lo->ktot * NPL;
  a.K = int32_t(lo->K);
  a.has_eta = mode;
  a.term = term ? 1 : 0;
  a.nb = nb;
  a.nT = int(grid_for(lo->ktot, kBlock * W - 2 * MS * 5));
  a.nsteps = nsteps;
  a.spin_limit = lo->sweep_spin_limit > 0 ? lo->sweep_spin_limit : dgr::kSweepSpinLimit;
  const unsigned grid = unsigned(int64_t(nb) * a.nT);
  if (hi->uniform)
    hipLaunchKernelGGL((k_adjp_flow<NPL, true, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, a);
  else
    hipLaunchKernelGGL((k_adjp_flow<NPL, false, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

// ---------------------------------------------------------------------------
// The p-estimate's WHOLE sweep -- the order-N snapshot forward and the estimate -- as ONE
// dataflow launch (k_psweep, dg_lserk4_sweep_p).  The forward's launches drain like the
// estimate's did (k_step at 8 steps per launch: 2,428 tiles are 3.16 rounds of the resident
// workgroups; SQ: 4.1 of 6-7 waves per SIMD resident on average, profiles/r05/p).  Items, in
// queue order: forward block 0 tiles 0..nT-1 (steps 0..MS-1), forward block 1, ..., then the
// estimate's blocks as k_adjp_flow.  Forward item (b, k) waits for forward block b-1's tiles
// k-1..k+1 (its input u^{b MS} is that block's last snapshot); estimate block 0 tile j waits
// for the last forward block's tiles j-1..j+1 -- whose completion implies every earlier
// forward block's snapshots around them, the cone growing a tile per block -- and later
// estimate blocks as k_adjp_flow.  Every snapshot is stored write-through and every load of
// one (the forward's input, the estimate's tiles, also direct-to-LDS) is sc1, after the poll.
// Forward and estimate tiles are both 256 * W elements with MS-step blocks (H = 5 MS), so the
// forward's arithmetic is k_step's at MS steps per launch: bit-identical to dg_lserk4_fwd
// with that steps-per-launch followed by dg_lserk4_adj_p.
// ---------------------------------------------------------------------------
constexpr int kPSMaxSteps = 32;  // 8 blocks of 4: the blocks' constants fit the kernarg segment

template <int NPL, int MS> struct PSweepArgs {
  static constexpr int kMaxBlocks = kPSMaxSteps / MS;
  // the estimate's (names as AdjPHArgs: adjph_tile reads them)
  EOArgs<NPL + 1> op;
  PrEO<NPL> pr;
  double sc;
  double beta[6];
  double bnd[kMaxBlocks * (MS * 5 + 1)];
  // the forward's: its operator (order N) and each block's stage inflow values (StepArgs uin)
  EOArgs<NPL> fop;
  double fuin[kMaxBlocks * (MS * 5 + 1)];
  double* snap;                          // u^0 (the caller's) .. u^nsteps, `stride` apart
  double* W[kMaxBlocks + 1];
  double* eta;
  double* part;
  const double* scale;                   // the estimate's metric (hi plan)
  const double* fscale;                  // the forward's (lo plan)
  uint32_t* sync;
  uint32_t* err_host;
  uint64_t* trace;                       // nullable: 8 words per item as k_adjp_flow's
  int64_t* am_idx;
  double* am_val;
  int64_t* am_nf;
  double* am_pv;
  int64_t* am_pi;
  int64_t ktot;
  int64_t stride;
  int32_t K;
  int32_t has_eta;
  int32_t nb;                            // blocks per direction
  int32_t nT;                            // tiles per block (both directions)
  int32_t nsteps;
  int32_t spin_limit;
};

// step_tile's view of the forward's arguments (StepArgs' names)
template <int NP> struct PFwdView {
  const EOArgs<NP>& op;
  double sc;
  int64_t ktot, stride, n0;
  int32_t K, jend;
};

template <int NPL, int W, int MS> struct PSGeo {
  static constexpr int kA = PHGeo<NPL, W>::kLds, kF = TileGeo<NPL, W>::kLds;
  static constexpr int kLds = (kA > kF ? kA : kF) + MS * 5 + 1;
};

template <int NPL, bool UNI, int W, int MS>
__global__ __launch_bounds__(kBlock * W) __attribute__((amdgpu_waves_per_eu(kPFWaves<NPL, UNI>)))
void k_psweep(PSweepArgs<NPL, MS> a) {
  using A = PSweepArgs<NPL, MS>;
  static_assert(sizeof(A) <= kKernargMax, "k_psweep's arguments exceed the kernarg segment");
  constexpr int NPH = NPL + 1, H = MS * 5, T = kBlock * W, TE = T - 2 * H, NW = T / 64;
  __shared__ __attribute__((aligned(16))) double lds[PSGeo<NPL, W, MS>::kLds];
  __shared__ uint32_t s_item, s_epoch, s_last, s_bad;
  __shared__ double s_av[NW];
  __shared__ int64_t s_ai[NW];
  uint32_t* sync = a.sync;
  uint32_t* flags = sync + dgr::kSyncFlags;
  const int tid = threadIdx.x;
  const int nT = a.nT, nb = a.nb;
  const int64_t nF = int64_t(nb) * nT;
  const uint64_t t_start = a.trace ? uint64_t(wall_clock64()) : 0;
  if (tid == 0) {
    uint32_t it, ep;
    dgr::flow_take(sync, 2 * nF, &it, &ep);
    s_item = it;
    s_epoch = ep;
    s_bad = 0u;
  }
  __syncthreads();
  const int64_t item = s_item;
  const uint32_t epoch = s_epoch;
  const uint64_t t_deq = a.trace ? uint64_t(wall_clock64()) : 0;
  uint64_t t_ready = 0;
  const bool fwd = item < nF;
  const int blk = int((fwd ? item : item - nF) / nT);
  const int j = int((fwd ? item : item - nF) - int64_t(blk) * nT);
  const int64_t ktot = a.ktot;
  // the poll: the previous block's tiles j-1..j+1 of the same direction; estimate block 0:
  // the last forward block's (items nF - nT ..)
  const auto wait_producers = [&]() {
    if ((blk > 0 || !fwd) && tid < 64) {
      const int lo = j > 0 ? j - 1 : 0, hi = j + 1 < nT ? j + 1 : nT - 1;
      const int64_t d0 = fwd ? int64_t(blk - 1) * nT : (blk == 0 ? nF - nT : nF + int64_t(blk - 1) * nT);
      const bool gave_up = dgr::sweep_wait(flags + d0 + lo, hi - lo + 1, epoch, sync, a.err_host,
                                           a.spin_limit);
      if (tid == 0 && gave_up) s_bad = 1u;
    }
    // no acquire fence: every load of handed-off bytes is an sc1 load; this only keeps the
    // compiler from hoisting them above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    if (a.trace) t_ready = uint64_t(wall_clock64());
  };
  dgr::EtaSink es;
  es.argmax = false;
  es.bv = -INFINITY;  // the weakest candidate (dg_argmax's convention)
  es.bi = INT64_MAX;
  const int64_t e0 = int64_t(j) * TE - H;
  const bool edge = edge_tile(e0, T, ktot, a.K);
  if (fwd) {
    wait_producers();
    const int64_t n0 = int64_t(blk) * MS;
    const PFwdView<NPL> v{a.fop, a.sc, ktot, a.stride, n0, a.K, 0};
    const double* kin = a.fuin + blk * (MS * 5 + 1);
    if (edge)
      step_tile<NPL, 5, UNI, W, MS, false, true, true>(lds, j, a.snap + n0 * a.stride,
                                                       a.snap + (n0 + 1) * a.stride, nullptr,
                                                       a.fscale, v, kin);
    else
      step_tile<NPL, 5, UNI, W, MS, false, false, true>(lds, j, a.snap + n0 * a.stride,
                                                        a.snap + (n0 + 1) * a.stride, nullptr,
                                                        a.fscale, v, kin);
    if (s_bad) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int64_t o0 = int64_t(j) * TE * NPL, nd = ktot * NPL;
      const int64_t cnt = (nd - o0) < int64_t(TE) * NPL ? nd - o0 : int64_t(TE) * NPL;
      for (int st = 0; st < MS; ++st)
        dgr::poison_run<T>(a.snap + (n0 + 1 + st) * a.stride, o0, cnt);
    }
  } else {
    const DG_KAS A* ka =
        reinterpret_cast<const DG_KAS A*>(kernarg_tail_k<decltype(&k_psweep<NPL, UNI, W, MS>), A>());
    const double* kbnd = reinterpret_cast<const double*>(
                             kernarg_tail<decltype(&k_psweep<NPL, UNI, W, MS>), A>() +
                             offsetof(A, bnd)) + blk * (MS * 5 + 1);
    const int64_t n0 = int64_t(a.nsteps) - int64_t(blk + 1) * MS;
    const bool lastb = blk == nb - 1;
    es.eta = a.eta;
    es.part_out = (a.has_eta && !lastb) ? a.part + int64_t(blk) * ktot : nullptr;
    es.part_in = a.part;
    es.part_ld = ktot;
    es.nparts = lastb ? nb - 1 : 0;
    es.mode = a.has_eta;
    es.argmax = lastb && a.am_idx != nullptr;
    const double* snap = a.snap + n0 * a.stride;
    const bool term = blk == 0;  // the terminal weight P u^nsteps
    using WP = decltype(wait_producers);
    if (edge)
      adjph_tile<NPL, UNI, W, MS, true, true, true, A, NoWait, true, WP>(
          lds, j, a.W[blk], a.W[blk + 1], snap, a.eta, a.scale, a, ka, kbnd, term, &es, NoWait(),
          wait_producers);
    else
      adjph_tile<NPL, UNI, W, MS, false, true, true, A, NoWait, true, WP>(
          lds, j, a.W[blk], a.W[blk + 1], snap, a.eta, a.scale, a, ka, kbnd, term, &es, NoWait(),
          wait_producers);
    if (s_bad) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int64_t o0 = int64_t(j) * TE, ndh = ktot * NPH;
      const int64_t ne = (ktot - o0) < TE ? ktot - o0 : int64_t(TE);
      dgr::poison_run<T>(a.W[blk + 1], o0 * NPH,
                         (ndh - o0 * NPH) < int64_t(TE) * NPH ? ndh - o0 * NPH : int64_t(TE) * NPH);
      if (a.has_eta) dgr::poison_run<T>(es.part_out ? es.part_out : a.eta, o0, ne);
      es.bv = __builtin_nan("");
    }
    if (es.argmax) {
      dgr::wg_argmax<NW>(es.bv, es.bi, s_av, s_ai);
      if (tid == 0) {
        dgr::st8_agent(a.am_pv + j, __builtin_bit_cast(uint64_t, es.bv));
        dgr::st8_agent(a.am_pi + j, uint64_t(es.bi));
      }
    }
  }
  const uint64_t t_body = a.trace ? uint64_t(wall_clock64()) : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) dgr::st_agent(flags + item, epoch);
  if (es.argmax)
    dgr::flow_refine_arrive<NW>(sync, nT, a.am_pv, a.am_pi, a.am_idx, a.am_val, a.am_nf, &s_last,
                                s_av, s_ai);
  if (a.trace && tid == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* tr = a.trace + 8 * item;
    tr[0] = t_start;
    tr[1] = t_deq;
    tr[2] = t_ready;
    tr[3] = t_body;
    tr[4] = uint64_t(wall_clock64());
    tr[5] = (uint64_t(xcc) << 32) | blockIdx.x;
  }
}

template <int NPL, int W, int MS>
int launch_psweep(dg_plan* lo, const dg_plan* hi, const PrEO<NPL>& pr, const PFlowBufs& b,
                  double* snapshots, double* eta, int mode, const double* tn, double dt,
                  int nsteps, hipStream_t st) {
  const dgr::RkPoly& P = dgr::rk_poly();
  if (!P.ok) return fail(DG_ERR_HIP, "LSERK4 stability polynomial: beta_0 = beta_1 = 1 expected");
  using A = PSweepArgs<NPL, MS>;
  const int nb = nsteps / MS;
  if (nb < 2 || nb > A::kMaxBlocks || nb * MS != nsteps)
    return fail(DG_ERR_ARG, "p sweep dataflow: nsteps must be 2..32/MS blocks of MS steps");
  A a;
  make_eo<NPL + 1>(hi, hi->uniform ? dt * hi->s_uniform : 1.0, &a.op, true);
  a.pr = pr;
  a.sc = dt;
  for (int k = 0; k < 6; ++k) a.beta[k] = P.beta[k];
  make_eo<NPL>(lo, lo->uniform ? dt * lo->s_uniform : 1.0, &a.fop, true);  // as launch_step_e
  for (int i = 0; i < A::kMaxBlocks * (MS * 5 + 1); ++i) a.bnd[i] = a.fuin[i] = 0.0;
  for (int bk = 0; bk < nb; ++bk) {
    const int n0 = nsteps - (bk + 1) * MS;  // estimate block b
    double bnd[MS * 6 + 1];
    dgr::rp_block_bnd(lo, MS, &tn[n0], dt, bnd);
    for (int i = 0; i < MS * 5; ++i) a.bnd[bk * (MS * 5 + 1) + i] = bnd[i];
    const int f0 = bk * MS;  // forward block b: StepArgs::uin of a launch at t_{f0}
    double* u = a.fuin + bk * (MS * 5 + 1);
    for (int m = 0; m < MS; ++m)
      for (int s = 0; s < 5; ++s) u[m * 5 + s] = inflow_value(lo, tn[f0 + m] + RK<5>::C(s) * dt);
    u[MS * 5] = inflow_value(lo, tn[f0 + MS]);
  }
  a.snap = snapshots;
  for (int i = 0; i <= A::kMaxBlocks; ++i) a.W[i] = i <= nb ? b.W[i] : nullptr;
  a.eta = eta;
  a.part = b.part;
  a.scale = hi->d_scale;
  a.fscale = lo->d_scale;
  a.sync = b.sync;
  a.err_host = lo->d_sweep_err;
  a.trace = lo->sweep_trace;
  a.am_idx = b.am_idx;
  a.am_val = b.am_val;
  a.am_nf = b.am_nf;
  a.am_pv = b.am_pv;
  a.am_pi = b.am_pi;
  a.ktot = lo->ktot;
  a.stride = lo->ktot * NPL;
  a.K = int32_t(lo->K);
  a.has_eta = mode;
  a.nb = nb;
  a.nT = int(grid_for(lo->ktot, kBlock * W - 2 * MS * 5));
  a.nsteps = nsteps;
  a.spin_limit = lo->sweep_spin_limit > 0 ? lo->sweep_spin_limit : dgr::kSweepSpinLimit;
  const unsigned grid = unsigned(2 * int64_t(nb) * a.nT);
  if (hi->uniform)
    hipLaunchKernelGGL((k_psweep<NPL, true, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, a);
  else
    hipLaunchKernelGGL((k_psweep<NPL, false, W, MS>), dim3(grid), dim3(kBlock * W), 0, st, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

// DG_P_HORNER (read once, A/B runs): 0 round 3's stage loop (k_adj_p), 1 Horner (k_adj_ph)
// with the next snapshot tile prefetched into registers (94 VGPRs at Np = 5: 5 waves per
// SIMD), 2 Horner pipelined (k_adj_pq: the forward recompute of step n-1 beside the reverse
// step n, half the barriers; 125 VGPRs, 4 waves per SIMD: measured 2-5 % slower than
// k_adj_ph, profiles/r05/p3), 3 (default) Horner with the snapshot tiles loaded straight into
// LDS (k_adj_ph<..., GL = true>: 80 VGPRs, 6 waves per SIMD; 1-2 % faster than 1,
// profiles/r05/p5, p13).  The dataflow launch (k_adjp_flow) always loads into LDS.
inline int p_horner() {
  static const int v = [] {
    const char* e = std::getenv("DG_P_HORNER");
    const int k = e ? std::atoi(e) : 3;
    return (k == 0 || k == 1 || k == 2) ? k : 3;
  }();
  return v;
}

// Shapes: 256-element tiles with 1, 2 or 4 steps per launch; 512-element tiles with 2, 4 or 8.
template <int NPL>
int launch_adj_p_t(const dg_plan* lo, const dg_plan* hi, const PrEO<NPL>& pr, int ms,
                   const double* win, double* wout, const double* snap, double* eta, int em,
                   const double* tn, double dt, hipStream_t st, bool term) {
  const bool w2 = lo->p_tile_width == 2;
  if (p_horner()) {
    if (w2 && ms == 8) return launch_adj_ph_e<NPL, 2, 8>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st, term);
    if (w2 && ms == 4) return launch_adj_ph_e<NPL, 2, 4>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st, term);
    if (w2 && ms == 2) return launch_adj_ph_e<NPL, 2, 2>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st, term);
    if (ms == 4) return launch_adj_ph_e<NPL, 1, 4>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st, term);
    if (ms == 2) return launch_adj_ph_e<NPL, 1, 2>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st, term);
    if (ms == 1) return launch_adj_ph_e<NPL, 1, 1>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st, term);
    return fail(DG_ERR_ARG, "p-estimate: unsupported steps per launch for this tile width");
  }
  if (w2 && ms == 8) return launch_adj_p_e<NPL, 2, 8>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st);
  if (w2 && ms == 4) return launch_adj_p_e<NPL, 2, 4>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st);
  if (w2 && ms == 2) return launch_adj_p_e<NPL, 2, 2>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st);
  if (ms == 4) return launch_adj_p_e<NPL, 1, 4>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st);
  if (ms == 2) return launch_adj_p_e<NPL, 1, 2>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st);
  if (ms == 1) return launch_adj_p_e<NPL, 1, 1>(lo, hi, pr, win, wout, snap, eta, em, tn, dt, st);
  return fail(DG_ERR_ARG, "p-estimate: unsupported steps per launch for this tile width");
}

// The estimate's steps per launch: the plan's setting (8 needs 512-element tiles), halved
// until it fits the steps left.
inline int p_msteps(const dg_plan* p) {
  int m = p->p_msteps;
  if (m == 8 && p->p_tile_width != 2) m = 4;
  return m;
}
inline int chunk_p(const dg_plan* p, int left) {
  int m = p_msteps(p);
  while (m > left) m >>= 1;
  return m < 1 ? 1 : m;
}

// Both plans describe one mesh and one problem (the order-(N+1) plan is the estimate's).
int check_pair(const dg_plan* lo, const dg_plan* hi) {
  if (hi->NP != lo->NP + 1) return fail(DG_ERR_ARG, "the enriched plan must have order N+1");
  if (hi->K != lo->K || hi->batch != lo->batch)
    return fail(DG_ERR_ARG, "the two plans differ in K or batch");
  if (hi->a != lo->a || hi->inflow != lo->inflow)
    return fail(DG_ERR_ARG, "the two plans differ in advection speed or inflow");
  if (lo->nstages != 5 || hi->nstages != 5)
    return fail(DG_ERR_ARG, "the p-estimate is the LSERK4 sweep's");
  if (lo->nonlinear() || hi->nonlinear())
    return fail(DG_ERR_ARG, "the p-estimate needs the linear flux without limiter");
  if (hi->uniform != lo->uniform ||
      (lo->uniform && std::fabs(hi->s_uniform - lo->s_uniform) > 1e-12 * lo->s_uniform))
    return fail(DG_ERR_ARG, "the two plans are not on the same mesh");
  return DG_OK;
}

// The dataflow form applies: the plan asks for it, the Horner kernels are selected, and the
// steps split into 2 .. 40/MS blocks of the plan's steps per launch (4 on 256-element tiles;
// 4 or 8 on 512-element tiles).
bool p_flow_shape(const dg_plan* lo, int nsteps) {
  const int m = p_msteps(lo);
  const int h = p_horner();
  return lo->p_flow && (h == 1 || h == 3) && (m == 4 || (m == 8 && lo->p_tile_width == 2)) &&
         nsteps > 0 && nsteps % m == 0 && nsteps / m >= 2 && nsteps <= dgr::kSweepMaxSteps;
}

// One dataflow launch of the whole estimate (k_adjp_flow).  Scratch: the lo plan's dataflow
// region (sweep_scratch: control words, then the blocks' w outputs W[1..nb-1] and partial
// indicator rows, sized for the reserved capacity).  W[0] = W[nb] = w: the first block reads
// it (unless the terminal weight is formed in the kernel) and the last rewrites it; with
// nb >= 2 the last block's tile j starts after every first-block tile whose input range
// overlaps its output range (j-1..j+1, through the chain of waits).
int p_flow_bufs(dg_plan* lo, const dg_plan* hi, uint64_t tag, int m, int W, int nsteps,
                int64_t items, int64_t items_cap, int64_t nT, int64_t nT_cap, int nb, double* w,
                bool eta, int64_t* idx, double* value, int64_t* nonfinite, hipStream_t st,
                PFlowBufs* b);

int adjp_flow(dg_plan* lo, const dg_plan* hi, const double* P, double* w,
              const double* snapshots, const double* tn, double dt, int nsteps, double* eta,
              int mode, bool term, int64_t* idx, double* value, int64_t* nonfinite,
              hipStream_t st) {
  const int m = p_msteps(lo), nb = nsteps / m, W = lo->p_tile_width;
  const int64_t TE = int64_t(kBlock) * W - 10 * m;
  const int64_t nT = (lo->ktot + TE - 1) / TE;
  const int64_t nT_cap = (lo->K_cap * lo->batch + TE - 1) / TE;
  PFlowBufs b;
  if (const int rc = p_flow_bufs(lo, hi, 0x5a, m, W, nsteps, int64_t(nb) * nT, int64_t(nb) * nT_cap,
                                 nT, nT_cap, nb, w, eta != nullptr, idx, value, nonfinite, st, &b))
    return rc;
  int rc = DG_OK;
  switch (lo->NP) {
#define DG_ADJPF_CASE(NPLV)                                                                  \
    case NPLV: {                                                                             \
      PrEO<NPLV> pr;                                                                         \
      if (!make_prolong_eo<NPLV>(P, &pr))                                                    \
        return fail(DG_ERR_ARG, "P does not commute with the node reversal (symmetric nodes)"); \
      if (W == 2 && m == 8)                                                                  \
        rc = launch_adjp_flow<NPLV, 2, 8>(lo, hi, pr, b, snapshots, eta, mode, tn, dt, nsteps, \
                                          term, st);                                         \
      else if (W == 2)                                                                       \
        rc = launch_adjp_flow<NPLV, 2, 4>(lo, hi, pr, b, snapshots, eta, mode, tn, dt, nsteps, \
                                          term, st);                                         \
      else                                                                                   \
        rc = launch_adjp_flow<NPLV, 1, 4>(lo, hi, pr, b, snapshots, eta, mode, tn, dt, nsteps, \
                                          term, st);                                         \
    } break;
    DG_ADJPF_CASE(2) DG_ADJPF_CASE(3) DG_ADJPF_CASE(4) DG_ADJPF_CASE(5)
    DG_ADJPF_CASE(6) DG_ADJPF_CASE(7) DG_ADJPF_CASE(8)
#undef DG_ADJPF_CASE
    default: return fail(DG_ERR_ARG, "the p-estimate supports N <= 7");
  }
  return rc;
}

// The whole sweep as one dataflow launch applies: the estimate's dataflow shape at 4-step
// blocks, the forward's stage-loop workgroup tiles (not the wave tiles of N <= 2), and
// 2..8 blocks.
bool p_sweep_shape(const dg_plan* lo, int nsteps) {
  return lo->p_sweep && p_flow_shape(lo, nsteps) && p_msteps(lo) == 4 && lo->lane_elems == 0 &&
         lo->nstages == 5 && nsteps <= kPSMaxSteps;
}

// Scratch and control words of a dataflow launch over `items` work items whose last block has
// nT tiles (the estimate's), with nb - 1 intermediate order-(N+1) fields and partial rows.
int p_flow_bufs(dg_plan* lo, const dg_plan* hi, uint64_t tag, int m, int W, int nsteps,
                int64_t items, int64_t items_cap, int64_t nT, int64_t nT_cap, int nb, double* w,
                bool eta, int64_t* idx, double* value, int64_t* nonfinite, hipStream_t st,
                PFlowBufs* b) {
  if (const int rc = sweep_watchdog(lo)) return rc;
  const int64_t kcap = lo->K_cap * lo->batch;
  const size_t sync_bytes =
      (sizeof(uint32_t) * size_t(sweep_sync_words() + items_cap) + 255) & ~size_t(255);
  const int64_t field_hi = lo->ktot * hi->NP;
  const size_t fcap = sizeof(double) * size_t(kcap) * size_t(hi->NP);
  const int nparts = eta ? nb - 1 : 0;
  const size_t data_bytes = fcap * size_t(nb - 1) + sizeof(double) * size_t(kcap) * size_t(nparts) +
                            (idx ? 16 * size_t(nT_cap) : 0);
  char* data = nullptr;
  if (const int rc = sweep_scratch(lo, sync_bytes, data_bytes, st, &data)) return rc;
  // the take counter numbers launches by items per launch, the refine's arrival counter by
  // the last block's tiles: another shape (or the jump sweep on this region) starts afresh
  const uint64_t sig = uint64_t(items) * 1000003u ^ (tag << 56) ^ (uint64_t(m) << 48) ^
                       (uint64_t(W) << 40) ^ (uint64_t(nsteps) << 32) ^ uint64_t(nT);
  if (lo->sweep_items != items || lo->sweep_sig != sig) {
    HIP_TRY(hipMemsetAsync(lo->d_sweep, 0, sync_bytes, st));
    lo->sweep_items = items;
    lo->sweep_sig = sig;
  }
  double* fld = reinterpret_cast<double*>(data);
  *b = PFlowBufs{};
  b->W[0] = w;
  for (int k = 1; k < nb; ++k) b->W[k] = fld + field_hi * (k - 1);
  b->W[nb] = w;
  double* rest = fld + field_hi * (nb - 1);
  b->part = nparts ? rest : nullptr;
  b->sync = static_cast<uint32_t*>(lo->d_sweep);
  b->am_idx = idx;
  b->am_val = value;
  b->am_nf = nonfinite;
  b->am_pv = idx ? rest + lo->ktot * nparts : nullptr;
  b->am_pi = idx ? reinterpret_cast<int64_t*>(b->am_pv + nT) : nullptr;
  return DG_OK;
}

// dg_lserk4_sweep_p's one dataflow launch (k_psweep).  Snapshot 0 holds u^0.
int psweep(dg_plan* lo, const dg_plan* hi, const double* P, double* snapshots, double* w,
           const double* tn, double dt, int nsteps, double* eta, int mode, int64_t* idx,
           double* value, int64_t* nonfinite, hipStream_t st) {
  const int m = 4, nb = nsteps / m, W = lo->p_tile_width;
  const int64_t TE = int64_t(kBlock) * W - 10 * m;
  const int64_t nT = (lo->ktot + TE - 1) / TE;
  const int64_t nT_cap = (lo->K_cap * lo->batch + TE - 1) / TE;
  PFlowBufs b;
  if (const int rc = p_flow_bufs(lo, hi, 0x5b, m, W, nsteps, 2 * int64_t(nb) * nT,
                                 2 * int64_t(nb) * nT_cap, nT, nT_cap, nb, w, eta != nullptr, idx,
                                 value, nonfinite, st, &b))
    return rc;
  int rc = DG_OK;
  switch (lo->NP) {
#define DG_PSWEEP_CASE(NPLV)                                                                 \
    case NPLV: {                                                                             \
      PrEO<NPLV> pr;                                                                         \
      if (!make_prolong_eo<NPLV>(P, &pr))                                                    \
        return fail(DG_ERR_ARG, "P does not commute with the node reversal (symmetric nodes)"); \
      if (W == 2)                                                                            \
        rc = launch_psweep<NPLV, 2, 4>(lo, hi, pr, b, snapshots, eta, mode, tn, dt, nsteps, st); \
      else                                                                                   \
        rc = launch_psweep<NPLV, 1, 4>(lo, hi, pr, b, snapshots, eta, mode, tn, dt, nsteps, st); \
    } break;
    DG_PSWEEP_CASE(2) DG_PSWEEP_CASE(3) DG_PSWEEP_CASE(4) DG_PSWEEP_CASE(5)
    DG_PSWEEP_CASE(6) DG_PSWEEP_CASE(7) DG_PSWEEP_CASE(8)
#undef DG_PSWEEP_CASE
    default: return fail(DG_ERR_ARG, "the p-estimate supports N <= 7");
  }
  return rc;
}

int adj_p_impl(dg_plan* lo, dg_plan* hi, const double* P, double* w, const double* snapshots,
               double t0, double dt, int nsteps, double* eta, int flags, int64_t* idx,
               double* value, int64_t* nonfinite, void* stream) {
  if (!lo || !hi || !P || !w || !snapshots) return fail(DG_ERR_ARG, "null argument");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (flags & ~(DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS | DG_ADJ_P_TERMINAL_PROLONG))
    return fail(DG_ERR_ARG, "unknown flags");
  bool term = (flags & DG_ADJ_P_TERMINAL_PROLONG) != 0;
  if (int rc = check_pair(lo, hi)) return rc;
  if (lo->NP > 8) return fail(DG_ERR_ARG, "the p-estimate supports N <= 7");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (eta != nullptr && nsteps == 0 && (flags & DG_ADJ_ETA_ASSIGN))
    HIP_TRY(hipMemsetAsync(eta, 0, sizeof(double) * lo->ktot, st));
  const int64_t field_lo = lo->ktot * lo->NP, field_hi = hi->ktot * hi->NP;
  if (term && (nsteps == 0 || p_horner() == 0)) {
    // the round-3 kernel (and an empty sweep) take the terminal weight from w: form it first
    if (const int rc = dg_prolong(lo, hi, P, snapshots + int64_t(nsteps) * field_lo, w, stream))
      return rc;
    term = false;
  }
  std::vector<double> tn(size_t(nsteps) + 1);  // time = time + dt, as the forward sweep
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  if (p_flow_shape(lo, nsteps)) {
    const int mode = eta ? (kEtaOn | ((flags & DG_ADJ_ETA_ASSIGN) ? kEtaAssign : 0) |
                            ((flags & DG_ADJ_ETA_ABS) ? kEtaAbs : 0))
                         : 0;
    return adjp_flow(lo, hi, P, w, snapshots, tn.data(), dt, nsteps, eta, mode, term, idx, value,
                     nonfinite, st);
  }
  if (nsteps > 0) {
    int launches = 0;
    for (int n = nsteps; n > 0; n -= chunk_p(lo, n)) ++launches;
    int l = 0;
    const double* in = w;
    for (int n = nsteps; n > 0; ++l) {  // this launch covers steps n-m .. n-1
      const int m = chunk_p(lo, n);
      const int n0 = n - m;
      double* out = (l == launches - 1 && launches > 1)
                        ? w : ((l % 2 == 0) ? hi->d_scratch : hi->d_scratch2);
      const int em = ((l == 0 && (flags & DG_ADJ_ETA_ASSIGN)) ? kEtaAssign : 0) |
                     ((n0 == 0 && (flags & DG_ADJ_ETA_ABS)) ? kEtaAbs : 0);
      const double* snap = snapshots + int64_t(n0) * field_lo;
      int rc = DG_OK;
      switch (lo->NP) {
#define DG_ADJP_CASE(NPLV)                                                                  \
        case NPLV: {                                                                        \
          PrEO<NPLV> pr;                                                                    \
          if (!make_prolong_eo<NPLV>(P, &pr))                                               \
            return fail(DG_ERR_ARG, "P does not commute with the node reversal (symmetric nodes)"); \
          rc = launch_adj_p_t<NPLV>(lo, hi, pr, m, in, out, snap, eta, em, &tn[n0], dt, st,  \
                                    term && l == 0);                                        \
        } break;
        DG_ADJP_CASE(2) DG_ADJP_CASE(3) DG_ADJP_CASE(4) DG_ADJP_CASE(5)
        DG_ADJP_CASE(6) DG_ADJP_CASE(7) DG_ADJP_CASE(8)
#undef DG_ADJP_CASE
        default: return fail(DG_ERR_ARG, "the p-estimate supports N <= 7");
      }
      if (rc) return rc;
      in = out;
      n = n0;
    }
    if (in != w)  // a one-launch sweep went through scratch
      HIP_TRY(hipMemcpyAsync(w, in, sizeof(double) * field_hi, hipMemcpyDeviceToDevice, st));
  }
  return idx ? dg_argmax_ex(lo, eta, lo->ktot, 1, idx, value, nonfinite, stream) : DG_OK;
}

}  // namespace

extern "C" {

int dg_prolong(const dg_plan* lo, const dg_plan* hi, const double* P, const double* u,
               double* u_hi, void* stream) {
  if (!lo || !hi || !P || !u || !u_hi) return fail(DG_ERR_ARG, "null argument");
  if (hi->NP != lo->NP + 1 || hi->ktot != lo->ktot)
    return fail(DG_ERR_ARG, "the enriched plan must have order N+1 and the same elements");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc = DG_OK;
  switch (lo->NP) {
#define DG_PROLONG_CASE(NPLV)                                                               \
    case NPLV: {                                                                            \
      PrEO<NPLV> pr;                                                                        \
      if (!make_prolong_eo<NPLV>(P, &pr))                                                   \
        return fail(DG_ERR_ARG, "P does not commute with the node reversal (symmetric nodes)"); \
      hipLaunchKernelGGL((k_prolong<NPLV>), dim3(grid_for(lo->ktot, kBlock)), dim3(kBlock), 0, \
                         st, u, u_hi, pr, lo->ktot);                                        \
      HIP_TRY(hipGetLastError());                                                           \
    } break;
    DG_PROLONG_CASE(2) DG_PROLONG_CASE(3) DG_PROLONG_CASE(4) DG_PROLONG_CASE(5)
    DG_PROLONG_CASE(6) DG_PROLONG_CASE(7) DG_PROLONG_CASE(8)
#undef DG_PROLONG_CASE
    default: return fail(DG_ERR_ARG, "the p-estimate supports N <= 7");
  }
  return rc;
}

int dg_lserk4_adj_p(dg_plan* lo, dg_plan* hi, const double* P, double* w, const double* snapshots,
                    double t0, double dt, int nsteps, double* eta, int flags, void* stream) {
  return adj_p_impl(lo, hi, P, w, snapshots, t0, dt, nsteps, eta, flags, nullptr, nullptr,
                    nullptr, stream);
}

int dg_lserk4_adj_p_refine(dg_plan* lo, dg_plan* hi, const double* P, double* w,
                           const double* snapshots, double t0, double dt, int nsteps,
                           double* eta, int flags, int64_t* idx, double* value,
                           int64_t* nonfinite_count, void* stream) {
  if (!idx || !eta) return fail(DG_ERR_ARG, "null argument (the refine decision needs eta)");
  return adj_p_impl(lo, hi, P, w, snapshots, t0, dt, nsteps, eta, flags, idx, value,
                    nonfinite_count, stream);
}

int dg_plan_query_p_flow(const dg_plan* lo, int nsteps, int* out) {
  if (!lo || !out) return fail(DG_ERR_ARG, "null argument");
  *out = p_flow_shape(lo, nsteps) ? 1 : 0;
  return DG_OK;
}

int dg_plan_query_p_sweep(const dg_plan* lo, int nsteps, int* out) {
  if (!lo || !out) return fail(DG_ERR_ARG, "null argument");
  *out = p_sweep_shape(lo, nsteps) ? 1 : 0;
  return DG_OK;
}

int dg_plan_query_p_trace(const dg_plan* lo, int nsteps, int64_t out[3]) {
  if (!lo || !out) return fail(DG_ERR_ARG, "null argument");
  // work items of each launch (k_adjp_flow: blocks x tiles; k_psweep: twice, forward and
  // estimate blocks), as adjp_flow / psweep size them
  const int W = lo->p_tile_width;
  out[0] = out[1] = 0;
  if (p_flow_shape(lo, nsteps)) {
    const int m = p_msteps(lo);
    const int64_t TE = int64_t(kBlock) * W - 10 * m;
    out[0] = int64_t(nsteps / m) * ((lo->ktot + TE - 1) / TE);
  }
  if (p_sweep_shape(lo, nsteps)) {
    const int64_t TE = int64_t(kBlock) * W - 10 * 4;
    out[1] = 2 * int64_t(nsteps / 4) * ((lo->ktot + TE - 1) / TE);
  }
  out[2] = 8;  // trace words per item
  return DG_OK;
}

int dg_lserk4_sweep_p(dg_plan* lo, dg_plan* hi, const double* P, double* snapshots, double* w,
                      double t0, double dt, int nsteps, double* eta, int flags, int64_t* idx,
                      double* value, int64_t* nonfinite_count, void* stream) {
  if (!lo || !hi || !P || !snapshots || !w) return fail(DG_ERR_ARG, "null argument");
  if (idx && !eta) return fail(DG_ERR_ARG, "the refine decision needs eta");
  if (nsteps < 0) return fail(DG_ERR_ARG, "nsteps < 0");
  if (flags & ~(DG_ADJ_ETA_ASSIGN | DG_ADJ_ETA_ABS))
    return fail(DG_ERR_ARG, "unknown flags (the terminal weight is always P u^nsteps)");
  if (int rc = check_pair(lo, hi)) return rc;
  if (lo->NP > 8) return fail(DG_ERR_ARG, "the p-estimate supports N <= 7");
  if (!p_sweep_shape(lo, nsteps)) {
    // the launch chains: the snapshot forward in place from snapshot 0 -- on the stage-loop
    // workgroup tiles at 4 steps per launch, the dataflow launch's forward blocks, so that the
    // result does not depend on whether nsteps fits that launch -- then the estimate
    const int ms = lo->msteps, sp = lo->snap_pairs, le = lo->lane_elems;
    lo->msteps = 4;
    lo->snap_pairs = 0;
    lo->lane_elems = 0;
    const int rf = dg_lserk4_fwd_ex(lo, snapshots, t0, dt, nsteps, snapshots, nullptr, stream);
    lo->msteps = ms;
    lo->snap_pairs = sp;
    lo->lane_elems = le;
    if (rf) return rf;
    return adj_p_impl(lo, hi, P, w, snapshots, t0, dt, nsteps, eta,
                      flags | DG_ADJ_P_TERMINAL_PROLONG, idx, value, nonfinite_count, stream);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::vector<double> tn(size_t(nsteps) + 1);  // time = time + dt (One_code.mlx:139)
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  const int mode = eta ? (kEtaOn | ((flags & DG_ADJ_ETA_ASSIGN) ? kEtaAssign : 0) |
                          ((flags & DG_ADJ_ETA_ABS) ? kEtaAbs : 0))
                       : 0;
  return psweep(lo, hi, P, snapshots, w, tn.data(), dt, nsteps, eta, mode, idx, value,
                nonfinite_count, st);
}

}  // extern "C"
