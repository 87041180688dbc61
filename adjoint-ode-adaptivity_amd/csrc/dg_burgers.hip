// dg_burgers.hip — the nonlinear-flux / per-stage-limiter path (BASELINE config 3,
// SURVEY §8(f)1): SlopeLimitN (utils/SlopeLimitN.m:1-33, SlopeLimitLin.m, minmod.m) applied
// after every LSERK4 stage update (utils/One_code.mlx:135-136) and, optionally, the
// build-defined Burgers-type flux f(u) = a*u^2/2 with AdvecRHS1D's central-flux structure
// (utils/AdvecRHS1D.m:9-19 with a*u -> a*f(u); CPU statement: oracle/burgers.py).
//
//   k_step_nl<NP,BURG,LIM,UNI,MS>  MS fused limited steps per launch.  Same tile scheme as
//       k_step (one element per lane, 256-element tiles, state in VGPRs, faces exchanged
//       through LDS); the limiter adds one cell-average exchange per stage, so the
//       dependency cone is 2 elements per stage (1 without the limiter).
//   k_adj_nl<NP,BURG,LIM,UNI>  one reverse step per launch: it recomputes the step's 5
//       stages from u^n in registers (keeping each stage input and the limiter's decision:
//       troubled or not, and which minmod argument was active), then runs the exact
//       transpose of the stages' tangent — the limiter with its decisions frozen, the flux
//       Jacobian diag(f'(u)) = diag(a*u) at the recomputed stage inputs — and accumulates
//       the dual-weighted jump residual of u^{n+1} into eta.
//   k_rhs_nl<NP>  the Burgers RHS for parity tests.
//
// Limiter arithmetic.  On a troubled cell SlopeLimitN replaces u by
//   y_i = v + (x_i - x0) m,   m = minmod(ux(1), (v+ - v)/h, (v - v-)/h)   (SlopeLimitLin.m:10-18)
// and x_i - x0 = h r_i / 2 for the LGL nodes, so with hm = h*m
//   y_i = v + (r_i / 2) hm,   hm = minmod(2 (Dr V)(1,1:2) uh(1:2), v+ - v, v - v-)
// (h > 0 scales all three arguments alike): no mesh coordinates are needed, on any mesh.
#include "dg_common.h"

namespace {
using namespace dgk;

// Limiter constants in even/odd coordinates (host: make_lim_eo).  The LGL nodes are
// symmetric, so row 1 of invV (P0) is even, row 2 (P1) odd and r odd: the parts that
// vanish in exact arithmetic (the odd part of row 1, the even part of row 2, the even part
// of r) are dropped; dg_plan_set_physics checks that they are below 1e-13.
template <int NP> struct LimEO {
  static constexpr int NE = (NP + 1) / 2, NO = NP / 2;
  double a0e[NE];           // cell average V(1,1) uh(1), uh(1) = sum_j invV(1,j) v_j  (SlopeLimitN.m:9)
  double a1o[NO];           // uh(2) = sum_j invV(2,j) v_j = a1o.o             (SlopeLimitN.m:28)
  double dv0, dv1;          // h ux(1) = 2 (Dr*ul)(1) = dv0 avg + dv1 uh(2)  (SlopeLimitLin.m:16)
  double rco[NO];           // r_i / 2, odd part: y = v + r/2 hm
  int32_t every;            // SlopeLimit1 (SlopeLimit1.m:21): every cell limited, no test
};

// minmod (utils/minmod.m:6-12) of three values and which one it returned: 1..3, or 0 when
// the signs differ (result 0).  Ties go to the first argument (min keeps the first).
__device__ __forceinline__ double minmod_br(double a, double b, double c, int& br) {
  const bool pos = a > 0.0 && b > 0.0 && c > 0.0;
  const bool neg = a < 0.0 && b < 0.0 && c < 0.0;
  br = 0;
  if (!pos && !neg) return 0.0;
  double m = fabs(a);
  br = 1;
  if (fabs(b) < m) {
    m = fabs(b);
    br = 2;
  }
  if (fabs(c) < m) {
    m = fabs(c);
    br = 3;
  }
  return pos ? m : -m;
}

// The troubled-cell test of SlopeLimitN.m:21-23.  Both minmods share the neighbour
// differences b = v - v-, c = v+ - v; with all three arguments of one sign minmod is the
// argument of least magnitude (minmod.m:9-11: s*min|.|), else 0.  Written as selects on
// magnitude compares (abs is a free operand modifier): no fmin/fmax, whose IEEE-mode
// operand canonicalisation costs two extra VALU ops each, and no branches.  On ties the two
// candidates are equal, so the pick is the same value s*min|.| gives; a NaN fails every
// sign test and yields 0, as in minmod.
__device__ __forceinline__ bool troubled(double v, double vm, double vp, double u0, double uN) {
  const double b = v - vm, c = vp - v;
  const bool bcp = b > 0.0 && c > 0.0, bcn = b < 0.0 && c < 0.0;
  const double bc = fabs(b) < fabs(c) ? b : c;
  const double a1 = v - u0, a2 = uN - v;
  const double s1 = fabs(a1) < fabs(bc) ? a1 : bc;
  const double s2 = fabs(a2) < fabs(bc) ? a2 : bc;
  const double m1 = ((bcp && a1 > 0.0) || (bcn && a1 < 0.0)) ? s1 : 0.0;
  const double m2 = ((bcp && a2 > 0.0) || (bcn && a2 < 0.0)) ? s2 : 0.0;
  return fabs((v - m1) - u0) > 1.0e-8 || fabs((v + m2) - uN) > 1.0e-8;
}

// Flux values divided by a, in even/odd coordinates: f = u (linear) or u^2/2 (Burgers):
//   fe_k = (f_k + f_{N-k})/2 = (e^2 + o^2)/2,  fo_k = (f_k - f_{N-k})/2 = e o.
// HQ (Burgers only): fe is returned doubled, for a Qoe the host pre-halved -- halving is
// exact, so (Qoe/2) (2 fe) rounds exactly as Qoe fe, and a face value fe_0 + fo_0 becomes
// fma(0.5, 2 fe_0, fo_0), the same number: NE multiplies fewer per stage, bit-identical.
template <int NP, bool BURG, bool HQ = false>
__device__ __forceinline__ void flux_eo(const double* ev, const double* od, double* fe,
                                        double* fo) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  static_assert(BURG || !HQ, "HQ is the Burgers flux's option");
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    fe[k] = BURG ? (HQ ? fma(ev[k], ev[k], od[k] * od[k])
                       : 0.5 * fma(ev[k], ev[k], od[k] * od[k]))
                 : ev[k];
    fo[k] = BURG ? ev[k] * od[k] : od[k];
  }
  if constexpr (NE > NO) fe[NO] = BURG ? (HQ ? ev[NO] * ev[NO] : 0.5 * ev[NO] * ev[NO]) : ev[NO];
}

// Exchange arrays in LDS (doubles, each padded by one slot on the left): two
// double-buffered face pairs [0, 4(T+2)), cell averages [4(T+2), 5(T+2)), the adjoint's
// limiter contributions to the left / right neighbour [5(T+2), 7(T+2)), the indicator's
// face values of u^{n+1} [7(T+2), 9(T+2)) (exchanged with the first reverse stage's).
template <int NP, int W = 1> struct NLGeo {
  static constexpr int T = kBlock * W;
  static constexpr int FA = 4 * (T + 2), CL = 5 * (T + 2), CR = 6 * (T + 2);
  static constexpr int IL = 7 * (T + 2), IR = 8 * (T + 2);
  static constexpr int kEx = 9 * (T + 2);
  static constexpr int kTileD = T * NP + 2;
  static constexpr int kLds = kTileD > kEx ? kTileD : kEx;  // boundary constants follow
};

// One LSERK4 stage s of the lane's element:  r = A_s r + dt RHS(u);  v = u + B_s r;
// u = SlopeLimitN(v) if LIM.  Returns the limiter's decision: 0 if the cell is not
// troubled, else 4 | (the active minmod argument, 1..3).  iin: LDS slot of the stage's
// inflow flux f(uin).  Barriers: one (faces), two with the limiter (cell averages).
//
// Metric: the operator constants carry dt (and 2/h on uniform meshes).  On non-uniform
// meshes the low-storage residual is kept divided by the element's 2/h = sc (r' = r / sc:
// r' = A_s r' + dt L u), so the stage is the uniform one except for the update
// v = u + (B_s sc) r' -- no per-node metric multiplies.
//
// KNOWN: the decisions come from the forward sweep's record `kc` (this stage's 3 bits)
// instead of the troubled-cell test, and `any` (workgroup-uniform: some lane of the tile is
// troubled in this stage) gates the cell-average exchange: a stage without a troubled cell
// in the tile runs no limiter work and no second barrier.
template <int NP, bool BURG, bool LIM, bool UNI, bool EDGE, bool KNOWN, int W, bool HQ = false>
__device__ __forceinline__ int nl_stage(double* __restrict__ lds, int el, int s, int par, int iin,
                                        const Elem& E, double sc, const EOArgs<NP>& op,
                                        const LimEO<NP>& lc, const LimEO<NP>& lk, double* ev,
                                        double* od, double* re, double* ro, int kc = 0,
                                        bool any = true) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, T = kBlock * W;
  constexpr int FA = NLGeo<NP, W>::FA;
  // par: face buffer, alternating over consecutive stages (across steps too: without the
  // limiter no barrier separates a step's last face reads from the next step's writes)
  const int fL = par * 2 * (T + 2), fR = fL + (T + 2);
  double fe[NE], fo[NO];
  flux_eo<NP, BURG, HQ>(ev, od, fe, fo);
  const double f0 = HQ ? fma(0.5, fe[0], fo[0]) : fe[0] + fo[0];
  const double fN = HQ ? fma(0.5, fe[0], -fo[0]) : fe[0] - fo[0];
  lds[fL + el + 1] = f0;
  lds[fR + el + 1] = fN;
  __builtin_amdgcn_sched_barrier(0);
  double pe[NE], po[NO];  // volume term + the carry A_s r'
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    double t = (s > 0) ? RK<5>::A(s) * re[k] : op.Qeo[k * NO] * fo[0];
#pragma unroll
    for (int j = (s > 0) ? 0 : 1; j < NO; ++j) t = fma(op.Qeo[k * NO + j], fo[j], t);
    pe[k] = t;
  }
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    double t = (s > 0) ? RK<5>::A(s) * ro[k] : op.Qoe[k * NE] * fe[0];
#pragma unroll
    for (int j = (s > 0) ? 0 : 1; j < NE; ++j) t = fma(op.Qoe[k * NE + j], fe[j], t);
    po[k] = t;
  }
#pragma unroll
  for (int k = 0; k < NE; ++k) pin(pe[k]);
#pragma unroll
  for (int k = 0; k < NO; ++k) pin(po[k]);
  __syncthreads();
  // Neighbour fluxes: left element's right face, right element's left face; a
  // trajectory's first element reads the inflow flux, its last one its own face (du1 = 0).
  const int iL = EDGE && E.first ? iin : fR + el;
  const int iR = EDGE && E.last ? fR + el + 1 : fL + el + 2;
  const double du0 = f0 - lds[iL];
  const double du1 = fN - lds[iR];
  const double dlt = du0 - du1, sig = du0 + du1;
  const double bs = UNI ? RK<5>::B(s) : RK<5>::B(s) * sc;
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    re[k] = fma(op.le[k], dlt, pe[k]);
    ev[k] = fma(bs, re[k], ev[k]);
  }
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    ro[k] = fma(op.lo[k], sig, po[k]);
    od[k] = fma(bs, ro[k], od[k]);
  }
  if constexpr (!LIM) {
    return 0;
  } else {
    if constexpr (KNOWN) {
      if (!any) return 0;  // workgroup-uniform: no troubled cell in the tile this stage
    }
    double avg = lc.a0e[0] * ev[0];
#pragma unroll
    for (int k = 1; k < NE; ++k) avg = fma(lc.a0e[k], ev[k], avg);
    lds[FA + el + 1] = avg;
    __syncthreads();
    // Neighbour averages, replicated at a trajectory's ends (SlopeLimitN.m:18).
    const double am = lds[EDGE && E.first ? FA + el + 1 : FA + el];
    const double ap = lds[EDGE && E.last ? FA + el + 1 : FA + el + 2];
    double uh1 = 0.0;
    int br;
    double hm;
    if constexpr (KNOWN) {
      if (!(kc & 4)) return 0;
      uh1 = lc.a1o[0] * od[0];
#pragma unroll
      for (int k = 1; k < NO; ++k) uh1 = fma(lc.a1o[k], od[k], uh1);
      // the recorded active minmod argument IS the minmod value (minmod.m:9-11: the
      // argument of least magnitude, all arguments of one sign)
      br = kc & 3;
      const double a1 = fma(lc.dv0, avg, lc.dv1 * uh1);
      hm = br == 1 ? a1 : (br == 2 ? ap - avg : (br == 3 ? avg - am : 0.0));
    } else {
      // (the test runs unconditionally: a branch on `every` only splits the code)
      if (!(troubled(avg, am, ap, ev[0] + od[0], ev[0] - od[0]) | (lc.every != 0))) return 0;
      uh1 = lk.a1o[0] * od[0];
#pragma unroll
      for (int k = 1; k < NO; ++k) uh1 = fma(lk.a1o[k], od[k], uh1);
      hm = minmod_br(fma(lk.dv0, avg, lk.dv1 * uh1), ap - avg, avg - am, br);
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) ev[k] = avg;
#pragma unroll
    for (int k = 0; k < NO; ++k) od[k] = lk.rco[k] * hm;
    return 4 | br;
  }
}

// Interior elements [H, T-H) of the tile to LDS (element-major, nodal); dual = adjoint
// coordinates (w_k = (we + wo)/2, w_{N-k} = (we - wo)/2).
template <int NP, int H, int W>
__device__ __forceinline__ void put_interior(double* __restrict__ lds, const double* ev,
                                             const double* od, bool dual) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1, T = kBlock * W;
  const int el = threadIdx.x;
  if (el >= H && el < T - H) {
    double* o = lds + (el - H) * NP;
    if (dual) {
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        o[k] = 0.5 * (ev[k] + od[k]);
        o[N - k] = 0.5 * (ev[k] - od[k]);
      }
      if constexpr (NE > NO) o[NO] = ev[NO];
    } else {
      from_eo<NP>(ev, od, o);
    }
  }
}

// ---------------------------------------------------------------------------
// Forward: MS limited steps per launch.
// ---------------------------------------------------------------------------
template <int NP, int MS> struct NLStepArgs {
  EOArgs<NP> op;
  LimEO<NP> lc;
  double sc;           // dt (non-uniform meshes multiply by scale[k]; uniform: folded in op)
  double fin[MS * 5];  // inflow flux f(uin) at each stage time
  int64_t ktot;
  int64_t stride;      // doubles between consecutive snapshots
  int32_t K;
  int32_t xcd;
};

template <bool LIM> constexpr int cone_per_stage() { return LIM ? 2 : 1; }

// Tile widths of the config-3 kernels: workgroups of 256*W lanes own tiles of 256*W
// elements.  Measured at K = 2^22 (bench.py --config 3): the forward (64 VGPRs, 8 waves per
// SIMD) gains from 512-element tiles (halo 4 % instead of 8 %: 101 -> 93 us per step with the
// SGPR cap); the adjoint (117 VGPRs, 4 waves per SIMD) loses (145 -> 151 us): with two
// 8-wave workgroups per CU each barrier stalls half the CU's waves.
constexpr int kNLStepW = 2, kNLAdjW = 1;

template <int NP, bool BURG, bool LIM, bool UNI, int MS>
__global__ __launch_bounds__(kBlock * kNLStepW) DG_NL_STEP_ATTR void k_step_nl(const double* __restrict__ uin,
                                                    double* __restrict__ snap,
                                                    double* __restrict__ last,
                                                    const double* __restrict__ scale,
                                                    uint16_t* __restrict__ codes,
                                                    NLStepArgs<NP, MS> args);

template <int NP, bool BURG, bool LIM, bool UNI, int MS, bool EDGE>
__device__ __forceinline__ void nl_step_tile(double* __restrict__ lds, int64_t tile,
                                             const double* __restrict__ uin,
                                             double* __restrict__ snap, double* __restrict__ last,
                                             const double* __restrict__ scale,
                                             uint16_t* __restrict__ codes,
                                             const NLStepArgs<NP, MS>& args) {
  constexpr int W = kNLStepW, T = kBlock * W, NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  constexpr int H = MS * 5 * cone_per_stage<LIM>();
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int CB = NLGeo<NP, W>::kLds;  // lds[CB + st*5 + s] = inflow flux of that stage
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;
  const int64_t o0 = tile * TE * NP;
  const int64_t rem = nd - o0;
  const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;

  const Elem E = elem_info<H, T, EDGE>(e0, lane, args.ktot, args.K);
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;  // issued with the tile's loads
  TileRegs<NP, W> pf;
  tile_issue<NP, W, EDGE>(uin, e0, nd, pf);
  tile_commit<NP, W>(pf, lds);
  if constexpr (EDGE) {
    // Lane-indexed read of fin straight from the kernel-argument segment (the args follow
    // the pointer arguments of k_step_nl; layout pinned by kernarg_tail), as in k_step.
    using SArgs = NLStepArgs<NP, MS>;
    const double* ka = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_step_nl<NP, BURG, LIM, UNI, MS>), SArgs>() +
        offsetof(SArgs, fin));
    if (lane < MS * 5) lds[CB + lane] = ka[lane];
  }
  __syncthreads();
  double ev[NE], od[NO];
  to_eo<NP>(lds + pf.off + lane * NP, ev, od);
  __syncthreads();  // the exchange arrays alias the staging image

  // The troubled-cell branch's constants are read from the kernel-argument segment where
  // they are used (scalar loads inside the rare branch) rather than kept live in SGPRs for
  // the whole tile: under the 80-SGPR cap that keeps every other constant unspilled.
  using SArgs = NLStepArgs<NP, MS>;
  const LimEO<NP>& lk = *reinterpret_cast<const LimEO<NP>*>(
      kernarg_tail<decltype(&k_step_nl<NP, BURG, LIM, UNI, MS>), SArgs>() + offsetof(SArgs, lc));
  double re[NE], ro[NO];
#pragma unroll
  for (int st = 0; st < MS; ++st) {
    int c15 = 0;  // this step's limiter decisions, 3 bits per stage
#pragma unroll
    for (int s = 0; s < 5; ++s)
      c15 |= nl_stage<NP, BURG, LIM, UNI, EDGE, false, W, BURG>(lds, lane, s, (st * 5 + s) & 1,
                                                          CB + st * 5 + s, E, sc, args.op, args.lc,
                                                          lk, ev, od, re, ro)
             << (3 * s);
    // The decision record for the adjoint (dg_lserk4_fwd_ex): one 16-bit word per element
    // and step, written by the lane that owns the element.
    if (LIM && codes != nullptr && E.valid) codes[st * args.ktot + E.e] = uint16_t(c15);
    if (snap != nullptr || st == MS - 1) {
      __syncthreads();  // the last stage's exchange reads are done before the image is rewritten
      put_interior<NP, H, W>(lds, ev, od, false);
      __syncthreads();
      if constexpr (EDGE) {
        if (snap != nullptr) store_run<T>(snap + st * args.stride, o0, count, lds);
        if (st == MS - 1 && last != nullptr) store_run<T>(last, o0, count, lds);
      } else {
        if (snap != nullptr) store_full<TE * NP, T>(snap + st * args.stride, o0, lds);
        if (st == MS - 1 && last != nullptr) store_full<TE * NP, T>(last, o0, lds);
      }
      if (st < MS - 1) __syncthreads();  // the next stage's exchange arrays alias the image
    }
  }
}

template <int NP, bool BURG, bool LIM, bool UNI, int MS>
__global__ __launch_bounds__(kBlock * kNLStepW) DG_NL_STEP_ATTR void k_step_nl(const double* __restrict__ uin,
                                                    double* __restrict__ snap,
                                                    double* __restrict__ last,
                                                    const double* __restrict__ scale,
                                                    uint16_t* __restrict__ codes,
                                                    NLStepArgs<NP, MS> args) {
  constexpr int T = kBlock * kNLStepW, H = MS * 5 * cone_per_stage<LIM>();
  __shared__ __attribute__((aligned(16))) double lds[NLGeo<NP, kNLStepW>::kLds + MS * 5];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  const int64_t e0 = tile * (T - 2 * H) - H;
  if (edge_tile(e0, T, args.ktot, args.K))
    nl_step_tile<NP, BURG, LIM, UNI, MS, true>(lds, tile, uin, snap, last, scale, codes, args);
  else
    nl_step_tile<NP, BURG, LIM, UNI, MS, false>(lds, tile, uin, snap, last, scale, codes, args);
}

// ---------------------------------------------------------------------------
// Adjoint: one reverse step per launch (w^{n+1} -> w^n), stages recomputed from u^n.
// ---------------------------------------------------------------------------
template <int NP> struct NLAdjArgs {
  EOArgs<NP> op;
  LimEO<NP> lc;
  double sc;
  double fin[6];   // inflow flux at the 5 stage times of step n, then at t_{n+1} (residual)
  double src;      // functional source coefficient of node n+1
  double qoe_h[EOArgs<NP>::NO * EOArgs<NP>::NE];  // Burgers: op.Qoe / 2 for the recompute (HQ)
  int64_t ktot;
  int32_t K;
  int32_t has_eta;  // kEta* bits
  int32_t xcd;
};

template <int NP, bool BURG, bool LIM, bool UNI, bool KNOWN>
__global__ __launch_bounds__(kBlock * kNLAdjW, kNLAdjMinWaves) void k_adj_nl(const double* __restrict__ win,
                                                   double* __restrict__ wout,
                                                   const double* __restrict__ snap,
                                                   double* __restrict__ eta,
                                                   const double* __restrict__ scale,
                                                   const uint16_t* __restrict__ codes,
                                                   int32_t* __restrict__ list,
                                                   int32_t* __restrict__ count,
                                                   NLAdjArgs<NP> args);

// One tile of the reverse step: the T elements from e0 on, of which lanes [H, H + nout)
// are outputs.  H is the dependency cone: 20 elements (10 stages of 2) in general, 10 (1 per
// stage) for a FAST tile, valid only when no cell of the tile is troubled in any stage of
// the step; a FAST tile finds that out from the decision record right after its loads and
// returns false, before any store, when it does not hold (the caller then recomputes its
// outputs on the wide cone).
template <int NP, bool BURG, bool LIM, bool UNI, bool KNOWN, bool EDGE, int H, bool FAST>
__device__ __forceinline__ bool nl_adj_tile(double* __restrict__ lds, int64_t e0, int nout,
                                            const double* __restrict__ win,
                                            double* __restrict__ wout,
                                            const double* __restrict__ snap,
                                            double* __restrict__ eta,
                                            const double* __restrict__ scale,
                                            const uint16_t* __restrict__ codes,
                                            const NLAdjArgs<NP>& args) {
  constexpr int W = kNLAdjW, T = kBlock * W, NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  static_assert(!FAST || KNOWN, "a FAST tile needs the decision record");
  static_assert(H > 0 && 2 * H < T, "tile geometry");
  constexpr int CB = NLGeo<NP, W>::kLds;  // lds[CB+s]: stage inflow flux; CB+5: residual's; CB+6: 0
  constexpr int CL = NLGeo<NP, W>::CL, CR = NLGeo<NP, W>::CR;
  const int lane = threadIdx.x;
  const int64_t nd = args.ktot * NP;

  // The decision record is loaded first, with the tiles, so its latency hides behind theirs.
  int kcode = 0;
  if constexpr (KNOWN) {
    const int64_t e = e0 + lane;
    kcode = (e >= 0 && e < args.ktot) ? int(codes[e]) : 0;
  }
  // the element's metric likewise
  Elem E = elem_info<H, T, EDGE>(e0, lane, args.ktot, args.K);
  E.valid = E.valid && lane < H + nout;
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;
  TileRegs<NP, W> pu, pw;
  tile_issue<NP, W, EDGE>(snap, e0, nd, pu);
  tile_issue<NP, W, EDGE>(win, e0, nd, pw);
  tile_commit<NP, W>(pu, lds);
  // KNOWN: bitwise OR of the tile's records (__syncthreads_or would only say "some
  // nonzero"), cleared here and OR-ed between the load phase's barriers
  __shared__ int wg_or;
  if (KNOWN && lane == 0) wg_or = 0;
  if constexpr (EDGE) {
    using AArgs = NLAdjArgs<NP>;  // the args follow the pointer arguments of k_adj_nl
    const double* ka = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_adj_nl<NP, BURG, LIM, UNI, KNOWN>), AArgs>() +
        offsetof(AArgs, fin));
    if (lane < 6) lds[CB + lane] = ka[lane];
    if (lane == 6) lds[CB + 6] = 0.0;
  }
  __syncthreads();
  double ev[NE], od[NO];
  to_eo<NP>(lds + pu.off + lane * NP, ev, od);
  if (KNOWN && kcode != 0) atomicOr(&wg_or, kcode);  // LDS atomic, rare lanes only
  __syncthreads();
  tile_commit<NP, W>(pw, lds);
  __syncthreads();
  double we[NE], wo[NO];  // the adjoint in dual even/odd coordinates
  {
    const double* w = lds + pw.off + lane * NP;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[k] = w[k] + w[N - k];
      wo[k] = w[k] - w[N - k];
    }
    if constexpr (NE > NO) we[NO] = w[NO];
  }
  __syncthreads();  // the exchange arrays alias the staging image

  // 1. Recompute the step's stages, keeping each stage's input and limiter decision.
  //    KNOWN: the decisions are the forward sweep's record; `wg` (the OR over the tile's
  //    lanes) says in which stages some cell of the tile is troubled at all -- in the
  //    others the limiter and its exchange are skipped, here and in the reverse pass.
  int wg = 0;
  if constexpr (KNOWN) wg = wg_or;  // the load phase's barriers ordered its init and ORs
  if constexpr (FAST) {
    if (wg != 0) return false;  // (workgroup-uniform) some cell is troubled: the wide cone
  }
  // The stage inputs u_s feed the Burgers flux Jacobian of the reverse pass.  Registers
  // hold u_2..u_4; u_1 goes to a lane-private LDS slot and u_0 = u^n is re-read from the
  // snapshot (L2-resident) at the end: 20 VGPRs fewer at the peak (5 waves per SIMD
  // instead of 4).
  constexpr int SE1 = CB + 8;  // lds[SE1 + k*T + lane]: u_1 in even/odd coordinates
  double se[5][NE], so[5][NO];
  int dcodes = 0;
  {
    // the recompute's operator: the Burgers even flux doubled against Qoe/2 (flux_eo HQ);
    // the reverse pass keeps Qoe
    EOArgs<NP> oph = args.op;
    if constexpr (BURG) {
#pragma unroll
      for (int k = 0; k < NO * NE; ++k) oph.Qoe[k] = args.qoe_h[k];
    }
    double re[NE], ro[NO];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      if (s >= 2) {
#pragma unroll
        for (int k = 0; k < NE; ++k) se[s][k] = ev[k];
#pragma unroll
        for (int k = 0; k < NO; ++k) so[s][k] = od[k];
      } else if (BURG && s == 1) {
#pragma unroll
        for (int k = 0; k < NE; ++k) lds[SE1 + k * T + lane] = ev[k];
#pragma unroll
        for (int k = 0; k < NO; ++k) lds[SE1 + (NE + k) * T + lane] = od[k];
      }
      const int c = nl_stage<NP, BURG, LIM, UNI, EDGE, KNOWN, W, BURG>(
          lds, lane, s, s & 1, CB + s, E, sc, oph, args.lc, args.lc, ev, od, re, ro,
          (kcode >> (3 * s)) & 7, ((wg >> (3 * s)) & 4) != 0);
      if constexpr (LIM) dcodes |= c << (3 * s);
    }
  }
  // (ev, od) = u^{n+1}.  2. Functional source w^{n+1} += src u^{n+1} (dual coordinates).
  if (args.src != 0.0) {
    const double s2 = 2.0 * args.src;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[k] = fma(s2, ev[k], we[k]);
      wo[k] = fma(s2, od[k], wo[k]);
    }
    if constexpr (NE > NO) we[NO] = fma(args.src, ev[NO], we[NO]);
  }
  // 3. Indicator: eta += dt sum_i w_i (LIFT Fscale du)_i at u^{n+1}, t_{n+1}.  The weights
  //    (le.we, lo.wo) are local; the neighbours' face fluxes of u^{n+1} travel with the
  //    first reverse stage's exchange below (one barrier fewer per step).
  double eacc = 0.0, ipe = 0.0, ipo = 0.0, uf0 = 0.0, ufN = 0.0;
  if (args.has_eta) {
    double fe[NE], fo[NO];
    flux_eo<NP, BURG>(ev, od, fe, fo);
    uf0 = fe[0] + fo[0];
    ufN = fe[0] - fo[0];
#pragma unroll
    for (int k = 0; k < NE; ++k) ipe = fma(args.op.le[k], we[k], ipe);
#pragma unroll
    for (int k = 0; k < NO; ++k) ipo = fma(args.op.lo[k], wo[k], ipo);
  }
  constexpr int IL = NLGeo<NP, W>::IL, IR = NLGeo<NP, W>::IR;

  // 4. Reverse stages s = 4..0 (forward: r = A_s r + dt L f(u); v = u + B_s r; u = Lim(v)):
  //      lv = Lim'(v)^T lu;  lr += B_s lv;  lu = lv + f'(u_s) (dt L^T lr);  lr = A_s lr.
  double un[NP];  // u_0 = u^n for the last reverse stage, re-read from the snapshot early
  double lre[NE], lro[NO];
#pragma unroll
  for (int k = 0; k < NE; ++k) lre[k] = 0.0;
#pragma unroll
  for (int k = 0; k < NO; ++k) lro[k] = 0.0;
#pragma unroll
  for (int ss = 0; ss < 5; ++ss) {
    const int s = 4 - ss;
    if (BURG && s == 2) {  // issue the re-read two stages ahead (u_4, u_3 are dead by now)
#pragma unroll
      for (int i = 0; i < NP; ++i) un[i] = E.inrange ? snap[E.e * NP + i] : 0.0;
    }
    if (LIM && (!KNOWN || ((wg >> (3 * s)) & 4))) {  // (workgroup-uniform)
      // Transposed limiter.  Troubled cell: y = v_avg + (r/2) hm, hm one of
      // {2 (Dr V)(1,:) uh(1:2), v+ - v, v - v-} (or 0): the cell's own nodal adjoint is
      // replaced by the branch-1 gradient, and avg-adjoints go to this cell (cs) and to the
      // left / right neighbour (cl / cr).  Every cell then adds the avg-adjoint it
      // receives times d avg / d v.
      const int code = (dcodes >> (3 * s)) & 7;
      double cs = 0.0, cl = 0.0, cr = 0.0;
      if (code & 4) {
        double ls = we[0];
#pragma unroll
        for (int k = 1; k < NE; ++k) ls += we[k];
        double mu = 0.0;  // adjoint of hm
#pragma unroll
        for (int k = 0; k < NO; ++k) mu = fma(args.lc.rco[k], wo[k], mu);
        const int br = code & 3;
        cs = ls;
        if (br == 2) {
          cs -= mu;
          cr = mu;
        }
        if (br == 3) {
          cs += mu;
          cl = -mu;
        }
        const double g = (br == 1) ? mu : 0.0;
        const double g0 = g * args.lc.dv0, g1 = g * args.lc.dv1;
#pragma unroll
        for (int k = 0; k < NE; ++k) we[k] = g0 * args.lc.a0e[k];
#pragma unroll
        for (int k = 0; k < NO; ++k) wo[k] = g1 * args.lc.a1o[k];
      }
      lds[CL + lane + 1] = cl;
      lds[CR + lane + 1] = cr;
      __syncthreads();
      // Received: the left neighbour's cr and the right neighbour's cl; at a trajectory's
      // ends the replicated neighbour average is the cell's own (SlopeLimitN.m:18).
      const double alpha = cs + lds[EDGE && E.first ? CL + lane + 1 : CR + lane] +
                           lds[EDGE && E.last ? CR + lane + 1 : CL + lane + 2];
#pragma unroll
      for (int k = 0; k < NE; ++k) we[k] = fma(alpha, args.lc.a0e[k], we[k]);
    }
    // Face buffers alternate starting with buffer 1: the recompute's last stage read
    // buffer 0 after its barrier, and no barrier separates it from this first write.
    const int f0 = ((ss + 1) & 1) * 2 * (T + 2), f1 = f0 + (T + 2);
    double qe[NE], qo[NO];
    double gd = 0.0, gs = 0.0;
    // transpose of v = u + (B_s sc) r' (nl_stage's metric folding): lr' += (B_s sc) lv
    const double bs = UNI ? RK<5>::B(s) : RK<5>::B(s) * sc;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      lre[k] = fma(bs, we[k], lre[k]);
      qe[k] = lre[k];
      gd = fma(args.op.le[k], qe[k], gd);
    }
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      lro[k] = fma(bs, wo[k], lro[k]);
      qo[k] = lro[k];
      gs = fma(args.op.lo[k], qo[k], gs);
    }
    const double g0 = gd + gs;  // adjoints of du0 and du1
    double g1 = gs - gd;
    if constexpr (EDGE) g1 = E.last ? 0.0 : g1;
    lds[f0 + lane + 1] = g0;
    lds[f1 + lane + 1] = g1;
    if (ss == 0 && args.has_eta) {  // the indicator's u^{n+1} faces ride along
      lds[IL + lane + 1] = uf0;
      lds[IR + lane + 1] = ufN;
    }
    __builtin_amdgcn_sched_barrier(0);
    double pe[NE], po[NO];  // transposed volume term: the adjoint of the flux values
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      double t = args.op.Qoe[j] * qo[0];
#pragma unroll
      for (int k = 1; k < NO; ++k) t = fma(args.op.Qoe[k * NE + j], qo[k], t);
      pe[j] = t;
    }
#pragma unroll
    for (int j = 0; j < NO; ++j) {
      double t = args.op.Qeo[j] * qe[0];
#pragma unroll
      for (int k = 1; k < NE; ++k) t = fma(args.op.Qeo[k * NO + j], qe[k], t);
      po[j] = t;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) lre[k] = RK<5>::A(s) * lre[k];
#pragma unroll
    for (int k = 0; k < NO; ++k) lro[k] = RK<5>::A(s) * lro[k];
#pragma unroll
    for (int k = 0; k < NE; ++k) pin(pe[k]);
#pragma unroll
    for (int k = 0; k < NO; ++k) pin(po[k]);
    __syncthreads();
    if (ss == 0 && args.has_eta) {
      // left neighbour's right face / right neighbour's left face of u^{n+1}; a
      // trajectory's first element reads the inflow flux at t_{n+1}, its last one its own
      // right face (du1 = 0)
      const double du0 = uf0 - lds[EDGE && E.first ? CB + 5 : IR + lane];
      const double du1 = ufN - lds[EDGE && E.last ? IR + lane + 1 : IL + lane + 2];
      eacc = fma(du0 - du1, ipe, (du0 + du1) * ipo);
      if constexpr (!UNI) eacc *= sc;
    }
    const double gl = lds[EDGE && E.first ? CB + 6 : f1 + lane];
    const double gr = lds[EDGE && E.last ? CB + 6 : f0 + lane + 2];
    pe[0] += (g0 + g1) - (gr + gl);
    po[0] += (g0 - g1) + (gr - gl);
    if constexpr (BURG) {  // f'(u) = u: the symmetric block [[e, o], [o, e]] per node pair
      double ue[NE], uo[NO];  // u_s (see the recompute)
      if (s >= 2) {
#pragma unroll
        for (int k = 0; k < NE; ++k) ue[k] = se[s][k];
#pragma unroll
        for (int k = 0; k < NO; ++k) uo[k] = so[s][k];
      } else if (s == 1) {
#pragma unroll
        for (int k = 0; k < NE; ++k) ue[k] = lds[SE1 + k * T + lane];
#pragma unroll
        for (int k = 0; k < NO; ++k) uo[k] = lds[SE1 + (NE + k) * T + lane];
      } else {
        to_eo<NP>(un, ue, uo);
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        const double e = ue[k], o = uo[k];
        we[k] = fma(e, pe[k], fma(o, po[k], we[k]));
        wo[k] = fma(o, pe[k], fma(e, po[k], wo[k]));
      }
      if constexpr (NE > NO) we[NO] = fma(ue[NO], pe[NO], we[NO]);
    } else {
#pragma unroll
      for (int k = 0; k < NE; ++k) we[k] += pe[k];
#pragma unroll
      for (int k = 0; k < NO; ++k) wo[k] += po[k];
    }
  }

  if (args.has_eta && E.valid) eta_update(eta, E.e, eacc, args.has_eta);
  // w^n: each lane stores its element straight from registers (the tile is latency-bound;
  // an LDS pass for wider stores costs two barriers and was 1.5 % slower)
  if (E.valid) {
    double* o = wout + E.e * NP;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      o[k] = 0.5 * (we[k] + wo[k]);
      o[N - k] = 0.5 * (we[k] - wo[k]);
    }
    if constexpr (NE > NO) o[NO] = we[NO];
  }
  return true;
}

template <int NP, bool BURG, bool LIM, bool UNI, bool KNOWN>
__global__ __launch_bounds__(kBlock * kNLAdjW, kNLAdjMinWaves) void k_adj_nl(const double* __restrict__ win,
                                                   double* __restrict__ wout,
                                                   const double* __restrict__ snap,
                                                   double* __restrict__ eta,
                                                   const double* __restrict__ scale,
                                                   const uint16_t* __restrict__ codes,
                                                   int32_t* __restrict__ list,
                                                   int32_t* __restrict__ count,
                                                   NLAdjArgs<NP> args) {
  // forward recompute and reverse sweep each widen the cone by one stage-cone per stage
  constexpr int T = kBlock * kNLAdjW, HW = 10 * cone_per_stage<LIM>();
  // With the decision record, tiles are laid out for the narrow cone (1 element per stage:
  // no troubled cell, the case of almost every tile); a tile with a troubled cell in its
  // range recomputes its outputs as two halves on the wide cone.  The results are the same
  // numbers either way: each output's value depends only on its cone.
  constexpr int H = KNOWN ? 10 : HW, TE = T - 2 * H, TH = TE / 2;
  static_assert(TE % 2 == 0 && TE > 0 && (!KNOWN || TH + 2 * HW <= T), "tile geometry");
  // boundary constants (8 slots), then the lane-private stage-1 input (Burgers only)
  __shared__ __attribute__((aligned(16)))
  double lds[NLGeo<NP, kNLAdjW>::kLds + 8 + (BURG ? T * NP : 0)];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  const int64_t e0 = tile * TE - H;
  bool done;
  if (edge_tile(e0, T, args.ktot, args.K))
    done = nl_adj_tile<NP, BURG, LIM, UNI, KNOWN, true, H, KNOWN>(lds, e0, TE, win, wout, snap,
                                                                   eta, scale, codes, args);
  else
    done = nl_adj_tile<NP, BURG, LIM, UNI, KNOWN, false, H, KNOWN>(lds, e0, TE, win, wout, snap,
                                                                    eta, scale, codes, args);
  if constexpr (KNOWN) {
    // a troubled tile goes on the list for k_adj_nl_wide (this step's count, zeroed per sweep)
    if (!done && threadIdx.x == 0) list[atomicAdd(count, 1)] = int32_t(tile);
  }
}

// The tiles k_adj_nl listed as troubled, each recomputed as two half tiles on the wide cone
// (20 elements of halo, 118 outputs each).  A separate launch so that neither kernel carries
// the other's registers (one kernel with both bodies spilled 69 VGPRs).  Grid-stride over
// the (tile, half) items -- almost always none.  Each step of a sweep has its own count
// (nl_adj zeroes them once per sweep), so nothing is reset here: an exit counter for a
// reset, one same-address atomic per workgroup, cost ~10 us per launch.  Same parameter list
// as k_adj_nl: the edge tiles read their constants at k_adj_nl's kernarg offsets.  4 waves
// per SIMD: at 5 the item loop's live kernel arguments spilled 20 VGPRs.
template <int NP, bool BURG, bool LIM, bool UNI>
__global__ __launch_bounds__(kBlock * kNLAdjW, 4) void k_adj_nl_wide(
    const double* __restrict__ win, double* __restrict__ wout, const double* __restrict__ snap,
    double* __restrict__ eta, const double* __restrict__ scale,
    const uint16_t* __restrict__ codes, int32_t* __restrict__ list, int32_t* __restrict__ count,
    NLAdjArgs<NP> args) {
  constexpr int T = kBlock * kNLAdjW, HW = 10 * cone_per_stage<LIM>(), TE = T - 20, TH = TE / 2;
  static_assert(TH % 2 == 0 && TH + 2 * HW <= T, "half-tile geometry");
  __shared__ __attribute__((aligned(16)))
  double lds[NLGeo<NP, kNLAdjW>::kLds + 8 + (BURG ? T * NP : 0)];
  const int n = *count;  // final: k_adj_nl has completed
  for (int i = blockIdx.x; i < 2 * n; i += gridDim.x) {
    if (i != int(blockIdx.x)) __syncthreads();  // the previous item's LDS reads are done
    const int64_t tile = list[i / 2];
    const int64_t e0 = tile * TE + (i & 1) * TH - HW;
    if (edge_tile(e0, T, args.ktot, args.K))
      nl_adj_tile<NP, BURG, LIM, UNI, true, true, HW, false>(lds, e0, TH, win, wout, snap, eta,
                                                             scale, codes, args);
    else
      nl_adj_tile<NP, BURG, LIM, UNI, true, false, HW, false>(lds, e0, TH, win, wout, snap, eta,
                                                              scale, codes, args);
  }
}

// ---------------------------------------------------------------------------
// Burgers RHS (parity entry point): one element per thread, global neighbour reads.
// ---------------------------------------------------------------------------
template <int NP>
__global__ __launch_bounds__(kBlock) void k_rhs_nl(const double* __restrict__ u,
                                                   double* __restrict__ rhs,
                                                   const double* __restrict__ scale,
                                                   OpArgs<NP> op, double s_uni, double fin,
                                                   int64_t ktot, int32_t K) {
  const int64_t e = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= ktot) return;
  const int32_t kl = int32_t(e % K);
  const bool first = (kl == 0), last = (kl == K - 1);
  double f[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const double v = u[e * NP + i];
    f[i] = 0.5 * v * v;
  }
  double fL = fin;
  if (!first) {
    const double v = u[(e - 1) * NP + NP - 1];
    fL = 0.5 * v * v;
  }
  const double du0 = f[0] - fL;
  double du1 = 0.0;
  if (!last) {
    const double v = u[(e + 1) * NP];
    du1 = f[NP - 1] - 0.5 * v * v;
  }
  const double s = scale ? scale[kl] : s_uni;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    double t = op.L0[i] * du0;
    t = fma(op.L1[i], du1, t);
#pragma unroll
    for (int j = 0; j < NP; ++j) t = fma(op.Dm[i * NP + j], f[j], t);
    rhs[e * NP + i] = s * t;
  }
}

__global__ __launch_bounds__(kBlock) void k_src_copy(const double* __restrict__ w,
                                                     const double* __restrict__ u, double c,
                                                     double* __restrict__ out, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = fma(c, u[i], w[i]);
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
template <int NP> LimEO<NP> make_lim_eo(const dg_plan* p) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  LimEO<NP> c;
  const double* i0 = p->invV;       // row 1 of invV
  const double* i1 = p->invV + NP;  // row 2
  for (int k = 0; k < NO; ++k) {
    c.a0e[k] = i0[k] + i0[N - k];
    c.a1o[k] = i1[k] - i1[N - k];
    c.rco[k] = 0.25 * (p->r[k] - p->r[N - k]);
  }
  if (NE > NO) {
    c.a0e[NO] = i0[NO];
  }
  const double V00 = p->V[0];  // V(1,1): the cell average is V(1,1) uh(1)
  for (int k = 0; k < NE; ++k) c.a0e[k] *= V00;
  double d0 = 0.0, d1 = 0.0;
  for (int l = 0; l < NP; ++l) {
    d0 += p->Dr[l] * p->V[l * NP + 0];
    d1 += p->Dr[l] * p->V[l * NP + 1];
  }
  c.dv0 = 2.0 * d0 / V00;  // uh(1) = avg / V(1,1)
  c.dv1 = 2.0 * d1;
  c.every = p->limiter == DG_LIMIT_PI1_EACH_STAGE;
  return c;
}

inline double flux_value(bool burg, double u) { return burg ? 0.5 * u * u : u; }

template <int NP, bool BURG, bool LIM, int MS>
int launch_step_nl(const dg_plan* p, const double* in, double* snap, double* last,
                   uint16_t* codes, const double* times, double dt, hipStream_t st) {
  NLStepArgs<NP, MS> a;
  // constants carry dt (and 2/h on uniform meshes); non-uniform meshes multiply the update
  // by the element's 2/h (nl_stage's metric folding)
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : dt, &a.op);
  if (BURG)  // the forward's nl_stage takes the Burgers fe doubled (flux_eo HQ)
    for (double& q : a.op.Qoe) q *= 0.5;
  a.lc = make_lim_eo<NP>(p);
  a.sc = 1.0;
  for (int m = 0; m < MS; ++m)
    for (int s = 0; s < 5; ++s)
      a.fin[m * 5 + s] = flux_value(BURG, inflow_value(p, times[m] + RK<5>::C(s) * dt));
  a.ktot = p->ktot;
  a.stride = p->ktot * NP;
  a.K = int32_t(p->K);
  a.xcd = p->xcd_order;
  constexpr int TE = kBlock * kNLStepW - 2 * MS * 5 * cone_per_stage<LIM>();
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_step_nl<NP, BURG, LIM, true, MS>), dim3(grid), dim3(kBlock * kNLStepW), 0, st, in,
                       snap, last, p->d_scale, codes, a);
  else
    hipLaunchKernelGGL((k_step_nl<NP, BURG, LIM, false, MS>), dim3(grid), dim3(kBlock * kNLStepW), 0, st,
                       in, snap, last, p->d_scale, codes, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP, bool BURG, bool LIM>
int launch_adj_nl(const dg_plan* p, const double* win, double* wout, const double* snap,
                  double* eta, int em, const uint16_t* codes, int32_t* count, double t_n,
                  double src, double dt, hipStream_t st) {
  NLAdjArgs<NP> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : dt, &a.op);  // see launch_step_nl
  for (int k = 0; k < EOArgs<NP>::NO * EOArgs<NP>::NE; ++k) a.qoe_h[k] = 0.5 * a.op.Qoe[k];
  a.lc = make_lim_eo<NP>(p);
  a.sc = 1.0;
  for (int s = 0; s < 5; ++s) a.fin[s] = flux_value(BURG, inflow_value(p, t_n + RK<5>::C(s) * dt));
  a.fin[5] = flux_value(BURG, inflow_value(p, t_n + dt));
  a.src = src;
  a.ktot = p->ktot;
  a.K = int32_t(p->K);
  a.has_eta = eta != nullptr ? (em | kEtaOn) : 0;
  a.xcd = p->xcd_order;
  // the recorded decisions are only kept with a limiter (without one there are none)
  const bool known = LIM && codes != nullptr;
  // tiles of the narrow cone with the record (k_adj_nl), else of the kernel's cone
  const int TE = kBlock * kNLAdjW - 20 * (known ? 1 : cone_per_stage<LIM>());
  const unsigned grid = grid_for(p->ktot, TE);
  int32_t* list = known ? p->d_nl_list : nullptr;
  if (known && (list == nullptr || count == nullptr || p->nl_list_tiles < int64_t(grid)))
    return fail(DG_ERR_ARG, "config-3 adjoint: tile list not sized (nl_adj)");
  if (p->uniform && known)
    hipLaunchKernelGGL((k_adj_nl<NP, BURG, LIM, true, true>), dim3(grid), dim3(kBlock * kNLAdjW), 0, st,
                       win, wout, snap, eta, p->d_scale, codes, list, count, a);
  else if (p->uniform)
    hipLaunchKernelGGL((k_adj_nl<NP, BURG, LIM, true, false>), dim3(grid), dim3(kBlock * kNLAdjW), 0, st,
                       win, wout, snap, eta, p->d_scale, codes, list, count, a);
  else if (known)
    hipLaunchKernelGGL((k_adj_nl<NP, BURG, LIM, false, true>), dim3(grid), dim3(kBlock * kNLAdjW), 0, st,
                       win, wout, snap, eta, p->d_scale, codes, list, count, a);
  else
    hipLaunchKernelGGL((k_adj_nl<NP, BURG, LIM, false, false>), dim3(grid), dim3(kBlock * kNLAdjW), 0, st,
                       win, wout, snap, eta, p->d_scale, codes, list, count, a);
  HIP_TRY(hipGetLastError());
  if (known) {
    const unsigned gw = std::min<unsigned>(grid, unsigned(p->cu_count));
    if (p->uniform)
      hipLaunchKernelGGL((k_adj_nl_wide<NP, BURG, LIM, true>), dim3(gw), dim3(kBlock * kNLAdjW), 0,
                         st, win, wout, snap, eta, p->d_scale, codes, list, count, a);
    else
      hipLaunchKernelGGL((k_adj_nl_wide<NP, BURG, LIM, false>), dim3(gw), dim3(kBlock * kNLAdjW),
                         0, st, win, wout, snap, eta, p->d_scale, codes, list, count, a);
    HIP_TRY(hipGetLastError());
  }
  return DG_OK;
}

// (flux, limiter) combinations: Burgers + limiter, Burgers alone, linear + limiter (the
// plain linear flux runs the k_step / k_adj kernels of dg_advec.hip).
template <int NP>
int step_np(const dg_plan* p, int ms, const double* in, double* snap, double* last,
            uint16_t* codes, const double* times, double dt, hipStream_t st) {
  const bool burg = p->flux == DG_FLUX_BURGERS, lim = p->limiter != 0;
  if (burg && lim)
    return ms == 2 ? launch_step_nl<NP, true, true, 2>(p, in, snap, last, codes, times, dt, st)
                   : launch_step_nl<NP, true, true, 1>(p, in, snap, last, codes, times, dt, st);
  if (burg)
    return ms == 2 ? launch_step_nl<NP, true, false, 2>(p, in, snap, last, codes, times, dt, st)
                   : launch_step_nl<NP, true, false, 1>(p, in, snap, last, codes, times, dt, st);
  return ms == 2 ? launch_step_nl<NP, false, true, 2>(p, in, snap, last, codes, times, dt, st)
                 : launch_step_nl<NP, false, true, 1>(p, in, snap, last, codes, times, dt, st);
}

template <int NP>
int adj_np(const dg_plan* p, const double* win, double* wout, const double* snap, double* eta,
           int em, const uint16_t* codes, int32_t* count, double t_n, double src, double dt,
           hipStream_t st) {
  const bool burg = p->flux == DG_FLUX_BURGERS, lim = p->limiter != 0;
  if (burg && lim)
    return launch_adj_nl<NP, true, true>(p, win, wout, snap, eta, em, codes, count, t_n, src, dt,
                                         st);
  if (burg)
    return launch_adj_nl<NP, true, false>(p, win, wout, snap, eta, em, codes, count, t_n, src,
                                          dt, st);
  return launch_adj_nl<NP, false, true>(p, win, wout, snap, eta, em, codes, count, t_n, src, dt,
                                        st);
}

int launch_nl_step(const dg_plan* p, int ms, const double* in, double* snap, double* last,
                   uint16_t* codes, const double* times, double dt, hipStream_t st) {
  int rc = DG_OK;
  DG_DISPATCH_NP(p->NP, rc = step_np<NP>(p, ms, in, snap, last, codes, times, dt, st));
  return rc;
}

// Steps per launch of the limited kernels: 1 or 2 (the cone is 10 elements per step).
// Steps per limited-forward launch.  The kernels are VALU-bound, so the 2-step cone's
// extra halo (20 instead of 10 elements per 256-element tile) costs more than the HBM
// round trip it saves whenever the snapshots are written anyway: the default (msteps 4)
// runs 1 step per launch with snapshots and 2 without (A/B at K = 2^22: 82 against 88 µs
// per step with snapshots, 84 against 80.5 without).  An explicit msteps of 1 or 2 is kept.
inline int chunk_nl(const dg_plan* p, int left, bool snapshots) {
  const int m = (p->msteps == 2 || (p->msteps > 2 && !snapshots)) ? 2 : 1;
  return m > left ? left : m;
}

}  // namespace

namespace dgk {

int nl_rhs(const dg_plan* p, const double* u, double* rhs, double t, hipStream_t st) {
  const double fin = flux_value(true, inflow_value(p, t));
  const unsigned grid = grid_for(p->ktot, kBlock);
  const double* sc = p->uniform ? nullptr : p->d_scale;
  DG_DISPATCH_NP(p->NP, hipLaunchKernelGGL((k_rhs_nl<NP>), dim3(grid), dim3(kBlock), 0, st, u,
                                           rhs, sc, make_op<NP>(p), p->s_uniform, fin, p->ktot,
                                           int32_t(p->K)));
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int nl_fwd(dg_plan* p, double* u, double t0, double dt, int nsteps, double* snapshots,
           uint16_t* decisions, hipStream_t st) {
  const int64_t field = p->ktot * p->NP;
  std::vector<double> tn(size_t(nsteps) + 1);  // time = time + dt (One_code.mlx:139)
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  if (snapshots) {
    if (snapshots != u)
      HIP_TRY(hipMemcpyAsync(snapshots, u, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    for (int n = 0; n < nsteps;) {
      const int m = chunk_nl(p, nsteps - n, true);
      double* last = (n + m == nsteps && snapshots != u) ? u : nullptr;
      uint16_t* dec = decisions ? decisions + int64_t(n) * p->ktot : nullptr;
      const int rc = launch_nl_step(p, m, snapshots + int64_t(n) * field,
                                    snapshots + int64_t(n + 1) * field, last, dec, &tn[n], dt,
                                    st);
      if (rc) return rc;
      n += m;
    }
    return DG_OK;
  }
  int launches = 0;  // ping-pong u <-> scratch, landing the last launch in u
  for (int n = 0; n < nsteps; n += chunk_nl(p, nsteps - n, false)) ++launches;
  double* a = u;
  double* b = p->d_scratch;
  if (launches % 2 == 1) {
    HIP_TRY(hipMemcpyAsync(b, a, sizeof(double) * field, hipMemcpyDeviceToDevice, st));
    std::swap(a, b);
  }
  for (int n = 0; n < nsteps;) {
    const int m = chunk_nl(p, nsteps - n, false);
    uint16_t* dec = decisions ? decisions + int64_t(n) * p->ktot : nullptr;
    const int rc = launch_nl_step(p, m, a, nullptr, b, dec, &tn[n], dt, st);
    if (rc) return rc;
    std::swap(a, b);
    n += m;
  }
  return DG_OK;
}

int nl_adj(dg_plan* p, double* w, const double* snapshots, double t0, double dt, int nsteps,
           double src_coef, double* eta, int flags, const uint16_t* decisions, hipStream_t st) {
  const int64_t field = p->ktot * p->NP;
  std::vector<double> tn(size_t(nsteps) + 1);
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  // k_adj_nl's troubled-tile list (shared by the steps: each step's wide pass has finished
  // before the next step lists) and one count per step, zeroed here once per sweep
  int32_t* counts = nullptr;
  if (decisions && p->limiter && nsteps > 0) {
    constexpr int64_t te = kBlock * kNLAdjW - 20;  // k_adj_nl's narrow-cone tile outputs
    const int64_t need = (p->ktot + te - 1) / te;
    if (p->nl_list_tiles < need || p->nl_list_steps < nsteps) {
      HIP_TRY(hipStreamSynchronize(st));  // an earlier sweep may still use it
      (void)hipFree(p->d_nl_list);
      p->d_nl_list = nullptr;
      p->nl_list_tiles = p->nl_list_steps = 0;
      const int64_t cap = (int64_t(p->K_cap) * p->batch + te - 1) / te;
      const int64_t tiles = cap > need ? cap : need;
      const int64_t steps = nsteps > 64 ? nsteps : 64;
      if (hipMalloc(&p->d_nl_list, sizeof(int32_t) * (tiles + steps)) != hipSuccess) {
        p->d_nl_list = nullptr;
        return fail(DG_ERR_NOMEM, "hipMalloc of the config-3 adjoint's tile list failed");
      }
      p->nl_list_tiles = tiles;
      p->nl_list_steps = steps;
    }
    counts = p->d_nl_list + p->nl_list_tiles;
    HIP_TRY(hipMemsetAsync(counts, 0, sizeof(int32_t) * nsteps, st));
  }
  // Launch for step n reads w^{n+1} and u^n and writes w^n; intermediate states alternate
  // between the plan scratch fields and the last launch lands in w.  (w may alias the
  // terminal snapshot: only the first launch reads w, and no launch reads snapshot nsteps.)
  const double* in = w;
  int l = 0;
  for (int n = nsteps - 1; n >= 0; --n, ++l) {
    double* out = (n == 0 && nsteps > 1) ? w : ((l % 2 == 0) ? p->d_scratch : p->d_scratch2);
    const double src = (n + 1 == nsteps) ? 0.0 : src_coef;  // left-endpoint rule
    // DG_ADJ_ETA_ASSIGN / DG_ADJ_ETA_ABS: first launch assigns eta, last one stores |eta|
    const int em = ((l == 0 && (flags & DG_ADJ_ETA_ASSIGN)) ? kEtaAssign : 0) |
                   ((n == 0 && (flags & DG_ADJ_ETA_ABS)) ? kEtaAbs : 0);
    int rc = DG_OK;
    const uint16_t* dec = decisions ? decisions + int64_t(n) * p->ktot : nullptr;
    DG_DISPATCH_NP(p->NP, rc = adj_np<NP>(p, in, out, snapshots + int64_t(n) * field, eta, em,
                                          dec, counts ? counts + n : nullptr, tn[n], src, dt,
                                          st));
    if (rc) return rc;
    in = out;
  }
  // Node-0 source w^0 += src u^0 (and the hand-back of a single-launch sweep).
  if ((src_coef != 0.0 && nsteps > 0) || in != w) {
    hipLaunchKernelGGL(k_src_copy, dim3(grid_for(field, kBlock)), dim3(kBlock), 0, st, in,
                       snapshots, nsteps > 0 ? src_coef : 0.0, w, field);
    HIP_TRY(hipGetLastError());
  }
  return DG_OK;
}

}  // namespace dgk
