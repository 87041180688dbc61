// dg_nl.h — the config-3 stage arithmetic (nonlinear flux, SlopeLimitN after every LSERK4
// stage, and their exact transposes), shared by the two tile layouts that run it:
//   dg_burgers.hip     workgroup tiles: one element per lane across a 256*W-lane workgroup,
//                      every exchange through LDS with a workgroup barrier (XLds);
//   dg_burgers_ov.hip  overlapped waves: every wave owns a window of 64 elements with its own
//                      ghosts, every exchange a DPP wave shift, no barrier inside a step (XDpp).
// The element arithmetic is the same source for both (nl_stage, nl_adj_body): only where a
// neighbour's value comes from differs, and a double is the same double whether it came
// through LDS or DPP, so the two layouts give the same bits.  Internal to libdgadv.so.
//
// Sources: SlopeLimitN (utils/SlopeLimitN.m:1-33), SlopeLimitLin.m:10-18, minmod.m:6-12, the
// per-stage limiter of utils/One_code.mlx:135-136, AdvecRHS1D's central-flux structure
// (utils/AdvecRHS1D.m:9-19, with a*u -> a*f(u)); CPU statement oracle/burgers.py.
//
// Limiter arithmetic.  On a troubled cell SlopeLimitN replaces u by
//   y_i = v + (x_i - x0) m,   m = minmod(ux(1), (v+ - v)/h, (v - v-)/h)   (SlopeLimitLin.m:10-18)
// and x_i - x0 = h r_i / 2 for the LGL nodes, so with hm = h*m
//   y_i = v + (r_i / 2) hm,   hm = minmod(2 (Dr V)(1,1:2) uh(1:2), v+ - v, v - v-)
// (h > 0 scales all three arguments alike): no mesh coordinates are needed, on any mesh.
#pragma once
#include "dg_common.h"

namespace dgn {
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

// An element's face fluxes f(u_0) = fe_0 + fo_0, f(u_N) = fe_0 - fo_0 (HQ: fe_0 doubled).
// Burgers' fo_0 = e o is a bare product, and fe_0 + e o may be contracted into fma(e, o, fe_0)
// -- or not, depending on the code around it: the two exchange layouts would then round the
// same face differently.  The product is materialised first (pin), so the face is always the
// rounded sum of the rounded product, which is also what HQ's fma(0.5, 2 fe_0, fo_0) gives.
template <bool BURG, bool HQ>
__device__ __forceinline__ void face_values(double fe0, double fo0, double& f0, double& fN) {
  if constexpr (HQ) {
    f0 = fma(0.5, fe0, fo0);
    fN = fma(0.5, fe0, -fo0);
  } else {
    if constexpr (BURG) pin(fo0);
    f0 = fe0 + fo0;
    fN = fe0 - fo0;
  }
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

// ---------------------------------------------------------------------------
// Neighbour exchange policies.  Every exchange in the stage arithmetic is a pair of calls:
// *_put with the lane's own values (as early as possible), *_get with the neighbours'
// values (left neighbour's right-side value, right neighbour's left-side value), with a
// trajectory's first / last element taking the boundary value instead (the inflow flux,
// its own value, or zero, as each exchange's comment says).
// ---------------------------------------------------------------------------

// Workgroup tiles: element el = lane of a T-lane tile, arrays of NLGeo, a workgroup barrier
// between put and get.  Boundary values are selected by LDS *index* (the edge tiles keep
// them at slots kCB + ...: the stage inflow fluxes, the residual's, a zero): a select of
// values or pointers lets the compiler fold a flat load onto every stage's critical path.
template <int NP, int W> struct XLds {
  using G = NLGeo<NP, W>;
  static constexpr int T = G::T;
  static constexpr int kCB = G::kLds;
  double* __restrict__ lds;
  int el;
  int se1;  // lane-private stage-input slots lds[se1 + k*T + el] (the adjoint's u_1)
  static constexpr int kSeLds = 1;  // stage inputs u_1 .. u_kSeLds kept in LDS
  static constexpr bool kHalfQ = true;  // the adjoint's recompute uses the host-halved Qoe (HQ)
  __device__ __forceinline__ double& se_slot(int k) { return lds[se1 + k * T + el]; }
  // faces (forward and reverse stages): a -> the left-face array, b -> the right-face array,
  // double-buffered by `par`
  __device__ __forceinline__ void face_put(int par, double a, double b) {
    const int fA = par * 2 * (T + 2), fB = fA + (T + 2);
    lds[fA + el + 1] = a;
    lds[fB + el + 1] = b;
  }
  __device__ __forceinline__ void sync() { __syncthreads(); }
  // forward: left element's right face (first element: the stage inflow flux at slot iin),
  // right element's left face (last element: its own right face, du1 = 0)
  template <bool EDGE>
  __device__ __forceinline__ void fwd_face_get(int par, int iin, double, double, const Elem& E,
                                               double& vl, double& vr) {
    const int fL = par * 2 * (T + 2), fR = fL + (T + 2);
    const int iL = EDGE && E.first ? iin : fR + el;
    const int iR = EDGE && E.last ? fR + el + 1 : fL + el + 2;
    vl = lds[iL];
    vr = lds[iR];
  }
  // reverse: the neighbours' face adjoints (zero at a trajectory's ends)
  template <bool EDGE>
  __device__ __forceinline__ void rev_face_get(int par, const Elem& E, double& gl, double& gr) {
    const int f0 = par * 2 * (T + 2), f1 = f0 + (T + 2);
    gl = lds[EDGE && E.first ? kCB + 6 : f1 + el];
    gr = lds[EDGE && E.last ? kCB + 6 : f0 + el + 2];
  }
  // the indicator's u^{n+1} faces, riding with the first reverse stage's exchange
  __device__ __forceinline__ void ind_put(double uf0, double ufN) {
    lds[G::IL + el + 1] = uf0;
    lds[G::IR + el + 1] = ufN;
  }
  template <bool EDGE>
  __device__ __forceinline__ void ind_get(const Elem& E, double, double, double& l, double& r) {
    l = lds[EDGE && E.first ? kCB + 5 : G::IR + el];
    r = lds[EDGE && E.last ? G::IR + el + 1 : G::IL + el + 2];
  }
  // cell averages (replicated at a trajectory's ends, SlopeLimitN.m:18)
  template <bool EDGE>
  __device__ __forceinline__ void avg_xchg(const Elem& E, double avg, double& am, double& ap) {
    lds[G::FA + el + 1] = avg;
    __syncthreads();
    am = lds[EDGE && E.first ? G::FA + el + 1 : G::FA + el];
    ap = lds[EDGE && E.last ? G::FA + el + 1 : G::FA + el + 2];
  }
  // the transposed limiter's contributions: left neighbour's cr, right neighbour's cl (a
  // trajectory's end receives its own)
  template <bool EDGE>
  __device__ __forceinline__ void lim_xchg(const Elem& E, double cl, double cr, double& fl,
                                           double& fr) {
    lds[G::CL + el + 1] = cl;
    lds[G::CR + el + 1] = cr;
    __syncthreads();
    fl = lds[EDGE && E.first ? G::CL + el + 1 : G::CR + el];
    fr = lds[EDGE && E.last ? G::CR + el + 1 : G::CL + el + 2];
  }
};

// DPP wave shifts of a double: lane l <- lane l-1 (lane 0 keeps its own x) / lane l <- lane
// l+1 (lane 63 keeps x); row-crossing wave_shr:1 / wave_shl:1, two 32-bit moves per double.
// The end lanes' results feed ghosts only.
__device__ __forceinline__ double nl_shr1(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = int(b), hi = int(b >> 32);
  const int rl = __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}
__device__ __forceinline__ double nl_shl1(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = int(b), hi = int(b >> 32);
  const int rl = __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}

// Overlapped waves: the element of a lane is its window lane; neighbours are the adjacent
// lanes of the same wave (every call is in wave-uniform control flow, all 64 lanes active),
// so no barrier anywhere.  Boundary values are plain selects of registers.
// SE: the adjoint's stage inputs u_1 .. u_SE are kept in lane-private LDS slots (the rest in
// registers).
template <int SE = 1, bool HALFQ = true> struct XDpp {
  static constexpr int kCB = 0;
  static constexpr int kSeLds = SE;
  static constexpr bool kHalfQ = HALFQ;
  double* __restrict__ sep;  // lane-private stage-input slots sep[k*64] (this lane's column)
  double fl_, fr_, il_, ir_;
  __device__ __forceinline__ double& se_slot(int k) { return sep[k * 64]; }
  __device__ __forceinline__ void face_put(int, double a, double b) {
    fl_ = nl_shr1(b);
    fr_ = nl_shl1(a);
  }
  __device__ __forceinline__ void sync() {}
  template <bool EDGE>
  __device__ __forceinline__ void fwd_face_get(int, int, double fin, double own_b, const Elem& E,
                                               double& vl, double& vr) {
    vl = EDGE && E.first ? fin : fl_;
    vr = EDGE && E.last ? own_b : fr_;
  }
  template <bool EDGE>
  __device__ __forceinline__ void rev_face_get(int, const Elem& E, double& gl, double& gr) {
    gl = EDGE && E.first ? 0.0 : fl_;
    gr = EDGE && E.last ? 0.0 : fr_;
  }
  __device__ __forceinline__ void ind_put(double uf0, double ufN) {
    il_ = nl_shr1(ufN);
    ir_ = nl_shl1(uf0);
  }
  template <bool EDGE>
  __device__ __forceinline__ void ind_get(const Elem& E, double fin, double own_ufN, double& l,
                                          double& r) {
    l = EDGE && E.first ? fin : il_;
    r = EDGE && E.last ? own_ufN : ir_;
  }
  template <bool EDGE>
  __device__ __forceinline__ void avg_xchg(const Elem& E, double avg, double& am, double& ap) {
    const double l = nl_shr1(avg), r = nl_shl1(avg);
    am = EDGE && E.first ? avg : l;
    ap = EDGE && E.last ? avg : r;
  }
  template <bool EDGE>
  __device__ __forceinline__ void lim_xchg(const Elem& E, double cl, double cr, double& fl,
                                           double& fr) {
    const double l = nl_shr1(cr), r = nl_shl1(cl);
    fl = EDGE && E.first ? cl : l;
    fr = EDGE && E.last ? cr : r;
  }
};

// One LSERK4 stage s of the lane's element:  r = A_s r + dt RHS(u);  v = u + B_s r;
// u = SlopeLimitN(v) if LIM.  Returns the limiter's decision: 0 if the cell is not
// troubled, else 4 | (the active minmod argument, 1..3).  iin / fin: the stage's inflow
// flux f(uin) (XLds: its LDS slot, XDpp: its value).  Exchanges: faces, and with the
// limiter the cell averages (XLds: one barrier each).
//
// Metric: the operator constants carry dt (and 2/h on uniform meshes).  On non-uniform
// meshes the low-storage residual is kept divided by the element's 2/h = sc (r' = r / sc:
// r' = A_s r' + dt L u), so the stage is the uniform one except for the update
// v = u + (B_s sc) r' -- no per-node metric multiplies.
//
// KNOWN: the decisions come from the forward sweep's record `kc` (this stage's 3 bits)
// instead of the troubled-cell test, and `any` (uniform over the exchange group: some
// element of the tile / window is troubled in this stage) gates the cell-average exchange:
// a stage without a troubled cell runs no limiter work and no second exchange.
template <int NP, bool BURG, bool LIM, bool UNI, bool EDGE, bool KNOWN, class X, bool HQ = false>
__device__ __forceinline__ int nl_stage(X& x, int s, int par, int iin, double fin,
                                        const Elem& E, double sc, const EOArgs<NP>& op,
                                        const LimEO<NP>& lc, const LimEO<NP>& lk, double* ev,
                                        double* od, double* re, double* ro, int kc = 0,
                                        bool any = true) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  // par: face buffer, alternating over consecutive stages (across steps too: without the
  // limiter no barrier separates a step's last face reads from the next step's writes)
  double fe[NE], fo[NO];
  flux_eo<NP, BURG, HQ>(ev, od, fe, fo);
  double f0, fN;
  face_values<BURG, HQ>(fe[0], fo[0], f0, fN);
  x.face_put(par, f0, fN);
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
  x.sync();
  // Neighbour fluxes: left element's right face, right element's left face; a
  // trajectory's first element reads the inflow flux, its last one its own face (du1 = 0).
  double vl, vr;
  x.template fwd_face_get<EDGE>(par, iin, fin, fN, E, vl, vr);
  const double du0 = f0 - vl;
  const double du1 = fN - vr;
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
      if (!any) return 0;  // uniform: no troubled cell in the group this stage
    }
    double avg = lc.a0e[0] * ev[0];
#pragma unroll
    for (int k = 1; k < NE; ++k) avg = fma(lc.a0e[k], ev[k], avg);
    // Neighbour averages, replicated at a trajectory's ends (SlopeLimitN.m:18).
    double am, ap;
    x.template avg_xchg<EDGE>(E, avg, am, ap);
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

// ---------------------------------------------------------------------------
// Launch arguments.
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

template <bool LIM> constexpr int cone_per_stage() { return LIM ? 2 : 1; }

// ---------------------------------------------------------------------------
// The reverse step of one element (k_adj_nl's body, both layouts): recompute the step's 5
// stages from u^n = (ev, od) in registers (keeping each stage's input and the limiter's
// decision: troubled or not, and which minmod argument was active), add the functional
// source, accumulate the dual-weighted jump residual of u^{n+1} (returned), then run the
// exact transpose of the stages' tangent on (we, wo) -- the limiter with its decisions
// frozen, the flux Jacobian diag(f'(u)) = diag(a*u) at the recomputed stage inputs.
// kcode / wg: the element's recorded decisions and their OR over the exchange group
// (KNOWN).  `snap`: u^n again (the stage-0 input is re-read there, L2-resident).
// ---------------------------------------------------------------------------
template <int NP, bool BURG, bool LIM, bool UNI, bool KNOWN, bool EDGE, class X>
__device__ __forceinline__ double nl_adj_body(X& x, const Elem& E, double sc, int kcode, int wg,
                                              const NLAdjArgs<NP>& args,
                                              const double* __restrict__ snap, double* ev,
                                              double* od, double* we, double* wo) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  // The stage inputs u_s feed the Burgers flux Jacobian of the reverse pass.  Registers
  // hold u_{L+1}..u_4; u_1..u_L go to lane-private LDS slots (L = X::kSeLds) and u_0 = u^n is
  // re-read from the snapshot (L2-resident) at the end: on the workgroup tiles (L = 1) 20
  // VGPRs fewer at the peak than all in registers (5 waves per SIMD instead of 4).
  double se[5][NE], so[5][NO];
  int dcodes = 0;
  {
    // the recompute's operator: the Burgers even flux doubled against Qoe/2 (flux_eo HQ);
    // the reverse pass keeps Qoe
    // (X::kHalfQ = false: the unhalved pair -- the same numbers, NE multiplies more per stage,
    // 12 SGPRs fewer)
    EOArgs<NP> oph = args.op;
    if constexpr (BURG && X::kHalfQ) {
#pragma unroll
      for (int k = 0; k < NO * NE; ++k) oph.Qoe[k] = args.qoe_h[k];
    }
    double re[NE], ro[NO];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      if (s > X::kSeLds) {
#pragma unroll
        for (int k = 0; k < NE; ++k) se[s][k] = ev[k];
#pragma unroll
        for (int k = 0; k < NO; ++k) so[s][k] = od[k];
      } else if (BURG && s >= 1) {
#pragma unroll
        for (int k = 0; k < NE; ++k) x.se_slot((s - 1) * NP + k) = ev[k];
#pragma unroll
        for (int k = 0; k < NO; ++k) x.se_slot((s - 1) * NP + NE + k) = od[k];
      }
      const int c = nl_stage<NP, BURG, LIM, UNI, EDGE, KNOWN, X, BURG && X::kHalfQ>(
          x, s, s & 1, X::kCB + s, args.fin[s], E, sc, oph, args.lc, args.lc, ev, od, re, ro,
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
    face_values<BURG, false>(fe[0], fo[0], uf0, ufN);
#pragma unroll
    for (int k = 0; k < NE; ++k) ipe = fma(args.op.le[k], we[k], ipe);
#pragma unroll
    for (int k = 0; k < NO; ++k) ipo = fma(args.op.lo[k], wo[k], ipo);
  }

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
    if (LIM && (!KNOWN || ((wg >> (3 * s)) & 4))) {  // (uniform over the exchange group)
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
      // Received: the left neighbour's cr and the right neighbour's cl; at a trajectory's
      // ends the replicated neighbour average is the cell's own (SlopeLimitN.m:18).
      double fl, fr;
      x.template lim_xchg<EDGE>(E, cl, cr, fl, fr);
      const double alpha = cs + fl + fr;
#pragma unroll
      for (int k = 0; k < NE; ++k) we[k] = fma(alpha, args.lc.a0e[k], we[k]);
    }
    // Face buffers alternate starting with buffer 1: the recompute's last stage read
    // buffer 0 after its barrier, and no barrier separates it from this first write.
    const int par = (ss + 1) & 1;
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
    x.face_put(par, g0, g1);
    if (ss == 0 && args.has_eta) x.ind_put(uf0, ufN);  // the indicator's u^{n+1} faces ride along
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
    x.sync();
    if (ss == 0 && args.has_eta) {
      // left neighbour's right face / right neighbour's left face of u^{n+1}; a
      // trajectory's first element reads the inflow flux at t_{n+1}, its last one its own
      // right face (du1 = 0)
      double l, r;
      x.template ind_get<EDGE>(E, args.fin[5], ufN, l, r);
      const double du0 = uf0 - l;
      const double du1 = ufN - r;
      eacc = fma(du0 - du1, ipe, (du0 + du1) * ipo);
      if constexpr (!UNI) eacc *= sc;
    }
    double gl, gr;
    x.template rev_face_get<EDGE>(par, E, gl, gr);
    pe[0] += (g0 + g1) - (gr + gl);
    po[0] += (g0 - g1) + (gr - gl);
    if constexpr (BURG) {  // f'(u) = u: the symmetric block [[e, o], [o, e]] per node pair
      double ue[NE], uo[NO];  // u_s (see the recompute)
      if (s > X::kSeLds) {
#pragma unroll
        for (int k = 0; k < NE; ++k) ue[k] = se[s][k];
#pragma unroll
        for (int k = 0; k < NO; ++k) uo[k] = so[s][k];
      } else if (s >= 1) {
#pragma unroll
        for (int k = 0; k < NE; ++k) ue[k] = x.se_slot((s - 1) * NP + k);
#pragma unroll
        for (int k = 0; k < NO; ++k) uo[k] = x.se_slot((s - 1) * NP + NE + k);
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
  return eacc;
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

// Arguments of MS limited forward steps from times[0..MS) (both layouts).  The constants
// carry dt (and 2/h on uniform meshes); non-uniform meshes multiply the update by the
// element's 2/h (nl_stage's metric folding).
template <int NP, bool BURG, int MS>
NLStepArgs<NP, MS> nl_step_args(const dg_plan* p, const double* times, double dt) {
  NLStepArgs<NP, MS> a;
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
  return a;
}

// Arguments of one reverse step from t_n (both layouts); has_eta: the kEta* bits.
template <int NP, bool BURG>
NLAdjArgs<NP> nl_adj_args(const dg_plan* p, int has_eta, double t_n, double src, double dt) {
  NLAdjArgs<NP> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : dt, &a.op);  // see nl_step_args
  for (int k = 0; k < EOArgs<NP>::NO * EOArgs<NP>::NE; ++k) a.qoe_h[k] = 0.5 * a.op.Qoe[k];
  a.lc = make_lim_eo<NP>(p);
  a.sc = 1.0;
  for (int s = 0; s < 5; ++s) a.fin[s] = flux_value(BURG, inflow_value(p, t_n + RK<5>::C(s) * dt));
  a.fin[5] = flux_value(BURG, inflow_value(p, t_n + dt));
  a.src = src;
  a.ktot = p->ktot;
  a.K = int32_t(p->K);
  a.has_eta = has_eta;
  a.xcd = p->xcd_order;
  return a;
}

// The overlapped-wave launches (dg_burgers_ov.hip).  ow_step: one limited step from `in`
// into `snap` (and `last`), the decision record into `codes`; ow_adj: one reverse step
// (`count`: the step's troubled-window count in the plan's list, zeroed by the caller).
// Each returns DG_OK, or 1 when the shape has no overlapped-wave kernel (the caller runs the
// workgroup tiles), or a negative error.
int ow_step(const dg_plan* p, const double* in, double* snap, double* last, uint16_t* codes,
            const double* times, double dt, hipStream_t st);
int ow_adj(const dg_plan* p, const double* win, double* wout, const double* snap, double* eta,
           int em, const uint16_t* codes, int32_t* count, double t_n, double src, double dt,
           hipStream_t st);
// Outputs of one overlapped-wave adjoint window (64 lanes less a 10-element cone per side): the
// unit of its troubled-window list (dg_plan d_nl_list); windows (waves) per tile.
constexpr int kOwAdjOwned = 44;
constexpr int kOwTileWindows = 4;

}  // namespace dgn
