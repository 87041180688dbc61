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
// These are the workgroup-tile kernels (exchanges through LDS, a barrier each); the stage
// arithmetic is dg_nl.h's, shared with the overlapped-wave kernels of dg_burgers_ov.hip,
// which nl_fwd / nl_adj run instead where the plan selects them (DG_TUNE_NL_EXCHANGE).
#include "dg_nl.h"

namespace {
using namespace dgk;
using namespace dgn;

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

// Tile widths of the config-3 kernels: workgroups of 256*W lanes own tiles of 256*W
// elements.  Measured at K = 2^22 (bench.py --config 3): the forward (64 VGPRs, 8 waves per
// SIMD) gains from 512-element tiles (halo 4 % instead of 8 %: 101 -> 93 us per step with the
// SGPR cap); the adjoint (117 VGPRs, 4 waves per SIMD) loses (145 -> 151 us): with two
// 8-wave workgroups per CU each barrier stalls half the CU's waves.  Round 6: 768- and
// 1024-element forward tiles (fewer tile rounds per launch, 2-3 % less halo) measured 99 and
// 94 us per step against 88 (profiles/r06/c3w/, patches in profiles/r06/variants/): 12- and
// 16-wave barriers cost more than the tail they save.
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
  XLds<NP, W> x{lds, lane, 0};
#pragma unroll
  for (int st = 0; st < MS; ++st) {
    int c15 = 0;  // this step's limiter decisions, 3 bits per stage
#pragma unroll
    for (int s = 0; s < 5; ++s)
      c15 |= nl_stage<NP, BURG, LIM, UNI, EDGE, false, XLds<NP, W>, BURG>(
                 x, s, (st * 5 + s) & 1, CB + st * 5 + s, 0.0, E, sc, args.op, args.lc, lk, ev,
                 od, re, ro)
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
  XLds<NP, W> x{lds, lane, CB + 8};  // lds[CB + 8 + k*T + lane]: u_1 in even/odd coordinates
  const double eacc = nl_adj_body<NP, BURG, LIM, UNI, KNOWN, EDGE>(x, E, sc, kcode, wg, args,
                                                                   snap, ev, od, we, wo);

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

template <int NP, bool BURG, bool LIM, int MS>
int launch_step_nl(const dg_plan* p, const double* in, double* snap, double* last,
                   uint16_t* codes, const double* times, double dt, hipStream_t st) {
  const NLStepArgs<NP, MS> a = nl_step_args<NP, BURG, MS>(p, times, dt);
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
  const NLAdjArgs<NP> a = nl_adj_args<NP, BURG>(p, eta != nullptr ? (em | kEtaOn) : 0, t_n, src, dt);
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

// One forward launch of ms steps: on overlapped waves (one step per launch) where the plan
// selects them (DG_TUNE_NL_EXCHANGE), else on workgroup tiles.
int launch_nl_step(const dg_plan* p, int ms, const double* in, double* snap, double* last,
                   uint16_t* codes, const double* times, double dt, hipStream_t st) {
  if (ms == 1 && p->nl_exchange) {
    const int rc = ow_step(p, in, snap, last, codes, times, dt, st);
    if (rc != 1) return rc;  // 1: no overlapped-wave kernel for this shape
  }
  int rc = DG_OK;
  DG_DISPATCH_NP(p->NP, rc = step_np<NP>(p, ms, in, snap, last, codes, times, dt, st));
  return rc;
}

// Steps per limited-forward launch: 1 or 2 (the cone is 10 elements per step).  The
// workgroup-tile kernels are barrier-bound, so the 2-step cone's extra halo (20 instead of
// 10 elements per 256-element tile) costs more than the HBM round trip it saves whenever the
// snapshots are written anyway: the default (msteps 4) runs 1 step per launch with snapshots
// and 2 without (A/B at K = 2^22: 82 against 88 µs per step with snapshots, 84 against 80.5
// without).  An explicit msteps of 1 or 2 is kept.  The overlapped waves run 1 step per
// launch (a 2-step window would own 24 of its 64 elements).
inline int chunk_nl(const dg_plan* p, int left, bool snapshots) {
  const int m = (p->msteps == 2 || (p->msteps > 2 && !snapshots && !p->nl_exchange)) ? 2 : 1;
  return m > left ? left : m;
}

}  // namespace

namespace dgk {

int nl_query(const dg_plan* p, int64_t out[3]) {
  out[0] = p->nl_exchange;
  out[1] = chunk_nl(p, 1 << 30, true);
  out[2] = chunk_nl(p, 1 << 30, false);
  return DG_OK;
}

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
  // The troubled-tile list of k_adj_nl (shared by the steps: each step's wide pass has
  // finished before the next step lists) and one count per step, zeroed here once per sweep.
  // The overlapped-wave adjoint (DG_TUNE_NL_EXCHANGE; it needs the record when limited) lists
  // troubled windows instead of tiles: kOwTileWindows per tile of kOwTileWindows*kOwAdjOwned.
  const bool ow = p->nl_exchange && (decisions != nullptr || !p->limiter);
  int32_t* counts = nullptr;
  if (decisions && p->limiter && nsteps > 0) {
    const int64_t te = ow ? kOwTileWindows * kOwAdjOwned : kBlock * kNLAdjW - 20;
    const int64_t per = ow ? kOwTileWindows : 1;  // list items per tile
    const int64_t need = (p->ktot + te - 1) / te * per;
    if (p->nl_list_tiles < need || p->nl_list_steps < nsteps) {
      HIP_TRY(hipStreamSynchronize(st));  // an earlier sweep may still use it
      (void)hipFree(p->d_nl_list);
      p->d_nl_list = nullptr;
      p->nl_list_tiles = p->nl_list_steps = 0;
      const int64_t cap = (int64_t(p->K_cap) * p->batch + te - 1) / te * per;
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
    int rc = 1;
    const uint16_t* dec = decisions ? decisions + int64_t(n) * p->ktot : nullptr;
    if (ow)
      rc = ow_adj(p, in, out, snapshots + int64_t(n) * field, eta, em, dec,
                  counts ? counts + n : nullptr, tn[n], src, dt, st);
    if (rc == 1) {
      if (ow) return fail(DG_ERR_ARG, "config-3 adjoint: no overlapped-wave kernel for this shape");
      DG_DISPATCH_NP(p->NP, rc = adj_np<NP>(p, in, out, snapshots + int64_t(n) * field, eta, em,
                                            dec, counts ? counts + n : nullptr, tn[n], src, dt,
                                            st));
    }
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
