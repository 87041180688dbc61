// dg_burgers_ov.hip — the config-3 kernels (BASELINE config 3: Burgers-type flux, SlopeLimitN
// after every LSERK4 stage, frozen-decision adjoint) on OVERLAPPED WAVES:
// no workgroup barrier inside a step.  Selected by DG_TUNE_NL_EXCHANGE = 1.
//
// The workgroup-tile kernels of dg_burgers.hip exchange every stage's faces, and with the
// limiter its cell averages, through LDS with a workgroup barrier each: 10 barriers per
// forward step, ~10 per reverse step, and their waves wait 55-58 % of their cycles there while
// the fp64 pipe idles (DESIGN.md §5 "Config 3", profiles/r05/config3/).  Here:
//   - every wave works on its own WINDOW of 64 consecutive elements, one per lane, and moves
//     every neighbour value (faces, cell averages, the transposed limiter's contributions, the
//     indicator's faces) between its lanes with DPP wave shifts (dg_nl.h XDpp);
//   - windows of neighbouring waves overlap by 2G elements, G = the step's dependency cone:
//     a wave OWNS the middle S = 64 - 2G elements of its window, whose values depend only on
//     the window (the G lanes at each end are ghosts whose results are never stored).  One
//     step per launch, so a window is loaded once and nothing is exchanged between waves;
//   - the workgroup's NW waves share one coalesced 16-byte load of their windows' union
//     (NW S + 2G elements) through LDS: one barrier after the load, one before the forward's
//     coalesced store.  The adjoint stores from registers.
// Cones (elements per side):
//   forward  G = 10: 5 stages x (faces + the limiter's neighbour averages); S = 44;
//   adjoint  G = 10 on the narrow cone: 5 recomputed stages + 5 reverse stages x faces, valid
//            when the forward's decision record shows no troubled cell in the window in this
//            step (almost every window) -- the limiter is then the identity in every stage.
//            A window with a troubled cell (wave-uniform, by ballot over the record) recomputes
//            its owned elements on the wide cone (G = 20: every stage also exchanges averages)
//            as two windows of 24 + 20 owned elements read straight from global memory, in the
//            same launch: no troubled-tile list and no second kernel (the workgroup tiles pay
//            a ~5 us k_adj_nl_wide launch per reverse step for it).
// The element arithmetic is dg_nl.h's nl_stage / nl_adj_body, the same source as the
// workgroup tiles with a different exchange policy: the results are the same bits (tested:
// tests/test_gpu_nl_exchange.py).  Cost: a window computes 64 elements and owns 44 (the
// ghosts redo 45 % of the work), which the barrier-free waves absorb in the fp64 pipe's idle
// cycles.
#include "dg_nl.h"

namespace {
using namespace dgk;
using namespace dgn;

constexpr int kOwWaves = kOwTileWindows;  // waves per workgroup (windows per tile)
constexpr int kOwAdjWaves = 5;  // occupancy target of the narrow adjoint (waves per SIMD)
// the adjoint's stage inputs kept in LDS (u_1 .. u_kOwSe; dg_nl.h nl_adj_body)
constexpr int kOwSe = 3;
constexpr bool kOwHalfQ = false;
template <int NP> using OwX = XDpp<kOwSe, kOwHalfQ>;

template <int NP, int G> struct OwGeo {
  static constexpr int LB = 64 * kOwWaves;         // lanes per workgroup
  static constexpr int S = 64 - 2 * G;             // elements a wave owns
  static constexpr int TE = kOwWaves * S;          // a tile's outputs
  static constexpr int T = TE + 2 * G;             // a tile's elements (incl. halo)
  static constexpr int kTileD = T * NP + 2;        // staging image (+2: 16-byte realignment)
  static constexpr int kVec = (kTileD + 2 * LB - 1) / (2 * LB);  // double2 loads per lane
  static constexpr int kImg = (kTileD + 1) & ~1;   // doubles per image (16-byte multiple)
  static_assert(S > 0 && TE % 2 == 0, "window geometry: outputs in 16-byte runs");
};

// Coalesced 16-byte loads of NS tile images [e0, e0 + T) (zeros outside [0, nd)), all issued
// before any is written to LDS.  Returns the images' offset (0 or 1 double).
template <class Geo, int NP, bool EDGE, int NS>
__device__ __forceinline__ int ow_load(const double* const (&g)[NS], int64_t e0, int64_t nd,
                                       double* __restrict__ lds) {
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  const int off = int(d0 - base);
  const int nvec = (Geo::T * NP + off + 1) >> 1;
  double2 rv[NS][Geo::kVec];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g[i]);
#pragma unroll
    for (int q = 0; q < Geo::kVec; ++q) {
      const int v = int(threadIdx.x) + q * Geo::LB;
      const int64_t gd = base + 2 * int64_t(v);
      double2 val = make_double2(0.0, 0.0);
      if (v < nvec) {
        if (!EDGE || (gd >= 0 && gd + 1 < nd)) {
          val = g2[gd >> 1];
        } else {
          if (gd >= 0 && gd < nd) val.x = g[i][gd];
          if (gd + 1 >= 0 && gd + 1 < nd) val.y = g[i][gd + 1];
        }
      }
      rv[i][q] = val;
    }
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) {
#pragma unroll
    for (int q = 0; q < Geo::kVec; ++q) {
      const int v = int(threadIdx.x) + q * Geo::LB;
      if (v < nvec) *reinterpret_cast<double2*>(&lds[i * Geo::kImg + 2 * v]) = rv[i][q];
    }
  }
  return off;
}

// ---------------------------------------------------------------------------
// Forward: one limited step per launch (u^n -> u^{n+1} and the decision record of step n).
// ---------------------------------------------------------------------------
template <int NP, bool BURG, bool LIM, bool UNI>
__global__ __launch_bounds__(64 * kOwWaves) DG_NL_STEP_ATTR void k_step_nlw(
    const double* __restrict__ uin, double* __restrict__ snap, double* __restrict__ last,
    const double* __restrict__ scale, uint16_t* __restrict__ codes, NLStepArgs<NP, 1> args);

template <int NP, bool BURG, bool LIM, bool UNI, bool EDGE>
__device__ __forceinline__ void ow_step_tile(double* __restrict__ lds, int64_t tile,
                                             const double* __restrict__ uin,
                                             double* __restrict__ snap, double* __restrict__ last,
                                             const double* __restrict__ scale,
                                             uint16_t* __restrict__ codes,
                                             const NLStepArgs<NP, 1>& args) {
  constexpr int G = 5 * cone_per_stage<LIM>();
  using Geo = OwGeo<NP, G>;
  constexpr int T = Geo::T, TE = Geo::TE, S = Geo::S, LB = Geo::LB;
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  const int lane = threadIdx.x, wv = lane >> 6, j = lane & 63;
  const int el = wv * S + j;  // the lane's tile element
  const bool own = j >= G && j < 64 - G;
  const int64_t e0 = tile * TE - G;
  const int64_t nd = args.ktot * NP;
  const int64_t o0 = tile * TE * NP;

  Elem E = elem_info<G, T, EDGE>(e0, el, args.ktot, args.K);
  E.valid = E.valid && own;
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;  // issued with the tile's loads
  const double* const src[1] = {uin};
  const int off = ow_load<Geo, NP, EDGE, 1>(src, e0, nd, lds);
  __syncthreads();
  double ev[NE], od[NO];
  to_eo<NP>(lds + off + el * NP, ev, od);

  // The troubled-cell branch's constants are read from the kernel-argument segment where
  // they are used (scalar loads inside the rare branch), as on the workgroup tiles.
  using SArgs = NLStepArgs<NP, 1>;
  const LimEO<NP>& lk = *reinterpret_cast<const LimEO<NP>*>(
      kernarg_tail<decltype(&k_step_nlw<NP, BURG, LIM, UNI>), SArgs>() + offsetof(SArgs, lc));
  double re[NE], ro[NO];
  XDpp<> x{nullptr};
  int c15 = 0;  // the step's limiter decisions, 3 bits per stage
#pragma unroll
  for (int s = 0; s < 5; ++s)
    c15 |= nl_stage<NP, BURG, LIM, UNI, EDGE, false, XDpp<>, BURG>(
               x, s, s & 1, 0, args.fin[s], E, sc, args.op, args.lc, lk, ev, od, re, ro)
           << (3 * s);
  // the decision record for the adjoint (dg_lserk4_fwd_ex): one 16-bit word per element
  if (LIM && codes != nullptr && E.valid) codes[E.e] = uint16_t(c15);
  // u^{n+1}: the owned elements to the output image (its own region: a slower wave may still
  // read its window from the input image), then 16-byte stores
  double* outi = lds + Geo::kImg;
  if (own) from_eo<NP>(ev, od, outi + (el - G) * NP);
  __syncthreads();
  if constexpr (EDGE) {
    const int64_t rem = nd - o0;
    const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;
    if (snap != nullptr) store_run<LB>(snap, o0, count, outi);
    if (last != nullptr) store_run<LB>(last, o0, count, outi);
  } else {
    if (snap != nullptr) store_full<TE * NP, LB>(snap, o0, outi);
    if (last != nullptr) store_full<TE * NP, LB>(last, o0, outi);
  }
}

template <int NP, bool BURG, bool LIM, bool UNI>
__global__ __launch_bounds__(64 * kOwWaves) DG_NL_STEP_ATTR void k_step_nlw(
    const double* __restrict__ uin, double* __restrict__ snap, double* __restrict__ last,
    const double* __restrict__ scale, uint16_t* __restrict__ codes, NLStepArgs<NP, 1> args) {
  using Geo = OwGeo<NP, 5 * cone_per_stage<LIM>()>;
  __shared__ __attribute__((aligned(16))) double lds[Geo::kImg + Geo::TE * NP];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  const int64_t e0 = tile * Geo::TE - (Geo::T - Geo::TE) / 2;
  if (edge_tile(e0, Geo::T, args.ktot, args.K))
    ow_step_tile<NP, BURG, LIM, UNI, true>(lds, tile, uin, snap, last, scale, codes, args);
  else
    ow_step_tile<NP, BURG, LIM, UNI, false>(lds, tile, uin, snap, last, scale, codes, args);
}

// ---------------------------------------------------------------------------
// Adjoint: one reverse step per launch (w^{n+1} -> w^n), stages recomputed from u^n.
// ---------------------------------------------------------------------------

// The lane's element of a reverse step, from its even/odd state: eta (owned lanes) and w^n
// straight from registers.
template <int NP>
__device__ __forceinline__ void ow_adj_out(const Elem& E, double eacc, const double* we,
                                           const double* wo, double* __restrict__ eta,
                                           double* __restrict__ wout, int has_eta) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  if (!E.valid) return;
  if (has_eta) eta_update(eta, E.e, eacc, has_eta);
  double* o = wout + E.e * NP;
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    o[k] = 0.5 * (we[k] + wo[k]);
    o[N - k] = 0.5 * (we[k] - wo[k]);
  }
  if constexpr (NE > NO) o[NO] = we[NO];
}

// Dual (adjoint) even/odd coordinates of a nodal w: we_k = w_k + w_{N-k}, wo_k = w_k - w_{N-k}.
template <int NP>
__device__ __forceinline__ void to_dual(const double* w, double* we, double* wo) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    we[k] = w[k] + w[N - k];
    wo[k] = w[k] - w[N - k];
  }
  if constexpr (NE > NO) we[NO] = w[NO];
}

// The adjoint's narrow cone: 1 element per stage, 10 stages (5 recomputed + 5 reverse).
constexpr int kOwAdjG = 10;
static_assert(64 - 2 * kOwAdjG == kOwAdjOwned, "dg_nl.h kOwAdjOwned: a narrow window's outputs");

// The narrow-cone reverse step of the tile's windows.  A wave whose window holds a troubled
// cell in this step (wave-uniform, by ballot over the record) stores nothing and appends its
// owned range to the step's list for k_adj_nlw_wide.
template <int NP, bool BURG, bool LIM, bool UNI, bool EDGE>
__device__ __forceinline__ void ow_adj_tile(double* __restrict__ lds, int64_t tile,
                                            const double* __restrict__ win,
                                            double* __restrict__ wout,
                                            const double* __restrict__ snap,
                                            double* __restrict__ eta,
                                            const double* __restrict__ scale,
                                            const uint16_t* __restrict__ codes,
                                            int32_t* __restrict__ list,
                                            int32_t* __restrict__ count,
                                            const NLAdjArgs<NP>& args) {
  constexpr int G = kOwAdjG;
  using Geo = OwGeo<NP, G>;
  constexpr int T = Geo::T, TE = Geo::TE, S = Geo::S;
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  const int lane = threadIdx.x, wv = lane >> 6, j = lane & 63;
  const int el = wv * S + j;
  const int64_t e0 = tile * TE - G;
  const int64_t nd = args.ktot * NP;

  // the decision record first, with the tiles, so its latency hides behind theirs
  int kcode = 0;
  if constexpr (LIM) {
    const int64_t e = e0 + el;
    kcode = (e >= 0 && e < args.ktot) ? int(codes[e]) : 0;
  }
  Elem E = elem_info<G, T, EDGE>(e0, el, args.ktot, args.K);
  E.valid = E.valid && j >= G && j < 64 - G;
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;
  const double* const src[2] = {snap, win};
  const int off = ow_load<Geo, NP, EDGE, 2>(src, e0, nd, lds);
  __syncthreads();
  double ev[NE], od[NO], we[NE], wo[NO];
  to_eo<NP>(lds + off + el * NP, ev, od);
  to_dual<NP>(lds + Geo::kImg + off + el * NP, we, wo);
  __syncthreads();  // the images are read: the stage-input slots alias them
  // (wave-uniform) a troubled cell anywhere in the window: its outputs need the wide cone
  if (LIM && __builtin_amdgcn_ballot_w64(kcode != 0) != 0) {
    if (j == 0) list[atomicAdd(count, 1)] = int32_t(e0 + el + G);  // the owned range's start
    return;
  }
  OwX<NP> x{lds + wv * 64 * kOwSe * NP + j};
  // no troubled cell in the window: the limiter is the identity in every stage (wg = 0)
  const double eacc = nl_adj_body<NP, BURG, LIM, UNI, LIM, EDGE>(x, E, sc, 0, 0, args, snap, ev,
                                                                 od, we, wo);
  ow_adj_out<NP>(E, eacc, we, wo, eta, wout, args.has_eta);
}

template <int NP, bool BURG, bool LIM, bool UNI>
__global__ __launch_bounds__(64 * kOwWaves, kOwAdjWaves) void k_adj_nlw(
    const double* __restrict__ win, double* __restrict__ wout, const double* __restrict__ snap,
    double* __restrict__ eta, const double* __restrict__ scale,
    const uint16_t* __restrict__ codes, int32_t* __restrict__ list, int32_t* __restrict__ count,
    NLAdjArgs<NP> args) {
  using Geo = OwGeo<NP, kOwAdjG>;
  // two images (u^n, w^{n+1}); once they are read, each wave's lane-private stage inputs
  constexpr int kSe = BURG ? kOwWaves * 64 * kOwSe * NP : 0;
  __shared__ __attribute__((aligned(16))) double lds[2 * Geo::kImg > kSe ? 2 * Geo::kImg : kSe];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  const int64_t e0 = tile * Geo::TE - kOwAdjG;
  if (edge_tile(e0, Geo::T, args.ktot, args.K))
    ow_adj_tile<NP, BURG, LIM, UNI, true>(lds, tile, win, wout, snap, eta, scale, codes, list,
                                          count, args);
  else
    ow_adj_tile<NP, BURG, LIM, UNI, false>(lds, tile, win, wout, snap, eta, scale, codes, list,
                                           count, args);
}

// The windows k_adj_nlw listed as troubled: each wave takes one (grid-stride; almost always
// none) and recomputes its S = 44 owned elements on the wide cone, as two windows of 64 lanes
// with HW = 20 ghosts per side owning 24 and 20 elements, loaded per lane from global memory
// (L2-resident), decisions from the record, the limiter's exchanges gated per stage by the OR
// of the window's records (as the workgroup tiles gate them by the tile's).  A separate launch
// (like k_adj_nl_wide): with both bodies in one kernel the compiler spilled ~80 SGPRs and
// 20-40 VGPRs, each body alone fits.  Each step of a sweep has its own count (nl_adj zeroes
// them once per sweep).
template <int NP, bool BURG, bool LIM, bool UNI>
__global__ __launch_bounds__(64 * kOwWaves, 4) void k_adj_nlw_wide(
    const double* __restrict__ win, double* __restrict__ wout, const double* __restrict__ snap,
    double* __restrict__ eta, const double* __restrict__ scale,
    const uint16_t* __restrict__ codes, int32_t* __restrict__ list, int32_t* __restrict__ count,
    NLAdjArgs<NP> args) {
  constexpr int HW = 20, S = kOwAdjOwned, P0 = 64 - 2 * HW;
  static_assert(P0 > 0 && S <= 2 * P0, "two wide windows cover a narrow window's outputs");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  __shared__ __attribute__((aligned(16))) double lds[BURG ? kOwWaves * 64 * kOwSe * NP : 1];
  const int lane = threadIdx.x, wv = lane >> 6, j = lane & 63;
  OwX<NP> x{lds + wv * 64 * kOwSe * NP + j};
  const int n = *count;  // final: k_adj_nlw has completed
  for (int i = blockIdx.x * kOwWaves + wv; i < 2 * n; i += gridDim.x * kOwWaves) {
    const int p = i & 1;  // which half of the window's outputs
    const int nown = p == 0 ? P0 : S - P0;
    const int64_t ew0 = int64_t(list[i >> 1]) + p * P0 - HW;
    Elem E = elem_info<HW, 64, true>(ew0, j, args.ktot, args.K);
    E.valid = E.valid && j < HW + nown;
    const int kcode = E.inrange ? int(codes[E.e]) : 0;
    int wg = 0;  // the window's OR of the troubled bits, per stage
#pragma unroll
    for (int s = 0; s < 5; ++s)
      if (__builtin_amdgcn_ballot_w64((kcode >> (3 * s)) & 4) != 0) wg |= 4 << (3 * s);
    double sc = args.sc;
    if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;
    double u[NP], w[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      u[k] = E.inrange ? snap[E.e * NP + k] : 0.0;
      w[k] = E.inrange ? win[E.e * NP + k] : 0.0;
    }
    double ev[NE], od[NO], we[NE], wo[NO];
    to_eo<NP>(u, ev, od);
    to_dual<NP>(w, we, wo);
    const double eacc = nl_adj_body<NP, BURG, LIM, UNI, LIM, true>(x, E, sc, kcode, wg, args,
                                                                   snap, ev, od, we, wo);
    ow_adj_out<NP>(E, eacc, we, wo, eta, wout, args.has_eta);
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
template <int NP, bool BURG, bool LIM>
int launch_step_ow(const dg_plan* p, const double* in, double* snap, double* last,
                   uint16_t* codes, const double* times, double dt, hipStream_t st) {
  const NLStepArgs<NP, 1> a = nl_step_args<NP, BURG, 1>(p, times, dt);
  using Geo = OwGeo<NP, 5 * cone_per_stage<LIM>()>;
  const unsigned grid = grid_for(p->ktot, Geo::TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_step_nlw<NP, BURG, LIM, true>), dim3(grid), dim3(Geo::LB), 0, st, in,
                       snap, last, p->d_scale, codes, a);
  else
    hipLaunchKernelGGL((k_step_nlw<NP, BURG, LIM, false>), dim3(grid), dim3(Geo::LB), 0, st, in,
                       snap, last, p->d_scale, codes, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP, bool BURG, bool LIM>
int launch_adj_ow(const dg_plan* p, const double* win, double* wout, const double* snap,
                  double* eta, int em, const uint16_t* codes, int32_t* count, double t_n,
                  double src, double dt, hipStream_t st) {
  if (LIM && (codes == nullptr || count == nullptr)) return 1;  // the narrow cone needs the record
  const NLAdjArgs<NP> a = nl_adj_args<NP, BURG>(p, eta != nullptr ? (em | kEtaOn) : 0, t_n, src, dt);
  using Geo = OwGeo<NP, kOwAdjG>;
  const unsigned grid = grid_for(p->ktot, Geo::TE);
  int32_t* list = LIM ? p->d_nl_list : nullptr;
  if (LIM && (list == nullptr || p->nl_list_tiles < int64_t(grid) * kOwWaves))
    return fail(DG_ERR_ARG, "config-3 adjoint: window list not sized (nl_adj)");
  if (p->uniform)
    hipLaunchKernelGGL((k_adj_nlw<NP, BURG, LIM, true>), dim3(grid), dim3(Geo::LB), 0, st, win,
                       wout, snap, eta, p->d_scale, codes, list, count, a);
  else
    hipLaunchKernelGGL((k_adj_nlw<NP, BURG, LIM, false>), dim3(grid), dim3(Geo::LB), 0, st, win,
                       wout, snap, eta, p->d_scale, codes, list, count, a);
  HIP_TRY(hipGetLastError());
  if constexpr (LIM) {
    // one wave per listed half window; a few workgroups suffice (a step lists a handful)
    const unsigned gw = std::min<unsigned>(grid, 64u);
    if (p->uniform)
      hipLaunchKernelGGL((k_adj_nlw_wide<NP, BURG, LIM, true>), dim3(gw), dim3(Geo::LB), 0, st,
                         win, wout, snap, eta, p->d_scale, codes, list, count, a);
    else
      hipLaunchKernelGGL((k_adj_nlw_wide<NP, BURG, LIM, false>), dim3(gw), dim3(Geo::LB), 0, st,
                         win, wout, snap, eta, p->d_scale, codes, list, count, a);
    HIP_TRY(hipGetLastError());
  }
  return DG_OK;
}

}  // namespace

namespace dgn {

// (flux, limiter) combinations as dg_burgers.hip step_np / adj_np: Burgers + limiter,
// Burgers alone, linear + limiter.
int ow_step(const dg_plan* p, const double* in, double* snap, double* last, uint16_t* codes,
            const double* times, double dt, hipStream_t st) {
  const bool burg = p->flux == DG_FLUX_BURGERS, lim = p->limiter != 0;
  int rc = DG_OK;
  if (burg && lim)
    DG_DISPATCH_NP(p->NP, rc = (launch_step_ow<NP, true, true>(p, in, snap, last, codes, times, dt, st)))
  else if (burg)
    DG_DISPATCH_NP(p->NP, rc = (launch_step_ow<NP, true, false>(p, in, snap, last, codes, times, dt, st)))
  else
    DG_DISPATCH_NP(p->NP, rc = (launch_step_ow<NP, false, true>(p, in, snap, last, codes, times, dt, st)))
  return rc;
}

int ow_adj(const dg_plan* p, const double* win, double* wout, const double* snap, double* eta,
           int em, const uint16_t* codes, int32_t* count, double t_n, double src, double dt,
           hipStream_t st) {
  const bool burg = p->flux == DG_FLUX_BURGERS, lim = p->limiter != 0;
  int rc = DG_OK;
  if (burg && lim)
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_ow<NP, true, true>(p, win, wout, snap, eta, em, codes, count, t_n, src, dt, st)))
  else if (burg)
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_ow<NP, true, false>(p, win, wout, snap, eta, em, codes, count, t_n, src, dt, st)))
  else
    DG_DISPATCH_NP(p->NP, rc = (launch_adj_ow<NP, false, true>(p, win, wout, snap, eta, em, codes, count, t_n, src, dt, st)))
  return rc;
}

}  // namespace dgn
