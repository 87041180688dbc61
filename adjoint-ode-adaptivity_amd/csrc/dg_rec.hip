// dg_rec.hip — the jump-record sweep pair (dg_lserk4_fwd_rec / dg_lserk4_adj_rec) on pair
// tiles, one launch per block of steps (k_step_rp / k_adj_rp; the tile bodies, their layout
// and the Horner-form step are in dg_rec_tiles.h, shared with the dataflow sweep of
// dg_sweep.hip).  Launches of 1, 2, 4, 5, 8, 10, 16 or 20 steps.
// Measured (N = 4, K = 2^20, bench, A/B pairs on one box, DESIGN.md §5 "Pair tiles"): with
// 8 + 8 + 4 launches 5.86-5.98e11 DOF-updates/s on 512-element tiles against 5.67-5.72e11 for
// the one-element-per-lane record kernels; 10 + 10 launches 6.07-6.12e11 (W = 1) and
// 6.15-6.16e11 (W = 2, the default).  Four elements per lane, raised wave priority, an
// unrolled step loop, no scheduling pins, 6 waves per SIMD for the adjoint: no gain.
// Sources: AdvecRHS1D (utils/AdvecRHS1D.m:9-19), the LSERK4 loop (utils/One_code.mlx:106-140),
// the indicator pattern (python/Main_finite_difference.py:54-94); DESIGN.md §5.
#include "dg_rec_tiles.h"

namespace {
using namespace dgk;
using namespace dgr;

// Arguments of a forward launch of MS steps.
template <int NP, int MS> struct RpStepArgs {
  RpOp<NP> c;
  double bnd[MS * 5 + MS + 1];  // rp_block_bnd's layout
  int64_t n0;                   // global index of the launch's first step
  int32_t jend;                 // the launch ends the sweep (record u^{n0+MS} too)
};

template <int NP, int MS> struct RpAdjArgs {
  RpOp<NP> c;
  int64_t n0;
  int32_t has_eta;  // kEta* bits
};

template <int NP, bool UNI, int NW, int E, int MS>
__global__ __launch_bounds__(64 * NW) void k_step_rp(const double* __restrict__ uin,
                                                        double* __restrict__ rec,
                                                        double* __restrict__ last,
                                                        const double* __restrict__ scale,
                                                        RpStepArgs<NP, MS> args) {
  using G = RpGeo<NP, NW, E>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 6 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.c.xcd);
  constexpr int H = RpHalo<MS>::F;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  using SArgs = RpStepArgs<NP, MS>;
  const OpSrc<NP> os = op_src<NP>(
      args.c, kernarg_tail_k<decltype(&k_step_rp<NP, UNI, NW, E, MS>), SArgs>() + offsetof(SArgs, c));
  if (edge_tile(e0, G::T, args.c.ktot, args.c.K)) {
    // lane-indexed kernarg read, see step_tile
    const double* kb = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_step_rp<NP, UNI, NW, E, MS>), SArgs>() + offsetof(SArgs, bnd));
    rp_step_tile<NP, UNI, NW, E, MS, true, false>(lds, tile, uin, rec, last, scale, args.c, os,
                                                  kb, args.n0, args.jend);
  } else {
    rp_step_tile<NP, UNI, NW, E, MS, false, false>(lds, tile, uin, rec, last, scale, args.c, os,
                                                   nullptr, args.n0, args.jend);
  }
}

template <int NP, bool UNI, int NW, int E, int MS>
__global__ __launch_bounds__(64 * NW) void k_adj_rp(const double* __restrict__ win,
                                                       double* __restrict__ wout,
                                                       const double* __restrict__ rec,
                                                       double* __restrict__ eta,
                                                       const double* __restrict__ scale,
                                                       RpAdjArgs<NP, MS> args) {
  using G = RpGeo<NP, NW, E>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.c.xcd);
  constexpr int H = RpHalo<MS>::A;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  EtaSink es{eta, nullptr, nullptr, 0, 0, args.has_eta, false, 0.0, 0};
  using AArgs = RpAdjArgs<NP, MS>;
  const OpSrc<NP> os = op_src<NP>(
      args.c, kernarg_tail_k<decltype(&k_adj_rp<NP, UNI, NW, E, MS>), AArgs>() + offsetof(AArgs, c));
  if (edge_tile(e0, G::T, args.c.ktot, args.c.K))
    rp_adj_tile<NP, UNI, NW, E, MS, true, false>(lds, tile, win, wout, rec, es, scale, args.c, os,
                                                 args.n0);
  else
    rp_adj_tile<NP, UNI, NW, E, MS, false, false>(lds, tile, win, wout, rec, es, scale, args.c,
                                                  os, args.n0);
}

// The snapshot forward on pair tiles (dg_lserk4_fwd with DG_TUNE_SNAP_PAIRS): MS steps of the
// Horner-form body, every step's state stored (snap = u^{n0+1}, stride one field).
template <int NP, bool UNI, int NW, int MS>
__global__ __launch_bounds__(64 * NW) void k_step_rps(const double* __restrict__ uin,
                                                         double* __restrict__ snap,
                                                         const double* __restrict__ scale,
                                                         RpStepArgs<NP, MS> args) {
  using G = RpGeo<NP, NW, 2>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 6 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.c.xcd);
  constexpr int H = RpHalo<MS>::F;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  using SArgs = RpStepArgs<NP, MS>;
  const OpSrc<NP> os = op_src<NP>(
      args.c, kernarg_tail_k<decltype(&k_step_rps<NP, UNI, NW, MS>), SArgs>() + offsetof(SArgs, c));
  const int64_t field = args.c.ktot * NP;
  double* last = snap + (MS - 1) * field;
  if (edge_tile(e0, G::T, args.c.ktot, args.c.K)) {
    const double* kb = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_step_rps<NP, UNI, NW, MS>), SArgs>() + offsetof(SArgs, bnd));
    rp_step_tile<NP, UNI, NW, 2, MS, true, false, true>(lds, tile, uin, snap, last, scale, args.c,
                                                        os, kb, 0, false, field);
  } else {
    rp_step_tile<NP, UNI, NW, 2, MS, false, false, true>(lds, tile, uin, snap, last, scale,
                                                         args.c, os, nullptr, 0, false, field);
  }
}

template <int NP, int NW, int MS>
int rp_snap_e(const dg_plan* p, const double* in, double* snap, const double* times, double dt,
              hipStream_t st) {
  RpStepArgs<NP, MS> a;
  if (const int rc = rp_make_op<NP>(p, dt, &a.c)) return rc;
  rp_block_bnd(p, MS, times, dt, a.bnd);
  a.n0 = 0;
  a.jend = 0;
  constexpr int TE = RpGeo<NP, NW, 2>::T - 2 * RpHalo<MS>::F;
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_step_rps<NP, true, NW, MS>), dim3(grid), dim3(64 * NW), 0, st, in, snap,
                       p->d_scale, a);
  else
    hipLaunchKernelGGL((k_step_rps<NP, false, NW, MS>), dim3(grid), dim3(64 * NW), 0, st, in,
                       snap, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP>
int rp_snap_np(const dg_plan* p, int ms, const double* in, double* snap, const double* times,
               double dt, hipStream_t st) {
  const bool w2 = p->tile_width == 2;
  switch (ms) {
    case 8: return w2 ? rp_snap_e<NP, 8, 8>(p, in, snap, times, dt, st)
                      : rp_snap_e<NP, 4, 8>(p, in, snap, times, dt, st);
    case 4: return w2 ? rp_snap_e<NP, 8, 4>(p, in, snap, times, dt, st)
                      : rp_snap_e<NP, 4, 4>(p, in, snap, times, dt, st);
    case 2: return w2 ? rp_snap_e<NP, 8, 2>(p, in, snap, times, dt, st)
                      : rp_snap_e<NP, 4, 2>(p, in, snap, times, dt, st);
    case 1: return w2 ? rp_snap_e<NP, 8, 1>(p, in, snap, times, dt, st)
                      : rp_snap_e<NP, 4, 1>(p, in, snap, times, dt, st);
    default: break;
  }
  return fail(DG_ERR_ARG, "pair snapshot forward: 1, 2, 4 or 8 steps per launch");
}

template <int NP, int NW, int E, int MS>
int rp_step_e(const dg_plan* p, const double* in, double* rec, double* last, const double* times,
              double dt, hipStream_t st, int64_t n0, bool jend) {
  RpStepArgs<NP, MS> a;
  if (const int rc = rp_make_op<NP>(p, dt, &a.c)) return rc;
  rp_block_bnd(p, MS, times, dt, a.bnd);
  a.n0 = n0;
  a.jend = jend ? 1 : 0;
  constexpr int TE = RpGeo<NP, NW, E>::T - 2 * RpHalo<MS>::F;
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_step_rp<NP, true, NW, E, MS>), dim3(grid), dim3(64 * NW), 0, st, in,
                       rec, last, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_step_rp<NP, false, NW, E, MS>), dim3(grid), dim3(64 * NW), 0, st, in,
                       rec, last, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP, int NW, int E, int MS>
int rp_adj_e(const dg_plan* p, const double* win, double* wout, const double* rec, double* eta,
             int eta_mode, const double* /*t_next*/, double dt, hipStream_t st, int64_t n0) {
  RpAdjArgs<NP, MS> a;
  if (const int rc = rp_make_op<NP>(p, dt, &a.c)) return rc;
  a.n0 = n0;
  a.has_eta = eta != nullptr ? (eta_mode | kEtaOn) : 0;
  constexpr int TE = RpGeo<NP, NW, E>::T - 2 * RpHalo<MS>::A;
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_adj_rp<NP, true, NW, E, MS>), dim3(grid), dim3(64 * NW), 0, st, win,
                       wout, rec, eta, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_adj_rp<NP, false, NW, E, MS>), dim3(grid), dim3(64 * NW), 0, st, win,
                       wout, rec, eta, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

// Shapes: 2 elements per lane on workgroups of NW = 4 or 8 waves (the plan's rec_tile_width
// 1 / 2: tiles of 512 / 1024 elements), 1, 2, 4, 5, 8, 10, 16 or 20 steps per launch (16 and 20
// only at NW = 8: the cone leaves too few output elements of a 512-element tile); Np <= 9.
// Wider workgroups (10, 12, 16 waves: less halo per tile, and 10 waves fill the adjoint's 5
// waves per SIMD) were measured slower in both directions (profiles/r03/waves/: adjoint
// 180 -> 200-244 us per sweep, forward 157-166 -> 183-220 us): the per-stage barrier waits
// for more waves.
template <int NP, int NW>
int rp_step_w(const dg_plan* p, int ms, const double* in, double* rec, double* last,
              const double* times, double dt, hipStream_t st, int64_t n0, bool jend) {
  switch (ms) {
    case 20: if constexpr (NW == 8) return rp_step_e<NP, NW, 2, 20>(p, in, rec, last, times, dt, st, n0, jend); break;
    case 16: if constexpr (NW == 8) return rp_step_e<NP, NW, 2, 16>(p, in, rec, last, times, dt, st, n0, jend); break;
    case 10: return rp_step_e<NP, NW, 2, 10>(p, in, rec, last, times, dt, st, n0, jend);
    case 8: return rp_step_e<NP, NW, 2, 8>(p, in, rec, last, times, dt, st, n0, jend);
    case 5: return rp_step_e<NP, NW, 2, 5>(p, in, rec, last, times, dt, st, n0, jend);
    case 4: return rp_step_e<NP, NW, 2, 4>(p, in, rec, last, times, dt, st, n0, jend);
    case 2: return rp_step_e<NP, NW, 2, 2>(p, in, rec, last, times, dt, st, n0, jend);
    case 1: return rp_step_e<NP, NW, 2, 1>(p, in, rec, last, times, dt, st, n0, jend);
    default: break;
  }
  return fail(DG_ERR_ARG, "pair tiles: unsupported steps per launch for this tile width");
}

template <int NP, int NW>
int rp_adj_w(const dg_plan* p, int ms, const double* win, double* wout, const double* rec,
             double* eta, int em, const double* t_next, double dt, hipStream_t st, int64_t n0) {
  switch (ms) {
    case 20: if constexpr (NW == 8) return rp_adj_e<NP, NW, 2, 20>(p, win, wout, rec, eta, em, t_next, dt, st, n0); break;
    case 16: if constexpr (NW == 8) return rp_adj_e<NP, NW, 2, 16>(p, win, wout, rec, eta, em, t_next, dt, st, n0); break;
    case 10: return rp_adj_e<NP, NW, 2, 10>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 8: return rp_adj_e<NP, NW, 2, 8>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 5: return rp_adj_e<NP, NW, 2, 5>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 4: return rp_adj_e<NP, NW, 2, 4>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 2: return rp_adj_e<NP, NW, 2, 2>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 1: return rp_adj_e<NP, NW, 2, 1>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    default: break;
  }
  return fail(DG_ERR_ARG, "pair tiles: unsupported steps per launch for this tile width");
}

template <int NP>
int rp_step_np(const dg_plan* p, int ms, const double* in, double* rec, double* last,
               const double* times, double dt, hipStream_t st, int64_t n0, bool jend) {
  if (rec_fwd_width(p) == 2) return rp_step_w<NP, 8>(p, ms, in, rec, last, times, dt, st, n0, jend);
  return rp_step_w<NP, 4>(p, ms, in, rec, last, times, dt, st, n0, jend);
}

template <int NP>
int rp_adj_np(const dg_plan* p, int ms, const double* win, double* wout, const double* rec,
              double* eta, int em, const double* t_next, double dt, hipStream_t st, int64_t n0) {
  if (p->rec_tile_width == 2)
    return rp_adj_w<NP, 8>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
  return rp_adj_w<NP, 4>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
}

}  // namespace

namespace dgk {

int pair_launch_step_rec(const dg_plan* p, int ms, const double* in, double* rec, double* last,
                         const double* times, double dt, hipStream_t st, int64_t n0, bool jend) {
  switch (p->NP) {
    case 2: return rp_step_np<2>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 3: return rp_step_np<3>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 4: return rp_step_np<4>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 5: return rp_step_np<5>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 6: return rp_step_np<6>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 7: return rp_step_np<7>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 8: return rp_step_np<8>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 9: return rp_step_np<9>(p, ms, in, rec, last, times, dt, st, n0, jend);
    default: return fail(DG_ERR_ARG, "pair tiles support Np <= 9");
  }
}

int pair_launch_step_snap(const dg_plan* p, int ms, const double* in, double* snap,
                          const double* times, double dt, hipStream_t st) {
  switch (p->NP) {
    case 2: return rp_snap_np<2>(p, ms, in, snap, times, dt, st);
    case 3: return rp_snap_np<3>(p, ms, in, snap, times, dt, st);
    case 4: return rp_snap_np<4>(p, ms, in, snap, times, dt, st);
    case 5: return rp_snap_np<5>(p, ms, in, snap, times, dt, st);
    case 6: return rp_snap_np<6>(p, ms, in, snap, times, dt, st);
    case 7: return rp_snap_np<7>(p, ms, in, snap, times, dt, st);
    case 8: return rp_snap_np<8>(p, ms, in, snap, times, dt, st);
    case 9: return rp_snap_np<9>(p, ms, in, snap, times, dt, st);
    default: return fail(DG_ERR_ARG, "pair tiles support Np <= 9");
  }
}

int pair_launch_adj_rec(const dg_plan* p, int ms, const double* win, double* wout,
                        const double* rec, double* eta, int em, const double* t_next, double dt,
                        hipStream_t st, int64_t n0) {
  switch (p->NP) {
    case 2: return rp_adj_np<2>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 3: return rp_adj_np<3>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 4: return rp_adj_np<4>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 5: return rp_adj_np<5>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 6: return rp_adj_np<6>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 7: return rp_adj_np<7>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 8: return rp_adj_np<8>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 9: return rp_adj_np<9>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    default: return fail(DG_ERR_ARG, "pair tiles support Np <= 9");
  }
}

}  // namespace dgk
