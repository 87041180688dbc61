// EXPERIMENT (not built; kept for the record, DESIGN.md §5 "Pair tiles"): the record sweep pair on
// one-wave tiles of 8 elements per lane.  Measured bit-identical and 20 % slower than the pair
// tiles (forward 96-97 us vs 80 us per 10-step launch); the adjoint needed 256 VGPRs + AGPRs.
// dg_wrec.hip — the jump-record sweep pair on wave tiles (plan->rec_lane_elems == 8):
// one-wave workgroups, 8 consecutive elements per lane (512-element tiles), no workgroup
// barrier in the time loop.  Faces between a lane's own elements are register reads; the two
// that cross lanes move with DPP wave shifts (dg_wave.hip).  A stage's 8 element updates
// are independent (each reads its neighbours' pre-update faces), so the fp64 pipe has 8-way
// instruction-level parallelism inside one wave instead of waiting on a barrier and an LDS
// round trip per stage (the pair tiles' limiter).
//
// Same arithmetic per element as k_step / k_adj<..., REC = true> and the pair tiles: results
// are bit-identical at equal steps per launch.
// Sources: AdvecRHS1D (utils/AdvecRHS1D.m:9-19), the LSERK4 loop (utils/One_code.mlx:106-140),
// the indicator pattern (python/Main_finite_difference.py:54-94).
#include "dg_common.h"

namespace {
using namespace dgk;

__device__ __forceinline__ double wr_shr1(double x) {  // lane l <- lane l-1
  const long long b = __double_as_longlong(x);
  const int rl = __builtin_amdgcn_update_dpp(int(b), int(b), 0x138, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(int(b >> 32), int(b >> 32), 0x138, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}

__device__ __forceinline__ double wr_shl1(double x) {  // lane l <- lane l+1
  const long long b = __double_as_longlong(x);
  const int rl = __builtin_amdgcn_update_dpp(int(b), int(b), 0x130, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(int(b >> 32), int(b >> 32), 0x130, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}

constexpr int kWE = 8;            // elements per lane
constexpr int kWT = 64 * kWE;     // elements per tile

template <int NP> struct WrGeo {
  static constexpr int kTileD = kWT * NP + 2;
  static constexpr int kVec = (kTileD + 127) / 128;  // double2 loads per lane
};

__device__ __forceinline__ double2* wr_slot(double* rec, int64_t n, int64_t ktot, int64_t e) {
  return reinterpret_cast<double2*>(rec) + (n * ktot + e);  // = dg_advec.hip jump_slot
}

// Coalesced 16-byte loads of [e0, e0 + kWT) elements into LDS; returns the image offset.
template <int NP, bool EDGE>
__device__ __forceinline__ int wr_load(const double* __restrict__ g, int64_t e0, int64_t nd,
                                       double* __restrict__ lds) {
  using G = WrGeo<NP>;
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  const int off = int(d0 - base);
  const int nvec = (kWT * NP + off + 1) >> 1;
  const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g);
  double2 r[G::kVec];
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = int(threadIdx.x) + q * 64;
    const int64_t gd = base + 2 * int64_t(v);
    double2 val = make_double2(0.0, 0.0);
    if (v < nvec) {
      if (!EDGE || (gd >= 0 && gd + 1 < nd)) {
        val = g2[gd >> 1];
      } else {
        if (gd >= 0 && gd < nd) val.x = g[gd];
        if (gd + 1 >= 0 && gd + 1 < nd) val.y = g[gd + 1];
      }
    }
    r[q] = val;
  }
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = int(threadIdx.x) + q * 64;
    if (v < nvec) *reinterpret_cast<double2*>(&lds[2 * v]) = r[q];
  }
  return off;
}

template <int NP, bool UNI, int MS>
__global__ __launch_bounds__(64) void k_wstep_rec(const double* __restrict__ uin,
                                                  double* __restrict__ rec,
                                                  double* __restrict__ last,
                                                  const double* __restrict__ scale,
                                                  StepArgs<NP, 5, MS> args);

template <int NP, bool UNI, int MS, bool EDGE>
__device__ __forceinline__ void wr_step_tile(double* __restrict__ lds, int64_t tile,
                                             const double* __restrict__ uin,
                                             double* __restrict__ rec, double* __restrict__ last,
                                             const double* __restrict__ scale,
                                             const StepArgs<NP, 5, MS>& args) {
  constexpr int NS = 5, E = kWE, T = kWT;
  constexpr int H = MS * NS + 1;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  constexpr int CB = WrGeo<NP>::kTileD + 1;  // lds[CB + st*NS + s] = inflow value
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;

  const int off = wr_load<NP, EDGE>(uin, e0, nd, lds);
  if constexpr (EDGE) {
    using SArgs = StepArgs<NP, NS, MS>;  // lane-indexed kernarg read, see step_tile
    const double* ka = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_wstep_rec<NP, UNI, MS>), SArgs>() + offsetof(SArgs, uin));
    for (int i = lane; i <= MS * NS; i += 64) lds[CB + i] = ka[i];
  }
  __syncthreads();
  double ev[E][NE], od[E][NO], re[E][NE], ro[E][NO];
  Elem El[E];
  double sc[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    const double* us = lds + off + el * NP;
    to_eo<NP>(us, ev[m], od[m]);
    El[m] = elem_info<H, T, EDGE>(e0, el, args.ktot, args.K);
    sc[m] = args.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    if (args.n0 >= 1 && El[m].valid) {  // u^{n0}'s jumps from the staged nodal values
      const double uL = (EDGE && El[m].first) ? lds[CB] : us[-1];
      const double uR = (EDGE && El[m].last) ? us[NP - 1] : us[NP];
      const double du0 = us[0] - uL, du1 = us[NP - 1] - uR;
      *wr_slot(rec, args.n0 - 1, args.ktot, El[m].e) = double2{du0 - du1, du0 + du1};
    }
  }

#pragma unroll 1
  for (int st = 0; st < MS; ++st) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // the cross-lane faces of the pre-update state
      const double fromL = wr_shr1(ev[E - 1][0] - od[E - 1][0]);
      const double fromR = wr_shl1(ev[0][0] + od[0][0]);
      double uin_s = 0.0;
      if constexpr (EDGE) uin_s = lds[CB + st * NS + s];
      double prevN = fromL;  // the left neighbour's pre-update u_N
#pragma unroll
      for (int m = 0; m < E; ++m) {
        const double u0 = ev[m][0] + od[m][0], uN = ev[m][0] - od[m][0];
        double uL = prevN;
        double uR = (m == E - 1) ? fromR : ev[m + 1][0] + od[m + 1][0];
        prevN = uN;
        if constexpr (EDGE) {
          uL = El[m].first ? uin_s : uL;
          uR = El[m].last ? uN : uR;
        }
        const double dlt = uR - uL, sig = -(uL + uR);
        if (s == 0 && st >= 1 && El[m].valid) {  // u^{n0+st}'s jumps (record n0+st-1)
          const double du0 = u0 - uL, du1 = uN - uR;
          *wr_slot(rec, args.n0 + st - 1, args.ktot, El[m].e) = double2{du0 - du1, du0 + du1};
        }
        double pe[NE], po[NO];
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          double t = (UNI && s > 0) ? RK<NS>::A(s) * re[m][k] : args.op.Qeo[k * NO] * od[m][0];
#pragma unroll
          for (int j = (UNI && s > 0) ? 0 : 1; j < NO; ++j)
            t = fma(args.op.Qeo[k * NO + j], od[m][j], t);
          pe[k] = t;
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          double t = (UNI && s > 0) ? RK<NS>::A(s) * ro[m][k] : args.op.Qoe[k * NE] * ev[m][0];
#pragma unroll
          for (int j = (UNI && s > 0) ? 0 : 1; j < NE; ++j)
            t = fma(args.op.Qoe[k * NE + j], ev[m][j], t);
          po[k] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          if constexpr (UNI) {
            re[m][k] = fma(args.op.le[k], dlt, pe[k]);
          } else {
            const double a = sc[m] * fma(args.op.le[k], dlt, pe[k]);
            re[m][k] = (s == 0) ? a : fma(RK<NS>::A(s), re[m][k], a);
          }
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          if constexpr (UNI) {
            ro[m][k] = fma(args.op.lo[k], sig, po[k]);
          } else {
            const double a = sc[m] * fma(args.op.lo[k], sig, po[k]);
            ro[m][k] = (s == 0) ? a : fma(RK<NS>::A(s), ro[m][k], a);
          }
        }
      }
      // the state update after all elements read their neighbours' pre-update faces
#pragma unroll
      for (int m = 0; m < E; ++m) {
#pragma unroll
        for (int k = 0; k < NE; ++k) ev[m][k] = fma(RK<NS>::B(s), re[m][k], ev[m][k]);
#pragma unroll
        for (int k = 0; k < NO; ++k) od[m][k] = fma(RK<NS>::B(s), ro[m][k], od[m][k]);
      }
    }
  }
  if (args.jend) {  // the sweep's final state's jumps (record n0+MS-1), inflow at t_{n0+MS}
    const double fromL = wr_shr1(ev[E - 1][0] - od[E - 1][0]);
    const double fromR = wr_shl1(ev[0][0] + od[0][0]);
    double prevN = fromL;
#pragma unroll
    for (int m = 0; m < E; ++m) {
      const double u0 = ev[m][0] + od[m][0], uN = ev[m][0] - od[m][0];
      double uL = prevN;
      double uR = (m == E - 1) ? fromR : ev[m + 1][0] + od[m + 1][0];
      prevN = uN;
      if constexpr (EDGE) {
        uL = El[m].first ? lds[CB + MS * NS] : uL;
        uR = El[m].last ? uN : uR;
      }
      if (El[m].valid) {
        const double du0 = u0 - uL, du1 = uN - uR;
        *wr_slot(rec, args.n0 + MS - 1, args.ktot, El[m].e) = double2{du0 - du1, du0 + du1};
      }
    }
  }
  // u^{n0+MS} through the image (its last reads were before the time loop)
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    if (el >= H && el < T - H) from_eo<NP>(ev[m], od[m], lds + (el - H) * NP);
  }
  __syncthreads();
  const int64_t o0 = tile * TE * NP;
  if constexpr (EDGE) {
    const int64_t rem = nd - o0;
    store_run<64>(last, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
  } else {
    store_full<TE * NP, 64>(last, o0, lds);
  }
}

template <int NP, bool UNI, int MS>
__global__ __launch_bounds__(64) void k_wstep_rec(const double* __restrict__ uin,
                                                  double* __restrict__ rec,
                                                  double* __restrict__ last,
                                                  const double* __restrict__ scale,
                                                  StepArgs<NP, 5, MS> args) {
  __shared__ __attribute__((aligned(16))) double lds[WrGeo<NP>::kTileD + 2 + MS * 5 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = MS * 5 + 1;
  const int64_t e0 = tile * (kWT - 2 * H) - H;
  if (edge_tile(e0, kWT, args.ktot, args.K))
    wr_step_tile<NP, UNI, MS, true>(lds, tile, uin, rec, last, scale, args);
  else
    wr_step_tile<NP, UNI, MS, false>(lds, tile, uin, rec, last, scale, args);
}

template <int NP, int MS>
int wr_step_e(const dg_plan* p, const double* in, double* rec, double* last, const double* times,
              double dt, hipStream_t st, int64_t n0, bool jend) {
  StepArgs<NP, 5, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;
  for (int m = 0; m < MS; ++m)
    for (int s = 0; s < 5; ++s) a.uin[m * 5 + s] = inflow_value(p, times[m] + RK<5>::C(s) * dt);
  a.uin[MS * 5] = inflow_value(p, times[MS]);
  a.ktot = p->ktot;
  a.stride = p->ktot * NP;
  a.n0 = n0;
  a.K = int32_t(p->K);
  a.xcd = p->xcd_order;
  a.jend = jend ? 1 : 0;
  constexpr int TE = kWT - 2 * (MS * 5 + 1);
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_wstep_rec<NP, true, MS>), dim3(grid), dim3(64), 0, st, in, rec, last,
                       p->d_scale, a);
  else
    hipLaunchKernelGGL((k_wstep_rec<NP, false, MS>), dim3(grid), dim3(64), 0, st, in, rec, last,
                       p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP>
int wr_step_np(const dg_plan* p, int ms, const double* in, double* rec, double* last,
               const double* times, double dt, hipStream_t st, int64_t n0, bool jend) {
  switch (ms) {
    case 10: return wr_step_e<NP, 10>(p, in, rec, last, times, dt, st, n0, jend);
    case 8: return wr_step_e<NP, 8>(p, in, rec, last, times, dt, st, n0, jend);
    case 5: return wr_step_e<NP, 5>(p, in, rec, last, times, dt, st, n0, jend);
    case 4: return wr_step_e<NP, 4>(p, in, rec, last, times, dt, st, n0, jend);
    case 2: return wr_step_e<NP, 2>(p, in, rec, last, times, dt, st, n0, jend);
    case 1: return wr_step_e<NP, 1>(p, in, rec, last, times, dt, st, n0, jend);
    default: return fail(DG_ERR_ARG, "wave record tiles: 1, 2, 4, 5, 8 or 10 steps per launch");
  }
}

template <int NP, bool UNI, int MS>
__global__ __launch_bounds__(64) void k_wadj_rec(const double* __restrict__ win,
                                                 double* __restrict__ wout,
                                                 const double* __restrict__ rec,
                                                 double* __restrict__ eta,
                                                 const double* __restrict__ scale,
                                                 AdjArgs<NP, MS> args);

// Adjoint: MS reverse steps of the tile (terminal functionals: no source), the indicator from
// the recorded jumps.  See adj_tile (dg_advec.hip) for the arithmetic.  The next step's
// record loads are issued during the current step's last reverse stage.
template <int NP, bool UNI, int MS, bool EDGE>
__device__ __forceinline__ void wr_adj_tile(double* __restrict__ lds, int64_t tile,
                                            const double* __restrict__ win,
                                            double* __restrict__ wout,
                                            const double* __restrict__ rec,
                                            double* __restrict__ eta,
                                            const double* __restrict__ scale,
                                            const AdjArgs<NP, MS>& args) {
  constexpr int NS = 5, E = kWE, T = kWT;
  constexpr int H = MS * NS;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;
  const int64_t eL = e0 + E * lane;  // the lane's first element

  const int off = wr_load<NP, EDGE>(win, e0, nd, lds);
  double2 jn[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const bool in = !EDGE || (eL + m >= 0 && eL + m < args.ktot);
    jn[m] = in ? *wr_slot(const_cast<double*>(rec), args.n0 + MS - 1, args.ktot, eL + m)
               : double2{0.0, 0.0};
  }
  __syncthreads();
  double we[E][NE], wo[E][NO], eacc[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const double* w = lds + off + (E * lane + m) * NP;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[m][k] = w[k] + w[N - k];
      wo[m][k] = w[k] - w[N - k];
    }
    if constexpr (NE > NO) we[m][NO] = w[NO];
    eacc[m] = 0.0;
  }

#pragma unroll 1
  for (int st = MS - 1; st >= 0; --st) {
    if (args.has_eta) {
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double pe = 0.0, po = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) pe = fma(args.op.le[k], we[m][k], pe);
#pragma unroll
        for (int k = 0; k < NO; ++k) po = fma(args.op.lo[k], wo[m][k], po);
        double c = fma(jn[m].x, pe, jn[m].y * po);
        if constexpr (!UNI) {
          const Elem El = elem_info<H, T, EDGE>(e0, E * lane + m, args.ktot, args.K);
          c *= args.sc * (El.inrange ? scale[El.kl] : 0.0);
        }
        eacc[m] += c;
      }
    }
    double le_[E][NE], lo_[E][NO];
#pragma unroll
    for (int m = 0; m < E; ++m) {
#pragma unroll
      for (int k = 0; k < NE; ++k) le_[m][k] = 0.0;
#pragma unroll
      for (int k = 0; k < NO; ++k) lo_[m][k] = 0.0;
    }
#pragma unroll
    for (int ss = 0; ss < NS; ++ss) {
      const int s = NS - 1 - ss;
      if (ss == NS - 1 && st > 0) {  // the next step's record (u^{n0+st}'s jumps)
#pragma unroll
        for (int m = 0; m < E; ++m) {
          const bool in = !EDGE || (eL + m >= 0 && eL + m < args.ktot);
          if (in) jn[m] = *wr_slot(const_cast<double*>(rec), args.n0 + st - 1, args.ktot, eL + m);
        }
      }
      double g0[E], g1[E];
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double scm = 1.0;
        if constexpr (!UNI) {
          const Elem El = elem_info<H, T, EDGE>(e0, E * lane + m, args.ktot, args.K);
          scm = args.sc * (El.inrange ? scale[El.kl] : 0.0);
        }
        double qe[NE], qo[NO], gd = 0.0, gs = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          le_[m][k] = fma(RK<NS>::B(s), we[m][k], le_[m][k]);
          qe[k] = UNI ? le_[m][k] : scm * le_[m][k];
          gd = fma(args.op.le[k], qe[k], gd);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          lo_[m][k] = fma(RK<NS>::B(s), wo[m][k], lo_[m][k]);
          qo[k] = UNI ? lo_[m][k] : scm * lo_[m][k];
          gs = fma(args.op.lo[k], qo[k], gs);
        }
        g0[m] = gd + gs;
        g1[m] = gs - gd;
#pragma unroll
        for (int j = 0; j < NE; ++j) {
          double t = we[m][j];
#pragma unroll
          for (int k = 0; k < NO; ++k) t = fma(args.op.Qoe[k * NE + j], qo[k], t);
          we[m][j] = t;
        }
#pragma unroll
        for (int j = 0; j < NO; ++j) {
          double t = wo[m][j];
#pragma unroll
          for (int k = 0; k < NE; ++k) t = fma(args.op.Qeo[k * NO + j], qe[k], t);
          wo[m][j] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) le_[m][k] = RK<NS>::A(s) * le_[m][k];
#pragma unroll
        for (int k = 0; k < NO; ++k) lo_[m][k] = RK<NS>::A(s) * lo_[m][k];
      }
      // lane-1's last element's g1 / lane+1's first element's g0
      const double fromL = wr_shr1(g1[E - 1]), fromR = wr_shl1(g0[0]);
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double gl = (m == 0) ? fromL : g1[m - 1];
        double gr = (m == E - 1) ? fromR : g0[m + 1];
        if constexpr (EDGE) {
          const Elem El = elem_info<H, T, EDGE>(e0, E * lane + m, args.ktot, args.K);
          gl = El.first ? 0.0 : gl;
          gr = El.last ? g1[m] : gr;
        }
        we[m][0] -= gl + gr;
        wo[m][0] += gr - gl;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const Elem El = elem_info<H, T, EDGE>(e0, E * lane + m, args.ktot, args.K);
    if (args.has_eta && El.valid) eta_update(eta, El.e, eacc[m], args.has_eta);
  }
  // w^{n0} through the image (dual coordinates back to nodal)
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    if (el >= H && el < T - H) {
      double* o = lds + (el - H) * NP;
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        o[k] = 0.5 * (we[m][k] + wo[m][k]);
        o[N - k] = 0.5 * (we[m][k] - wo[m][k]);
      }
      if constexpr (NE > NO) o[NO] = we[m][NO];
    }
  }
  __syncthreads();
  const int64_t o0 = tile * TE * NP;
  if constexpr (EDGE) {
    const int64_t rem = nd - o0;
    store_run<64>(wout, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
  } else {
    store_full<TE * NP, 64>(wout, o0, lds);
  }
}

template <int NP, bool UNI, int MS>
__global__ __launch_bounds__(64) void k_wadj_rec(const double* __restrict__ win,
                                                 double* __restrict__ wout,
                                                 const double* __restrict__ rec,
                                                 double* __restrict__ eta,
                                                 const double* __restrict__ scale,
                                                 AdjArgs<NP, MS> args) {
  __shared__ __attribute__((aligned(16))) double lds[WrGeo<NP>::kTileD + 2];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = MS * 5;
  const int64_t e0 = tile * (kWT - 2 * H) - H;
  if (edge_tile(e0, kWT, args.ktot, args.K))
    wr_adj_tile<NP, UNI, MS, true>(lds, tile, win, wout, rec, eta, scale, args);
  else
    wr_adj_tile<NP, UNI, MS, false>(lds, tile, win, wout, rec, eta, scale, args);
}

template <int NP, int MS>
int wr_adj_e(const dg_plan* p, const double* win, double* wout, const double* rec, double* eta,
             int eta_mode, const double* t_next, double dt, hipStream_t st, int64_t n0) {
  AdjArgs<NP, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;
  for (int m = 0; m < MS; ++m) {
    a.uin_res[m] = inflow_value(p, t_next[m]);
    a.src[m] = 0.0;
  }
  a.ktot = p->ktot;
  a.stride = p->ktot * NP;
  a.n0 = n0;
  a.K = int32_t(p->K);
  a.has_eta = eta != nullptr ? (eta_mode | kEtaOn) : 0;
  a.xcd = p->xcd_order;
  constexpr int TE = kWT - 2 * MS * 5;
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_wadj_rec<NP, true, MS>), dim3(grid), dim3(64), 0, st, win, wout, rec,
                       eta, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_wadj_rec<NP, false, MS>), dim3(grid), dim3(64), 0, st, win, wout, rec,
                       eta, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP>
int wr_adj_np(const dg_plan* p, int ms, const double* win, double* wout, const double* rec,
              double* eta, int em, const double* t_next, double dt, hipStream_t st, int64_t n0) {
  switch (ms) {
    case 10: return wr_adj_e<NP, 10>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 8: return wr_adj_e<NP, 8>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 5: return wr_adj_e<NP, 5>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 4: return wr_adj_e<NP, 4>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 2: return wr_adj_e<NP, 2>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 1: return wr_adj_e<NP, 1>(p, win, wout, rec, eta, em, t_next, dt, st, n0);
    default: return fail(DG_ERR_ARG, "wave record tiles: 1, 2, 4, 5, 8 or 10 steps per launch");
  }
}

}  // namespace

namespace dgk {

int wave_launch_step_rec(const dg_plan* p, int ms, const double* in, double* rec, double* last,
                         const double* times, double dt, hipStream_t st, int64_t n0, bool jend) {
  switch (p->NP) {
    case 2: return wr_step_np<2>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 3: return wr_step_np<3>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 4: return wr_step_np<4>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 5: return wr_step_np<5>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 6: return wr_step_np<6>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 7: return wr_step_np<7>(p, ms, in, rec, last, times, dt, st, n0, jend);
    case 8: return wr_step_np<8>(p, ms, in, rec, last, times, dt, st, n0, jend);
    default: return fail(DG_ERR_ARG, "wave record tiles support Np <= 8");
  }
}

int wave_launch_adj_rec(const dg_plan* p, int ms, const double* win, double* wout,
                        const double* rec, double* eta, int em, const double* t_next, double dt,
                        hipStream_t st, int64_t n0) {
  switch (p->NP) {
    case 2: return wr_adj_np<2>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 3: return wr_adj_np<3>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 4: return wr_adj_np<4>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 5: return wr_adj_np<5>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 6: return wr_adj_np<6>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 7: return wr_adj_np<7>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    case 8: return wr_adj_np<8>(p, ms, win, wout, rec, eta, em, t_next, dt, st, n0);
    default: return fail(DG_ERR_ARG, "wave record tiles support Np <= 8");
  }
}

}  // namespace dgk
