// dg_wave.hip — wave-tile variants of the fused linear LSERK4 step kernels (see
// dg_advec.hip for the workgroup-tile kernels k_step / k_adj and DESIGN.md for the
// layout).  Selected per plan by DG_TUNE_LANE_ELEMENTS.
#include "dg_common.h"

namespace {
using namespace dgk;

// ---------------------------------------------------------------------------
// Wave tiles: one-wave workgroups, E consecutive elements per lane (tile T = 64*E), no
// workgroup barriers.  Faces between a lane's own elements are plain register reads; the
// two faces that cross lanes move with DPP wave shifts (row-crossing wave_shr:1 /
// wave_shl:1, two 32-bit moves per double).  LDS only stages the coalesced 16-byte tile
// loads and stores.  The E independent element chains per lane give the fp64 pipe
// instruction-level parallelism that the one-element-per-lane kernel gets only from
// other waves.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double dpp_shr1(double x) {  // lane l <- lane l-1 (lane 0 keeps x)
  const long long b = __double_as_longlong(x);
  const int lo = int(b), hi = int(b >> 32);
  const int rl = __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}

__device__ __forceinline__ double dpp_shl1(double x) {  // lane l <- lane l+1 (lane 63 keeps x)
  const long long b = __double_as_longlong(x);
  const int lo = int(b), hi = int(b >> 32);
  const int rl = __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}

template <int NP, int E, int MS, int NS> struct WaveGeo {
  static constexpr int LB = 64;
  static constexpr int T = 64 * E;
  static constexpr int H = MS * NS;
  static constexpr int TE = T - 2 * H;
  static constexpr int kTileD = T * NP + 2;
  static constexpr int kVec = (kTileD + 2 * LB - 1) / (2 * LB);  // double2 loads per lane
};

template <int NP, int NS, bool UNI, int E, int MS>
__global__ __launch_bounds__(64) void k_wstep(const double* __restrict__ uin,
                                              double* __restrict__ snap,
                                              double* __restrict__ last,
                                              const double* __restrict__ scale,
                                              StepArgs<NP, NS, MS> args);

template <int NP, int NS, bool UNI, int E, int MS, bool EDGE>
__device__ __forceinline__ void wstep_tile(double* __restrict__ lds, int64_t tile,
                                           const double* __restrict__ uin,
                                           double* __restrict__ snap, double* __restrict__ last,
                                           const double* __restrict__ scale,
                                           const StepArgs<NP, NS, MS>& args) {
  using G = WaveGeo<NP, E, MS, NS>;
  constexpr int T = G::T, H = G::H, TE = G::TE, LB = G::LB;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  constexpr int CB = G::kTileD;  // lds[CB + st*NS + s] = inflow value of that stage
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;
  const int64_t o0 = tile * TE * NP;
  const int64_t rem = nd - o0;
  const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;

  int off;
  {  // coalesced 16-byte loads of the tile image, staged through LDS
    const int64_t d0 = e0 * NP;
    const int64_t base = d0 & ~int64_t(1);
    off = int(d0 - base);
    const int nvec = (T * NP + off + 1) >> 1;
    const double2* __restrict__ g2 = reinterpret_cast<const double2*>(uin);
    double2 r[G::kVec];
#pragma unroll
    for (int q = 0; q < G::kVec; ++q) {
      const int v = lane + q * LB;
      const int64_t gd = base + 2 * int64_t(v);
      double2 val = make_double2(0.0, 0.0);
      if (v < nvec) {
        if (!EDGE || (gd >= 0 && gd + 1 < nd)) {
          val = g2[gd >> 1];
        } else {
          if (gd >= 0 && gd < nd) val.x = uin[gd];
          if (gd + 1 >= 0 && gd + 1 < nd) val.y = uin[gd + 1];
        }
      }
      r[q] = val;
    }
#pragma unroll
    for (int q = 0; q < G::kVec; ++q) {
      const int v = lane + q * LB;
      if (v < nvec) *reinterpret_cast<double2*>(&lds[2 * v]) = r[q];
    }
    if constexpr (EDGE) {
      using SArgs = StepArgs<NP, NS, MS>;  // kernarg read of uin[], see step_tile
      const double* ka = reinterpret_cast<const double*>(
          kernarg_tail<decltype(&k_wstep<NP, NS, UNI, E, MS>), SArgs>() + offsetof(SArgs, uin));
      if (lane < MS * NS) lds[CB + lane] = ka[lane];
    }
    __syncthreads();
  }
  double ev[E][NE], od[E][NO];
  Elem El[E];
  double sc[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    to_eo<NP>(lds + off + el * NP, ev[m], od[m]);
    El[m] = elem_info<H, T, EDGE>(e0, el, args.ktot, args.K);
    sc[m] = args.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
  }

  double re[E][NE], ro[E][NO];
#pragma unroll
  for (int st = 0; st < MS; ++st) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      double u0[E], uN[E];
#pragma unroll
      for (int m = 0; m < E; ++m) {
        u0[m] = ev[m][0] + od[m][0];
        uN[m] = ev[m][0] - od[m][0];
      }
      const double fromL = dpp_shr1(uN[E - 1]);  // lane l-1's last element, right face
      const double fromR = dpp_shl1(u0[0]);      // lane l+1's first element, left face
      double uin_s = 0.0;
      if constexpr (EDGE) uin_s = lds[CB + st * NS + s];
#pragma unroll
      for (int m = 0; m < E; ++m) {
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
        double uL = (m == 0) ? fromL : uN[m - 1];
        double uR = (m == E - 1) ? fromR : u0[m + 1];
        if constexpr (EDGE) {
          uL = El[m].first ? uin_s : uL;
          uR = El[m].last ? uN[m] : uR;
        }
        const double dlt = uR - uL, sig = -(uL + uR);  // folded operator (make_eo, fold)
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          if constexpr (UNI) {
            re[m][k] = fma(args.op.le[k], dlt, pe[k]);
          } else {
            const double a = sc[m] * fma(args.op.le[k], dlt, pe[k]);
            re[m][k] = (s == 0) ? a : fma(RK<NS>::A(s), re[m][k], a);
          }
          ev[m][k] = fma(RK<NS>::B(s), re[m][k], ev[m][k]);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          if constexpr (UNI) {
            ro[m][k] = fma(args.op.lo[k], sig, po[k]);
          } else {
            const double a = sc[m] * fma(args.op.lo[k], sig, po[k]);
            ro[m][k] = (s == 0) ? a : fma(RK<NS>::A(s), ro[m][k], a);
          }
          od[m][k] = fma(RK<NS>::B(s), ro[m][k], od[m][k]);
        }
      }
    }
    if (snap != nullptr || st == MS - 1) {
      __syncthreads();  // previous reads of the image are done
#pragma unroll
      for (int m = 0; m < E; ++m) {
        const int el = E * lane + m;
        if (el >= H && el < T - H) from_eo<NP>(ev[m], od[m], lds + (el - H) * NP);
      }
      __syncthreads();
      if constexpr (EDGE) {
        if (snap != nullptr) store_run<LB>(snap + st * args.stride, o0, count, lds);
        if (st == MS - 1 && last != nullptr) store_run<LB>(last, o0, count, lds);
      } else {
        if (snap != nullptr) store_full<TE * NP, LB>(snap + st * args.stride, o0, lds);
        if (st == MS - 1 && last != nullptr) store_full<TE * NP, LB>(last, o0, lds);
      }
    }
  }
}

template <int NP, int NS, bool UNI, int E, int MS>
__global__ __launch_bounds__(64) void k_wstep(const double* __restrict__ uin,
                                              double* __restrict__ snap,
                                              double* __restrict__ last,
                                              const double* __restrict__ scale,
                                              StepArgs<NP, NS, MS> args) {
  using G = WaveGeo<NP, E, MS, NS>;
  __shared__ __attribute__((aligned(16))) double lds[G::kTileD + MS * NS];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  const int64_t e0 = tile * G::TE - G::H;
  if (edge_tile(e0, G::T, args.ktot, args.K))
    wstep_tile<NP, NS, UNI, E, MS, true>(lds, tile, uin, snap, last, scale, args);
  else
    wstep_tile<NP, NS, UNI, E, MS, false>(lds, tile, uin, snap, last, scale, args);
}


template <int NP, int E, int MS>
int launch_wstep_e(const dg_plan* p, const double* in, double* snap, double* last,
                   const double* times, double dt, hipStream_t st) {
  StepArgs<NP, 5, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;
  for (int m = 0; m < MS; ++m)
    for (int s = 0; s < 5; ++s) a.uin[m * 5 + s] = inflow_value(p, times[m] + RK<5>::C(s) * dt);
  a.ktot = p->ktot;
  a.stride = p->ktot * NP;
  a.K = int32_t(p->K);
  a.xcd = p->xcd_order;
  a.uin[MS * 5] = 0.0;  // (no jump record on the wave path)
  a.n0 = 0;
  a.jend = 0;
  constexpr int TE = WaveGeo<NP, E, MS, 5>::TE;
  const unsigned grid = grid_for(p->ktot, TE);
  if (p->uniform)
    hipLaunchKernelGGL((k_wstep<NP, 5, true, E, MS>), dim3(grid), dim3(64), 0, st, in, snap,
                       last, p->d_scale, a);
  else
    hipLaunchKernelGGL((k_wstep<NP, 5, false, E, MS>), dim3(grid), dim3(64), 0, st, in, snap,
                       last, p->d_scale, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP>
int wstep_np(const dg_plan* p, int ms, const double* in, double* snap, double* last,
             const double* times, double dt, hipStream_t st) {
  if (p->lane_elems == 8) {
    if (ms == 8) return launch_wstep_e<NP, 8, 8>(p, in, snap, last, times, dt, st);
    if (ms == 4) return launch_wstep_e<NP, 8, 4>(p, in, snap, last, times, dt, st);
    if (ms == 2) return launch_wstep_e<NP, 8, 2>(p, in, snap, last, times, dt, st);
    return launch_wstep_e<NP, 8, 1>(p, in, snap, last, times, dt, st);
  }
  if (p->lane_elems == 4) {
    if (ms == 8) return launch_wstep_e<NP, 4, 8>(p, in, snap, last, times, dt, st);
    if (ms == 4) return launch_wstep_e<NP, 4, 4>(p, in, snap, last, times, dt, st);
    if (ms == 2) return launch_wstep_e<NP, 4, 2>(p, in, snap, last, times, dt, st);
    if (ms == 1) return launch_wstep_e<NP, 4, 1>(p, in, snap, last, times, dt, st);
    return fail(DG_ERR_ARG, "wave tiles: unsupported steps per launch");
  }
  // 2 elements per lane: a 128-element tile leaves no room for the 8-step cone
  // (effective_msteps caps these plans at 4)
  if (ms == 4) return launch_wstep_e<NP, 2, 4>(p, in, snap, last, times, dt, st);
  if (ms == 2) return launch_wstep_e<NP, 2, 2>(p, in, snap, last, times, dt, st);
  if (ms == 1) return launch_wstep_e<NP, 2, 1>(p, in, snap, last, times, dt, st);
  return fail(DG_ERR_ARG, "wave tiles of 2 elements per lane take at most 4 steps per launch");
}

}  // namespace

namespace dgk {

int wave_launch_step(const dg_plan* p, int ms, const double* in, double* snap, double* last,
                     const double* times, double dt, hipStream_t st) {
  int rc = DG_OK;
  switch (p->NP) {
    case 2: rc = wstep_np<2>(p, ms, in, snap, last, times, dt, st); break;
    case 3: rc = wstep_np<3>(p, ms, in, snap, last, times, dt, st); break;
    case 4: rc = wstep_np<4>(p, ms, in, snap, last, times, dt, st); break;
    case 5: rc = wstep_np<5>(p, ms, in, snap, last, times, dt, st); break;
    case 6: rc = wstep_np<6>(p, ms, in, snap, last, times, dt, st); break;
    case 7: rc = wstep_np<7>(p, ms, in, snap, last, times, dt, st); break;
    case 8: rc = wstep_np<8>(p, ms, in, snap, last, times, dt, st); break;
    default: return fail(DG_ERR_ARG, "wave tiles support Np <= 8");
  }
  return rc;
}

}  // namespace dgk
