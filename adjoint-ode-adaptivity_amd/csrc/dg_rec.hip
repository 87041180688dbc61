// dg_rec.hip — the jump-record sweep pair (dg_lserk4_fwd_rec / dg_lserk4_adj_rec) on
// workgroup tiles with E consecutive elements per lane ("pair tiles", plan->rec_lane_elems).
//
// Same arithmetic per element as k_step / k_adj<..., REC = true> in dg_advec.hip (so the
// results are bit-identical at equal steps per launch); what changes is the layout:
//   - lane l owns tile elements E*l .. E*l+E-1.  The face between a lane's own elements is a
//     register read; only the lane's outer two faces go through LDS, so a stage writes and
//     reads half the LDS words per element and a barrier covers twice the elements;
//   - the E independent element chains per lane give the fp64 pipe instruction-level
//     parallelism between a stage's barrier and its update;
//   - a 256*W-lane workgroup covers 256*W*E elements: 512 per tile on 4 waves (W = 1) or
//     1024 on 8 waves (W = 2, the default with 10 steps per launch: 41 KB of LDS, 3
//     workgroups per CU);
//   - the face arrays alias the staging image (one barrier after the image is read and one
//     before it is rewritten, per launch);
//   - launches of 5, 10, 16 or 20 steps (no one-element-per-lane counterpart).
// Measured (N = 4, K = 2^20, bench, A/B pairs on one box, DESIGN.md §5 "Pair tiles"): with
// 8 + 8 + 4 launches 5.86-5.98e11 DOF-updates/s on 512-element tiles against 5.67-5.72e11 for
// the one-element-per-lane record kernels; 10 + 10 launches 6.07-6.12e11 (W = 1) and
// 6.15-6.16e11 (W = 2, the default).  Four elements per lane, raised wave priority, an
// unrolled step loop, no scheduling pins, 6 waves per SIMD for the adjoint: no gain.
// Sources: AdvecRHS1D (utils/AdvecRHS1D.m:9-19), the LSERK4 loop (utils/One_code.mlx:106-140),
// the indicator pattern (python/Main_finite_difference.py:54-94); DESIGN.md §5.
#include "dg_common.h"

namespace {
using namespace dgk;

template <int NP, int NW, int E> struct RpGeo {
  static constexpr int LB = 64 * NW;  // lanes per workgroup
  static constexpr int T = E * LB;       // elements per tile (incl. halo)
  static constexpr int kTileD = T * NP + 2;  // staging image (+2: 16-byte realignment)
  static constexpr int kVec = (kTileD + 2 * LB - 1) / (2 * LB);  // double2 loads per lane
  static constexpr int kFaceD = 4 * (LB + 2);  // 2 double-buffered lane-face arrays, padded
  static constexpr int kLds = ((kTileD > kFaceD ? kTileD : kFaceD) + 1) & ~1;
};

// Coalesced 16-byte loads of the tile image [e0, e0 + T) (zeros outside [0, nd)), issued
// together, then written to LDS.  Returns the image's offset (0 or 1 double).
template <int NP, int NW, int E, bool EDGE>
__device__ __forceinline__ int rp_load(const double* __restrict__ g, int64_t e0, int64_t nd,
                                       double* __restrict__ lds) {
  using G = RpGeo<NP, NW, E>;
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  const int off = int(d0 - base);
  const int nvec = (G::T * NP + off + 1) >> 1;
  const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g);
  double2 r[G::kVec];
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = int(threadIdx.x) + q * G::LB;
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
    const int v = int(threadIdx.x) + q * G::LB;
    if (v < nvec) *reinterpret_cast<double2*>(&lds[2 * v]) = r[q];
  }
  return off;
}

// The TE interior elements from registers to the image (nodal; `dual`: from the adjoint's
// dual coordinates), then 16-byte stores.  Callers barrier before (face reads done).
template <int NP, int NW, int E, int H, bool EDGE>
__device__ __forceinline__ void rp_store(double* __restrict__ g, int64_t o0, int64_t nd,
                                         double* __restrict__ lds,
                                         const double (*ev)[(NP + 1) / 2],
                                         const double (*od)[NP / 2], bool dual) {
  using G = RpGeo<NP, NW, E>;
  constexpr int T = G::T, TE = T - 2 * H;
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  const int lane = threadIdx.x;
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    if (el >= H && el < T - H) {
      double* o = lds + (el - H) * NP;
      if (dual) {
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          o[k] = 0.5 * (ev[m][k] + od[m][k]);
          o[N - k] = 0.5 * (ev[m][k] - od[m][k]);
        }
        if constexpr (NE > NO) o[NO] = ev[m][NO];
      } else {
        from_eo<NP>(ev[m], od[m], o);
      }
    }
  }
  __syncthreads();
  if constexpr (EDGE) {
    const int64_t rem = nd - o0;
    store_run<G::LB>(g, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
  } else {
    store_full<TE * NP, G::LB>(g, o0, lds);
  }
}

// Halo widths (elements per side): the forward's stage cone MS*5 + the final state's
// neighbours, the adjoint's MS*5; both rounded up to even, so every lane's element pair starts
// at an even element and its two record entries are one aligned 16-byte access.
template <int MS> struct RpHalo {
  static constexpr int F = (MS * 5 + 2) & ~1;
  static constexpr int A = (MS * 5 + 1) & ~1;
};

// Record row n: the lane's two left-face jumps (dg_common.h rec_ld), one 16-byte store; an
// edge tile stores them one by one where its valid range ends between them.
template <bool EDGE>
__device__ __forceinline__ void rp_rec_put(double* __restrict__ rec, int64_t n, int64_t ktot,
                                           const Elem* El, double j0, double j1) {
  double* row = rec + n * rec_ld(ktot);
  if (!EDGE || (El[0].valid && El[1].valid)) {
    if (El[0].valid) *reinterpret_cast<double2*>(row + El[0].e) = double2{j0, j1};
  } else {
    if (El[0].valid) row[El[0].e] = j0;
    if (El[1].valid) row[El[1].e] = j1;
  }
}

// Record row n for the lane's pair starting at element ea (even): j_ea, j_ea+1 and the right
// neighbour's j_ea+2.  Interior tiles never reach a trajectory's end, so all three are in
// range; edge tiles read zeros outside [0, ktot).
template <bool EDGE>
__device__ __forceinline__ void rp_rec_get(const double* __restrict__ rec, int64_t n,
                                           int64_t ktot, int64_t ea, double2& j01, double& j2) {
  const double* row = rec + n * rec_ld(ktot);
  if constexpr (!EDGE) {
    j01 = *reinterpret_cast<const double2*>(row + ea);
    j2 = row[ea + 2];
  } else {
    j01.x = (ea >= 0 && ea < ktot) ? row[ea] : 0.0;
    j01.y = (ea + 1 >= 0 && ea + 1 < ktot) ? row[ea + 1] : 0.0;
    j2 = (ea + 2 >= 0 && ea + 2 < ktot) ? row[ea + 2] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// The LSERK4 step as its stability polynomial, in Horner form (round 3).
//
// For the linear sweep du/dt = L u + (inflow at a trajectory's first element) the five
// low-storage stages (utils/One_code.mlx:120-137, coefficients utils/Globals1D.m:19-34) are
//   u^{n+1} = P(z) u^n + sum_{k<5} z^k zb b_k,    P(z) = sum_{k<=5} beta_k z^k,  z = dt L,
// zb the lift of a left boundary value and b_k = sum_s g_{s,k} uin(t_n + c_s dt) (the stage
// inflow values' weights, rk_poly below).  Evaluated as
//   t = beta_4 u + beta_5 Z_{b_4/beta_5}(u);  t = beta_k u + Z_{b_k}(t), k = 3, 2, 1;
//   u^{n+1} = u + Z_{b_0}(t),          Z_b(v) = z v + zb b  (b: the first element's uL)
// it is still five applications of z -- five face exchanges per step -- but 125 fp64
// operations per element-step at Np = 5 instead of the stage loop's 155 (no low-storage
// carry A_s r, no B_s update), and the adjoint's P(z^T) w 135 instead of 170.  Equal to the
// stage loop to rounding: 2e-16 relative per step (profiles/r03/horner_check.py; the oracle
// keeps the stage loop).  beta_0 = beta_1 = 1 exactly in double (checked on the host), so the
// last two levels take u itself as the accumulator's start.
// ---------------------------------------------------------------------------
struct RkPoly {
  double beta[6];   // P(z) = sum_k beta_k z^k
  double g[5][5];   // g[s][k]: weight of stage s's inflow value in b_k
  bool ok;
};

// The polynomial coefficients from the stage recursion (r = A_s r + z u + zb uin_s;
// u = u + B_s r) on coefficient vectors in z, in long double, rounded once.
inline const RkPoly& rk_poly() {
  static const RkPoly P = [] {
    long double uc[6] = {1}, rc[6] = {0}, uf[5][6] = {}, rf[5][6] = {};
    for (int s = 0; s < 5; ++s) {
      const long double A = RK<5>::A(s), B = RK<5>::B(s);
      for (int k = 5; k >= 0; --k) rc[k] = A * rc[k] + (k ? uc[k - 1] : 0.0L);
      for (int q = 0; q < 5; ++q)
        for (int k = 5; k >= 0; --k)
          rf[q][k] = A * rf[q][k] + (k ? uf[q][k - 1] : 0.0L) + ((q == s && k == 0) ? 1.0L : 0.0L);
      for (int k = 0; k < 6; ++k) uc[k] += B * rc[k];
      for (int q = 0; q < 5; ++q)
        for (int k = 0; k < 6; ++k) uf[q][k] += B * rf[q][k];
    }
    RkPoly r{};
    for (int k = 0; k < 6; ++k) r.beta[k] = double(uc[k]);
    for (int q = 0; q < 5; ++q)
      for (int k = 0; k < 5; ++k) r.g[q][k] = double(uf[q][k]);
    r.ok = r.beta[0] == 1.0 && r.beta[1] == 1.0 && r.beta[5] != 0.0;
    return r;
  }();
  return P;
}

// Arguments of a forward launch of MS steps.
template <int NP, int MS> struct RpStepArgs {
  EOArgs<NP> op;
  double sc;                    // dt (non-uniform meshes multiply by scale[k]; uniform: in op)
  double beta[6];               // P's coefficients
  double bnd[MS * 5 + MS + 1];  // step st, level l = 0..4: bnd[5 st + l] = b_4/beta_5, b_3,
                                // b_2, b_1, b_0; then bnd[5 MS + st] = uin(t_{n0+st}), the
                                // record's inflow value, st = 0..MS
  int64_t ktot;
  int64_t n0;                   // global index of the launch's first step
  int32_t K;
  int32_t xcd;
  int32_t jend;                 // the launch ends the sweep (record u^{n0+MS} too)
};

template <int NP, int MS> struct RpAdjArgs {
  EOArgs<NP> op;
  double sc;
  double beta[6];
  int64_t ktot;
  int64_t n0;
  int32_t K;
  int32_t has_eta;  // kEta* bits
  int32_t xcd;
};

template <int NP, bool UNI, int NW, int E, int MS>
__global__ __launch_bounds__(64 * NW) void k_step_rp(const double* __restrict__ uin,
                                                        double* __restrict__ rec,
                                                        double* __restrict__ last,
                                                        const double* __restrict__ scale,
                                                        RpStepArgs<NP, MS> args);

// Forward: MS steps of the tile; records u^{n0}..u^{n0+MS-1}'s jumps (and u^{n0+MS}'s when
// the launch ends the sweep), writes u^{n0+MS} to `last`.  Per step five Horner levels, each
// one face exchange of its input vector v (u at level 0, t after) through LDS.
template <int NP, bool UNI, int NW, int E, int MS, bool EDGE>
__device__ __forceinline__ void rp_step_tile(double* __restrict__ lds, int64_t tile,
                                             const double* __restrict__ uin,
                                             double* __restrict__ rec, double* __restrict__ last,
                                             const double* __restrict__ scale,
                                             const RpStepArgs<NP, MS>& args) {
  using G = RpGeo<NP, NW, E>;
  constexpr int T = G::T, LB = G::LB;
  constexpr int H = RpHalo<MS>::F;  // the level cone + the final state's neighbours, even
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0 && H % 2 == 0 && E == 2, "pair tiles: aligned pairs");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  constexpr int CB = G::kLds;  // lds[CB + i] = args.bnd[i] (edge tiles)
  constexpr int CR = CB + MS * 5;  // the record's inflow values
  constexpr int FB = LB + 2;   // one face array
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;

  const int off = rp_load<NP, NW, E, EDGE>(uin, e0, nd, lds);
  if constexpr (EDGE) {
    using SArgs = RpStepArgs<NP, MS>;  // lane-indexed kernarg read, see step_tile
    const double* ka = reinterpret_cast<const double*>(
        kernarg_tail<decltype(&k_step_rp<NP, UNI, NW, E, MS>), SArgs>() + offsetof(SArgs, bnd));
    if (lane <= MS * 6) lds[CB + lane] = ka[lane];
  }
  __syncthreads();
  double ue[E][NE], uo[E][NO];  // u in even/odd coordinates
  Elem El[E];
  double sc[E], jv[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    const double* us = lds + off + el * NP;
    to_eo<NP>(us, ue[m], uo[m]);
    El[m] = elem_info<H, T, EDGE>(e0, el, args.ktot, args.K);
    sc[m] = args.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    // u^{n0}'s left-face jumps (record n0-1) from the staged nodal values, as step_tile
    jv[m] = us[0] - ((EDGE && El[m].first) ? lds[CR] : us[-1]);
  }
  if (args.n0 >= 1) rp_rec_put<EDGE>(rec, args.n0 - 1, args.ktot, El, jv[0], jv[1]);
  __syncthreads();  // the image is read: the face arrays alias it

  const double b4 = args.beta[4], b5 = args.beta[5], b3 = args.beta[3], b2 = args.beta[2];
  double te[E][NE], to[E][NO];  // the Horner accumulator t
  // The step loop stays rolled; the level loop inside is unrolled.
#pragma unroll 1
  for (int st = 0; st < MS; ++st) {
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      const int fL = ((st * 5 + l) & 1) * 2 * FB;  // buffers alternate over the global level
      const int fR = fL + FB;
      // the level's input v: u at level 0, t after
      double v0[E], vN[E];
#pragma unroll
      for (int m = 0; m < E; ++m) {
        const double e = (l == 0) ? ue[m][0] : te[m][0], o = (l == 0) ? uo[m][0] : to[m][0];
        v0[m] = e + o;
        vN[m] = e - o;
      }
      lds[fL + lane + 1] = v0[0];      // the lane's left face
      lds[fR + lane + 1] = vN[E - 1];  // the lane's right face
      __builtin_amdgcn_sched_barrier(0);
      // Volume part, before the barrier: pe = c u + Qeo vo, po = c u + Qoe ve on uniform
      // meshes (c = beta_{4-l}; level 0 has no u term here, c = 1 from level 3 on), the bare
      // products on non-uniform ones (the metric multiplies them after the lift).
      double pe[E][NE], po[E][NO];
#pragma unroll
      for (int m = 0; m < E; ++m) {
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          const double* vo = (l == 0) ? uo[m] : to[m];
          double a;
          int j0 = 0;
          if (UNI && l >= 3) {
            a = ue[m][k];
          } else if (UNI && l >= 1) {
            a = (l == 1 ? b3 : b2) * ue[m][k];
          } else {
            a = args.op.Qeo[k * NO] * vo[0];
            j0 = 1;
          }
#pragma unroll
          for (int j = j0; j < NO; ++j) a = fma(args.op.Qeo[k * NO + j], vo[j], a);
          pe[m][k] = a;
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          const double* ve = (l == 0) ? ue[m] : te[m];
          double a;
          int j0 = 0;
          if (UNI && l >= 3) {
            a = uo[m][k];
          } else if (UNI && l >= 1) {
            a = (l == 1 ? b3 : b2) * uo[m][k];
          } else {
            a = args.op.Qoe[k * NE] * ve[0];
            j0 = 1;
          }
#pragma unroll
          for (int j = j0; j < NE; ++j) a = fma(args.op.Qoe[k * NE + j], ve[j], a);
          po[m][k] = a;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(pe[m][k]);
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(po[m][k]);
      }
      __syncthreads();
      // lane-1's right face / lane+1's left face (the pads feed halo elements only)
      const double fromL = lds[fR + lane], fromR = lds[fL + lane + 2];
      double bnd = 0.0, urec = 0.0;
      if constexpr (EDGE) {
        bnd = lds[CB + st * 5 + l];
        if (l == 0) urec = lds[CR + st];
      }
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double vL = (m == 0) ? fromL : vN[m - 1];
        double vR = (m == E - 1) ? fromR : v0[m + 1];
        if (l == 0) jv[m] = v0[m] - ((EDGE && El[m].first) ? urec : vL);  // u^{n0+st}'s jump
        if constexpr (EDGE) {
          vL = El[m].first ? bnd : vL;
          vR = El[m].last ? vN[m] : vR;
        }
        const double dlt = vR - vL, sig = -(vL + vR);
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          const double z = fma(args.op.le[k], dlt, pe[m][k]);
          if constexpr (UNI) {
            if (l == 0) te[m][k] = fma(b5, z, b4 * ue[m][k]);
            else if (l < 4) te[m][k] = z;
            else ue[m][k] = z;
          } else {
            if (l == 0) te[m][k] = fma(b5 * sc[m], z, b4 * ue[m][k]);
            else if (l < 3) te[m][k] = fma(sc[m], z, (l == 1 ? b3 : b2) * ue[m][k]);
            else if (l == 3) te[m][k] = fma(sc[m], z, ue[m][k]);
            else ue[m][k] = fma(sc[m], z, ue[m][k]);
          }
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          const double z = fma(args.op.lo[k], sig, po[m][k]);
          if constexpr (UNI) {
            if (l == 0) to[m][k] = fma(b5, z, b4 * uo[m][k]);
            else if (l < 4) to[m][k] = z;
            else uo[m][k] = z;
          } else {
            if (l == 0) to[m][k] = fma(b5 * sc[m], z, b4 * uo[m][k]);
            else if (l < 3) to[m][k] = fma(sc[m], z, (l == 1 ? b3 : b2) * uo[m][k]);
            else if (l == 3) to[m][k] = fma(sc[m], z, uo[m][k]);
            else uo[m][k] = fma(sc[m], z, uo[m][k]);
          }
        }
      }
      if (l == 0 && st >= 1) rp_rec_put<EDGE>(rec, args.n0 + st - 1, args.ktot, El, jv[0], jv[1]);
    }
  }
  if (args.jend) {
    // the sweep's final state u^{n0+MS}: one more face exchange for its jumps (record
    // n0+MS-1), inflow at t_{n0+MS}
    const int fL = ((MS * 5) & 1) * 2 * FB, fR = fL + FB;
    double u0[E], uN[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
      u0[m] = ue[m][0] + uo[m][0];
      uN[m] = ue[m][0] - uo[m][0];
    }
    lds[fL + lane + 1] = u0[0];
    lds[fR + lane + 1] = uN[E - 1];
    __syncthreads();
    const double fromL = lds[fR + lane];
#pragma unroll
    for (int m = 0; m < E; ++m) {
      double uL = (m == 0) ? fromL : uN[m - 1];
      if constexpr (EDGE) uL = El[m].first ? lds[CR + MS] : uL;
      jv[m] = u0[m] - uL;
    }
    rp_rec_put<EDGE>(rec, args.n0 + MS - 1, args.ktot, El, jv[0], jv[1]);
  }
  __syncthreads();  // the last face reads are done: the image is rewritten
  rp_store<NP, NW, E, H, EDGE>(last, tile * TE * NP, nd, lds, ue, uo, false);
}

template <int NP, bool UNI, int NW, int E, int MS>
__global__ __launch_bounds__(64 * NW) void k_step_rp(const double* __restrict__ uin,
                                                        double* __restrict__ rec,
                                                        double* __restrict__ last,
                                                        const double* __restrict__ scale,
                                                        RpStepArgs<NP, MS> args) {
  using G = RpGeo<NP, NW, E>;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MS * 6 + 1];
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = RpHalo<MS>::F;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  if (edge_tile(e0, G::T, args.ktot, args.K))
    rp_step_tile<NP, UNI, NW, E, MS, true>(lds, tile, uin, rec, last, scale, args);
  else
    rp_step_tile<NP, UNI, NW, E, MS, false>(lds, tile, uin, rec, last, scale, args);
}

// Adjoint: MS reverse steps st = MS-1..0 of the tile, each
//   eta += DWR(u^{n0+st+1}'s recorded jumps, w^{n0+st+1});  w^{n0+st} = P(z^T) w^{n0+st+1}
// (terminal functionals only: no source; the inflow forcing does not depend on u).  Horner
// in z^T: t = beta_4 w + beta_5 z^T w; t = beta_k w + z^T t, k = 3, 2, 1; w = w + z^T t, with
// z^T v = L^T (sc v): the face adjoints g0 = le.ve + lo.vo, g1 = lo.vo - le.ve of each element
// go to its neighbours (one exchange per level), the transposed volume blocks stay local.
template <int NP, bool UNI, int NW, int E, int MS, bool EDGE>
__device__ __forceinline__ void rp_adj_tile(double* __restrict__ lds, int64_t tile,
                                            const double* __restrict__ win,
                                            double* __restrict__ wout,
                                            const double* __restrict__ rec,
                                            double* __restrict__ eta,
                                            const double* __restrict__ scale,
                                            const RpAdjArgs<NP, MS>& args) {
  using G = RpGeo<NP, NW, E>;
  constexpr int T = G::T, LB = G::LB;
  constexpr int H = RpHalo<MS>::A;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0 && H % 2 == 0 && E == 2, "pair tiles: aligned pairs");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  constexpr int FB = LB + 2;
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;
  const int64_t ea = e0 + E * lane;  // the lane's first element (even)

  const int off = rp_load<NP, NW, E, EDGE>(win, e0, nd, lds);
  // the left-face jumps of u^{n0+st+1} (record n0+st) of the lane's two elements and of its
  // right neighbour: one 16-byte and one 8-byte load per lane and step, prefetched a step ahead
  double2 jn;
  double jn2;
  rp_rec_get<EDGE>(rec, args.n0 + MS - 1, args.ktot, ea, jn, jn2);
  __syncthreads();
  double we[E][NE], wo[E][NO];
  Elem El[E];
  double sc[E], eacc[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = E * lane + m;
    const double* w = lds + off + el * NP;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[m][k] = w[k] + w[N - k];
      wo[m][k] = w[k] - w[N - k];
    }
    if constexpr (NE > NO) we[m][NO] = w[NO];
    El[m] = elem_info<H, T, EDGE>(e0, el, args.ktot, args.K);
    sc[m] = args.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    eacc[m] = 0.0;
  }
  __syncthreads();  // the image is read: the face arrays alias it

  const double b4 = args.beta[4], b5 = args.beta[5], b3 = args.beta[3], b2 = args.beta[2];
  double te[E][NE], to[E][NO];  // the Horner accumulator
#pragma unroll 1
  for (int st = MS - 1; st >= 0; --st) {
    // du0 = j_e; du1 = -j_{e+1} (0 at a trajectory's last element): du0 - du1 and du0 + du1
    // are the snapshot path's doubles bit for bit (dg_common.h rec_ld).  The next step's
    // record is loaded after this step's indicator has read the current one.
    const double jc[E + 1] = {jn.x, jn.y, jn2};
    if (args.has_eta) {
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double pe = 0.0, po = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) pe = fma(args.op.le[k], we[m][k], pe);
#pragma unroll
        for (int k = 0; k < NO; ++k) po = fma(args.op.lo[k], wo[m][k], po);
        const bool lst = EDGE && El[m].last;
        const double dd = lst ? jc[m] : jc[m] + jc[m + 1];
        const double ds = lst ? jc[m] : jc[m] - jc[m + 1];
        double c = fma(dd, pe, ds * po);
        if constexpr (!UNI) c *= sc[m];
        eacc[m] += c;
      }
    }
    if (st > 0) rp_rec_get<EDGE>(rec, args.n0 + st - 1, args.ktot, ea, jn, jn2);
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      // buffers alternate over the launch's global level index (no barrier between a step's
      // last level and the next step's first)
      const int f0 = (((MS - 1 - st) * 5 + l) & 1) * 2 * FB, f1 = f0 + FB;
      // the level's input v (w at level 0, t after), scaled by the metric: q = sc v
      double g0[E], g1[E], qe[E][NE], qo[E][NO];
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double gd = 0.0, gs = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          const double v = (l == 0) ? we[m][k] : te[m][k];
          qe[m][k] = UNI ? v : sc[m] * v;
          gd = fma(args.op.le[k], qe[m][k], gd);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          const double v = (l == 0) ? wo[m][k] : to[m][k];
          qo[m][k] = UNI ? v : sc[m] * v;
          gs = fma(args.op.lo[k], qo[m][k], gs);
        }
        g0[m] = gd + gs;
        g1[m] = gs - gd;
      }
      lds[f0 + lane + 1] = g0[0];      // the lane's first element: adjoint of its uL
      lds[f1 + lane + 1] = g1[E - 1];  // the lane's last element: adjoint of its uR
      __builtin_amdgcn_sched_barrier(0);
      // the transposed volume term, before the barrier: a = c w + Qoe^T qo (even), c w +
      // Qeo^T qe (odd); level 0 starts from the bare products
      double ae[E][NE], ao[E][NO];
#pragma unroll
      for (int m = 0; m < E; ++m) {
#pragma unroll
        for (int j = 0; j < NE; ++j) {
          double t;
          int k0 = 0;
          if (l >= 3) {
            t = we[m][j];
          } else if (l >= 1) {
            t = (l == 1 ? b3 : b2) * we[m][j];
          } else {
            t = args.op.Qoe[j] * qo[m][0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NO; ++k) t = fma(args.op.Qoe[k * NE + j], qo[m][k], t);
          ae[m][j] = t;
        }
#pragma unroll
        for (int j = 0; j < NO; ++j) {
          double t;
          int k0 = 0;
          if (l >= 3) {
            t = wo[m][j];
          } else if (l >= 1) {
            t = (l == 1 ? b3 : b2) * wo[m][j];
          } else {
            t = args.op.Qeo[j] * qe[m][0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NE; ++k) t = fma(args.op.Qeo[k * NO + j], qe[m][k], t);
          ao[m][j] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(ae[m][k]);
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(ao[m][k]);
      }
      __syncthreads();
      // lane-1's last element's g1 / lane+1's first element's g0
      const double fromL = lds[f1 + lane], fromR = lds[f0 + lane + 2];
#pragma unroll
      for (int m = 0; m < E; ++m) {
        // edge tiles: nothing arrives at a trajectory's first element from the left (uL is
        // the inflow); its last element's uR is its own u_N (du1 = 0)
        double gl = (m == 0) ? fromL : g1[m - 1];
        double gr = (m == E - 1) ? fromR : g0[m + 1];
        if constexpr (EDGE) {
          gl = El[m].first ? 0.0 : gl;
          gr = El[m].last ? g1[m] : gr;
        }
        ae[m][0] -= gl + gr;
        ao[m][0] += gr - gl;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          if (l == 0) te[m][k] = fma(b5, ae[m][k], b4 * we[m][k]);
          else if (l < 4) te[m][k] = ae[m][k];
          else we[m][k] = ae[m][k];
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          if (l == 0) to[m][k] = fma(b5, ao[m][k], b4 * wo[m][k]);
          else if (l < 4) to[m][k] = ao[m][k];
          else wo[m][k] = ao[m][k];
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < E; ++m)
    if (args.has_eta && El[m].valid) eta_update(eta, El[m].e, eacc[m], args.has_eta);
  __syncthreads();  // the last face reads are done: the image is rewritten
  rp_store<NP, NW, E, H, EDGE>(wout, tile * TE * NP, nd, lds, we, wo, true);
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
  const int64_t tile = tile_of(blockIdx.x, gridDim.x, args.xcd);
  constexpr int H = RpHalo<MS>::A;
  const int64_t e0 = tile * (G::T - 2 * H) - H;
  if (edge_tile(e0, G::T, args.ktot, args.K))
    rp_adj_tile<NP, UNI, NW, E, MS, true>(lds, tile, win, wout, rec, eta, scale, args);
  else
    rp_adj_tile<NP, UNI, NW, E, MS, false>(lds, tile, win, wout, rec, eta, scale, args);
}

template <int NP, int NW, int E, int MS>
int rp_step_e(const dg_plan* p, const double* in, double* rec, double* last, const double* times,
              double dt, hipStream_t st, int64_t n0, bool jend) {
  const RkPoly& P = rk_poly();
  if (!P.ok) return fail(DG_ERR_HIP, "LSERK4 stability polynomial: beta_0 = beta_1 = 1 expected");
  RpStepArgs<NP, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;
  for (int k = 0; k < 6; ++k) a.beta[k] = P.beta[k];
  for (int m = 0; m < MS; ++m) {
    double u[5], b[5];
    for (int s = 0; s < 5; ++s) u[s] = inflow_value(p, times[m] + RK<5>::C(s) * dt);
    for (int k = 0; k < 5; ++k) {
      double acc = 0.0;
      for (int s = 0; s < 5; ++s) acc = std::fma(P.g[s][k], u[s], acc);
      b[k] = acc;
    }
    a.bnd[m * 5 + 0] = b[4] / P.beta[5];
    for (int l = 1; l < 5; ++l) a.bnd[m * 5 + l] = b[4 - l];
  }
  for (int m = 0; m <= MS; ++m) a.bnd[MS * 5 + m] = inflow_value(p, times[m]);
  a.ktot = p->ktot;
  a.n0 = n0;
  a.K = int32_t(p->K);
  a.xcd = p->xcd_order;
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
  const RkPoly& P = rk_poly();
  if (!P.ok) return fail(DG_ERR_HIP, "LSERK4 stability polynomial: beta_0 = beta_1 = 1 expected");
  RpAdjArgs<NP, MS> a;
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &a.op, true);
  a.sc = dt;
  for (int k = 0; k < 6; ++k) a.beta[k] = P.beta[k];
  a.ktot = p->ktot;
  a.n0 = n0;
  a.K = int32_t(p->K);
  a.has_eta = eta != nullptr ? (eta_mode | kEtaOn) : 0;
  a.xcd = p->xcd_order;
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
