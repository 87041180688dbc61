// dg_ovl_tiles.h — the dataflow sweep's tile bodies with one workgroup barrier per time step
// instead of one per Horner level ("overlapped waves"; DG_TUNE_SWEEP_EXCHANGE = 1).
// Internal to libdgadv.so.
//
// The pair-tile bodies of dg_rec_tiles.h exchange every level's faces through LDS: write, a
// workgroup barrier, read -- five barriers per step across all of a tile's waves, and a wave
// spends ~40 % of its cycles waiting there (profiles/r04/headline_w12/).  Here:
//   - every wave works on its own window of 128 consecutive elements (lane j: window
//     elements 2j, 2j+1, as the pair tiles) and moves the faces between its lanes with DPP
//     wave shifts (wave_shr:1 / wave_shl:1, two 32-bit moves per double; dg_wave.hip), so a
//     level needs no LDS and no barrier;
//   - windows of neighbouring waves overlap by 2 G elements: wave w's window starts at tile
//     element w*S, S = 128 - 2G, and the wave OWNS the middle S elements [G, 128 - G).  The
//     G = 6 elements at each end (3 lanes) are ghosts.  A step's cone is 5 elements (one per
//     level), so after a step the ghosts are stale (the lanes at the wave's ends read no real
//     neighbour) but every owned element is exact;
//   - after each step the lanes next to the ghosts publish their state (the G owned elements
//     at each end of the window) in LDS, one workgroup barrier, and every wave replaces its
//     ghosts with its neighbours' owned values: the whole window is exact again.  The first
//     wave's left and the last wave's right ghosts have no neighbour and are the tile's halo
//     (H >= G), which the cone accounting of the pair tiles covers unchanged.
// Each element's arithmetic is the pair tiles' (the same fma sequence on the same doubles; a
// face value is the same double whether it came through LDS or DPP), so the results are bit-
// identical to the launch-per-block pair and to the level-barrier dataflow launch.  The cost:
// a wave computes 128 elements and owns 116 (the ghost lanes redo 9.4 % of the work), and a
// tile of NW waves covers NW*S + 2G elements instead of 128*NW.
// Sources: AdvecRHS1D (utils/AdvecRHS1D.m:9-19), the LSERK4 loop (utils/One_code.mlx:106-140),
// the indicator pattern (python/Main_finite_difference.py:54-94); DESIGN.md §5.
#pragma once
#include "dg_rec_tiles.h"

namespace dgr {

constexpr int kOvG = 6;               // ghost elements per window end: >= 5 (a step's cone), even
constexpr int kOvGL = kOvG / 2;       // ghost lanes per window end
constexpr int kOvS = 128 - 2 * kOvG;  // elements a wave owns

template <int NP, int NW> struct OvGeo {
  static constexpr int LB = 64 * NW;
  static constexpr int T = NW * kOvS + 2 * kOvG;  // elements per tile (incl. halo)
  static constexpr int kTileD = T * NP + 2;       // staging image (+2: 16-byte realignment)
  static constexpr int kVec = (kTileD + 2 * LB - 1) / (2 * LB);
  // the step exchange: per wave a left and a right slot of kOvGL lanes x 2 elements x NP
  // doubles, double-buffered over the step index (a wave may publish step s+1 while a slower
  // one still reads step s; two barriers separate s and s+2).  Aliases the image, which is
  // dead between the prologue's last read and the epilogue's store (both behind a barrier).
  static constexpr int kXSlot = 2 * NP;
  static constexpr int kXBuf = NW * 2 * kOvGL * kXSlot;
  static constexpr int kXD = 2 * kXBuf;
  static constexpr int kLds = ((kTileD > kXD ? kTileD : kXD) + 1) & ~1;
  static_assert(kOvS % 2 == 0 && T % 2 == 0, "lane pairs at even elements");
};

// DPP wave shifts of a double (dg_wave.hip): lane l <- lane l-1 (lane 0 keeps its own x) /
// lane l <- lane l+1 (lane 63 keeps x).  The end lanes' results feed ghosts only.  (Measured
// against ds_bpermute, which runs on the LDS pipe instead of the VALU: 8-13 % slower at N = 1,
// 2, 4, profiles/r05/ovl3 -- the crossbar's latency sits on every level's critical path.)
__device__ __forceinline__ double ov_shr1(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = int(b), hi = int(b >> 32);
  const int rl = __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}
__device__ __forceinline__ double ov_shl1(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = int(b), hi = int(b >> 32);
  const int rl = __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false);
  const int rh = __builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false);
  return __hiloint2double(rh, rl);
}

// The lane's wave, window lane and first tile element; whether it owns its two elements.
struct OvLane {
  int wv, j, el0;
  bool own;
};
__device__ __forceinline__ OvLane ov_lane() {
  OvLane L;
  const int lane = threadIdx.x;
  L.wv = lane >> 6;
  L.j = lane & 63;
  L.el0 = L.wv * kOvS + 2 * L.j;
  L.own = L.j >= kOvGL && L.j < 64 - kOvGL;
  return L;
}

// The step exchange of the lane pair's state (even/odd or dual coordinates), `xb` the step's
// buffer: the owned lanes next to the ghosts publish, a workgroup barrier, the ghost lanes
// take their neighbour wave's values.
template <int NP, int NW>
__device__ __forceinline__ void ov_exchange(double* __restrict__ xb, const OvLane& L,
                                            double (*se)[(NP + 1) / 2], double (*so)[NP / 2]) {
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, SL = 2 * NP;
  static_assert(SL % 2 == 0, "16-byte slots");
  int slot = -1;
  if (L.j >= kOvGL && L.j < 2 * kOvGL) slot = (L.wv * 2 + 0) * kOvGL + (L.j - kOvGL);
  else if (L.j >= 64 - 2 * kOvGL && L.j < 64 - kOvGL)
    slot = (L.wv * 2 + 1) * kOvGL + (L.j - (64 - 2 * kOvGL));
  if (slot >= 0) {
    double v[SL];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
      for (int k = 0; k < NE; ++k) v[m * NP + k] = se[m][k];
#pragma unroll
      for (int k = 0; k < NO; ++k) v[m * NP + NE + k] = so[m][k];
    }
    double2* p = reinterpret_cast<double2*>(xb + slot * SL);
#pragma unroll
    for (int q = 0; q < NP; ++q) p[q] = double2{v[2 * q], v[2 * q + 1]};
  }
  __syncthreads();
  int src = -1;
  if (L.j < kOvGL) {
    if (L.wv > 0) src = ((L.wv - 1) * 2 + 1) * kOvGL + L.j;
  } else if (L.j >= 64 - kOvGL) {
    if (L.wv < NW - 1) src = ((L.wv + 1) * 2 + 0) * kOvGL + (L.j - (64 - kOvGL));
  }
  if (src >= 0) {
    double v[SL];
    const double2* p = reinterpret_cast<const double2*>(xb + src * SL);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const double2 t = p[q];
      v[2 * q] = t.x;
      v[2 * q + 1] = t.y;
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
      for (int k = 0; k < NE; ++k) se[m][k] = v[m * NP + k];
#pragma unroll
      for (int k = 0; k < NO; ++k) so[m][k] = v[m * NP + NE + k];
    }
  }
}

// The TE interior elements of the tile (each written by its owning lane) to the image, then
// 16-byte stores.  Callers barrier before (the exchange's last reads are done).
template <int NP, int NW, int H, bool EDGE, bool WT>
__device__ __forceinline__ void ov_store(double* __restrict__ g, int64_t o0, int64_t nd,
                                         double* __restrict__ lds, const OvLane& L,
                                         const double (*ev)[(NP + 1) / 2],
                                         const double (*od)[NP / 2], bool dual) {
  using G = OvGeo<NP, NW>;
  constexpr int T = G::T, TE = T - 2 * H;
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  if (L.own) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int el = L.el0 + m;
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
  }
  __syncthreads();
  const int64_t rem = nd - o0;
  if constexpr (EDGE) {
    if constexpr (WT) store_run_wt<G::LB>(g, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
    else store_run<G::LB>(g, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
  } else {
    if constexpr (WT) store_full_wt<TE * NP, G::LB>(g, o0, lds);
    else store_full<TE * NP, G::LB>(g, o0, lds);
  }
}

// Forward: rp_step_tile's MS steps on overlapped waves (same arguments, same outputs).
template <int NP, bool UNI, int NW, int MS, bool EDGE, bool WT>
__device__ __forceinline__ void ov_step_tile(double* __restrict__ lds, int64_t tile,
                                             const double* __restrict__ uin,
                                             double* __restrict__ rec, double* __restrict__ last,
                                             const double* __restrict__ scale,
                                             const RpOp<NP>& c, OpSrc<NP> os,
                                             const double* kb, int64_t n0, bool jend) {
  using G = OvGeo<NP, NW>;
  constexpr int T = G::T, E = 2;
  constexpr int H = RpHalo<MS>::F;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0 && H % 2 == 0 && H >= kOvG, "overlapped tiles");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  constexpr int CB = G::kLds;      // lds[CB + i] = bnd[i] (edge tiles)
  constexpr int CR = CB + MS * 5;  // the record's inflow values
  const int lane = threadIdx.x;
  const OvLane L = ov_lane();
  const int64_t e0 = tile * TE - H;
  const int64_t ec = e0 > 0 ? e0 : 0;
  const int64_t nd = c.ktot * NP;

  const int off = tile_load<G, NP, EDGE, WT>(uin, e0, nd, lds);
  if constexpr (EDGE) {
    if (lane <= MS * 6) lds[CB + lane] = kb[lane];
  }
  __syncthreads();
  double ue[E][NE], uo[E][NO];
  Elem El[E];
  double sc[E], jv[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = L.el0 + m;
    const double* us = lds + off + el * NP;
    to_eo<NP>(us, ue[m], uo[m]);
    El[m] = elem_info<H, T, EDGE>(e0, el, c.ktot, c.K);
    El[m].valid = El[m].valid && L.own;  // a ghost never publishes
    sc[m] = c.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    jv[m] = us[0] - ((EDGE && El[m].first) ? lds[CR] : us[-1]);
  }
  if (n0 >= 1) rp_rec_put<E, EDGE, WT>(rec, n0 - 1, c.ktot, El, jv, ec);
  __syncthreads();  // the image is read: the exchange buffers alias it

  const double b4 = c.beta[4], b5 = c.beta[5], b3 = c.beta[3], b2 = c.beta[2];
  double te[E][NE], to[E][NO];
#pragma unroll 1
  for (int st = 0; st < MS; ++st) {
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      double v0[E], vN[E];
#pragma unroll
      for (int m = 0; m < E; ++m) {
        const double e = (l == 0) ? ue[m][0] : te[m][0], o = (l == 0) ? uo[m][0] : to[m][0];
        v0[m] = e + o;
        vN[m] = e - o;
      }
      // lane-1's right face / lane+1's left face
      const double fromL = ov_shr1(vN[E - 1]), fromR = ov_shl1(v0[0]);
      double pe[E][NE], po[E][NO];
      {
        const auto& op = os.get();
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
              a = op.Qeo[k * NO] * vo[0];
              j0 = 1;
            }
#pragma unroll
            for (int j = j0; j < NO; ++j) a = fma(op.Qeo[k * NO + j], vo[j], a);
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
              a = op.Qoe[k * NE] * ve[0];
              j0 = 1;
            }
#pragma unroll
            for (int j = j0; j < NE; ++j) a = fma(op.Qoe[k * NE + j], ve[j], a);
            po[m][k] = a;
          }
        }
      }
#pragma unroll
      for (int m = 0; m < E; ++m) {  // as the pair tiles (no contraction across the update)
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(pe[m][k]);
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(po[m][k]);
      }
      double bnd = 0.0, urec = 0.0;
      if constexpr (EDGE) {
        bnd = lds[CB + st * 5 + l];
        if (l == 0) urec = lds[CR + st];
      }
      const auto& ol = os.get();
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
          const double z = fma(ol.le[k], dlt, pe[m][k]);
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
          const double z = fma(ol.lo[k], sig, po[m][k]);
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
      if (l == 0 && st >= 1) rp_rec_put<E, EDGE, WT>(rec, n0 + st - 1, c.ktot, El, jv, ec);
    }
    // the ghosts take their neighbours' exact values (not needed after the last step unless
    // the final state's jumps are recorded)
    if (st < MS - 1 || jend) ov_exchange<NP, NW>(lds + (st & 1) * G::kXBuf, L, ue, uo);
  }
  if (jend) {
    // the sweep's final state u^{n0+MS}: its jumps (record n0+MS-1), inflow at t_{n0+MS}
    double u0[E], uN[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
      u0[m] = ue[m][0] + uo[m][0];
      uN[m] = ue[m][0] - uo[m][0];
    }
    const double fromL = ov_shr1(uN[E - 1]);
#pragma unroll
    for (int m = 0; m < E; ++m) {
      double uL = (m == 0) ? fromL : uN[m - 1];
      if constexpr (EDGE) uL = El[m].first ? lds[CR + MS] : uL;
      jv[m] = u0[m] - uL;
    }
    rp_rec_put<E, EDGE, WT>(rec, n0 + MS - 1, c.ktot, El, jv, ec);
  }
  __syncthreads();  // the exchange's last reads are done: the image is rewritten
  ov_store<NP, NW, H, EDGE, WT>(last, tile * TE * NP, nd, lds, L, ue, uo, false);
}

// Adjoint: rp_adj_tile's MS reverse steps on overlapped waves (same arguments and outputs).
template <int NP, bool UNI, int NW, int MS, bool EDGE, bool WT>
__device__ __forceinline__ void ov_adj_tile(double* __restrict__ lds, int64_t tile,
                                            const double* __restrict__ win,
                                            double* __restrict__ wout,
                                            const double* __restrict__ rec,
                                            EtaSink& es,
                                            const double* __restrict__ scale,
                                            const RpOp<NP>& c, OpSrc<NP> os, int64_t n0) {
  using G = OvGeo<NP, NW>;
  constexpr int T = G::T, E = 2;
  constexpr int H = RpHalo<MS>::A;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0 && H % 2 == 0 && H >= kOvG, "overlapped tiles");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  const OvLane L = ov_lane();
  const int64_t e0 = tile * TE - H;
  const int64_t ec = e0 > 0 ? e0 : 0;
  const int64_t nd = c.ktot * NP;
  const int64_t ea = e0 + L.el0;  // the lane's first element (even)
  const int has_eta = es.mode;

  const int off = tile_load<G, NP, EDGE, WT>(win, e0, nd, lds);
  double jn[E + 1];
  rp_rec_get<E, EDGE, WT>(rec, n0 + MS - 1, c.ktot, ea, ec, jn);
  __syncthreads();
  double we[E][NE], wo[E][NO];
  Elem El[E];
  double sc[E], eacc[E];
#pragma unroll
  for (int m = 0; m < E; ++m) {
    const int el = L.el0 + m;
    const double* w = lds + off + el * NP;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[m][k] = w[k] + w[N - k];
      wo[m][k] = w[k] - w[N - k];
    }
    if constexpr (NE > NO) we[m][NO] = w[NO];
    El[m] = elem_info<H, T, EDGE>(e0, el, c.ktot, c.K);
    El[m].valid = El[m].valid && L.own;
    sc[m] = c.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    eacc[m] = 0.0;
  }
  __syncthreads();  // the image is read: the exchange buffers alias it

  const double b4 = c.beta[4], b5 = c.beta[5], b3 = c.beta[3], b2 = c.beta[2];
  double te[E][NE], to[E][NO];
#pragma unroll 1
  for (int st = MS - 1; st >= 0; --st) {
    double jc[E + 1];
#pragma unroll
    for (int m = 0; m <= E; ++m) jc[m] = jn[m];
    if (has_eta) {
      const auto& op = os.get();
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double pe = 0.0, po = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) pe = fma(op.le[k], we[m][k], pe);
#pragma unroll
        for (int k = 0; k < NO; ++k) po = fma(op.lo[k], wo[m][k], po);
        const bool lst = EDGE && El[m].last;
        const double dd = lst ? jc[m] : jc[m] + jc[m + 1];
        const double ds = lst ? jc[m] : jc[m] - jc[m + 1];
        double cc = fma(dd, pe, ds * po);
        if constexpr (!UNI) cc *= sc[m];
        eacc[m] += cc;
      }
    }
    if (st > 0) rp_rec_get<E, EDGE, WT>(rec, n0 + st - 1, c.ktot, ea, ec, jn);
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      double g0[E], g1[E], qe[E][NE], qo[E][NO];
      const auto& ol = os.get();
#pragma unroll
      for (int m = 0; m < E; ++m) {
        double gd = 0.0, gs = 0.0;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          const double v = (l == 0) ? we[m][k] : te[m][k];
          qe[m][k] = UNI ? v : sc[m] * v;
          gd = fma(ol.le[k], qe[m][k], gd);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          const double v = (l == 0) ? wo[m][k] : to[m][k];
          qo[m][k] = UNI ? v : sc[m] * v;
          gs = fma(ol.lo[k], qo[m][k], gs);
        }
        g0[m] = gd + gs;
        g1[m] = gs - gd;
      }
      // lane-1's last element's g1 / lane+1's first element's g0
      const double fromL = ov_shr1(g1[E - 1]), fromR = ov_shl1(g0[0]);
      double ae[E][NE], ao[E][NO];
      const auto& oq = os.get();
#pragma unroll
      for (int m = 0; m < E; ++m) {
#pragma unroll
        for (int j = 0; j < NO; ++j) {
          double t;
          int k0 = 0;
          if (l >= 3) {
            t = wo[m][j];
          } else if (l >= 1) {
            t = (l == 1 ? b3 : b2) * wo[m][j];
          } else {
            t = oq.Qeo[j] * qe[m][0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NE; ++k) t = fma(oq.Qeo[k * NO + j], qe[m][k], t);
          ao[m][j] = t;
        }
#pragma unroll
        for (int j = 0; j < NE; ++j) {
          double t;
          int k0 = 0;
          if (l >= 3) {
            t = we[m][j];
          } else if (l >= 1) {
            t = (l == 1 ? b3 : b2) * we[m][j];
          } else {
            t = oq.Qoe[j] * qo[m][0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NO; ++k) t = fma(oq.Qoe[k * NE + j], qo[m][k], t);
          ae[m][j] = t;
        }
        // materialised as the pair tiles do (their barrier-ordering pins): a bare product at
        // level 0 (Np = 2: one term) must not contract with the face update below into an fma
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(ao[m][k]);
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(ae[m][k]);
      }
#pragma unroll
      for (int m = 0; m < E; ++m) {
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
    if (st > 0) ov_exchange<NP, NW>(lds + ((MS - 1 - st) & 1) * G::kXBuf, L, we, wo);
  }
  if (has_eta) {
    if constexpr (WT) {
      const __amdgpu_buffer_rsrc_t ro = wt_rsrc(es.part_out ? es.part_out + ec : es.eta + ec);
#pragma unroll
      for (int m = 0; m < E; ++m) {
        if (!El[m].valid) continue;
        const uint32_t o = uint32_t(El[m].e - ec) * 8u;
        if (es.part_out) {
          wt_st8(ro, o, eacc[m]);
        } else {
          double v;
          if (es.nparts > 0) {
            v = wt_ld8(wt_rsrc(es.part_in + ec), o);
            if (!(has_eta & kEtaAssign)) v = es.eta[El[m].e] + v;
            for (int q = 1; q < es.nparts; ++q)
              v = v + wt_ld8(wt_rsrc(es.part_in + q * es.part_ld + ec), o);
            v = v + eacc[m];
          } else {
            v = (has_eta & kEtaAssign) ? eacc[m] : es.eta[El[m].e] + eacc[m];
          }
          if (has_eta & kEtaAbs) v = fabs(v);
          wt_st8(ro, o, v);
          if (es.argmax && am_better(fabs(v), El[m].e, es.bv, es.bi)) {
            es.bv = fabs(v);
            es.bi = El[m].e;
          }
        }
      }
    } else {
#pragma unroll
      for (int m = 0; m < E; ++m)
        if (El[m].valid) eta_update(es.eta, El[m].e, eacc[m], has_eta);
    }
  }
  __syncthreads();  // the exchange's last reads are done: the image is rewritten
  ov_store<NP, NW, H, EDGE, WT>(wout, tile * TE * NP, nd, lds, L, we, wo, true);
}

}  // namespace dgr
