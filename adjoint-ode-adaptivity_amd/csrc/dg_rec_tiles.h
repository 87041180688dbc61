// dg_rec_tiles.h — the jump-record sweep pair's tile bodies on pair tiles (E = 2 consecutive
// elements per lane), shared by the launch-per-block kernels of dg_rec.hip (k_step_rp /
// k_adj_rp) and the dataflow sweep of dg_sweep.hip (k_sweep_rp, forward + adjoint in one
// launch).  Internal to libdgadv.so.
//
// Same arithmetic per element as k_step / k_adj<..., REC = true> in dg_advec.hip; what the
// pair tiles change is the layout (DESIGN.md §5 "Pair tiles"):
//   - lane l owns tile elements E*l .. E*l+E-1.  The face between a lane's own elements is a
//     register read; only the lane's outer two faces go through LDS, so a stage writes and
//     reads half the LDS words per element and a barrier covers twice the elements;
//   - the E independent element chains per lane give the fp64 pipe instruction-level
//     parallelism between a level's barrier and its update;
//   - a 256*W-lane workgroup covers 256*W*E elements: 512 per tile on 4 waves (W = 1) or
//     1024 on 8 waves (W = 2, the default: 41 KB of LDS);
//   - the face arrays alias the staging image (one barrier after the image is read and one
//     before it is rewritten, per tile).
//
// Memory policy `WT` (template flag of every function that touches global memory):
//   false  plain loads and stores (a launch hands its results to the next one at the kernel
//          boundary);
//   true   the dataflow sweep's in-launch hand-offs (cdna_hip_programming.md §6 Guideline 16,
//          R1): every store another workgroup reads in the same launch is write-through
//          (`sc1`: the line leaves this XCD's L2 for memory, so a consumer on any XCD reads
//          it), every load of such bytes is an `sc1` load (it bypasses the CU's L1, which other
//          CUs' stores never refresh).  The consumer polls its producers' flags before loading;
//          no acquire fence is needed because every handed-off byte is loaded `sc1` and no
//          buffer is rewritten inside the launch (dg_sweep.hip).
// Sources: AdvecRHS1D (utils/AdvecRHS1D.m:9-19), the LSERK4 loop (utils/One_code.mlx:106-140),
// the indicator pattern (python/Main_finite_difference.py:54-94); DESIGN.md §5.
#pragma once
#include "dg_common.h"

namespace dgr {
using namespace dgk;

template <int NP, int NW, int E> struct RpGeo {
  static constexpr int LB = 64 * NW;  // lanes per workgroup
  static constexpr int T = E * LB;       // elements per tile (incl. halo)
  static constexpr int kTileD = T * NP + 2;  // staging image (+2: 16-byte realignment)
  static constexpr int kVec = (kTileD + 2 * LB - 1) / (2 * LB);  // double2 loads per lane
  static constexpr int kFaceD = 4 * (LB + 2);  // 2 double-buffered lane-face arrays, padded
  static constexpr int kLds = ((kTileD > kFaceD ? kTileD : kFaceD) + 1) & ~1;
};

// Halo widths (elements per side): the forward's stage cone MS*5 + the final state's
// neighbours, the adjoint's MS*5; both rounded up to even, so every lane's element pair starts
// at an even element and its two record entries are one aligned 16-byte access.
template <int MS> struct RpHalo {
  static constexpr int F = (MS * 5 + 2) & ~1;
  static constexpr int A = (MS * 5 + 1) & ~1;
};

// ---------------------------------------------------------------------------
// Global-memory access under the policy WT.  The write-through / L1-bypassing forms are
// buffer instructions with the `sc1` cache-policy bit (aux 16) on a descriptor whose base is
// wave-uniform (read-first-lane'd, so hipcc emits no waterfall loop); offsets are 32-bit
// bytes from that base, which every caller keeps inside one tile's range.
// ---------------------------------------------------------------------------
typedef unsigned rp_v4u __attribute__((ext_vector_type(4)));
typedef unsigned rp_v2u __attribute__((ext_vector_type(2)));
constexpr int kSc1 = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(b));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(b >> 32));
  void* p = reinterpret_cast<void*>((uint64_t(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ void wt_st16(__amdgpu_buffer_rsrc_t r, uint32_t off, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(rp_v4u, v), r, off, 0, kSc1);
}
__device__ __forceinline__ void wt_st8(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(rp_v2u, v), r, off, 0, kSc1);
}
__device__ __forceinline__ double2 wt_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}
__device__ __forceinline__ double wt_ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSc1));
}

// Coalesced 16-byte loads of the tile image [e0, e0 + G::T) (zeros outside [0, nd)), issued
// together, then written to LDS.  Returns the image's offset (0 or 1 double).  G: the tile
// geometry (G::T elements, G::LB lanes, G::kVec double2 per lane).
template <class G, int NP, bool EDGE, bool WT>
__device__ __forceinline__ int tile_load(const double* __restrict__ g, int64_t e0, int64_t nd,
                                         double* __restrict__ lds) {
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  const int off = int(d0 - base);
  const int nvec = (G::T * NP + off + 1) >> 1;
  const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g);
  // WT: descriptor at the first in-range double of the image (base < 0 only in edge tiles,
  // whose out-of-range lanes load nothing)
  const int64_t bc = base > 0 ? base : 0;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(g + bc);  // (unused, and dropped, unless WT)
  double2 rv[G::kVec];
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = int(threadIdx.x) + q * G::LB;
    const int64_t gd = base + 2 * int64_t(v);
    double2 val = make_double2(0.0, 0.0);
    if (v < nvec) {
      if (!EDGE || (gd >= 0 && gd + 1 < nd)) {
        if constexpr (WT) val = wt_ld16(r, uint32_t(gd - bc) * 8u);
        else val = g2[gd >> 1];
      } else {
        if constexpr (WT) {
          if (gd >= 0 && gd < nd) val.x = wt_ld8(r, uint32_t(gd - bc) * 8u);
          if (gd + 1 >= 0 && gd + 1 < nd) val.y = wt_ld8(r, uint32_t(gd + 1 - bc) * 8u);
        } else {
          if (gd >= 0 && gd < nd) val.x = g[gd];
          if (gd + 1 >= 0 && gd + 1 < nd) val.y = g[gd + 1];
        }
      }
    }
    rv[q] = val;
  }
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = int(threadIdx.x) + q * G::LB;
    if (v < nvec) *reinterpret_cast<double2*>(&lds[2 * v]) = rv[q];
  }
  return off;
}

template <int NP, int NW, int E, bool EDGE, bool WT>
__device__ __forceinline__ int rp_load(const double* __restrict__ g, int64_t e0, int64_t nd,
                                       double* __restrict__ lds) {
  return tile_load<RpGeo<NP, NW, E>, NP, EDGE, WT>(g, e0, nd, lds);
}

// Store `count` doubles from lds[0..count) to g[o0..o0+count) (o0 even), write-through.
template <int LB>
__device__ __forceinline__ void store_run_wt(double* __restrict__ g, int64_t o0, int64_t count,
                                             const double* __restrict__ lds) {
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(g + o0);
  for (int64_t v = threadIdx.x; 2 * v < count; v += LB) {
    const double2 val = *reinterpret_cast<const double2*>(&lds[2 * v]);
    if (2 * v + 1 < count) wt_st16(r, uint32_t(v) * 16u, val);
    else wt_st8(r, uint32_t(v) * 16u, val.x);
  }
}

template <int COUNT, int LB>
__device__ __forceinline__ void store_full_wt(double* __restrict__ g, int64_t o0,
                                              const double* __restrict__ lds) {
  static_assert(COUNT % 2 == 0, "16-byte runs");
  constexpr int NV = COUNT / 2, NQ = (NV + LB - 1) / LB;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(g + o0);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int v = int(threadIdx.x) + q * LB;
    if ((q + 1) * LB <= NV || v < NV)
      wt_st16(r, uint32_t(v) * 16u, *reinterpret_cast<const double2*>(&lds[2 * v]));
  }
}

// The TE interior elements from registers to the image (nodal; `dual`: from the adjoint's
// dual coordinates), then 16-byte stores.  Callers barrier before (face reads done).
template <int NP, int NW, int E, int H, bool EDGE, bool WT>
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
  const int64_t rem = nd - o0;
  if constexpr (EDGE) {
    if constexpr (WT) store_run_wt<G::LB>(g, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
    else store_run<G::LB>(g, o0, rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP, lds);
  } else {
    if constexpr (WT) store_full_wt<TE * NP, G::LB>(g, o0, lds);
    else store_full<TE * NP, G::LB>(g, o0, lds);
  }
}

// Record row n: the lane's E left-face jumps jv[0..E) (dg_common.h rec_ld), one 16-byte store
// per pair of them; an edge tile stores a pair one by one where its valid range ends between
// them.  (A tile's valid range [H, T - H) starts and ends at even elements, so in interior
// tiles a pair is valid or invalid as a whole.)  `ec` (WT): the tile's first in-range element,
// the descriptor's base.
template <int E, bool EDGE, bool WT>
__device__ __forceinline__ void rp_rec_put(double* __restrict__ rec, int64_t n, int64_t ktot,
                                           const Elem* El, const double* jv, int64_t ec) {
  double* row = rec + n * rec_ld(ktot);
  if constexpr (WT) {
    const __amdgpu_buffer_rsrc_t r = wt_rsrc(row + ec);
    const uint32_t o = uint32_t(El[0].e - ec) * 8u;
#pragma unroll
    for (int q = 0; q < E; q += 2) {
      if (!EDGE || (El[q].valid && El[q + 1].valid)) {
        if (El[q].valid) wt_st16(r, o + 8u * q, double2{jv[q], jv[q + 1]});
      } else {
        if (El[q].valid) wt_st8(r, o + 8u * q, jv[q]);
        if (El[q + 1].valid) wt_st8(r, o + 8u * (q + 1), jv[q + 1]);
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < E; q += 2) {
      if (!EDGE || (El[q].valid && El[q + 1].valid)) {
        if (El[q].valid) *reinterpret_cast<double2*>(row + El[q].e) = double2{jv[q], jv[q + 1]};
      } else {
        if (El[q].valid) row[El[q].e] = jv[q];
        if (El[q + 1].valid) row[El[q + 1].e] = jv[q + 1];
      }
    }
  }
}

// Record row n for the lane's E elements starting at element ea (even): j[0..E) = j_ea..
// j_ea+E-1 and the right neighbour's j[E] = j_ea+E.  Interior tiles never reach a
// trajectory's end, so all are in range; edge tiles read zeros outside [0, ktot).  `ec` as
// for rp_rec_put.
template <int E, bool EDGE, bool WT>
__device__ __forceinline__ void rp_rec_get(const double* __restrict__ rec, int64_t n,
                                           int64_t ktot, int64_t ea, int64_t ec, double* j) {
  const double* row = rec + n * rec_ld(ktot);
  if constexpr (WT) {
    const __amdgpu_buffer_rsrc_t r = wt_rsrc(row + ec);
    const uint32_t o = uint32_t(ea - ec) * 8u;
    if constexpr (!EDGE) {
#pragma unroll
      for (int q = 0; q < E; q += 2) {
        const double2 v = wt_ld16(r, o + 8u * q);
        j[q] = v.x;
        j[q + 1] = v.y;
      }
      j[E] = wt_ld8(r, o + 8u * E);
    } else {
#pragma unroll
      for (int m = 0; m <= E; ++m) j[m] = (ea + m >= 0 && ea + m < ktot) ? wt_ld8(r, o + 8u * m) : 0.0;
    }
  } else {
    if constexpr (!EDGE) {
#pragma unroll
      for (int q = 0; q < E; q += 2) {
        const double2 v = *reinterpret_cast<const double2*>(row + ea + q);
        j[q] = v.x;
        j[q + 1] = v.y;
      }
      j[E] = row[ea + E];
    } else {
#pragma unroll
      for (int m = 0; m <= E; ++m) j[m] = (ea + m >= 0 && ea + m < ktot) ? row[ea + m] : 0.0;
    }
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

// Per-step edge constants of a forward block of MS steps (the layout rp_step_tile copies into
// LDS): bnd[5 st + l] = b_4/beta_5, b_3, b_2, b_1, b_0 of step st, level l = 0..4; then
// bnd[5 MS + st] = uin(t_{n0+st}), the record's inflow value, st = 0..MS.  times[0..MS].
inline void rp_block_bnd(const dg_plan* p, int MS, const double* times, double dt, double* bnd) {
  const RkPoly& P = rk_poly();
  for (int m = 0; m < MS; ++m) {
    double u[5], b[5];
    for (int s = 0; s < 5; ++s) u[s] = inflow_value(p, times[m] + RK<5>::C(s) * dt);
    for (int k = 0; k < 5; ++k) {
      double acc = 0.0;
      for (int s = 0; s < 5; ++s) acc = std::fma(P.g[s][k], u[s], acc);
      b[k] = acc;
    }
    bnd[m * 5 + 0] = b[4] / P.beta[5];
    for (int l = 1; l < 5; ++l) bnd[m * 5 + l] = b[4 - l];
  }
  for (int m = 0; m <= MS; ++m) bnd[MS * 5 + m] = inflow_value(p, times[m]);
}

// Launch constants shared by both directions and every block of a sweep.
template <int NP> struct RpOp {
  EOArgs<NP> op;
  double sc;       // dt (non-uniform meshes multiply by scale[k]; uniform: in op)
  double beta[6];  // P's coefficients
  int64_t ktot;
  int32_t K;
  int32_t xcd;
};

template <int NP> int rp_make_op(const dg_plan* p, double dt, RpOp<NP>* c) {
  const RkPoly& P = rk_poly();
  if (!P.ok) return fail(DG_ERR_HIP, "LSERK4 stability polynomial: beta_0 = beta_1 = 1 expected");
  make_eo<NP>(p, p->uniform ? dt * p->s_uniform : 1.0, &c->op, true);
  c->sc = dt;
  for (int k = 0; k < 6; ++k) c->beta[k] = P.beta[k];
  c->ktot = p->ktot;
  c->K = int32_t(p->K);
  c->xcd = p->xcd_order;
  return DG_OK;
}

// Where the tile bodies read the operator blocks (Qeo, Qoe, le, lo: 2 NE NO + NP doubles).
// Up to Np = 5 (at most 40 SGPRs) as the kernel argument they are, which the compiler keeps in
// SGPRs for the whole kernel.  From Np = 6 on they do not fit the SGPR file beside the rest
// (98 SGPRs at Np = 9): kept as one hoisted argument they were spilled to VGPR lanes and read
// back with a v_readlane per use -- 2,120 v_readlane in the Np = 9 sweep kernel, a third of
// the VALU instructions it issued.  OpSrc<NP, true> re-reads each block from the kernarg
// segment where it is used: scalar loads through a pointer laundered by an empty asm (so not
// hoisted), only the block in use occupying SGPRs.
template <int NP> constexpr bool kOpReload = NP >= 6;
template <int NP, bool R = kOpReload<NP>> struct OpSrc {
  const EOArgs<NP>* p;
  __device__ __forceinline__ const EOArgs<NP>& get() const { return *p; }
};
template <int NP> struct OpSrc<NP, true> {
  const DG_KAS EOArgs<NP>* p;
  __device__ __forceinline__ const DG_KAS EOArgs<NP>& get() const {
    const DG_KAS EOArgs<NP>* q = p;
    asm volatile("" : "+s"(q));
    return *q;
  }
};
// kc: the RpOp argument's address in the kernarg segment (kernarg_tail_k + its offset).
template <int NP>
__device__ __forceinline__ OpSrc<NP> op_src(const RpOp<NP>& rc, const DG_KAS char* kc) {
  if constexpr (kOpReload<NP>)
    return OpSrc<NP>{reinterpret_cast<const DG_KAS EOArgs<NP>*>(kc + offsetof(RpOp<NP>, op))};
  else
    return OpSrc<NP>{&rc.op};
}

// Forward: MS steps of the tile; records u^{n0}..u^{n0+MS-1}'s jumps (and u^{n0+MS}'s when
// the block ends the sweep), writes u^{n0+MS} to `last`.  Per step five Horner levels, each
// one face exchange of its input vector v (u at level 0, t after) through LDS.  `kb` (edge
// tiles only): the block's rp_block_bnd constants in kernarg memory (lane-indexed reads);
// lds must hold G::kLds + MS*6 + 1 doubles.
// Snapshot variant (SNAP, round 5: the snapshot forward on pair tiles, dg_lserk4_fwd with
// DG_TUNE_SNAP_PAIRS): no record; `rec` is the launch's first output state u^{n0+1} and step st's
// state u^{n0+st+1} is stored at rec + st * sstride straight from the registers (each lane's
// two elements are 2 Np consecutive doubles), the last one through `last` as usual.
template <int NP, int E, bool EDGE>
__device__ __forceinline__ void rp_snap_put(double* __restrict__ g, const Elem* El,
                                            const double (*ue)[(NP + 1) / 2],
                                            const double (*uo)[NP / 2]) {
  double v[E][NP];
#pragma unroll
  for (int m = 0; m < E; ++m) from_eo<NP>(ue[m], uo[m], v[m]);
  const bool pair = El[0].valid && El[1].valid;
  double* o = g + El[0].e * NP;
  if (pair && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
#pragma unroll
    for (int q = 0; q < NP; ++q)
      reinterpret_cast<double2*>(o)[q] = double2{v[(2 * q) / NP][(2 * q) % NP],
                                                 v[(2 * q + 1) / NP][(2 * q + 1) % NP]};
  } else {
#pragma unroll
    for (int m = 0; m < E; ++m)
      if (El[m].valid) {
#pragma unroll
        for (int i = 0; i < NP; ++i) g[El[m].e * NP + i] = v[m][i];
      }
  }
}

template <int NP, bool UNI, int NW, int E, int MS, bool EDGE, bool WT, bool SNAP = false>
__device__ __forceinline__ void rp_step_tile(double* __restrict__ lds, int64_t tile,
                                             const double* __restrict__ uin,
                                             double* __restrict__ rec, double* __restrict__ last,
                                             const double* __restrict__ scale,
                                             const RpOp<NP>& c, OpSrc<NP> os,
                                             const double* kb, int64_t n0, bool jend,
                                             int64_t sstride = 0) {
  static_assert(!SNAP || (E == 2 && !WT), "snapshots: launch chains on pair tiles");
  using G = RpGeo<NP, NW, E>;
  constexpr int T = G::T, LB = G::LB;
  constexpr int H = RpHalo<MS>::F;  // the level cone + the final state's neighbours, even
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0 && H % 2 == 0 && (E == 2 || E == 4),
                "pair tiles: aligned pairs");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  constexpr int CB = G::kLds;  // lds[CB + i] = bnd[i] (edge tiles)
  constexpr int CR = CB + MS * 5;  // the record's inflow values
  constexpr int FB = LB + 2;   // one face array
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t ec = e0 > 0 ? e0 : 0;
  const int64_t nd = c.ktot * NP;

  const int off = rp_load<NP, NW, E, EDGE, WT>(uin, e0, nd, lds);
  if constexpr (EDGE) {
    if (lane <= MS * 6) lds[CB + lane] = kb[lane];
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
    El[m] = elem_info<H, T, EDGE>(e0, el, c.ktot, c.K);
    sc[m] = c.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    // u^{n0}'s left-face jumps (record n0-1) from the staged nodal values, as step_tile
    jv[m] = us[0] - ((EDGE && El[m].first) ? lds[CR] : us[-1]);
  }
  if constexpr (!SNAP)
    if (n0 >= 1) rp_rec_put<E, EDGE, WT>(rec, n0 - 1, c.ktot, El, jv, ec);
  __syncthreads();  // the image is read: the face arrays alias it

  const double b4 = c.beta[4], b5 = c.beta[5], b3 = c.beta[3], b2 = c.beta[2];
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
        }
      }
      {
        const auto& op = os.get();
#pragma unroll
        for (int m = 0; m < E; ++m) {
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
      for (int m = 0; m < E; ++m) {
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
      if constexpr (!SNAP)
        if (l == 0 && st >= 1) rp_rec_put<E, EDGE, WT>(rec, n0 + st - 1, c.ktot, El, jv, ec);
    }
    if constexpr (SNAP)
      if (st < MS - 1) rp_snap_put<NP, E, EDGE>(rec + st * sstride, El, ue, uo);
  }
  if (!SNAP && jend) {
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
    rp_rec_put<E, EDGE, WT>(rec, n0 + MS - 1, c.ktot, El, jv, ec);
  }
  __syncthreads();  // the last face reads are done: the image is rewritten
  rp_store<NP, NW, E, H, EDGE, WT>(last, tile * TE * NP, nd, lds, ue, uo, false);
}

// Where the adjoint tile's indicator goes.  Launch-per-block kernels: eta_update with the
// launch's mode bits.  The dataflow sweep (WT): a block other than the last stores its partial
// sum to `part_out`; the last block adds the earlier blocks' partials `part_in[0..np)` (rows of
// ktot, in block order) in the order the separate launches would have, then applies the mode:
//   v = (assign ? p_0 : eta + p_0) + p_1 + ... + own;  abs  -- bit-identical to launches.
struct EtaSink {
  double* eta;         // the caller's indicator (final value)
  double* part_out;    // WT, not the last block: this block's partial sums
  const double* part_in;
  int64_t part_ld;
  int32_t nparts;      // partial rows to combine (last block)
  int32_t mode;        // kEta* bits; 0: no indicator
  // WT, last block: the lane's best (|eta|, element) of its final values under numpy's
  // argmax order (am_better), for the dataflow sweep's fused refine decision
  bool argmax;
  double bv;
  int64_t bi;
};

// numpy.argmax order: NaN is the maximum, ties go to the lowest index (a strict total order
// on (value, index), so any reduction tree gives the same winner; dg_argmax's rule).
__device__ __forceinline__ bool am_better(double va, int64_t ia, double vb, int64_t ib) {
  const bool na = isnan(va), nb = isnan(vb);
  if (na != nb) return na;
  if (!na && va != vb) return va > vb;
  return ia < ib;
}

// Adjoint: MS reverse steps st = MS-1..0 of the tile, each
//   eta += DWR(u^{n0+st+1}'s recorded jumps, w^{n0+st+1});  w^{n0+st} = P(z^T) w^{n0+st+1}
// (terminal functionals only: no source; the inflow forcing does not depend on u).  Horner
// in z^T: t = beta_4 w + beta_5 z^T w; t = beta_k w + z^T t, k = 3, 2, 1; w = w + z^T t, with
// z^T v = L^T (sc v): the face adjoints g0 = le.ve + lo.vo, g1 = lo.vo - le.ve of each element
// go to its neighbours (one exchange per level), the transposed volume blocks stay local.
template <int NP, bool UNI, int NW, int E, int MS, bool EDGE, bool WT>
__device__ __forceinline__ void rp_adj_tile(double* __restrict__ lds, int64_t tile,
                                            const double* __restrict__ win,
                                            double* __restrict__ wout,
                                            const double* __restrict__ rec,
                                            EtaSink& es,
                                            const double* __restrict__ scale,
                                            const RpOp<NP>& c, OpSrc<NP> os, int64_t n0) {
  using G = RpGeo<NP, NW, E>;
  constexpr int T = G::T, LB = G::LB;
  constexpr int H = RpHalo<MS>::A;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0 && H % 2 == 0 && (E == 2 || E == 4),
                "pair tiles: aligned pairs");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO, N = NP - 1;
  constexpr int FB = LB + 2;
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t ec = e0 > 0 ? e0 : 0;
  const int64_t nd = c.ktot * NP;
  const int64_t ea = e0 + E * lane;  // the lane's first element (even)
  const int has_eta = es.mode;

  const int off = rp_load<NP, NW, E, EDGE, WT>(win, e0, nd, lds);
  // the left-face jumps of u^{n0+st+1} (record n0+st) of the lane's two elements and of its
  // right neighbour: one 16-byte and one 8-byte load per lane and step, prefetched a step ahead
  double jn[E + 1];
  rp_rec_get<E, EDGE, WT>(rec, n0 + MS - 1, c.ktot, ea, ec, jn);
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
    El[m] = elem_info<H, T, EDGE>(e0, el, c.ktot, c.K);
    sc[m] = c.sc;
    if constexpr (!UNI) sc[m] *= El[m].inrange ? scale[El[m].kl] : 0.0;
    eacc[m] = 0.0;
  }
  __syncthreads();  // the image is read: the face arrays alias it

  const double b4 = c.beta[4], b5 = c.beta[5], b3 = c.beta[3], b2 = c.beta[2];
  double te[E][NE], to[E][NO];  // the Horner accumulator
#pragma unroll 1
  for (int st = MS - 1; st >= 0; --st) {
    // du0 = j_e; du1 = -j_{e+1} (0 at a trajectory's last element): du0 - du1 and du0 + du1
    // are the snapshot path's doubles bit for bit (dg_common.h rec_ld).  The next step's
    // record is loaded after this step's indicator has read the current one.
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
      // buffers alternate over the launch's global level index (no barrier between a step's
      // last level and the next step's first)
      const int f0 = (((MS - 1 - st) * 5 + l) & 1) * 2 * FB, f1 = f0 + FB;
      // the level's input v (w at level 0, t after), scaled by the metric: q = sc v
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
      lds[f0 + lane + 1] = g0[0];      // the lane's first element: adjoint of its uL
      lds[f1 + lane + 1] = g1[E - 1];  // the lane's last element: adjoint of its uR
      __builtin_amdgcn_sched_barrier(0);
      // the transposed volume term, before the barrier: a = c w + Qoe^T qo (even), c w +
      // Qeo^T qe (odd); level 0 starts from the bare products
      // odd outputs first (they read the even inputs, which then die), then the even ones
      // (reading the odd inputs): fewer values live at once than one loop over both
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
        for (int k = 0; k < NO; ++k) pin(ao[m][k]);
      }
      __builtin_amdgcn_sched_barrier(0);
      const auto& or_ = os.get();
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
            t = or_.Qoe[j] * qo[m][0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NO; ++k) t = fma(or_.Qoe[k * NE + j], qo[m][k], t);
          ae[m][j] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(ae[m][k]);
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
  if (has_eta) {
    if constexpr (WT) {
      // partial rows and the final combine; pairs are 16-byte aligned (ea even, ktot rows of
      // even length are not required: 8-byte accesses)
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
  __syncthreads();  // the last face reads are done: the image is rewritten
  rp_store<NP, NW, E, H, EDGE, WT>(wout, tile * TE * NP, nd, lds, we, wo, true);
}

}  // namespace dgr
