// dg_dwr_tiles.h — the p-enriched DWR estimate's reverse steps in Horner form (round 5).
// Internal to libdgadv.so; included by dg_dwr.hip.
//
// Per reverse step n (dg_dwr.hip, "k_adj_p"): prolong the order-N snapshot u^n to order N+1
// (v = P u^n), recompute S_{N+1}(v), pair the residual R^n = P u^{n+1} - S_{N+1}(v) with the
// order-(N+1) adjoint w^{n+1} (eta -= w^{n+1} . R^n), then w^n = S_{N+1}^T w^{n+1}.  Round 3
// ran both S and S^T as the five low-storage stages (utils/One_code.mlx:120-137).  Here both
// are the LSERK4 step's stability polynomial in Horner form (dg_rec_tiles.h "Horner form"):
//   S(v)    = v + Z_{b0}(t),  t = v + Z_{b1}(t'), ...,  t'' = beta_4 v + beta_5 Z_{b4/beta5}(v)
//   S^T w   = w + z^T t,      t = w + z^T t', ...,     t'' = beta_4 w + beta_5 z^T w
// five applications of the order-(N+1) operator each way (one face exchange each), with no
// low-storage carry: at Np = 6 about 290 + 300 fp64 operations per element and step instead
// of the stage loop's 368 + 360.  The prolongation (even/odd blocks), the residual pairing,
// the tile layout (one element per lane, the next snapshot tile loaded into registers during
// the reverse levels and committed to LDS after them), the halo (5 per step) and the outputs
// are round 3's.  The order-(N+1) operator and prolongation blocks are re-read
// from the kernel-argument segment where they are used (OpSrc, dg_rec_tiles.h): together they
// are 39 doubles at Np = 6, which held as arguments spilled SGPRs into VGPR lanes.
// Sources: matlab/MAIN.m:32-34 (adjoint at order Ns+1), matlab/adj_march.m:103-117 (err(k) =
// v_k' R_k), python/Main_finite_difference.py:79-94 (errEst); DESIGN.md §6c.
#pragma once
#include "dg_step_tile.h"

namespace dgk {

// Prolongation in even/odd coordinates: e_hi = Pe e_lo, o_hi = Po o_lo.
template <int NPL> struct PrEO {
  static constexpr int NPH = NPL + 1;
  static constexpr int NEL = (NPL + 1) / 2, NOL = NPL / 2;
  static constexpr int NEH = (NPH + 1) / 2, NOH = NPH / 2;
  double Pe[NEH * NEL];
  double Po[NOH * NOL];
};

// The Horner-form estimate's launch arguments (MS reverse steps n0+MS-1 .. n0).  op: the
// order-(N+1) operator, folded, dt*2/h folded on uniform meshes; bnd[5 st + l]: the inflow
// weights of level l of step n0+st's forward recompute (rp_block_bnd: b_4/beta_5, b_3, b_2,
// b_1, b_0), then one 0.
template <int NPL, int MS> struct AdjPHArgs {
  EOArgs<NPL + 1> op;
  PrEO<NPL> pr;
  double sc;        // dt (non-uniform meshes multiply by scale[k])
  double beta[6];   // the stability polynomial's coefficients (rk_poly)
  double bnd[MS * 5 + 1];
  int64_t ktot;
  int64_t stride;   // doubles between consecutive order-N snapshots
  int32_t K;
  int32_t has_eta;  // kEta* bits
  int32_t xcd;
  int32_t term;     // 1: the terminal weight is P u^{n0+MS} (w's input is not read)
};

// The terminal weight w = P u (J = |P u|^2 / 2) in dual even/odd coordinates from the primal
// even/odd P u, through the nodal values exactly as dg_prolong (k_prolong: from_eo) + the
// adjoint's load (w_k + w_{N-k}, w_k - w_{N-k}) compute it: bit-identical to that pair.
template <int NPH>
__device__ __forceinline__ void terminal_from_prolong(const double* ne, const double* no,
                                                      double* we, double* wo) {
  constexpr int NE = EOArgs<NPH>::NE, NO = EOArgs<NPH>::NO;
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    const double a = ne[k] + no[k], b = ne[k] - no[k];
    we[k] = a + b;
    wo[k] = a - b;
  }
  if constexpr (NE > NO) we[NO] = ne[NO];
}

template <int NPL, class PR>
__device__ __forceinline__ void prolong_eo(const double* __restrict__ u, const PR& pr,
                                           double* ev, double* od) {
  using R = PrEO<NPL>;
  double el[R::NEL], ol[R::NOL];
  to_eo<NPL>(u, el, ol);
#pragma unroll
  for (int k = 0; k < R::NEH; ++k) {
    double t = pr.Pe[k * R::NEL] * el[0];
#pragma unroll
    for (int j = 1; j < R::NEL; ++j) t = fma(pr.Pe[k * R::NEL + j], el[j], t);
    ev[k] = t;
  }
#pragma unroll
  for (int k = 0; k < R::NOH; ++k) {
    double t = pr.Po[k * R::NOL] * ol[0];
#pragma unroll
    for (int j = 1; j < R::NOL; ++j) t = fma(pr.Po[k * R::NOL + j], ol[j], t);
    od[k] = t;
  }
  // Materialised: at NPL <= 3 a block row is one bare product, which fp-contract would fuse
  // into whatever adds it next -- differently in k_prolong (from_eo) and in the estimate's
  // tiles (the terminal weight, the residual), so the two paths would not agree bit for bit.
#pragma unroll
  for (int k = 0; k < R::NEH; ++k) pin(ev[k]);
#pragma unroll
  for (int k = 0; k < R::NOH; ++k) pin(od[k]);
}

// A kernel-argument block read where it is used (dgr::OpSrc's technique for any block).
template <class T> struct KaSrc {
  const DG_KAS T* p;
  __device__ __forceinline__ const DG_KAS T& get() const {
    const DG_KAS T* q = p;
    asm volatile("" : "+s"(q));
    return *q;
  }
};

// A workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup release fence
// as well, and with a direct-to-LDS load in flight the compiler drains vmcnt(0) before it;
// between the levels nothing but LDS is exchanged, so the loads stay in flight across these.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// tile_issue's interior load straight into the LDS image (global_load_lds_dwordx4: the lanes
// of a wave write 64 consecutive 16-byte slots from M0, the wave's base): no registers held
// while the loads are in flight.  Interior tiles only (every 16-byte slot in range).  The
// image is complete after `s_waitcnt vmcnt(0)` and a barrier.  Returns the image offset.
// AUX: the cache-policy bits (dgr::kSc1 for bytes written earlier in the same launch).
template <int NP, int W, int AUX = 0>
__device__ __forceinline__ int tile_issue_lds(const double* __restrict__ g, int64_t e0,
                                              double* __restrict__ lds) {
  using G = TileGeo<NP, W>;
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) void glb_void;
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  const int off = int(d0 - base);
  const int nvec = (G::T * NP + off + 1) >> 1;
  const double* gb = g + base;
  const int wb = int(threadIdx.x) & ~63;
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = threadIdx.x + q * G::LB;
    if (v < nvec)
      __builtin_amdgcn_global_load_lds((glb_void*)(gb + 2 * v),
                                       (lds_void*)(lds + 2 * (q * G::LB + wb)), 16, 0, AUX);
  }
  return off;
}

// One element's indicator in a dataflow launch (rp_adj_tile's WT branch): a block other than
// the last writes its partial sum to its own row; the last adds the caller's eta (unless
// assigning) and the earlier blocks' rows in launch order, then its own -- the additions of
// the launch-per-block chain, bit for bit -- and keeps the lane's (|eta|, element) winner for
// the fused refine decision.  ec: the tile's first output element (wave-uniform).
__device__ __forceinline__ void eta_sink_put(dgr::EtaSink& es, int64_t ec, int64_t e,
                                             double acc) {
  const uint32_t o = uint32_t(e - ec) * 8u;
  if (es.part_out) {
    dgr::wt_st8(dgr::wt_rsrc(es.part_out + ec), o, acc);
    return;
  }
  double v;
  if (es.nparts > 0) {
    v = dgr::wt_ld8(dgr::wt_rsrc(es.part_in + ec), o);
    if (!(es.mode & kEtaAssign)) v = es.eta[e] + v;
    for (int q = 1; q < es.nparts; ++q)
      v = v + dgr::wt_ld8(dgr::wt_rsrc(es.part_in + q * es.part_ld + ec), o);
    v = v + acc;
  } else {
    v = (es.mode & kEtaAssign) ? acc : es.eta[e] + acc;
  }
  if (es.mode & kEtaAbs) v = fabs(v);
  dgr::wt_st8(dgr::wt_rsrc(es.eta + ec), o, v);
  if (es.argmax && dgr::am_better(fabs(v), e, es.bv, es.bi)) {
    es.bv = fabs(v);
    es.bi = e;
  }
}

template <int NPL, int W> struct PHGeo {
  static constexpr int NPH = NPL + 1;
  static constexpr int LB = kBlock * W, T = LB;
  static constexpr int kImgD = T * NPH + 2;  // the image holds the w tile or a snapshot tile
  static constexpr int kFB = (kImgD + 1) & ~1;
  static constexpr int kFaceD = 4 * (T + 2);  // two double-buffered face arrays, padded by 1
  static constexpr int kLds = kFB + kFaceD;
};

// One tile of a Horner-form estimate launch.  snap = u^{n0}; reads u^{n0} .. u^{n0+MS}.
// `ka`: the argument block in the kernarg segment (operator and prolongation reads); `kbnd`:
// its bnd array there (the edge tiles' lane-indexed reads).
// GL: interior tiles load the next snapshot straight into LDS (tile_issue_lds).  WT: a work
// item of the one-launch sweep (k_adjp_flow): w is loaded sc1 and stored write-through, and
// the indicator goes to `es` (this block's partial row, or the final combine in the last
// block), as the jump sweep's rp_adj_tile does.  A: the argument struct (op, pr, sc, beta,
// ktot, stride, K, has_eta).  term: the terminal weight is P u^{n0+MS} (win is not read).
// wait_inputs: called by all threads once the snapshot loads are issued, before w is loaded
// (a dataflow item's poll of its producers and the barrier after it); wait_snapshots: before
// the snapshot loads.  SWT: the snapshots are loaded sc1 (written earlier in the same launch).
struct NoWait {
  __device__ void operator()() const {}
};

template <int NPL, bool UNI, int W, int MS, bool EDGE, bool GL = false, bool WT = false,
          class A = AdjPHArgs<NPL, MS>, class WaitF = NoWait, bool SWT = false,
          class WaitS = NoWait>
__device__ __forceinline__ void adjph_tile(double* __restrict__ lds, int64_t tile,
                                           const double* __restrict__ win,
                                           double* __restrict__ wout,
                                           const double* __restrict__ snap,
                                           double* __restrict__ eta,
                                           const double* __restrict__ scale,
                                           const A& args, const DG_KAS A* ka,
                                           const double* kbnd, bool term,
                                           dgr::EtaSink* es = nullptr,
                                           const WaitF& wait_inputs = WaitF(),
                                           const WaitS& wait_snapshots = WaitS()) {
  static_assert(!SWT || GL, "sc1 snapshot loads: direct-to-LDS tiles only");
  constexpr int NPH = NPL + 1;
  using G = PHGeo<NPL, W>;
  constexpr int T = G::T, LB = G::LB;
  // the reverse cone is 5 elements per step; the forward recompute of a step needs 5 more
  // around the output elements, which the halo of the steps still to come covers
  constexpr int H = MS * 5;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NPH>::NE, NO = EOArgs<NPH>::NO, NH = NPH - 1;
  const KaSrc<EOArgs<NPH>> os{reinterpret_cast<const DG_KAS EOArgs<NPH>*>(
      reinterpret_cast<const DG_KAS char*>(ka) + offsetof(A, op))};
  const KaSrc<PrEO<NPL>> ps{reinterpret_cast<const DG_KAS PrEO<NPL>*>(
      reinterpret_cast<const DG_KAS char*>(ka) + offsetof(A, pr))};
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t ndh = args.ktot * NPH, ndl = args.ktot * NPL;
  constexpr int CB = G::kLds;  // lds[CB + 5 st + l]: level inflow weights; lds[CB + 5 MS] = 0

  TileRegs<NPH, W> pw;
  TileRegs<NPL, W> pa, pb;
  // the snapshots (an earlier launch's) are loaded while a dataflow item waits for its
  // producers (wait_inputs), then w
  wait_snapshots();  // (SWT: the snapshots are this launch's: their producers first)
  if constexpr (SWT) {
    tile_issue_wt<NPL, W, EDGE>(snap + MS * args.stride, e0, ndl, pa);
    tile_issue_wt<NPL, W, EDGE>(snap + (MS - 1) * args.stride, e0, ndl, pb);
  } else {
    tile_issue<NPL, W, EDGE>(snap + MS * args.stride, e0, ndl, pa);
    tile_issue<NPL, W, EDGE>(snap + (MS - 1) * args.stride, e0, ndl, pb);
  }
  wait_inputs();
  if (!term) {
    if constexpr (WT) tile_issue_wt<NPH, W, EDGE>(win, e0, ndh, pw);
    else tile_issue<NPH, W, EDGE>(win, e0, ndh, pw);
  }
  if (!term) tile_commit<NPH, W>(pw, lds);
  if constexpr (EDGE) {
    if (lane <= MS * 5) lds[CB + lane] = kbnd[lane];  // lane-indexed: from the kernarg segment
  }
  __syncthreads();
  double we[NE], wo[NO];  // the order-(N+1) adjoint in dual even/odd coordinates
  if (!term) {
    const double* w = lds + pw.off + lane * NPH;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[k] = w[k] + w[NH - k];
      wo[k] = w[k] - w[NH - k];
    }
    if constexpr (NE > NO) we[NO] = w[NO];
  }
  const Elem E = elem_info<H, T, EDGE>(e0, lane, args.ktot, args.K);
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;
  __syncthreads();  // the w image is read
  tile_commit<NPL, W>(pa, lds);
  __syncthreads();
  double ne[NE], no[NO];  // P u^{n+1} of this lane's element
  prolong_eo<NPL>(lds + pa.off + lane * NPL, ps.get(), ne, no);
  if (term) terminal_from_prolong<NPH>(ne, no, we, wo);
  __syncthreads();
  tile_commit<NPL, W>(pb, lds);
  int off = pb.off;
  __syncthreads();
  double eacc = 0.0;
  const double b4 = args.beta[4], b5 = args.beta[5], b3 = args.beta[3], b2 = args.beta[2];

#pragma unroll 1
  for (int st = MS - 1; st >= 0; --st) {
    // ---- v = P u^n ----
    double ve[NE], vo[NO];
    prolong_eo<NPL>(lds + off + lane * NPL, ps.get(), ve, vo);

    // ---- S_{N+1}(v) by Horner (rp_step_tile's level arithmetic at order N+1) ----
    double te[NE], to[NO];
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      const int fL = G::kFB + (l & 1) * 2 * (T + 2), fR = fL + (T + 2);
      {
        const double e = (l == 0) ? ve[0] : te[0], o = (l == 0) ? vo[0] : to[0];
        lds[fL + lane + 1] = e + o;
        lds[fR + lane + 1] = e - o;
      }
      __builtin_amdgcn_sched_barrier(0);
      double pe[NE], po[NO];
      {
        const auto& op = os.get();
        const double* xo = (l == 0) ? vo : to;
        const double* xe = (l == 0) ? ve : te;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          double a;
          int j0 = 0;
          if (UNI && l >= 3) {
            a = ve[k];
          } else if (UNI && l >= 1) {
            a = (l == 1 ? b3 : b2) * ve[k];
          } else {
            a = op.Qeo[k * NO] * xo[0];
            j0 = 1;
          }
#pragma unroll
          for (int j = j0; j < NO; ++j) a = fma(op.Qeo[k * NO + j], xo[j], a);
          pe[k] = a;
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          double a;
          int j0 = 0;
          if (UNI && l >= 3) {
            a = vo[k];
          } else if (UNI && l >= 1) {
            a = (l == 1 ? b3 : b2) * vo[k];
          } else {
            a = op.Qoe[k * NE] * xe[0];
            j0 = 1;
          }
#pragma unroll
          for (int j = j0; j < NE; ++j) a = fma(op.Qoe[k * NE + j], xe[j], a);
          po[k] = a;
        }
      }
#pragma unroll
      for (int k = 0; k < NE; ++k) pin(pe[k]);
#pragma unroll
      for (int k = 0; k < NO; ++k) pin(po[k]);
      __syncthreads();
      // a trajectory's first element reads the level's inflow weight, its last one its own
      // right node (index selection: dg_common.h)
      const int iL = EDGE && E.first ? CB + st * 5 + l : fR + lane;
      const int iR = EDGE && E.last ? fR + lane + 1 : fL + lane + 2;
      const double vL = lds[iL], vR = lds[iR];
      const double dlt = vR - vL, sig = -(vL + vR);
      const auto& ol = os.get();
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const double z = fma(ol.le[k], dlt, pe[k]);
        if constexpr (UNI) {
          if (l == 0) te[k] = fma(b5, z, b4 * ve[k]);
          else te[k] = z;  // level 4: S itself
        } else {
          if (l == 0) te[k] = fma(b5 * sc, z, b4 * ve[k]);
          else if (l < 3) te[k] = fma(sc, z, (l == 1 ? b3 : b2) * ve[k]);
          else te[k] = fma(sc, z, ve[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        const double z = fma(ol.lo[k], sig, po[k]);
        if constexpr (UNI) {
          if (l == 0) to[k] = fma(b5, z, b4 * vo[k]);
          else to[k] = z;
        } else {
          if (l == 0) to[k] = fma(b5 * sc, z, b4 * vo[k]);
          else if (l < 3) to[k] = fma(sc, z, (l == 1 ? b3 : b2) * vo[k]);
          else to[k] = fma(sc, z, vo[k]);
        }
      }
    }

    // ---- eta -= w^{n+1} . (P u^{n+1} - S_{N+1}(P u^n)) in dual x primal even/odd ----
    if (args.has_eta) {
      double c = 0.0;
#pragma unroll
      for (int k = 0; k < NE; ++k) c = fma(we[k], ne[k] - te[k], c);
#pragma unroll
      for (int k = 0; k < NO; ++k) c = fma(wo[k], no[k] - to[k], c);
      eacc -= c;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) ne[k] = ve[k];
#pragma unroll
    for (int k = 0; k < NO; ++k) no[k] = vo[k];
    // the next snapshot's loads, in flight behind the reverse levels (issued here rather than
    // at the step start: the forward levels hold the most values, and 12 more VGPRs there
    // would cost a workgroup per CU).  GL: interior tiles load straight into the image (its
    // readers, the prolongation at the step start, are 5 barriers behind) and edge tiles load
    // at the step end, so no prefetch registers are held.
    constexpr bool kGL = GL && !EDGE;
    int offn = 0;
    if constexpr (kGL) {
      if (st > 0)
        offn = tile_issue_lds<NPL, W, SWT ? dgr::kSc1 : 0>(snap + (st - 1) * args.stride, e0, lds);
    } else if constexpr (!GL) {
      if (st > 0) tile_issue<NPL, W, EDGE>(snap + (st - 1) * args.stride, e0, ndl, pa);
    }

    // ---- w^n = S_{N+1}^T w^{n+1} by Horner (rp_adj_tile's level arithmetic at order N+1) ----
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      const int f0 = G::kFB + ((l + 1) & 1) * 2 * (T + 2), f1 = f0 + (T + 2);
      double qe[NE], qo[NO], gd = 0.0, gs = 0.0;
      {
        const auto& op = os.get();
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          const double v = (l == 0) ? we[k] : te[k];
          qe[k] = UNI ? v : sc * v;
          gd = fma(op.le[k], qe[k], gd);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          const double v = (l == 0) ? wo[k] : to[k];
          qo[k] = UNI ? v : sc * v;
          gs = fma(op.lo[k], qo[k], gs);
        }
      }
      const double g0 = gd + gs, g1 = gs - gd;
      lds[f0 + lane + 1] = g0;
      lds[f1 + lane + 1] = g1;
      __builtin_amdgcn_sched_barrier(0);
      double ae[NE], ao[NO];
      {
        const auto& op = os.get();
#pragma unroll
        for (int j = 0; j < NO; ++j) {
          double t;
          int k0 = 0;
          if (l >= 3) {
            t = wo[j];
          } else if (l >= 1) {
            t = (l == 1 ? b3 : b2) * wo[j];
          } else {
            t = op.Qeo[j] * qe[0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NE; ++k) t = fma(op.Qeo[k * NO + j], qe[k], t);
          ao[j] = t;
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(ao[k]);
      }
      __builtin_amdgcn_sched_barrier(0);
      {
        const auto& op = os.get();
#pragma unroll
        for (int j = 0; j < NE; ++j) {
          double t;
          int k0 = 0;
          if (l >= 3) {
            t = we[j];
          } else if (l >= 1) {
            t = (l == 1 ? b3 : b2) * we[j];
          } else {
            t = op.Qoe[j] * qo[0];
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < NO; ++k) t = fma(op.Qoe[k * NE + j], qo[k], t);
          ae[j] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(ae[k]);
      }
      if constexpr (GL) lds_barrier();
      else __syncthreads();
      // nothing arrives at a trajectory's first element from the left (its uL is the
      // inflow); its last element's uR is its own u_N (du1 = 0)
      const double gl = lds[EDGE && E.first ? CB + MS * 5 : f1 + lane];
      const double gr = lds[EDGE && E.last ? f1 + lane + 1 : f0 + lane + 2];
      ae[0] -= gl + gr;
      ao[0] += gr - gl;
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        if (l == 0) te[k] = fma(b5, ae[k], b4 * we[k]);
        else if (l < 4) te[k] = ae[k];
        else we[k] = ae[k];
      }
#pragma unroll
      for (int k = 0; k < NO; ++k) {
        if (l == 0) to[k] = fma(b5, ao[k], b4 * wo[k]);
        else if (l < 4) to[k] = ao[k];
        else wo[k] = ao[k];
      }
    }
    // the image's readers (the prolongation at the step start) are 10 level barriers behind;
    // the next step's prolongation reads what every wave commits here
    if (st > 0) {
      if constexpr (kGL) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        off = offn;
      } else {
        if constexpr (GL && SWT) tile_issue_wt<NPL, W, EDGE>(snap + (st - 1) * args.stride, e0, ndl, pa);
        else if constexpr (GL) tile_issue<NPL, W, EDGE>(snap + (st - 1) * args.stride, e0, ndl, pa);
        tile_commit<NPL, W>(pa, lds);
        off = pa.off;
      }
      __syncthreads();
    }
  }

  if constexpr (WT) {
    if (args.has_eta && E.valid) eta_sink_put(*es, tile * TE, E.e, eacc);
  } else {
    if (args.has_eta && E.valid) eta_update(eta, E.e, eacc, args.has_eta);
  }
  {
    const double(*pwe)[NE] = &we;
    const double(*pwo)[NO] = &wo;
    stage_out<NPH, W, H>(lds, pwe, pwo, true);  // the image's last reads are 5 barriers behind
  }
  __syncthreads();
  const int64_t o0 = tile * TE * NPH;
  if constexpr (EDGE) {
    const int64_t rem = ndh - o0;
    if constexpr (WT)
      dgr::store_run_wt<LB>(wout, o0, rem < int64_t(TE) * NPH ? rem : int64_t(TE) * NPH, lds);
    else
      store_run<LB>(wout, o0, rem < int64_t(TE) * NPH ? rem : int64_t(TE) * NPH, lds);
  } else {
    if constexpr (WT) dgr::store_full_wt<TE * NPH, LB>(wout, o0, lds);
    else store_full<TE * NPH, LB>(wout, o0, lds);
  }
}


// ---------------------------------------------------------------------------
// The pipelined form (k_adj_pq): the forward recompute of step n-1 runs beside the reverse
// step n, level by level, sharing each level's barrier.  The two chains are independent (S
// reads the snapshot, S^T reads w^{n+1}); the residual of step n-1 pairs with w^n, which the
// same iteration produces:
//   prologue:     S(P u^{n0+MS-1})                 -> eta_{n0+MS-1} with w^{n0+MS}
//   iteration n:  S(P u^{n-1})  ||  w^n = S^T w^{n+1} -> eta_{n-1} with w^n   (n = n0+MS-1 .. n0+1)
//   last:         w^{n0} = S^T w^{n0+1}
// 5 (MS + 1) level barriers per launch instead of 10 MS, and two independent dependency chains
// per lane between barriers.  Same arithmetic per element as adjph_tile (bit-identical).
// ---------------------------------------------------------------------------
template <int NPL, int W> struct PQGeo {
  static constexpr int NPH = NPL + 1;
  static constexpr int LB = kBlock * W, T = LB;
  static constexpr int kImgD = T * NPH + 2;
  static constexpr int kFB = (kImgD + 1) & ~1;
  static constexpr int kFA = T + 2;              // one face array (padded by one each side)
  static constexpr int kFaceD = 2 * 4 * kFA;     // 4 arrays (F left/right, R left/right), x2
  static constexpr int kLds = kFB + kFaceD;
};

// One level l of the forward chain (DOF: tF <- level l of S(v), l == 4: S itself) and/or the
// reverse chain (DOR: tR <- level l of S^T w, l == 4: w itself), one barrier.  ibF: the inflow
// weight's LDS slot of this level (edge tiles).
template <int NPH, bool UNI, bool EDGE, bool DOF, bool DOR, int L, class OP>
__device__ __forceinline__ void pq_level(double* __restrict__ lds, int fb, const Elem& E, double sc,
                                         const OP& os, const double* beta, int ibF, int izR,
                                         double* ve, double* vo, double* fe, double* fo,
                                         double* we, double* wo, double* re, double* ro) {
  constexpr int NE = EOArgs<NPH>::NE, NO = EOArgs<NPH>::NO;
  constexpr int FA = (kBlock * 0) + 0;  // (unused)
  (void)FA;
  const int lane = threadIdx.x;
  const int T2 = int(blockDim.x) + 2;
  // face arrays of this level: F left/right faces at fb, fb + T2; R g0/g1 at fb + 2 T2, + 3 T2
  const int fF0 = fb, fFN = fb + T2, fR0 = fb + 2 * T2, fR1 = fb + 3 * T2;
  const double b4 = beta[4], b5 = beta[5], b3 = beta[3], b2 = beta[2];
  double pe[NE], po[NO], qe[NE], qo[NO], ae[NE], ao[NO];
  if constexpr (DOF) {
    const double e = (L == 0) ? ve[0] : fe[0], o = (L == 0) ? vo[0] : fo[0];
    lds[fF0 + lane + 1] = e + o;
    lds[fFN + lane + 1] = e - o;
  }
  if constexpr (DOR) {
    const auto& op = os.get();
    double gd = 0.0, gs = 0.0;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const double v = (L == 0) ? we[k] : re[k];
      qe[k] = UNI ? v : sc * v;
      gd = fma(op.le[k], qe[k], gd);
    }
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      const double v = (L == 0) ? wo[k] : ro[k];
      qo[k] = UNI ? v : sc * v;
      gs = fma(op.lo[k], qo[k], gs);
    }
    lds[fR0 + lane + 1] = gd + gs;
    lds[fR1 + lane + 1] = gs - gd;
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (DOF) {
    const auto& op = os.get();
    const double* xo = (L == 0) ? vo : fo;
    const double* xe = (L == 0) ? ve : fe;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      double a;
      int j0 = 0;
      if (UNI && L >= 3) {
        a = ve[k];
      } else if (UNI && L >= 1) {
        a = (L == 1 ? b3 : b2) * ve[k];
      } else {
        a = op.Qeo[k * NO] * xo[0];
        j0 = 1;
      }
#pragma unroll
      for (int j = j0; j < NO; ++j) a = fma(op.Qeo[k * NO + j], xo[j], a);
      pe[k] = a;
    }
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      double a;
      int j0 = 0;
      if (UNI && L >= 3) {
        a = vo[k];
      } else if (UNI && L >= 1) {
        a = (L == 1 ? b3 : b2) * vo[k];
      } else {
        a = op.Qoe[k * NE] * xe[0];
        j0 = 1;
      }
#pragma unroll
      for (int j = j0; j < NE; ++j) a = fma(op.Qoe[k * NE + j], xe[j], a);
      po[k] = a;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) pin(pe[k]);
#pragma unroll
    for (int k = 0; k < NO; ++k) pin(po[k]);
  }
  if constexpr (DOR) {
    const auto& op = os.get();
#pragma unroll
    for (int j = 0; j < NO; ++j) {
      double t;
      int k0 = 0;
      if (L >= 3) {
        t = wo[j];
      } else if (L >= 1) {
        t = (L == 1 ? b3 : b2) * wo[j];
      } else {
        t = op.Qeo[j] * qe[0];
        k0 = 1;
      }
#pragma unroll
      for (int k = k0; k < NE; ++k) t = fma(op.Qeo[k * NO + j], qe[k], t);
      ao[j] = t;
    }
#pragma unroll
    for (int k = 0; k < NO; ++k) pin(ao[k]);
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      double t;
      int k0 = 0;
      if (L >= 3) {
        t = we[j];
      } else if (L >= 1) {
        t = (L == 1 ? b3 : b2) * we[j];
      } else {
        t = op.Qoe[j] * qo[0];
        k0 = 1;
      }
#pragma unroll
      for (int k = k0; k < NO; ++k) t = fma(op.Qoe[k * NE + j], qo[k], t);
      ae[j] = t;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) pin(ae[k]);
  }
  __syncthreads();
  if constexpr (DOF) {
    const int iL = EDGE && E.first ? ibF : fFN + lane;
    const int iR = EDGE && E.last ? fFN + lane + 1 : fF0 + lane + 2;
    const double vL = lds[iL], vR = lds[iR];
    const double dlt = vR - vL, sig = -(vL + vR);
    const auto& ol = os.get();
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const double z = fma(ol.le[k], dlt, pe[k]);
      if constexpr (UNI) {
        if (L == 0) fe[k] = fma(b5, z, b4 * ve[k]);
        else fe[k] = z;
      } else {
        if (L == 0) fe[k] = fma(b5 * sc, z, b4 * ve[k]);
        else if (L < 3) fe[k] = fma(sc, z, (L == 1 ? b3 : b2) * ve[k]);
        else fe[k] = fma(sc, z, ve[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      const double z = fma(ol.lo[k], sig, po[k]);
      if constexpr (UNI) {
        if (L == 0) fo[k] = fma(b5, z, b4 * vo[k]);
        else fo[k] = z;
      } else {
        if (L == 0) fo[k] = fma(b5 * sc, z, b4 * vo[k]);
        else if (L < 3) fo[k] = fma(sc, z, (L == 1 ? b3 : b2) * vo[k]);
        else fo[k] = fma(sc, z, vo[k]);
      }
    }
  }
  if constexpr (DOR) {
    const double gl = lds[EDGE && E.first ? izR : fR1 + lane];
    const double gr = lds[EDGE && E.last ? fR1 + lane + 1 : fR0 + lane + 2];
    ae[0] -= gl + gr;
    ao[0] += gr - gl;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      if (L == 0) re[k] = fma(b5, ae[k], b4 * we[k]);
      else if (L < 4) re[k] = ae[k];
      else we[k] = ae[k];
    }
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      if (L == 0) ro[k] = fma(b5, ao[k], b4 * wo[k]);
      else if (L < 4) ro[k] = ao[k];
      else wo[k] = ao[k];
    }
  }
}

// The five levels of one iteration; buffers alternate over the level index (5 per iteration:
// `parity` carries it across iterations).
template <int NPH, bool UNI, bool EDGE, bool DOF, bool DOR, class OP>
__device__ __forceinline__ void pq_iteration(double* __restrict__ lds, int fbase, int& parity,
                                             const Elem& E, double sc, const OP& os,
                                             const double* beta, int ibF0, int izR, double* ve,
                                             double* vo, double* fe, double* fo, double* we,
                                             double* wo, double* re, double* ro) {
  const int T2 = int(blockDim.x) + 2;
#define DG_PQ_LEVEL(LV)                                                                        \
  pq_level<NPH, UNI, EDGE, DOF, DOR, LV>(lds, fbase + ((parity + LV) & 1) * 4 * T2, E, sc, os, \
                                         beta, ibF0 + LV, izR, ve, vo, fe, fo, we, wo, re, ro)
  DG_PQ_LEVEL(0);
  DG_PQ_LEVEL(1);
  DG_PQ_LEVEL(2);
  DG_PQ_LEVEL(3);
  DG_PQ_LEVEL(4);
#undef DG_PQ_LEVEL
  parity ^= 1;  // 5 levels: the next iteration starts on the other buffer
}

template <int NPL, bool UNI, int W, int MS, bool EDGE>
__device__ __forceinline__ void adjpq_tile(double* __restrict__ lds, int64_t tile,
                                           const double* __restrict__ win,
                                           double* __restrict__ wout,
                                           const double* __restrict__ snap,
                                           double* __restrict__ eta,
                                           const double* __restrict__ scale,
                                           const AdjPHArgs<NPL, MS>& args,
                                           const DG_KAS AdjPHArgs<NPL, MS>* ka,
                                           const double* kbnd) {
  constexpr int NPH = NPL + 1;
  using G = PQGeo<NPL, W>;
  using A = AdjPHArgs<NPL, MS>;
  constexpr int T = G::T, LB = G::LB;
  constexpr int H = MS * 5;
  constexpr int TE = T - 2 * H;
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NPH>::NE, NO = EOArgs<NPH>::NO, NH = NPH - 1;
  const KaSrc<EOArgs<NPH>> os{reinterpret_cast<const DG_KAS EOArgs<NPH>*>(
      reinterpret_cast<const DG_KAS char*>(ka) + offsetof(A, op))};
  const KaSrc<PrEO<NPL>> ps{reinterpret_cast<const DG_KAS PrEO<NPL>*>(
      reinterpret_cast<const DG_KAS char*>(ka) + offsetof(A, pr))};
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t ndh = args.ktot * NPH, ndl = args.ktot * NPL;
  constexpr int CB = G::kLds;  // lds[CB + 5 st + l]: level inflow weights; lds[CB + 5 MS] = 0

  TileRegs<NPH, W> pw;
  TileRegs<NPL, W> pa, pb;
  const bool term = args.term != 0;
  if (!term) tile_issue<NPH, W, EDGE>(win, e0, ndh, pw);
  tile_issue<NPL, W, EDGE>(snap + MS * args.stride, e0, ndl, pa);
  tile_issue<NPL, W, EDGE>(snap + (MS - 1) * args.stride, e0, ndl, pb);
  if (!term) tile_commit<NPH, W>(pw, lds);
  if constexpr (EDGE) {
    if (lane <= MS * 5) lds[CB + lane] = kbnd[lane];  // lane-indexed: from the kernarg segment
  }
  __syncthreads();
  double we[NE], wo[NO];
  if (!term) {
    const double* w = lds + pw.off + lane * NPH;
#pragma unroll
    for (int k = 0; k < NO; ++k) {
      we[k] = w[k] + w[NH - k];
      wo[k] = w[k] - w[NH - k];
    }
    if constexpr (NE > NO) we[NO] = w[NO];
  }
  const Elem E = elem_info<H, T, EDGE>(e0, lane, args.ktot, args.K);
  double sc = args.sc;
  if constexpr (!UNI) sc *= E.inrange ? scale[E.kl] : 0.0;
  __syncthreads();  // the w image is read
  tile_commit<NPL, W>(pa, lds);
  __syncthreads();
  double ne[NE], no[NO];  // P u^{n+1}
  prolong_eo<NPL>(lds + pa.off + lane * NPL, ps.get(), ne, no);
  if (term) terminal_from_prolong<NPH>(ne, no, we, wo);
  __syncthreads();
  tile_commit<NPL, W>(pb, lds);
  int off = pb.off;
  __syncthreads();
  double eacc = 0.0;
  double beta[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) beta[k] = args.beta[k];
  int parity = 0;
  double ve[NE], vo[NO], fe[NE], fo[NO], re[NE], ro[NO];

  // prologue: S(P u^{n0+MS-1}) alone, its residual paired with w^{n0+MS}
  prolong_eo<NPL>(lds + off + lane * NPL, ps.get(), ve, vo);
  if (MS > 1) tile_issue<NPL, W, EDGE>(snap + (MS - 2) * args.stride, e0, ndl, pa);
  pq_iteration<NPH, UNI, EDGE, true, false>(lds, G::kFB, parity, E, sc, os, beta,
                                            CB + (MS - 1) * 5, CB + MS * 5, ve, vo, fe, fo, we,
                                            wo, re, ro);
  if (args.has_eta) {
    double c = 0.0;
#pragma unroll
    for (int k = 0; k < NE; ++k) c = fma(we[k], ne[k] - fe[k], c);
#pragma unroll
    for (int k = 0; k < NO; ++k) c = fma(wo[k], no[k] - fo[k], c);
    eacc -= c;
  }
#pragma unroll
  for (int k = 0; k < NE; ++k) ne[k] = ve[k];
#pragma unroll
  for (int k = 0; k < NO; ++k) no[k] = vo[k];
  if (MS > 1) {
    tile_commit<NPL, W>(pa, lds);  // the prologue's prolongation read is 5 barriers behind
    off = pa.off;
    __syncthreads();
  }

  // iterations: S(P u^{n0+st-1}) beside w^{n0+st} = S^T w^{n0+st+1}, st = MS-1 .. 1
#pragma unroll 1
  for (int st = MS - 1; st >= 1; --st) {
    prolong_eo<NPL>(lds + off + lane * NPL, ps.get(), ve, vo);
    if (st >= 2) tile_issue<NPL, W, EDGE>(snap + (st - 2) * args.stride, e0, ndl, pa);
    pq_iteration<NPH, UNI, EDGE, true, true>(lds, G::kFB, parity, E, sc, os, beta,
                                             CB + (st - 1) * 5, CB + MS * 5, ve, vo, fe, fo, we,
                                             wo, re, ro);
    if (args.has_eta) {  // step n0+st-1's residual with w^{n0+st}, just produced
      double c = 0.0;
#pragma unroll
      for (int k = 0; k < NE; ++k) c = fma(we[k], ne[k] - fe[k], c);
#pragma unroll
      for (int k = 0; k < NO; ++k) c = fma(wo[k], no[k] - fo[k], c);
      eacc -= c;
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) ne[k] = ve[k];
#pragma unroll
    for (int k = 0; k < NO; ++k) no[k] = vo[k];
    if (st >= 2) {
      tile_commit<NPL, W>(pa, lds);
      off = pa.off;
      __syncthreads();
    }
  }
  // last: w^{n0} = S^T w^{n0+1}
  pq_iteration<NPH, UNI, EDGE, false, true>(lds, G::kFB, parity, E, sc, os, beta, CB, CB + MS * 5,
                                            ve, vo, fe, fo, we, wo, re, ro);

  if (args.has_eta && E.valid) eta_update(eta, E.e, eacc, args.has_eta);
  {
    const double(*pwe)[NE] = &we;
    const double(*pwo)[NO] = &wo;
    stage_out<NPH, W, H>(lds, pwe, pwo, true);  // the image's last reads are 5 barriers behind
  }
  __syncthreads();
  const int64_t o0 = tile * TE * NPH;
  if constexpr (EDGE) {
    const int64_t rem = ndh - o0;
    store_run<LB>(wout, o0, rem < int64_t(TE) * NPH ? rem : int64_t(TE) * NPH, lds);
  } else {
    store_full<TE * NPH, LB>(wout, o0, lds);
  }
}

}  // namespace dgk
