// dg_step_tile.h — the stage-loop forward tile (k_step's body, dg_advec.hip) and the sc1
// tile load, shared by dg_advec.hip (k_step) and dg_dwr.hip (k_psweep: the p-estimate's
// forward and adjoint as one dataflow launch).  Internal to libdgadv.so.
#pragma once
#include "dg_rec_tiles.h"

namespace dgk {

// The jump record (dg_lserk4_fwd_rec / dg_lserk4_adj_rec; layout in dg_common.h rec_ld): per
// element and step the left-face jump j_e = u_0 - uL -- 8 bytes where a snapshot takes 8 Np --
// computed from the face values stage 0 exchanges anyway; the adjoint rebuilds
// du0 - du1 = j_e + j_{e+1} and du0 + du1 = j_e - j_{e+1} (du1 = 0 at a trajectory's last
// element), the snapshot path's doubles, so eta is bit-identical to the snapshot sweep's.
__device__ __forceinline__ double* jump_row(double* rec, int64_t n, int64_t ktot) {
  return rec + n * rec_ld(ktot);
}

// tile_issue with sc1 loads (dg_rec_tiles.h tile_load's WT policy): the input of a work item
// of a dataflow launch, written write-through by an earlier item of the same launch.
template <int NP, int W, bool EDGE>
__device__ __forceinline__ void tile_issue_wt(const double* __restrict__ g, int64_t e0,
                                              int64_t nd, TileRegs<NP, W>& r) {
  using G = TileGeo<NP, W>;
  const int64_t d0 = e0 * NP;
  const int64_t base = d0 & ~int64_t(1);
  r.off = int(d0 - base);
  const int nvec = (G::T * NP + r.off + 1) >> 1;
  const int64_t bc = base > 0 ? base : 0;  // (base < 0 only in edge tiles: those lanes load nothing)
  const __amdgpu_buffer_rsrc_t rs = dgr::wt_rsrc(g + bc);
#pragma unroll
  for (int q = 0; q < G::kVec; ++q) {
    const int v = threadIdx.x + q * G::LB;
    const int64_t gd = base + 2 * int64_t(v);
    double2 val = make_double2(0.0, 0.0);
    if (v < nvec) {
      if (!EDGE || (gd >= 0 && gd + 1 < nd)) {
        val = dgr::wt_ld16(rs, uint32_t(gd - bc) * 8u);
      } else {
        if (gd >= 0 && gd < nd) val.x = dgr::wt_ld8(rs, uint32_t(gd - bc) * 8u);
        if (gd + 1 >= 0 && gd + 1 < nd) val.y = dgr::wt_ld8(rs, uint32_t(gd + 1 - bc) * 8u);
      }
    }
    r.v[q] = val;
  }
}

// ---------------------------------------------------------------------------
// Forward fused kernel: MS time steps of NS stages (AdvecRHS1D + the low-storage update)
// for the EPL elements of each lane.  After each step st the interior elements go to
// snap + st*stride (if snap) and after the last step also to `last` (if non-null).
// UNI: the operator constants already carry dt*2/h.
// ---------------------------------------------------------------------------
// kin: the MS*NS+1 inflow values (edge tiles read them lane-indexed).  WT: a work item of a
// dataflow launch (dg_dwr.hip k_psweep): the input is loaded sc1 and the snapshots are stored
// write-through.  SA: the argument struct (op, sc, ktot, K, stride, n0, jend).
template <int NP, int NS, bool UNI, int W, int MS, bool REC, bool EDGE, bool WT = false,
          class SA = StepArgs<NP, NS, MS>>
__device__ __forceinline__ void step_tile(double* __restrict__ lds, int64_t tile,
                                          const double* __restrict__ uin,
                                          double* __restrict__ snap, double* __restrict__ last,
                                          const double* __restrict__ scale, const SA& args,
                                          const double* __restrict__ kin) {
  using G = TileGeo<NP, W>;
  constexpr int T = G::T, LB = G::LB, EPL = 1;
  // dependency cone: one element per stage (+1 with the jump record: the final state's
  // jumps need the output elements' neighbours after the last stage)
  constexpr int H = MS * NS + (REC ? 1 : 0);
  constexpr int TE = T - 2 * H;  // output elements per tile (even)
  static_assert(TE % 2 == 0 && TE > 0, "tile output must be 16-byte aligned");
  constexpr int NE = EOArgs<NP>::NE, NO = EOArgs<NP>::NO;
  const int lane = threadIdx.x;
  const int64_t e0 = tile * TE - H;
  const int64_t nd = args.ktot * NP;
  const int64_t o0 = tile * TE * NP;
  const int64_t rem = nd - o0;
  const int64_t count = rem < int64_t(TE) * NP ? rem : int64_t(TE) * NP;

  constexpr int CB = G::kLds;  // lds[CB + st*NS + s] = inflow value of that stage
  TileRegs<NP, W> pf;
  if constexpr (WT) tile_issue_wt<NP, W, EDGE>(uin, e0, nd, pf);
  else tile_issue<NP, W, EDGE>(uin, e0, nd, pf);
  tile_commit<NP, W>(pf, lds);
  if constexpr (EDGE) {
    if (lane <= MS * NS) lds[CB + lane] = kin[lane];
  }
  __syncthreads();
  double ev[EPL][NE], od[EPL][NO];  // the element state in even/odd coordinates
  Elem E[EPL];
  double sc[EPL];
#pragma unroll
  for (int m = 0; m < EPL; ++m) {
    const int el = m * LB + lane;
    to_eo<NP>(lds + pf.off + el * NP, ev[m], od[m]);
    E[m] = elem_info<H, T, EDGE>(e0, el, args.ktot, args.K);
    sc[m] = args.sc;
    if constexpr (!UNI) sc[m] *= E[m].inrange ? scale[E[m].kl] : 0.0;
    if constexpr (REC) {
      // The launch's input state u^{n0} (record n0-1) from its nodal values in the staged
      // image -- the values a snapshot holds; the even/odd round trip ev_0 + od_0 can differ
      // from them in the last bit.  Inflow at t_{n0} = the first stage's, own node at the end.
      if (args.n0 >= 1 && E[m].valid) {
        const double* us = lds + pf.off + el * NP;
        const double uL = (EDGE && E[m].first) ? lds[CB] : us[-1];
        jump_row(snap, args.n0 - 1, args.ktot)[E[m].e] = us[0] - uL;
      }
    }
  }

  double re[EPL][NE], ro[EPL][NO];
#pragma unroll
  for (int st = 0; st < MS; ++st) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // Face buffers alternate over the global stage index: consecutive stages (also across
      // steps, where no barrier separates the last stage's reads from the next writes)
      // never share one.
      const int fL = G::kFB + ((st * NS + s) & 1) * 2 * (T + 2);  // faceL = lds[fL ...]
      const int fR = fL + (T + 2);  // faceR = lds[fR ...]
      double u0[EPL], uN[EPL];
      double pe[EPL][NE], po[EPL][NO];
#pragma unroll
      for (int m = 0; m < EPL; ++m) {
        const int el = m * LB + lane;
        u0[m] = ev[m][0] + od[m][0];
        uN[m] = ev[m][0] - od[m][0];
        lds[fL + el + 1] = u0[m];
        lds[fR + el + 1] = uN[m];
        __builtin_amdgcn_sched_barrier(0);  // face writes first, then hide their latency:
        // Everything that does not need the neighbours' faces is issued before the barrier
        // (s_barrier is a scheduling boundary): the volume term and, on uniform meshes,
        // the low-storage carry A_s*r.  Only the lift term and the update follow it.
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          double t = (UNI && s > 0) ? RK<NS>::A(s) * re[m][k] : args.op.Qeo[k * NO] * od[m][0];
#pragma unroll
          for (int j = (UNI && s > 0) ? 0 : 1; j < NO; ++j)
            t = fma(args.op.Qeo[k * NO + j], od[m][j], t);
          pe[m][k] = t;
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          double t = (UNI && s > 0) ? RK<NS>::A(s) * ro[m][k] : args.op.Qoe[k * NE] * ev[m][0];
#pragma unroll
          for (int j = (UNI && s > 0) ? 0 : 1; j < NE; ++j)
            t = fma(args.op.Qoe[k * NE + j], ev[m][j], t);
          po[m][k] = t;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) pin(pe[m][k]);
#pragma unroll
        for (int k = 0; k < NO; ++k) pin(po[m][k]);
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < EPL; ++m) {
        const int el = m * LB + lane;
        // faceR[el] is element el-1's right node, faceL[el+2] element el+1's left node; the
        // pad entries are only read by the outermost halo elements, whose results are dropped.
        // Interior tiles: neighbours' faces.  Edge tiles: the first element of a
        // trajectory reads the inflow value, the last one its own right face (du1 = 0).
        const int iL = EDGE && E[m].first ? CB + st * NS + s : fR + el;
        const int iR = EDGE && E[m].last ? fR + el + 1 : fL + el + 2;
        // The own faces' lift parts sit in the folded volume blocks (make_eo, fold):
        // only uR - uL and uL + uR remain.
        const double uL = lds[iL], uR = lds[iR];
        const double dlt = uR - uL, sig = -(uL + uR);
        if constexpr (REC) {  // u^{n0+st}'s jumps (record n0+st-1), stage 0 of its step
          if (s == 0 && st >= 1 && E[m].valid)
            jump_row(snap, args.n0 + st - 1, args.ktot)[E[m].e] = u0[m] - uL;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) {
          if constexpr (UNI) {  // r = A_s r + dt*L u, dt*2/h folded into the operator
            re[m][k] = fma(args.op.le[k], dlt, pe[m][k]);
          } else {
            const double a = sc[m] * fma(args.op.le[k], dlt, pe[m][k]);
            re[m][k] = (s == 0) ? a : fma(RK<NS>::A(s), re[m][k], a);  // rk4a(1) = 0
          }
          ev[m][k] = fma(RK<NS>::B(s), re[m][k], ev[m][k]);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) {
          if constexpr (UNI) {
            ro[m][k] = fma(args.op.lo[k], sig, po[m][k]);
          } else {
            const double a = sc[m] * fma(args.op.lo[k], sig, po[m][k]);
            ro[m][k] = (s == 0) ? a : fma(RK<NS>::A(s), ro[m][k], a);
          }
          od[m][k] = fma(RK<NS>::B(s), ro[m][k], od[m][k]);
        }
      }
    }
    if (REC && st == MS - 1 && args.jend) {
      // The sweep's final state u^{n0+MS}: one more face exchange (the buffer parity of the
      // stage after the last) for its jumps, record n0+MS-1; inflow at t_{n0+MS}.
      const int fL = G::kFB + ((MS * NS) & 1) * 2 * (T + 2), fR = fL + (T + 2);
      const int el = lane;
      const double u0 = ev[0][0] + od[0][0], uN = ev[0][0] - od[0][0];
      lds[fL + el + 1] = u0;
      lds[fR + el + 1] = uN;
      __syncthreads();
      const int iL = EDGE && E[0].first ? CB + MS * NS : fR + el;
      if (E[0].valid) jump_row(snap, args.n0 + MS - 1, args.ktot)[E[0].e] = u0 - lds[iL];
    }
    if ((!REC && snap != nullptr) || st == MS - 1) {
      // The image's last readers (staging reads, the previous step's store) are at least
      // one stage barrier behind; the faces live elsewhere.
      stage_out<NP, W, H>(lds, ev, od, false);
      __syncthreads();
      if constexpr (WT) {  // (dataflow items: snapshots only)
        if constexpr (EDGE) dgr::store_run_wt<LB>(snap + st * args.stride, o0, count, lds);
        else dgr::store_full_wt<TE * NP, LB>(snap + st * args.stride, o0, lds);
      } else if constexpr (EDGE) {
        if (!REC && snap != nullptr) store_run<LB>(snap + st * args.stride, o0, count, lds);
        if (st == MS - 1 && last != nullptr) store_run<LB>(last, o0, count, lds);
      } else {
        if (!REC && snap != nullptr) store_full<TE * NP, LB>(snap + st * args.stride, o0, lds);
        if (st == MS - 1 && last != nullptr) store_full<TE * NP, LB>(last, o0, lds);
      }
    }
  }
}

}  // namespace dgk
