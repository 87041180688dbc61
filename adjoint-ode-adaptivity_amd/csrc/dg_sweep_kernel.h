// dg_sweep_kernel.h — the jump-record sweep pair as ONE dataflow launch (dg_lserk4_sweep_rec):
// the kernel and its launch templates, instantiated by dg_sweep.hip (Np <= 5, per-level
// exchange), dg_sweep_hi.hip (Np >= 6) and dg_sweep_ov.hip (overlapped waves).
//
// The launch-per-block sweep (dg_lserk4_fwd_rec + dg_lserk4_adj_rec, dg_rec.hip) runs three
// launches per 20-step sweep at the default shape (forward 20, adjoint 10 + 10), and each
// launch pays a fill (the first round of workgroups loading their tiles with nothing to
// overlap) and a drain (the last round running partly empty: at K = 2^20 the forward's 1,279
// tiles are 1.66 rounds of the 768 resident workgroups).  Here the same tile bodies
// (dg_rec_tiles.h, policy WT = write-through hand-offs) are the work items of ONE launch:
//   items, in queue order: forward block 0 tiles 0..nTF-1, forward block 1 tiles, ...,
//   adjoint block 0 tiles 0..nTA-1 (reverse steps nsteps-MSA..nsteps-1), adjoint block 1, ...
//   The grid has one workgroup per item; each takes the next item from one counter when the
//   hardware starts it (not by blockIdx), so items start in queue order.  An item waits only
//   for items earlier in the queue -- the previous block's tiles whose output ranges its
//   input range (tile + halo) touches; the first adjoint block for the last forward block's
//   tiles covering its range (whose completion implies every earlier forward block's records
//   there) -- so the sweep cannot deadlock at any residency: the earliest waiting item's
//   producers were taken before it by workgroups that are running and wait on nothing later.
//   (A persistent grid looping over items measured 143 VGPRs: the compiler keeps both
//   bodies' constants live across the loop; one item per workgroup keeps the registers of
//   the separate kernels.)
// Hand-offs (cdna_hip_programming.md §6 Guideline 16, R1; MI355X_MICROARCH.md, visibility):
//   producer: every store of handed-off bytes (block states, the record, indicator partials)
//     is write-through (`sc1`); every wave drains (`s_waitcnt vmcnt(0)`), a workgroup barrier,
//     then one lane stores the item's flag (an agent-scope atomic store of the epoch);
//   consumer: wave 0 polls the producers' flags (relaxed agent loads, one lane per flag,
//     `s_sleep` between polls), a workgroup barrier, then EVERY load of handed-off bytes is
//     an `sc1` load (bypasses the CU's L1), so no acquire fence is needed;
//   no buffer is written twice in a launch (every block writes its own state buffer; the
//   adjoint's indicator partials have one row per block), so no cache line another
//   workgroup reads can change after it was read.
// Epochs: a 64-bit take counter that only grows numbers the launches (value / items) and the
// items (value % items); the flags hold the launch's epoch, so no memset precedes a launch
// of the same shape and HIP-graph replays work.  Every poll is bounded: a producer that never
// finishes (a bug) sets the error word after ~2^20 polls and every waiter gives up, so the
// launch always ends.  A work item that gave up writes NaN over what it publishes, so the
// indicator and the fused refine value turn non-finite; the error is also raised in mapped
// host memory, which makes the plan's next sweep call fail, and dg_sweep_status() reports
// and clears it.
// The results are bit-identical to the launch-per-block pair with the same steps per block
// (same tile arithmetic; the indicator's block partials are added in launch order).
#pragma once
#include "dg_ovl_tiles.h"
#include "dg_flow.h"

namespace {
using namespace dgk;
using namespace dgr;

template <int NP, int MSF> struct SweepArgs {
  RpOp<NP> c;
  double bnd[(kSweepMaxSteps / MSF) * (MSF * 6 + 1)];  // block b's rp_block_bnd at b*(6 MSF+1)
  double* U[kSweepMaxBlocks + 1];  // forward block b reads U[b] (U[0] = u0), writes U[b+1]
  double* W[kSweepMaxBlocks + 1];  // adjoint block a reads W[a] (terminal weight), writes W[a+1]
  double* rec;
  double* eta;
  double* part;                    // (nbA - 1) rows of ktot: the adjoint blocks' partial eta
  const double* scale;
  uint32_t* sync;                  // kSync* words, then one flag per item
  uint64_t* trace;                 // nullable: per item {dequeued, producers done, published,
                                   // XCC id << 32 | workgroup id} (wall clock, 100 MHz)
  int64_t* am_idx;                 // nullable: the fused refine decision, dg_argmax_ex(|eta|)
  double* am_val;
  int64_t* am_nf;
  double* am_pv;                   // per last-block tile: its (|eta|, element) winner
  int64_t* am_pi;
  uint32_t* err_host;              // nullable: mapped host word, raised with the error word
  int32_t nbF, nbA, nTF, nTA;
  int32_t nsteps;
  int32_t mode;                    // kEta* bits (0: no indicator)
  int32_t spin_limit;
};

// Occupancy target.  Both bodies live in one kernel, so its registers are the adjoint's
// (82-92 VGPRs at Np = 4, 5 unconstrained: 2 eight-wave workgroups per CU).  Capped at 80
// (6 waves per SIMD: 3 workgroups per CU, 3 x 41 KB of LDS) the allocator keeps every level
// loop of the uniform-mesh kernels spill-free at Np <= 5; the few spills it adds sit outside
// the loops (the edge tiles' prologue, the indicator's partial-row combine).  Np = 6 spills
// inside a loop at 80, and the non-uniform bodies (the metric per element) spill more: they
// keep the unconstrained count.  (Np 2, 3 fit 6 waves unconstrained.)
// At Np = 2 the bodies fit 8 waves per SIMD by VGPRs (57) but not by SGPRs: 99 SGPRs admit 6
// (MI355X_MICROARCH.md, residency: floor(800 / (ceil(sgpr/16)*16 + 16))).  Asked for 8, the
// compiler keeps 78 SGPRs and 58 VGPRs without spilling, and 4- or 8-wave workgroups then fill
// 32 wave slots per CU: N = 1 +4-6 % (6.09 / 6.17e11 against 5.88 / 5.79e11 for the 12-wave
// default, profiles/r04/wpe8/).  Np = 3 spills 28 B per lane at 8 and gains nothing.
template <int NP, bool UNI, int NW = 8, int X = 0> struct SweepOcc {
  static constexpr int waves_per_simd =
      (UNI && NP == 2 && (NW == 4 || NW == 8 || (X == 1 && NW == 16))) ? 8
      : (UNI && NP <= 5)                                               ? 6
                                                                       : 1;  // 1: none
};

// The tile geometry of an exchange mode X: 0 the pair tiles (a face exchange through LDS and a
// workgroup barrier per Horner level, dg_rec_tiles.h), 1 overlapped waves (DPP faces, one
// barrier per step, dg_ovl_tiles.h).
template <int NP, int NW, int E, int X>
using SwGeo = std::conditional_t<X == 1, OvGeo<NP, NW>, RpGeo<NP, NW, E>>;

template <int NP, bool UNI, int NW, int MSF, int MSA, int E, int X>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(
    E == 2 ? SweepOcc<NP, UNI, NW, X>::waves_per_simd : 1))) void k_sweep_rp(SweepArgs<NP, MSF> a) {
  static_assert(X == 0 || E == 2, "overlapped waves hold element pairs");
  static_assert(sizeof(SweepArgs<NP, MSF>) <= kKernargMax,
                "k_sweep_rp's arguments exceed the kernarg segment");
  using G = SwGeo<NP, NW, E, X>;
  constexpr int HF = RpHalo<MSF>::F, HA = RpHalo<MSA>::A;
  constexpr int TEF = G::T - 2 * HF, TEA = G::T - 2 * HA;
  __shared__ __attribute__((aligned(16))) double lds[G::kLds + MSF * 6 + 1];
  __shared__ uint32_t s_item, s_epoch, s_last, s_bad;
  __shared__ double s_av[NW];
  __shared__ int64_t s_ai[NW];
  uint32_t* sync = a.sync;
  uint32_t* flags = sync + kSyncFlags;
  const int tid = threadIdx.x;
  const int64_t ktot = a.c.ktot;
  const int nTF = a.nTF, nTA = a.nTA, nbF = a.nbF, nbA = a.nbA;
  const int64_t nF = int64_t(nbF) * nTF;
  const int64_t nItems = nF + int64_t(nbA) * nTA;
  if (tid == 0) {
    uint32_t it, ep;
    flow_take(sync, nItems, &it, &ep);  // items start in queue order (dg_flow.h)
    s_epoch = ep;
    s_item = it;
    s_bad = 0u;
  }
  __syncthreads();
  const int64_t item = s_item;
  const uint32_t epoch = s_epoch;
  const uint64_t t_deq = a.trace ? uint64_t(wall_clock64()) : 0;
  {
    // decode the item and the range of flags it waits for
    const bool fwd = item < nF;
    int blk, j;
    int64_t d0 = 0;
    int nd = 0;
    if (fwd) {
      blk = int(item / nTF);
      j = int(item - int64_t(blk) * nTF);
      if (blk > 0) {  // the previous block's tiles j-1..j+1 (halo < TEF)
        const int lo = j > 0 ? j - 1 : 0, hi = j + 1 < nTF ? j + 1 : nTF - 1;
        d0 = int64_t(blk - 1) * nTF + lo;
        nd = hi - lo + 1;
      }
    } else {
      const int64_t i2 = item - nF;
      blk = int(i2 / nTA);
      j = int(i2 - int64_t(blk) * nTA);
      if (blk == 0) {  // the last forward block's tiles covering the input + record range
        int64_t elo = int64_t(j) * TEA - HA, ehi = int64_t(j + 1) * TEA + HA;
        elo = elo > 0 ? elo : 0;
        ehi = ehi < ktot - 1 ? ehi : ktot - 1;
        const int lo = int(elo / TEF), hi = int(ehi / TEF);
        d0 = int64_t(nbF - 1) * nTF + lo;
        nd = hi - lo + 1;
      } else {
        const int lo = j > 0 ? j - 1 : 0, hi = j + 1 < nTA ? j + 1 : nTA - 1;
        d0 = nF + int64_t(blk - 1) * nTA + lo;
        nd = hi - lo + 1;
      }
    }
    if (tid < 64 && nd > 0) {
      const bool gave_up = sweep_wait(flags + d0, nd, epoch, sync, a.err_host, a.spin_limit);
      if (tid == 0 && gave_up) s_bad = 1u;
    }
    // no acquire fence: every load of handed-off bytes below is an sc1 load; this only keeps
    // the compiler from hoisting them above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    const uint64_t t_ready = a.trace ? uint64_t(wall_clock64()) : 0;
    using SA = SweepArgs<NP, MSF>;
    const DG_KAS char* ka = kernarg_tail_k<decltype(&k_sweep_rp<NP, UNI, NW, MSF, MSA, E, X>), SA>();
    const OpSrc<NP> os = op_src<NP>(a.c, ka + offsetof(SA, c));
    if (fwd) {
      const int64_t e0 = int64_t(j) * TEF - HF;
      const double* kb = reinterpret_cast<const double*>(
                             kernarg_tail<decltype(&k_sweep_rp<NP, UNI, NW, MSF, MSA, E, X>), SA>() +
                             offsetof(SA, bnd)) + blk * (MSF * 6 + 1);
      const int64_t n0 = int64_t(blk) * MSF;
      const bool jend = blk == a.nbF - 1;
      if constexpr (X == 1) {
        if (edge_tile(e0, G::T, ktot, a.c.K))
          ov_step_tile<NP, UNI, NW, MSF, true, true>(lds, j, a.U[blk], a.rec, a.U[blk + 1],
                                                     a.scale, a.c, os, kb, n0, jend);
        else
          ov_step_tile<NP, UNI, NW, MSF, false, true>(lds, j, a.U[blk], a.rec, a.U[blk + 1],
                                                      a.scale, a.c, os, kb, n0, jend);
      } else {
        if (edge_tile(e0, G::T, ktot, a.c.K))
          rp_step_tile<NP, UNI, NW, E, MSF, true, true>(lds, j, a.U[blk], a.rec, a.U[blk + 1],
                                                        a.scale, a.c, os, kb, n0, jend);
        else
          rp_step_tile<NP, UNI, NW, E, MSF, false, true>(lds, j, a.U[blk], a.rec, a.U[blk + 1],
                                                         a.scale, a.c, os, kb, n0, jend);
      }
      if (s_bad) {
        // the body's own write-through stores (another lane mapping) complete first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int64_t o0 = int64_t(j) * TEF * NP, nd = ktot * NP;
        poison_run<64 * NW>(a.U[blk + 1], o0, (nd - o0) < int64_t(TEF) * NP ? nd - o0
                                                                            : int64_t(TEF) * NP);
        // and the record rows it wrote from possibly unready inputs (rows n0-1 .. n0+MS-1 over
        // its output elements): an adjoint that reads them (a caller-supplied terminal weight
        // never reads U) turns its eta non-finite too
        const int64_t ee = int64_t(j) * TEF, ne = (ktot - ee) < TEF ? ktot - ee : int64_t(TEF);
        const int64_t n0 = int64_t(blk) * MSF, r0 = n0 >= 1 ? n0 - 1 : 0;
        const int64_t r1 = (blk == a.nbF - 1) ? n0 + MSF : n0 + MSF - 1;
        for (int64_t r = r0; r < r1; ++r) poison_run<64 * NW>(a.rec + r * rec_ld(ktot), ee, ne);
      }
    } else {
      const int64_t e0 = int64_t(j) * TEA - HA;
      const bool lastb = blk == a.nbA - 1;
      EtaSink es;
      es.eta = a.eta;
      es.part_out = (a.mode && !lastb) ? a.part + int64_t(blk) * ktot : nullptr;
      es.part_in = a.part;
      es.part_ld = ktot;
      es.nparts = lastb ? a.nbA - 1 : 0;
      es.mode = a.mode;
      es.argmax = lastb && a.am_idx != nullptr;
      es.bv = -INFINITY;  // the weakest candidate (dg_argmax's convention)
      es.bi = INT64_MAX;
      const int64_t n0 = int64_t(a.nsteps) - int64_t(blk + 1) * MSA;
      if constexpr (X == 1) {
        if (edge_tile(e0, G::T, ktot, a.c.K))
          ov_adj_tile<NP, UNI, NW, MSA, true, true>(lds, j, a.W[blk], a.W[blk + 1], a.rec, es,
                                                    a.scale, a.c, os, n0);
        else
          ov_adj_tile<NP, UNI, NW, MSA, false, true>(lds, j, a.W[blk], a.W[blk + 1], a.rec, es,
                                                     a.scale, a.c, os, n0);
      } else {
        if (edge_tile(e0, G::T, ktot, a.c.K))
          rp_adj_tile<NP, UNI, NW, E, MSA, true, true>(lds, j, a.W[blk], a.W[blk + 1], a.rec, es,
                                                       a.scale, a.c, os, n0);
        else
          rp_adj_tile<NP, UNI, NW, E, MSA, false, true>(lds, j, a.W[blk], a.W[blk + 1], a.rec,
                                                        es, a.scale, a.c, os, n0);
      }
      if (s_bad) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int64_t o0 = int64_t(j) * TEA, nd = ktot * NP;
        const int64_t ne = (ktot - o0) < TEA ? ktot - o0 : int64_t(TEA);
        poison_run<64 * NW>(a.W[blk + 1], o0 * NP, (nd - o0 * NP) < int64_t(TEA) * NP
                                                       ? nd - o0 * NP : int64_t(TEA) * NP);
        if (a.mode) poison_run<64 * NW>(es.part_out ? es.part_out : a.eta, o0, ne);
        es.bv = __builtin_nan("");
      }
      if (es.argmax) {  // the tile's winner, a hand-off to the last arriving tile
        wg_argmax<NW>(es.bv, es.bi, s_av, s_ai);
        if (tid == 0) {
          st8_agent(a.am_pv + j, __builtin_bit_cast(uint64_t, es.bv));
          st8_agent(a.am_pi + j, uint64_t(es.bi));
        }
      }
    }
    // publish: every wave's write-through stores have completed, then one flag store
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_agent(flags + item, epoch);
    if (!fwd && blk == nbA - 1 && a.am_idx != nullptr) {
      // Fused refine decision: the last block's tiles arrive on a counter; the one whose add
      // completes a launch's count reduces the nTA winners (published above, drained)
      flow_refine_arrive<NW>(sync, nTA, a.am_pv, a.am_pi, a.am_idx, a.am_val, a.am_nf, &s_last,
                             s_av, s_ai);
    }
    if (a.trace && tid == 0) {
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint64_t* tr = a.trace + 4 * item;
      tr[0] = t_deq;
      tr[1] = t_ready;
      tr[2] = uint64_t(wall_clock64());
      tr[3] = (uint64_t(xcc) << 32) | blockIdx.x;
    }
  }
}

static_assert(kSweepMaxBlocks + 1 == sizeof(SweepBufs::U) / sizeof(double*), "SweepBufs");

template <int NP, bool UNI, int NW, int MSF, int MSA, int E, int X>
int sweep_launch(dg_plan* p, const dgk::SweepBufs& b, double t0, double dt, int nsteps,
                 int mode, hipStream_t st) {
  SweepArgs<NP, MSF> a;
  if (const int rc = rp_make_op<NP>(p, dt, &a.c)) return rc;
  const int nbF = nsteps / MSF, nbA = nsteps / MSA;
  std::vector<double> tn(size_t(nsteps) + 1);  // time = time + dt (One_code.mlx:139)
  tn[0] = t0;
  for (int n = 0; n < nsteps; ++n) tn[n + 1] = tn[n] + dt;
  for (int bk = 0; bk < nbF; ++bk)
    rp_block_bnd(p, MSF, &tn[size_t(bk) * MSF], dt, a.bnd + bk * (MSF * 6 + 1));
  for (int i = 0; i <= kSweepMaxBlocks; ++i) {
    a.U[i] = b.U[i];
    a.W[i] = b.W[i];
  }
  a.rec = b.rec;
  a.eta = b.eta;
  a.part = b.part;
  a.scale = p->d_scale;
  a.sync = b.sync;
  a.trace = p->sweep_trace;
  a.am_idx = b.am_idx;
  a.am_val = b.am_val;
  a.am_nf = b.am_nf;
  a.am_pv = b.am_pv;
  a.am_pi = b.am_pi;
  a.nbF = nbF;
  a.nbA = nbA;
  using G = SwGeo<NP, NW, E, X>;
  a.nTF = int(grid_for(p->ktot, G::T - 2 * RpHalo<MSF>::F));
  a.nTA = int(grid_for(p->ktot, G::T - 2 * RpHalo<MSA>::A));
  a.nsteps = nsteps;
  a.mode = mode;
  a.err_host = b.err_host;
  a.spin_limit = b.spin_limit > 0 ? b.spin_limit : kSweepSpinLimit;
  const int64_t items = int64_t(nbF) * a.nTF + int64_t(nbA) * a.nTA;
  hipLaunchKernelGGL((k_sweep_rp<NP, UNI, NW, MSF, MSA, E, X>), dim3(unsigned(items)), dim3(64 * NW), 0,
                     st, a);
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

template <int NP, bool UNI, int NW, int E, int X>
int sweep_shape_launch(dg_plan* p, int msf, int msa, const dgk::SweepBufs& b, double t0,
                       double dt, int nsteps, int mode, hipStream_t st) {
  if constexpr (NW > 8 || X == 1) {
    // the wide tiles and the overlapped waves: 20- or 10-step forward, 10-step adjoint blocks
    if (msa == 10 && msf == 20) return sweep_launch<NP, UNI, NW, 20, 10, E, X>(p, b, t0, dt, nsteps, mode, st);
    if (msa == 10 && msf == 10) return sweep_launch<NP, UNI, NW, 10, 10, E, X>(p, b, t0, dt, nsteps, mode, st);
    return fail(DG_ERR_ARG, "dataflow sweep: 12 or 16 waves, or overlapped waves, take 10- or "
                            "20-step forward and 10-step adjoint blocks");
  } else {
    if (msa == 10) {
      if constexpr (NW * E >= 16)  // 20-step forward blocks need 1024-element tiles
        if (msf == 20) return sweep_launch<NP, UNI, NW, 20, 10, E, 0>(p, b, t0, dt, nsteps, mode, st);
      if (msf == 10) return sweep_launch<NP, UNI, NW, 10, 10, E, 0>(p, b, t0, dt, nsteps, mode, st);
      if (msf == 5) return sweep_launch<NP, UNI, NW, 5, 10, E, 0>(p, b, t0, dt, nsteps, mode, st);
    } else if (msa == 5) {
      if constexpr (NW * E >= 16)
        if (msf == 20) return sweep_launch<NP, UNI, NW, 20, 5, E, 0>(p, b, t0, dt, nsteps, mode, st);
      if (msf == 10) return sweep_launch<NP, UNI, NW, 10, 5, E, 0>(p, b, t0, dt, nsteps, mode, st);
      if (msf == 5) return sweep_launch<NP, UNI, NW, 5, 5, E, 0>(p, b, t0, dt, nsteps, mode, st);
    }
    return fail(DG_ERR_ARG, "dataflow sweep: unsupported steps per block for this tile width");
  }
}

template <int NP, int NW, int E = 2, int X = 0>
int sweep_uni(dg_plan* p, int msf, int msa, const dgk::SweepBufs& b, double t0, double dt,
              int nsteps, int mode, hipStream_t st) {
  return p->uniform
             ? sweep_shape_launch<NP, true, NW, E, X>(p, msf, msa, b, t0, dt, nsteps, mode, st)
             : sweep_shape_launch<NP, false, NW, E, X>(p, msf, msa, b, t0, dt, nsteps, mode, st);
}

}  // namespace
