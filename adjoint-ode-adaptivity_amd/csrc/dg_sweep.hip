// dg_sweep.hip — the dataflow sweep (dg_sweep_kernel.h) at Np = 2..5, per-level exchange; the host
// helpers and the dispatch over the three translation units.
#include "dg_sweep_kernel.h"

namespace {
// Tiles of 128 * waves elements on workgroups of `waves` waves: 8 (1024 elements, the
// default) or 4 (512: tile width 1).  Workgroups of 5, 6 and 10 waves (which fill the 20 wave
// slots per CU the 88-VGPR bodies leave, where 8-wave groups use 16) measured 17-27 % slower
// at N = 4, K = 2^20 (profiles/r03/waves2/: more items and their per-item latency, or a
// barrier over 10 waves) and were dropped.  With the overlapped waves (p->sweep_exchange = 1,
// dg_ovl_tiles.h) tiles of waves * 116 + 12 elements on 8, 12 or 16 waves.
template <int NP>
int sweep_np_x0(dg_plan* p, int waves, int msf, int msa, const dgk::SweepBufs& b, double t0,
             double dt, int nsteps, int mode, hipStream_t st) {
  if constexpr (NP <= 3) {  // four elements per lane (DG_TUNE_SWEEP_LANE_ELEMENTS)
    if (p->sweep_lane_elems == 4) {
      if (waves == 8) return sweep_uni<NP, 8, 4>(p, msf, msa, b, t0, dt, nsteps, mode, st);
      if (waves == 4) return sweep_uni<NP, 4, 4>(p, msf, msa, b, t0, dt, nsteps, mode, st);
      return fail(DG_ERR_ARG, "dataflow sweep: four elements per lane on 4 or 8 waves");
    }
  }
  if (waves == 8) return sweep_uni<NP, 8>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  if (waves == 4) return sweep_uni<NP, 4>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  if (waves == 12) return sweep_uni<NP, 12>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  if constexpr (NP <= 5)  // 2048 * Np doubles of LDS; larger Np would not fit 4 waves per SIMD
    if (waves == 16) return sweep_uni<NP, 16>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  return fail(DG_ERR_ARG, "dataflow sweep: workgroups of 4, 8, 12 or 16 (Np <= 5) waves");
}

}  // namespace

namespace dgk {

int sweep_launch_lo(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b,
                    double t0, double dt, int nsteps, int mode, hipStream_t st) {
  int rc = DG_OK;
  switch (p->NP) {
    case 2: rc = sweep_np_x0<2>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 3: rc = sweep_np_x0<3>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 4: rc = sweep_np_x0<4>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 5: rc = sweep_np_x0<5>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    default: return fail(DG_ERR_ARG, "unsupported Np");
  }
  return rc;
}


int sweep_launch_lo(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b, double t0,
                    double dt, int nsteps, int mode, hipStream_t st);
int sweep_launch_hi(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b, double t0,
                    double dt, int nsteps, int mode, hipStream_t st);
int sweep_launch_ov(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b, double t0,
                    double dt, int nsteps, int mode, hipStream_t st);


int sweep_tile_elems(const dg_plan* p, int waves) {
  return p->sweep_exchange == 1 ? waves * kOvS + 2 * kOvG : 64 * p->sweep_lane_elems * waves;
}

int sweep_waves_per_simd(const dg_plan* p, int waves) {
  const int E = p->sweep_lane_elems, X = p->sweep_exchange;
  if (E != 2) return 0;
  int w = 0;
  // SweepOcc<NP, UNI, NW, X>::waves_per_simd, evaluated on the host (1 there means none)
  auto occ = [&](auto np_tag) {
    constexpr int NP = decltype(np_tag)::value;
    auto pick = [&](auto uni_tag) {
      constexpr bool UNI = decltype(uni_tag)::value;
      switch (waves) {
        case 4: return X ? 0 : SweepOcc<NP, UNI, 4, 0>::waves_per_simd;
        case 8: return X ? SweepOcc<NP, UNI, 8, 1>::waves_per_simd : SweepOcc<NP, UNI, 8, 0>::waves_per_simd;
        case 12: return X ? SweepOcc<NP, UNI, 12, 1>::waves_per_simd : SweepOcc<NP, UNI, 12, 0>::waves_per_simd;
        case 16: return X ? SweepOcc<NP, UNI, 16, 1>::waves_per_simd : SweepOcc<NP, UNI, 16, 0>::waves_per_simd;
        default: return 0;
      }
    };
    w = p->uniform ? pick(std::true_type{}) : pick(std::false_type{});
  };
  switch (p->NP) {
    case 2: occ(std::integral_constant<int, 2>{}); break;
    case 3: occ(std::integral_constant<int, 3>{}); break;
    case 4: occ(std::integral_constant<int, 4>{}); break;
    case 5: occ(std::integral_constant<int, 5>{}); break;
    case 6: occ(std::integral_constant<int, 6>{}); break;
    case 7: occ(std::integral_constant<int, 7>{}); break;
    case 8: occ(std::integral_constant<int, 8>{}); break;
    case 9: occ(std::integral_constant<int, 9>{}); break;
    default: break;
  }
  return w == 1 ? 0 : w;
}

int64_t sweep_items(const dg_plan* p, int waves, int msf, int msa, int nsteps, int64_t elems) {
  const int64_t n = elems >= 0 ? elems : p->ktot;
  const int T = sweep_tile_elems(p, waves);
  const int64_t nTF = grid_for(n, T - 2 * ((msf * 5 + 2) & ~1));
  const int64_t nTA = grid_for(n, T - 2 * ((msa * 5 + 1) & ~1));
  return int64_t(nsteps / msf) * nTF + int64_t(nsteps / msa) * nTA;
}

int64_t sweep_tiles_adj(const dg_plan* p, int waves, int msa, int64_t elems) {
  const int64_t n = elems >= 0 ? elems : p->ktot;
  return grid_for(n, sweep_tile_elems(p, waves) - 2 * ((msa * 5 + 1) & ~1));
}

int sweep_launch_rec(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b, double t0,
                     double dt, int nsteps, int mode, hipStream_t st) {
  if (p->sweep_exchange == 1) return sweep_launch_ov(p, waves, msf, msa, b, t0, dt, nsteps, mode, st);
  if (p->NP <= 5) return sweep_launch_lo(p, waves, msf, msa, b, t0, dt, nsteps, mode, st);
  return sweep_launch_hi(p, waves, msf, msa, b, t0, dt, nsteps, mode, st);
}

int sweep_sync_words() { return kSyncFlags; }
int sweep_max_steps() { return kSweepMaxSteps; }
int sweep_err_word() { return kSyncErr; }

}  // namespace dgk
