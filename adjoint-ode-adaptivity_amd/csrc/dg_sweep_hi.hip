// dg_sweep_hi.hip — the dataflow sweep (dg_sweep_kernel.h) at Np = 6..9, per-level exchange.
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

int sweep_launch_hi(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b,
                    double t0, double dt, int nsteps, int mode, hipStream_t st) {
  int rc = DG_OK;
  switch (p->NP) {
    case 6: rc = sweep_np_x0<6>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 7: rc = sweep_np_x0<7>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 8: rc = sweep_np_x0<8>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 9: rc = sweep_np_x0<9>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    default: return fail(DG_ERR_ARG, "unsupported Np");
  }
  return rc;
}

}  // namespace dgk
