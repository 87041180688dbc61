// dg_sweep_ov.hip — the dataflow sweep (dg_sweep_kernel.h) on overlapped waves (dg_ovl_tiles.h), every Np.
#include "dg_sweep_kernel.h"

namespace {
// The overlapped-wave tiles (p->sweep_exchange = 1, dg_ovl_tiles.h): waves * 116 + 12 elements
// on 8, 12 or 16 waves.
template <int NP>
int sweep_np_x1(dg_plan* p, int waves, int msf, int msa, const dgk::SweepBufs& b, double t0,
                double dt, int nsteps, int mode, hipStream_t st) {
  if (p->sweep_lane_elems != 2)
    return fail(DG_ERR_ARG, "dataflow sweep: overlapped waves hold two elements per lane");
  if (waves == 8) return sweep_uni<NP, 8, 2, 1>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  if (waves == 12) return sweep_uni<NP, 12, 2, 1>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  if constexpr (NP <= 5)
    if (waves == 16) return sweep_uni<NP, 16, 2, 1>(p, msf, msa, b, t0, dt, nsteps, mode, st);
  return fail(DG_ERR_ARG, "dataflow sweep: overlapped waves on 8, 12 or 16 (Np <= 5) waves");
}
}  // namespace

namespace dgk {

int sweep_launch_ov(dg_plan* p, int waves, int msf, int msa, const SweepBufs& b,
                    double t0, double dt, int nsteps, int mode, hipStream_t st) {
  int rc = DG_OK;
  switch (p->NP) {
    case 2: rc = sweep_np_x1<2>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 3: rc = sweep_np_x1<3>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 4: rc = sweep_np_x1<4>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 5: rc = sweep_np_x1<5>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 6: rc = sweep_np_x1<6>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 7: rc = sweep_np_x1<7>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 8: rc = sweep_np_x1<8>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    case 9: rc = sweep_np_x1<9>(p, waves, msf, msa, b, t0, dt, nsteps, mode, st); break;
    default: return fail(DG_ERR_ARG, "unsupported Np");
  }
  return rc;
}

}  // namespace dgk
