// dg_fd.hip — the finite-difference DWR adapt step of python/Main_finite_difference.py for
// ensembles of du/dt = sin(u) with J = int u^2: forward Euler on the coarse
// grid (forwardSolve, :34-51), the discrete adjoint on the ref_factor-refined grid
// (adjSolve, :54-76: (J_F^T - I) v = -K is upper bidiagonal with -1 on the diagonal, so its
// solve is the backward recursion v_n = K_n + (1 + cos(u_n) dt_n) v_{n+1}), the
// adjoint-weighted residual (errEst, :79-94) and the windowed per-step sums (:270-277).
// One lane per ensemble member; the fine-grid solution is the np.interp of the coarse one
// (:24-31), evaluated on the fly with numpy's arithmetic (host-computed interval codes,
// no FMA contraction) instead of being stored.
// Layouts: U[n*n_ics + ic] (coarse nodes), V[n*n_ics + ic] (fine nodes, optional),
// err_steps[ic*n_steps + r] (steps contiguous per member, for dg_sum_rows).
#include "dg_common.h"

namespace {
using namespace dgk;

constexpr int kFdBlock = 256;
constexpr int kMaxRf = 16;  // ref_factor bound (one kernel per value, window in registers)

// np.interp(t_fine[i], t_coarse, u) with numpy's case split (numpy/core/src/multiarray/
// compiled_base.c arr_interp): code >= 0 -> slope*(x - xp[j]) + fp[j] in interval j,
// code < 0 -> the coarse node -(code+1) exactly.
__device__ __forceinline__ double fine_u(int32_t code, double x, const double* __restrict__ tc,
                                         const double* __restrict__ U, int64_t n_ics,
                                         int64_t ic) {
  if (code < 0) return U[int64_t(-(code + 1)) * n_ics + ic];
  const double u0 = U[int64_t(code) * n_ics + ic], u1 = U[int64_t(code + 1) * n_ics + ic];
  const double slope = __ddiv_rn(__dsub_rn(u1, u0), __dsub_rn(tc[code + 1], tc[code]));
  return __dadd_rn(__dmul_rn(slope, __dsub_rn(x, tc[code])), u0);
}

// np.sum(err_steps, 1) over one window (Main_finite_difference.py:276): on that strided
// 2-D view numpy reduces the last axis sequentially from the window's first element
// (checked against numpy 2.2 with values whose sum depends on the order), so the window
// is summed in ascending fine-step order.
template <int W>
__device__ __forceinline__ double numpy_window_sum(const double* a) {
  double acc = a[0];
#pragma unroll
  for (int i = 1; i < W; ++i) acc = __dadd_rn(acc, a[i]);
  return acc;
}

template <int RF>
__global__ __launch_bounds__(kFdBlock) void k_fd_sweep(
    int n_steps, const double* __restrict__ dt_n, const double* __restrict__ tc,
    const double* __restrict__ tf, const int32_t* __restrict__ code, const double* __restrict__ u0,
    int64_t n_ics, double* __restrict__ U, double* __restrict__ V,
    double* __restrict__ err_steps) {
  const int64_t ic = int64_t(blockIdx.x) * kFdBlock + threadIdx.x;
  if (ic >= n_ics) return;
  // forwardSolve: u_n = u_{n-1} + sin(u_{n-1}) dt_{n-1} (Main_finite_difference.py:131-132)
  double u = u0[ic];
  U[ic] = u;
  for (int n = 1; n <= n_steps; ++n) {
    u = __dadd_rn(u, __dmul_rn(sin(u), dt_n[n - 1]));
    U[int64_t(n) * n_ics + ic] = u;
  }
  // Backward over the fine grid: v_Nf = K_Nf = v0 = 0 (getK of J = int u^2, :225-227);
  // v_n = 2 u_n dt_n + (1 + cos(u_n) dt_n) v_{n+1};  err_n = (u_n - u_{n-1} - sin(u_{n-1}) dt_{n-1}) v_n
  // Coarse step m's window (fine steps n = m RF + 2 .. (m+1) RF, :270-277) is kept in
  // registers and summed once it is complete, in numpy's order, then stored once.
  const int nf = n_steps * RF;
  double v = 0.0;
  double un = fine_u(code[nf], tf[nf], tc, U, n_ics, ic);
  if (V) V[int64_t(nf) * n_ics + ic] = v;
  double* __restrict__ erow = err_steps + ic * n_steps;
  for (int m = n_steps - 1; m >= 0; --m) {
    const double dtp = dt_n[m] / double(RF);  // dt_fine of coarse step m (refineAll, :16-21)
    double term[RF];
#pragma unroll
    for (int p = RF - 1; p >= 0; --p) {
      const int n = m * RF + 1 + p;  // fine step n: nodes n-1 -> n
      const double up = fine_u(code[n - 1], tf[n - 1], tc, U, n_ics, ic);
      double su, cu;
      sincos(up, &su, &cu);
      // residual of fine step n (errEst, :88-90) times v_n; |err|[2:] drops the first fine
      // step of each coarse step (p = 0)
      const double res = __dsub_rn(un, __dadd_rn(up, __dmul_rn(su, dtp)));
      term[p] = fabs(__dmul_rn(res, v));
      // adjoint recursion to node n-1
      v = __dadd_rn(__dmul_rn(2.0 * up, dtp), __dmul_rn(__dadd_rn(1.0, __dmul_rn(cu, dtp)), v));
      if (V) V[int64_t(n - 1) * n_ics + ic] = v;
      un = up;
    }
    erow[m] = numpy_window_sum<RF - 1>(term + 1);
  }
}

}  // namespace

extern "C" {

int dg_fd_adapt_sweep(int n_steps, int ref_factor, const double* dt_n, const double* t_coarse,
                      const double* t_fine, const int32_t* interp_code, const double* u0,
                      int64_t n_ics, double* U, double* V, double* err_steps, void* stream) {
  if (!dt_n || !t_coarse || !t_fine || !interp_code || !u0 || !U || !err_steps)
    return fail(DG_ERR_ARG, "null argument");
  if (n_steps < 1 || ref_factor < 2 || n_ics < 1) return fail(DG_ERR_ARG, "bad sizes");
  if (ref_factor > kMaxRf) return fail(DG_ERR_ARG, "ref_factor > 16 is not supported");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(grid_for(n_ics, kFdBlock));
  switch (ref_factor) {
#define DG_FD_CASE(R)                                                                          \
  case R:                                                                                      \
    hipLaunchKernelGGL(k_fd_sweep<R>, grid, dim3(kFdBlock), 0, st, n_steps, dt_n, t_coarse,    \
                       t_fine, interp_code, u0, n_ics, U, V, err_steps);                       \
    break;
    DG_FD_CASE(2) DG_FD_CASE(3) DG_FD_CASE(4) DG_FD_CASE(5) DG_FD_CASE(6) DG_FD_CASE(7)
    DG_FD_CASE(8) DG_FD_CASE(9) DG_FD_CASE(10) DG_FD_CASE(11) DG_FD_CASE(12) DG_FD_CASE(13)
    DG_FD_CASE(14) DG_FD_CASE(15) DG_FD_CASE(16)
#undef DG_FD_CASE
  }
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

}  // extern "C"
