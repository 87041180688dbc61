// dg_time.hip — batched DG-in-time marches for ensembles of the scalar ODE du/dt = sin(u):
// matlab/dg_march.m (forward, nonlinear branch), matlab/adj_march.m (adjoint + DWR
// indicator, nonlinear branch) with the operators of matlab/fem_setup.m, as driven by
// matlab/MAIN.m.  CPU statement: oracle/dgtime.py.
//
// One lane per initial condition.  Slabs are marched in order inside the lane (the
// recursion is sequential in time); every slab is a Newton iteration on
//   R(U) = (S^T + B) U + hk/2 Phi^T (w .* sin(Phi U)) + e_1 uR_prev        (dg_march.m:47-64)
// with an Np x Np partial-pivoting LU solve in registers, or, backwards, one linear solve
// for the adjoint and the dual-weighted residual err(k) = v_k^T R_k(u_h)  (adj_march.m:98-117).
// The reference-element operators (Gauss points and weights, Phi, stiffness, mass) are
// the same for every slab and lane; they are staged in LDS once per workgroup.
// Layouts (device arrays): Y[(k*Np + i)*n_ics + ic] (ICs contiguous: coalesced per node),
// iters[k*n_ics + ic], err[ic*n_slabs + k] (slabs contiguous per IC, for dg_sum_rows).
#include "dg_common.h"

namespace {
using namespace dgk;

constexpr int kTimeBlock = 128;

// Solve A x = b in place (x returned in b): Gaussian elimination with partial pivoting,
// first maximal row on ties (LAPACK dgesv, MATLAB mldivide).  Row swaps are selects, so
// the unrolled arrays stay in registers.
template <int NP>
__device__ __forceinline__ void lu_solve(double (&A)[NP][NP], double (&b)[NP]) {
#pragma unroll
  for (int c = 0; c < NP; ++c) {
    int p = c;
    double m = fabs(A[c][c]);
#pragma unroll
    for (int r = c + 1; r < NP; ++r) {
      const double a = fabs(A[r][c]);
      if (a > m) {
        m = a;
        p = r;
      }
    }
#pragma unroll
    for (int r = c + 1; r < NP; ++r) {
      const bool sw = (r == p);
#pragma unroll
      for (int j = c; j < NP; ++j) {
        const double t = A[c][j];
        A[c][j] = sw ? A[r][j] : t;
        A[r][j] = sw ? t : A[r][j];
      }
      const double t = b[c];
      b[c] = sw ? b[r] : t;
      b[r] = sw ? t : b[r];
    }
    const double inv = 1.0 / A[c][c];
#pragma unroll
    for (int r = c + 1; r < NP; ++r) {
      const double f = A[r][c] * inv;
#pragma unroll
      for (int j = c + 1; j < NP; ++j) A[r][j] = fma(-f, A[c][j], A[r][j]);
      b[r] = fma(-f, b[c], b[r]);
    }
  }
#pragma unroll
  for (int c = NP - 1; c >= 0; --c) {
    double x = b[c];
#pragma unroll
    for (int j = c + 1; j < NP; ++j) x = fma(-A[c][j], b[j], x);
    b[c] = x / A[c][c];
  }
}

// x(end) - x(1) of fem_setup on [ta, tb]: x = VX(1) + (r+1)/2 (VX(2) - VX(1)) (StartUp1D.m:21)
__device__ __forceinline__ double slab_width(double ta, double tb) { return (ta + (tb - ta)) - ta; }

// Forward march, order NP-1.  LDS: S[NP*NP] (row-major S = (V V')\Dr), Phi[nq*NP], w[nq].
template <int NP>
__global__ __launch_bounds__(kTimeBlock) void k_dgt_march(
    const double* __restrict__ S, const double* __restrict__ Phi, const double* __restrict__ wq,
    int nq, const double* __restrict__ times, int n_slabs, const double* __restrict__ y0,
    int64_t n_ics, double tol, int maxit, double* __restrict__ Y, int32_t* __restrict__ iters) {
  extern __shared__ double sm[];
  double* sS = sm;
  double* sPhi = sm + NP * NP;
  double* sw = sPhi + nq * NP;
  for (int i = threadIdx.x; i < NP * NP; i += kTimeBlock) sS[i] = S[i];
  for (int i = threadIdx.x; i < nq * NP; i += kTimeBlock) sPhi[i] = Phi[i];
  for (int i = threadIdx.x; i < nq; i += kTimeBlock) sw[i] = wq[i];
  __syncthreads();
  const int64_t ic = int64_t(blockIdx.x) * kTimeBlock + threadIdx.x;
  if (ic >= n_ics) return;
  double uR = y0[ic];
  for (int k = 0; k < n_slabs; ++k) {
    const double hh = 0.5 * slab_width(times[k], times[k + 1]);
    double U[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) U[i] = uR;  // dg_march.m:46
    int it = 0;
    double err = 1.0;
    while (it <= maxit && err > tol) {  // dg_march.m:53
      double Mt[NP], J[NP][NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        Mt[i] = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) J[i][j] = 0.0;
      }
      for (int q = 0; q < nq; ++q) {  // Phi' (w.*sin(Phi U)),  Phi' diag(w.*cos(Phi U)) Phi
        const double* ph = sPhi + q * NP;
        double ur = 0.0;
#pragma unroll
        for (int i = 0; i < NP; ++i) ur = fma(ph[i], U[i], ur);
        double s, c;
        sincos(ur, &s, &c);
        const double ws = sw[q] * s, wc = sw[q] * c;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          Mt[i] = fma(ph[i], ws, Mt[i]);
          const double pi = ph[i] * wc;
#pragma unroll
          for (int j = i; j < NP; ++j) J[i][j] = fma(pi, ph[j], J[i][j]);
        }
      }
      double R[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        double a = hh * Mt[i] + (i == 0 ? uR : 0.0);  // + F (dg_march.m:59)
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const double Aij = sS[j * NP + i] + ((i == NP - 1 && j == NP - 1) ? -1.0 : 0.0);
          a = fma(Aij, U[j], a);  // A = S' + B (:61)
        }
        R[i] = a;
      }
      double D[NP][NP];  // dRdU = A + dMt/dU (:62); dMt/dU is symmetric (upper half in J)
#pragma unroll
      for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const double m = hh * (j >= i ? J[i][j] : J[j][i]);
          D[i][j] = m + sS[j * NP + i] + ((i == NP - 1 && j == NP - 1) ? -1.0 : 0.0);
        }
      lu_solve<NP>(D, R);  // delta_u = dRdU \ R (:65)
      double e2 = 0.0;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const double un = U[i] - R[i];
        const double d = U[i] - un;
        e2 = fma(d, d, e2);
        U[i] = un;
      }
      err = sqrt(e2);  // norm(U_old - U_next) (:67)
      ++it;
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) Y[(int64_t(k) * NP + i) * n_ics + ic] = U[i];
    if (iters) iters[int64_t(k) * n_ics + ic] = it;
    uR = U[NP - 1];  // (:75)
  }
}

// Adjoint march and DWR indicator, adjoint order NA-1 on the forward order NF-1 solution.
// LDS: Sa[NA*NA] (inv(V V')*Dr), Ma[NA*NA] (inv(V V')), Phia[nq*NA] (adjoint basis at the
// Gauss points), Pext[nq*NF] (forward basis at the evaluation points of adj_march.m:79),
// Ifa[NA*NF] (forward basis at the adjoint nodes), w[nq].
template <int NA, int NF>
__global__ __launch_bounds__(kTimeBlock) void k_dgt_adjoint(
    const double* __restrict__ Sa, const double* __restrict__ Ma, const double* __restrict__ Phia,
    const double* __restrict__ Pext, const double* __restrict__ Ifa,
    const double* __restrict__ wq, int nq, const double* __restrict__ times, int n_slabs,
    const double* __restrict__ y0, const double* __restrict__ Y, int64_t n_ics,
    double* __restrict__ Vout, double* __restrict__ err) {
  extern __shared__ double sm[];
  double* sS = sm;
  double* sM = sS + NA * NA;
  double* sPa = sM + NA * NA;
  double* sPe = sPa + nq * NA;
  double* sI = sPe + nq * NF;
  double* sw = sI + NA * NF;
  for (int i = threadIdx.x; i < NA * NA; i += kTimeBlock) {
    sS[i] = Sa[i];
    sM[i] = Ma[i];
  }
  for (int i = threadIdx.x; i < nq * NA; i += kTimeBlock) sPa[i] = Phia[i];
  for (int i = threadIdx.x; i < nq * NF; i += kTimeBlock) sPe[i] = Pext[i];
  for (int i = threadIdx.x; i < NA * NF; i += kTimeBlock) sI[i] = Ifa[i];
  for (int i = threadIdx.x; i < nq; i += kTimeBlock) sw[i] = wq[i];
  __syncthreads();
  const int64_t ic = int64_t(blockIdx.x) * kTimeBlock + threadIdx.x;
  if (ic >= n_ics) return;
  double vL = 0.0;
  for (int k = n_slabs - 1; k >= 0; --k) {
    double U[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) U[i] = Y[(int64_t(k) * NF + i) * n_ics + ic];
    const double hh = -0.5 * slab_width(times[k], times[k + 1]);  // hk = x(1) - x(end) < 0 (:73)
    double uh[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < NF; ++i) a = fma(sI[j * NF + i], U[i], a);
      uh[j] = a;  // polyval(pu, x) (:78)
    }
    double Mv[NA][NA], Mt[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      Mt[i] = 0.0;
#pragma unroll
      for (int j = 0; j < NA; ++j) Mv[i][j] = 0.0;
    }
    for (int q = 0; q < nq; ++q) {
      const double* pe = sPe + q * NF;
      double ur = 0.0;  // polyval(pu, r_interp) (:79-80)
#pragma unroll
      for (int i = 0; i < NF; ++i) ur = fma(pe[i], U[i], ur);
      double s, c;
      sincos(ur, &s, &c);
      const double ws = sw[q] * s, wc = sw[q] * c;
      const double* pa = sPa + q * NA;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        Mt[i] = fma(pa[i], ws, Mt[i]);
        const double pi = pa[i] * wc;
#pragma unroll
        for (int j = i; j < NA; ++j) Mv[i][j] = fma(pi, pa[j], Mv[i][j]);
      }
    }
    double A[NA][NA], F[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      double f = 0.0;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        f += sM[i * NA + j];
        const double mv = hh * (j >= i ? Mv[i][j] : Mv[j][i]);
        A[i][j] = -sS[j * NA + i] + ((i == 0 && j == 0) ? -1.0 : 0.0) - mv;  // -S' + B - M_v (:87)
      }
      F[i] = hh * f;  // M_k * ones (:96)
    }
    F[NA - 1] -= vL;
    lu_solve<NA>(A, F);  // v_k = A \ F (:98)
    vL = F[0];
    const double uprev = (k == 0) ? y0[ic] : Y[(int64_t(k - 1) * NF + NF - 1) * n_ics + ic];
    double e = 0.0;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      // -A2 uh - M_tilde + F2 with A2 = -S' - B, B(end,end) = -1 (:105-117)
      double res = -hh * Mt[i] + (i == 0 ? uprev : 0.0);
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const double a2 = -sS[j * NA + i] + ((i == NA - 1 && j == NA - 1) ? 1.0 : 0.0);
        res = fma(-a2, uh[j], res);
      }
      e = fma(F[i], res, e);
      Vout[(int64_t(k) * NA + i) * n_ics + ic] = F[i];
    }
    err[ic * n_slabs + k] = e;
  }
}

}  // namespace

extern "C" {

int dg_time_march(int Np, int nq, const double* S, const double* Phi, const double* wq,
                  int n_slabs, const double* times, int64_t n_ics, const double* y0, double tol,
                  int maxit, double* Y, int32_t* iters, void* stream) {
  if (!S || !Phi || !wq || !times || !y0 || !Y) return fail(DG_ERR_ARG, "null argument");
  if (Np < 2 || Np > kMaxNP) return fail(DG_ERR_ARG, "Np must be in 2..9");
  if (nq < 1 || n_slabs < 1 || n_ics < 1 || maxit < 0) return fail(DG_ERR_ARG, "bad sizes");
  const size_t lds = sizeof(double) * size_t(Np * Np + nq * Np + nq);
  if (lds > 64 * 1024) return fail(DG_ERR_ARG, "operators exceed 64 KiB of LDS");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = grid_for(n_ics, kTimeBlock);
  DG_DISPATCH_NP(Np, hipLaunchKernelGGL((k_dgt_march<NP>), dim3(grid), dim3(kTimeBlock), lds, st,
                                        S, Phi, wq, nq, times, n_slabs, y0, n_ics, tol, maxit, Y,
                                        iters));
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

int dg_time_adjoint(int Np_fwd, int nq, const double* Sa, const double* Ma, const double* Phia,
                    const double* Pext, const double* Ifa, const double* wq, int n_slabs,
                    const double* times, int64_t n_ics, const double* y0, const double* Y,
                    double* V, double* err, void* stream) {
  if (!Sa || !Ma || !Phia || !Pext || !Ifa || !wq || !times || !y0 || !Y || !V || !err)
    return fail(DG_ERR_ARG, "null argument");
  if (Np_fwd < 2 || Np_fwd > kMaxNP - 1) return fail(DG_ERR_ARG, "forward Np must be in 2..8");
  if (nq < 1 || n_slabs < 1 || n_ics < 1) return fail(DG_ERR_ARG, "bad sizes");
  const int NA = Np_fwd + 1;
  const size_t lds =
      sizeof(double) * size_t(2 * NA * NA + nq * NA + nq * Np_fwd + NA * Np_fwd + nq);
  if (lds > 64 * 1024) return fail(DG_ERR_ARG, "operators exceed 64 KiB of LDS");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = grid_for(n_ics, kTimeBlock);
#define DGT_ADJ(NF)                                                                         \
  hipLaunchKernelGGL((k_dgt_adjoint<NF + 1, NF>), dim3(grid), dim3(kTimeBlock), lds, st, Sa, \
                     Ma, Phia, Pext, Ifa, wq, nq, times, n_slabs, y0, Y, n_ics, V, err)
  switch (Np_fwd) {
    case 2: DGT_ADJ(2); break;
    case 3: DGT_ADJ(3); break;
    case 4: DGT_ADJ(4); break;
    case 5: DGT_ADJ(5); break;
    case 6: DGT_ADJ(6); break;
    case 7: DGT_ADJ(7); break;
    case 8: DGT_ADJ(8); break;
  }
#undef DGT_ADJ
  HIP_TRY(hipGetLastError());
  return DG_OK;
}

}  // extern "C"
