/* advec_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): a plain-C restatement of
 * the numpy oracle's config-2 sweep, for bench.py's cpu_baseline leg (a compiled, OpenMP
 * CPU port of the same algorithm, timed on the host cores) and checked against the numpy
 * oracle by tests/test_oracle_cport.py.  Nothing in the product package links or loads it.
 *
 *   oc_forward_sweep  -- oracle/advec.py forward_sweep: the LSERK4 stage loop of
 *                        utils/One_code.mlx:120-139 over AdvecRHS1D (utils/AdvecRHS1D.m:9-19,
 *                        central flux alpha = 1, inflow uin = -sin(a t), du(mapO) = 0).
 *   oc_p_estimate     -- oracle/effectivity.py p_estimate (inflow uin = -sin(a t)): the
 *                        order-(N+1) adjoint from the terminal weight g (adj_march.m:103-117
 *                        at order N+1, MAIN.m:32-34) paired with the prolonged one-step
 *                        residual R^n = P u^{n+1} - S_{N+1}(P u^n, t_n): eta -= w^{n+1}.R^n
 *                        (summed here from the last step back, the oracle sums forward).
 *   oc_adjoint_sweep  -- oracle/adjoint.py adjoint_sweep (src = 0): eta += dt sum_i w^{n+1}
 *                        R(u^{n+1}, t_{n+1}) with R = LIFT (Fscale .* du) (AdvecRHS1D.m:19),
 *                        then w^n = S^T w^{n+1} through the reversed stages
 *                        (lr += B_s lu; lu += dt L^T lr; lr = A_s lr), L^T as
 *                        adjoint.py advec_linear_T's scatter through vmapM / vmapP, written
 *                        as a gather over each element's two faces.
 *
 * Layout: fields element-major, u[k*Np + i] (the product's and oracle.setup1d.to_elem_major's);
 * Dr row-major Np x Np, LIFT row-major Np x 2 (column 0: left face, 1: right face); rx and
 * the face scales per element (the oracle's metric="element"). */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OC_MAXNP 16

typedef struct {
  int np;
  long k;
  const double* dr;   /* Np x Np */
  const double* lift; /* Np x 2 */
  const double* rx;   /* K */
  const double* fsl;  /* K: Fscale of the left face */
  const double* fsr;  /* K: Fscale of the right face */
  double a;
} oc_mesh;

void oc_set_threads(int n) {
#ifdef _OPENMP
  omp_set_num_threads(n > 0 ? n : 1);
#else
  (void)n;
#endif
}

int oc_max_np(void) { return OC_MAXNP; }

/* du of AdvecRHS1D.m:11-16 for element k: (u^- - u^+) (a nx) / 2, the inflow at the first
 * element's left face, 0 at the last element's right face. */
static void face_jumps(const oc_mesh* m, const double* u, double uin, long k, double* dul,
                       double* dur) {
  const int np = m->np;
  const double* uk = u + k * np;
  const double left = (k == 0) ? uin : u[(k - 1) * np + np - 1];
  *dul = (uk[0] - left) * (-m->a) / 2.0;
  *dur = (k == m->k - 1) ? 0.0 : (uk[np - 1] - u[(k + 1) * np]) * m->a / 2.0;
}

/* The element loops below take Np as a compile-time constant (NP_DISPATCH), so the small
 * matrix products unroll. */
#define OC_INLINE static inline __attribute__((always_inline))
#define NP_DISPATCH(fn, ...)                       \
  switch (m->np) {                                 \
    case 1: fn(1, __VA_ARGS__); break;             \
    case 2: fn(2, __VA_ARGS__); break;             \
    case 3: fn(3, __VA_ARGS__); break;             \
    case 4: fn(4, __VA_ARGS__); break;             \
    case 5: fn(5, __VA_ARGS__); break;             \
    case 6: fn(6, __VA_ARGS__); break;             \
    case 7: fn(7, __VA_ARGS__); break;             \
    case 8: fn(8, __VA_ARGS__); break;             \
    case 9: fn(9, __VA_ARGS__); break;             \
    default: fn(m->np, __VA_ARGS__); break;        \
  }

/* rhsu = -a rx (Dr u) + LIFT (Fscale .* du)  (AdvecRHS1D.m:19) into r; lift_only: the
 * residual R = LIFT (Fscale .* du) alone (oracle/advec.py lift_residual). */
OC_INLINE void rhs_np(const int np, const oc_mesh* m, const double* u, double uin, double* r,
                      int lift_only) {
  const long K = m->k;
#pragma omp parallel for schedule(static)
  for (long k = 0; k < K; ++k) {
    double dul, dur;
    face_jumps(m, u, uin, k, &dul, &dur);
    const double fl = m->fsl[k] * dul, fr = m->fsr[k] * dur;
    const double c = -m->a * m->rx[k];
    const double* uk = u + k * np;
    double* rk = r + k * np;
    for (int i = 0; i < np; ++i) {
      const double lift = m->lift[2 * i] * fl + m->lift[2 * i + 1] * fr;
      if (lift_only) {
        rk[i] = lift;
      } else {
        double d = 0.0;
        for (int j = 0; j < np; ++j) d += m->dr[i * np + j] * uk[j];
        rk[i] = c * d + lift;
      }
    }
  }
}

static void rhs(const oc_mesh* m, const double* u, double uin, double* r, int lift_only) {
  NP_DISPATCH(rhs_np, m, u, uin, r, lift_only)
}

/* One LSERK4 stage (One_code.mlx:135-136) fused with its right-hand side, element by element:
 * res = A res + dt rhs(uin_field); uout = uin_field + B res.  The rhs reads the neighbours'
 * stage input, so the stage writes a second field (ping-pong); res is element-local. */
OC_INLINE void stage_np(const int np, const oc_mesh* m, const double* __restrict__ u,
                        double uin, double A, double B, double dt, double* __restrict__ res,
                        double* __restrict__ uo) {
  const long K = m->k;
  double dr[OC_MAXNP * OC_MAXNP], l0[OC_MAXNP], l1[OC_MAXNP];
  for (int i = 0; i < np * np; ++i) dr[i] = m->dr[i];
  for (int i = 0; i < np; ++i) {
    l0[i] = m->lift[2 * i];
    l1[i] = m->lift[2 * i + 1];
  }
#pragma omp parallel for schedule(static)
  for (long k = 0; k < K; ++k) {
    double dul, dur;
    face_jumps(m, u, uin, k, &dul, &dur);
    const double fl = m->fsl[k] * dul, fr = m->fsr[k] * dur;
    const double c = -m->a * m->rx[k];
    const double* uk = u + k * np;
    double* rk = res + k * np;
    double* ok = uo + k * np;
    for (int i = 0; i < np; ++i) {
      double d = 0.0;
      for (int j = 0; j < np; ++j) d += dr[i * np + j] * uk[j];
      const double rhsu = c * d + (l0[i] * fl + l1[i] * fr);
      rk[i] = A * rk[i] + dt * rhsu;
      ok[i] = uk[i] + B * rk[i];
    }
  }
}

static void stage(const oc_mesh* m, const double* u, double uin, double A, double B, double dt,
                  double* res, double* uo) {
  NP_DISPATCH(stage_np, m, u, uin, A, B, dt, res, uo)
}

/* out = L^T w (oracle/adjoint.py advec_linear_T): Dr^T (-a rx w) plus the face terms.  The
 * face weights z = Fscale .* (LIFT^T w) scaled by c = a nx / 2 land on the own face node
 * (vmapM) with + and on the neighbour's face node (vmapP) with -, except at the inflow face
 * (no neighbour term) and the outflow face (du = 0: no term at all).  zc: 2K scratch. */
OC_INLINE void lin_t_np(const int np, const oc_mesh* m, const double* __restrict__ w,
                        double* __restrict__ out, double* __restrict__ zc) {
  const long K = m->k;
  double dr[OC_MAXNP * OC_MAXNP];
  for (int i = 0; i < np * np; ++i) dr[i] = m->dr[i];
#pragma omp parallel for schedule(static)
  for (long k = 0; k < K; ++k) {
    const double* wk = w + k * np;
    double zl = 0.0, zr = 0.0;
    for (int i = 0; i < np; ++i) {
      zl += m->lift[2 * i] * wk[i];
      zr += m->lift[2 * i + 1] * wk[i];
    }
    zc[2 * k] = (-m->a / 2.0) * (m->fsl[k] * zl);
    zc[2 * k + 1] = (k == K - 1) ? 0.0 : (m->a / 2.0) * (m->fsr[k] * zr);
  }
#pragma omp parallel for schedule(static)
  for (long k = 0; k < K; ++k) {
    const double* wk = w + k * np;
    double* ok = out + k * np;
    const double c = -m->a * m->rx[k];
    for (int i = 0; i < np; ++i) {
      double d = 0.0;
      for (int j = 0; j < np; ++j) d += dr[j * np + i] * (c * wk[j]);
      ok[i] = d;
    }
    ok[0] += zc[2 * k];
    if (k >= 1) ok[0] -= zc[2 * k - 1];          /* element k-1's right face, P side */
    ok[np - 1] += zc[2 * k + 1];
    if (k + 1 < K) ok[np - 1] -= zc[2 * k + 2];  /* element k+1's left face, P side */
  }
}

static void lin_t(const oc_mesh* m, const double* w, double* out, double* zc) {
  NP_DISPATCH(lin_t_np, m, w, out, zc)
}

/* dst = 0 over n doubles, in parallel (first touch of fresh pages too) */
static void par_zero(double* dst, long n) {
#pragma omp parallel for schedule(static)
  for (long q = 0; q < n; ++q) dst[q] = 0.0;
}

/* snaps: (nsteps + 1) fields, snaps[0] = u^0 on entry; fills u^1..u^nsteps.  rk: A[5], B[5],
 * C[5] (oracle.setup1d RK4A / RK4B / RK4C).  Time levels t_{n+1} = t_n + dt. */
int oc_forward_sweep(int np, long K, const double* dr, const double* lift, const double* rx,
                     const double* fsl, const double* fsr, double a, double t0, double dt,
                     int nsteps, const double* rk, double* snaps) {
  if (np < 1 || np > OC_MAXNP || K < 1 || nsteps < 0) return 1;
  const oc_mesh m = {np, K, dr, lift, rx, fsl, fsr, a};
  const long n = (long)np * K;
  double* res = (double*)malloc(sizeof(double) * (size_t)n);
  double* tmp = (double*)malloc(sizeof(double) * (size_t)n);
  if (!res || !tmp) {
    free(res);
    free(tmp);
    return 2;
  }
  double time = t0;
  for (int step = 0; step < nsteps; ++step) {
    /* stages 0..4 ping-pong between tmp and the step's snapshot so that the last (s = 4)
     * lands in the snapshot: in -> tmp -> out -> tmp -> out -> ... would end in tmp, so the
     * first stage writes the snapshot field */
    const double* u = snaps + (long)step * n;
    double* out = snaps + (long)(step + 1) * n;
    par_zero(res, n);  /* resu is step-local: rk4a(1) = 0 */
    for (int s = 0; s < 5; ++s) {
      const double tl = time + rk[10 + s] * dt;
      double* dst = (s % 2 == 0) ? out : tmp;
      stage(&m, u, -sin(a * tl), rk[s], rk[5 + s], dt, res, dst);
      u = dst;
    }
    time = time + dt;
  }
  free(res);
  free(tmp);
  return 0;
}

/* w: w^nsteps on entry, w^0 on exit; eta (K): the indicator (assigned).  times: t_0..t_nsteps.
 * snaps: u^0..u^nsteps from oc_forward_sweep. */
int oc_adjoint_sweep(int np, long K, const double* dr, const double* lift, const double* rx,
                     const double* fsl, const double* fsr, double a, double dt, int nsteps,
                     const double* rk, const double* times, const double* snaps, double* w,
                     double* eta) {
  if (np < 1 || np > OC_MAXNP || K < 1 || nsteps < 0) return 1;
  const oc_mesh m = {np, K, dr, lift, rx, fsl, fsr, a};
  const long n = (long)np * K;
  double* lr = (double*)malloc(sizeof(double) * (size_t)n);
  double* t = (double*)malloc(sizeof(double) * (size_t)n);
  double* zc = (double*)malloc(sizeof(double) * (size_t)(2 * K));
  if (!lr || !t || !zc) {
    free(lr);
    free(t);
    free(zc);
    return 2;
  }
  par_zero(eta, K);
  for (int step = nsteps - 1; step >= 0; --step) {
    /* eta += dt * sum_i w^{n+1} R(u^{n+1}, t_{n+1}) */
    rhs(&m, snaps + (long)(step + 1) * n, -sin(a * times[step + 1]), t, 1);
#pragma omp parallel for schedule(static)
    for (long k = 0; k < K; ++k) {
      double s = 0.0;
      for (int i = 0; i < np; ++i) s += w[k * np + i] * t[k * np + i];
      eta[k] = eta[k] + dt * s;
    }
    /* w^n = S^T w^{n+1}: for s = 4..0: lr += B_s lu; lu += dt L^T lr; lr = A_s lr */
    par_zero(lr, n);
    for (int s = 4; s >= 0; --s) {
      const double A = rk[s], B = rk[5 + s];
#pragma omp parallel for schedule(static)
      for (long q = 0; q < n; ++q) lr[q] = lr[q] + B * w[q];
      lin_t(&m, lr, t, zc);
#pragma omp parallel for schedule(static)
      for (long q = 0; q < n; ++q) {
        w[q] = w[q] + dt * t[q];
        lr[q] = A * lr[q];
      }
    }
  }
  free(lr);
  free(t);
  free(zc);
  return 0;
}

/* out = P u element by element (oracle/effectivity.py prolong_matrix: order-N nodal values to
 * the order-(N+1) LGL nodes); P row-major nph x npl. */
static void prolong(int npl, int nph, long K, const double* P, const double* u, double* out) {
#pragma omp parallel for schedule(static)
  for (long k = 0; k < K; ++k) {
    const double* uk = u + k * npl;
    double* ok = out + k * nph;
    for (int i = 0; i < nph; ++i) {
      double d = 0.0;
      for (int j = 0; j < npl; ++j) d += P[i * npl + j] * uk[j];
      ok[i] = d;
    }
  }
}

/* snaps: u^0..u^nsteps at order N (npl nodes); the operators are the order-(N+1) mesh's (nph
 * nodes; the same per-element metric); w: the terminal weight g at order N+1 on entry, w^0 on
 * exit; eta (K) assigned.  times: t_0..t_nsteps. */
int oc_p_estimate(int npl, int nph, long K, const double* dr, const double* lift,
                  const double* rx, const double* fsl, const double* fsr, const double* P,
                  double a, double dt, int nsteps, const double* rk, const double* times,
                  const double* snaps, double* w, double* eta) {
  if (npl < 1 || nph < 1 || nph > OC_MAXNP || K < 1 || nsteps < 0) return 1;
  const oc_mesh m = {nph, K, dr, lift, rx, fsl, fsr, a};
  const long nl = (long)npl * K, nh = (long)nph * K;
  double* pa = (double*)malloc(sizeof(double) * (size_t)nh);
  double* pb = (double*)malloc(sizeof(double) * (size_t)nh);
  double* s1 = (double*)malloc(sizeof(double) * (size_t)nh);
  double* s2 = (double*)malloc(sizeof(double) * (size_t)nh);
  double* res = (double*)malloc(sizeof(double) * (size_t)nh);
  double* lr = (double*)malloc(sizeof(double) * (size_t)nh);
  double* zc = (double*)malloc(sizeof(double) * (size_t)(2 * K));
  int rc = 0;
  if (!pa || !pb || !s1 || !s2 || !res || !lr || !zc) {
    rc = 2;
    goto done;
  }
  par_zero(eta, K);
  for (int step = nsteps - 1; step >= 0; --step) {
    /* R = P u^{n+1} - S_{N+1}(P u^n, t_n): the stage loop of oracle/advec.py lserk4_step */
    prolong(npl, nph, K, P, snaps + (long)(step + 1) * nl, pa);
    prolong(npl, nph, K, P, snaps + (long)step * nl, pb);
    par_zero(res, nh);
    const double* u = pb;
    for (int s = 0; s < 5; ++s) {
      double* dst = (s % 2 == 0) ? s1 : s2;
      stage(&m, u, -sin(a * (times[step] + rk[10 + s] * dt)), rk[s], rk[5 + s], dt, res, dst);
      u = dst;
    }
    /* eta -= w^{n+1} . R (u = s1: the step's result) */
#pragma omp parallel for schedule(static)
    for (long k = 0; k < K; ++k) {
      double c = 0.0;
      for (int i = 0; i < nph; ++i) c += w[k * nph + i] * (pa[k * nph + i] - u[k * nph + i]);
      eta[k] = eta[k] - c;
    }
    /* w^n = S_{N+1}^T w^{n+1} (oracle/adjoint.py adjoint_step) */
    par_zero(lr, nh);
    for (int s = 4; s >= 0; --s) {
      const double A = rk[s], B = rk[5 + s];
#pragma omp parallel for schedule(static)
      for (long q = 0; q < nh; ++q) lr[q] = lr[q] + B * w[q];
      lin_t(&m, lr, s2, zc);
#pragma omp parallel for schedule(static)
      for (long q = 0; q < nh; ++q) {
        w[q] = w[q] + dt * s2[q];
        lr[q] = A * lr[q];
      }
    }
  }
done:
  free(pa);
  free(pb);
  free(s1);
  free(s2);
  free(res);
  free(lr);
  free(zc);
  return rc;
}
