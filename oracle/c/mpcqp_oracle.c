/*
 * mpcqp_oracle.c -- plain-C restatement of the condensed box-QP MPC step,
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY (never linked into the product).
 *
 * Per instance (x0 and optionally its own A, B):
 *   condense: explicit Gamma / Phi of session_4/main.py:86-106 for
 *             x_{k+1} = A x_k + B u_k, Qhat = blkdiag(Q,..,Q,Qf), Rhat = I (x) R
 *             H = Gam' Qhat Gam + Rhat,  f = Gam' Qhat Phi x0
 *   solve:    min 1/2 z'Hz + f'z,  lb <= z <= ub  by the Goldfarb-Idnani dual
 *             active set on the swept inverse (same algorithm family as the
 *             device kernel; checked against the NumPy primal active set and
 *             SciPy BVLS in tests/test_oracle.py).
 * Threads: OpenMP over instances (bench.py reports the thread count).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static void sweep(double* M, int n, int k, double sigma) {
  const double d = M[k * n + k];
  double* rk = (double*)alloca(sizeof(double) * n);
  memcpy(rk, M + k * n, sizeof(double) * n);
  for (int i = 0; i < n; ++i) {
    double* mi = M + i * n;
    const double a = mi[k] / d;
    const double beta = (i == k) ? (sigma / d - 1.0) : -a;
    for (int j = 0; j < n; ++j) mi[j] += beta * rk[j];
    mi[k] += (i == k) ? (-1.0 / d - sigma) : sigma * a;
  }
}

/* returns iterations (>=0), or -1 not convex, -2 max_iter */
static int gi_box(const double* H, const double* f, const double* lb, const double* ub, int n,
                  double* z, double* M, double* g, int* st, int max_iter) {
  memcpy(M, H, sizeof(double) * n * n);
  for (int k = 0; k < n; ++k) {
    if (!(M[k * n + k] > 0)) return -1;
    sweep(M, n, k, 1.0);
  }
  for (int i = 0; i < n; ++i) st[i] = 0;
  int it = 0;
  for (;;) {
    /* refresh: s = M w */
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int j = 0; j < n; ++j) {
        const double w = st[j] == 0 ? f[j] : -(st[j] == 1 ? lb[j] : ub[j]);
        s += M[i * n + j] * w;
      }
      z[i] = st[i] == 0 ? s : (st[i] == 1 ? lb[i] : ub[i]);
      g[i] = st[i] == 0 ? 0.0 : f[i] - s;
    }
    int p = -1;
    double best = 1e-12;
    for (int i = 0; i < n; ++i) {
      if (st[i]) continue;
      double v = -INFINITY;
      if (isfinite(lb[i])) v = (lb[i] - z[i]) / (1 + fabs(lb[i]));
      if (isfinite(ub[i])) { double u = (z[i] - ub[i]) / (1 + fabs(ub[i])); if (u > v) v = u; }
      if (v > best) { best = v; p = i; }
    }
    if (p < 0) return it;
    const int side = z[p] < lb[p] ? 1 : 2;
    const double tgt = side == 1 ? lb[p] : ub[p];
    for (int i = 0; i < n; ++i) g[i] = st[i] == 1 ? g[i] : (st[i] == 2 ? -g[i] : 0.0); /* mu */
    for (;;) {
      if (++it > max_iter) return -2;
      const double mpp = M[p * n + p];
      const double sgn = tgt > z[p] ? 1.0 : -1.0;
      const double t2 = fabs(tgt - z[p]);
      double t1 = INFINITY;
      int k = -1;
      for (int i = 0; i < n; ++i) {
        if (!st[i]) continue;
        const double cr = M[i * n + p] / mpp;
        const double dmu = (st[i] == 1 ? -cr : cr) * sgn;
        if (dmu < 0 && g[i] / (-dmu) < t1) { t1 = g[i] / (-dmu); k = i; }
      }
      if (t1 < t2) {
        for (int i = 0; i < n; ++i) {
          const double cr = M[i * n + p] / mpp;
          if (st[i] == 0) z[i] += sgn * t1 * cr;
          else g[i] += t1 * (st[i] == 1 ? -cr : cr) * sgn;
        }
        g[k] = 0; st[k] = 0;
        if (!(M[k * n + k] > 0)) return -1;
        sweep(M, n, k, 1.0);
      } else {
        st[p] = side;
        if (!(M[p * n + p] < 0)) return -1;
        sweep(M, n, p, -1.0);
        break;
      }
    }
  }
}

static void condense1(const double* A, const double* B, const double* Q, const double* R,
                      const double* Qf, int nx, int nu, int N, const double* x0, double* H,
                      double* f, double* Gam, double* Phi, double* QG, double* tmp) {
  const int n = N * nu, m = N * nx;
  memset(Gam, 0, sizeof(double) * m * n);
  double* P = tmp;            /* nx*nx current power */
  double* P2 = tmp + nx * nx;
  for (int i = 0; i < nx * nx; ++i) P[i] = (i / nx == i % nx);
  for (int k = 0; k < N; ++k) {
    for (int r = 0; r < nx; ++r)
      for (int c = 0; c < nx; ++c) {
        double s = 0;
        for (int q = 0; q < nx; ++q) s += A[r * nx + q] * P[q * nx + c];
        P2[r * nx + c] = s;
      }
    memcpy(P, P2, sizeof(double) * nx * nx);
    memcpy(Phi + k * nx * nx, P, sizeof(double) * nx * nx);
    if (k > 0)
      for (int r = 0; r < nx; ++r)
        for (int c = 0; c < k * nu; ++c) {
          double s = 0;
          for (int q = 0; q < nx; ++q) s += A[r * nx + q] * Gam[((k - 1) * nx + q) * n + c];
          Gam[(k * nx + r) * n + c] = s;
        }
    for (int r = 0; r < nx; ++r)
      for (int c = 0; c < nu; ++c) Gam[(k * nx + r) * n + k * nu + c] = B[r * nu + c];
  }
  /* QG = Qhat Gam, xb = Phi x0 */
  for (int k = 0; k < N; ++k) {
    const double* Qk = (k == N - 1) ? Qf : Q;
    for (int r = 0; r < nx; ++r)
      for (int c = 0; c < n; ++c) {
        double s = 0;
        for (int q = 0; q < nx; ++q) s += Qk[r * nx + q] * Gam[(k * nx + q) * n + c];
        QG[(k * nx + r) * n + c] = s;
      }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int r = 0; r < m; ++r) s += Gam[r * n + i] * QG[r * n + j];
      if (i / nu == j / nu) s += R[(i % nu) * nu + (j % nu)];
      H[i * n + j] = H[j * n + i] = s;
    }
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int r = 0; r < m; ++r) {
      double xb = 0;
      for (int q = 0; q < nx; ++q) xb += Phi[r * nx + q] * x0[q];
      s += QG[r * n + i] * xb;
    }
    f[i] = s;
  }
}

/* Batched condense + box solve.  A, B per instance when strideA/strideB > 0.
 * z (batch x n), iters (batch) = iterations or <0 on failure. */
int oracle_mpc_box(int batch, int nx, int nu, int N, const double* A, long strideA,
                   const double* B, long strideB, const double* Q, const double* R,
                   const double* Qf, const double* x0, const double* lb, const double* ub,
                   double* z, int* iters, int nthreads) {
  const int n = N * nu, m = N * nx;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    double* H = (double*)malloc(sizeof(double) * n * n);
    double* M = (double*)malloc(sizeof(double) * n * n);
    double* f = (double*)malloc(sizeof(double) * n);
    double* g = (double*)malloc(sizeof(double) * n);
    int* st = (int*)malloc(sizeof(int) * n);
    double* Gam = (double*)malloc(sizeof(double) * m * n);
    double* QG = (double*)malloc(sizeof(double) * m * n);
    double* Phi = (double*)malloc(sizeof(double) * m * nx);
    double* tmp = (double*)malloc(sizeof(double) * 2 * nx * nx);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int b = 0; b < batch; ++b) {
      condense1(A + (long)b * strideA, B + (long)b * strideB, Q, R, Qf, nx, nu, N,
                x0 + (long)b * nx, H, f, Gam, Phi, QG, tmp);
      iters[b] = gi_box(H, f, lb, ub, n, z + (long)b * n, M, g, st, 3 * n + 30);
    }
    free(H); free(M); free(f); free(g); free(st); free(Gam); free(QG); free(Phi); free(tmp);
  }
  return 0;
}
