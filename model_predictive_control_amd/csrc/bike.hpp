// bike.hpp -- the kinematic bicycle of session_4 (forward Euler and RK4) as
// scalar device functions (one instance per lane): the step, its Jacobians
// and the curvature sum_i lam_i d2 x+_i / d(x,u)2 an exact-Hessian SQP needs.
// Model (rcracers is absent; restated from parameters.py:7-8,47-48 -- parity
// unpinned), x = [p_x, p_y, psi, v], u = [a, delta]:
//   beta = atan(k tan delta), k = l_r / (l_f + l_r)
//   f = [v cos(psi+beta), v sin(psi+beta), v / l_r sin(beta), acc a - fric v]
//   fe(x, u) = x + ts f(x, u)                               (main.py:132-135)
#pragma once

#include "common.hpp"

namespace mpcqp {

struct Bike {
  double ts, lf, lr, acc, fric;
  __device__ __forceinline__ double k() const { return lr / (lf + lr); }
};

// trig terms of one point
struct BikePt {
  double st, ct;      // sin, cos of psi + beta
  double sb, cb;      // sin, cos of beta
  double db, ddb;     // dbeta/ddelta, d2beta/ddelta2
};

__device__ __forceinline__ BikePt bike_pt(const Bike& p, const double* x, const double* u) {
  const double kk = p.k();
  const double t = tan(u[1]);
  const double beta = atan(kk * t);
  const double den = 1.0 + kk * kk * t * t;
  BikePt q;
  sincos(x[2] + beta, &q.st, &q.ct);
  sincos(beta, &q.sb, &q.cb);
  q.db = kk * (1.0 + t * t) / den;
  q.ddb = 2.0 * kk * t * (1.0 - kk * kk) * (1.0 + t * t) / (den * den);
  return q;
}

__device__ __forceinline__ void bike_step(const Bike& p, const BikePt& q, const double* x,
                                          const double* u, double* xn) {
  const double v = x[3];
  xn[0] = x[0] + p.ts * v * q.ct;
  xn[1] = x[1] + p.ts * v * q.st;
  xn[2] = x[2] + p.ts * v / p.lr * q.sb;
  xn[3] = x[3] + p.ts * (p.acc * u[0] - p.fric * v);
}

// A = d fe / dx (4 x 4), B = d fe / du (4 x 2)
__device__ __forceinline__ void bike_jac(const Bike& p, const BikePt& q, const double* x,
                                         double (&A)[4][4], double (&B)[4][2]) {
  const double v = x[3], ts = p.ts;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) A[i][j] = i == j ? 1.0 : 0.0;
  A[0][2] = -ts * v * q.st;  A[0][3] = ts * q.ct;
  A[1][2] = ts * v * q.ct;   A[1][3] = ts * q.st;
  A[2][3] = ts * q.sb / p.lr;
  A[3][3] = 1.0 - ts * p.fric;
  B[0][0] = 0.0; B[0][1] = -ts * v * q.st * q.db;
  B[1][0] = 0.0; B[1][1] = ts * v * q.ct * q.db;
  B[2][0] = 0.0; B[2][1] = ts * v * q.cb * q.db / p.lr;
  B[3][0] = ts * p.acc; B[3][1] = 0.0;
}

// sum_i lam_i d2 fe_i / dw2 over w = [x; u] (6 x 6, row-major): only
// (psi, v, delta) = w[2], w[3], w[5] couple.
__device__ __forceinline__ void bike_lag_hess(const Bike& p, const BikePt& q, const double* x,
                                              const double* lam, double* H) {
  const double v = x[3], ts = p.ts;
  const double l0 = lam[0], l1 = lam[1], l2 = lam[2];
  // d2 f0: v cos th, d2 f1: v sin th, d2 f2: v / lr sin beta
  const double hpp = -v * (l0 * q.ct + l1 * q.st);
  const double hpv = -l0 * q.st + l1 * q.ct;
  const double hpd = q.db * hpp;
  const double hvd = q.db * hpv + l2 * q.cb * q.db / p.lr;
  const double hdd = q.db * q.db * hpp + q.ddb * v * (-l0 * q.st + l1 * q.ct) +
                     l2 * v / p.lr * (q.cb * q.ddb - q.sb * q.db * q.db);
  for (int i = 0; i < 36; ++i) H[i] = 0.0;
  H[2 * 6 + 2] = ts * hpp;
  H[2 * 6 + 3] = H[3 * 6 + 2] = ts * hpv;
  H[2 * 6 + 5] = H[5 * 6 + 2] = ts * hpd;
  H[3 * 6 + 5] = H[5 * 6 + 3] = ts * hvd;
  H[5 * 6 + 5] = ts * hdd;
}

// f(x, u) and its Jacobians (continuous time)
__device__ __forceinline__ void bike_f_jac(const Bike& p, const double* x, const double* u,
                                           double* f, double (&Jx)[4][4], double (&Ju)[4][2]) {
  const BikePt q = bike_pt(p, x, u);
  const double v = x[3];
  f[0] = v * q.ct;
  f[1] = v * q.st;
  f[2] = v / p.lr * q.sb;
  f[3] = p.acc * u[0] - p.fric * v;
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) Jx[i][j] = 0.0;
    Ju[i][0] = Ju[i][1] = 0.0;
  }
  Jx[0][2] = -v * q.st;  Jx[0][3] = q.ct;
  Jx[1][2] = v * q.ct;   Jx[1][3] = q.st;
  Jx[2][3] = q.sb / p.lr;
  Jx[3][3] = -p.fric;
  Ju[0][1] = -v * q.st * q.db;
  Ju[1][1] = v * q.ct * q.db;
  Ju[2][1] = v * q.cb * q.db / p.lr;
  Ju[3][0] = p.acc;
}

// One RK4 step (runge_kutta4, main.py:138-147) and, when A != nullptr, its
// Jacobians A = d x+ / dx, B = d x+ / du by forward sensitivities through
// the four stages (tangent S = d(stage point)/d(x, u), 4 x 6).
__device__ __forceinline__ void bike_rk4_step_jac(const Bike& p, const double* x,
                                                  const double* u, double* xn,
                                                  double (*A)[4], double (*B)[2]) {
  const double h = p.ts;
  const double cw[4] = {h / 6.0, h / 3.0, h / 3.0, h / 6.0};  // stage weights
  const double cs[4] = {0.0, 0.5 * h, 0.5 * h, h};            // stage offsets
  double k[4] = {0, 0, 0, 0}, dk[4][6];
  double acc[4], dacc[4][6];
  for (int i = 0; i < 4; ++i) {
    acc[i] = x[i];
    for (int j = 0; j < 6; ++j) { dk[i][j] = 0.0; dacc[i][j] = (j == i) ? 1.0 : 0.0; }
  }
  for (int s = 0; s < 4; ++s) {
    double xs[4], S[4][6];
    for (int i = 0; i < 4; ++i) {
      xs[i] = x[i] + cs[s] * k[i];
      for (int j = 0; j < 6; ++j) S[i][j] = ((j == i) ? 1.0 : 0.0) + cs[s] * dk[i][j];
    }
    double f[4], Jx[4][4], Ju[4][2];
    bike_f_jac(p, xs, u, f, Jx, Ju);
    for (int i = 0; i < 4; ++i) {
      k[i] = f[i];
      acc[i] += cw[s] * f[i];
    }
    if (A) {
      double nk[4][6];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 6; ++j) {
          double t = j >= 4 ? Ju[i][j - 4] : 0.0;
          for (int q2 = 0; q2 < 4; ++q2) t = fma(Jx[i][q2], S[q2][j], t);
          nk[i][j] = t;
        }
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 6; ++j) {
          dk[i][j] = nk[i][j];
          dacc[i][j] += cw[s] * nk[i][j];
        }
    }
  }
  for (int i = 0; i < 4; ++i) xn[i] = acc[i];
  if (A)
    for (int i = 0; i < 4; ++i) {
      for (int j = 0; j < 4; ++j) A[i][j] = dacc[i][j];
      B[i][0] = dacc[i][4];
      B[i][1] = dacc[i][5];
    }
}

// sum_i lam_i d2 F_i / dw2 (6 x 6, row-major) of one RK4 step F(x, u) by the
// second-order adjoint of its computational graph: with stage points z_j =
// (s_j, u), s_j = x + c_j k_{j-1}, k_j = f(z_j) and F = x + sum_j w_j k_j,
//   d2 (lam'F) = sum_j Dz_j' [sum_i rho_j,i d2 f_i(z_j)] Dz_j,
// rho_j the adjoint of k_j (rho_4 = w_4 lam, rho_j = w_j lam + c_{j+1}
// Jx_{j+1}' rho_{j+1}) and Dz_j = d z_j / dw (the forward sensitivities of
// bike_rk4_step_jac); the continuous curvature is bike_lag_hess at ts = 1.
__device__ __forceinline__ void bike_rk4_lag_hess(const Bike& p, const double* x, const double* u,
                                                  const double* lam, double* H) {
  const double h = p.ts;
  const double cw[4] = {h / 6.0, h / 3.0, h / 3.0, h / 6.0};
  const double cs[4] = {0.0, 0.5 * h, 0.5 * h, h};
  double zs[4][4], S[4][4][6], J[4][4][4];
  double k[4] = {0, 0, 0, 0}, dk[4][6];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 6; ++j) dk[i][j] = 0.0;
  for (int s = 0; s < 4; ++s) {
    for (int i = 0; i < 4; ++i) {
      zs[s][i] = x[i] + cs[s] * k[i];
      for (int j = 0; j < 6; ++j) S[s][i][j] = ((j == i) ? 1.0 : 0.0) + cs[s] * dk[i][j];
    }
    double f[4], Ju[4][2];
    bike_f_jac(p, zs[s], u, f, J[s], Ju);
    for (int i = 0; i < 4; ++i) {
      k[i] = f[i];
      for (int j = 0; j < 6; ++j) {
        double t = j >= 4 ? Ju[i][j - 4] : 0.0;
        for (int q = 0; q < 4; ++q) t = fma(J[s][i][q], S[s][q][j], t);
        dk[i][j] = t;
      }
    }
  }
  Bike pc = p;
  pc.ts = 1.0;
  for (int i = 0; i < 36; ++i) H[i] = 0.0;
  double rho[4];
  for (int i = 0; i < 4; ++i) rho[i] = cw[3] * lam[i];
  for (int s = 3; s >= 0; --s) {
    // W = sum_i rho_i d2 f_i at z_s: non-zero only on (psi, v, delta)
    double W[36];
    const BikePt q = bike_pt(pc, zs[s], u);
    bike_lag_hess(pc, q, zs[s], rho, W);
    // G: the rows psi, v, delta of Dz_s (3 x 6)
    double G[3][6];
    for (int j = 0; j < 6; ++j) {
      G[0][j] = S[s][2][j];
      G[1][j] = S[s][3][j];
      G[2][j] = j == 5 ? 1.0 : 0.0;
    }
    const int id[3] = {2, 3, 5};
    double Wc[3][3];
    for (int a = 0; a < 3; ++a)
      for (int c = 0; c < 3; ++c) Wc[a][c] = W[id[a] * 6 + id[c]];
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) {
        double t = 0.0;
        for (int a = 0; a < 3; ++a)
          for (int c = 0; c < 3; ++c) t = fma(G[a][i] * Wc[a][c], G[c][j], t);
        H[i * 6 + j] += t;
      }
    if (s > 0) {  // rho_{s-1} = w_{s-1} lam + c_s J_s' rho_s
      double rn[4];
      for (int i = 0; i < 4; ++i) {
        double t = 0.0;
        for (int q2 = 0; q2 < 4; ++q2) t = fma(J[s][q2][i], rho[q2], t);
        rn[i] = fma(cs[s], t, cw[s - 1] * lam[i]);
      }
      for (int i = 0; i < 4; ++i) rho[i] = rn[i];
    }
  }
}

// sum_i lam_i d2 x+_i / dw2 of the prediction model (integ as model_step)
__device__ __forceinline__ void model_lag_hess(const Bike& p, int integ, const double* x,
                                               const double* u, const double* lam, double* H) {
  if (integ == 1) {
    bike_rk4_lag_hess(p, x, u, lam, H);
  } else {
    const BikePt q = bike_pt(p, x, u);
    bike_lag_hess(p, q, x, lam, H);
  }
}

// the prediction model of the OCP: 0 = forward Euler (main.py:132-135),
// 1 = RK4 (main.py:138-147, the model template.py:141 builds on)
__device__ __forceinline__ void model_step(const Bike& p, int integ, const double* x,
                                           const double* u, double* xn) {
  if (integ == 1) {
    bike_rk4_step_jac(p, x, u, xn, nullptr, nullptr);
  } else {
    const BikePt q = bike_pt(p, x, u);
    bike_step(p, q, x, u, xn);
  }
}

__device__ __forceinline__ void model_step_jac(const Bike& p, int integ, const double* x,
                                               const double* u, double* xn, double (&A)[4][4],
                                               double (&B)[4][2]) {
  if (integ == 1) {
    bike_rk4_step_jac(p, x, u, xn, A, B);
  } else {
    const BikePt q = bike_pt(p, x, u);
    bike_step(p, q, x, u, xn);
    bike_jac(p, q, x, A, B);
  }
}

}  // namespace mpcqp
