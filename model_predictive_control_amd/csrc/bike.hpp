// bike.hpp -- the forward-Euler kinematic bicycle of session_4 as scalar
// device functions (one instance per lane): the step, its Jacobians and the
// curvature sum_i lam_i d2 fe_i / d(x,u)2 an exact-Hessian SQP needs.
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

}  // namespace mpcqp
