// sqp_core.hpp -- the per-instance pieces of the device SQP of
// MPCController.solve (session_4/main.py:115-116): the Hessian of one stage,
// the merit line search + update + KKT residual of one instance, and their
// constants.  sqp.hip runs them as batched kernels (one launch per piece and
// SQP iteration, mpc.SqpSolver.iterate); sqp_solve.hip runs a whole solve of
// one instance in one workgroup (mpcqp_bicycle_sqp_solve).
#pragma once

#include <algorithm>
#include <cstdlib>

#include "bike.hpp"

namespace mpcqp {

constexpr int kSqpDone = 1, kSqpExact = 2, kSqpFail = 4, kSqpProj = 8;
// an exact-Hessian QP that is not convex switches the instance to the
// per-stage projected curvature (mpcqp_bicycle_hessian_convex) for this many
// full steps (bits 24..27 count down), then the exact curvature is tried again
constexpr int kSqpProjSteps = 4;
// a Gauss-Newton QP (convex by construction) that fails this many times in a
// row stops the instance: DONE | FAIL, the QP's status code in bits 28..30
constexpr int kSqpMaxFails = 3;
// KKT residual below which the exact Hessian is used (Gauss-Newton before:
// far from a solution the costates that weight the curvature are poor, and
// the Gauss-Newton path picks the same local minimum as the oracle's)
constexpr double kSqpSwitch = 0.3;
// ... or after this many Gauss-Newton iterations (a large-residual instance
// converges only linearly under Gauss-Newton)
constexpr int kSqpGnMax = 15;
// Levenberg-Marquardt damping of the exact-Hessian QPs: x4 after a failed QP
// or a shortened step (at least kMuFloor), x1/4 after a full step
constexpr double kMuFloor = 1e-4, kMuDec = 0.25;
// watchdog: after this many shortened exact-Hessian steps in a row, one full
// step is taken without the merit test (a curved constraint or a poorly
// scaled merit can reject Newton steps that make progress; 5 moves 0.2 % of
// the bench x0 under the 60-iteration budget and keeps every saturated-tail
// fixture on the oracle's minimum, 2-3 move one to another minimum)
constexpr int kSqpWatchdog = 5;
constexpr double kFixRho = 1e2;
// Inputs held at their bound: an input at a bound whose NLP gradient pushes
// against it by more than kFixGrad (the bound is strongly active) gets the
// proximal curvature kFixRho in the next exact-Hessian QP, so the QP keeps it
// there.  The full Hessian of this NLP is indefinite along such inputs (the
// steering saturates where turning the other way would also pay); without
// the term the QP, started inside the box, may run to the far bound and
// its step is rejected, while the Hessian on the free inputs -- the one
// second-order optimality needs -- is positive definite.
constexpr double kFixGrad = 1e-6;

// Symmetric eigen-decomposition of a 6 x 6 matrix by cyclic Jacobi sweeps,
// fully unrolled (every index a compile-time constant: the matrix and the
// rotation accumulate in registers).  On exit W is diagonal (the
// eigenvalues) and V holds the eigenvectors as columns.
__device__ __forceinline__ void jacobi6(double (&W)[6][6], double (&V)[6][6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 8; ++sweep) {
    double off = 0.0, dia = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      dia = fma(W[i][i], W[i][i], dia);
#pragma unroll
      for (int j = i + 1; j < 6; ++j) off = fma(W[i][j], W[i][j], off);
    }
    if (!(off > 1e-30 * dia)) break;
#pragma unroll
    for (int pp = 0; pp < 5; ++pp) {
#pragma unroll
      for (int q = pp + 1; q < 6; ++q) {
        const double apq = W[pp][q];
        if (apq == 0.0) continue;
        const double th = (W[q][q] - W[pp][pp]) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
        const double c = 1.0 / sqrt(fma(t, t, 1.0)), sn = t * c;
#pragma unroll
        for (int k = 0; k < 6; ++k) {  // columns pp, q
          const double wkp = W[k][pp], wkq = W[k][q];
          W[k][pp] = c * wkp - sn * wkq;
          W[k][q] = sn * wkp + c * wkq;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {  // rows pp, q
          const double wpk = W[pp][k], wqk = W[q][k];
          W[pp][k] = c * wpk - sn * wqk;
          W[q][k] = sn * wpk + c * wqk;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const double vkp = V[k][pp], vkq = V[k][q];
          V[k][pp] = c * vkp - sn * vkq;
          V[k][q] = sn * vkp + c * vkq;
        }
      }
    }
  }
}

// Per-stage convexification (eigenvalue projection of the stage Hessian):
// the stage's full QP Hessian is W = blkdiag(Q, R) + Hl (Hl the Lagrangian
// curvature of the dynamics, whose (psi, v) block is always indefinite:
// d2(v cos psi) couples them bilinearly).  Where W is not positive definite
// (a Cholesky pivot below eps), its eigenvalues are lifted to eps and Hl is
// replaced by W' - blkdiag(Q, R), so the QP is convex by construction; where
// W is positive definite, Hl is left exact (Newton's rate near a solution).
__device__ __forceinline__ void project_stage(double* Hl, const double* Qw, const double* Rw,
                                              double eps) {
  double W[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const double bd = (i < 4 && j < 4) ? Qw[i * 4 + j] : ((i >= 4 && j >= 4) ? Rw[(i - 4) * 2 + (j - 4)] : 0.0);
      W[i][j] = Hl[i * 6 + j] + bd;
    }
  // Cholesky test
  bool pd = true;
  {
    double L[6][6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double d = W[j][j];
#pragma unroll
      for (int k = 0; k < j; ++k) d = fma(-L[j][k], L[j][k], d);
      pd = pd && d > eps;
      const double ljj = sqrt(fmax(d, eps));
      L[j][j] = ljj;
#pragma unroll
      for (int i = j + 1; i < 6; ++i) {
        double s = W[i][j];
#pragma unroll
        for (int k = 0; k < j; ++k) s = fma(-L[i][k], L[j][k], s);
        L[i][j] = s / ljj;
      }
    }
  }
  if (pd) return;
  double V[6][6];
  const double W0[6][6] = {{W[0][0], W[0][1], W[0][2], W[0][3], W[0][4], W[0][5]},
                           {W[1][0], W[1][1], W[1][2], W[1][3], W[1][4], W[1][5]},
                           {W[2][0], W[2][1], W[2][2], W[2][3], W[2][4], W[2][5]},
                           {W[3][0], W[3][1], W[3][2], W[3][3], W[3][4], W[3][5]},
                           {W[4][0], W[4][1], W[4][2], W[4][3], W[4][4], W[4][5]},
                           {W[5][0], W[5][1], W[5][2], W[5][3], W[5][4], W[5][5]}};
  jacobi6(W, V);
  double lam[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) lam[i] = fmax(W[i][i], eps);
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s = fma(V[i][k] * lam[k], V[j][k], s);
      Hl[i * 6 + j] += s - W0[i][j];
    }
}

// project_stage with its two 6 x 6 work matrices in memory (W, V: 36
// doubles each, row-major; the one-launch SQP passes dead LDS of the QP's
// workspace) and plain loops: the same cyclic Jacobi sweeps without the
// register file the unrolled version needs (it would set the register
// allocation of a whole fused kernel).  Hl <- V diag(max(lambda, eps)) V' -
// blkdiag(Q, R) where W = Hl + blkdiag(Q, R) is not positive definite.
__device__ __forceinline__ void project_stage_mem(double* Hl, const double* Qw, const double* Rw,
                                                  double eps, double* W, double* V) {
#pragma unroll 1
  for (int i = 0; i < 6; ++i)
#pragma unroll 1
    for (int j = 0; j < 6; ++j) {
      const double bd = (i < 4 && j < 4) ? Qw[i * 4 + j] : ((i >= 4 && j >= 4) ? Rw[(i - 4) * 2 + (j - 4)] : 0.0);
      W[i * 6 + j] = Hl[i * 6 + j] + bd;
    }
  // Cholesky test (L in V)
  bool pd = true;
#pragma unroll 1
  for (int j = 0; j < 6; ++j) {
    double d = W[j * 6 + j];
#pragma unroll 1
    for (int k = 0; k < j; ++k) d = fma(-V[j * 6 + k], V[j * 6 + k], d);
    pd = pd && d > eps;
    const double ljj = sqrt(fmax(d, eps));
    V[j * 6 + j] = ljj;
#pragma unroll 1
    for (int i = j + 1; i < 6; ++i) {
      double t = W[i * 6 + j];
#pragma unroll 1
      for (int k = 0; k < j; ++k) t = fma(-V[i * 6 + k], V[j * 6 + k], t);
      V[i * 6 + j] = t / ljj;
    }
  }
  if (pd) return;
#pragma unroll 1
  for (int i = 0; i < 36; ++i) V[i] = (i % 7 == 0) ? 1.0 : 0.0;
#pragma unroll 1
  for (int sweep = 0; sweep < 8; ++sweep) {
    double off = 0.0, dia = 0.0;
#pragma unroll 1
    for (int i = 0; i < 6; ++i) {
      dia = fma(W[i * 7], W[i * 7], dia);
#pragma unroll 1
      for (int j = i + 1; j < 6; ++j) off = fma(W[i * 6 + j], W[i * 6 + j], off);
    }
    if (!(off > 1e-30 * dia)) break;
#pragma unroll 1
    for (int pp = 0; pp < 5; ++pp) {
#pragma unroll 1
      for (int q = pp + 1; q < 6; ++q) {
        const double apq = W[pp * 6 + q];
        if (apq == 0.0) continue;
        const double th = (W[q * 7] - W[pp * 7]) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(fma(th, th, 1.0)));
        const double c = 1.0 / sqrt(fma(t, t, 1.0)), sn = t * c;
#pragma unroll 1
        for (int k = 0; k < 6; ++k) {  // columns pp, q
          const double wkp = W[k * 6 + pp], wkq = W[k * 6 + q];
          W[k * 6 + pp] = c * wkp - sn * wkq;
          W[k * 6 + q] = sn * wkp + c * wkq;
        }
#pragma unroll 1
        for (int k = 0; k < 6; ++k) {  // rows pp, q
          const double wpk = W[pp * 6 + k], wqk = W[q * 6 + k];
          W[pp * 6 + k] = c * wpk - sn * wqk;
          W[q * 6 + k] = sn * wpk + c * wqk;
        }
#pragma unroll 1
        for (int k = 0; k < 6; ++k) {
          const double vkp = V[k * 6 + pp], vkq = V[k * 6 + q];
          V[k * 6 + pp] = c * vkp - sn * vkq;
          V[k * 6 + q] = sn * vkp + c * vkq;
        }
      }
    }
  }
#pragma unroll 1
  for (int i = 0; i < 6; ++i) W[i] = fmax(W[i * 7], eps);  // the eigenvalues, lifted (row 0 of W)
#pragma unroll 1
  for (int i = 0; i < 6; ++i)
#pragma unroll 1
    for (int j = 0; j < 6; ++j) {
      double s = 0.0;
#pragma unroll 1
      for (int k = 0; k < 6; ++k) s = fma(V[i * 6 + k] * W[k], V[j * 6 + k], s);
      const double bd = (i < 4 && j < 4) ? Qw[i * 4 + j] : ((i >= 4 && j >= 4) ? Rw[(i - 4) * 2 + (j - 4)] : 0.0);
      Hl[i * 6 + j] = s - bd;
    }
}

// H2, q2 of stage k of instance b (the body of bike_hess_kernel): the
// Lagrangian curvature of the prediction model's step at (x_k, u_k) weighted
// by the costate of x_{k+1}, projected per stage in PROJ mode (Qw, Rw given),
// plus the damping mu and the proximal term of held inputs; zero in
// Gauss-Newton mode.  H (36) and q (6) are written whole.
__device__ __forceinline__ void hess_stage(int64_t b, int N, int k, const Bike& p, int integ,
                                           const double* X, const double* U, const double* pi,
                                           const int32_t* flags, const double* mu,
                                           const int32_t* fix, double fix_rho, const double* Qw,
                                           const double* Rw, double eps, double* H, double* q,
                                           double* pw = nullptr, double* pv = nullptr) {
  const bool exact = flags == nullptr || (flags[b] & kSqpExact);
  const bool proj = Qw && Rw && (flags == nullptr || (flags[b] & kSqpProj));
  if (!exact) {
    for (int i = 0; i < 36; ++i) H[i] = 0.0;
    for (int i = 0; i < 6; ++i) q[i] = 0.0;
    return;
  }
  const double* x = X + (b * (N + 1) + k) * 4;
  const double* u = U + (b * N + k) * 2;
  const double* lam = pi + (b * N + k) * 4;  // costate of x_{k+1} = fe(x_k, u_k)
  double Hl[36];
  model_lag_hess(p, integ, x, u, lam, Hl);
  if (proj) {
    if (pw) {  // work matrices pw, pv and the stage block itself (H) in memory
      for (int i = 0; i < 36; ++i) H[i] = Hl[i];
      project_stage_mem(H, Qw, Rw, eps, pw, pv);
      for (int i = 0; i < 36; ++i) Hl[i] = H[i];
    } else {
      project_stage(Hl, Qw, Rw, eps);
    }
  }
  if (mu)
    for (int i = 0; i < 6; ++i) Hl[i * 6 + i] += mu[b];
  if (fix) {
    const int32_t fb = fix[b * N + k];
    for (int r = 0; r < 2; ++r)
      if ((fb >> r) & 1) Hl[(4 + r) * 6 + 4 + r] += fix_rho;
  }
  const double w[6] = {x[0], x[1], x[2], x[3], u[0], u[1]};
  // 1/2 (w - wbar)' H (w - wbar) = 1/2 w'H w - (H wbar)'w + const
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
    for (int j = 0; j < 6; ++j) s = fma(Hl[i * 6 + j], w[j], s);
    q[i] = -s;
  }
  for (int i = 0; i < 36; ++i) H[i] = Hl[i];
}

struct SqpArgs {
  int batch, N, integ;  // integ: prediction model, 0 = forward Euler, 1 = RK4
  Bike p;
  const double* x0; int64_t sX0;
  const double *Q, *R, *Qf;
  const double *xlo, *xhi; int64_t sXb;
  const double *lb, *ub; int64_t sLb;
  double* U;
  const double *Z, *yq, *piq;
  const int32_t* qp_status;
  double *y, *pi, *X;
  double *rho, *kkt, *mu;
  int32_t* flags;
  int32_t* fix;  // (batch, N): bit q = input q held at its bound (nullable)
  double tol;
  int proj_steps;  // kSqpProjSteps (MPCQP_SQP_PROJ_STEPS overrides; 0: damping only)
  int fix_mode;    // 1 (MPCQP_SQP_FIX=0 disables holding inputs at their bounds)
  double fix_grad; // kFixGrad (MPCQP_SQP_FIX_GRAD overrides)
  double sw;       // kSqpSwitch (MPCQP_SQP_SWITCH overrides)
  double mu_dec;   // kMuDec (MPCQP_SQP_MU_DEC overrides)
  int gn_max;      // kSqpGnMax (MPCQP_SQP_GN_MAX overrides)
  int watchdog;    // kSqpWatchdog (MPCQP_SQP_WATCHDOG overrides; 0: off)
};

// 1/2 J(U) and the l1 violation of the state box along a rollout
struct Merit {
  double J, viol;
};

__device__ inline double sq_form(const double* M, int n, const double* v) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    double t = 0.0;
    for (int j = 0; j < n; ++j) t = fma(M[i * n + j], v[j], t);
    s = fma(v[i], t, s);
  }
  return s;
}

__device__ inline double box_viol(const SqpArgs& a, int64_t b, int k, const double* x) {
  double v = 0.0;
  for (int i = 0; i < 4; ++i) {
    const int64_t o = b * a.sXb + (int64_t)k * 4 + i;
    if (a.xhi) v += fmax(0.0, x[i] - a.xhi[o]);
    if (a.xlo) v += fmax(0.0, a.xlo[o] - x[i]);
  }
  return v;
}

// Search direction component i of instance b: Z - U, except for an input
// the QP held at its bound (fix bit set when the QP was built), which stays
// put -- the interior-point QP leaves such an input a barrier gap inside.
// An exact-Hessian QP holds it by the proximal term of bike_hess_kernel; in
// the Gauss-Newton phase before the switch the zeroed components make the
// step a projected one (an input on its bound whose gradient pushes outward
// stays there), checked by the merit line search like any other step.
// Measured on the saturated-tail fixtures (tests/golden/nlp_tail.npz):
// holding only in exact mode, or giving the Gauss-Newton QP the proximal
// term as well, sends 1-2 of the 10 to another local minimum.  A controller
// that never builds H2 (hessian="gauss-newton") passes no fix array.
__device__ __forceinline__ double sqp_dir(const SqpArgs& a, int64_t b, int i) {
  const int64_t o = b * a.N * 2 + i;
  if (a.fix && ((a.fix[b * a.N + (i >> 1)] >> (i & 1)) & 1)) return 0.0;
  return a.Z[o] - a.U[o];
}

// rollout of U + alpha d (d = sqp_dir), merit terms only
__device__ inline Merit merit_at(const SqpArgs& a, int64_t b, double alpha) {
  const int N = a.N;
  const double* U = a.U + b * N * 2;
  double x[4];
  for (int i = 0; i < 4; ++i) x[i] = a.x0[b * a.sX0 + i];
  Merit m{0.0, 0.0};
  for (int k = 0; k < N; ++k) {
    double u[2];
    for (int r = 0; r < 2; ++r) u[r] = fma(alpha, sqp_dir(a, b, k * 2 + r), U[k * 2 + r]);
    m.J += 0.5 * (sq_form(a.Q, 4, x) + sq_form(a.R, 2, u));
    double xn[4];
    model_step(a.p, a.integ, x, u, xn);
    for (int i = 0; i < 4; ++i) x[i] = xn[i];
    m.viol += box_viol(a, b, k, x);
  }
  m.J += 0.5 * sq_form(a.Qf, 4, x);
  return m;
}

// The QP of instance b failed (not converged within its budget, or non-
// convex beyond the inertia correction with the unprojected Hessian): no step.
// An exact-Hessian iteration raises the damping mu (x4, at least kMuFloor),
// which changes the next QP; a Gauss-Newton QP would be rebuilt unchanged, so
// kSqpMaxFails failures in a row stop the instance with the QP's status
// (never OPTIMAL).  Returns false (nothing written) when the QP succeeded.
__device__ __forceinline__ bool sqp_qp_failed(const SqpArgs& a, int64_t b, int fl) {
  if (!a.qp_status || (a.qp_status[b] & 0xFF) == MPCQP_STATUS_OPTIMAL) return false;
  const int iters = ((fl >> 8) & 0xFFFF) + 1;
  const int fails = ((fl >> 24) & 0xF) + 1;
  const int code = a.qp_status[b] & 0x7;
  if ((fl & kSqpExact) && !(fl & kSqpProj) && a.proj_steps > 0) {
    // the exact curvature made the QP fail (non-convex): the projected one
    // next (mpcqp_bicycle_hessian_convex; a caller of the plain
    // mpcqp_bicycle_hessian gets the damping below at the next failure)
    a.flags[b] = (iters << 8) | kSqpExact | kSqpProj | (a.proj_steps << 24);
  } else if (fl & kSqpExact) {
    a.mu[b] = fmax(4.0 * a.mu[b], kMuFloor);
    a.flags[b] = (iters << 8) | (fl & (kSqpExact | kSqpProj | (0xF << 24)));
  } else if (fails >= kSqpMaxFails) {
    a.flags[b] = (iters << 8) | kSqpDone | kSqpFail | (code << 28);
  } else {
    a.flags[b] = (iters << 8) | (fails << 24);
  }
  return true;
}

// After a step of length alpha with KKT residual r at the new point: the
// damping mu, the Hessian mode (the exact Hessian once r < sw or after gn_max
// iterations, sticky), the projected-curvature countdown, the watchdog count,
// DONE below tol; rho and kkt stored.
__device__ __forceinline__ void sqp_finish(const SqpArgs& a, int64_t b, int fl, double alpha,
                                           double r, double rho, bool force, int wd) {
  if (fl & kSqpExact) {
    double mu = a.mu[b];
    mu = alpha == 1.0 ? (mu > 4e-12 ? a.mu_dec * mu : 0.0) : fmax(4.0 * mu, kMuFloor);
    a.mu[b] = mu;
  }
  const int iters = ((fl >> 8) & 0xFFFF) + 1;
  const bool exact = (fl & kSqpExact) || r < a.sw || iters >= a.gn_max;  // sticky
  // projected curvature: count full steps down, then back to the exact one
  int pc = (fl & kSqpProj) ? ((fl >> 24) & 0xF) : 0;
  if (pc > 0 && alpha == 1.0) --pc;
  const int wdn = (force || alpha == 1.0) ? 0 : (wd < 15 ? wd + 1 : 15);
  fl = (iters << 8) | (r <= a.tol ? kSqpDone : 0) | (exact ? kSqpExact : 0) |
       (pc > 0 ? kSqpProj | (pc << 24) : 0) | (wdn << 4);
  a.flags[b] = fl;
  a.rho[b] = rho;
  a.kkt[b] = r;
}

// One SQP step of instance b (the body of sqp_step_kernel): line search,
// update, KKT residual, flags.
__device__ __forceinline__ void sqp_step_one(const SqpArgs& a, int64_t b) {
  int fl = a.flags[b];
  if (fl & kSqpDone) return;
  const int N = a.N;
  if (sqp_qp_failed(a, b, fl)) return;
  double* U = a.U + b * N * 2;
  const double* yq = a.yq + b * N * 4;
  const double* piq = a.piq + b * N * 4;
  double* y = a.y + b * N * 4;
  double* pi = a.pi + b * N * 4;
  double* X = a.X + b * (N + 1) * 4;

  // ----------------------------------------- merit, directional derivative
  double ymax = 0.0, dmax = 0.0, umax = 0.0;
  for (int i = 0; i < 4 * N; ++i) ymax = fmax(ymax, fabs(yq[i]));
  for (int i = 0; i < 2 * N; ++i) {
    dmax = fmax(dmax, fabs(sqp_dir(a, b, i)));
    umax = fmax(umax, fabs(U[i]));
  }
  const double rho = fmax(a.rho[b], 2.0 * ymax);
  double D = 0.0;  // d(1/2 J)/dU . d
  Merit m0{0.0, 0.0};
  {
    double x[4], dx[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < 4; ++i) x[i] = a.x0[b * a.sX0 + i];
    for (int k = 0; k < N; ++k) {
      const double u[2] = {U[2 * k], U[2 * k + 1]};
      const double d[2] = {sqp_dir(a, b, 2 * k), sqp_dir(a, b, 2 * k + 1)};
      m0.J += 0.5 * (sq_form(a.Q, 4, x) + sq_form(a.R, 2, u));
      for (int i = 0; i < 4; ++i) {
        double t = 0.0;
        for (int j = 0; j < 4; ++j) t = fma(a.Q[i * 4 + j], x[j], t);
        D = fma(t, dx[i], D);
      }
      for (int r = 0; r < 2; ++r) {
        double t = 0.0;
        for (int q = 0; q < 2; ++q) t = fma(a.R[r * 2 + q], u[q], t);
        D = fma(t, d[r], D);
      }
      double A[4][4], B[4][2], xn[4], dxn[4];
      model_step_jac(a.p, a.integ, x, u, xn, A, B);
      for (int i = 0; i < 4; ++i) {
        double s = B[i][0] * d[0] + B[i][1] * d[1];
        for (int j = 0; j < 4; ++j) s = fma(A[i][j], dx[j], s);
        dxn[i] = s;
      }
      for (int i = 0; i < 4; ++i) { x[i] = xn[i]; dx[i] = dxn[i]; }
      m0.viol += box_viol(a, b, k, x);
    }
    m0.J += 0.5 * sq_form(a.Qf, 4, x);
    for (int i = 0; i < 4; ++i) {
      double t = 0.0;
      for (int j = 0; j < 4; ++j) t = fma(a.Qf[i * 4 + j], x[j], t);
      D = fma(t, dx[i], D);
    }
  }
  const double phi0 = m0.J + rho * m0.viol;
  const double Dm = D - rho * m0.viol;

  // --------------------------- backtracking (quadratic interpolation), Armijo
  // the acceptance test is relaxed by the rounding noise of phi: near a
  // solution the predicted decrease (|d| * residual) falls below it and an
  // exact test would reject every step
  double alpha = 1.0;
  const double noise = 1e-14 * (1.0 + fabs(phi0));
  // watchdog: after a.watchdog shortened steps in a row (exact Hessian), one
  // full step is taken without the merit test
  const int wd = (fl >> 4) & 0xF;
  const bool force = a.watchdog > 0 && (fl & kSqpExact) && wd >= a.watchdog;
  if (!force && dmax > 1e-14 * (1.0 + umax)) {
    for (int t = 0; t < 40; ++t) {
      const Merit m = merit_at(a, b, alpha);
      const double phi = m.J + rho * m.viol;
      if (phi <= phi0 + 1e-4 * alpha * Dm + noise) break;
      const double den = 2.0 * (phi - phi0 - alpha * Dm);
      const double at = den > 0.0 ? -Dm * alpha * alpha / den : 0.5 * alpha;
      alpha = fmin(0.5 * alpha, fmax(0.1 * alpha, at));
      if (alpha < 1e-10) break;
    }
  }
  // inputs within 1e-9 (relative) of a bound are put on it: an interior-point
  // QP that ends unpolished leaves its active inputs that far inside, and
  // the projected gradient would count the gap as a residual
  for (int i = 0; i < 2 * N; ++i) {
    double u = fma(alpha, sqp_dir(a, b, i), U[i]);
    const int64_t o = b * a.sLb + i;
    if (a.lb && u <= a.lb[o] + 1e-9 * (1.0 + fabs(a.lb[o]))) u = a.lb[o];
    if (a.ub && u >= a.ub[o] - 1e-9 * (1.0 + fabs(a.ub[o]))) u = a.ub[o];
    U[i] = u;
  }
  for (int i = 0; i < 4 * N; ++i) {
    y[i] = fma(alpha, yq[i] - y[i], y[i]);
    pi[i] = fma(alpha, piq[i] - pi[i], pi[i]);
  }

  // ------------------------------------------ KKT residual at the new point
  // gradient of 1/2 J + y'[x_1..x_N] by the adjoint, projected on the input
  // box; state-box violation; complementarity of the state multipliers
  {
    double x[4];
    for (int i = 0; i < 4; ++i) X[i] = x[i] = a.x0[b * a.sX0 + i];
    for (int k = 0; k < N; ++k) {
      const double u[2] = {U[2 * k], U[2 * k + 1]};
      double xn[4];
      model_step(a.p, a.integ, x, u, xn);
      for (int i = 0; i < 4; ++i) X[(k + 1) * 4 + i] = x[i] = xn[i];
    }
  }
  double r = 0.0;
  {
    double lam[4];
    const double* xN = X + N * 4;
    for (int i = 0; i < 4; ++i) {
      double s = y[(N - 1) * 4 + i];
      for (int j = 0; j < 4; ++j) s = fma(a.Qf[i * 4 + j], xN[j], s);
      lam[i] = s;
    }
    for (int k = N - 1; k >= 0; --k) {
      const double* x = X + k * 4;
      const double u[2] = {U[2 * k], U[2 * k + 1]};
      double A[4][4], B[4][2], xn[4];
      model_step_jac(a.p, a.integ, x, u, xn, A, B);
      int32_t fb = 0;
      for (int q = 0; q < 2; ++q) {
        double g = 0.0;
        for (int j = 0; j < 2; ++j) g = fma(a.R[q * 2 + j], u[j], g);
        for (int i = 0; i < 4; ++i) g = fma(B[i][q], lam[i], g);
        const int64_t o = b * a.sLb + (int64_t)k * 2 + q;
        const double lo = a.lb ? a.lb[o] : -Lim<double>::inf();
        const double hi = a.ub ? a.ub[o] : Lim<double>::inf();
        const double t = fmin(fmax(u[q] - g, lo), hi);
        r = fmax(r, fabs(u[q] - t));
        if ((u[q] <= lo + 1e-9 * (1.0 + fabs(lo)) && g > a.fix_grad) ||
            (u[q] >= hi - 1e-9 * (1.0 + fabs(hi)) && g < -a.fix_grad))
          fb |= 1 << q;
      }
      if (a.fix) a.fix[b * N + k] = a.fix_mode ? fb : 0;
      // state x_{k+1}: feasibility and complementarity of y_k
      const double* xk1 = X + (k + 1) * 4;
      for (int i = 0; i < 4; ++i) {
        const int64_t o = b * a.sXb + (int64_t)k * 4 + i;
        const double hi = a.xhi ? a.xhi[o] : Lim<double>::inf();
        const double lo = a.xlo ? a.xlo[o] : -Lim<double>::inf();
        const double yi = y[k * 4 + i];
        r = fmax(r, fmax(xk1[i] - hi, lo - xk1[i]));
        if (yi > 0.0) r = fmax(r, fmin(yi, hi - xk1[i]));
        if (yi < 0.0) r = fmax(r, fmin(-yi, xk1[i] - lo));
      }
      if (k > 0) {
        double ln[4];
        for (int i = 0; i < 4; ++i) {
          double s = y[(k - 1) * 4 + i];
          for (int j = 0; j < 4; ++j) s = fma(a.Q[i * 4 + j], x[j], s);
          for (int j = 0; j < 4; ++j) s = fma(A[j][i], lam[j], s);
          ln[i] = s;
        }
        for (int i = 0; i < 4; ++i) lam[i] = ln[i];
      }
    }
  }
  if (!(r == r)) r = Lim<double>::inf();

  sqp_finish(a, b, fl, alpha, r, rho, force, wd);
}

// ------------------------------------------- the closed loop's plant
// (rcracers.simulate(x0, dynamics, n_steps, policy), main.py:270-271)
__device__ inline void bike_f(const Bike& p, const double* x, const double* u, double* f) {
  const double kk = p.k();
  const double beta = atan(kk * tan(u[1]));
  double s, c;
  sincos(x[2] + beta, &s, &c);
  f[0] = x[3] * c;
  f[1] = x[3] * s;
  f[2] = x[3] / p.lr * sin(beta);
  f[3] = p.acc * u[0] - p.fric * x[3];
}

__device__ inline void bike_rk4(const Bike& p, double h, const double* x, const double* u, double* xn) {
  double k1[4], k2[4], k3[4], k4[4], t[4];
  bike_f(p, x, u, k1);
  for (int i = 0; i < 4; ++i) t[i] = x[i] + 0.5 * h * k1[i];
  bike_f(p, t, u, k2);
  for (int i = 0; i < 4; ++i) t[i] = x[i] + 0.5 * h * k2[i];
  bike_f(p, t, u, k3);
  for (int i = 0; i < 4; ++i) t[i] = x[i] + h * k3[i];
  bike_f(p, t, u, k4);
  for (int i = 0; i < 4; ++i) xn[i] = x[i] + h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
}


// One step of the closed loop's plant, in place on x: 0 forward Euler, 1 RK4,
// 2 RK4 over `substeps` sub-intervals (the stand-in for odeint)
__device__ inline void plant_step(const Bike& p, int integrator, int substeps, double* xs,
                                  const double* u) {
  if (integrator == 0) {
    double f[4];
    bike_f(p, xs, u, f);
    for (int i = 0; i < 4; ++i) xs[i] += p.ts * f[i];
  } else {
    const int m = integrator == 1 ? 1 : substeps;
    const double h = p.ts / m;
    for (int s = 0; s < m; ++s) {
      double t[4];
      bike_rk4(p, h, xs, u, t);
      for (int i = 0; i < 4; ++i) xs[i] = t[i];
    }
  }
}

// ------------------------------------------------------------ host side
inline Bike bike_of(double ts, const double* prm) {
  Bike p;
  p.ts = ts; p.lf = prm[0]; p.lr = prm[1]; p.acc = prm[2]; p.fric = prm[3];
  return p;
}

// proximal curvature of an input held at its bound (kFixRho; the
// environment variable MPCQP_SQP_FIX_RHO overrides it for experiments)
inline double fix_rho() {
  static const double r = [] {
    const char* e = getenv("MPCQP_SQP_FIX_RHO");
    return e ? atof(e) : kFixRho;
  }();
  return r;
}

// The step's constants, each overridable by an environment variable for
// experiments (read once per process): MPCQP_SQP_PROJ_STEPS, _FIX (0: no
// held inputs), _FIX_GRAD, _SWITCH, _MU_DEC, _GN_MAX, _WATCHDOG.
inline void sqp_knobs(SqpArgs& a) {
  auto env_i = [](const char* n, int d) { const char* e = getenv(n); return e ? atoi(e) : d; };
  auto env_d = [](const char* n, double d) { const char* e = getenv(n); return e ? atof(e) : d; };
  static const int proj_steps = std::min(15, std::max(0, env_i("MPCQP_SQP_PROJ_STEPS", kSqpProjSteps)));
  static const int fix_mode = env_i("MPCQP_SQP_FIX", 1);
  static const double fix_grad = env_d("MPCQP_SQP_FIX_GRAD", kFixGrad);
  static const double sw = env_d("MPCQP_SQP_SWITCH", kSqpSwitch);
  static const double mu_dec = env_d("MPCQP_SQP_MU_DEC", kMuDec);
  static const int gn_max = env_i("MPCQP_SQP_GN_MAX", kSqpGnMax);
  static const int watchdog = env_i("MPCQP_SQP_WATCHDOG", kSqpWatchdog);
  a.proj_steps = proj_steps;
  a.fix_mode = fix_mode;
  a.fix_grad = fix_grad;
  a.sw = sw;
  a.mu_dec = mu_dec;
  a.gn_max = gn_max;
  a.watchdog = watchdog;
}

}  // namespace mpcqp
