// ipm_lane.hpp -- one instance of the box-constrained, time-varying LQ
// problem of an MPC step, solved by a primal-dual interior-point method on the
// NON-condensed (stage-wise) structure with a Riccati factorisation per
// iteration.  Included by ipm.hip (one instance per lane) with
// MPCQP_HD = __host__ __device__.
//
// Problem (the OCP of session_4/main.py:41-113 / session4_sol.py:132-217 on
// linear(ised) dynamics, cost scaled by 1/2 like the condensed QP):
//   min  1/2 sum_{k<N} (x_k'Q x_k + u_k'R u_k) + 1/2 x_N'Qf x_N
//        [+ 1/2 sum_k w_k'H2_k w_k + q2_k'w_k,  w_k = [x_k; u_k]]
//   s.t. x_{k+1} = A_k x_k + B_k u_k + c_k,   x_0 given,
//        lb_k <= u_k <= ub_k,   xlo_k <= x_{k+1} <= xhi_k     (k = 0..N-1)
// Any bound may be infinite.  No limit on N: the work is O(N (nx+nu)^3) per
// iteration and nothing is dense in N (the condensed kernels need
// N (nx+nu) <= 192, which the reference's N = 50 controllers,
// session4_sol.py:342,391,445, exceed).
//
// Method: Mehrotra predictor-corrector.  The bounded variables stay strictly
// inside their boxes (slacks s = v - lo, hi - v are derived, never stored);
// the dynamics may be violated by the iterate (infeasible start) and are
// driven to zero by the Newton steps.  Each iteration is four sweeps over the
// horizon:
//   1. backward: apply the previous step, residuals, Sigma = lam/s, Riccati
//      factorisation (P_k, K_k, G_k^-1) and the predictor right-hand side;
//   2. forward: predictor direction, its step to the boundary and the
//      affine complementarity (a quadratic in alpha, accumulated on the way);
//   3. backward: corrector right-hand side on the stored factorisation;
//   4. forward: corrector direction, step length.
// Once mu is small the active set is guessed and polished to the exact
// vertex (method of multipliers on the same Riccati structure).
// Stage k owns u_k, x_{k+1}, pi_{k+1} (the costate of x_{k+1} = ...), the
// bound duals of u_k and x_{k+1}, and the factor data; everything lives in a
// stage-major, field-major workspace (global: instance-minor, one fp64 per
// lane per field, so every wavefront access is one coalesced row; or a slice
// of LDS).
//
// Register economy (one lane holds a whole instance): symmetric matrices are
// packed, the backward sweeps carry only the cost-to-go (Ph, ph) and one
// vector gx1 = A_{k+1}'pi_{k+2} + H2xu_{k+1} u_{k+1} + q2x_{k+1} from the
// later stage, every helper is inlined (arrays passed by pointer to a
// non-inlined call would live in scratch), and the stage data are reloaded
// from the workspace where a sweep needs them again.
#pragma once

#include <stdint.h>

#include <cmath>

#ifndef MPCQP_HD
#error "define MPCQP_HD before including ipm_lane.hpp"
#endif

#define MPCQP_IL MPCQP_HD inline __attribute__((always_inline))

namespace mpcqp {
namespace ipm {

// per-stage field offsets (in doubles) of the workspace
template <int NX, int NU>
struct Layout {
  static constexpr int NB = NU + NX;  // bounded components of stage k: u_k then x_{k+1}
  static constexpr int SX = NX * (NX + 1) / 2, SU = NU * (NU + 1) / 2;
  // iterate
  static constexpr int U = 0, X = U + NU, PI = X + NX, LL = PI + NX, LU = LL + NB;
  // corrector direction (du, dx, dpi) and predictor direction (duA, dxA)
  static constexpr int DU = LU + NB, DX = DU + NU, DPI = DX + NX, DUA = DPI + NX, DXA = DUA + NU;
  // factorisation and right-hand sides
  static constexpr int PP = DXA + NX;   // P_{k+1}, packed lower
  static constexpr int KM = PP + SX;    // K_k (NU x NX)
  static constexpr int GI = KM + NU * NX;  // G_k^-1, packed lower
  static constexpr int E = GI + SU;     // e_k: dynamics residual
  static constexpr int KV = E + NX;     // k_k: feed-forward
  static constexpr int PV = KV + NU;    // p_{k+1}
  static constexpr int GA = PV + NX;    // gradient without bound duals
  // the stage data, converted to fp64 and padded once at the start: the
  // sweeps read nothing else (no runtime nx/nu tests, no per-lane pointers)
  static constexpr int DA = GA + NB, DB = DA + NX * NX, DC = DB + NX * NU;
  static constexpr int WXX = DC + NX;     // Q (Qf at k = N-1) + H2xx_{k+1}: cost of x_{k+1}, packed
  static constexpr int WUU = WXX + SX;    // R + H2uu_k, packed
  static constexpr int WXU = WUU + SU;    // H2xu_k (NX x NU): coupling of x_k and u_k
  static constexpr int QX = WXU + NX * NU;  // q2x_{k+1}
  static constexpr int QU = QX + NX;      // q2u_k
  static constexpr int LO = QU + NU, HI = LO + NB;  // bounds of u_k, x_{k+1} (+-inf: none)
  static constexpr int F = HI + NB;
};

template <typename T>
struct Args {
  int batch, nx, nu, N, tv, max_iter;
  int strict;                    // > 0: at most this many inertia corrections, then NOT_CONVEX
  double tol, tol_mu;            // convergence of the interior-point iteration
  double tol_polish, mu_polish;  // first polish attempt: residuals and mu below these
  const T* A; int64_t sA;
  const T* B; int64_t sB;
  const T* c; int64_t sC;
  const T* Q; int64_t sQ;
  const T* R; int64_t sR;
  const T* Qf; int64_t sQf;
  const T* x0; int64_t sX0;
  const T* xlo; const T* xhi; int64_t sXb;
  const T* lb; int64_t sLb;
  const T* ub; int64_t sUb;
  const T* U0; int64_t sU0;  // optional starting inputs (N x nu); NULL = 0
  // optional extra stage cost 1/2 [x_k; u_k]'H2_k [x_k; u_k] + q2_k'[x_k; u_k],
  // k = 0..N-1, (nx+nu)^2 and nx+nu per stage (the curvature of the dynamics
  // in an exact-Hessian SQP); NULL = none
  const T* H2; int64_t sH2;
  const T* q2; int64_t sq2;
  T* z;                      // N*nu
  T* y;                      // optional N*nx: state-bound multipliers, > 0 at xhi
  T* X;                      // optional N*nx: x_1..x_N
  T* lam_u;                  // optional N*nu: input-bound multipliers, > 0 at ub
  T* pi;                     // optional N*nx: costates of x_{k+1} = A x_k + B u_k + c_k
  int32_t* status;
  // optional: instances with (skip[b] & skip_mask) != 0 are left untouched
  // (outputs and status keep their values; e.g. the SQP's converged ones)
  const int32_t* skip; int32_t skip_mask;
  double* ws;
  // optional: solve only the instances list[0 .. *list_count) (device
  // memory; the fp64 fallback of mpcqp_mpc_qp), on a grid sized for a few
  // of them -- an empty list costs one short launch, not one per instance
  const int* list; const int* list_count;
  int list_begin;  // list mode: entries list_begin .. *list_count
};

constexpr double kInf = __builtin_huge_val();

MPCQP_IL bool fin(double v) { return __builtin_isfinite(v); }
MPCQP_IL constexpr int pk(int i, int j) {
  return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i;
}

// Workspace accessor: field f of stage k of this lane's instance, LD
// instances interleaved (a compile-time stride, so every field offset is an
// immediate of the load instead of a hoisted per-field register).
template <int F, int LD>
struct Ws {
  double* W;
  MPCQP_IL double& operator()(int k, int f) const { return W[(k * F + f) * LD]; }
};

// Stage bounds of the NB components (u_k then x_{k+1}); +-inf where absent.
template <typename T, int NX, int NU>
MPCQP_IL void load_bounds(const Args<T>& a, int b, int k, double* lo, double* hi) {
  for (int j = 0; j < NU; ++j) {
    const bool on = j < a.nu;
    lo[j] = (on && a.lb) ? (double)a.lb[(int64_t)b * a.sLb + (int64_t)k * a.nu + j] : -kInf;
    hi[j] = (on && a.ub) ? (double)a.ub[(int64_t)b * a.sUb + (int64_t)k * a.nu + j] : kInf;
  }
  for (int i = 0; i < NX; ++i) {
    const bool on = i < a.nx;
    const int64_t o = (int64_t)b * a.sXb + (int64_t)k * a.nx + i;
    lo[NU + i] = (on && a.xlo) ? (double)a.xlo[o] : -kInf;
    hi[NU + i] = (on && a.xhi) ? (double)a.xhi[o] : kInf;
  }
}

// Bounds of stage k from the workspace.
template <int NX, int NU, class W>
MPCQP_IL void ws_bounds(const W& at, int k, double* lo, double* hi) {
  using L = Layout<NX, NU>;
  for (int j = 0; j < L::NB; ++j) {
    lo[j] = at(k, L::LO + j);
    hi[j] = at(k, L::HI + j);
  }
}

// Q (stage < N) or Qf, entry (i, j) with zero padding.
template <typename T>
MPCQP_IL double wq(const Args<T>& a, int b, bool term, int i, int j) {
  if (i >= a.nx || j >= a.nx) return 0.0;
  const T* M = term ? a.Qf + (int64_t)b * a.sQf : a.Q + (int64_t)b * a.sQ;
  return (double)M[i * a.nx + j];
}
// R, padded with the identity (a padded input has zero B column: it stays 0)
template <typename T>
MPCQP_IL double wr(const Args<T>& a, int b, int i, int j) {
  if (i >= a.nu || j >= a.nu) return i == j ? 1.0 : 0.0;
  return (double)a.R[(int64_t)b * a.sR + i * a.nu + j];
}

// Extra stage cost of stage k (zero when absent, for k = N, and on padding):
// xx block (i, j < nx), xu block (i < nx, r < nu), uu block, linear terms.
template <typename T>
MPCQP_IL const T* h2_stage(const Args<T>& a, int b, int k) {
  const int n2 = a.nx + a.nu;
  return a.H2 + (int64_t)b * a.sH2 + (int64_t)k * n2 * n2;
}
template <typename T>
MPCQP_IL double h2xx(const Args<T>& a, int b, int k, int i, int j) {
  if (!a.H2 || k >= a.N || i >= a.nx || j >= a.nx) return 0.0;
  return (double)h2_stage(a, b, k)[i * (a.nx + a.nu) + j];
}
template <typename T>
MPCQP_IL double h2xu(const Args<T>& a, int b, int k, int i, int r) {
  if (!a.H2 || k >= a.N || i >= a.nx || r >= a.nu) return 0.0;
  return (double)h2_stage(a, b, k)[i * (a.nx + a.nu) + a.nx + r];
}
template <typename T>
MPCQP_IL double h2uu(const Args<T>& a, int b, int k, int r, int q) {
  if (!a.H2 || k >= a.N || r >= a.nu || q >= a.nu) return 0.0;
  return (double)h2_stage(a, b, k)[(a.nx + r) * (a.nx + a.nu) + a.nx + q];
}
template <typename T>
MPCQP_IL double q2x(const Args<T>& a, int b, int k, int i) {
  if (!a.q2 || k >= a.N || i >= a.nx) return 0.0;
  return (double)a.q2[(int64_t)b * a.sq2 + (int64_t)k * (a.nx + a.nu) + i];
}
template <typename T>
MPCQP_IL double q2u(const Args<T>& a, int b, int k, int r) {
  if (!a.q2 || k >= a.N || r >= a.nu) return 0.0;
  return (double)a.q2[(int64_t)b * a.sq2 + (int64_t)k * (a.nx + a.nu) + a.nx + r];
}

// Stage data of stage k from the workspace.
template <int NX, int NU, class W>
MPCQP_IL void load_ab(const W& at, int k, double (&Am)[NX][NX], double (&Bm)[NX][NU]) {
  using L = Layout<NX, NU>;
  for (int i = 0; i < NX; ++i) {
    for (int j = 0; j < NX; ++j) Am[i][j] = at(k, L::DA + i * NX + j);
    for (int j = 0; j < NU; ++j) Bm[i][j] = at(k, L::DB + i * NU + j);
  }
}

// Gradient of the cost plus the dynamics terms (no bound duals) for u_k
// (g[0..NU)) and x_{k+1} (g[NU..NB)): v = [u_k; x_{k+1}], pi = pi_{k+1},
// xk = x_k, gx1 = A_{k+1}'pi_{k+2} + H2xu_{k+1} u_{k+1} (from the later
// stage; 0 at k = N-1).
template <int NX, int NU, class W>
MPCQP_IL void stage_grad(const W& at, int k, const double (&Bm)[NX][NU], const double* v,
                         const double (&pi)[NX], const double (&xk)[NX], const double (&gx1)[NX],
                         double* g) {
  using L = Layout<NX, NU>;
  for (int j = 0; j < NU; ++j) {
    double s = at(k, L::QU + j);
    for (int q = 0; q < NU; ++q) s = fma(at(k, L::WUU + pk(j, q)), v[q], s);
    for (int i = 0; i < NX; ++i) s = fma(at(k, L::WXU + i * NU + j), xk[i], s);
    for (int i = 0; i < NX; ++i) s = fma(Bm[i][j], pi[i], s);
    g[j] = s;
  }
  for (int i = 0; i < NX; ++i) {
    double s = gx1[i] - pi[i] + at(k, L::QX + i);
    for (int q = 0; q < NX; ++q) s = fma(at(k, L::WXX + pk(i, q)), v[NU + q], s);
    g[NU + i] = s;
  }
}

// gx1 for the stage before k: A_k'pi_{k+1} + H2xu_k u_k.
template <int NX, int NU, class W>
MPCQP_IL void next_gx1(const W& at, int k, const double (&Am)[NX][NX], const double (&pi)[NX],
                       const double* u, double (&gx1)[NX]) {
  using L = Layout<NX, NU>;
  for (int i = 0; i < NX; ++i) {
    double s = 0.0;
    for (int q = 0; q < NX; ++q) s = fma(Am[q][i], pi[q], s);
    for (int r = 0; r < NU; ++r) s = fma(at(k, L::WXU + i * NU + r), u[r], s);
    gx1[i] = s;
  }
}

// Symmetric positive-definite NU x NU inverse, packed lower in and out.
// Returns false on a non-positive pivot.
template <int NU>
MPCQP_IL bool spd_inv(const double* G, double* Gi) {
  if constexpr (NU == 1) {
    if (!(G[0] > 0.0)) return false;
    Gi[0] = 1.0 / G[0];
    return true;
  } else {
    static_assert(NU == 2, "spd_inv: NU <= 2");
    const double det = G[0] * G[2] - G[1] * G[1];
    if (!(G[0] > 0.0) || !(det > 0.0)) return false;
    const double r = 1.0 / det;
    Gi[0] = G[2] * r;
    Gi[1] = -G[1] * r;
    Gi[2] = G[0] * r;
    return true;
  }
}

// One backward Riccati step of the Newton system.  In: the cost-to-go of
// x_{k+1} from the stages after k (Ph packed, ph), the stage data, the
// gradient g and the diagonal barrier/penalty Sigma of u_k (first NU) and
// x_{k+1} (next NX).  Out: P_{k+1} (packed), p_{k+1} (the full cost-to-go of
// x_{k+1}), K_k, k_k, G_k^-1, and Ph, ph overwritten with the cost-to-go of
// x_k.  dreg is added to every Hessian diagonal (inertia correction of a
// non-convex stage cost, H2).  False on a non-positive pivot of
// G = R + Sigma_u + B'P B: the reduced Hessian is not positive definite.
template <int NX, int NU, class W>
MPCQP_IL bool riccati_stage(const W& at, int k, const double (&Am)[NX][NX],
                            const double (&Bm)[NX][NU], const double (&e)[NX], const double* g,
                            const double* sig, double* Ph, double (&ph)[NX], double* P,
                            double (&p)[NX], double (&K)[NU][NX], double (&kk)[NU], double* Gi,
                            double dreg) {
  using L = Layout<NX, NU>;
  // P_{k+1} = Q' + H2xx_{k+1} + Sigma_x + Ph,  p_{k+1} = g_x + ph
  for (int i = 0; i < NX; ++i) {
    for (int j = 0; j <= i; ++j)
      P[pk(i, j)] = at(k, L::WXX + pk(i, j)) + Ph[pk(i, j)] + (i == j ? sig[NU + i] + dreg : 0.0);
    p[i] = g[NU + i] + ph[i];
  }
  // Pe = P e + p
  double Pe[NX];
  for (int i = 0; i < NX; ++i) {
    double s = p[i];
    for (int j = 0; j < NX; ++j) s = fma(P[pk(i, j)], e[j], s);
    Pe[i] = s;
  }
  // G = R + H2uu + Sigma_u + B'PB,  h = g_u + B'Pe
  double G[NU * (NU + 1) / 2], h[NU];
  {
    double PB[NX][NU];
    for (int i = 0; i < NX; ++i)
      for (int r = 0; r < NU; ++r) {
        double t = 0.0;
        for (int q = 0; q < NX; ++q) t = fma(P[pk(i, q)], Bm[q][r], t);
        PB[i][r] = t;
      }
    for (int r = 0; r < NU; ++r) {
      for (int q = 0; q <= r; ++q) {
        double s = at(k, L::WUU + pk(r, q)) + (r == q ? sig[r] + dreg : 0.0);
        for (int i = 0; i < NX; ++i) s = fma(Bm[i][r], PB[i][q], s);
        G[pk(r, q)] = s;
      }
      double s = g[r];
      for (int i = 0; i < NX; ++i) s = fma(Bm[i][r], Pe[i], s);
      h[r] = s;
    }
  }
  // Hx = H2xu' + B'PA,  Ph = A'PA (then + Hx'K below)
  double Hx[NU][NX];
  {
    double PA[NX][NX];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) {
        double t = 0.0;
        for (int q = 0; q < NX; ++q) t = fma(P[pk(i, q)], Am[q][j], t);
        PA[i][j] = t;
      }
    for (int r = 0; r < NU; ++r)
      for (int j = 0; j < NX; ++j) {
        double s = at(k, L::WXU + j * NU + r);
        for (int i = 0; i < NX; ++i) s = fma(Bm[i][r], PA[i][j], s);
        Hx[r][j] = s;
      }
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = 0.0;
        for (int q = 0; q < NX; ++q) s = fma(Am[q][i], PA[q][j], s);
        Ph[pk(i, j)] = s;
      }
  }
  for (int r = 0; r < NU * (NU + 1) / 2; ++r) Gi[r] = 0.0;
  const bool ok = spd_inv<NU>(G, Gi);
  // K = -Gi Hx,  kk = -Gi h
  for (int r = 0; r < NU; ++r) {
    for (int j = 0; j < NX; ++j) {
      double s = 0.0;
      for (int q = 0; q < NU; ++q) s = fma(Gi[pk(r, q)], Hx[q][j], s);
      K[r][j] = -s;
    }
    double s = 0.0;
    for (int q = 0; q < NU; ++q) s = fma(Gi[pk(r, q)], h[q], s);
    kk[r] = -s;
  }
  // Ph += Hx'K,  ph = A'Pe + Hx'kk   (the cost-to-go of x_k)
  for (int i = 0; i < NX; ++i) {
    for (int j = 0; j <= i; ++j) {
      double s = Ph[pk(i, j)];
      for (int r = 0; r < NU; ++r) s = fma(Hx[r][i], K[r][j], s);
      Ph[pk(i, j)] = s;
    }
    double s = 0.0;
    for (int q = 0; q < NX; ++q) s = fma(Am[q][i], Pe[q], s);
    for (int r = 0; r < NU; ++r) s = fma(Hx[r][i], kk[r], s);
    ph[i] = s;
  }
  return ok;
}

// Store the factor data of stage k.
template <int NX, int NU, class W>
MPCQP_IL void store_factor(const W& at, int k, const double* P, const double (&p)[NX],
                           const double (&K)[NU][NX], const double (&kk)[NU], const double* Gi,
                           const double (&e)[NX]) {
  using L = Layout<NX, NU>;
  for (int q = 0; q < L::SX; ++q) at(k, L::PP + q) = P[q];
  for (int i = 0; i < NX; ++i) {
    for (int r = 0; r < NU; ++r) at(k, L::KM + r * NX + i) = K[r][i];
    at(k, L::E + i) = e[i];
    at(k, L::PV + i) = p[i];
  }
  for (int q = 0; q < L::SU; ++q) at(k, L::GI + q) = Gi[q];
  for (int r = 0; r < NU; ++r) at(k, L::KV + r) = kk[r];
}

// Forward sweep of the Newton direction from the stored factors:
// du = K dx + kk, dx+ = A dx + B du + e (dx_0 = 0); calls body(k, du, dxn).
template <int NX, int NU, class W, class Body>
MPCQP_IL void forward_sweep(const W& at, int N, Body&& body) {
  using L = Layout<NX, NU>;
  double dx[NX];
  for (int i = 0; i < NX; ++i) dx[i] = 0.0;
  for (int k = 0; k < N; ++k) {
    double du[NU], dxn[NX];
    for (int r = 0; r < NU; ++r) {
      double s = at(k, L::KV + r);
      for (int j = 0; j < NX; ++j) s = fma(at(k, L::KM + r * NX + j), dx[j], s);
      du[r] = s;
    }
    for (int i = 0; i < NX; ++i) {
      double s = at(k, L::E + i);
      for (int j = 0; j < NX; ++j) s = fma(at(k, L::DA + i * NX + j), dx[j], s);
      for (int r = 0; r < NU; ++r) s = fma(at(k, L::DB + i * NU + r), du[r], s);
      dxn[i] = s;
    }
    body(k, du, dxn);
    for (int i = 0; i < NX; ++i) dx[i] = dxn[i];
  }
}

// Starting margin inside a box: a point at least this far from a finite bound.
MPCQP_IL double interior(double v, double lo, double hi) {
  const bool fl = fin(lo), fh = fin(hi);
  if (fl && fh) {
    const double m = 0.05 * (hi - lo);
    return fmin(fmax(v, lo + m), hi - m);
  }
  if (fl) return fmax(v, lo + 0.05 * (1.0 + fabs(lo)));
  if (fh) return fmin(v, hi - 0.05 * (1.0 + fabs(hi)));
  return v;
}

// ------------------------------------------------------------- polish
// Guess the active set from the interior-point iterate (lam > s), then
// solve the QP with those bounds as equalities exactly: method of
// multipliers on  L = J + y'(v - b) + rho/2 |v - b|^2  over the active
// components, each step one Riccati sweep pair on the same structure.
// Accepted when the inactive bounds hold and the multipliers have the
// right sign; the result is then the vertex solution itself, not a
// barrier-perturbed point (weakly active bounds would otherwise leave an
// O(sqrt(mu)) error).  The iterate lives in DU/DX/DPI (v, pi), the
// multipliers in DUA/DXA and the active flags in GA; the interior-point
// iterate in U/X/PI/LL/LU is not touched.
template <typename T, int NX, int NU, class W>
MPCQP_IL bool polish(const Args<T>& a, int b, const W& at, const double (&x0)[NX]) {
  using L = Layout<NX, NU>;
  constexpr int NB = L::NB;
  const int N = a.N;
  for (int k = 0; k < N; ++k) {
    double lo[NB], hi[NB];
    ws_bounds<NX, NU>(at, k, lo, hi);
    for (int j = 0; j < NB; ++j) {
      const double vj = j < NU ? at(k, L::U + j) : at(k, L::X + j - NU);
      const double l = at(k, L::LL + j), u = at(k, L::LU + j);
      const double rl = fin(lo[j]) ? l / (vj - lo[j]) : 0.0;
      const double ru = fin(hi[j]) ? u / (hi[j] - vj) : 0.0;
      const double act = (ru > 1.0 && ru >= rl) ? 1.0 : ((rl > 1.0) ? -1.0 : 0.0);
      at(k, L::GA + j) = act;
      const double y = act > 0.0 ? u : (act < 0.0 ? -l : 0.0);
      if (j < NU) { at(k, L::DU + j) = vj; at(k, L::DUA + j) = y; }
      else { at(k, L::DX + j - NU) = vj; at(k, L::DXA + j - NU) = y; }
    }
    for (int i = 0; i < NX; ++i) at(k, L::DPI + i) = at(k, L::PI + i);
  }
  // rounds: after each, violated inactive bounds join the active set and
  // active ones with a wrong-sign multiplier leave it (a primal-dual
  // active-set step from the interior-point guess); accepted when a round
  // changes nothing.  Penalty per step: a large rho pins the active
  // components and moves the multipliers close in one step, but rho (v - b)
  // carries rho times the rounding of v - b (~1e-16 |b|) into y; the smaller
  // ones that follow contract the remaining error by ~curvature / rho each
  // with a floor of 1e-12 (rho = 1e4)
  constexpr int kSteps = 4, kRounds = 4;
  const double kRho[kSteps] = {1e8, 1e6, 1e4, 1e4};
  for (int round = 0; round < kRounds; ++round) {
    bool good = true, changed = false;
    for (int step = 0; step < kSteps; ++step) {
      const double rho = kRho[step];
      double Ph[L::SX], ph[NX], gx1[NX];
      for (int q = 0; q < L::SX; ++q) Ph[q] = 0.0;
      for (int i = 0; i < NX; ++i) ph[i] = gx1[i] = 0.0;
      for (int k = N - 1; k >= 0; --k) {
        double v[NB], pi[NX], lo[NB], hi[NB], xk[NX];
        for (int j = 0; j < NU; ++j) v[j] = at(k, L::DU + j);
        for (int i = 0; i < NX; ++i) { v[NU + i] = at(k, L::DX + i); pi[i] = at(k, L::DPI + i); }
        for (int i = 0; i < NX; ++i) xk[i] = k == 0 ? x0[i] : at(k - 1, L::DX + i);
        ws_bounds<NX, NU>(at, k, lo, hi);
        double Am[NX][NX], Bm[NX][NU], e[NX];
        load_ab<NX, NU>(at, k, Am, Bm);
        for (int i = 0; i < NX; ++i) {
          double s = at(k, L::DC + i) - v[NU + i];
          for (int j = 0; j < NX; ++j) s = fma(Am[i][j], xk[j], s);
          for (int j = 0; j < NU; ++j) s = fma(Bm[i][j], v[j], s);
          e[i] = s;
        }
        double g[NB], sig[NB];
        stage_grad<NX, NU>(at, k, Bm, v, pi, xk, gx1, g);
        for (int j = 0; j < NB; ++j) {
          const double act = at(k, L::GA + j);
          const double y = j < NU ? at(k, L::DUA + j) : at(k, L::DXA + j - NU);
          sig[j] = act != 0.0 ? rho : 0.0;
          if (act != 0.0) g[j] += y + rho * (v[j] - (act > 0.0 ? hi[j] : lo[j]));
        }
        double P[L::SX], p[NX], K[NU][NX], kk[NU], Gi[L::SU];
        good = riccati_stage<NX, NU>(at, k, Am, Bm, e, g, sig, Ph, ph, P, p, K, kk, Gi, 0.0) &&
               good;
        store_factor<NX, NU>(at, k, P, p, K, kk, Gi, e);
        next_gx1<NX, NU>(at, k, Am, pi, v, gx1);
      }
      // forward: full Newton step, then the multiplier update
      const bool last = step == kSteps - 1;
      forward_sweep<NX, NU>(at, N, [&](int k, const double (&du)[NU], const double (&dxn)[NX]) {
        for (int i = 0; i < NX; ++i) {
          double s = at(k, L::PV + i);
          for (int j = 0; j < NX; ++j) s = fma(at(k, L::PP + pk(i, j)), dxn[j], s);
          at(k, L::DPI + i) += s;
        }
        double lo[NB], hi[NB];
        ws_bounds<NX, NU>(at, k, lo, hi);
        for (int j = 0; j < NB; ++j) {
          double& vr = j < NU ? at(k, L::DU + j) : at(k, L::DX + j - NU);
          const double vj = vr + (j < NU ? du[j] : dxn[j - NU]);
          vr = vj;
          const double act = at(k, L::GA + j);
          if (act != 0.0) {
            double& yr = j < NU ? at(k, L::DUA + j) : at(k, L::DXA + j - NU);
            const double bnd = act > 0.0 ? hi[j] : lo[j];
            const double y = yr + rho * (vj - bnd);
            yr = y;
            if (last) {
              good = good && fabs(vj - bnd) <= 1e-9 * (1.0 + fabs(bnd));
              if (act > 0.0 ? y < -1e-9 * (1.0 + fabs(y)) : y > 1e-9 * (1.0 + fabs(y))) {
                at(k, L::GA + j) = 0.0;  // wrong sign: release
                yr = 0.0;
                changed = true;
              }
            }
          } else if (last) {
            const double jl = (lo[j] - vj) / (1.0 + fabs(lo[j]));
            const double jh = (vj - hi[j]) / (1.0 + fabs(hi[j]));
            if (jl > 1e-9 || jh > 1e-9) {  // violated: fix at the violated side
              at(k, L::GA + j) = jl > jh ? -1.0 : 1.0;
              changed = true;
            }
          }
        }
      });
    }
    if (good && !changed) return true;
    if (!good) return false;
  }
  return false;
}

// Outputs of one instance.  polished: v in DU/DX, multipliers (> 0 at the
// upper bound) in DUA/DXA; else the interior-point iterate, multipliers
// lam_u - lam_l.
template <typename T, int NX, int NU, class W>
MPCQP_IL void emit(const Args<T>& a, int b, const W& at, bool polished, int code, int it) {
  using L = Layout<NX, NU>;
  const int N = a.N, nx = a.nx, nu = a.nu;
  const int fu = polished ? L::DU : L::U, fx = polished ? L::DX : L::X;
  for (int k = 0; k < N; ++k) {
    for (int j = 0; j < nu; ++j) a.z[(int64_t)b * N * nu + (int64_t)k * nu + j] = (T)at(k, fu + j);
    if (a.lam_u)
      for (int j = 0; j < nu; ++j)
        a.lam_u[(int64_t)b * N * nu + (int64_t)k * nu + j] =
            (T)(polished ? at(k, L::DUA + j) : at(k, L::LU + j) - at(k, L::LL + j));
    if (a.X)
      for (int i = 0; i < nx; ++i)
        a.X[(int64_t)b * N * nx + (int64_t)k * nx + i] = (T)at(k, fx + i);
    if (a.pi)
      for (int i = 0; i < nx; ++i)
        a.pi[(int64_t)b * N * nx + (int64_t)k * nx + i] = (T)at(k, (polished ? L::DPI : L::PI) + i);
    if (a.y)
      for (int i = 0; i < nx; ++i)
        a.y[(int64_t)b * N * nx + (int64_t)k * nx + i] =
            (T)(polished ? at(k, L::DXA + i)
                         : at(k, L::LU + NU + i) - at(k, L::LL + NU + i));
  }
  a.status[b] = code | ((it & 0xFFFF) << 8) | (polished ? (1 << 24) : 0);
}

// One instance; its workspace rows start at W, LD instances interleaved: a
// block of the global workspace (LD = 64, one block per wave) or a slice of
// LDS.
template <typename T, int NX, int NU, int LD>
MPCQP_IL void solve_lane(const Args<T>& a, int b, double* W) {
  using L = Layout<NX, NU>;
  constexpr int NB = L::NB;
  const int N = a.N, nx = a.nx, nu = a.nu;
  const Ws<L::F, LD> at{W};
  if (a.skip && (a.skip[b] & a.skip_mask)) return;

  double x0[NX];
  for (int i = 0; i < NX; ++i) x0[i] = i < nx ? (double)a.x0[(int64_t)b * a.sX0 + i] : 0.0;

  // ---------------------------------------------------------------- start
  // copy the stage data (fp64, padded), inputs strictly inside their box,
  // states rolled out and pushed inside theirs, pi = 0, duals = 1
  int mcount = 0;
  {
    double x[NX];
    for (int i = 0; i < NX; ++i) x[i] = x0[i];
    for (int k = 0; k < N; ++k) {
      const T* Ak = a.A + (int64_t)b * a.sA + (a.tv ? (int64_t)k * nx * nx : 0);
      const T* Bk = a.B + (int64_t)b * a.sB + (a.tv ? (int64_t)k * nx * nu : 0);
      const T* ck = a.c ? a.c + (int64_t)b * a.sC + (int64_t)k * nx : nullptr;
      double lo[NB], hi[NB], u[NU], xn[NX];
      load_bounds<T, NX, NU>(a, b, k, lo, hi);
      for (int j = 0; j < NB; ++j) {
        at(k, L::LO + j) = lo[j];
        at(k, L::HI + j) = hi[j];
      }
      // stage cost: x_{k+1} (Q or Qf, H2xx_{k+1}, q2x_{k+1}); u_k (R, H2uu_k,
      // q2u_k); the x_k-u_k coupling H2xu_k
      const bool term = (k == N - 1);
      for (int i = 0; i < NX; ++i) {
        for (int j = 0; j <= i; ++j)
          at(k, L::WXX + pk(i, j)) = wq(a, b, term, i, j) + h2xx(a, b, k + 1, i, j);
        for (int r = 0; r < NU; ++r) at(k, L::WXU + i * NU + r) = h2xu(a, b, k, i, r);
        at(k, L::QX + i) = q2x(a, b, k + 1, i);
      }
      for (int r = 0; r < NU; ++r) {
        for (int q = 0; q <= r; ++q) at(k, L::WUU + pk(r, q)) = wr(a, b, r, q) + h2uu(a, b, k, r, q);
        at(k, L::QU + r) = q2u(a, b, k, r);
      }
      for (int j = 0; j < NU; ++j) {
        const double u0 =
            (a.U0 && j < nu) ? (double)a.U0[(int64_t)b * a.sU0 + (int64_t)k * nu + j] : 0.0;
        u[j] = interior(u0, lo[j], hi[j]);
      }
      for (int i = 0; i < NX; ++i) {
        const double ci = (ck && i < nx) ? (double)ck[i] : 0.0;
        at(k, L::DC + i) = ci;
        double s = ci;
        for (int j = 0; j < NX; ++j) {
          const double aij = (i < nx && j < nx) ? (double)Ak[i * nx + j] : 0.0;
          at(k, L::DA + i * NX + j) = aij;
          s = fma(aij, x[j], s);
        }
        for (int j = 0; j < NU; ++j) {
          const double bij = (i < nx && j < nu) ? (double)Bk[i * nu + j] : 0.0;
          at(k, L::DB + i * NU + j) = bij;
          s = fma(bij, u[j], s);
        }
        xn[i] = interior(s, lo[NU + i], hi[NU + i]);
      }
      for (int j = 0; j < NU; ++j) at(k, L::U + j) = u[j];
      for (int i = 0; i < NX; ++i) {
        at(k, L::X + i) = xn[i];
        at(k, L::PI + i) = 0.0;
        x[i] = xn[i];
      }
      for (int j = 0; j < NB; ++j) {
        at(k, L::LL + j) = fin(lo[j]) ? 1.0 : 0.0;
        at(k, L::LU + j) = fin(hi[j]) ? 1.0 : 0.0;
        mcount += (fin(lo[j]) ? 1 : 0) + (fin(hi[j]) ? 1 : 0);
      }
    }
  }

  // every exit writes the outputs and returns from inside the loop
  double alpha = 0.0, sigmu = 0.0;  // step and sigma*mu of the last corrector
  double mu_pol = a.mu_polish;      // next polish attempt below this mu
  // inertia correction (only a non-convex H2 needs it): on a non-positive
  // pivot pass 1 runs again with a growing dreg; each iteration starts a third
  // below the last one that worked (0 once it falls below 1e-12).  It changes
  // the Newton direction, not the residuals, so the iterate still converges
  // to a KKT point of the QP.  Strict mode (an SQP's QP, whose caller can
  // damp the Hessian instead) gives up after a.strict corrections: a QP that
  // is non-convex only away from its active face needs a few while the
  // barrier terms of the active bounds grow; one that keeps needing them is
  // handed back to the caller.
  double dreg = 0.0, dlast = 0.0;
  int ncorr = 0;
  const int max_iter = a.max_iter;
  for (int it = 0;; ++it) {
    // ======================================== pass 1: backward factorisation
    double Ph[L::SX], ph[NX], gx1[NX];
    for (int q = 0; q < L::SX; ++q) Ph[q] = 0.0;
    for (int i = 0; i < NX; ++i) ph[i] = gx1[i] = 0.0;
    double rstat = 0.0, rdyn = 0.0, musum = 0.0;
    bool pd = true;
    for (int k = N - 1; k >= 0; --k) {
      double v[NB], ll[NB], lu[NB], pi[NX], lo[NB], hi[NB], xk[NX];
      for (int j = 0; j < NU; ++j) v[j] = at(k, L::U + j);
      for (int i = 0; i < NX; ++i) { v[NU + i] = at(k, L::X + i); pi[i] = at(k, L::PI + i); }
      for (int j = 0; j < NB; ++j) { ll[j] = at(k, L::LL + j); lu[j] = at(k, L::LU + j); }
      // x_k: the previous stage's state (its own pass applies the same step)
      for (int i = 0; i < NX; ++i) {
        xk[i] = k == 0 ? x0[i] : at(k - 1, L::X + i);
        if (alpha > 0.0 && k > 0) xk[i] += alpha * at(k - 1, L::DX + i);
      }
      ws_bounds<NX, NU>(at, k, lo, hi);
      if (alpha > 0.0) {  // apply the corrector step of the previous iteration
        for (int j = 0; j < NB; ++j) {
          const double dv = j < NU ? at(k, L::DU + j) : at(k, L::DX + j - NU);
          const double dva = j < NU ? at(k, L::DUA + j) : at(k, L::DXA + j - NU);
          if (fin(lo[j])) {
            const double sl = v[j] - lo[j];
            const double dla = -ll[j] * (1.0 + dva / sl);
            const double rc = sigmu - sl * ll[j] - dva * dla;
            ll[j] += alpha * ((rc - ll[j] * dv) / sl);
          }
          if (fin(hi[j])) {
            const double su = hi[j] - v[j];
            const double dua = -lu[j] * (1.0 - dva / su);
            const double rc = sigmu - su * lu[j] + dva * dua;
            lu[j] += alpha * ((rc + lu[j] * dv) / su);
          }
          v[j] += alpha * dv;
        }
        for (int i = 0; i < NX; ++i) pi[i] += alpha * at(k, L::DPI + i);
        for (int j = 0; j < NU; ++j) at(k, L::U + j) = v[j];
        for (int i = 0; i < NX; ++i) { at(k, L::X + i) = v[NU + i]; at(k, L::PI + i) = pi[i]; }
        for (int j = 0; j < NB; ++j) { at(k, L::LL + j) = ll[j]; at(k, L::LU + j) = lu[j]; }
      }
      double Am[NX][NX], Bm[NX][NU], e[NX];
      load_ab<NX, NU>(at, k, Am, Bm);
      // dynamics residual e_k = A x_k + B u_k + c_k - x_{k+1}
      for (int i = 0; i < NX; ++i) {
        double s = at(k, L::DC + i) - v[NU + i];
        for (int j = 0; j < NX; ++j) s = fma(Am[i][j], xk[j], s);
        for (int j = 0; j < NU; ++j) s = fma(Bm[i][j], v[j], s);
        e[i] = s;
        rdyn = fmax(rdyn, fabs(s));
      }
      // gradients without the bound duals
      double g[NB];
      stage_grad<NX, NU>(at, k, Bm, v, pi, xk, gx1, g);
      // stationarity residual, complementarity, Sigma
      double sig[NB];
      for (int j = 0; j < NB; ++j) {
        double sj = 0.0;
        double r = g[j];
        if (fin(lo[j])) {
          const double sl = v[j] - lo[j];
          sj += ll[j] / sl;
          musum += sl * ll[j];
          r -= ll[j];
        }
        if (fin(hi[j])) {
          const double su = hi[j] - v[j];
          sj += lu[j] / su;
          musum += su * lu[j];
          r += lu[j];
        }
        sig[j] = sj;
        rstat = fmax(rstat, fabs(r));
      }
      for (int j = 0; j < NB; ++j) at(k, L::GA + j) = g[j];
      double P[L::SX], p[NX], K[NU][NX], kk[NU], Gi[L::SU];
      const bool ok = riccati_stage<NX, NU>(at, k, Am, Bm, e, g, sig, Ph, ph, P, p, K, kk, Gi, dreg);
      pd = pd && ok;
      store_factor<NX, NU>(at, k, P, p, K, kk, Gi, e);
      next_gx1<NX, NU>(at, k, Am, pi, v, gx1);
    }
    const double mu = mcount ? musum / mcount : 0.0;
#ifdef MPCQP_IPM_TRACE  // host build of tools/ipm_host.cpp only
    printf("it %3d mu %.3e rstat %.3e rdyn %.3e pd %d dreg %.2e alpha %.3e\n", it, mu, rstat,
           rdyn, (int)pd, dreg, alpha);
#endif
    if (!fin(rstat) || !fin(rdyn) || !fin(mu)) {
      emit<T, NX, NU>(a, b, at, false, MPCQP_STATUS_NONFINITE, it);
      return;
    }
    if (!pd) {
      dreg = dreg > 0.0 ? 8.0 * dreg : (dlast > 0.0 ? dlast : 1e-4);
      if ((a.strict > 0 && ++ncorr > a.strict) || dreg > 1e12 || it >= max_iter) {
        emit<T, NX, NU>(a, b, at, false, MPCQP_STATUS_NOT_CONVEX, it);
        return;
      }
      alpha = 0.0;  // the pending step is applied already
      continue;
    }
    if (dreg > 0.0) {  // next iteration starts a third lower
      dlast = dreg;
      dreg = dreg / 3.0 > 1e-12 ? dreg / 3.0 : 0.0;
    }

    const bool conv = rstat <= a.tol && rdyn <= a.tol && mu <= a.tol_mu;
    if (mcount && mu_pol > 0.0 && mu <= mu_pol && rstat <= a.tol_polish && rdyn <= a.tol_polish) {
      if (polish<T, NX, NU>(a, b, at, x0)) {
        emit<T, NX, NU>(a, b, at, true, MPCQP_STATUS_OPTIMAL, it);
        return;
      }
      // wrong active-set guess: keep iterating, try again at a smaller mu;
      // the polish overwrote the factorisation, so pass 1 runs again
      mu_pol *= 1e-2;
      alpha = 0.0;
      if (conv || it >= max_iter) {
        emit<T, NX, NU>(a, b, at, false, conv ? MPCQP_STATUS_OPTIMAL : MPCQP_STATUS_MAXITER, it);
        return;
      }
      continue;
    }
    if (conv || it >= max_iter) {
      emit<T, NX, NU>(a, b, at, false, conv ? MPCQP_STATUS_OPTIMAL : MPCQP_STATUS_MAXITER, it);
      return;
    }

    // ========================================== pass 2: forward predictor
    double amax = 1.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
    forward_sweep<NX, NU>(at, N, [&](int k, const double (&du)[NU], const double (&dxn)[NX]) {
      for (int r = 0; r < NU; ++r) at(k, L::DUA + r) = du[r];
      for (int i = 0; i < NX; ++i) at(k, L::DXA + i) = dxn[i];
      double lo[NB], hi[NB];
      ws_bounds<NX, NU>(at, k, lo, hi);
      for (int j = 0; j < NB; ++j) {
        const double vj = j < NU ? at(k, L::U + j) : at(k, L::X + j - NU);
        const double dv = j < NU ? du[j] : dxn[j - NU];
        if (fin(lo[j])) {
          const double sl = vj - lo[j], l = at(k, L::LL + j);
          const double dl = -l * (1.0 + dv / sl);
          if (dv < 0.0) amax = fmin(amax, -sl / dv);
          if (dl < 0.0) amax = fmin(amax, -l / dl);
          c0 += sl * l;
          c1 += sl * dl + l * dv;
          c2 += dv * dl;
        }
        if (fin(hi[j])) {
          const double su = hi[j] - vj, l = at(k, L::LU + j);
          const double dl = -l * (1.0 - dv / su);
          if (dv > 0.0) amax = fmin(amax, su / dv);
          if (dl < 0.0) amax = fmin(amax, -l / dl);
          c0 += su * l;
          c1 += su * dl - l * dv;
          c2 -= dv * dl;
        }
      }
    });
    if (mcount) {
      const double mua = (c0 + amax * (c1 + amax * c2)) / mcount;
      const double r = fmax(0.0, fmin(1.0, mua / mu));
      sigmu = r * r * r * mu;
    } else {
      sigmu = 0.0;
    }

    // ================================ pass 3: backward corrector right side
    {
      double phc[NX];
      for (int i = 0; i < NX; ++i) phc[i] = 0.0;
      for (int k = N - 1; k >= 0; --k) {
        double lo[NB], hi[NB], g[NB];
        ws_bounds<NX, NU>(at, k, lo, hi);
        for (int j = 0; j < NB; ++j) {
          const double vj = j < NU ? at(k, L::U + j) : at(k, L::X + j - NU);
          const double dva = j < NU ? at(k, L::DUA + j) : at(k, L::DXA + j - NU);
          double s = at(k, L::GA + j);
          if (fin(lo[j])) {
            const double sl = vj - lo[j], l = at(k, L::LL + j);
            s += (-sigmu - dva * l * (1.0 + dva / sl)) / sl;
          }
          if (fin(hi[j])) {
            const double su = hi[j] - vj, l = at(k, L::LU + j);
            s += (sigmu - dva * l * (1.0 - dva / su)) / su;
          }
          g[j] = s;
        }
        double p[NX], Pe[NX];
        for (int i = 0; i < NX; ++i) p[i] = g[NU + i] + phc[i];
        for (int i = 0; i < NX; ++i) {
          double s = p[i];
          for (int j = 0; j < NX; ++j) s = fma(at(k, L::PP + pk(i, j)), at(k, L::E + j), s);
          Pe[i] = s;
        }
        double h[NU];
        for (int r = 0; r < NU; ++r) {
          double s = g[r];
          for (int i = 0; i < NX; ++i) s = fma(at(k, L::DB + i * NU + r), Pe[i], s);
          h[r] = s;
        }
        for (int r = 0; r < NU; ++r) {
          double s = 0.0;
          for (int q = 0; q < NU; ++q) s = fma(at(k, L::GI + pk(r, q)), h[q], s);
          at(k, L::KV + r) = -s;
        }
        // ph = A'Pe + Hx'kk = A'Pe + K'h
        for (int i = 0; i < NX; ++i) {
          double s = 0.0;
          for (int q = 0; q < NX; ++q) s = fma(at(k, L::DA + q * NX + i), Pe[q], s);
          for (int r = 0; r < NU; ++r) s = fma(at(k, L::KM + r * NX + i), h[r], s);
          phc[i] = s;
        }
        for (int i = 0; i < NX; ++i) at(k, L::PV + i) = p[i];
      }
    }

    // ========================================== pass 4: forward corrector
    amax = 1.0;
    forward_sweep<NX, NU>(at, N, [&](int k, const double (&du)[NU], const double (&dxn)[NX]) {
      // dpi_{k+1} = P_{k+1} dx_{k+1} + p_{k+1}
      for (int i = 0; i < NX; ++i) {
        double s = at(k, L::PV + i);
        for (int j = 0; j < NX; ++j) s = fma(at(k, L::PP + pk(i, j)), dxn[j], s);
        at(k, L::DPI + i) = s;
      }
      for (int r = 0; r < NU; ++r) at(k, L::DU + r) = du[r];
      for (int i = 0; i < NX; ++i) at(k, L::DX + i) = dxn[i];
      double lo[NB], hi[NB];
      ws_bounds<NX, NU>(at, k, lo, hi);
      for (int j = 0; j < NB; ++j) {
        const double vj = j < NU ? at(k, L::U + j) : at(k, L::X + j - NU);
        const double dv = j < NU ? du[j] : dxn[j - NU];
        const double dva = j < NU ? at(k, L::DUA + j) : at(k, L::DXA + j - NU);
        if (fin(lo[j])) {
          const double sl = vj - lo[j], l = at(k, L::LL + j);
          const double dla = -l * (1.0 + dva / sl);
          const double dl = (sigmu - sl * l - dva * dla - l * dv) / sl;
          if (dv < 0.0) amax = fmin(amax, -sl / dv);
          if (dl < 0.0) amax = fmin(amax, -l / dl);
        }
        if (fin(hi[j])) {
          const double su = hi[j] - vj, l = at(k, L::LU + j);
          const double dua = -l * (1.0 - dva / su);
          const double dl = (sigmu - su * l + dva * dua + l * dv) / su;
          if (dv > 0.0) amax = fmin(amax, su / dv);
          if (dl < 0.0) amax = fmin(amax, -l / dl);
        }
      }
    });
    // fraction to the boundary.  Fixed, not tightened towards 1 as mu -> 0:
    // the slacks are differences v - lo, and a slack driven below the rounding
    // of v would turn Sigma = lam / s into inf
    alpha = fmin(1.0, 0.995 * amax);
  }
}

// Global workspace: blocks of 64 instances, [block][stage][field][64].
template <typename T, int NX, int NU>
MPCQP_IL void solve_lane(const Args<T>& a, int b) {
  constexpr int F = Layout<NX, NU>::F;
  solve_lane<T, NX, NU, 64>(a, b, a.ws + (int64_t)(b / 64) * a.N * F * 64 + (b % 64));
}

}  // namespace ipm
}  // namespace mpcqp
