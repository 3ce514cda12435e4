// ipm_quad.hpp -- the interior-point MPC step of ipm_lane.hpp run by FOUR
// lanes per instance (one DPP quad): lane i of the quad owns state row i of
// every stage quantity (x_{k+1}, pi_{k+1}, the rows of P_{k+1}, A_k, B_k, the
// state bound duals) and lanes 0, 1 also own the inputs u_k.  The O(nx^3)
// products of the Riccati factorisation are split by rows; rows travel to the
// other lanes by quad_perm DPP broadcasts; the small replicated pieces (the
// 2 x 2 input block, its inverse, the gains) are computed by every lane.  The
// per-instance chain of dependent instructions is ~10x shorter than one lane
// per instance, and a wave holds 16 instances instead of 1-4.
//
// Same algorithm, workspace layout (Layout<4, 2>), arguments and outputs as
// ipm_lane.hpp (solve_lane); the workspace is a slice of LDS (LD instances
// interleaved), so a value one lane stores is read by the others in program
// order.  Every decision (step length, convergence, polish, inertia) is made
// on quad-reduced values, so the four lanes of an instance take the same
// branches.  Device only (DPP).
#pragma once

#include "sym2d.hpp"

namespace mpcqp {
namespace ipmq {

using ipm::Args;
using ipm::fin;
using ipm::interior;
using ipm::kInf;
using ipm::Layout;
using ipm::pk;
using ipm::Ws;

#define MPCQP_QD __device__ inline __attribute__((always_inline))

template <int Q>
MPCQP_QD double qb(double v) {  // value of quad lane Q
  return dpp<Q | (Q << 2) | (Q << 4) | (Q << 6)>(v);
}
MPCQP_QD double qsum(double v) {
  v += dpp<0xB1>(v);
  return v + dpp<0x4E>(v);
}
MPCQP_QD double qmax(double v) {
  v = fmax(v, dpp<0xB1>(v));
  return fmax(v, dpp<0x4E>(v));
}
MPCQP_QD double qmin(double v) {
  v = fmin(v, dpp<0xB1>(v));
  return fmin(v, dpp<0x4E>(v));
}
MPCQP_QD void bcast4(double v, double (&o)[4]) {
  o[0] = qb<0>(v);
  o[1] = qb<1>(v);
  o[2] = qb<2>(v);
  o[3] = qb<3>(v);
}
MPCQP_QD double sel4(const double (&v)[4], int i) {
  return i == 0 ? v[0] : (i == 1 ? v[1] : (i == 2 ? v[2] : v[3]));
}
MPCQP_QD double sel2(const double (&v)[2], int i) { return i == 0 ? v[0] : v[1]; }
// M[i][j] for a runtime row i
MPCQP_QD double sel4Row(const double (&M)[4][4], int i, int j) {
  return i == 0 ? M[0][j] : (i == 1 ? M[1][j] : (i == 2 ? M[2][j] : M[3][j]));
}
MPCQP_QD double sel4RowB(const double (&M)[4][2], int i, int r) {
  return i == 0 ? M[0][r] : (i == 1 ? M[1][r] : (i == 2 ? M[2][r] : M[3][r]));
}

constexpr int NX = 4, NU = 2;
using L = Layout<NX, NU>;

// Workspace accessor of one quad: field f of stage k, and the lane-relative
// fields with the lane's row offset folded into a per-lane base pointer, so
// every access is a base + compile-time immediate (a runtime row index in
// the field offset costs address arithmetic on every access):
//   r(k, f) = f + i,  ra(k, f) = f + i*NX,  rb(k, f) = f + i*NU,
//   p(k, f, j) = f + pk(i, j)  (row i of a packed symmetric block).
template <int LD>
struct WsQ {
  double* W;
  double* Wi;
  double* Wa;
  double* Wb;
  double* Wp[4];
  MPCQP_QD WsQ(double* w, int i)
      : W(w), Wi(w + i * LD), Wa(w + i * NX * LD), Wb(w + i * NU * LD),
        Wp{w + pk(i, 0) * LD, w + pk(i, 1) * LD, w + pk(i, 2) * LD, w + pk(i, 3) * LD} {}
  MPCQP_QD double& operator()(int k, int f) const { return W[(k * L::F + f) * LD]; }
  MPCQP_QD double& r(int k, int f) const { return Wi[(k * L::F + f) * LD]; }
  MPCQP_QD double& ra(int k, int f) const { return Wa[(k * L::F + f) * LD]; }
  MPCQP_QD double& rb(int k, int f) const { return Wb[(k * L::F + f) * LD]; }
  MPCQP_QD double& p(int k, int f, int j) const { return Wp[j][(k * L::F + f) * LD]; }
};

// The stage data every lane reads several times per stage, in registers.
struct StageQ {
  double A[4][4], B[4][2], WXU[4][2], WUU[3];
  template <class W>
  MPCQP_QD void load(const W& at, int k) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) A[q][j] = at(k, L::DA + q * NX + j);
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        B[q][r] = at(k, L::DB + q * NU + r);
        WXU[q][r] = at(k, L::WXU + q * NU + r);
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) WUU[c] = at(k, L::WUU + c);
  }
};

// 2 x 2 SPD inverse, packed (G[0] = (0,0), G[1] = (1,0), G[2] = (1,1)).
MPCQP_QD bool inv2(const double (&G)[3], double (&Gi)[3]) {
  const double det = G[0] * G[2] - G[1] * G[1];
  const bool ok = (G[0] > 0.0) && (det > 0.0);
  const double r = 1.0 / det;
  Gi[0] = ok ? G[2] * r : 0.0;
  Gi[1] = ok ? -G[1] * r : 0.0;
  Gi[2] = ok ? G[0] * r : 0.0;
  return ok;
}

// One backward Riccati step, lane i: the row-i parts of P, p, Pe, the
// replicated input block.  In: Ph (row i of the cost-to-go of x_{k+1} from the
// later stages), ph_i, e_i, gx (the state gradient g_x[i]), gu[2] (input
// gradients, replicated), sx (Sigma of state comp i), su2[2] (Sigma of the
// inputs, replicated).  Out: P row i, p_i, K (2 x 4, replicated), kk, Gi,
// Kc = column i of K, and Ph, ph overwritten with the cost-to-go of x_k.
template <class W>
MPCQP_QD bool riccati_q(const W& at, const StageQ& S, int k, int i, double (&Ph)[4], double& ph,
                        double e,
                        double gx, const double (&gu)[2], double sx, const double (&su2)[2],
                        double dreg, double (&P)[4], double& p, double (&K)[2][4],
                        double (&kk)[2], double (&Gi)[3], double (&Kc)[2]) {
  // P_{k+1} row i = Q' + H2xx_{k+1} + Sigma_x + Ph,  p = g_x + ph
#pragma unroll
  for (int j = 0; j < 4; ++j)
    P[j] = at.p(k, L::WXX, j) + Ph[j] + (i == j ? sx + dreg : 0.0);
  p = gx + ph;
  double ea[4];
  bcast4(e, ea);
  double Pe = p;
#pragma unroll
  for (int j = 0; j < 4; ++j) Pe = fma(P[j], ea[j], Pe);
  // rows of P B and P A, then to every lane
  double PB[2], PA[4];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fma(P[q], S.B[q][c], s);
    PB[c] = s;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fma(P[q], S.A[q][j], s);
    PA[j] = s;
  }
  double PBa[4][2], PAa[4][4], Pea[4];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    PBa[0][c] = qb<0>(PB[c]);
    PBa[1][c] = qb<1>(PB[c]);
    PBa[2][c] = qb<2>(PB[c]);
    PBa[3][c] = qb<3>(PB[c]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    PAa[0][j] = qb<0>(PA[j]);
    PAa[1][j] = qb<1>(PA[j]);
    PAa[2][j] = qb<2>(PA[j]);
    PAa[3][j] = qb<3>(PA[j]);
  }
  bcast4(Pe, Pea);
  // replicated: G = R + H2uu + Sigma_u + B'PB, h = g_u + B'Pe
  double G[3], h[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int c = 0; c <= r; ++c) {
      double s = S.WUU[pk(r, c)] + (r == c ? su2[r] + dreg : 0.0);
#pragma unroll
      for (int q = 0; q < 4; ++q) s = fma(S.B[q][r], PBa[q][c], s);
      G[pk(r, c)] = s;
    }
    double s = gu[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fma(S.B[q][r], Pea[q], s);
    h[r] = s;
  }
  const bool ok = inv2(G, Gi);
#pragma unroll
  for (int r = 0; r < 2; ++r) kk[r] = -(Gi[pk(r, 0)] * h[0] + Gi[pk(r, 1)] * h[1]);
  // column i of Hx = H2xu' + B'PA from the lane's own column of A:
  // (B'PA)_ri = (A'PB)_ir (P symmetric); the gains K = -G^-1 Hx by columns
  // (Kc, lane i), then to every lane -- replicating Hx and K on the four lanes
  // cost 48 VALU per stage against 16 DPP moves
  double Ai[4], Hxi[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) Ai[q] = at.r(k, L::DA + q * NX);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    double t = at.rb(k, L::WXU + r);
#pragma unroll
    for (int q = 0; q < 4; ++q) t = fma(Ai[q], PBa[q][r], t);
    Hxi[r] = t;
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    Kc[r] = -(Gi[pk(r, 0)] * Hxi[0] + Gi[pk(r, 1)] * Hxi[1]);
    bcast4(Kc[r], K[r]);
  }
  // row i of the cost-to-go of x_k: A'PA + Hx'K,  ph_i = (A'Pe)_i + (Hx'kk)_i
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fma(Ai[q], PAa[q][j], s);
    Ph[j] = fma(Hxi[1], K[1][j], fma(Hxi[0], K[0][j], s));
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s = fma(Ai[q], Pea[q], s);
  ph = fma(Hxi[1], kk[1], fma(Hxi[0], kk[0], s));
  return ok;
}

// Store the factor data of stage k (lane i: its rows / columns).
template <class W>
MPCQP_QD void store_factor_q(const W& at, int k, int i, const double (&P)[4], double p,
                             const double (&Kc)[2], const double (&kk)[2], const double (&Gi)[3],
                             double e) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j <= i) at.p(k, L::PP, j) = P[j];
#pragma unroll
  for (int r = 0; r < 2; ++r) at.r(k, L::KM + r * NX) = Kc[r];
  at.r(k, L::E) = e;
  at.r(k, L::PV) = p;
  if (i < 2) at.r(k, L::KV) = sel2(kk, i);
  if (i == 0) {
    at(k, L::GI + 0) = Gi[0];
    at(k, L::GI + 1) = Gi[1];
    at(k, L::GI + 2) = Gi[2];
  }
}

// Gradients of stage k without the bound duals, lane i: gx = g_x[i]
// (x_{k+1} row i) and gu (both inputs, replicated).  xa = x_k, x1a =
// x_{k+1}, pia = pi_{k+1}, ua = u_k (all replicated), gx1 = the later
// stage's A'pi + H2xu u, row i.
template <class W>
MPCQP_QD void grad_q(const W& at, const StageQ& S, int k, int i, const double (&xa)[4],
                     const double (&x1a)[4],
                     const double (&pia)[4], const double (&ua)[2], double pii, double gx1,
                     double& gx, double (&gu)[2]) {
  double s = gx1 - pii + at.r(k, L::QX);
#pragma unroll
  for (int q = 0; q < 4; ++q) s = fma(at.p(k, L::WXX, q), x1a[q], s);
  gx = s;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    double t = at(k, L::QU + r);
#pragma unroll
    for (int q = 0; q < 2; ++q) t = fma(S.WUU[pk(r, q)], ua[q], t);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      t = fma(S.WXU[q][r], xa[q], t);
      t = fma(S.B[q][r], pia[q], t);
    }
    gu[r] = t;
  }
}

// gx1 for the stage before k, row i: (A_k'pi_{k+1})_i + (H2xu_k u_k)_i
template <class W>
MPCQP_QD double next_gx1_q(const W& at, const StageQ& S, int k, int i, const double (&pia)[4],
                           const double (&ua)[2]) {
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s = fma(at.r(k, L::DA + q * NX), pia[q], s);
#pragma unroll
  for (int r = 0; r < 2; ++r) s = fma(at.rb(k, L::WXU + r), ua[r], s);
  return s;
}

// dynamics residual row i: c_i + (A x_k)_i + (B u_k)_i - x_{k+1,i}
template <class W>
MPCQP_QD double resid_q(const W& at, const StageQ& S, int k, int i, const double (&xa)[4],
                        const double (&ua)[2],
                        double x1i) {
  double s = at.r(k, L::DC) - x1i;
#pragma unroll
  for (int j = 0; j < 4; ++j) s = fma(at.ra(k, L::DA + j), xa[j], s);
#pragma unroll
  for (int r = 0; r < 2; ++r) s = fma(at.rb(k, L::DB + r), ua[r], s);
  return s;
}

// Forward sweep of the Newton direction from the stored factors: du = K dx +
// kk (replicated), dx+_i = (A dx)_i + (B du)_i + e_i; body(k, du, dxn_i,
// dxn_all).
template <class W, class Body>
MPCQP_QD void forward_q(const W& at, int N, int i, Body&& body) {
  double dx[4] = {0.0, 0.0, 0.0, 0.0};
  for (int k = 0; k < N; ++k) {
    double du[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      double s = at(k, L::KV + r);
#pragma unroll
      for (int j = 0; j < 4; ++j) s = fma(at(k, L::KM + r * NX + j), dx[j], s);
      du[r] = s;
    }
    double s = at.r(k, L::E);
#pragma unroll
    for (int j = 0; j < 4; ++j) s = fma(at.ra(k, L::DA + j), dx[j], s);
#pragma unroll
    for (int r = 0; r < 2; ++r) s = fma(at.rb(k, L::DB + r), du[r], s);
    double dxa[4];
    bcast4(s, dxa);
    body(k, du, s, dxa);
#pragma unroll
    for (int j = 0; j < 4; ++j) dx[j] = dxa[j];
  }
}

// ------------------------------------------------------------- polish
// The polish of ipm_lane.hpp (see there), lane i owning state comp i and
// (i < 2) input comp i.
// warm: the active set is the one GA already holds (the previous QP's polish,
// solve_quad's warm start) and the multipliers start at 0; otherwise it is
// guessed from the interior-point iterate (lambda > slack) with its duals.
template <typename T, class W>
MPCQP_QD bool polish_q(const Args<T>& a, const W& at, int i, double x0i, bool warm = false) {
  const int N = a.N;
  const bool ou = i < NU;
  for (int k = 0; k < N; ++k) {
    // state comp i, then input comp i
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      if (part == 1 && !ou) continue;
      const int j = part == 0 ? NU + i : i;
      const double vj = part == 0 ? at.r(k, L::X) : at.r(k, L::U);
      double y = 0.0;
      if (!warm) {
        const double lo = at(k, L::LO + j), hi = at(k, L::HI + j);
        const double l = at(k, L::LL + j), u = at(k, L::LU + j);
        const double rl = fin(lo) ? l / (vj - lo) : 0.0;
        const double ru = fin(hi) ? u / (hi - vj) : 0.0;
        const double act = (ru > 1.0 && ru >= rl) ? 1.0 : ((rl > 1.0) ? -1.0 : 0.0);
        at(k, L::GA + j) = act;
        y = act > 0.0 ? u : (act < 0.0 ? -l : 0.0);
      }
      if (part == 1) { at.r(k, L::DU) = vj; at.r(k, L::DUA) = y; }
      else { at.r(k, L::DX) = vj; at.r(k, L::DXA) = y; }
    }
    at.r(k, L::DPI) = at.r(k, L::PI);
  }
  constexpr int kSteps = 4, kRounds = 4;
#ifdef MPCQP_POLISH_EARLY
  constexpr int kPolishEarly = MPCQP_POLISH_EARLY;
#else
  constexpr int kPolishEarly = kSteps;  // (off: every round runs all four steps)
#endif
#ifdef MPCQP_WARM_ROUNDS
  // a warm polish whose active set needs corrections hands over to the
  // interior point after this many rounds (timing builds)
  const int rounds = warm ? MPCQP_WARM_ROUNDS : kRounds;
#else
  const int rounds = kRounds;
#endif
  for (int round = 0; round < rounds; ++round) {
    bool good = true, changed = false;
    for (int step = 0; step < kSteps; ++step) {
      const double rho = step == 0 ? 1e8 : (step == 1 ? 1e6 : 1e4);
      double Ph[4] = {0.0, 0.0, 0.0, 0.0}, ph = 0.0, gx1 = 0.0;
      for (int k = N - 1; k >= 0; --k) {
        const double xi = at.r(k, L::DX), pii = at.r(k, L::DPI);
        const double ui = ou ? at.r(k, L::DU) : 0.0;
        const double xki = k == 0 ? x0i : at.r(k - 1, L::DX);
        double xa[4], x1a[4], pia[4], ua[2];
        bcast4(xki, xa);
        bcast4(xi, x1a);
        bcast4(pii, pia);
        ua[0] = qb<0>(ui);
        ua[1] = qb<1>(ui);
        StageQ S;
        S.load(at, k);
        const double e = resid_q(at, S, k, i, xa, ua, xi);
        double gx, gu[2];
        grad_q(at, S, k, i, xa, x1a, pia, ua, pii, gx1, gx, gu);
        // the penalty of the active components: state comp i, inputs (owners)
        double sx = 0.0, sui = 0.0;
        {
          const int j = NU + i;
          const double act = at(k, L::GA + j);
          if (act != 0.0) {
            const double bnd = act > 0.0 ? at(k, L::HI + j) : at(k, L::LO + j);
            sx = rho;
            gx += at.r(k, L::DXA) + rho * (xi - bnd);
          }
        }
        double gum = 0.0;
        if (ou) {
          const double act = at.r(k, L::GA);
          if (act != 0.0) {
            const double bnd = act > 0.0 ? at.r(k, L::HI) : at.r(k, L::LO);
            sui = rho;
            gum = at.r(k, L::DUA) + rho * (ui - bnd);
          }
        }
        double su2[2] = {qb<0>(sui), qb<1>(sui)};
        gu[0] += qb<0>(gum);
        gu[1] += qb<1>(gum);
        double P[4], p, K[2][4], kk[2], Gi[3], Kc[2];
        good = riccati_q(at, S, k, i, Ph, ph, e, gx, gu, sx, su2, 0.0, P, p, K, kk, Gi, Kc) && good;
        store_factor_q(at, k, i, P, p, Kc, kk, Gi, e);
        gx1 = next_gx1_q(at, S, k, i, pia, ua);
      }
      const bool last = step == kSteps - 1;
      // early exit (MPCQP_POLISH_EARLY builds / kPolishEarly): from step
      // kPolishEarly on, a step whose result already passes the last step's
      // test (active components on their bound to 1e-9, multipliers of the
      // right sign, no inactive component violated) ends the polish
      const bool probe = !last && step >= kPolishEarly;
      bool pass = true;
      forward_q(at, N, i, [&](int k, const double (&du)[2], double dxn, const double (&dxa)[4]) {
        double s = at.r(k, L::PV);
#pragma unroll
        for (int j = 0; j < 4; ++j) s = fma(at.p(k, L::PP, j), dxa[j], s);
        at.r(k, L::DPI) += s;
#pragma unroll
        for (int part = 0; part < 2; ++part) {
          if (part == 1 && !ou) continue;
          const int j = part == 0 ? NU + i : i;
          double& vr = part == 0 ? at.r(k, L::DX) : at.r(k, L::DU);
          const double vj = vr + (part == 0 ? dxn : sel2(du, i));
          vr = vj;
          const double lo = at(k, L::LO + j), hi = at(k, L::HI + j);
          const double act = at(k, L::GA + j);
          if (act != 0.0) {
            double& yr = part == 0 ? at.r(k, L::DXA) : at.r(k, L::DUA);
            const double bnd = act > 0.0 ? hi : lo;
            const double y = yr + rho * (vj - bnd);
            yr = y;
            if (probe)
              pass = pass && fabs(vj - bnd) <= 1e-9 * (1.0 + fabs(bnd)) &&
                     !(act > 0.0 ? y < -1e-9 * (1.0 + fabs(y)) : y > 1e-9 * (1.0 + fabs(y)));
            if (last) {
              good = good && fabs(vj - bnd) <= 1e-9 * (1.0 + fabs(bnd));
              if (act > 0.0 ? y < -1e-9 * (1.0 + fabs(y)) : y > 1e-9 * (1.0 + fabs(y))) {
                at(k, L::GA + j) = 0.0;
                yr = 0.0;
                changed = true;
              }
            }
          } else if (last || probe) {
            const double jl = (lo - vj) / (1.0 + fabs(lo));
            const double jh = (vj - hi) / (1.0 + fabs(hi));
            if (jl > 1e-9 || jh > 1e-9) {
              if (last) {
                at(k, L::GA + j) = jl > jh ? -1.0 : 1.0;
                changed = true;
              }
              pass = false;
            }
          }
        }
      });
      if (probe && good && qmin(pass ? 1.0 : 0.0) > 0.5) return true;
    }
    // quad-uniform verdicts
    good = qmin(good ? 1.0 : 0.0) > 0.5;
    changed = qmax(changed ? 1.0 : 0.0) > 0.5;
    if (good && !changed) return true;
    if (!good) return false;
  }
  return false;
}

template <typename T, class W>
MPCQP_QD void emit_q(const Args<T>& a, int b, const W& at, int i, bool polished, int code,
                     int it) {
  const int N = a.N, nx = a.nx, nu = a.nu;
  for (int k = 0; k < N; ++k) {
    if (i < nu) {
      a.z[(int64_t)b * N * nu + (int64_t)k * nu + i] = (T)at.r(k, polished ? L::DU : L::U);
      if (a.lam_u)
        a.lam_u[(int64_t)b * N * nu + (int64_t)k * nu + i] =
            (T)(polished ? at.r(k, L::DUA) : at.r(k, L::LU) - at.r(k, L::LL));
    }
    if (i < nx) {
      if (a.X)
        a.X[(int64_t)b * N * nx + (int64_t)k * nx + i] = (T)at.r(k, polished ? L::DX : L::X);
      if (a.pi)
        a.pi[(int64_t)b * N * nx + (int64_t)k * nx + i] =
            (T)at.r(k, polished ? L::DPI : L::PI);
      if (a.y)
        a.y[(int64_t)b * N * nx + (int64_t)k * nx + i] =
            (T)(polished ? at.r(k, L::DXA) : at.r(k, L::LU + NU) - at.r(k, L::LL + NU));
    }
  }
  if (i == 0) a.status[b] = code | ((it & 0xFFFF) << 8) | (polished ? (1 << 24) : 0);
}

// One instance on the four lanes of a quad (i = lane & 3), workspace slice W
// (LD instances interleaved).  Requires nx <= 4, nu <= 2.
// Stage k's data into the workspace, lane i's rows: the bounds, A, B, c, the
// x_{k+1} cost with H2xx, the coupling H2xu, R + H2uu and q2 (the first half
// of solve_quad's start; the one-launch SQP runs it one quad per stage).
template <typename T, class W>
MPCQP_QD void stage_in_q(const Args<T>& a, int b, const W& at, int i, int k) {
  const int nx = a.nx, nu = a.nu;
  const bool ou = i < NU;
  const T* Ak = a.A + (int64_t)b * a.sA + (a.tv ? (int64_t)k * nx * nx : 0);
  const T* Bk = a.B + (int64_t)b * a.sB + (a.tv ? (int64_t)k * nx * nu : 0);
  const T* ck = a.c ? a.c + (int64_t)b * a.sC + (int64_t)k * nx : nullptr;
  // bounds of the lane's components (ipm::load_bounds order: u then x)
  double lo[L::NB], hi[L::NB];
  ipm::load_bounds<T, NX, NU>(a, b, k, lo, hi);
  at.r(k, L::LO + NU) = sel4({lo[2], lo[3], lo[4], lo[5]}, i);
  at.r(k, L::HI + NU) = sel4({hi[2], hi[3], hi[4], hi[5]}, i);
  if (ou) {
    at.r(k, L::LO) = sel2({lo[0], lo[1]}, i);
    at.r(k, L::HI) = sel2({hi[0], hi[1]}, i);
  }
  // stage data, row i (A, B, c, the x_{k+1} cost, the coupling H2xu)
  const bool term = (k == a.N - 1);
  const double ci = (ck && i < nx) ? (double)ck[i] : 0.0;
  at.r(k, L::DC) = ci;
#pragma unroll
  for (int j = 0; j < NX; ++j)
    at.ra(k, L::DA + j) = (i < nx && j < nx) ? (double)Ak[i * nx + j] : 0.0;
#pragma unroll
  for (int r = 0; r < NU; ++r) {
    at.rb(k, L::DB + r) = (i < nx && r < nu) ? (double)Bk[i * nu + r] : 0.0;
    at.rb(k, L::WXU + r) = ipm::h2xu(a, b, k, i, r);
  }
#pragma unroll
  for (int j = 0; j < NX; ++j)
    if (j <= i)
      at.p(k, L::WXX, j) = ipm::wq(a, b, term, i, j) + ipm::h2xx(a, b, k + 1, i, j);
  at.r(k, L::QX) = ipm::q2x(a, b, k + 1, i);
  if (ou) {
#pragma unroll
    for (int q = 0; q < NU; ++q)
      if (q <= i) at(k, L::WUU + pk(i, q)) = ipm::wr(a, b, i, q) + ipm::h2uu(a, b, k, i, q);
    at.r(k, L::QU) = ipm::q2u(a, b, k, i);
  }
}

// warm (the one-launch SQP, sqp_solve.hip): the previous QP of this
// instance ended polished and its active set is still in W's GA fields; the
// QP is first polished on that active set from the start point, and the
// interior point runs only if that is not a certified vertex.  Returns true
// when the QP ended polished (its active set is then in GA for the next one).
// MPCQP_IPM_PASSCLK (timing builds, tools/sqp_latency.py): s_memrealtime
// ticks accumulated into pclk[0..7]: the four passes, the polish, factorisations
// that failed the inertia test (solve_wave; solve_quad: + the loop head), the
// start, the warm polish (solve_wave)
#ifdef MPCQP_IPM_PASSCLK
#define MPCQP_PCLK(i) do { if (pclk) { const uint64_t _t = __builtin_amdgcn_s_memrealtime(); pclk[i] += _t - pclk_t; pclk_t = _t; } } while (0)
#else
#define MPCQP_PCLK(i) do { } while (0)
#endif
template <typename T, int LD>
MPCQP_QD bool solve_quad(const Args<T>& a, int b, double* W, bool warm = false,
                         uint64_t* pclk = nullptr, bool staged = false) {
#ifdef MPCQP_IPM_PASSCLK
  uint64_t pclk_t = __builtin_amdgcn_s_memrealtime();
#endif
  const int i = (int)(threadIdx.x & 3);
  const WsQ<LD> at(W, i);
  const bool ou = i < NU;
  const int N = a.N, nx = a.nx, nu = a.nu;
  if (a.skip && (a.skip[b] & a.skip_mask)) return false;
  const double x0i = i < nx ? (double)a.x0[(int64_t)b * a.sX0 + i] : 0.0;

  // ---------------------------------------------------------------- start
  double mc = 0.0;  // finite bounds owned by this lane
  {
    double xi = x0i;
    for (int k = 0; k < N; ++k) {
      if (!staged) stage_in_q(a, b, at, i, k);
      const double ci = at.r(k, L::DC);
      // start point: inputs inside their box, states rolled out and pushed
      // inside theirs, pi = 0, duals = 1
      double ui = 0.0;
      if (ou) {
        const double u0 =
            (a.U0 && i < nu) ? (double)a.U0[(int64_t)b * a.sU0 + (int64_t)k * nu + i] : 0.0;
        ui = interior(u0, at.r(k, L::LO), at.r(k, L::HI));
        at.r(k, L::U) = ui;
      }
      double xa[4], ua[2];
      bcast4(xi, xa);
      ua[0] = qb<0>(ui);
      ua[1] = qb<1>(ui);
      double s = ci;
#pragma unroll
      for (int j = 0; j < NX; ++j) s = fma(at.ra(k, L::DA + j), xa[j], s);
#pragma unroll
      for (int r = 0; r < NU; ++r) s = fma(at.rb(k, L::DB + r), ua[r], s);
      const double lox = at.r(k, L::LO + NU), hix = at.r(k, L::HI + NU);
      xi = interior(s, lox, hix);
      at.r(k, L::X) = xi;
      at.r(k, L::PI) = 0.0;
      at.r(k, L::LL + NU) = fin(lox) ? 1.0 : 0.0;
      at.r(k, L::LU + NU) = fin(hix) ? 1.0 : 0.0;
      mc += (fin(lox) ? 1.0 : 0.0) + (fin(hix) ? 1.0 : 0.0);
      if (ou) {
        const double lou = at.r(k, L::LO), hiu = at.r(k, L::HI);
        at.r(k, L::LL) = fin(lou) ? 1.0 : 0.0;
        at.r(k, L::LU) = fin(hiu) ? 1.0 : 0.0;
        mc += (fin(lou) ? 1.0 : 0.0) + (fin(hiu) ? 1.0 : 0.0);
      }
    }
  }
  const double mcount = qsum(mc);
  MPCQP_PCLK(6);
  if (warm && mcount > 0.0 && polish_q<T>(a, at, i, x0i, true)) {
    emit_q<T>(a, b, at, i, true, MPCQP_STATUS_OPTIMAL, 0);
    return true;
  }

  double alpha = 0.0, sigmu = 0.0;
  double mu_pol = a.mu_polish;
  double dreg = 0.0, dlast = 0.0;
  int ncorr = 0;
  const int max_iter = a.max_iter;
  for (int it = 0;; ++it) {
    MPCQP_PCLK(5);
    // ======================================== pass 1: backward factorisation
    double Ph[4] = {0.0, 0.0, 0.0, 0.0}, ph = 0.0, gx1 = 0.0;
    double rstat = 0.0, rdyn = 0.0, musum = 0.0;
    bool pd = true;
    for (int k = N - 1; k >= 0; --k) {
      double xi = at.r(k, L::X), pii = at.r(k, L::PI);
      double llx = at.r(k, L::LL + NU), lux = at.r(k, L::LU + NU);
      double ui = 0.0, llu = 0.0, luu = 0.0;
      if (ou) { ui = at.r(k, L::U); llu = at.r(k, L::LL); luu = at.r(k, L::LU); }
      const double lox = at.r(k, L::LO + NU), hix = at.r(k, L::HI + NU);
      const double lou = ou ? at.r(k, L::LO) : -kInf, hiu = ou ? at.r(k, L::HI) : kInf;
      double xki = k == 0 ? x0i : at.r(k - 1, L::X);
      if (alpha > 0.0 && k > 0) xki += alpha * at.r(k - 1, L::DX);
      if (alpha > 0.0) {  // apply the corrector step of the previous iteration
        auto apply = [&](double& v, double& ll, double& lu, double lo, double hi, double dv,
                         double dva) {
          if (fin(lo)) {
            const double sl = v - lo;
            const double dla = -ll * (1.0 + dva / sl);
            const double rc = sigmu - sl * ll - dva * dla;
            ll += alpha * ((rc - ll * dv) / sl);
          }
          if (fin(hi)) {
            const double su = hi - v;
            const double dua = -lu * (1.0 - dva / su);
            const double rc = sigmu - su * lu + dva * dua;
            lu += alpha * ((rc + lu * dv) / su);
          }
          v += alpha * dv;
        };
        apply(xi, llx, lux, lox, hix, at.r(k, L::DX), at.r(k, L::DXA));
        if (ou) apply(ui, llu, luu, lou, hiu, at.r(k, L::DU), at.r(k, L::DUA));
        pii += alpha * at.r(k, L::DPI);
        at.r(k, L::X) = xi;
        at.r(k, L::PI) = pii;
        at.r(k, L::LL + NU) = llx;
        at.r(k, L::LU + NU) = lux;
        if (ou) { at.r(k, L::U) = ui; at.r(k, L::LL) = llu; at.r(k, L::LU) = luu; }
      }
      double xa[4], x1a[4], pia[4], ua[2];
      bcast4(xki, xa);
      bcast4(xi, x1a);
      bcast4(pii, pia);
      ua[0] = qb<0>(ui);
      ua[1] = qb<1>(ui);
      StageQ S;
      S.load(at, k);
      const double e = resid_q(at, S, k, i, xa, ua, xi);
      rdyn = fmax(rdyn, fabs(e));
      double gx, gu[2];
      grad_q(at, S, k, i, xa, x1a, pia, ua, pii, gx1, gx, gu);
      // stationarity, complementarity, Sigma of the lane's components
      double sx = 0.0, sui = 0.0;
      {
        double r = gx;
        if (fin(lox)) { const double sl = xi - lox; sx += llx / sl; musum += sl * llx; r -= llx; }
        if (fin(hix)) { const double su = hix - xi; sx += lux / su; musum += su * lux; r += lux; }
        rstat = fmax(rstat, fabs(r));
        at.r(k, L::GA + NU) = gx;
      }
      if (ou) {
        const double gui = sel2(gu, i);
        double r = gui;
        if (fin(lou)) { const double sl = ui - lou; sui += llu / sl; musum += sl * llu; r -= llu; }
        if (fin(hiu)) { const double su = hiu - ui; sui += luu / su; musum += su * luu; r += luu; }
        rstat = fmax(rstat, fabs(r));
        at.r(k, L::GA) = gui;
      }
      const double su2[2] = {qb<0>(sui), qb<1>(sui)};
      double P[4], p, K[2][4], kk[2], Gi[3], Kc[2];
      const bool ok = riccati_q(at, S, k, i, Ph, ph, e, gx, gu, sx, su2, dreg, P, p, K, kk, Gi, Kc);
      pd = pd && ok;
      store_factor_q(at, k, i, P, p, Kc, kk, Gi, e);
      gx1 = next_gx1_q(at, S, k, i, pia, ua);
    }
    rstat = qmax(rstat);
    rdyn = qmax(rdyn);
    const double mu = mcount > 0.0 ? qsum(musum) / mcount : 0.0;
    if (!fin(rstat) || !fin(rdyn) || !fin(mu)) {
      emit_q<T>(a, b, at, i, false, MPCQP_STATUS_NONFINITE, it);
      return false;
    }
    if (!pd) {
      dreg = dreg > 0.0 ? 8.0 * dreg : (dlast > 0.0 ? dlast : 1e-4);
      if ((a.strict > 0 && ++ncorr > a.strict) || dreg > 1e12 || it >= max_iter) {
        emit_q<T>(a, b, at, i, false, MPCQP_STATUS_NOT_CONVEX, it);
        return false;
      }
      alpha = 0.0;
      continue;
    }
    if (dreg > 0.0) {
      dlast = dreg;
      dreg = dreg / 3.0 > 1e-12 ? dreg / 3.0 : 0.0;
    }
    const bool conv = rstat <= a.tol && rdyn <= a.tol && mu <= a.tol_mu;
    if (mcount > 0.0 && mu_pol > 0.0 && mu <= mu_pol && rstat <= a.tol_polish &&
        rdyn <= a.tol_polish) {
      MPCQP_PCLK(0);
      const bool pol = polish_q<T>(a, at, i, x0i);
      MPCQP_PCLK(4);
      if (pol) {
        emit_q<T>(a, b, at, i, true, MPCQP_STATUS_OPTIMAL, it);
        return true;
      }
      mu_pol *= 1e-2;
      alpha = 0.0;
      if (conv || it >= max_iter) {
        emit_q<T>(a, b, at, i, false, conv ? MPCQP_STATUS_OPTIMAL : MPCQP_STATUS_MAXITER, it);
        return false;
      }
      continue;
    }
    if (conv || it >= max_iter) {
      emit_q<T>(a, b, at, i, false, conv ? MPCQP_STATUS_OPTIMAL : MPCQP_STATUS_MAXITER, it);
      return false;
    }

    MPCQP_PCLK(0);
    // ========================================== pass 2: forward predictor
    double amax = 1.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
    forward_q(at, N, i, [&](int k, const double (&du)[2], double dxn, const double (&)[4]) {
      at.r(k, L::DXA) = dxn;
      if (ou) at.r(k, L::DUA) = sel2(du, i);
      auto comp = [&](double vj, double dv, double lo, double hi, double l, double lu) {
        if (fin(lo)) {
          const double sl = vj - lo;
          const double dl = -l * (1.0 + dv / sl);
          if (dv < 0.0) amax = fmin(amax, -sl / dv);
          if (dl < 0.0) amax = fmin(amax, -l / dl);
          c0 += sl * l;
          c1 += sl * dl + l * dv;
          c2 += dv * dl;
        }
        if (fin(hi)) {
          const double su = hi - vj;
          const double dl = -lu * (1.0 - dv / su);
          if (dv > 0.0) amax = fmin(amax, su / dv);
          if (dl < 0.0) amax = fmin(amax, -lu / dl);
          c0 += su * lu;
          c1 += su * dl - lu * dv;
          c2 -= dv * dl;
        }
      };
      comp(at.r(k, L::X), dxn, at.r(k, L::LO + NU), at.r(k, L::HI + NU),
           at.r(k, L::LL + NU), at.r(k, L::LU + NU));
      if (ou)
        comp(at.r(k, L::U), sel2(du, i), at.r(k, L::LO), at.r(k, L::HI), at.r(k, L::LL),
             at.r(k, L::LU));
    });
    amax = qmin(amax);
    if (mcount > 0.0) {
      const double mua = (qsum(c0) + amax * (qsum(c1) + amax * qsum(c2))) / mcount;
      const double r = fmax(0.0, fmin(1.0, mua / mu));
      sigmu = r * r * r * mu;
    } else {
      sigmu = 0.0;
    }

    MPCQP_PCLK(1);
    // ================================ pass 3: backward corrector right side
    {
      double phc = 0.0;
      for (int k = N - 1; k >= 0; --k) {
        auto rhs = [&](double vj, double dva, double lo, double hi, double l, double lu,
                       double g) {
          double s = g;
          if (fin(lo)) {
            const double sl = vj - lo;
            s += (-sigmu - dva * l * (1.0 + dva / sl)) / sl;
          }
          if (fin(hi)) {
            const double su = hi - vj;
            s += (sigmu - dva * lu * (1.0 - dva / su)) / su;
          }
          return s;
        };
        const double gx = rhs(at.r(k, L::X), at.r(k, L::DXA), at.r(k, L::LO + NU),
                              at.r(k, L::HI + NU), at.r(k, L::LL + NU),
                              at.r(k, L::LU + NU), at.r(k, L::GA + NU));
        const double gum = ou ? rhs(at.r(k, L::U), at.r(k, L::DUA), at.r(k, L::LO),
                                    at.r(k, L::HI), at.r(k, L::LL), at.r(k, L::LU),
                                    at.r(k, L::GA))
                              : 0.0;
        const double gu[2] = {qb<0>(gum), qb<1>(gum)};
        const double p = gx + phc;
        double Pe = p;
#pragma unroll
        for (int j = 0; j < 4; ++j) Pe = fma(at.p(k, L::PP, j), at(k, L::E + j), Pe);
        double Pea[4];
        bcast4(Pe, Pea);
        double h[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          double s = gu[r];
#pragma unroll
          for (int q = 0; q < 4; ++q) s = fma(at(k, L::DB + q * NU + r), Pea[q], s);
          h[r] = s;
        }
        const double Gi[3] = {at(k, L::GI + 0), at(k, L::GI + 1), at(k, L::GI + 2)};
        double kk[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) kk[r] = -(Gi[pk(r, 0)] * h[0] + Gi[pk(r, 1)] * h[1]);
        if (ou) at.r(k, L::KV) = sel2(kk, i);
        // ph = A'Pe + K'h
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) s = fma(at.r(k, L::DA + q * NX), Pea[q], s);
#pragma unroll
        for (int r = 0; r < 2; ++r) s = fma(at.r(k, L::KM + r * NX), h[r], s);
        phc = s;
        at.r(k, L::PV) = p;
      }
    }

    MPCQP_PCLK(2);
    // ========================================== pass 4: forward corrector
    amax = 1.0;
    forward_q(at, N, i, [&](int k, const double (&du)[2], double dxn, const double (&dxa)[4]) {
      double s = at.r(k, L::PV);
#pragma unroll
      for (int j = 0; j < 4; ++j) s = fma(at.p(k, L::PP, j), dxa[j], s);
      at.r(k, L::DPI) = s;
      at.r(k, L::DX) = dxn;
      if (ou) at.r(k, L::DU) = sel2(du, i);
      auto comp = [&](double vj, double dv, double dva, double lo, double hi, double l,
                      double lu) {
        if (fin(lo)) {
          const double sl = vj - lo;
          const double dla = -l * (1.0 + dva / sl);
          const double dl = (sigmu - sl * l - dva * dla - l * dv) / sl;
          if (dv < 0.0) amax = fmin(amax, -sl / dv);
          if (dl < 0.0) amax = fmin(amax, -l / dl);
        }
        if (fin(hi)) {
          const double su = hi - vj;
          const double dua = -lu * (1.0 - dva / su);
          const double dl = (sigmu - su * lu + dva * dua + lu * dv) / su;
          if (dv > 0.0) amax = fmin(amax, su / dv);
          if (dl < 0.0) amax = fmin(amax, -lu / dl);
        }
      };
      comp(at.r(k, L::X), dxn, at.r(k, L::DXA), at.r(k, L::LO + NU), at.r(k, L::HI + NU),
           at.r(k, L::LL + NU), at.r(k, L::LU + NU));
      if (ou)
        comp(at.r(k, L::U), sel2(du, i), at.r(k, L::DUA), at.r(k, L::LO), at.r(k, L::HI),
             at.r(k, L::LL), at.r(k, L::LU));
    });
    alpha = fmin(1.0, 0.995 * qmin(amax));
    MPCQP_PCLK(3);
  }
}

}  // namespace ipmq
}  // namespace mpcqp
