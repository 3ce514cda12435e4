// ipm_wave.hpp -- the interior point of ipm_quad.hpp (solve_quad) for one
// instance on a WHOLE wavefront: the one-launch SQP (sqp_solve.hip) runs each
// instance in its own single-wave workgroup, where solve_quad kept 60 of the
// 64 lanes idle while one quad walked the horizon four times per iteration.
// Here only the serial chains stay on quad 0 (lanes 0..3):
//   pass 1  the Riccati factorisation (riccati_q, store_factor_q),
//   pass 2  the predictor's forward sweep (du = K dx + k, dx+ = A dx + B du + e),
//   pass 3  the corrector's backward right-hand side (p, Pe, h, k, the cost-to-go),
//   pass 4  the corrector's forward sweep,
// and everything per stage runs one quad per stage on the 16 quads of the wave
// before or after its chain: applying the previous step, the dynamics residual,
// the gradients, Sigma and the complementarity of pass 1; the step to the
// boundary and the affine complementarity of pass 2; the corrector right-hand
// side of pass 3; the costate direction and the step to the boundary of pass 4.
// Every per-stage quantity is the same expression of the same fields as in
// solve_quad (the helpers are shared), so the iterates agree with it to the
// summation order of the wave-wide reductions.  The polish is split the same
// way (polish_w); the start and the output are solve_quad's (quad 0).  The
// QP's workspace in LDS (LD = 1), stage data already staged (stage_in_q).
//
// Between the per-stage and the serial parts the values go through the
// workspace: pass 1's per-stage part leaves e in E, the gradients in GA and
// Sigma of the lane's components in DXA / DUA (dead until pass 2 writes the
// predictor); its first half leaves x_k (after the step) in E and the later
// stage's A'pi + H2xu u term in PV (both dead until the factorisation).
#pragma once

#include "ipm_quad.hpp"

namespace mpcqp {
namespace ipmw {

using namespace ipmq;

// sum over the whole wave (every lane ends with the total)
MPCQP_QD double wsum(double v) {
  v += lane_step<1>(v);
  v += lane_step<2>(v);
  v += lane_step<4>(v);
  v += lane_step<8>(v);
  v += lane_step<16>(v);
  v += lane_step<32>(v);
  return v;
}
MPCQP_QD double wave_max(double v) {
  v = fmax(v, lane_step<1>(v));
  v = fmax(v, lane_step<2>(v));
  v = fmax(v, lane_step<4>(v));
  v = fmax(v, lane_step<8>(v));
  v = fmax(v, lane_step<16>(v));
  return fmax(v, lane_step<32>(v));
}
MPCQP_QD double wave_min(double v) {
  v = fmin(v, lane_step<1>(v));
  v = fmin(v, lane_step<2>(v));
  v = fmin(v, lane_step<4>(v));
  v = fmin(v, lane_step<8>(v));
  v = fmin(v, lane_step<16>(v));
  return fmin(v, lane_step<32>(v));
}
MPCQP_QD double from_lane0(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(bits & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(bits >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
MPCQP_QD bool from_lane0(bool v) { return __builtin_amdgcn_readfirstlane(v ? 1 : 0) != 0; }

constexpr int kQuads = kWave / 4;

// ------------------------------------------------ Riccati on the matrix cores
// The factorisation sweep of riccati_q as 4 x 4 fp64 matrix products on
// v_mfma_f64_4x4x4_4b_f64 (measured on gfx950, tools/mfma64_probe): four
// independent 4 x 4 x 4 blocks, block m = (lane >> 2) & 3; in a block the B,
// C and D operands hold X[r][c] at lane 16 r + 4 m + c ("D layout") and the A
// operand reads a D-layout matrix as its transpose.  So with every stage
// matrix in D layout (lane (r, c) loads its element):
//   M1a = P'A = PA,  M1b = P [B | e] + [0 | p]        (2 products)
//   A'PA, A'M1b, B'PA, B'M1b                           (4 products)
//   K = -G^-1 Hx,  Ph = A'PA + Hx'K,  ph = A'Pe + Hx'k (3 products)
// with Hx = H2xu' + B'PA; the 2 x 2 block G, h is read from block 0 and
// inverted on every lane.  One stage is ~50 instructions with a dependency
// chain of 5 products, against ~285 VALU for the quad step (each fp64 VALU
// op issues in 4 cycles; a dependent 4x4x4 product returns in 23-29, a
// dependent FMA in 6.5: profiles/r06/mfma64_probe.txt).  All four blocks
// compute the same stage; block 0 stores.  Fields: the factor data as
// store_factor_q writes them (PP, KM, GI, KV, PV; E is not rewritten);
// the gradient g_x, the input gradients, Sigma_x and Sigma_u come from the
// lane-relative field FGX, the fields FGU, FGU+1, the lane-relative FSX and
// FSU, FSU+1.  Returns (uniformly) whether every G was positive definite.
MPCQP_QD double mfma44(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
MPCQP_QD double lane_bcast(double v, int l) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int FGX, int FGU, int FSX, int FSU>
MPCQP_QD bool riccati_mfma(double* W, int N, double dreg) {
  const int lane = (int)threadIdx.x;
  const int r = lane >> 4, c = lane & 3;
  const bool store = ((lane >> 2) & 3) == 0;
  const bool isB = c < 2, isE = c == 2, isD = r == c, rowU = r < 2;
  // lane-constant offsets of the lane's element in a stage's fields
  const int oA = L::DA + r * NX + c;
  const int oB = L::DB + r * NU + (c & 1);
  const int oE = L::E + r;
  const int oWXX = L::WXX + pk(r, c);
  const int oSX = FSX + r, oGX = FGX + r;
  const int oWXU = L::WXU + c * NU + (r & 1);
  const int oPP = L::PP + pk(r, c), oKM = L::KM + (r & 1) * NX + c;
  // the stage's operands, loaded one stage ahead (the LDS round trip then
  // overlaps the previous stage's products instead of opening each stage)
  struct Ops {
    double a, bq, e, wxx, sx, gx, wxu, wuu0, wuu1, wuu2, su0, su1, gu0, gu1;
  };
  auto load = [&](int k) {
    const double* S = W + k * L::F;
    Ops o;
    o.a = S[oA]; o.bq = S[oB]; o.e = S[oE]; o.wxx = S[oWXX];
    o.sx = S[oSX]; o.gx = S[oGX]; o.wxu = S[oWXU];
    o.wuu0 = S[L::WUU]; o.wuu1 = S[L::WUU + 1]; o.wuu2 = S[L::WUU + 2];
    o.su0 = S[FSU]; o.su1 = S[FSU + 1]; o.gu0 = S[FGU]; o.gu1 = S[FGU + 1];
    return o;
  };
  double Ph = 0.0, phc = 0.0;
  bool ok = true;
  Ops nx = load(N - 1);
  for (int k = N - 1; k >= 0; --k) {
    double* S = W + k * L::F;
    const Ops o = nx;
    // P = Q' + H2xx + Ph + Sigma_x (+ shift), p = g_x + ph (column 2)
    const double P = o.wxx + Ph + (isD ? o.sx + dreg : 0.0);
    const double p = o.gx + phc;
    const double M1a = mfma44(P, o.a, 0.0);
    const double M1b = mfma44(P, isB ? o.bq : (isE ? o.e : 0.0), isE ? p : 0.0);
    // the next stage's operands, issued behind the first products (the
    // scheduler would otherwise sink them to their use: an LDS round trip
    // at the head of every stage)
    __builtin_amdgcn_sched_barrier(0);
    nx = load(k > 0 ? k - 1 : 0);
    __builtin_amdgcn_sched_barrier(0);
    const double Bz = isB ? o.bq : 0.0;
    const double AtPA = mfma44(o.a, M1a, 0.0);
    const double AtM1b = mfma44(o.a, M1b, 0.0);
    const double BtPA = mfma44(Bz, M1a, 0.0);
    const double BtM1b = mfma44(Bz, M1b, 0.0);
    // G = R + H2uu + Sigma_u + B'PB, h = g_u + B'Pe (block 0, lanes 0, 16, 17; 2, 18)
    double G[3], Gi[3];
    G[0] = o.wuu0 + o.su0 + dreg + lane_bcast(BtM1b, 0);
    G[1] = o.wuu1 + lane_bcast(BtM1b, 16);
    G[2] = o.wuu2 + o.su1 + dreg + lane_bcast(BtM1b, 17);
    const double h0 = o.gu0 + lane_bcast(BtM1b, 2), h1 = o.gu1 + lane_bcast(BtM1b, 18);
    ok = inv2(G, Gi) && ok;
    const double kk0 = -(Gi[0] * h0 + Gi[1] * h1), kk1 = -(Gi[1] * h0 + Gi[2] * h1);
    const double Hx = rowU ? BtPA + o.wxu : 0.0;
    const double mGi = (rowU && isB) ? -(r == c ? (r == 0 ? Gi[0] : Gi[2]) : Gi[1]) : 0.0;
    const double K = mfma44(mGi, Hx, 0.0);
    const double kkv = (rowU && isE) ? (r == 0 ? kk0 : kk1) : 0.0;
    Ph = mfma44(Hx, K, AtPA);
    phc = mfma44(Hx, kkv, AtM1b);
    if (store) {
      if (c <= r) S[oPP] = P;
      if (rowU) {
        S[oKM] = K;
        if (isE) S[L::KV + r] = kkv;
      }
      if (isE) S[L::PV + r] = p;
      if (r == 0 && c < 3) S[L::GI + c] = Gi[c];
    }
  }
  return ok;
}

// The two recursions that remain after the factorisation, on the matrix cores
// (same operand layouts as riccati_mfma; block 0 stores):
//  forward_mfma  dx_{k+1} = Acl_k dx_k + (e_k + B_k k_k), Acl = A + B K, the
//                state direction of x_{k+1} into the lane-relative field FOUT
//                (one dependent product per stage; the input direction
//                du_k = K_k dx_k + k_k is left to the per-stage phase after it,
//                du_of_stage);
//  rhs_mfma      the right-hand side sweep of rhs_sweep_q: p = g_x + phc,
//                Pe = P e + p, k = -G^-1 (g_u + B'Pe), phc = Acl'Pe + K'g_u
//                (one dependent product per stage).
// Acl' / Acl, P e + g_x and K'g_u do not depend on the recursion and are
// formed from the stage's fields ahead of it.
template <int FOUT>
MPCQP_QD void forward_mfma(double* W, int N) {
  const int lane = (int)threadIdx.x;
  const int r = lane >> 4, c = lane & 3;
  const bool store = ((lane >> 2) & 3) == 0 && c == 0, rowU = r < 2, col0 = c == 0;
  const int oKM = L::KM + (r & 1) * NX + c;
  const int oBt = L::DB + c * NU + (r & 1);
  const int oAt = L::DA + c * NX + r;
  const int oB0 = L::DB + r * NU, oE = L::E + r;
  // pipeline: the stage's raw operands two stages ahead, its closed-loop
  // matrix and offset (products that do not depend on the recursion) one
  // stage ahead, each behind a scheduling barrier after the recursion's
  // product of the current stage
  struct Raw {
    double Kd, Bt, At, b0, b1, e, kk0, kk1;
  };
  auto load = [&](int k) {
    const double* S = W + k * L::F;
    Raw o;
    o.Kd = rowU ? S[oKM] : 0.0; o.Bt = rowU ? S[oBt] : 0.0; o.At = S[oAt];
    o.b0 = S[oB0]; o.b1 = S[oB0 + 1]; o.e = S[oE];
    o.kk0 = S[L::KV]; o.kk1 = S[L::KV + 1];
    return o;
  };
  auto prep = [&](const Raw& o, double& AclT, double& ccl) {
    AclT = mfma44(o.Kd, o.Bt, o.At);  // (A + B K)'
    ccl = col0 ? fma(o.b1, o.kk1, fma(o.b0, o.kk0, o.e)) : 0.0;
  };
  double dx = 0.0;  // column 0: the direction of x_k
  double AclT, ccl;
  prep(load(0), AclT, ccl);
  Raw nx = load(N > 1 ? 1 : 0);
  for (int k = 0; k < N; ++k) {
    dx = mfma44(AclT, dx, ccl);
    __builtin_amdgcn_sched_barrier(0);
    prep(nx, AclT, ccl);
    nx = load(k + 2 < N ? k + 2 : N - 1);
    __builtin_amdgcn_sched_barrier(0);
    if (store) W[k * L::F + FOUT + r] = dx;
  }
}

template <int FGX, int FGU>
MPCQP_QD void rhs_mfma(double* W, int N) {
  const int lane = (int)threadIdx.x;
  const int r = lane >> 4, c = lane & 3;
  const bool store = ((lane >> 2) & 3) == 0 && c == 0, rowU = r < 2, col0 = c == 0;
  const int oPP = L::PP + pk(r, c), oE = L::E + r, oGX = FGX + r;
  const int oA = L::DA + r * NX + c, oKM = L::KM + (r & 1) * NX + c;
  const int oBt = L::DB + c * NU + (r & 1);
  // pipeline as forward_mfma: raw operands two stages ahead, the products
  // that do not depend on the recursion one stage ahead
  struct Raw {
    double P, e, gx, A, Kd, Bt, guc;
  };
  auto load = [&](int k) {
    const double* S = W + k * L::F;
    Raw o;
    o.P = S[oPP]; o.e = col0 ? S[oE] : 0.0; o.gx = col0 ? S[oGX] : 0.0;
    o.A = S[oA]; o.Kd = rowU ? S[oKM] : 0.0; o.Bt = rowU ? S[oBt] : 0.0;
    o.guc = (rowU && col0) ? S[FGU + (r & 1)] : 0.0;
    return o;
  };
  auto prep = [&](const Raw& o, double& Pe0, double& Acl, double& Ktgu, double& gx) {
    Pe0 = mfma44(o.P, o.e, o.gx);      // P e + g_x (column 0)
    Acl = mfma44(o.Bt, o.Kd, o.A);     // A + B K
    Ktgu = mfma44(o.Kd, o.guc, 0.0);   // K'g_u (column 0)
    gx = o.gx;
  };
  double phc = 0.0;  // column 0
  double Pe0, Acl, Ktgu, gx;
  prep(load(N - 1), Pe0, Acl, Ktgu, gx);
  Raw nx = load(N > 1 ? N - 2 : 0);
  for (int k = N - 1; k >= 0; --k) {
    const double p = gx + phc;
    phc = mfma44(Acl, Pe0 + phc, Ktgu);
    __builtin_amdgcn_sched_barrier(0);
    prep(nx, Pe0, Acl, Ktgu, gx);
    nx = load(k > 1 ? k - 2 : 0);
    __builtin_amdgcn_sched_barrier(0);
    if (store) W[k * L::F + L::PV + r] = p;
  }
}

// The feed-forward of stage k after rhs_mfma, lane i of a quad (lanes 0, 1
// store): k = -G^-1 (g_u + B'(P e + p)), g_u from FGU, FGU+1
template <int FGU>
MPCQP_QD void rhs_kk_stage(const WsQ<1>& at, int k, int i) {
  double Pe = at.r(k, L::PV);
#pragma unroll
  for (int j = 0; j < 4; ++j) Pe = fma(at.p(k, L::PP, j), at(k, L::E + j), Pe);
  double Pea[4];
  bcast4(Pe, Pea);
  double h[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    double s = at(k, FGU + r);
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fma(at(k, L::DB + q * NU + r), Pea[q], s);
    h[r] = s;
  }
  const double Gi[3] = {at(k, L::GI + 0), at(k, L::GI + 1), at(k, L::GI + 2)};
  if (i < 2) {
    const double kk = -(Gi[pk(i, 0)] * h[0] + Gi[pk(i, 1)] * h[1]);
    at.r(k, L::KV) = kk;
  }
}

// du_k = K_k dx_k + k_k of stage k, lane i < 2 (dx_k: the state direction of
// stage k-1 in the lane-relative field FDX, 0 at k = 0)
template <int FDX>
MPCQP_QD double du_of_stage(const WsQ<1>& at, int k, int i) {
  double s = at(k, L::KV + (i & 1));
  if (k > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) s = fma(at(k, L::KM + (i & 1) * NX + j), at(k - 1, FDX + j), s);
  }
  return s;
}

// The backward sweep of a right-hand side on the stored factorisation (quad
// 0; pass 3 of the interior point, solve_quad's expressions): g_x row i from
// field FGX (lane-relative), g_u (both inputs) from FGU; writes k -> KV and
// p -> PV (each stage's fields are read before they are written).
template <int FGX, int FGU>
MPCQP_QD void rhs_sweep_q(const WsQ<1>& at, int N, int i) {
  const bool ou = i < NU;
  double phc = 0.0;
  for (int k = N - 1; k >= 0; --k) {
    const double gx = at.r(k, FGX);
    const double gu[2] = {at(k, FGU), at(k, FGU + 1)};
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
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) s = fma(at.r(k, L::DA + q * NX), Pea[q], s);
#pragma unroll
    for (int r = 0; r < 2; ++r) s = fma(at.r(k, L::KM + r * NX), h[r], s);
    phc = s;
    at.r(k, L::PV) = p;
  }
}

// polish_q (ipm_quad.hpp) on the whole wave: each method-of-multipliers step
// is the per-stage residual / gradient / penalty (one quad per stage, into
// the factor fields the serial sweep overwrites after reading: e -> E, g_x ->
// PV, g_u -> KV, the penalties -> KM / GI), the Riccati sweep on quad 0, the
// forward sweep on quad 0 (the state direction of stage k -> E, the iterate
// updated), then per stage the costate update, the multipliers and the
// active-set tests.  Same expressions as polish_q; returns (wave-uniform)
// whether the polish certified its vertex.
template <typename T>
MPCQP_QD bool polish_w(const Args<T>& a, const WsQ<1>& at, int qd, int i, double x0i,
                       bool warm) {
  const int N = a.N;
  const bool ou = i < NU;
#ifdef MPCQP_RICCATI_QUAD
  const bool q0 = qd == 0;
#endif
  for (int k = qd; k < N; k += kQuads) {
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
  wave_lds_sync();
  constexpr int kSteps = 4, kRounds = 4;
#ifdef MPCQP_POLISH_EARLY
  constexpr int kPolishEarly = MPCQP_POLISH_EARLY;
#else
  constexpr int kPolishEarly = kSteps;
#endif
#ifdef MPCQP_WARM_ROUNDS
  const int rounds = warm ? MPCQP_WARM_ROUNDS : kRounds;
#else
  const int rounds = kRounds;
#endif
  for (int round = 0; round < rounds; ++round) {
    bool good = true, changed = false;
    for (int step = 0; step < kSteps; ++step) {
      const double rho = step == 0 ? 1e8 : (step == 1 ? 1e6 : 1e4);
      // the last step keeps the penalty of the one before: same factorisation
      const bool refactor = step < 3;
      // per stage: residual, gradients and the active components' penalty
      for (int k = qd; k < N; k += kQuads) {
        const double xi = at.r(k, L::DX), pii = at.r(k, L::DPI);
        const double ui = ou ? at.r(k, L::DU) : 0.0;
        const double xki = k == 0 ? x0i : at.r(k - 1, L::DX);
        double gx1 = 0.0;
        if (k + 1 < N) {
          const double pin = at.r(k + 1, L::DPI), un = ou ? at.r(k + 1, L::DU) : 0.0;
          double pia[4], ua[2];
          bcast4(pin, pia);
          ua[0] = qb<0>(un);
          ua[1] = qb<1>(un);
          StageQ S1;
          gx1 = next_gx1_q(at, S1, k + 1, i, pia, ua);
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
        double gx, gu[2];
        grad_q(at, S, k, i, xa, x1a, pia, ua, pii, gx1, gx, gu);
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
        gu[0] += qb<0>(gum);
        gu[1] += qb<1>(gum);
        at.r(k, L::E) = e;
        at.r(k, L::PV) = gx;
        if (ou) at.r(k, L::KV) = sel2(gu, i);
        if (refactor) {  // (a kept factorisation keeps its K and G^-1 fields)
          at.r(k, L::KM) = sx;
          if (ou) at.r(k, L::GI) = sui;
        }
      }
      wave_lds_sync();
#ifndef MPCQP_RICCATI_QUAD
      if (refactor) {
        good = riccati_mfma<L::PV, L::KV, L::KM, L::GI>(at.W, N, 0.0) && good;
      } else {
        // the penalty and the active set of the previous step: its factors
        // stand, only the right-hand side is swept (e back in E first)
        rhs_mfma<L::PV, L::KV>(at.W, N);
        wave_lds_sync();
        // (g_u is in KV: every stage reads its own before writing k there)
        for (int k = qd; k < N; k += kQuads) rhs_kk_stage<L::KV>(at, k, i);
      }
      wave_lds_sync();
      forward_mfma<L::E>(at.W, N);
      wave_lds_sync();
      // the step: x, u += the directions (the state direction of stage k is
      // in E(k); du_k needs that of stage k-1, so the updates of DX follow)
      for (int k = qd; k < N; k += kQuads)
        if (ou) at.r(k, L::DU) += du_of_stage<L::E>(at, k, i);
      wave_lds_sync();
      for (int k = qd; k < N; k += kQuads) at.r(k, L::DX) += at.r(k, L::E);
#else
      if (q0 && refactor) {
        double Ph[4] = {0.0, 0.0, 0.0, 0.0}, ph = 0.0;
        for (int k = N - 1; k >= 0; --k) {
          StageQ S;
          S.load(at, k);
          const double e = at.r(k, L::E), gx = at.r(k, L::PV), sx = at.r(k, L::KM);
          const double gu[2] = {at(k, L::KV), at(k, L::KV + 1)};
          const double su2[2] = {at(k, L::GI), at(k, L::GI + 1)};
          double P[4], p, K[2][4], kk[2], Gi[3], Kc[2];
          good = riccati_q(at, S, k, i, Ph, ph, e, gx, gu, sx, su2, 0.0, P, p, K, kk, Gi, Kc) && good;
          store_factor_q(at, k, i, P, p, Kc, kk, Gi, e);
        }
      } else if (q0) {
        rhs_sweep_q<L::PV, L::KV>(at, N, i);
      }
      if (q0) {
        forward_q(at, N, i, [&](int k, const double (&du)[2], double dxn, const double (&)[4]) {
          at.r(k, L::E) = dxn;
          at.r(k, L::DX) += dxn;
          if (ou) at.r(k, L::DU) += sel2(du, i);
        });
      }
#endif
      wave_lds_sync();
      const bool last = step == kSteps - 1;
      const bool probe = !last && step >= kPolishEarly;
      bool pass = true;
      for (int k = qd; k < N; k += kQuads) {
        double s = at.r(k, L::PV);
#pragma unroll
        for (int j = 0; j < 4; ++j) s = fma(at.p(k, L::PP, j), at(k, L::E + j), s);
        at.r(k, L::DPI) += s;
#pragma unroll
        for (int part = 0; part < 2; ++part) {
          if (part == 1 && !ou) continue;
          const int j = part == 0 ? NU + i : i;
          const double vj = part == 0 ? at.r(k, L::DX) : at.r(k, L::DU);
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
      }
      wave_lds_sync();
      if (probe && wave_min(good && pass ? 1.0 : 0.0) > 0.5) return true;
    }
    good = wave_min(good ? 1.0 : 0.0) > 0.5;
    changed = wave_max(changed ? 1.0 : 0.0) > 0.5;
    if (good && !changed) return true;
    if (!good) return false;
  }
  return false;
}

// All 64 lanes, uniform control flow; returns true (on every lane) when the
// QP ended polished.  warm, pclk: as solve_quad.
template <typename T>
MPCQP_QD bool solve_wave(const Args<T>& a, int b, double* W, bool warm = false,
                         uint64_t* pclk = nullptr) {
#ifdef MPCQP_IPM_PASSCLK
  uint64_t pclk_t = __builtin_amdgcn_s_memrealtime();
#endif
  const int lane = (int)threadIdx.x, qd = lane >> 2;
  const int i = lane & 3;
  const bool q0 = qd == 0;
  const WsQ<1> at(W, i);
  const bool ou = i < NU;
  const int N = a.N, nx = a.nx, nu = a.nu;
  const double x0i = i < nx ? (double)a.x0[(int64_t)b * a.sX0 + i] : 0.0;

  // ------------------------------------------------- start (quad 0, serial)
  double mc = 0.0;
  if (q0) {
    double xi = x0i;
    for (int k = 0; k < N; ++k) {
      const double ci = at.r(k, L::DC);
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
  const double mcount = wsum(mc);
  wave_lds_sync();
  MPCQP_PCLK(6);
  if (warm && mcount > 0.0) {
    const bool wp = polish_w<T>(a, at, qd, i, x0i, true);
    MPCQP_PCLK(7);
    if (wp) {
      if (q0) emit_q<T>(a, b, at, i, true, MPCQP_STATUS_OPTIMAL, 0);
      return true;
    }
  }

  double alpha = 0.0, sigmu = 0.0;
  double mu_pol = a.mu_polish;
  double dreg = 0.0, dlast = 0.0;
  int ncorr = 0;
  const int max_iter = a.max_iter;
  for (int it = 0;; ++it) {
    // ========================= pass 1a: per stage, the neighbours' values
    // x_k after the previous step (stage k-1's state, not yet updated in
    // solve_quad's backward order) -> E; the later stage's A'pi + H2xu u
    // after the step -> PV
    for (int k = qd; k < N; k += kQuads) {
      double xki = k == 0 ? x0i : at.r(k - 1, L::X);
      if (alpha > 0.0 && k > 0) xki += alpha * at.r(k - 1, L::DX);
      double gx1 = 0.0;
      if (k + 1 < N) {
        double pin = at.r(k + 1, L::PI), un = ou ? at.r(k + 1, L::U) : 0.0;
        if (alpha > 0.0) {
          pin += alpha * at.r(k + 1, L::DPI);
          if (ou) un += alpha * at.r(k + 1, L::DU);
        }
        double pia[4], ua[2];
        bcast4(pin, pia);
        ua[0] = qb<0>(un);
        ua[1] = qb<1>(un);
        StageQ S;
        gx1 = next_gx1_q(at, S, k + 1, i, pia, ua);
      }
      at.r(k, L::E) = xki;
      at.r(k, L::PV) = gx1;
    }
    wave_lds_sync();
    MPCQP_PCLK(8);
    // ============ pass 1b: per stage, the step, residual, gradients, Sigma
    double rstat = 0.0, rdyn = 0.0, musum = 0.0;
    for (int k = qd; k < N; k += kQuads) {
      double xi = at.r(k, L::X), pii = at.r(k, L::PI);
      double llx = at.r(k, L::LL + NU), lux = at.r(k, L::LU + NU);
      double ui = 0.0, llu = 0.0, luu = 0.0;
      if (ou) { ui = at.r(k, L::U); llu = at.r(k, L::LL); luu = at.r(k, L::LU); }
      const double lox = at.r(k, L::LO + NU), hix = at.r(k, L::HI + NU);
      const double lou = ou ? at.r(k, L::LO) : -kInf, hiu = ou ? at.r(k, L::HI) : kInf;
      const double xki = at.r(k, L::E), gx1 = at.r(k, L::PV);
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
        at.r(k, L::DUA) = sui;
      }
      at.r(k, L::E) = e;
      at.r(k, L::DXA) = sx;
    }
    wave_lds_sync();
    MPCQP_PCLK(9);
    // ==================== pass 1c: the Riccati factorisation (quad 0, serial)
    bool pd = true;
#ifndef MPCQP_RICCATI_QUAD
    pd = riccati_mfma<L::GA + NU, L::GA, L::DXA, L::DUA>(W, N, dreg);
#else
    if (q0) {
      double Ph[4] = {0.0, 0.0, 0.0, 0.0}, ph = 0.0;
      for (int k = N - 1; k >= 0; --k) {
        StageQ S;
        S.load(at, k);
        const double e = at.r(k, L::E), gx = at.r(k, L::GA + NU), sx = at.r(k, L::DXA);
        const double gu[2] = {at(k, L::GA), at(k, L::GA + 1)};
        const double su2[2] = {at(k, L::DUA), at(k, L::DUA + 1)};
        double P[4], p, K[2][4], kk[2], Gi[3], Kc[2];
        const bool ok = riccati_q(at, S, k, i, Ph, ph, e, gx, gu, sx, su2, dreg, P, p, K, kk, Gi, Kc);
        pd = pd && ok;
        store_factor_q(at, k, i, P, p, Kc, kk, Gi, e);
      }
    }
    pd = from_lane0(pd);
#endif
    MPCQP_PCLK(10);
    rstat = wave_max(rstat);
    rdyn = wave_max(rdyn);
    const double mu = mcount > 0.0 ? wsum(musum) / mcount : 0.0;
    wave_lds_sync();
    if (!fin(rstat) || !fin(rdyn) || !fin(mu)) {
      if (q0) emit_q<T>(a, b, at, i, false, MPCQP_STATUS_NONFINITE, it);
      return false;
    }
    if (!pd) {
      dreg = dreg > 0.0 ? 8.0 * dreg : (dlast > 0.0 ? dlast : 1e-4);
      if ((a.strict > 0 && ++ncorr > a.strict) || dreg > 1e12 || it >= max_iter) {
        if (q0) emit_q<T>(a, b, at, i, false, MPCQP_STATUS_NOT_CONVEX, it);
        return false;
      }
      MPCQP_PCLK(5);
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
      const bool pol = polish_w<T>(a, at, qd, i, x0i, false);
      MPCQP_PCLK(4);
      if (pol) {
        if (q0) emit_q<T>(a, b, at, i, true, MPCQP_STATUS_OPTIMAL, it);
        return true;
      }
      mu_pol *= 1e-2;
      alpha = 0.0;
      if (conv || it >= max_iter) {
        if (q0) emit_q<T>(a, b, at, i, false, conv ? MPCQP_STATUS_OPTIMAL : MPCQP_STATUS_MAXITER, it);
        return false;
      }
      continue;
    }
    if (conv || it >= max_iter) {
      if (q0) emit_q<T>(a, b, at, i, false, conv ? MPCQP_STATUS_OPTIMAL : MPCQP_STATUS_MAXITER, it);
      return false;
    }

    MPCQP_PCLK(0);
    // ============ pass 2: the predictor's forward sweep (quad 0), then per stage
#ifndef MPCQP_RICCATI_QUAD
    forward_mfma<L::DXA>(W, N);
    wave_lds_sync();
#else
    if (q0)
      forward_q(at, N, i, [&](int k, const double (&du)[2], double dxn, const double (&)[4]) {
        at.r(k, L::DXA) = dxn;
        if (ou) at.r(k, L::DUA) = sel2(du, i);
      });
    wave_lds_sync();
#endif
    double amax = 1.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
    for (int k = qd; k < N; k += kQuads) {
#ifndef MPCQP_RICCATI_QUAD
      if (ou) at.r(k, L::DUA) = du_of_stage<L::DXA>(at, k, i);
#endif
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
      comp(at.r(k, L::X), at.r(k, L::DXA), at.r(k, L::LO + NU), at.r(k, L::HI + NU),
           at.r(k, L::LL + NU), at.r(k, L::LU + NU));
      if (ou)
        comp(at.r(k, L::U), at.r(k, L::DUA), at.r(k, L::LO), at.r(k, L::HI), at.r(k, L::LL),
             at.r(k, L::LU));
    }
    amax = wave_min(amax);
    if (mcount > 0.0) {
      const double mua = (wsum(c0) + amax * (wsum(c1) + amax * wsum(c2))) / mcount;
      const double r = fmax(0.0, fmin(1.0, mua / mu));
      sigmu = r * r * r * mu;
    } else {
      sigmu = 0.0;
    }

    MPCQP_PCLK(1);
    // ==== pass 3: per stage the corrector right-hand side (-> GA), then the
    // backward chain (quad 0)
    for (int k = qd; k < N; k += kQuads) {
      auto rhs = [&](double vj, double dva, double lo, double hi, double l, double lu, double g) {
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
                            at.r(k, L::HI + NU), at.r(k, L::LL + NU), at.r(k, L::LU + NU),
                            at.r(k, L::GA + NU));
      if (ou) {
        const double gum = rhs(at.r(k, L::U), at.r(k, L::DUA), at.r(k, L::LO), at.r(k, L::HI),
                               at.r(k, L::LL), at.r(k, L::LU), at.r(k, L::GA));
        at.r(k, L::GA) = gum;
      }
      at.r(k, L::GA + NU) = gx;
    }
    wave_lds_sync();
#ifndef MPCQP_RICCATI_QUAD
    rhs_mfma<L::GA + NU, L::GA>(W, N);
    wave_lds_sync();
    for (int k = qd; k < N; k += kQuads) rhs_kk_stage<L::GA>(at, k, i);
#else
    if (q0) rhs_sweep_q<L::GA + NU, L::GA>(at, N, i);
#endif
    wave_lds_sync();

    MPCQP_PCLK(2);
    // ========== pass 4: the corrector's forward sweep (quad 0), then per stage
#ifndef MPCQP_RICCATI_QUAD
    forward_mfma<L::DX>(W, N);
    wave_lds_sync();
#else
    if (q0)
      forward_q(at, N, i, [&](int k, const double (&du)[2], double dxn, const double (&)[4]) {
        at.r(k, L::DX) = dxn;
        if (ou) at.r(k, L::DU) = sel2(du, i);
      });
    wave_lds_sync();
#endif
    amax = 1.0;
    for (int k = qd; k < N; k += kQuads) {
#ifndef MPCQP_RICCATI_QUAD
      if (ou) at.r(k, L::DU) = du_of_stage<L::DX>(at, k, i);
#endif
      const double dxn = at.r(k, L::DX);
      double s = at.r(k, L::PV);
#pragma unroll
      for (int j = 0; j < 4; ++j) s = fma(at.p(k, L::PP, j), at(k, L::DX + j), s);
      at.r(k, L::DPI) = s;
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
        comp(at.r(k, L::U), at.r(k, L::DU), at.r(k, L::DUA), at.r(k, L::LO), at.r(k, L::HI),
             at.r(k, L::LL), at.r(k, L::LU));
    }
    alpha = fmin(1.0, 0.995 * wave_min(amax));
    wave_lds_sync();
    MPCQP_PCLK(3);
  }
}

}  // namespace ipmw
}  // namespace mpcqp
