// sqp_solve.hip -- mpcqp_bicycle_sqp_solve: a whole MPCController.solve
// (session_4/main.py:115-116, the NLP of main.py:41-113) per instance in ONE
// launch.  The batched SQP of mpc.SqpSolver.iterate is four launches per
// iteration over the whole batch (re-linearisation, Hessian, interior-point
// QP, step), so every iteration lasts as long as its slowest instance's QP,
// and an iteration with 50 instances still iterating costs as much as one
// with 4096 (profiles/r05/sqp_iters_nlp.txt: half the nlp step).  Here one
// single-wave workgroup runs one instance's iterations back to back:
//   1. rollout of U and the per-stage linearisation A_k, B_k, c_k;
//   2. the stage Hessians H2_k, q2_k (exact-Hessian iterations);
//   3. the QP on the interior point, the horizon in LDS (ipmw::solve_wave:
//      ipmq::solve_quad's algorithm with the per-stage work on all 16 quads
//      and the Riccati chains on one);
//   4. the merit line search, update and KKT residual (sqp_step_one, the
//      body of mpcqp_bicycle_sqp_step)
// until the KKT residual is below tol or max_iter iterations.  The launch
// lasts as long as the slowest instance's own solve, and workgroups that
// finish free their CU slot for the next ones (one workgroup per instance:
// the dispatcher balances the load, no atomics).  Same device functions as
// the four-launch iteration, so the iterates are those of SqpSolver.iterate
// with the linearisation of mpcqp_bicycle_linearise.
//
// Lanes: the whole wave.  Stage k's trig terms, Jacobians and Hessian on lane
// k; the QP's per-stage work on quad k % 16; the scalar scans on lane 0.
// Data between the phases goes through the caller's workspace (HBM) with a
// workgroup-scope fence after each phase (one wave: no barrier needed).
#include <algorithm>
#include <cstdlib>

#include "sqp_core.hpp"

#define MPCQP_HD __host__ __device__
// the SQP's QPs end their polish as soon as a step passes the final test (from
// the second step on; ipm_quad.hpp): A/B on the nlp line (tools/sqp_knobs.py,
// libmpcqp_pe1): sum of instance times -7 %, launch 291 -> 249 ms, the same
// converged set and fixture optima, 16.79 -> 17.09 SQP iterations on average
#ifndef MPCQP_POLISH_EARLY
#define MPCQP_POLISH_EARLY 1
#endif
#include "ipm_lane.hpp"
#include "ipm_quad.hpp"
// the QPs on the whole wave (ipm_wave.hpp: per-stage work on 16 quads, the
// Riccati chains on one): A/B on the nlp line (tools/sqp_knobs.py, the quad
// solver built with -DMPCQP_IPM_QUAD): sum of instance times 113.4 -> 73.8 s
// with the interior point alone, launch 259 -> 170 ms, the same fixture optima
#ifndef MPCQP_IPM_QUAD
#define MPCQP_IPM_WAVE 1
#include "ipm_wave.hpp"
#endif

namespace mpcqp {

// Hessian of the QPs: Gauss-Newton (none), the exact Lagrangian curvature
// projected per stage in PROJ mode ("exact"), or never projected ("exact-raw")
enum SqpHessian { kHessGN = MPCQP_SQP_HESS_GN, kHessExact = MPCQP_SQP_HESS_EXACT, kHessRaw = MPCQP_SQP_HESS_RAW };

struct SqpSolveArgs {
  SqpArgs s;            // the step: weights, bounds, U, y, pi, X, rho, kkt, mu, flags, fix
  ipm::Args<double> q;  // the QP: stage data and outputs in the workspace
  int max_iter, hmode;
  // polish a QP first on the previous QP's active set (MPCQP_SQP_WARM): 0 never,
  // 1 Gauss-Newton QPs, 2 those and exact-Hessian ones once kkt < warm_kkt
  // (MPCQP_SQP_WARM_KKT), 3 always
  int warm;
  double warm_kkt;
  double fix_rho, eps;  // proximal curvature of held inputs, projection floor
  double* Xr;           // (batch, N+1, 4): rollout states of the linearisation
  // per-instance timing of the launch (the workspace's last region, read by
  // tools/sqp_latency.py): s_memrealtime ticks (100 MHz) in all and in the
  // QPs, interior-point iterations, SQP iterations
  int64_t* stats;
};

// workspace regions (doubles per instance): A, B, c, H2, q2, Xr, z, y, pi,
// lam_u, X of the QP; then the QP's int32 status per instance
constexpr int kWsPerStage = 16 + 8 + 4 + 36 + 6 + 4 + 2 + 4 + 4 + 2 + 4;

__device__ __forceinline__ void wg_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// ------------------------------------------------- wave-parallel FE pieces
// The forward-Euler model splits into per-stage trig terms and cheap scalar
// recurrences: beta_k = atan(k tan delta_k) and sin/cos beta_k depend on u_k
// alone; psi_{k+1} = psi_k + ts v_k / l_r sin beta_k and v_{k+1} = v_k +
// ts (acc a_k - fric v_k) need no trig; sin/cos(psi_k + beta_k) then come
// per stage again, and p_x, p_y are running sums.  So a rollout is two trig
// rounds on one lane per stage and three short serial scans on lane 0 --
// every expression written as bike_pt / bike_step write it, so the rollout
// is bit-identical to model_step's.  Per-stage scratch in LDS after the QP's
// workspace (kScr doubles per stage, N + 1 stages, then the broadcast slots).
// the step's serial sweeps read their operands from the QP's LDS workspace
// (dead between QPs except the active flags GA): A_k, B_k in the stage-data
// fields DA, DB (the QP's own copy of the linearisation, then the new one
// from fe_linearise_wave), the multipliers y_k in DX
constexpr int kQF = ipm::Layout<4, 2>::F, kQA = ipm::Layout<4, 2>::DA, kQB = ipm::Layout<4, 2>::DB;
constexpr int kQY = ipm::Layout<4, 2>::DX;
constexpr int kScr = 14;
enum { kU0 = 0, kU1, kBeta, kSb, kPx, kPy, kPsi, kV, kSt, kCt, kTJ, kTV, kL0, kL1 };

__device__ __forceinline__ double* scr_at(double* scr, int k) { return scr + k * kScr; }

// Rollout of U + alpha d (use_d; d = sqp_dir) or of U; the states of stage k
// land in scr (kPx, kPy, kPsi, kV) and, when X != nullptr, in X ((N+1) x 4,
// global); returns 1/2 J and the state-box violation (merit_at's sums, in
// its order) on every lane.
__device__ __forceinline__ Merit fe_merit_wave(const SqpArgs& a, int64_t b, double alpha, bool use_d, double* X,
                               double* scr, int lane) {
  const int N = a.N;
  const Bike& p = a.p;
  const double* U = a.U + b * N * 2;
  const double kk = p.k();
  for (int k = lane; k < N; k += kWave) {
    double u0 = U[2 * k], u1 = U[2 * k + 1];
    if (use_d) {
      u0 = fma(alpha, sqp_dir(a, b, 2 * k), u0);
      u1 = fma(alpha, sqp_dir(a, b, 2 * k + 1), u1);
    }
    const double t = tan(u1);
    const double beta = atan(kk * t);
    double sb, cb;
    sincos(beta, &sb, &cb);
    double* q = scr_at(scr, k);
    q[kU0] = u0; q[kU1] = u1; q[kBeta] = beta; q[kSb] = sb;
  }
  wave_lds_sync();
  if (lane == 0) {  // psi and v (bike_step's xn[2], xn[3])
    double x2 = a.x0[b * a.sX0 + 2], x3 = a.x0[b * a.sX0 + 3];
    for (int k = 0; k < N; ++k) {
      double* q = scr_at(scr, k);
      q[kPsi] = x2;
      q[kV] = x3;
      const double v = x3;
      const double n2 = x2 + p.ts * v / p.lr * q[kSb];
      const double n3 = x3 + p.ts * (p.acc * q[kU0] - p.fric * v);
      x2 = n2;
      x3 = n3;
    }
    scr_at(scr, N)[kPsi] = x2;
    scr_at(scr, N)[kV] = x3;
  }
  wave_lds_sync();
  for (int k = lane; k < N; k += kWave) {
    double* q = scr_at(scr, k);
    double st, ct;
    sincos(q[kPsi] + q[kBeta], &st, &ct);
    q[kSt] = st;
    q[kCt] = ct;
  }
  wave_lds_sync();
  if (lane == 0) {  // p_x, p_y (xn[0], xn[1])
    double x0 = a.x0[b * a.sX0], x1 = a.x0[b * a.sX0 + 1];
    for (int k = 0; k < N; ++k) {
      double* q = scr_at(scr, k);
      q[kPx] = x0;
      q[kPy] = x1;
      const double v = q[kV];
      const double n0 = x0 + p.ts * v * q[kCt];
      const double n1 = x1 + p.ts * v * q[kSt];
      x0 = n0;
      x1 = n1;
    }
    scr_at(scr, N)[kPx] = x0;
    scr_at(scr, N)[kPy] = x1;
  }
  wave_lds_sync();
  // per-stage merit terms, and the states out
  for (int k = lane; k <= N; k += kWave) {
    const double* q = scr_at(scr, k);
    const double x[4] = {q[kPx], q[kPy], q[kPsi], q[kV]};
    if (X) {
#pragma unroll
      for (int i = 0; i < 4; ++i) X[k * 4 + i] = x[i];
    }
    if (k < N) {
      const double u[2] = {q[kU0], q[kU1]};
      const double* q1 = scr_at(scr, k + 1);
      const double x1[4] = {q1[kPx], q1[kPy], q1[kPsi], q1[kV]};
      scr_at(scr, k)[kTJ] = 0.5 * (sq_form(a.Q, 4, x) + sq_form(a.R, 2, u));
      scr_at(scr, k)[kTV] = box_viol(a, b, k, x1);
    }
  }
  wave_lds_sync();
  double* bc = scr_at(scr, N + 1);
  if (lane == 0) {  // merit_at's running sums
    Merit m{0.0, 0.0};
    for (int k = 0; k < N; ++k) {
      m.J += scr_at(scr, k)[kTJ];
      m.viol += scr_at(scr, k)[kTV];
    }
    const double* q = scr_at(scr, N);
    const double xN[4] = {q[kPx], q[kPy], q[kPsi], q[kV]};
    m.J += 0.5 * sq_form(a.Qf, 4, xN);
    bc[0] = m.J;
    bc[1] = m.viol;
  }
  wave_lds_sync();
  return Merit{bc[0], bc[1]};
}

// A_k, B_k, c_k of every stage from the rollout in scr (model_step_jac at
// (x_k, u_k), as mpcqp_bicycle_linearise writes them), lane per stage.
__device__ __forceinline__ void fe_linearise_wave(const SqpArgs& a, int N, double* A, double* B, double* c,
                                  const double* scr, int lane, double* qlds = nullptr) {
  for (int k = lane; k < N; k += kWave) {
    const double* q = scr_at(const_cast<double*>(scr), k);
    const double x[4] = {q[kPx], q[kPy], q[kPsi], q[kV]};
    const double u[2] = {q[kU0], q[kU1]};
    double Aj[4][4], Bj[4][2], xn[4];
    model_step_jac(a.p, 0, x, u, xn, Aj, Bj);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double t = xn[i] - Bj[i][0] * u[0] - Bj[i][1] * u[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        A[k * 16 + i * 4 + j] = Aj[i][j];
        if (qlds) qlds[(size_t)k * kQF + kQA + i * 4 + j] = Aj[i][j];
        t -= Aj[i][j] * x[j];
      }
      B[k * 8 + i * 2] = Bj[i][0];
      B[k * 8 + i * 2 + 1] = Bj[i][1];
      c[k * 4 + i] = t;
    }
  }
}

// sqp_step_one on the whole wave for the forward-Euler model: the same line
// search, update, KKT residual and flags, with every rollout from
// fe_merit_wave and the per-stage work one lane per stage; the serial parts
// (the directional derivative's forward sensitivities, the adjoint) run on
// lane 0 from the stored Jacobians.  The Jacobians at the accepted point are
// the next iteration's linearisation: they overwrite A, B, c, and the
// function returns true when it wrote them.
#ifdef MPCQP_IPM_PASSCLK
#define MPCQP_STCLK(i) do { if (sclk) { const uint64_t _t = __builtin_amdgcn_s_memrealtime(); sclk[i] += _t - st_t; st_t = _t; } } while (0)
#else
#define MPCQP_STCLK(i) do { } while (0)
#endif
__device__ __forceinline__ bool sqp_step_wave(const SqpArgs& a, int64_t b, double* A, double* B, double* c,
                              double* scr, int lane, double* qlds, uint64_t* sclk = nullptr) {
#ifdef MPCQP_IPM_PASSCLK
  uint64_t st_t = __builtin_amdgcn_s_memrealtime();
#endif
  const int fl = a.flags[b];
  if (fl & kSqpDone) return false;
  const int N = a.N;
  if (a.qp_status && (a.qp_status[b] & 0xFF) != MPCQP_STATUS_OPTIMAL) {
    if (lane == 0) sqp_qp_failed(a, b, fl);
    return false;
  }
  double* U = a.U + b * N * 2;
  const double* yq = a.yq + b * N * 4;
  const double* piq = a.piq + b * N * 4;
  double* y = a.y + b * N * 4;
  double* pi = a.pi + b * N * 4;
  double* X = a.X + b * (N + 1) * 4;

  // ----------------------------------------- merit, directional derivative
  double ymax = 0.0, dmax = 0.0, umax = 0.0;
  for (int i = lane; i < 4 * N; i += kWave) ymax = fmax(ymax, fabs(yq[i]));
  for (int i = lane; i < 2 * N; i += kWave) {
    dmax = fmax(dmax, fabs(sqp_dir(a, b, i)));
    umax = fmax(umax, fabs(U[i]));
  }
  ymax = wave_max(ymax);
  dmax = wave_max(dmax);
  umax = wave_max(umax);
  const double rho = fmax(a.rho[b], 2.0 * ymax);
  const Merit m0 = fe_merit_wave(a, b, 0.0, false, nullptr, scr, lane);
  MPCQP_STCLK(0);
  // the direction into LDS beside U (scr: kL0, kL1 free until the adjoint)
  for (int k = lane; k < N; k += kWave) {
    scr_at(scr, k)[kL0] = sqp_dir(a, b, 2 * k);
    scr_at(scr, k)[kL1] = sqp_dir(a, b, 2 * k + 1);
  }
  wave_lds_sync();
  double* bc = scr_at(scr, N + 1);
  if (lane == 0) {  // D = d(1/2 J)/dU . d, sqp_step_one's loop on the QP's A_k, B_k (LDS)
    // the weights in registers: through the generic pointers the compiler
    // could not rule out that the loop's LDS traffic aliases them, and
    // reloaded them from global memory at every stage (15 us of the step)
    double Qr[16], Rr[4], Qfr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { Qr[i] = a.Q[i]; Qfr[i] = a.Qf[i]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) Rr[i] = a.R[i];
    double D = 0.0;
    double dx[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < N; ++k) {
      const double* q = scr_at(scr, k);
      const double x[4] = {q[kPx], q[kPy], q[kPsi], q[kV]};
      const double u[2] = {q[kU0], q[kU1]};
      const double d[2] = {q[kL0], q[kL1]};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) t = fma(Qr[i * 4 + j], x[j], t);
        D = fma(t, dx[i], D);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        double t = 0.0;
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) t = fma(Rr[r * 2 + q2], u[q2], t);
        D = fma(t, d[r], D);
      }
      const double* Ak = qlds + (size_t)k * kQF + kQA;
      const double* Bk = qlds + (size_t)k * kQF + kQB;
      double dxn[4];
      for (int i = 0; i < 4; ++i) {
        double s = Bk[i * 2] * d[0] + Bk[i * 2 + 1] * d[1];
        for (int j = 0; j < 4; ++j) s = fma(Ak[i * 4 + j], dx[j], s);
        dxn[i] = s;
      }
      for (int i = 0; i < 4; ++i) dx[i] = dxn[i];
    }
    const double* q = scr_at(scr, N);
    const double xN[4] = {q[kPx], q[kPy], q[kPsi], q[kV]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) t = fma(Qfr[i * 4 + j], xN[j], t);
      D = fma(t, dx[i], D);
    }
    bc[2] = D;
  }
  wave_lds_sync();
  MPCQP_STCLK(1);
  const double D = bc[2];
  const double phi0 = m0.J + rho * m0.viol;
  const double Dm = D - rho * m0.viol;

  // --------------------------- backtracking (quadratic interpolation), Armijo
  double alpha = 1.0;
  const double noise = 1e-14 * (1.0 + fabs(phi0));
  const int wd = (fl >> 4) & 0xF;
  const bool force = a.watchdog > 0 && (fl & kSqpExact) && wd >= a.watchdog;
  if (!force && dmax > 1e-14 * (1.0 + umax)) {
    for (int t = 0; t < 40; ++t) {
      const Merit m = fe_merit_wave(a, b, alpha, true, nullptr, scr, lane);
      const double phi = m.J + rho * m.viol;
      if (phi <= phi0 + 1e-4 * alpha * Dm + noise) break;
      const double den = 2.0 * (phi - phi0 - alpha * Dm);
      const double at = den > 0.0 ? -Dm * alpha * alpha / den : 0.5 * alpha;
      alpha = fmin(0.5 * alpha, fmax(0.1 * alpha, at));
      if (alpha < 1e-10) break;
    }
  }
  MPCQP_STCLK(2);
  // the update (inputs within 1e-9 of a bound put on it), elementwise
  for (int i = lane; i < 2 * N; i += kWave) {
    double u = fma(alpha, sqp_dir(a, b, i), U[i]);
    const int64_t o = b * a.sLb + i;
    if (a.lb && u <= a.lb[o] + 1e-9 * (1.0 + fabs(a.lb[o]))) u = a.lb[o];
    if (a.ub && u >= a.ub[o] - 1e-9 * (1.0 + fabs(a.ub[o]))) u = a.ub[o];
    U[i] = u;
  }
  for (int i = lane; i < 4 * N; i += kWave) {
    const double yi = fma(alpha, yq[i] - y[i], y[i]);
    y[i] = yi;
    qlds[(size_t)(i >> 2) * kQF + kQY + (i & 3)] = yi;
    pi[i] = fma(alpha, piq[i] - pi[i], pi[i]);
  }
  wg_fence();

  MPCQP_STCLK(3);
  // ------------------------------------------ KKT residual at the new point
  fe_merit_wave(a, b, 0.0, false, X, scr, lane);
  fe_linearise_wave(a, N, A, B, c, scr, lane, qlds);
  wg_fence();
  MPCQP_STCLK(4);
  if (lane == 0) {  // the adjoint lambda_{k+1} of every stage, sqp_step_one's order
    double Qr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Qr[i] = a.Q[i];
    double lam[4];
    const double* q = scr_at(scr, N);
    const double xN[4] = {q[kPx], q[kPy], q[kPsi], q[kV]};
    for (int i = 0; i < 4; ++i) {
      double s = qlds[(size_t)(N - 1) * kQF + kQY + i];
      for (int j = 0; j < 4; ++j) s = fma(a.Qf[i * 4 + j], xN[j], s);
      lam[i] = s;
    }
    for (int k = N - 1; k >= 0; --k) {
      double* qk = scr_at(scr, k);
      qk[kL0] = lam[0];  // (lambda_{k+1} in four slots: kL0, kL1, kTJ, kTV)
      qk[kL1] = lam[1];
      qk[kTJ] = lam[2];
      qk[kTV] = lam[3];
      if (k > 0) {
        const double x[4] = {qk[kPx], qk[kPy], qk[kPsi], qk[kV]};
        const double* Ak = qlds + (size_t)k * kQF + kQA;
        double ln[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double s = qlds[(size_t)(k - 1) * kQF + kQY + i];
#pragma unroll
          for (int j = 0; j < 4; ++j) s = fma(Qr[i * 4 + j], x[j], s);
          for (int j = 0; j < 4; ++j) s = fma(Ak[j * 4 + i], lam[j], s);
          ln[i] = s;
        }
        for (int i = 0; i < 4; ++i) lam[i] = ln[i];
      }
    }
  }
  wave_lds_sync();
  MPCQP_STCLK(5);
  double r = 0.0;
  for (int k = lane; k < N; k += kWave) {
    const double* qk = scr_at(scr, k);
    const double lam[4] = {qk[kL0], qk[kL1], qk[kTJ], qk[kTV]};
    const double u[2] = {U[2 * k], U[2 * k + 1]};
    const double* Bk = B + k * 8;
    int32_t fb = 0;
    for (int q = 0; q < 2; ++q) {
      double g = 0.0;
      for (int j = 0; j < 2; ++j) g = fma(a.R[q * 2 + j], u[j], g);
      for (int i = 0; i < 4; ++i) g = fma(Bk[i * 2 + q], lam[i], g);
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
    const double* q1 = scr_at(const_cast<double*>(scr), k + 1);
    const double xk1[4] = {q1[kPx], q1[kPy], q1[kPsi], q1[kV]};
    for (int i = 0; i < 4; ++i) {
      const int64_t o = b * a.sXb + (int64_t)k * 4 + i;
      const double hi = a.xhi ? a.xhi[o] : Lim<double>::inf();
      const double lo = a.xlo ? a.xlo[o] : -Lim<double>::inf();
      const double yi = y[k * 4 + i];
      r = fmax(r, fmax(xk1[i] - hi, lo - xk1[i]));
      if (yi > 0.0) r = fmax(r, fmin(yi, hi - xk1[i]));
      if (yi < 0.0) r = fmax(r, fmin(-yi, xk1[i] - lo));
    }
  }
  r = wave_max(r);
  if (!(r == r)) r = Lim<double>::inf();
  if (lane == 0) sqp_finish(a, b, fl, alpha, r, rho, force, wd);
  MPCQP_STCLK(6);
  return true;
}
#undef MPCQP_STCLK


// Per-instance clocks of a launch (the workspace's stats region).
struct SolveClock {
  uint64_t tqp = 0;
  int64_t ipm_its = 0, warm_hits = 0, sqp_its = 0;
#ifdef MPCQP_IPM_PASSCLK
  // timing builds: passes 1-4, polish, failed factorisations, start, warm
  // polish, and pass 1's parts 1a, 1b, 1c (index 0 then keeps its reductions)
  // + the SQP's own phases: linearisation, Hessians + stage-in, the step
  // + the step's parts: merit at U, directional derivative, line search,
  // update, merit + linearisation at the new point, adjoint, KKT + flags
  uint64_t pass[22] = {};
#endif
};

// Up to max_iter SQP iterations of instance b, to its own convergence: the
// body of both kernels below.  All 64 lanes (the QP on lanes 0..3).
__device__ __forceinline__ void sqp_solve_instance(const SqpSolveArgs& g, int64_t b, int max_iter,
                                                   double* ipm_lds, double* scr, int lane,
                                                   SolveClock& clk) {
  const SqpArgs& s = g.s;
  const int N = s.N;
  const Bike p = s.p;
  double* A = const_cast<double*>(g.q.A) + b * N * 16;
  double* B = const_cast<double*>(g.q.B) + b * N * 8;
  double* c = const_cast<double*>(g.q.c) + b * N * 4;
  double* X = s.X + b * (N + 1) * 4;
  const double* U = s.U + b * N * 2;
  const bool fe = s.integ == MPCQP_MODEL_FE;
  bool lin = false;   // A, B, c and X hold the linearisation at the current U
  bool warm = false;  // the last QP ended polished: its active set is in LDS
  int it = 0;
#ifdef MPCQP_IPM_PASSCLK
  uint64_t ph_t = __builtin_amdgcn_s_memrealtime();
#define MPCQP_SCLK(i) do { const uint64_t _t = __builtin_amdgcn_s_memrealtime(); clk.pass[i] += _t - ph_t; ph_t = _t; } while (0)
#else
#define MPCQP_SCLK(i) do { } while (0)
#endif
  for (; it < max_iter; ++it) {
    if (s.flags[b] & kSqpDone) break;
    MPCQP_SCLK(14);
    // ------------------------------------------- 1. rollout + linearisation
    if (fe) {
      if (!lin) {
        fe_merit_wave(s, b, 0.0, false, X, scr, lane);
        fe_linearise_wave(s, N, A, B, c, scr, lane);
        wg_fence();
        lin = true;
      }
    } else {  // RK4: the serial rollout on every lane, stage k's Jacobians on lane k
      double x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) X[i] = x[i] = s.x0[b * s.sX0 + i];
      for (int k = 0; k < N; ++k) {
        const double u[2] = {U[2 * k], U[2 * k + 1]};
        double xn[4];
        model_step(p, s.integ, x, u, xn);
#pragma unroll
        for (int i = 0; i < 4; ++i) X[(k + 1) * 4 + i] = x[i] = xn[i];
      }
      for (int k = lane; k < N; k += kWave) {
        const double* xk = X + k * 4;
        const double u[2] = {U[2 * k], U[2 * k + 1]};
        double Aj[4][4], Bj[4][2], xn[4];
        model_step_jac(p, s.integ, xk, u, xn, Aj, Bj);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double t = xn[i] - Bj[i][0] * u[0] - Bj[i][1] * u[1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            A[k * 16 + i * 4 + j] = Aj[i][j];
            t -= Aj[i][j] * xk[j];
          }
          B[k * 8 + i * 2] = Bj[i][0];
          B[k * 8 + i * 2 + 1] = Bj[i][1];
          c[k * 4 + i] = t;
        }
      }
      wg_fence();
    }
    MPCQP_SCLK(11);
    // ------------------------------------------------ 2. stage Hessians
    if (g.hmode != kHessGN) {
      const bool cvx = g.hmode == kHessExact;
      // the projection's work matrices in stage k's slice of the QP's LDS
      // workspace, dead between QPs except the active flags GA the warm
      // polish keeps: fields U..PV (69 doubles) and DA..QU (55)
      using LQ = ipm::Layout<4, 2>;
      static_assert(LQ::GA >= 36 && LQ::LO - LQ::DA >= 36, "projection scratch");
      for (int k = lane; k < N; k += kWave)
        hess_stage(b, N, k, p, s.integ, s.X, s.U, s.pi, s.flags, s.mu, s.fix, g.fix_rho,
                   cvx ? s.Q : nullptr, cvx ? s.R : nullptr, g.eps,
                   const_cast<double*>(g.q.H2) + (b * N + k) * 36,
                   const_cast<double*>(g.q.q2) + (b * N + k) * 6,
                   ipm_lds + (size_t)k * LQ::F + LQ::DA, ipm_lds + (size_t)k * LQ::F);
    }
    wg_fence();
    // ------------------------------------------------------------- 3. QP
    // (the whole wave, ipm_wave.hpp; the warm polish where the QP's solution is the one the
    // interior point would find: Gauss-Newton QPs are convex, a unique
    // solution; an exact-Hessian QP may have several KKT points, and far from
    // the NLP's solution the previous active set can pick another one than
    // the interior point -- which changes the local minimum the SQP ends in
    // -- so there only once the KKT residual is below warm_kkt)
    const uint64_t q0 = __builtin_amdgcn_s_memrealtime();
    {  // the QP's stage data into LDS, one quad per stage (solve_quad's copy, in parallel)
      const ipmq::WsQ<1> at(ipm_lds, lane & 3);
      for (int k = lane >> 2; k < N; k += kWave / 4) ipmq::stage_in_q(g.q, (int)b, at, lane & 3, k);
    }
    wave_lds_sync();
    MPCQP_SCLK(12);
#ifdef MPCQP_IPM_WAVE
    {
      const int fl = s.flags[b];
      const bool use_warm = warm && (g.warm == 3 || (g.warm >= 1 && !(fl & kSqpExact)) ||
                                     (g.warm == 2 && s.kkt[b] < g.warm_kkt));
      warm = ipmw::solve_wave<double>(g.q, (int)b, ipm_lds, use_warm,
#ifdef MPCQP_IPM_PASSCLK
                                      clk.pass
#else
                                      nullptr
#endif
      );
      if (lane == 0)
        clk.warm_hits += (use_warm && warm && ((g.q.status[b] >> 8) & 0xFFFF) == 0) ? 1 : 0;
    }
#else
    if (lane < 4) {
      const int fl = s.flags[b];
      const bool use_warm = warm && (g.warm == 3 || (g.warm >= 1 && !(fl & kSqpExact)) ||
                                     (g.warm == 2 && s.kkt[b] < g.warm_kkt));
      warm = ipmq::solve_quad<double, 1>(g.q, (int)b, ipm_lds, use_warm,
#ifdef MPCQP_IPM_PASSCLK
                                         clk.pass,
#else
                                         nullptr,
#endif
                                         true);
      clk.warm_hits += (use_warm && warm && ((g.q.status[b] >> 8) & 0xFFFF) == 0) ? 1 : 0;
    }
#endif
    wg_fence();
    clk.tqp += __builtin_amdgcn_s_memrealtime() - q0;
    clk.ipm_its += (g.q.status[b] >> 8) & 0xFFFF;
#ifdef MPCQP_IPM_PASSCLK
    ph_t = __builtin_amdgcn_s_memrealtime();
#endif
    // ----------------------------------------------------------- 4. step
    if (fe) {
#ifdef MPCQP_IPM_PASSCLK
      sqp_step_wave(s, b, A, B, c, scr, lane, ipm_lds, clk.pass + 15);
#else
      sqp_step_wave(s, b, A, B, c, scr, lane, ipm_lds);
#endif
    } else if (lane == 0) {
      sqp_step_one(s, b);
    }
    wg_fence();
    MPCQP_SCLK(13);
  }
  clk.sqp_its += it;
#undef MPCQP_SCLK
}

__device__ __forceinline__ void write_clock(const SqpSolveArgs& g, int64_t b, uint64_t t0,
                                            const SolveClock& clk, int lane) {
  if (lane == 0) {
    int64_t* st = g.stats + b * 4;
    st[0] = (int64_t)(__builtin_amdgcn_s_memrealtime() - t0);
    st[1] = (int64_t)clk.tqp;
    st[2] = clk.ipm_its;
    st[3] = clk.sqp_its | (clk.warm_hits << 32);
#ifdef MPCQP_IPM_PASSCLK
    // (the workspace region of g.Xr, unused by sqp_solve_kernel)
    for (int i = 0; i < 22; ++i) reinterpret_cast<int64_t*>(g.Xr)[b * 22 + i] = (int64_t)clk.pass[i];
#endif
  }
}

__global__ __launch_bounds__(64, 1) void sqp_solve_kernel(SqpSolveArgs g) {
  extern __shared__ __attribute__((aligned(16))) double ipm_lds[];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  double* scr = ipm_lds + (size_t)g.s.N * ipm::Layout<4, 2>::F;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  SolveClock clk;
  sqp_solve_instance(g, b, g.max_iter, ipm_lds, scr, lane, clk);
  write_clock(g, b, t0, clk, lane);
}

// ------------------------------------------------ the whole closed loop
// rcracers.simulate(x0, dynamics, n_steps, policy=controller) of main.py:
// 270-271 (session4_sol.py:458,465) for one instance per workgroup: per
// sample t the controller's SQP from the shifted previous solution
// (sqp_solve_instance, up to iters_first / iters iterations), the
// ControllerLog record (session_2/log.py:8-12), the plant x_{t+1} =
// F(x_t, u_0), and the warm-start shift -- ClosedLoop._step's sequence, in
// one launch.  Every instance runs its own episode: the launch lasts as long
// as the slowest episode, not the sum over samples of each sample's slowest
// solve.
struct SqpLoopArgs {
  int T, iters_first, iters;
  double mu0;
  Bike plant;
  int plant_integ, substeps;
  double* xs;           // (T+1, batch, 4); xs[0] given
  double* us;           // (T, batch, 2)
  int8_t* success;      // (T, batch)
  int32_t* iters_out;   // (T, batch)
  double* state_pred;   // (T, batch, N+1, 4)
  double* input_pred;   // (T, batch, N, 2)
  double* x0buf;        // (batch, 4): the sample's x0 (g.s.x0, g.q.x0)
};

__global__ __launch_bounds__(64, 1) void sqp_loop_kernel(SqpSolveArgs g, SqpLoopArgs e) {
  extern __shared__ __attribute__((aligned(16))) double ipm_lds[];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const SqpArgs& s = g.s;
  const int N = s.N, batch = s.batch;
  double* scr = ipm_lds + (size_t)N * ipm::Layout<4, 2>::F;
  double* U = s.U + b * N * 2;
  double* y = s.y + b * N * 4;
  double* pi = s.pi + b * N * 4;
  const double* X = s.X + b * (N + 1) * 4;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  SolveClock clk;
  for (int t = 0; t < e.T; ++t) {
    const double* xt = e.xs + ((int64_t)t * batch + b) * 4;
    if (lane < 4) e.x0buf[b * 4 + lane] = xt[lane];
    wg_fence();
    sqp_solve_instance(g, b, t == 0 ? e.iters_first : e.iters, ipm_lds, scr, lane, clk);
    // ControllerLog: solver_success, the iteration count, [x_t; X], U
    const int fl = s.flags[b];
    const int64_t tb = (int64_t)t * batch + b;
    if (lane == 0) {
      e.success[tb] = ((fl & kSqpDone) && !(fl & kSqpFail)) ? 1 : 0;
      e.iters_out[tb] = (fl >> 8) & 0xFFFF;
    }
    for (int j = lane; j < (N + 1) * 4; j += kWave) e.state_pred[tb * (N + 1) * 4 + j] = X[j];
    for (int j = lane; j < N * 2; j += kWave) e.input_pred[tb * N * 2 + j] = U[j];
    // the plant with u_t = U[0] (mpcqp_bicycle_plant)
    if (lane == 0) {
      double x[4] = {xt[0], xt[1], xt[2], xt[3]};
      const double u[2] = {U[0], U[1]};
      plant_step(e.plant, e.plant_integ, e.substeps, x, u);
      double* xn = e.xs + ((int64_t)(t + 1) * batch + b) * 4;
      for (int i = 0; i < 4; ++i) xn[i] = x[i];
      e.us[tb * 2] = u[0];
      e.us[tb * 2 + 1] = u[1];
    }
    // the warm start of the next sample (mpcqp_sqp_shift): every per-stage
    // array one stage forward, the last stage repeated; the SQP state reset
    double su[2] = {0.0, 0.0}, sy[4] = {0.0, 0.0, 0.0, 0.0}, sp[4] = {0.0, 0.0, 0.0, 0.0};
    const int k = lane;
    const bool mv = k + 1 < N;
    if (mv) {
      for (int j = 0; j < 2; ++j) su[j] = U[(k + 1) * 2 + j];
      for (int j = 0; j < 4; ++j) {
        sy[j] = y[(k + 1) * 4 + j];
        sp[j] = pi[(k + 1) * 4 + j];
      }
    }
    wg_fence();
    if (mv) {
      for (int j = 0; j < 2; ++j) U[k * 2 + j] = su[j];
      for (int j = 0; j < 4; ++j) {
        y[k * 4 + j] = sy[j];
        pi[k * 4 + j] = sp[j];
      }
    }
    if (lane == 0) {
      s.flags[b] = 0;
      s.rho[b] = 0.0;
      s.mu[b] = e.mu0;
      s.kkt[b] = Lim<double>::inf();
    }
    wg_fence();
  }
  write_clock(g, b, t0, clk, lane);
}

}  // namespace mpcqp

using namespace mpcqp;

extern "C" size_t mpcqp_bicycle_sqp_solve_workspace(int batch, int N) {
  if (batch <= 0 || N < 1) return 0;
  return (size_t)batch * ((size_t)N * kWsPerStage + 4 + 4) * sizeof(double) + (size_t)batch * 4 +
         256;
}

// The arguments both entry points share (checks, the step's and the QP's
// argument blocks, the workspace regions); x0 with stride strideX0.
static int setup_solve(const char* fn, SqpSolveArgs& g, int batch, int N, double ts,
                       const double* params, int integrator, int hessian, const void* x0,
                       int64_t strideX0, const void* Q, const void* R, const void* Qf,
                       const void* xlo, const void* xhi, int64_t strideXb, const void* lb,
                       const void* ub, int64_t strideLb, void* U, void* y, void* pi, void* X,
                       double* rho, double* kkt, double* mu, int32_t* flags, int32_t* fix,
                       void* lam_u, int32_t* qp_status, int max_iter, int qp_max_iter, double tol,
                       void* ws, size_t ws_bytes, size_t& lds) {
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1 && max_iter >= 0, "%s: bad sizes", fn);
  MPCQP_CHECK_ARG(params && x0 && Q && R && Qf && U && y && pi && X && rho && kkt && mu && flags,
                  "%s: null pointer", fn);
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0, "%s: bad axle lengths", fn);
  MPCQP_CHECK_ARG(strideX0 >= 4 && strideXb >= 0 && strideLb >= 0, "%s: bad strides", fn);
  MPCQP_CHECK_ARG(integrator == MPCQP_MODEL_FE || integrator == MPCQP_MODEL_RK4,
                  "%s: integrator %d", fn, integrator);
  MPCQP_CHECK_ARG(hessian >= kHessGN && hessian <= kHessRaw, "%s: hessian mode %d", fn, hessian);
  const size_t need = mpcqp_bicycle_sqp_solve_workspace(batch, N);
  MPCQP_CHECK_ARG(batch == 0 || (ws && ws_bytes >= need), "%s: workspace %zu bytes < %zu", fn,
                  ws_bytes, need);
  // the QP's workspace, then the step's per-stage scratch (N + 2 rows)
  lds = ((size_t)N * ipm::Layout<4, 2>::F + (size_t)(N + 2) * kScr) * sizeof(double);
  MPCQP_CHECK_ARG(lds <= 160 * 1024, "%s: N = %d exceeds the LDS horizon", fn, N);
  // ---- the step (mpcqp_bicycle_sqp_step's arguments)
  SqpArgs& a = g.s;
  a.batch = batch; a.N = N; a.p = bike_of(ts, params); a.integ = integrator;
  a.x0 = (const double*)x0; a.sX0 = strideX0;
  a.Q = (const double*)Q; a.R = (const double*)R; a.Qf = (const double*)Qf;
  a.xlo = (const double*)xlo; a.xhi = (const double*)xhi; a.sXb = strideXb;
  a.lb = (const double*)lb; a.ub = (const double*)ub; a.sLb = strideLb;
  a.U = (double*)U; a.y = (double*)y; a.pi = (double*)pi; a.X = (double*)X;
  a.rho = rho; a.kkt = kkt; a.mu = mu; a.flags = flags;
  // held inputs exist only for exact-Hessian QPs (the proximal term of the
  // Hessian); a Gauss-Newton controller passes no fix array
  a.fix = hessian == kHessGN ? nullptr : fix;
  a.tol = tol > 0 ? tol : 1e-9;
  sqp_knobs(a);
  // ---- workspace regions
  double* w = (double*)ws;
  const int64_t bN = (int64_t)batch * N;
  double* wA = w;                 w += bN * 16;
  double* wB = w;                 w += bN * 8;
  double* wc = w;                 w += bN * 4;
  double* wH = w;                 w += bN * 36;
  double* wq = w;                 w += bN * 6;
  double* wx0 = w;                w += bN * 4 + (int64_t)batch * 4;  // (the loop's x0 per sample)
  double* wz = w;                 w += bN * 2;
  double* wy = w;                 w += bN * 4;
  double* wpi = w;                w += bN * 4;
  double* wlu = lam_u ? (double*)lam_u : w;  w += bN * 2;
  double* wX = w;                 w += bN * 4;
  g.stats = (int64_t*)w;          w += (int64_t)batch * 4;  // (tools/sqp_latency.py reads it here)
  int32_t* wst = qp_status ? qp_status : (int32_t*)w;
  g.Xr = wx0;
  a.Z = wz; a.yq = wy; a.piq = wpi; a.qp_status = wst;
  // ---- the QP (mpc.SqpSolver.iterate's mpcqp_mpc_ipm call)
  ipm::Args<double>& q = g.q;
  q.batch = batch; q.nx = 4; q.nu = 2; q.N = N; q.tv = 1;
  q.max_iter = qp_max_iter > 0 ? qp_max_iter : 25;
  q.strict = 0;  // as many inertia corrections as the QP needs (SqpSolver.STRICT)
  // the first polish attempt: mu and the residuals below this
  // (MPCQP_SQP_MU_POLISH, an A/B knob)
  static const double mu_pol = [] {
    const char* e = getenv("MPCQP_SQP_MU_POLISH");
    return e ? atof(e) : 1e-6;
  }();
  q.tol = 1e-10; q.tol_mu = 1e-12; q.tol_polish = mu_pol; q.mu_polish = mu_pol;
  q.A = wA; q.sA = (int64_t)N * 16; q.B = wB; q.sB = (int64_t)N * 8; q.c = wc; q.sC = (int64_t)N * 4;
  q.Q = a.Q; q.sQ = 0; q.R = a.R; q.sR = 0; q.Qf = a.Qf; q.sQf = 0;
  q.x0 = a.x0; q.sX0 = strideX0;
  q.xlo = a.xlo; q.xhi = a.xhi; q.sXb = strideXb;
  q.lb = a.lb; q.sLb = strideLb; q.ub = a.ub; q.sUb = strideLb;
  q.U0 = nullptr; q.sU0 = 0;
  q.H2 = hessian == kHessGN ? nullptr : wH; q.sH2 = (int64_t)N * 36;
  q.q2 = hessian == kHessGN ? nullptr : wq; q.sq2 = (int64_t)N * 6;
  q.z = wz; q.y = wy; q.X = wX; q.lam_u = wlu; q.pi = wpi; q.status = wst;
  q.skip = nullptr; q.skip_mask = 0;
  q.ws = nullptr; q.list = nullptr; q.list_count = nullptr; q.list_begin = 0;
  static const int warm_qp = [] {
    const char* e = getenv("MPCQP_SQP_WARM");
    return e ? atoi(e) : 2;
  }();
  // 1e-2 (round 6, with the QP on the matrix cores; tools/sqp_knobs.py and the
  // loop line, profiles/r06/sqp_warm_kkt.txt): nlp instance time -3 %, loop
  // line +5 %, the same fixture optima; 1e-4 and 1e-6 lose 2-4 % / 10-30 %;
  // 1e-1 gains more but sends 8 of 4096 bench instances to higher-cost minima
  // (tools/sqp_minima.py; 1e-2: 2 instances, both to lower-cost ones)
  static const double warm_kkt = [] {
    const char* e = getenv("MPCQP_SQP_WARM_KKT");
    return e ? atof(e) : 1e-2;
  }();
  g.warm = warm_qp;
  g.warm_kkt = warm_kkt;
  g.max_iter = max_iter;
  g.hmode = hessian;
  g.fix_rho = fix_rho();
  g.eps = 1e-6;  // mpcqp_bicycle_hessian_convex's floor (batched.bicycle_hessian)
  return MPCQP_OK;
}

template <class K>
static int set_lds(K kern, size_t lds) {
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(sqp_solve)");
  }
  return MPCQP_OK;
}

extern "C" int mpcqp_bicycle_sqp_solve(int dtype, int batch, int N, double ts,
                                       const double* params, int integrator, int hessian,
                                       const void* x0, int64_t strideX0, const void* Q,
                                       const void* R, const void* Qf, const void* xlo,
                                       const void* xhi, int64_t strideXb, const void* lb,
                                       const void* ub, int64_t strideLb, void* U, void* y, void* pi,
                                       void* X, double* rho, double* kkt, double* mu,
                                       int32_t* flags, int32_t* fix, void* lam_u,
                                       int32_t* qp_status, int max_iter, int qp_max_iter,
                                       double tol, void* ws, size_t ws_bytes, void* stream) {
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "mpcqp_bicycle_sqp_solve: MPCQP_F64 only");
  SqpSolveArgs g{};
  size_t lds = 0;
  const int rc = setup_solve("mpcqp_bicycle_sqp_solve", g, batch, N, ts, params, integrator,
                             hessian, x0, strideX0, Q, R, Qf, xlo, xhi, strideXb, lb, ub, strideLb,
                             U, y, pi, X, rho, kkt, mu, flags, fix, lam_u, qp_status, max_iter,
                             qp_max_iter, tol, ws, ws_bytes, lds);
  if (rc != MPCQP_OK) return rc;
  if (batch == 0 || max_iter == 0) return MPCQP_OK;
  if (set_lds(sqp_solve_kernel, lds) != MPCQP_OK) return MPCQP_EHIP;
  hipLaunchKernelGGL(sqp_solve_kernel, dim3((unsigned)batch), dim3(64), lds, (hipStream_t)stream, g);
  MPCQP_CHECK_LAUNCH("sqp_solve_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_bicycle_mpc_loop(int dtype, int batch, int N, int T, double ts,
                                      const double* params, int integrator, int hessian,
                                      const double* plant_params, int plant, int substeps,
                                      const void* Q, const void* R, const void* Qf,
                                      const void* xlo, const void* xhi, int64_t strideXb,
                                      const void* lb, const void* ub, int64_t strideLb, void* U,
                                      void* y, void* pi, void* X, double* rho, double* kkt,
                                      double* mu, int32_t* flags, int32_t* fix, int iters_first,
                                      int iters, int qp_max_iter, double tol, double mu0, void* xs,
                                      void* us, void* success, int32_t* iters_out,
                                      void* state_prediction, void* input_prediction, void* ws,
                                      size_t ws_bytes, void* stream) {
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "mpcqp_bicycle_mpc_loop: MPCQP_F64 only");
  MPCQP_CHECK_ARG(T >= 0 && iters_first >= 0 && iters >= 0 && N <= kWave,
                  "mpcqp_bicycle_mpc_loop: bad sizes (T=%d, N=%d <= 64)", T, N);
  MPCQP_CHECK_ARG(plant_params && plant_params[1] > 0 && plant_params[0] + plant_params[1] > 0,
                  "mpcqp_bicycle_mpc_loop: bad plant parameters");
  MPCQP_CHECK_ARG(plant >= MPCQP_PLANT_FE && plant <= MPCQP_PLANT_RK4_SUB &&
                      (plant != MPCQP_PLANT_RK4_SUB || substeps >= 1),
                  "mpcqp_bicycle_mpc_loop: plant %d / substeps %d", plant, substeps);
  MPCQP_CHECK_ARG(xs && us && success && iters_out && state_prediction && input_prediction,
                  "mpcqp_bicycle_mpc_loop: null output");
  SqpSolveArgs g{};
  size_t lds = 0;
  // the sample's x0 lives in the workspace (written per sample by the kernel)
  double* x0buf = (double*)ws + (int64_t)batch * N * (16 + 8 + 4 + 36 + 6);
  const int rc = setup_solve("mpcqp_bicycle_mpc_loop", g, batch, N, ts, params, integrator,
                             hessian, x0buf, 4, Q, R, Qf, xlo, xhi, strideXb, lb, ub, strideLb,
                             U, y, pi, X, rho, kkt, mu, flags, fix, nullptr, nullptr,
                             std::max(iters_first, iters), qp_max_iter, tol, ws, ws_bytes, lds);
  if (rc != MPCQP_OK) return rc;
  if (batch == 0 || T == 0) return MPCQP_OK;
  SqpLoopArgs e{};
  e.T = T; e.iters_first = iters_first; e.iters = iters; e.mu0 = mu0;
  e.plant = bike_of(ts, plant_params); e.plant_integ = plant; e.substeps = substeps;
  e.xs = (double*)xs; e.us = (double*)us; e.success = (int8_t*)success; e.iters_out = iters_out;
  e.state_pred = (double*)state_prediction; e.input_pred = (double*)input_prediction;
  e.x0buf = x0buf;
  if (set_lds(sqp_loop_kernel, lds) != MPCQP_OK) return MPCQP_EHIP;
  hipLaunchKernelGGL(sqp_loop_kernel, dim3((unsigned)batch), dim3(64), lds, (hipStream_t)stream, g, e);
  MPCQP_CHECK_LAUNCH("sqp_loop_kernel");
  return MPCQP_OK;
}
