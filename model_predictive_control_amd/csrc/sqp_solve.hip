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
//   3. the QP on the interior point, four lanes per instance, the horizon in
//      LDS (ipmq::solve_quad, the kernel of mpcqp_mpc_ipm);
//   4. the merit line search, update and KKT residual (sqp_step_one, the
//      body of mpcqp_bicycle_sqp_step)
// until the KKT residual is below tol or max_iter iterations.  The launch
// lasts as long as the slowest instance's own solve, and workgroups that
// finish free their CU slot for the next ones (one workgroup per instance:
// the dispatcher balances the load, no atomics).  Same device functions as
// the four-launch iteration, so the iterates are those of SqpSolver.iterate
// with the linearisation of mpcqp_bicycle_linearise.
//
// Lanes: 0..3 (one DPP quad; 4..63 exit at once).  The rollout runs on every
// lane; stage k's Jacobians and Hessian on lane k % 4; the step on lane 0.
// Data between the phases goes through the caller's workspace (HBM) with a
// workgroup-scope fence after each phase (one wave: no barrier needed).
#include <algorithm>
#include <cstdlib>

#include "sqp_core.hpp"

#define MPCQP_HD __host__ __device__
#include "ipm_lane.hpp"
#include "ipm_quad.hpp"

namespace mpcqp {

// Hessian of the QPs: Gauss-Newton (none), the exact Lagrangian curvature
// projected per stage in PROJ mode ("exact"), or never projected ("exact-raw")
enum SqpHessian { kHessGN = MPCQP_SQP_HESS_GN, kHessExact = MPCQP_SQP_HESS_EXACT, kHessRaw = MPCQP_SQP_HESS_RAW };

struct SqpSolveArgs {
  SqpArgs s;            // the step: weights, bounds, U, y, pi, X, rho, kkt, mu, flags, fix
  ipm::Args<double> q;  // the QP: stage data and outputs in the workspace
  int max_iter, hmode;
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

__global__ __launch_bounds__(64, 1) void sqp_solve_kernel(SqpSolveArgs g) {
  extern __shared__ __attribute__((aligned(16))) double ipm_lds[];
  const int lane = threadIdx.x;
  if (lane >= 4) return;
  const int64_t b = blockIdx.x;
  const SqpArgs& s = g.s;
  const int N = s.N;
  const Bike p = s.p;
  double* A = const_cast<double*>(g.q.A) + b * N * 16;
  double* B = const_cast<double*>(g.q.B) + b * N * 8;
  double* c = const_cast<double*>(g.q.c) + b * N * 4;
  double* Xr = g.Xr + b * (N + 1) * 4;
  const double* U = s.U + b * N * 2;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t tqp = 0;
  int64_t ipm_its = 0;
  int it = 0;
  for (; it < g.max_iter; ++it) {
    if (s.flags[b] & kSqpDone) break;
    // ------------------------------------------- 1. rollout + linearisation
    {
      double x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) Xr[i] = x[i] = s.x0[b * s.sX0 + i];
      for (int k = 0; k < N; ++k) {
        const double u[2] = {U[2 * k], U[2 * k + 1]};
        double xn[4];
        model_step(p, s.integ, x, u, xn);
#pragma unroll
        for (int i = 0; i < 4; ++i) Xr[(k + 1) * 4 + i] = x[i] = xn[i];
      }
    }
    // every lane wrote the same rollout; stage k's data on lane k % 4 from
    // its own copy
    for (int k = lane; k < N; k += 4) {
      const double* x = Xr + k * 4;
      const double u[2] = {U[2 * k], U[2 * k + 1]};
      double Aj[4][4], Bj[4][2], xn[4];
      model_step_jac(p, s.integ, x, u, xn, Aj, Bj);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double t = xn[i] - Bj[i][0] * u[0] - Bj[i][1] * u[1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          A[k * 16 + i * 4 + j] = Aj[i][j];
          t -= Aj[i][j] * x[j];
        }
        B[k * 8 + i * 2] = Bj[i][0];
        B[k * 8 + i * 2 + 1] = Bj[i][1];
        c[k * 4 + i] = t;
      }
      if (g.hmode != kHessGN) {
        const bool cvx = g.hmode == kHessExact;
        hess_stage(b, N, k, p, s.integ, g.Xr, s.U, s.pi, s.flags, s.mu, s.fix, g.fix_rho,
                   cvx ? s.Q : nullptr, cvx ? s.R : nullptr, g.eps,
                   const_cast<double*>(g.q.H2) + (b * N + k) * 36,
                   const_cast<double*>(g.q.q2) + (b * N + k) * 6);
      }
    }
    wg_fence();
    // ------------------------------------------------------------- 2. QP
    const uint64_t q0 = __builtin_amdgcn_s_memrealtime();
    ipmq::solve_quad<double, 1>(g.q, (int)b, ipm_lds);
    wg_fence();
    tqp += __builtin_amdgcn_s_memrealtime() - q0;
    ipm_its += (g.q.status[b] >> 8) & 0xFFFF;
    // ----------------------------------------------------------- 3. step
    if (lane == 0) sqp_step_one(s, b);
    wg_fence();
  }
  if (lane == 0) {
    int64_t* st = g.stats + b * 4;
    st[0] = (int64_t)(__builtin_amdgcn_s_memrealtime() - t0);
    st[1] = (int64_t)tqp;
    st[2] = ipm_its;
    st[3] = it;
  }
}

}  // namespace mpcqp

using namespace mpcqp;

extern "C" size_t mpcqp_bicycle_sqp_solve_workspace(int batch, int N) {
  if (batch <= 0 || N < 1) return 0;
  return (size_t)batch * ((size_t)N * kWsPerStage + 4 + 4) * sizeof(double) + (size_t)batch * 4 +
         256;
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
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1 && max_iter >= 0, "mpcqp_bicycle_sqp_solve: bad sizes");
  MPCQP_CHECK_ARG(params && x0 && Q && R && Qf && U && y && pi && X && rho && kkt && mu && flags,
                  "mpcqp_bicycle_sqp_solve: null pointer");
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0,
                  "mpcqp_bicycle_sqp_solve: bad axle lengths");
  MPCQP_CHECK_ARG(strideX0 >= 4 && strideXb >= 0 && strideLb >= 0,
                  "mpcqp_bicycle_sqp_solve: bad strides");
  MPCQP_CHECK_ARG(integrator == MPCQP_MODEL_FE || integrator == MPCQP_MODEL_RK4,
                  "mpcqp_bicycle_sqp_solve: integrator %d", integrator);
  MPCQP_CHECK_ARG(hessian >= kHessGN && hessian <= kHessRaw,
                  "mpcqp_bicycle_sqp_solve: hessian mode %d", hessian);
  if (batch == 0 || max_iter == 0) return MPCQP_OK;
  const size_t need = mpcqp_bicycle_sqp_solve_workspace(batch, N);
  MPCQP_CHECK_ARG(ws && ws_bytes >= need, "mpcqp_bicycle_sqp_solve: workspace %zu bytes < %zu",
                  ws_bytes, need);
  const size_t lds = (size_t)N * ipm::Layout<4, 2>::F * sizeof(double);
  MPCQP_CHECK_ARG(lds <= 160 * 1024, "mpcqp_bicycle_sqp_solve: N = %d exceeds the LDS horizon", N);
  SqpSolveArgs g{};
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
  double* wXr = w;                w += bN * 4 + (int64_t)batch * 4;
  double* wz = w;                 w += bN * 2;
  double* wy = w;                 w += bN * 4;
  double* wpi = w;                w += bN * 4;
  double* wlu = lam_u ? (double*)lam_u : w;  w += bN * 2;
  double* wX = w;                 w += bN * 4;
  g.stats = (int64_t*)w;          w += (int64_t)batch * 4;  // (tools/sqp_latency.py reads it here)
  int32_t* wst = qp_status ? qp_status : (int32_t*)w;
  g.Xr = wXr;
  a.Z = wz; a.yq = wy; a.piq = wpi; a.qp_status = wst;
  // ---- the QP (mpc.SqpSolver.iterate's mpcqp_mpc_ipm call)
  ipm::Args<double>& q = g.q;
  q.batch = batch; q.nx = 4; q.nu = 2; q.N = N; q.tv = 1;
  q.max_iter = qp_max_iter > 0 ? qp_max_iter : 25;
  q.strict = 0;  // as many inertia corrections as the QP needs (SqpSolver.STRICT)
  q.tol = 1e-10; q.tol_mu = 1e-12; q.tol_polish = 1e-6; q.mu_polish = 1e-6;
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
  g.max_iter = max_iter;
  g.hmode = hessian;
  g.fix_rho = fix_rho();
  g.eps = 1e-6;  // mpcqp_bicycle_hessian_convex's floor (batched.bicycle_hessian)
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)sqp_solve_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(sqp_solve)");
  }
  hipLaunchKernelGGL(sqp_solve_kernel, dim3((unsigned)batch), dim3(64), lds, (hipStream_t)stream, g);
  MPCQP_CHECK_LAUNCH("sqp_solve_kernel");
  return MPCQP_OK;
}
