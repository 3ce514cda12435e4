// sqp.hip -- the outer loop of a CONVERGED MPCController.solve: the
// reference's per-step call hands IPOPT the single-shooting NLP of
// session_4/main.py:41-113 (session4_sol.py:132-217) and returns its optimum
// (main.py:115-116).  Here that NLP is solved by SQP on device, batched over
// initial states; every QP is the stage-wise interior point (ipm.hip), so
// the horizon is unbounded.  Per iteration:
//   mpcqp_bicycle_rti      linearise at U            (bicycle.hip)
//   mpcqp_bicycle_hessian  sum_i pi_i d2 fe_i (exact-Hessian iterations)
//   mpcqp_mpc_ipm          QP -> Z, state multipliers, costates
//   mpcqp_bicycle_sqp_step line search on an L1 merit function, update, and
//                          the first-order optimality (KKT) residual of the
//                          NLP at the new point -- the stopping test.
// Far from a solution the QP uses the Gauss-Newton Hessian (positive
// definite, globally well behaved); once the KKT residual is below 0.3 (or
// after 15 Gauss-Newton iterations) the exact Hessian of the Lagrangian
// takes over (quadratic local convergence), damped Levenberg-Marquardt style
// by a proximal term mu/2 |w - w_k|^2 per stage: a full step divides mu by 4
// (down to 0), a step that needs backtracking multiplies it by 4 (at least
// 1e-4).  An exact-Hessian QP that fails switches the instance to the
// per-stage projected curvature for a few steps.  Inputs at a bound their
// gradient pushes against are held there in the next exact-Hessian QP (a
// proximal term on them, their search direction zero): the full Hessian is
// indefinite along them even at the solution, while second-order
// optimality only needs it positive definite on the free inputs.
#include "sqp_core.hpp"

namespace mpcqp {

__global__ __launch_bounds__(256) void bike_hess_kernel(int batch, int N, Bike p, int integ,
                                 const double* X, const double* U,
                                 const double* pi, const int32_t* flags, const double* mu,
                                 const int32_t* fix, double fix_rho, const double* Qw,
                                 const double* Rw, double eps, double* H2, double* q2) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)batch * N) return;
  const int64_t b = e / N;
  const int k = (int)(e - b * N);
  hess_stage(b, N, k, p, integ, X, U, pi, flags, mu, fix, fix_rho, Qw, Rw, eps, H2 + e * 36,
             q2 + e * 6);
}

__global__ __launch_bounds__(64) void sqp_step_kernel(SqpArgs a) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= a.batch) return;
  sqp_step_one(a, b);
}

// ------------------------------------------------------- linearisation
// The prediction model linearised along the rollout of U (the RTI / SQP
// linearisation, main.py:41-113 on fwd_euler or runge_kutta4,
// main.py:132-147; template.py:141 builds its OCP on RK4): phase 1 (lane =
// instance) rolls out X, phase 2 (lane = (instance, stage)) writes
//   A_k = d x+/dx, B_k = d x+/du at (x_k, u_k), c_k = x_{k+1} - A_k x_k - B_k u_k
// in the layout of mpcqp_condense(MPCQP_TV) and mpcqp_mpc_ipm.
__global__ void model_rollout_kernel(int batch, int N, Bike p, int integ, const double* x0,
                                     int64_t sX0, const double* U, int64_t sU, double* X) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double x[4];
  for (int i = 0; i < 4; ++i) X[(int64_t)b * (N + 1) * 4 + i] = x[i] = x0[(int64_t)b * sX0 + i];
  for (int k = 0; k < N; ++k) {
    const double u[2] = {U[(int64_t)b * sU + 2 * k], U[(int64_t)b * sU + 2 * k + 1]};
    double xn[4];
    model_step(p, integ, x, u, xn);
    for (int i = 0; i < 4; ++i) X[((int64_t)b * (N + 1) + k + 1) * 4 + i] = x[i] = xn[i];
  }
}

__global__ void model_jac_kernel(int batch, int N, Bike p, int integ, const double* U, int64_t sU,
                                 const double* X, double* Ao, double* Bo, double* co) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)batch * N) return;
  const int64_t b = e / N;
  const int k = (int)(e - b * N);
  const double* x = X + (b * (N + 1) + k) * 4;
  const double u[2] = {U[b * sU + 2 * k], U[b * sU + 2 * k + 1]};
  double A[4][4], B[4][2], xn[4];
  model_step_jac(p, integ, x, u, xn, A, B);
  for (int i = 0; i < 4; ++i) {
    double s = xn[i] - B[i][0] * u[0] - B[i][1] * u[1];
    for (int j = 0; j < 4; ++j) {
      Ao[e * 16 + i * 4 + j] = A[i][j];
      s -= A[i][j] * x[j];
    }
    Bo[e * 8 + i * 2] = B[i][0];
    Bo[e * 8 + i * 2 + 1] = B[i][1];
    co[e * 4 + i] = s;
  }
}

// -------------------------------------------------- receding-horizon loop
// The plant of the closed loop (rcracers.simulate(x0, dynamics, n_steps,
// policy), main.py:270-271; session4_sol.py:458,465): x_{t+1} = F(x_t, u_t)
// with u_t = U[0] (the first input of the step's solution, __call__
// main.py:121-129) and F one of
//   0: forward Euler (fwd_euler, main.py:132-135)
//   1: RK4 (runge_kutta4, main.py:138-147)
//   2: RK4 over `substeps` sub-intervals -- the stand-in for odeint
//      (exact_integration, main.py:150-170)
// with the plant's own parameters (e.g. friction x 0.8, session4_sol.py:
// 461-462).  One lane per instance; writes x_{t+1} and records u_t.
__global__ void plant_kernel(int batch, Bike p, int integrator, int substeps, const double* x,
                             const double* U, int64_t sU, double* xn, double* u_rec) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double xs[4], u[2] = {U[(int64_t)b * sU], U[(int64_t)b * sU + 1]};
  for (int i = 0; i < 4; ++i) xs[i] = x[(int64_t)b * 4 + i];
  plant_step(p, integrator, substeps, xs, u);
  for (int i = 0; i < 4; ++i) xn[(int64_t)b * 4 + i] = xs[i];
  if (u_rec) {
    u_rec[(int64_t)b * 2] = u[0];
    u_rec[(int64_t)b * 2 + 1] = u[1];
  }
}

// Warm start of the next receding-horizon step: every per-stage array moves
// one stage forward (the last stage repeated) and the SQP state restarts.
__global__ void sqp_shift_kernel(int batch, int N, double* U, double* y, double* pi,
                                 int32_t* flags, double* rho, double* mu, double* kkt,
                                 double mu0) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  auto shift = [&](double* a, int w) {
    if (!a) return;
    double* r = a + (int64_t)b * N * w;
    for (int k = 0; k + 1 < N; ++k)
      for (int j = 0; j < w; ++j) r[k * w + j] = r[(k + 1) * w + j];
  };
  shift(U, 2);
  shift(y, 4);
  shift(pi, 4);
  if (flags) flags[b] = 0;
  if (rho) rho[b] = 0.0;
  if (mu) mu[b] = mu0;
  if (kkt) kkt[b] = Lim<double>::inf();
}

}  // namespace mpcqp

using mpcqp::Bike;

static int bicycle_hessian_impl(const char* fn, int dtype, int batch, int N, double ts,
                                const double* params, int integrator, const void* X, const void* U,
                                const void* pi, const int32_t* flags, const double* mu,
                                const int32_t* fix, const void* Q, const void* R, double eps,
                                void* H2, void* q2, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "%s: MPCQP_F64 only", fn);
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "%s: bad sizes", fn);
  MPCQP_CHECK_ARG(params && X && U && pi && H2 && q2, "%s: null pointer", fn);
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0, "%s: bad axle lengths", fn);
  MPCQP_CHECK_ARG(integrator == MPCQP_MODEL_FE || integrator == MPCQP_MODEL_RK4,
                  "%s: integrator %d", fn, integrator);
  if (batch == 0) return MPCQP_OK;
  const int64_t total = (int64_t)batch * N;
  hipLaunchKernelGGL(bike_hess_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, batch, N, bike_of(ts, params), integrator, (const double*)X,
                     (const double*)U, (const double*)pi, flags, mu, fix, fix_rho(), (const double*)Q,
                     (const double*)R, eps, (double*)H2, (double*)q2);
  MPCQP_CHECK_LAUNCH("bike_hess_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_bicycle_hessian(int dtype, int batch, int N, double ts, const double* params,
                                     int integrator, const void* X, const void* U, const void* pi,
                                     const int32_t* flags, const double* mu, const int32_t* fix,
                                     void* H2, void* q2, void* stream) {
  return bicycle_hessian_impl("mpcqp_bicycle_hessian", dtype, batch, N, ts, params, integrator,
                              X, U, pi,
                              flags, mu, fix, nullptr, nullptr, 0.0, H2, q2, stream);
}

extern "C" int mpcqp_bicycle_hessian_convex(int dtype, int batch, int N, double ts,
                                            const double* params, int integrator, const void* X,
                                            const void* U,
                                            const void* pi, const int32_t* flags,
                                            const double* mu, const int32_t* fix, const void* Q,
                                            const void* R, double eps, void* H2, void* q2,
                                            void* stream) {
  MPCQP_CHECK_ARG(Q && R && eps > 0.0, "mpcqp_bicycle_hessian_convex: Q, R and eps > 0 required");
  return bicycle_hessian_impl("mpcqp_bicycle_hessian_convex", dtype, batch, N, ts, params,
                              integrator, X, U,
                              pi, flags, mu, fix, Q, R, eps, H2, q2, stream);
}

extern "C" int mpcqp_bicycle_sqp_step(int dtype, int batch, int N, double ts,
                                      const double* params, int integrator, const void* x0,
                                      int64_t strideX0,
                                      const void* Q, const void* R, const void* Qf,
                                      const void* xlo, const void* xhi, int64_t strideXb,
                                      const void* lb, const void* ub, int64_t strideLb, void* U,
                                      const void* Z, const void* yq, const void* piq,
                                      const int32_t* qp_status, void* y, void* pi, void* X,
                                      double* rho, double* kkt, double* mu, int32_t* flags,
                                      int32_t* fix, double tol, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "mpcqp_bicycle_sqp_step: MPCQP_F64 only");
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "mpcqp_bicycle_sqp_step: bad sizes");
  MPCQP_CHECK_ARG(params && x0 && Q && R && Qf && U && Z && yq && piq && y && pi && X && rho &&
                      kkt && mu && flags,
                  "mpcqp_bicycle_sqp_step: null pointer");
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0,
                  "mpcqp_bicycle_sqp_step: bad axle lengths");
  MPCQP_CHECK_ARG(strideX0 >= 0 && strideXb >= 0 && strideLb >= 0,
                  "mpcqp_bicycle_sqp_step: negative stride");
  MPCQP_CHECK_ARG(integrator == MPCQP_MODEL_FE || integrator == MPCQP_MODEL_RK4,
                  "mpcqp_bicycle_sqp_step: integrator %d", integrator);
  if (batch == 0) return MPCQP_OK;
  SqpArgs a;
  a.batch = batch; a.N = N; a.p = bike_of(ts, params); a.integ = integrator;
  a.x0 = (const double*)x0; a.sX0 = strideX0;
  a.Q = (const double*)Q; a.R = (const double*)R; a.Qf = (const double*)Qf;
  a.xlo = (const double*)xlo; a.xhi = (const double*)xhi; a.sXb = strideXb;
  a.lb = (const double*)lb; a.ub = (const double*)ub; a.sLb = strideLb;
  a.U = (double*)U; a.Z = (const double*)Z; a.yq = (const double*)yq; a.piq = (const double*)piq;
  a.qp_status = qp_status;
  a.y = (double*)y; a.pi = (double*)pi; a.X = (double*)X;
  a.rho = rho; a.kkt = kkt; a.mu = mu; a.flags = flags; a.tol = tol > 0 ? tol : 1e-9;
  a.fix = fix;
  sqp_knobs(a);
  hipLaunchKernelGGL(sqp_step_kernel, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0,
                     (hipStream_t)stream, a);
  MPCQP_CHECK_LAUNCH("sqp_step_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_bicycle_plant(int dtype, int batch, double ts, const double* params,
                                   int integrator, int substeps, const void* x, const void* U,
                                   int64_t strideU, void* x_next, void* u_rec, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "mpcqp_bicycle_plant: MPCQP_F64 only");
  MPCQP_CHECK_ARG(batch >= 0 && strideU >= 2, "mpcqp_bicycle_plant: bad sizes");
  MPCQP_CHECK_ARG(integrator >= 0 && integrator <= 2 && (integrator != 2 || substeps >= 1),
                  "mpcqp_bicycle_plant: integrator %d / substeps %d", integrator, substeps);
  MPCQP_CHECK_ARG(params && x && U && x_next, "mpcqp_bicycle_plant: null pointer");
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0,
                  "mpcqp_bicycle_plant: bad axle lengths");
  if (batch == 0) return MPCQP_OK;
  hipLaunchKernelGGL(plant_kernel, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     batch, bike_of(ts, params), integrator, substeps, (const double*)x,
                     (const double*)U, strideU, (double*)x_next, (double*)u_rec);
  MPCQP_CHECK_LAUNCH("plant_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_sqp_shift(int dtype, int batch, int N, void* U, void* y, void* pi,
                               int32_t* flags, double* rho, double* mu, double* kkt, double mu0,
                               void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "mpcqp_sqp_shift: MPCQP_F64 only");
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "mpcqp_sqp_shift: bad sizes");
  if (batch == 0) return MPCQP_OK;
  hipLaunchKernelGGL(sqp_shift_kernel, dim3((batch + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, batch, N, (double*)U, (double*)y, (double*)pi, flags,
                     rho, mu, kkt, mu0);
  MPCQP_CHECK_LAUNCH("sqp_shift_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_bicycle_linearise(int dtype, int batch, int N, double ts,
                                       const double* params, int integrator, const void* x0,
                                       int64_t strideX0, const void* U, int64_t strideU, void* X,
                                       void* A, void* B, void* c, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64, "mpcqp_bicycle_linearise: MPCQP_F64 only");
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "mpcqp_bicycle_linearise: bad sizes");
  MPCQP_CHECK_ARG(integrator == MPCQP_MODEL_FE || integrator == MPCQP_MODEL_RK4,
                  "mpcqp_bicycle_linearise: integrator %d", integrator);
  MPCQP_CHECK_ARG(params && x0 && U && X && A && B && c, "mpcqp_bicycle_linearise: null pointer");
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0,
                  "mpcqp_bicycle_linearise: bad axle lengths");
  MPCQP_CHECK_ARG(strideX0 >= 4 && strideU >= 2 * N, "mpcqp_bicycle_linearise: bad strides");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  const Bike p = bike_of(ts, params);
  hipLaunchKernelGGL(model_rollout_kernel, dim3((batch + 63) / 64), dim3(64), 0, st, batch, N, p,
                     integrator, (const double*)x0, strideX0, (const double*)U, strideU,
                     (double*)X);
  MPCQP_CHECK_LAUNCH("model_rollout_kernel");
  const int64_t total = (int64_t)batch * N;
  hipLaunchKernelGGL(model_jac_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     batch, N, p, integrator, (const double*)U, strideU, (const double*)X,
                     (double*)A, (double*)B, (double*)c);
  MPCQP_CHECK_LAUNCH("model_jac_kernel");
  return MPCQP_OK;
}
