/*
 * mpcqp.h -- C ABI of libmpcqp.so, the MI355X-native batched condensed-QP
 * MPC solver (gfx950 / CDNA4, HIP).
 *
 * The reference (konnpaku-youmu/Model_Predictive_Control) has no FFI: its hot
 * path is a set of Python call surfaces that today reach NumPy and
 * CasADi/IPOPT.  Each entry point below replaces one of them; the Python
 * shim in model_predictive_control_amd/ keeps the reference's call surface
 * and calls these through ctypes:
 *
 *   mpcqp_condense   <- the symbolic single-shooting elimination of
 *                       session_4/main.py:86-106 (and session4_sol.py:195-204)
 *                       written as dense H, F, f, Gamma, Phi, xbar.
 *   mpcqp_solve_box  <- the per-step IPOPT call of session_4/main.py:115-116
 *                       (session4_sol.py:128-129) for an input box
 *                       (lbx/ubx, main.py:68-69,97-98).
 *   mpcqp_mpc_box    <- both of the above fused for the input-box OCP
 *                       (MPCController.solve end to end, one launch).
 *   mpcqp_mpc_qp     <- MPCController.solve end to end with the input box AND
 *                       the state box (main.py:58-61,68-69; session4_sol.py:
 *                       176-181): condense + QP in one call, fp32 refined
 *                       against the dynamics in fp64.
 *   mpcqp_solve_poly <- the same call with general rows hl <= G z <= hu (state box
 *                       lbg/ubg of main.py:58-61,99-100 after condensing, or
 *                       arbitrary polytopes -- BASELINE config 4).
 *   mpcqp_riccati    <- ricatti_recursion(A,B,Q,R,P_f,N), session_1/FHC.py:51-61
 *                       (and riccati_recursion, session1_sol.py:44-65).
 *   mpcqp_gemv       <- the batched  f = F x0  /  z = -W x0 - U lambda  products
 *                       that sit between condense and solve.
 *   mpcqp_rollout    <- LinearSystem.simulate (session_1/LinearSystem.py:20-26)
 *                       under a linear state-feedback policy
 *                       (AutoCruising.control_law, FHC.py:25-26).
 *
 * Conventions (all entry points):
 *  - dtype: MPCQP_F64 or MPCQP_F32; every floating buffer of a call has it.
 *  - Buffers are caller-owned DEVICE pointers (hipMalloc / torch tensors),
 *    row-major, batch-outermost.  A "stride" is the element distance between
 *    consecutive instances; stride 0 means one buffer shared by the batch.
 *    The library keeps no pointer after the call returns.
 *  - z is stage-major: z = [u_0; u_1; ...; u_{N-1}] (main.py:46,110).
 *  - Symmetric n x n matrices (H, the dual M) are stored PACKED LOWER,
 *    row-major: element (i, j<=i) at i*(i+1)/2 + j, n(n+1)/2 per instance.
 *  - stream is a hipStream_t (NULL = default stream).  Calls only enqueue
 *    work; they never synchronise, allocate or free (graph-capturable).
 *  - Return value: MPCQP_OK (0) or a negative error code; the message is
 *    available from mpcqp_last_error() (thread-local).
 *  - Per-instance outcome goes to status[b]: low byte = MPCQP_STATUS_*, bits
 *    8..23 = active-set iterations used.
 *    This mirrors the per-step ``solver_success`` of session_2/log.py:10.
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCQP_ABI_VERSION 1

/* dtypes */
#define MPCQP_F64 0
#define MPCQP_F32 1

/* return codes */
#define MPCQP_OK 0
#define MPCQP_EINVAL (-1)   /* bad argument (shape, pointer, dtype) */
#define MPCQP_EHIP (-2)     /* HIP runtime error (launch / no device) */
#define MPCQP_ENOTSUP (-3)  /* size outside the compiled kernel set */

/* per-instance status (low byte of status[b]) */
#define MPCQP_STATUS_OPTIMAL 0
#define MPCQP_STATUS_MAXITER 1
#define MPCQP_STATUS_NOT_CONVEX 2  /* non-positive pivot: H not positive definite */
#define MPCQP_STATUS_INFEASIBLE 3  /* lb > ub, or polytope empty */
#define MPCQP_STATUS_NONFINITE 4   /* NaN/Inf in the data */

/* condense / MPC-step flags */
#define MPCQP_TV 1  /* A, B are per-stage: N*nx*nx / N*nx*nu per instance */
#define MPCQP_IPM 2 /* mpcqp_mpc_qp: solve on the stage-wise interior point (mpcqp_mpc_ipm) */
/* mpcqp_mpc_ipm: after a few (6) inertia corrections of non-positive
   Riccati pivots the solve ends with MPCQP_STATUS_NOT_CONVEX instead of
   regularising further (an SQP caller raises its own damping and retries) */
#define MPCQP_STRICT 4
/* mpcqp_condense: Gam is written as its lower block triangle only, block row
   k (rows k*nx .. k*nx+nx-1, the state x_{k+1}) holding its (k+1)*nu leading
   columns from element offset nx*nu*k*(k+1)/2, column by column: entry
   (k*nx + q, col) at nx*nu*k*(k+1)/2 + col*nx + q -- nx*nu*N*(N+1)/2
   elements per instance instead of N*nx*N*nu (the upper block triangle is
   structurally zero; SURVEY 8(d) counts only this part) */
#define MPCQP_GAM_PACKED 8

/* status bit 24: the solution was polished to the exact active-set vertex */
#define MPCQP_STATUS_POLISHED (1 << 24)
/* status bit 25 (mpcqp_mpc_qp, fp32): more than 64 active constraints sent the
   instance to the workgroup kernel, which solves the fp32 condensed QP without
   the refinement against the dynamics -- z is at the fp32 condensing floor
   (~1e-5 relative) instead of the fp64 solution of the step */
#define MPCQP_STATUS_UNREFINED (1 << 25)

int mpcqp_abi_version(void);
const char* mpcqp_last_error(void);
/* Largest n (= N*nu) accepted by mpcqp_solve_box and the dual size accepted
 * by mpcqp_solve_poly for the given dtype. */
int mpcqp_max_box_n(int dtype);

/*
 * Batched condensing of  x_{k+1} = A_k x_k + B_k u_k + c_k,  k = 0..N-1, with
 * cost  sum_{k<N} x_k'Q x_k + u_k'R u_k + x_N'Qf x_N  (session_4/main.py:86-106):
 *
 *   X = [x_1;..;x_N] = Phi x0 + Gam z + w,   xbar = Phi x0 + w
 *   H = Gam' Qhat Gam + Rhat  (packed lower, n(n+1)/2),   n = N*nu
 *   F = Gam' Qhat Phi  (n x nx),   f = Gam' Qhat xbar (n)
 *
 * Inputs (per-instance strides in elements; 0 = shared):
 *   A  nx*nx (or N*nx*nx with MPCQP_TV), Bm nx*nu (or N*nx*nu), Q nx*nx,
 *   R nu*nu, Qf nx*nx, c (optional, N*nx), x0 (optional, nx).
 * Outputs (NULL to skip; per-instance, densely packed):
 *   H (required), F, f (uses x0 and c; x0 = NULL means x0 = 0),
 *   Gam (N*nx x n; with MPCQP_GAM_PACKED its lower block triangle,
 *   nx*nu*N*(N+1)/2), Phi (N*nx x nx), xbar (N*nx).
 * Limits: 1 <= nx <= 16, 1 <= nu <= 16, N >= 1.
 */
int mpcqp_condense(int dtype, int batch, int nx, int nu, int N, int flags,
                   const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                   const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                   const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                   const void* x0, int64_t strideX0,
                   void* H, void* F, void* f, void* Gam, void* Phi, void* xbar,
                   void* stream);

/*
 * Batched box QP:  min 1/2 z'Hz + f'z   s.t.  lb <= z <= ub
 * (n <= mpcqp_max_box_n(dtype); n > 64 runs on the mpcqp_solve_qp kernel).
 * H packed lower (stride 0 = shared), f/lb/ub per instance or shared
 * (lb/ub NULL = -inf/+inf).  One QP per wavefront: Goldfarb-Idnani dual
 * active set specialised to bounds, on H swept over the free set (one row per
 * lane, pivot rows broadcast by v_readlane).  Finite termination; iterations
 * ~ number of active bounds.  max_iter <= 0 selects the default (3n + 30);
 * tol <= 0 the default relative feasibility tolerance (1e-12 f64, 1e-6 f32).
 */
int mpcqp_solve_box(int dtype, int batch, int n,
                    const void* H, int64_t strideH, const void* f, int64_t stridef,
                    const void* lb, int64_t strideLb, const void* ub, int64_t strideUb,
                    void* z, int32_t* status, int max_iter, double tol, void* stream);

/*
 * Fused per-instance condense + input-box QP (the whole MPCController.solve of
 * session_4/main.py:115-116 for an input-box OCP, session4_sol.py:128-129):
 * plant (A, B [, c]) per instance or shared exactly as in mpcqp_condense, x0
 * per instance, bounds lb/ub (N*nu; stride 0 = shared; NULL = +-inf) -> z, status.
 * -H^{-1} is built from a per-instance Riccati factorisation (one lane per
 * column) instead of being formed and inverted; nothing but the plant, x0,
 * the bounds and z cross HBM.  Limits: nx <= 4, nu <= 2, N*nu <= 32 (larger
 * problems: mpcqp_condense + mpcqp_solve_box).
 */
int mpcqp_mpc_box(int dtype, int batch, int nx, int nu, int N, int flags,
                  const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                  const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                  const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                  const void* x0, int64_t strideX0,
                  const void* lb, int64_t strideLb, const void* ub, int64_t strideUb,
                  void* z, int32_t* status, int max_iter, double tol, void* stream);

/*
 * Batched polytope QP:
 *     min 1/2 z'Hz + f'z   s.t.  hl <= G z <= hu,   lbz <= z <= ubz
 * H (n x n, packed lower) and G (m x n) are SHARED by the batch (the
 * shared-structure form of BASELINE config 4 and of LTI state boxes);
 * f (n) and the row bounds hl/hu (m) vary per instance (stride 0 = shared;
 * NULL = -inf / +inf).  The box rows are appended to C = [G; I] when lbz or
 * ubz is given (then m_total = m + n, else m_total = m; m_total <= 64).
 * Solved through the dual: Hinv, Ut = C Hinv and M = C Hinv C' are formed once
 * per call on device; per instance a wavefront runs a dual range active set
 * (Goldfarb-Idnani in the row space, tolerant of linearly dependent rows) and
 * recovers z = -Hinv f - Ut' y.  y (batch x m_total): row multipliers,
 * y > 0 at the upper bound, y < 0 at the lower bound.
 * workspace: device scratch of at least mpcqp_solve_poly_workspace() bytes
 * (nbox = 1 when lbz or ubz is given).
 */
int64_t mpcqp_solve_poly_workspace(int dtype, int batch, int n, int m, int nbox);
int mpcqp_solve_poly(int dtype, int batch, int n, int m,
                     const void* H, const void* f, int64_t stridef,
                     const void* G, const void* hl, const void* hu, int64_t strideh,
                     const void* lbz, const void* ubz,
                     void* z, void* y, int32_t* status, int max_iter, double tol,
                     void* workspace, int64_t workspace_bytes, void* stream);

/*
 * The same polytope QP split into a shared setup and a per-batch solve, for
 * the receding-horizon loop where H, G (and the condensed x0 -> gradient map
 * F, n x nx) stay fixed and only x0 changes (BASELINE config 4):
 *   mpcqp_poly_setup: Hinv, Ut = C Hinv, M = C Hinv C', Kt = (-Hinv F)',
 *                     L = -Ut F  into the workspace (once);
 *   mpcqp_poly_solve: gradient f = F x0 + f1 per instance (x0 and/or f1,
 *                     either may be NULL), rows hl/hu per instance or shared;
 *                     one wavefront per instance computes s0 = L x0 - Ut f1,
 *                     runs the dual range active set and writes
 *                     z = Kt' x0 - Hinv f1 - Ut' y.
 * nbox = 1 appends the box rows (lbz/ubz given to poly_solve) to C = [G; I].
 * Limits: m_total <= 64, nx <= 16.  The workspace (mpcqp_poly_workspace
 * bytes) is read-only during poly_solve, so concurrent solves may share it.
 */
int64_t mpcqp_poly_workspace(int dtype, int n, int m, int nbox, int nx);
int mpcqp_poly_setup(int dtype, int n, int m, int nbox, int nx, const void* H,
                     const void* G, const void* F, void* workspace,
                     int64_t workspace_bytes, void* stream);
int mpcqp_poly_solve(int dtype, int batch, int n, int m, int nbox, int nx,
                     const void* workspace, const void* x0, int64_t strideX0,
                     const void* f, int64_t stridef, const void* hl, const void* hu,
                     int64_t strideh, const void* lbz, const void* ubz,
                     void* z, void* y, int32_t* status, int max_iter, double tol,
                     void* stream);

/*
 * Batched QP with per-instance data and general rows:
 *     min 1/2 z'Hz + f'z   s.t.  lb <= z <= ub,   hl <= G z <= hu
 * (session_4/main.py:115-116 with the input box lbx/ubx, main.py:68-69, AND
 * the state box lbg/ubg, main.py:58-61, after condensing: G = Gam,
 * hl/hu = x_min/x_max - xbar -- BASELINE config 3; with m = 0 the large
 * input-box QPs of config 5).  Every operand has its own per-instance stride
 * (0 = shared): H packed lower n(n+1)/2, f n, G m*n row-major, hl/hu m,
 * lb/ub n (NULL = unbounded).  One instance per workgroup: the augmented
 * matrix [[H, G'], [G, 0]] lives in registers, every z is swept in (which
 * yields -H^-1 and the dual G H^-1 G' without forming either separately),
 * then a mixed primal/dual Goldfarb-Idnani active set handles bounds and
 * rows together, including rows that depend on the active set.
 * y (batch x m, optional): row multipliers, > 0 at hu, < 0 at hl.
 * Limits: n + m <= mpcqp_max_qp_size(dtype).  mpcqp_solve_box uses the same
 * kernel for n > 64.
 */
int mpcqp_max_qp_size(int dtype);
int mpcqp_solve_qp(int dtype, int batch, int n, int m,
                   const void* H, int64_t strideH, const void* f, int64_t stridef,
                   const void* G, int64_t strideG, const void* hl, const void* hu,
                   int64_t strideh, const void* lb, int64_t strideLb,
                   const void* ub, int64_t strideUb,
                   void* z, void* y, int32_t* status, int max_iter, double tol,
                   void* stream);

/*
 * Two-kernel fp32 path for the large QPs of mpcqp_solve_qp / mpcqp_solve_box
 * (configs 3 and 5; replaces the same per-step IPOPT call,
 * session_4/main.py:115-116): the "sweep every z in" phase runs as its own
 * MFMA kernel (mpcqp_sweep) into a caller workspace, then the active set runs
 * on the pre-swept matrix.  Same arguments, results and status codes as
 * mpcqp_solve_qp / mpcqp_solve_box.
 *   mpcqp_solve_qp_workspace: bytes the _ws calls need for (dtype, batch, n,
 *     m) -- about batch * (n+m)^2 floats -- or 0 where the path does not
 *     apply (fp64, n + m <= 64, padded n + m > 192); with 0 or ws == NULL the
 *     _ws calls are the plain ones.
 *   mpcqp_sweep: M = SWEEP_z([[H, G'], [G, 0]]) = [[-H^-1, H^-1 G'],
 *     [G H^-1, -G H^-1 G']] over n + m per instance, packed lower (full = 0)
 *     or dense row-major (full = 1); status[b] = 0 / MPCQP_STATUS_NOT_CONVEX /
 *     MPCQP_STATUS_NONFINITE.  MPCQP_F32 only; 64 < 16*ceil(n/16) + m <= 192.
 *   The _ws solves run mpcqp_sweep (dense) -> a product-form active set on
 *     the swept matrix (one instance per wavefront, solve_pf.hip) -> the
 *     workgroup kernel for any instance with more than 64 active constraints.
 */
size_t mpcqp_solve_qp_workspace(int dtype, int batch, int n, int m);
int mpcqp_sweep(int dtype, int batch, int n, int m, const void* H, int64_t strideH,
                const void* G, int64_t strideG, void* M, int full, int32_t* status,
                void* stream);
int mpcqp_solve_qp_ws(int dtype, int batch, int n, int m,
                      const void* H, int64_t strideH, const void* f, int64_t stridef,
                      const void* G, int64_t strideG, const void* hl, const void* hu,
                      int64_t strideh, const void* lb, int64_t strideLb,
                      const void* ub, int64_t strideUb,
                      void* z, void* y, int32_t* status, int max_iter, double tol,
                      void* ws, size_t ws_bytes, void* stream);
int mpcqp_solve_box_ws(int dtype, int batch, int n,
                       const void* H, int64_t strideH, const void* f, int64_t stridef,
                       const void* lb, int64_t strideLb, const void* ub, int64_t strideUb,
                       void* z, int32_t* status, int max_iter, double tol,
                       void* ws, size_t ws_bytes, void* stream);

/*
 * One MPC step with input box and state box, end to end (the whole
 * MPCController.solve of session_4/main.py:115-116 for the OCP of
 * main.py:41-113 with lbx/ubx, main.py:68-69, and lbg/ubg on x_1..x_N,
 * main.py:58-61; session4_sol.py:176-181):
 *     min  sum_{k<N} x_k'Q x_k + u_k'R u_k + x_N'Qf x_N
 *     s.t. x_{k+1} = A_k x_k + B_k u_k + c_k,   lb <= z <= ub,
 *          xlo <= [x_1; ..; x_N] <= xhi
 * Plant, weights, c and x0 exactly as in mpcqp_condense (flags MPCQP_TV);
 * xlo/xhi (N*nx, stride strideXb, 0 = shared; both NULL = no state box,
 * one NULL = unbounded on that side); lb/ub (N*nu) as in mpcqp_solve_box.
 * Outputs: z (N*nu), y (optional, N*nx: state-row multipliers, > 0 at xhi),
 * X (optional, N*nx: x_1..x_N of z, the IPOPT "g" rows), status.
 * Pipeline: mpcqp_condense -> rows -> (fp32, N(nu+nx) > 64) MFMA sweep ->
 * product-form active set -> iterative refinement whose KKT residual is
 * computed from the DYNAMICS in fp64 (forward rollout + adjoint), so the
 * fp32 path converges to the solution of the QP its inputs define rather
 * than to that of the fp32-rounded condensed matrices; fp64 or small QPs:
 * the workgroup QP kernel.  Steps beyond the dense size limit (N*(nu + nx)
 * with the state box, or N*nu, > mpcqp_max_qp_size(dtype)) -- and every step
 * when flags has MPCQP_IPM -- run on the stage-wise interior point
 * (mpcqp_mpc_ipm) when nx <= 4 and nu <= 2.  Limits: nx, nu <= 16.
 * workspace: mpcqp_mpc_qp_workspace() bytes of device scratch (state_box = 1
 * when xlo or xhi is given).
 */
size_t mpcqp_mpc_qp_workspace(int dtype, int batch, int nx, int nu, int N, int state_box);
int mpcqp_mpc_qp(int dtype, int batch, int nx, int nu, int N, int flags,
                 const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                 const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                 const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                 const void* x0, int64_t strideX0,
                 const void* xlo, const void* xhi, int64_t strideXb,
                 const void* lb, int64_t strideLb, const void* ub, int64_t strideUb,
                 void* z, void* y, void* X, int32_t* status, int max_iter, double tol,
                 void* ws, size_t ws_bytes, void* stream);
/*
 * Stage timing of mpcqp_mpc_qp (profiling, one host thread): after
 * mpcqp_mpc_qp_profile(1) every mpcqp_mpc_qp call records HIP events on its
 * stream around its stages; mpcqp_mpc_qp_stage_ms(ms) waits for the last
 * call's events and writes 5 floats, the milliseconds of condense, sweep,
 * solve, fp64 fallback and states (-1 for a stage the call did not run).
 * An enabled call cannot be captured in a graph; mpcqp_mpc_qp_profile(0)
 * turns it off.
 */
int mpcqp_mpc_qp_profile(int enable);
int mpcqp_mpc_qp_stage_ms(float* ms);

/*
 * The same MPC step (same problem, arguments and outputs as mpcqp_mpc_qp) on
 * the NON-condensed structure, for any horizon N: the reference's own
 * controllers run N = 50 with the state box (session4_sol.py:342,391,445,
 * bounds session4_sol.py:176-181), n + m = 300, beyond the dense kernels.
 * One instance per lane; primal-dual interior point (Mehrotra
 * predictor-corrector) whose Newton systems are solved by a Riccati sweep
 * over the stages, O(N (nx+nu)^3) per iteration, then an exact polish on the
 * identified active set (status bit MPCQP_STATUS_POLISHED).  Arithmetic is
 * fp64 for both dtypes.
 * Extra arguments: U0 (optional, N*nu per instance, stride strideU0): the
 * starting inputs; H2, q2 (optional, (nx+nu)^2 and nx+nu per stage, N
 * stages per instance, strides strideH2/strideq2): an extra stage cost
 * 1/2 [x_k; u_k]'H2_k [x_k; u_k] + q2_k'[x_k; u_k] -- the curvature of the
 * dynamics in an exact-Hessian SQP; it may be indefinite (the interior
 * point corrects the inertia of its Newton systems).  Outputs: lam_u
 * (optional, N*nu): input-bound multipliers, > 0 at ub; pi (optional, N*nx):
 * costates of x_{k+1} = A_k x_k + B_k u_k + c_k; y (optional, N*nx):
 * state-bound multipliers, > 0 at xhi.  status: MPCQP_STATUS_NOT_CONVEX when
 * no inertia correction up to 1e12 makes the Newton system definite (at the
 * sixth inertia correction with flags & MPCQP_STRICT).  skip (optional, one
 * int32 per instance): instances with (skip[b] & skip_mask) != 0 are not
 * solved and their outputs and status are left as they are (an SQP passes
 * its per-instance flags to freeze the converged instances).
 * Limits: nx <= 4, nu <= 2.  workspace: mpcqp_mpc_ipm_workspace() bytes
 * (N * ~100 doubles per instance).
 */
size_t mpcqp_mpc_ipm_workspace(int dtype, int batch, int nx, int nu, int N);
int mpcqp_mpc_ipm(int dtype, int batch, int nx, int nu, int N, int flags,
                  const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                  const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                  const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                  const void* x0, int64_t strideX0,
                  const void* xlo, const void* xhi, int64_t strideXb,
                  const void* lb, int64_t strideLb, const void* ub, int64_t strideUb,
                  const void* U0, int64_t strideU0, const void* H2, int64_t strideH2,
                  const void* q2, int64_t strideq2,
                  void* z, void* y, void* X, void* lam_u, void* pi, int32_t* status,
                  const int32_t* skip, int32_t skip_mask,
                  int max_iter, double tol, void* ws, size_t ws_bytes, void* stream);

/*
 * Converged MPCController.solve (session_4/main.py:115-116: IPOPT's optimum
 * of the single-shooting NLP of main.py:41-113 / session4_sol.py:132-217)
 * as an SQP over batched initial states, one iteration =
 *   mpcqp_bicycle_rti (linearise at U, states X) -> [mpcqp_bicycle_hessian]
 *   -> mpcqp_mpc_ipm (H2, q2; outputs z, y, pi) -> mpcqp_bicycle_sqp_step.
 * mpcqp_bicycle_hessian: per instance and stage, H2_k = sum_i pi_{k+1,i}
 *   d2 F_i / d(x,u)2 at (x_k, u_k) (F the prediction model's step:
 *   integrator MPCQP_MODEL_FE or MPCQP_MODEL_RK4, the latter by the
 *   second-order adjoint through its four stages) + mu I (6 x 6 over [x; u]; mu the
 *   instance's Levenberg-Marquardt damping, NULL = 0) and q2_k = -H2_k w_k,
 *   so that the QP's extra cost is 1/2 (w - w_k)'H2_k (w - w_k); zeros for
 *   instances whose flags lack MPCQP_SQP_EXACT (flags NULL = all exact).
 *   fix (NULL = none): one int32 per instance and stage, bit q set = input
 *   q is held at its bound: its diagonal gets a proximal 100 (the QP keeps
 *   the input at its bound; the step kernel gives it no search direction).  X ((N+1) x 4), U (N x 2), pi (N x 4) per
 *   instance.
 * mpcqp_bicycle_sqp_step: per instance not yet MPCQP_SQP_DONE: step d = Z - U
 *   (Z the QP solution; an instance whose qp_status is not OPTIMAL takes no
 *   step: in exact-Hessian mode it switches to the projected curvature
 *   (MPCQP_SQP_PROJ) and, if that QP fails too, its damping mu grows x4; in Gauss-Newton mode
 *   three failures in a row stop it with flags DONE | MPCQP_SQP_FAIL and the
 *   QP's status code in bits 28..30), L1 merit 1/2 J + rho |state-box violation|_1 with
 *   rho >= 2 max|yq|, Armijo backtracking by quadratic interpolation (after
 *   five shortened exact-Hessian steps in a row, one full step without the
 *   test; flags bits 4..7 count them); then
 *   U += alpha d, y += alpha (yq - y), pi += alpha (piq - pi), the rollout X
 *   ((N+1) x 4) at the new U and the first-order optimality residual of the
 *   NLP there (projected gradient of the Lagrangian on the input box,
 *   state-box violation, complementarity of y) -> kkt.  flags: DONE when
 *   kkt <= tol; EXACT (use the exact Hessian from now on) once kkt < 0.3
 *   or after 15 Gauss-Newton iterations;
 *   bits 8..23 count the iterations.  fix (NULL = not written; batch x N
 *   int32, for mpcqp_bicycle_hessian): bit q of stage k set when u_k,q sits
 *   at a bound that its NLP gradient pushes against by more than 1e-6.  mu (Levenberg-Marquardt damping of the
 *   exact-Hessian QPs, caller-initialised, e.g. 0.1): divided by 4 after a
 *   full step (to 0 below 1e-11), multiplied by 4 (at least 1e-3) after a
 *   step that needed backtracking or a failed QP.  rho, mu, kkt: one double
 *   per instance (rho initialised to 0).  Q, R, Qf shared (4x4, 2x2, 4x4);
 *   bounds as in mpcqp_mpc_qp (lb/ub stride strideLb).  integrator: the
 *   prediction model of the NLP (MPCQP_MODEL_FE / MPCQP_MODEL_RK4; pass
 *   the same one to mpcqp_bicycle_hessian).  fp64.
 */
#define MPCQP_SQP_DONE 1
#define MPCQP_SQP_EXACT 2
#define MPCQP_SQP_FAIL 4  /* with DONE: stopped by failing QPs; QP status in bits 28..30 */
#define MPCQP_SQP_PROJ 8  /* projected curvature for the next steps (bits 24..27 count) */
/* prediction models (integrator argument) */
#define MPCQP_MODEL_FE 0  /* fwd_euler, main.py:132-135 */
#define MPCQP_MODEL_RK4 1 /* runge_kutta4, main.py:138-147 (template.py:141) */
/*
 * mpcqp_bicycle_linearise: the prediction model (FE or RK4) rolled out from
 * x0 under U (N x 2) -> X ((N+1) x 4), and linearised along it:
 * A_k = d x+/dx, B_k = d x+/du (RK4: forward sensitivities through the four
 * stages), c_k = x_{k+1} - A_k x_k - B_k u_k, in the layout of
 * mpcqp_condense(MPCQP_TV).  fp64.  (mpcqp_bicycle_rti is the FE case in
 * fp32 or fp64.)
 */
int mpcqp_bicycle_linearise(int dtype, int batch, int N, double ts, const double* params,
                            int integrator, const void* x0, int64_t strideX0, const void* U,
                            int64_t strideU, void* X, void* A, void* B, void* c, void* stream);
int mpcqp_bicycle_hessian(int dtype, int batch, int N, double ts, const double* params,
                          int integrator, const void* X, const void* U, const void* pi, const int32_t* flags,
                          const double* mu, const int32_t* fix, void* H2, void* q2, void* stream);
/*
 * mpcqp_bicycle_hessian_convex: mpcqp_bicycle_hessian with a per-stage
 * convexification for the instances whose flags carry MPCQP_SQP_PROJ (all
 * when flags is NULL): where the stage's QP Hessian W_k = blkdiag(Q, R) +
 * H2_k (Q 4 x 4, R 2 x 2 shared, the stage weights) is not positive definite,
 * its eigenvalues are lifted to eps and H2_k = W_k' - blkdiag(Q, R)
 * (eigenvalue projection; stages with W_k > 0 keep the exact curvature), then
 * + mu I.  mpcqp_bicycle_sqp_step sets MPCQP_SQP_PROJ when an exact-Hessian QP
 * fails (non-convex) and clears it after four full steps, so the exact
 * curvature (Newton's rate) is used wherever its QP is convex and a convex
 * QP is taken instead of a rejected one where it is not.
 */
int mpcqp_bicycle_hessian_convex(int dtype, int batch, int N, double ts, const double* params,
                                 int integrator, const void* X, const void* U, const void* pi,
                                 const int32_t* flags, const double* mu, const int32_t* fix,
                                 const void* Q, const void* R, double eps, void* H2, void* q2,
                                 void* stream);
int mpcqp_bicycle_sqp_step(int dtype, int batch, int N, double ts, const double* params,
                           int integrator, const void* x0, int64_t strideX0, const void* Q, const void* R,
                           const void* Qf, const void* xlo, const void* xhi, int64_t strideXb,
                           const void* lb, const void* ub, int64_t strideLb, void* U,
                           const void* Z, const void* yq, const void* piq,
                           const int32_t* qp_status, void* y, void* pi, void* X, double* rho,
                           double* kkt, double* mu, int32_t* flags, int32_t* fix, double tol,
                           void* stream);

/*
 * mpcqp_bicycle_sqp_solve: the whole SQP above -- up to max_iter iterations
 * of linearise -> Hessian -> interior-point QP -> step per instance -- in ONE
 * launch, one single-wave workgroup per instance (replaces session_4/
 * main.py:115-116's per-step IPOPT call like the four-call iteration does;
 * mpc.SqpSolver.solve).  Every instance stops at its own convergence: the
 * launch lasts as long as the slowest instance's solve, not the sum over
 * iterations of each iteration's slowest QP.  Arguments as
 * mpcqp_bicycle_sqp_step (the SQP state U, y, pi, X, rho, kkt, mu, flags,
 * fix in and out: a warm start continues from them) plus
 *   hessian: MPCQP_SQP_HESS_GN (Gauss-Newton QPs; fix unused),
 *            MPCQP_SQP_HESS_EXACT (the exact Lagrangian curvature after the
 *            switch, projected per stage in PROJ mode: Q and R are the
 *            projection's stage weights), MPCQP_SQP_HESS_RAW (never projected);
 *   lam_u (optional, batch x N*2): the last QP's input-bound multipliers;
 *   qp_status (optional, batch): the last QP's status word;
 *   qp_max_iter: interior-point iterations per QP (<= 0: 25);
 *   tol: the KKT tolerance (<= 0: 1e-9).
 * The linearisation is mpcqp_bicycle_linearise's (FE or RK4).  The QP's
 * horizon lives in LDS: N * 142 doubles <= 160 KB (N <= 144).  fp64.
 * workspace: mpcqp_bicycle_sqp_solve_workspace() bytes (N * 90 doubles per
 * instance).
 */
#define MPCQP_SQP_HESS_GN 0
#define MPCQP_SQP_HESS_EXACT 1
#define MPCQP_SQP_HESS_RAW 2
size_t mpcqp_bicycle_sqp_solve_workspace(int batch, int N);
int mpcqp_bicycle_sqp_solve(int dtype, int batch, int N, double ts, const double* params,
                            int integrator, int hessian, const void* x0, int64_t strideX0,
                            const void* Q, const void* R, const void* Qf, const void* xlo,
                            const void* xhi, int64_t strideXb, const void* lb, const void* ub,
                            int64_t strideLb, void* U, void* y, void* pi, void* X, double* rho,
                            double* kkt, double* mu, int32_t* flags, int32_t* fix, void* lam_u,
                            int32_t* qp_status, int max_iter, int qp_max_iter, double tol,
                            void* ws, size_t ws_bytes, void* stream);

/*
 * mpcqp_bicycle_mpc_loop: the receding-horizon loop of the controller above
 * (rcracers.simulate(x0, dynamics, n_steps, policy=controller), session_4/
 * main.py:270-271; session4_sol.py:458,465) for T samples in ONE launch, one
 * workgroup per instance (closed_loop.ClosedLoop in fused mode).  Per sample
 * t: the SQP of mpcqp_bicycle_sqp_solve from x_t = xs[t] (up to iters_first
 * iterations at t = 0, iters after), the ControllerLog record
 * (session_2/log.py:8-12: success[t] (int8), iters_out[t], state_prediction
 * [t] = the SQP's X ((N+1) x 4), input_prediction[t] = U (N x 2)), the plant
 * xs[t+1] = F(x_t, U[0]) with its own parameters plant_params and model
 * plant (MPCQP_PLANT_*, substeps) and us[t] = U[0], then the warm start of
 * mpcqp_sqp_shift (U, y, pi one stage forward; flags, rho 0; mu = mu0; kkt
 * = inf).  Every instance runs its own episode.  xs (T+1) x batch x 4 with
 * xs[0] given; the SQP state as mpcqp_bicycle_sqp_solve's (reset by the
 * caller before the first sample).  N <= 64.  workspace:
 * mpcqp_bicycle_sqp_solve_workspace().  fp64.
 */
int mpcqp_bicycle_mpc_loop(int dtype, int batch, int N, int T, double ts, const double* params,
                           int integrator, int hessian, const double* plant_params, int plant,
                           int substeps, const void* Q, const void* R, const void* Qf,
                           const void* xlo, const void* xhi, int64_t strideXb, const void* lb,
                           const void* ub, int64_t strideLb, void* U, void* y, void* pi, void* X,
                           double* rho, double* kkt, double* mu, int32_t* flags, int32_t* fix,
                           int iters_first, int iters, int qp_max_iter, double tol, double mu0,
                           void* xs, void* us, void* success, int32_t* iters_out,
                           void* state_prediction, void* input_prediction, void* ws,
                           size_t ws_bytes, void* stream);

/*
 * The receding-horizon loop on device (rcracers.simulate(x0, dynamics,
 * n_steps, policy=controller), session_4/main.py:270-271; session4_sol.py:
 * 458,465), one step of it per call pair:
 * mpcqp_bicycle_plant: x_next = F(x, u) with u = U[b][0..1] (instance stride
 *   strideU: the first input of each instance's solution, __call__
 *   main.py:121-129), F = MPCQP_PLANT_FE (fwd_euler, main.py:132-135),
 *   MPCQP_PLANT_RK4 (runge_kutta4, main.py:138-147) or MPCQP_PLANT_RK4_SUB
 *   (RK4 over `substeps` sub-intervals: the stand-in for odeint,
 *   exact_integration main.py:150-170) with the PLANT's parameters (which
 *   may differ from the controller's, session4_sol.py:461-462); u_rec
 *   (optional, 2 per instance) records u.  x, x_next: 4 per instance.
 * mpcqp_sqp_shift: warm start of the next step -- U (N x 2), y, pi (N x 4)
 *   move one stage forward (last stage repeated; NULL = skip) and the SQP
 *   state restarts (flags 0, rho 0, mu = mu0, kkt = inf; NULL = skip).
 * Both are plain launches on the stream, so a T-step loop of
 * (MPC step; plant; shift) can be captured in one HIP graph.  fp64.
 */
#define MPCQP_PLANT_FE 0
#define MPCQP_PLANT_RK4 1
#define MPCQP_PLANT_RK4_SUB 2
int mpcqp_bicycle_plant(int dtype, int batch, double ts, const double* params, int integrator,
                        int substeps, const void* x, const void* U, int64_t strideU,
                        void* x_next, void* u_rec, void* stream);
int mpcqp_sqp_shift(int dtype, int batch, int N, void* U, void* y, void* pi, int32_t* flags,
                    double* rho, double* mu, double* kkt, double mu0, void* stream);

/*
 * The receding-horizon loop of an input-box MPC on a linear plant, T steps in
 * one launch (session_1 LinearSystem.simulate, LinearSystem.py:20-26, under
 * the box-constrained MPC policy of session_4 MPCController.solve,
 * main.py:115-116 / input box main.py:68-69; simulate(...) main.py:270-271):
 *   for t = 0..steps-1:  z_t = argmin 1/2 z'Hz + (F x_t)'z,  lb <= z <= ub
 *                        x_{t+1} = A x_t + B u_0(z_t)
 * H (packed lower n(n+1)/2, n = N*nu) and F (n x nx) are the instance's
 * condensed problem (mpcqp_condense of the same plant, once per episode);
 * A (nx x nx), Bm (nx x nu) the plant (stride 0 = shared).  Each step is
 * warm-started from the previous active set shifted one stage.  Outputs:
 * xs ((steps+1) x batch x nx: x_0..x_T), us (steps x batch x nu: the applied
 * u_0), zs (optional, steps x batch x n: the input plans, the
 * input_prediction of ControllerLog), status (steps x batch; bits 8..23 =
 * sweeps + active-set iterations of the step; us and status may be NULL
 * when steps = 0).  Limits: nx <= 4, nu <= 2, N*nu <= 32.
 */
int mpcqp_mpc_box_loop(int dtype, int batch, int nx, int nu, int N, int steps,
                       const void* H, int64_t strideH, const void* F, int64_t strideF,
                       const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                       const void* x0, int64_t strideX0, const void* lb, int64_t strideLb,
                       const void* ub, int64_t strideUb, void* xs, void* us, void* zs,
                       int32_t* status, int max_iter, double tol, void* stream);

/*
 * Batched finite-horizon Riccati recursion, FHC.py:51-61:
 *   K_k = -(R + B'P B)^{-1} B'P A,  P_k = Q + A'P A + A'P B K_k,  P_N = Pf
 * Outputs in the reference's order (lists reversed: K[0] is the first-stage
 * gain): P (N+1)*nx*nx, K N*nu*nx per instance.  nx, nu <= 4.
 */
int mpcqp_riccati(int dtype, int batch, int nx, int nu, int N,
                  const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                  const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                  const void* Pf, int64_t stridePf, void* P, void* K, void* stream);

/*
 * Batched re-linearisation of the kinematic bicycle for the RTI step of
 * MPCController (session_4/main.py:41-113 on fwd_euler(KinematicBicycle),
 * main.py:132-135, 250-251): per instance, roll the forward-Euler model out
 * from x0 (4) under U (N x 2, the warm start) and write, for k = 0..N-1,
 *   A_k = I + ts df/dx (N x 4 x 4), B_k = ts df/du (N x 4 x 2),
 *   c_k = fd(x_k,u_k) - A_k x_k - B_k u_k (N x 4),
 * and optionally the rolled-out states X (N+1 x 4).  Layouts match
 * mpcqp_condense with MPCQP_TV.  params = {l_f, l_r, acceleration, friction}
 * (parameters.py:7-8,47-48).  x = [p_x, p_y, psi, v], u = [a, delta].
 */
int mpcqp_bicycle_rti(int dtype, int batch, int N, double ts, const double* params,
                      const void* x0, int64_t strideX0, const void* U, int64_t strideU,
                      void* X, void* A, void* B, void* c, void* stream);

/* Batched  y_b = alpha * M_b x_b + beta * y_b,  M_b (rows x cols) row-major. */
int mpcqp_gemv(int dtype, int batch, int rows, int cols, double alpha,
               const void* M, int64_t strideM, const void* x, int64_t strideX,
               double beta, void* y, int64_t strideY, void* stream);

/*
 * Batched closed-loop rollout of LinearSystem.simulate (LinearSystem.py:20-26)
 * with u_t = K x_t (AutoCruising.control_law, FHC.py:25-26):
 *   x_{t+1} = A x_t + B K x_t,  t = 1..steps-1.
 * A, Bm, K shared; x0 (batch x nx); xs out TIME-MAJOR (steps x batch x nx),
 * whose (2,1,0) permutation is the reference's (nx, batch, steps) state
 * tensor (LinearSystem.py:21,26).  nx, nu <= 16.
 */
int mpcqp_rollout(int dtype, int batch, int nx, int nu, int steps,
                  const void* A, const void* Bm, const void* K,
                  const void* x0, void* xs, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPCQP_H */
