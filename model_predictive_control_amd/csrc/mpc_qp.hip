// mpc_qp.hip -- one MPC step with input box AND state box, end to end:
// the whole MPCController.solve of session_4/main.py:115-116 for the OCP of
// main.py:41-113 with the input bounds lbx/ubx (main.py:68-69) and the state
// bounds lbg/ubg on x_1..x_N (main.py:58-61, session4_sol.py:176-181),
// linear(ised) dynamics.  BASELINE configs 3 (state + input box) and 5
// (input box only, the large horizon).
//
//   1. mpcqp_condense (TV or shared plant)    -> H, f [, Gam, xbar]   (workspace)
//   2. rows_kernel                            -> hl = xlo - xbar, hu = xhi - xbar
//   3. fp32 with n + m > 64: sweep (MFMA) -> product-form active set whose
//      iterative refinement takes its KKT residual from the DYNAMICS in fp64
//      (solve_pf.hip, PfDyn) -> workgroup kernel for hand-offs;
//      otherwise (fp64, small QPs): mpcqp_solve_box (input box only) or the
//      workgroup kernel (mpcqp_solve_qp).
//   4. optional: states_kernel -> X = x_1..x_N of the solution (fp64 rollout),
//      the "g" rows IPOPT reports and the state_prediction of the
//      ControllerLog (session_2/log.py:12).
//
// The refinement residual from the dynamics is what lets the fp32 path reach
// the fp64 solution of the QP its inputs define: the condensed H, Gam, xbar
// carry fp32 rounding of the recursion (cond(H) ~ 1e4 at config 3), which a
// residual from them cannot see.
#include <cstdlib>

#include "pf.hpp"
#include "quad_api.hpp"

namespace mpcqp {

template <typename T>
__global__ void rows_kernel(int64_t total, int m, const T* xlo, const T* xhi, int64_t sXb,
                            const T* xbar, T* hl, T* hu) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int64_t b = e / m;
  const int j = (int)(e - b * m);
  const T xb = xbar[e];
  const T inf = Lim<T>::inf();
  hl[e] = (xlo ? xlo[b * sXb + j] : -inf) - xb;
  hu[e] = (xhi ? xhi[b * sXb + j] : inf) - xb;
}

// X = [x_1; ..; x_N] of z, one instance per lane, fp64 accumulation.
template <typename T, int NX>
__global__ void states_kernel(int batch, int nx, int nu, int N, int tv, const T* A, int64_t sA,
                              const T* Bm, int64_t sB, const T* c, int64_t sC, const T* x0,
                              int64_t sX0, const T* z, T* X) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double x[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) x[i] = i < nx ? (double)x0[(int64_t)b * sX0 + i] : 0.0;
  const T* Ab = A + (int64_t)b * sA;
  const T* Bb = Bm + (int64_t)b * sB;
  const T* cb = c ? c + (int64_t)b * sC : nullptr;
  const T* zb = z + (int64_t)b * N * nu;
  T* Xb = X + (int64_t)b * N * nx;
  for (int s = 0; s < N; ++s) {
    const T* As = Ab + (tv ? (int64_t)s * nx * nx : 0);
    const T* Bs = Bb + (tv ? (int64_t)s * nx * nu : 0);
    double xn[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      double acc = (cb && i < nx) ? (double)cb[s * nx + i] : 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j)
        if (i < nx && j < nx) acc = fma((double)As[i * nx + j], x[j], acc);
      for (int a = 0; a < nu; ++a)
        if (i < nx) acc = fma((double)Bs[i * nu + a], (double)zb[s * nu + a], acc);
      xn[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      x[i] = xn[i];
      if (i < nx) Xb[s * nx + i] = (T)xn[i];
    }
  }
}

static size_t al256(size_t v) { return (v + 255) / 256 * 256; }

// workspace of the dense path with its fp64 fallback: the dense layout (the
// hand-off list is in it), then the interior point's workspace
// the fp64 hand-off's workspace (the interior point's or fallback64.hip's
// slots, which run one after the other) after the dense path's data
static size_t mpc_fallback_bytes(size_t dense, size_t ipm, size_t fb64) {
  return al256(dense) + (ipm > fb64 ? ipm : fb64);
}

struct MpcWs {
  size_t H, f, Gam, xbar, hl, hu, qp, total;
};

static MpcWs mpc_ws_layout(int dtype, int batch, int nx, int nu, int N, int sbox) {
  const size_t es = dtype_size(dtype), B = (size_t)batch;
  const size_t n = (size_t)N * nu, m = sbox ? (size_t)N * nx : 0;
  MpcWs w{};
  size_t o = 0;
  w.H = o; o += al256(B * n * (n + 1) / 2 * es);
  w.f = o; o += al256(B * n * es);
  w.Gam = o; o += al256(B * m * n * es);
  w.xbar = o; o += al256(B * m * es);
  w.hl = o; o += al256(B * m * es);
  w.hu = o; o += al256(B * m * es);
  w.qp = o; o += al256(qp_ws_bytes(dtype, batch, (int)n, (int)m));
  w.total = o;
  return w;
}

// most refinement steps with the dynamics residual (MPCQP_MPC_REFINE
// overrides); each instance stops once its correction is below kDynStop
static int mpc_refine() {
  const char* v = getenv("MPCQP_MPC_REFINE");
  return v ? atoi(v) : 4;
}

// MPCQP_MPC_DYN=0 refines against the condensed matrices instead (A/B checks)
static bool mpc_dyn() {
  const char* v = getenv("MPCQP_MPC_DYN");
  return v ? atoi(v) != 0 : true;
}

// MPCQP_MPC_ZF=0 keeps configs of the z-space kernel (solve_zf.hip) on the
// dense sweep + product-form path (A/B)
static bool mpc_zf() {
  const char* v = getenv("MPCQP_MPC_ZF");
  return v ? atoi(v) != 0 : true;
}

// MPCQP_MPC_FALLBACK=wg sends uncertified instances to the fp32 workgroup
// kernel (flagged MPCQP_STATUS_UNREFINED) instead of the fp64 hand-off;
// =ipm keeps the whole hand-off on the fp64 interior point (A/B)
static bool mpc_fallback_f64() {
  const char* v = getenv("MPCQP_MPC_FALLBACK");
  return !(v && v[0] == 'w');
}
// MPCQP_MPC_FALLBACK=none (diagnostics): no hand-off, the fp32 kernels'
// hand-off status (0x7f, reason in bits 24..27) is left in place
static bool mpc_fallback_none() {
  const char* v = getenv("MPCQP_MPC_FALLBACK");
  return v && v[0] == 'n';
}
static bool mpc_fallback_ipm_only() {
  const char* v = getenv("MPCQP_MPC_FALLBACK");
  return v && v[0] == 'i';
}

template <typename T>
static int launch_states(int batch, int nx, int nu, int N, int tv, const void* A, int64_t sA,
                         const void* Bm, int64_t sB, const void* c, int64_t sC, const void* x0,
                         int64_t sX0, const void* z, void* X, hipStream_t st) {
  const dim3 grid((batch + 255) / 256), blk(256);
#define MPCQP_STATES(NXT)                                                                     \
  hipLaunchKernelGGL((states_kernel<T, NXT>), grid, blk, 0, st, batch, nx, nu, N, tv,         \
                     (const T*)A, sA, (const T*)Bm, sB, (const T*)c, sC, (const T*)x0, sX0,   \
                     (const T*)z, (T*)X)
  if (nx <= 4) MPCQP_STATES(4);
  else if (nx <= 8) MPCQP_STATES(8);
  else if (nx <= 12) MPCQP_STATES(12);
  else MPCQP_STATES(16);
#undef MPCQP_STATES
  MPCQP_CHECK_LAUNCH("states_kernel");
  return MPCQP_OK;
}

// Stage timing of mpcqp_mpc_qp (bench.py's per-kernel rooflines): while
// enabled, every call records a HIP event on its stream before its first
// launch and after each stage (condense, sweep, solve, fp64 fallback,
// states); mpcqp_mpc_qp_stage_ms reads the last call's stage times.  A
// profiling facility for one host thread, off by default (an enabled call
// cannot be captured in a graph).
struct StageProf {
  int on = 0;
  bool done[kProfN] = {};
  hipEvent_t ev[kProfN] = {};
};
static StageProf g_prof;

void prof_mark(int stage, hipStream_t st) {
  if (!g_prof.on) return;
  if (hipEventRecord(g_prof.ev[stage], st) == hipSuccess) g_prof.done[stage] = true;
}

}  // namespace mpcqp

extern "C" int mpcqp_mpc_qp_profile(int enable) {
  using namespace mpcqp;
  if (enable && !g_prof.ev[0])
    for (int i = 0; i < kProfN; ++i) {
      const hipError_t e = hipEventCreate(&g_prof.ev[i]);
      if (e != hipSuccess) return hip_fail(e, "mpcqp_mpc_qp_profile: hipEventCreate");
    }
  g_prof.on = enable ? 1 : 0;
  return MPCQP_OK;
}

extern "C" int mpcqp_mpc_qp_stage_ms(float* ms) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(ms, "mpcqp_mpc_qp_stage_ms: null pointer");
  for (int i = 0; i + 1 < kProfN; ++i) ms[i] = -1.0f;
  if (!g_prof.done[kProfStart]) return MPCQP_OK;
  hipError_t e;
  int prev = kProfStart;
  for (int i = 1; i < kProfN; ++i) {
    if (!g_prof.done[i]) continue;
    e = hipEventSynchronize(g_prof.ev[i]);
    if (e != hipSuccess) return hip_fail(e, "mpcqp_mpc_qp_stage_ms: hipEventSynchronize");
    float t = 0.0f;
    e = hipEventElapsedTime(&t, g_prof.ev[prev], g_prof.ev[i]);
    if (e != hipSuccess) return hip_fail(e, "mpcqp_mpc_qp_stage_ms: hipEventElapsedTime");
    ms[i - 1] = t;
    prev = i;
  }
  return MPCQP_OK;
}

// the stage-wise interior point takes the step when the caller asks for it
// (MPCQP_IPM) or when the condensed QP exceeds the dense kernels' size
static bool mpc_use_ipm(int dtype, int nx, int nu, int N, int sbox, int flags) {
  if (!mpcqp::ipm_supported(nx, nu)) return false;
  if (flags & MPCQP_IPM) return true;
  return N * (nu + (sbox ? nx : 0)) > mpcqp::max_qp_size_dtype(dtype);
}

extern "C" size_t mpcqp_mpc_qp_workspace(int dtype, int batch, int nx, int nu, int N,
                                         int state_box) {
  if ((dtype != MPCQP_F64 && dtype != MPCQP_F32) || batch <= 0 || nx < 1 || nu < 1 || N < 1)
    return 0;
  const size_t dense = mpcqp::mpc_ws_layout(dtype, batch, nx, nu, N, state_box ? 1 : 0).total;
  // room for either path (the flags are not known here)
  const size_t ipm = mpcqp::ipm_supported(nx, nu) ? mpcqp::ipm_ws_bytes(batch, nx, nu, N) : 0;
  if (mpc_use_ipm(dtype, nx, nu, N, state_box ? 1 : 0, 0)) return ipm;
  // the dense path's fp64 hand-off after the condensed data
  const size_t fb64 =
      dtype == MPCQP_F32 ? mpcqp::fallback64_bytes(batch, nx, nu, N, state_box ? 1 : 0) : 0;
  return mpcqp::mpc_fallback_bytes(dense, ipm, fb64);
}

extern "C" int mpcqp_mpc_qp(int dtype, int batch, int nx, int nu, int N, int flags,
                            const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                            const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                            const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                            const void* x0, int64_t strideX0, const void* xlo, const void* xhi,
                            int64_t strideXb, const void* lb, int64_t strideLb, const void* ub,
                            int64_t strideUb, void* z, void* y, void* X, int32_t* status,
                            int max_iter, double tol, void* ws, size_t ws_bytes, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_mpc_qp: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_mpc_qp: batch < 0");
  MPCQP_CHECK_ARG(nx >= 1 && nx <= 16 && nu >= 1 && nu <= 16 && N >= 1,
                  "mpcqp_mpc_qp: nx=%d nu=%d N=%d outside nx, nu in [1,16], N >= 1", nx, nu, N);
  MPCQP_CHECK_ARG(A && Bm && Q && R && Qf && x0 && z && status,
                  "mpcqp_mpc_qp: A, B, Q, R, Qf, x0, z, status are required");
  MPCQP_CHECK_ARG(strideA >= 0 && strideB >= 0 && strideQ >= 0 && strideR >= 0 && strideQf >= 0 &&
                      strideC >= 0 && strideX0 >= 0 && strideXb >= 0 && strideLb >= 0 &&
                      strideUb >= 0,
                  "mpcqp_mpc_qp: negative stride");
  const int sbox = (xlo || xhi) ? 1 : 0;
  const int n = N * nu, m = sbox ? N * nx : 0;
  // stage timing: only a profiled call touches the (process-global) record,
  // and it clears it first, so a call routed to the interior point reports
  // -1 for every stage instead of the previous call's times
  if (g_prof.on)
    for (int i = 0; i < kProfN; ++i) g_prof.done[i] = false;
  if (mpc_use_ipm(dtype, nx, nu, N, sbox, flags)) {
    if (batch == 0) return MPCQP_OK;
    return mpc_ipm_impl(dtype, batch, nx, nu, N, flags, A, strideA, Bm, strideB, Q, strideQ, R,
                        strideR, Qf, strideQf, c, strideC, x0, strideX0, xlo, xhi, strideXb, lb,
                        strideLb, ub, strideUb, nullptr, 0, nullptr, 0, nullptr, 0, z, y, X,
                        nullptr, nullptr, status, nullptr, 0, max_iter, tol, ws, ws_bytes,
                        (hipStream_t)stream);
  }
  MPCQP_CHECK_ARG(n + m <= max_qp_size_dtype(dtype),
                  "mpcqp_mpc_qp: N*(nu%s) = %d exceeds the QP size limit %d", sbox ? "+nx" : "",
                  n + m, max_qp_size_dtype(dtype));
  if (batch == 0) return MPCQP_OK;
  const MpcWs L = mpc_ws_layout(dtype, batch, nx, nu, N, sbox);
  MPCQP_CHECK_ARG(ws && ws_bytes >= L.total, "mpcqp_mpc_qp: workspace %zu bytes < %zu", ws_bytes,
                  L.total);
  hipStream_t st = (hipStream_t)stream;
  prof_mark(kProfStart, st);
  char* w = (char*)ws;
  const int tv = (flags & MPCQP_TV) ? 1 : 0;
  void* Hw = w + L.H;
  void* fw = w + L.f;
  const size_t qpb = qp_ws_bytes(dtype, batch, n, m);
  const int64_t sH = (int64_t)n * (n + 1) / 2, sG = (int64_t)m * n;
  PfDyn d{};
  const bool dyn_ok = dtype == MPCQP_F32 && qpb > 0 && mpc_dyn() && dyn_nxp(nx, nu) > 0 &&
                      dyn_chunk_stages(nx, nu, N) >= 1;
  if (dyn_ok) {
    d.nx = nx; d.nu = nu; d.N = N; d.tv = tv;
    d.A = (const float*)A; d.sA = strideA;
    d.B = (const float*)Bm; d.sB = strideB;
    d.c = (const float*)c; d.sC = strideC;
    d.x0 = (const float*)x0; d.sX0 = strideX0;
    d.Q = (const float*)Q; d.sQ = strideQ;
    d.R = (const float*)R; d.sR = strideR;
    d.Qf = (const float*)Qf; d.sQf = strideQf;
    d.xlo = (const float*)xlo; d.xhi = (const float*)xhi; d.sXb = strideXb;
  }
  // An instance the fp32 kernels hand back -- more than 64 active
  // constraints, a non-finite state, or (DYN) a refined point they could not
  // certify as the QP's KKT point -- is solved again by the stage-wise fp64
  // interior point with its exact polish (status bit MPCQP_STATUS_POLISHED),
  // on the same inputs; it never returns OPTIMAL from the fp32 path
  // uncertified.  The fallback runs over the whole batch with every other
  // instance skipped, its workspace over the (then dead) condensed data.
  const QpWsParts P = qp_ws_parts(w + L.qp, batch, n, m);
  const size_t ipmb = ipm_supported(nx, nu) ? ipm_ws_bytes(batch, nx, nu, N) : 0;
  const size_t fb64b = fallback64_bytes(batch, nx, nu, N, sbox);
  const bool f64_fb = dyn_ok && mpc_fallback_f64() && ipmb > 0 &&
                      ws_bytes >= mpc_fallback_bytes(L.total, ipmb, fb64b);
  const bool use_fb64 = f64_fb && !mpc_fallback_ipm_only() && n + m <= max_qp_size_dtype(MPCQP_F64);
  // the first fallback64_cap(batch) listed instances: fp64 re-condensing +
  // the fp64 workgroup active set (fallback64.hip); the rest of the list on
  // the interior point in list mode (an empty remainder costs one short
  // launch)
  auto fallback_f64 = [&]() -> int {
    if (mpc_fallback_none()) return MPCQP_OK;
    if (use_fb64) {
      Fallback64In in;
      in.batch = batch; in.nx = nx; in.nu = nu; in.N = N; in.tv = tv;
      in.A = (const float*)A; in.sA = strideA; in.B = (const float*)Bm; in.sB = strideB;
      in.c = (const float*)c; in.sC = strideC; in.x0 = (const float*)x0; in.sX0 = strideX0;
      in.Q = (const float*)Q; in.sQ = strideQ; in.R = (const float*)R; in.sR = strideR;
      in.Qf = (const float*)Qf; in.sQf = strideQf;
      in.xlo = (const float*)xlo; in.xhi = (const float*)xhi; in.sXb = strideXb;
      in.lb = (const float*)lb; in.sLb = strideLb; in.ub = (const float*)ub; in.sUb = strideUb;
      const int rc = fallback64(in, P.list, P.cnt, (float*)z, (float*)y, status,
                                w + al256(L.total), fb64b, st);
      if (rc != MPCQP_OK) return rc;
    }
    return mpc_ipm_impl(MPCQP_F32, batch, nx, nu, N, flags & MPCQP_TV, A, strideA, Bm, strideB, Q,
                        strideQ, R, strideR, Qf, strideQf, c, strideC, x0, strideX0, xlo, xhi,
                        strideXb, lb, strideLb, ub, strideUb, nullptr, 0, nullptr, 0, nullptr, 0, z,
                        y, nullptr, nullptr, nullptr, status, nullptr, 0, 0, 0.0,
                        w + al256(L.total), ipmb, st, P.list, P.cnt,
                        use_fb64 ? fallback64_cap(batch) : 0);
  };
  // fp32 with 48 < n <= 64 (config 3): the z-space product form -- H and f
  // (and Gamma for the row normals) are condensed, H^-1 by the MFMA sweep
  const bool zf = dyn_ok && f64_fb && mpc_zf() && zf_supported(n, m, nx, nu, N);
  void* Gw = sbox ? w + L.Gam : nullptr;
  void* xbw = (sbox && !zf) ? w + L.xbar : nullptr;
  // the z-space kernel reads Gamma rows as normals: its lower block triangle
  // is all it needs (the upper one is structurally zero)
  const int cflags = (flags & MPCQP_TV) | (zf ? MPCQP_GAM_PACKED : 0);
  int rc = mpcqp_condense(dtype, batch, nx, nu, N, cflags, A, strideA, Bm, strideB, Q, strideQ, R,
                          strideR, Qf, strideQf, c, strideC, x0, strideX0, Hw, nullptr, fw, Gw,
                          nullptr, xbw, stream);
  if (rc != MPCQP_OK) return rc;
  prof_mark(kProfCondense, st);
  if (zf) {
    hipError_t e = hipMemsetAsync(P.cnt, 0, sizeof(int), st);
    if (e != hipSuccess) return hip_fail(e, "mpcqp_mpc_qp: hipMemsetAsync");
    const int mi = max_iter > 0 ? max_iter : 3 * (n + m) + 30;
    const float tl = tol > 0 ? (float)tol : 1e-6f;
    rc = sweep_hinv(batch, n, Hw, sH, fw, n, P.m0, P.s0, status, st);
    if (rc != MPCQP_OK) return rc;
    prof_mark(kProfSweep, st);
    rc = launch_zf(batch, n, m, (const float*)P.m0, (const float*)P.s0, (const float*)Gw,
                   (const float*)fw, n, (const float*)lb, strideLb, (const float*)ub, strideUb,
                   (float*)z, (float*)y, status, P.cnt, P.list, mi, mpc_refine(), tl, d, st);
    prof_mark(kProfSolve, st);
    if (rc == MPCQP_OK) rc = fallback_f64();
    if (rc != MPCQP_OK) return rc;
    prof_mark(kProfFallback, st);
    if (X) {
      rc = launch_states<float>(batch, nx, nu, N, tv, A, strideA, Bm, strideB, c, strideC, x0,
                                strideX0, z, X, st);
      prof_mark(kProfStates, st);
    }
    return rc;
  }
  void* hl = sbox ? w + L.hl : nullptr;
  void* hu = sbox ? w + L.hu : nullptr;
  if (sbox) {
    const int64_t total = (int64_t)batch * m;
    const dim3 grid((unsigned)((total + 255) / 256)), blk(256);
    if (dtype == MPCQP_F64)
      hipLaunchKernelGGL((rows_kernel<double>), grid, blk, 0, st, total, m, (const double*)xlo,
                         (const double*)xhi, strideXb, (const double*)xbw, (double*)hl,
                         (double*)hu);
    else
      hipLaunchKernelGGL((rows_kernel<float>), grid, blk, 0, st, total, m, (const float*)xlo,
                         (const float*)xhi, strideXb, (const float*)xbw, (float*)hl, (float*)hu);
    MPCQP_CHECK_LAUNCH("rows_kernel");
  }
  if (qpb > 0) {
    // a missing side of the state box has no finite bound: no row can be
    // active on it, so the residual never reads it
    rc = solve_two_kernel(batch, n, m, Hw, sH, fw, n, Gw, sG, hl, hu, m, lb, strideLb, ub,
                          strideUb, z, y, status, max_iter, tol, w + L.qp, st,
                          dyn_ok ? &d : nullptr, dyn_ok ? mpc_refine() : -1, f64_fb ? 0 : 1);
    prof_mark(kProfSolve, st);
    if (rc == MPCQP_OK && f64_fb) rc = fallback_f64();
    if (rc == MPCQP_OK && f64_fb) prof_mark(kProfFallback, st);
  } else if (m == 0) {  // input box only: the wavefront box kernels
    rc = mpcqp_solve_box(dtype, batch, n, Hw, sH, fw, n, lb, strideLb, ub, strideUb, z, status,
                         max_iter, tol, stream);
  } else {
    rc = mpcqp_solve_qp(dtype, batch, n, m, Hw, sH, fw, n, Gw, sG, hl, hu, m, lb, strideLb, ub,
                        strideUb, z, y, status, max_iter, tol, stream);
  }
  if (rc != MPCQP_OK) return rc;
  if (!(qpb > 0)) prof_mark(kProfSolve, st);
  if (X) {
    rc = dtype == MPCQP_F64
             ? launch_states<double>(batch, nx, nu, N, tv, A, strideA, Bm, strideB, c, strideC,
                                     x0, strideX0, z, X, st)
             : launch_states<float>(batch, nx, nu, N, tv, A, strideA, Bm, strideB, c, strideC,
                                    x0, strideX0, z, X, st);
    prof_mark(kProfStates, st);
  }
  return rc;
}
