// ipm.hip -- mpcqp_mpc_ipm: one MPC step with input box and state box on the
// stage-wise (non-condensed) structure, one instance per lane, for any
// horizon.  The algorithm is in ipm_lane.hpp (primal-dual interior point,
// Mehrotra predictor-corrector, Riccati factorisation per iteration).
//
// Where it sits: the condensed kernels (mpcqp_mpc_qp's sweep + product-form
// and workgroup active sets) hold dense (N(nu+nx))^2 matrices and stop at
// N(nu+nx) = 192.  The reference's own controllers go beyond that:
// session4_sol.py:342,391,445 run N = 50 with the state box of
// session4_sol.py:176-181 and the input box, i.e. n + m = 100 + 200.  Here the
// work per iteration is O(N (nx+nu)^3) and the memory O(N), so the horizon is
// unbounded; mpcqp_mpc_qp routes such steps here.
//
// Mapping: lane = instance, 64 instances per workgroup (one wave).  Every lane
// runs the same sequence of operations on its own data (no divergence except
// the iteration count, which the wave pays as its maximum), and every
// workspace access is one fp64 per lane at consecutive addresses.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

#define MPCQP_HD __host__ __device__
#include "ipm_lane.hpp"
#include "ipm_quad.hpp"
#include "ipm_wave.hpp"

namespace mpcqp {

template <typename T, int NX, int NU>
__global__ __launch_bounds__(64) void ipm_kernel(ipm::Args<T> a) {
  if (a.list) {
    const int cnt = *a.list_count;
    for (int k = a.list_begin + blockIdx.x * 64 + threadIdx.x; k < cnt; k += gridDim.x * 64)
      ipm::solve_lane<T, NX, NU>(a, a.list[k]);
    return;
  }
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= a.batch) return;
  ipm::solve_lane<T, NX, NU>(a, b);
}

// The same lane routine with the instance's workspace in LDS: G instances
// per single-wave workgroup (lanes >= G idle), field stride G doubles so the
// active lanes hit consecutive banks.  Every workspace access is then an LDS
// round trip instead of an HBM one; it is the latency-bound small/medium-batch
// variant (the per-stage sweeps are serial in each lane either way).
template <typename T, int NX, int NU, int G>
__global__ __launch_bounds__(64) void ipm_lds_kernel(ipm::Args<T> a) {
  extern __shared__ __attribute__((aligned(16))) double ipm_lds[];
  const int lane = threadIdx.x;
  if (lane >= G) return;
  if (a.list) {
    const int cnt = *a.list_count;
    for (int k = a.list_begin + blockIdx.x * G + lane; k < cnt; k += gridDim.x * G)
      ipm::solve_lane<T, NX, NU, G>(a, a.list[k], ipm_lds + lane);
    return;
  }
  const int b = blockIdx.x * G + lane;
  if (b >= a.batch) return;
  ipm::solve_lane<T, NX, NU, G>(a, b, ipm_lds + lane);
}

// Four lanes per instance (ipm_quad.hpp), G instances per workgroup, the
// workspace in LDS.  The (4, 2) shapes whose horizon fits 160 KB of LDS.
template <typename T, int G>
__global__ __launch_bounds__(64, 1) void ipm_quad_kernel(ipm::Args<T> a) {
  extern __shared__ __attribute__((aligned(16))) double ipm_lds[];
  const int g = threadIdx.x >> 2;
  if (g >= G) return;
  if (a.list) {
    // the group's four lanes take the same entries (uniform trip count)
    const int cnt = *a.list_count;
    for (int k = a.list_begin + blockIdx.x * G + g; k < cnt; k += gridDim.x * G)
      ipmq::solve_quad<T, G>(a, a.list[k], ipm_lds + g);
    return;
  }
  const int b = blockIdx.x * G + g;
  if (b >= a.batch) return;
  ipmq::solve_quad<T, G>(a, b, ipm_lds + g);
}

// One instance per single-wave workgroup on the whole wave (ipm_wave.hpp):
// the stage data staged one quad per stage, the per-stage work of every pass
// on the 16 quads, the Riccati chains on quad 0.  Same iterates as
// ipm_quad_kernel<T, 1> up to the summation order of the reductions.
template <typename T>
__global__ __launch_bounds__(64, 1) void ipm_wave_kernel(ipm::Args<T> a) {
  extern __shared__ __attribute__((aligned(16))) double ipm_lds[];
  const int lane = threadIdx.x;
  const ipmq::WsQ<1> at(ipm_lds, lane & 3);
  auto one = [&](int b) {
    if (a.skip && (a.skip[b] & a.skip_mask)) return;
    for (int k = lane >> 2; k < a.N; k += kWave / 4) ipmq::stage_in_q(a, b, at, lane & 3, k);
    wave_lds_sync();
    ipmw::solve_wave<T>(a, b, ipm_lds);
    wave_lds_sync();
  };
  if (a.list) {
    const int cnt = *a.list_count;
    for (int k = a.list_begin + blockIdx.x; k < cnt; k += gridDim.x) one(a.list[k]);
    return;
  }
  if ((int)blockIdx.x < a.batch) one((int)blockIdx.x);
}

static int64_t ipm_ldb(int batch) { return ((int64_t)batch + 63) / 64 * 64; }

// list mode: workgroups of the launch (each loops over its share of the list)
constexpr int kListGrid = 1024;
static unsigned ipm_grid(const int64_t units, bool list) {
  return (unsigned)(list && units > kListGrid ? kListGrid : units);
}

// LDS variant: instances per workgroup (1, 2 or 4; 0 = the global-workspace
// kernel), within the 160 KB of one CU.  MPCQP_IPM_LDS=0/1 forces the choice.
static int ipm_lds_group(int batch, int F, int N) {
  const size_t per = (size_t)N * F * sizeof(double);
  const char* env = getenv("MPCQP_IPM_LDS");
  if (env && atoi(env) == 0) return 0;
  const size_t budget = 160 * 1024;
  if (per > budget) return 0;
  const int G = per * 4 <= budget ? 4 : (per * 2 <= budget ? 2 : 1);
  // large batches: the global-workspace kernel keeps 64 lanes busy per wave
  const bool small = (int64_t)batch <= (int64_t)256 * 4 * G;
  if (!small && !(env && atoi(env) == 1)) return 0;
  return G;
}

static bool ipm_dims(int nx, int nu, int& NX, int& NU) {
  if (nx <= 2 && nu <= 1) { NX = 2; NU = 1; return true; }
  if (nx <= 4 && nu <= 2) { NX = 4; NU = 2; return true; }
  return false;
}

size_t ipm_ws_bytes(int batch, int nx, int nu, int N) {
  int NX, NU;
  if (batch <= 0 || N < 1 || !ipm_dims(nx, nu, NX, NU)) return 0;
  const int F = (NX == 2) ? ipm::Layout<2, 1>::F : ipm::Layout<4, 2>::F;
  return (size_t)N * F * ipm_ldb(batch) * sizeof(double);
}

bool ipm_supported(int nx, int nu) {
  int NX, NU;
  return ipm_dims(nx, nu, NX, NU);
}

template <typename T>
static int ipm_quad_launch(ipm::Args<T>& a, hipStream_t st) {
  const int F = ipm::Layout<4, 2>::F;
  const size_t per = (size_t)a.N * F * sizeof(double);
  // One instance per single-wave workgroup: the CU's four SIMDs then each run
  // a wave (four instances in one wave left three SIMDs idle, LDS allowing one
  // such workgroup per CU).  Measured at the nlp line (N = 30, B = 4096, the
  // SQP's strict QPs): 12.2 ms per interior-point launch against 15.0 ms
  // (four per workgroup) and 13.4 ms (two).
  int G = 1;
  if (const char* env = getenv("MPCQP_IPM_G")) {  // A/B: instances per workgroup
    const int g = atoi(env);
    if ((g == 1 || g == 2 || g == 4) && (size_t)g * per <= 160 * 1024) G = g;
  }
  const size_t bytes = (size_t)G * per;
  const char* wenv = getenv("MPCQP_IPM_WAVE");  // A/B: 0 = the quad kernel at G = 1
  const bool wave = G == 1 && !(wenv && atoi(wenv) == 0);
  auto launch = [&](auto kern) -> int {
    if (bytes > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)kern,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
      if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(ipm_quad)");
    }
    hipLaunchKernelGGL(kern, dim3(ipm_grid((a.batch + G - 1) / G, a.list)), dim3(64), bytes, st, a);
    MPCQP_CHECK_LAUNCH("ipm_quad_kernel");
    return MPCQP_OK;
  };
  if (G == 4) return launch(ipm_quad_kernel<T, 4>);
  if (G == 2) return launch(ipm_quad_kernel<T, 2>);
  if (wave) return launch(ipm_wave_kernel<T>);
  return launch(ipm_quad_kernel<T, 1>);
}

// The quad kernel for the (4, 2) shapes whose horizon fits LDS;
// MPCQP_IPM_QUAD=0 selects the lane-per-instance kernels instead.
static bool ipm_use_quad(int N) {
  const char* env = getenv("MPCQP_IPM_QUAD");
  if (env && atoi(env) == 0) return false;
  return (size_t)N * ipm::Layout<4, 2>::F * sizeof(double) <= 160 * 1024;
}

template <typename T, int NX, int NU>
static int ipm_launch_t(ipm::Args<T>& a, hipStream_t st) {
  if constexpr (NX == 4 && NU == 2) {
    if (ipm_use_quad(a.N)) return ipm_quad_launch(a, st);
  }
  const int F = ipm::Layout<NX, NU>::F;
  const int G = ipm_lds_group(a.batch, F, a.N);
  const dim3 blk(64);
  if (G > 0) {
    const size_t bytes = (size_t)G * a.N * F * sizeof(double);
    auto launch = [&](auto kern) -> int {
      if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(ipm_lds)");
      }
      hipLaunchKernelGGL(kern, dim3(ipm_grid((a.batch + G - 1) / G, a.list)), blk, bytes, st, a);
      MPCQP_CHECK_LAUNCH("ipm_lds_kernel");
      return MPCQP_OK;
    };
    if (G == 4) return launch(ipm_lds_kernel<T, NX, NU, 4>);
    if (G == 2) return launch(ipm_lds_kernel<T, NX, NU, 2>);
    return launch(ipm_lds_kernel<T, NX, NU, 1>);
  }
  hipLaunchKernelGGL((ipm_kernel<T, NX, NU>), dim3(ipm_grid((a.batch + 63) / 64, a.list)), blk, 0,
                     st, a);
  MPCQP_CHECK_LAUNCH("ipm_kernel");
  return MPCQP_OK;
}

template <typename T>
static int ipm_launch(ipm::Args<T>& a, hipStream_t st) {
  int NX, NU;
  ipm_dims(a.nx, a.nu, NX, NU);
  return NX == 2 ? ipm_launch_t<T, 2, 1>(a, st) : ipm_launch_t<T, 4, 2>(a, st);
}

// inertia corrections a strict QP may take before NOT_CONVEX (6; the
// environment variable MPCQP_IPM_STRICT overrides it for experiments)
static int strict_corrections() {
  static const int n = [] {
    const char* e = getenv("MPCQP_IPM_STRICT");
    return e ? atoi(e) : 6;
  }();
  return n;
}

int mpc_ipm_impl(int dtype, int batch, int nx, int nu, int N, int flags, const void* A,
                 int64_t sA, const void* Bm, int64_t sB, const void* Q, int64_t sQ, const void* R,
                 int64_t sR, const void* Qf, int64_t sQf, const void* c, int64_t sC,
                 const void* x0, int64_t sX0, const void* xlo, const void* xhi, int64_t sXb,
                 const void* lb, int64_t sLb, const void* ub, int64_t sUb, const void* U0,
                 int64_t sU0, const void* H2, int64_t sH2, const void* q2, int64_t sq2, void* z,
                 void* y, void* X, void* lam_u, void* pi, int32_t* status,
                 const int32_t* skip, int32_t skip_mask, int max_iter, double tol, void* ws,
                 size_t ws_bytes, hipStream_t st, const int* list, const int* list_count,
                 int list_begin) {
  const size_t need = ipm_ws_bytes(batch, nx, nu, N);
  MPCQP_CHECK_ARG(ws && ws_bytes >= need, "mpcqp_mpc_ipm: workspace %zu bytes < %zu", ws_bytes,
                  need);
  auto fill = [&](auto& a, auto tp) {
    using T = decltype(tp);
    a.batch = batch; a.nx = nx; a.nu = nu; a.N = N; a.tv = (flags & MPCQP_TV) ? 1 : 0;
    a.max_iter = max_iter > 0 ? max_iter : 100;
    a.strict = (flags & MPCQP_STRICT) ? strict_corrections() : 0;  // before NOT_CONVEX
    a.tol = tol > 0 ? tol : 1e-10;
    a.tol_mu = 1e-2 * a.tol;
    a.tol_polish = 1e-6;
    a.mu_polish = 1e-6;
    a.A = (const T*)A; a.sA = sA; a.B = (const T*)Bm; a.sB = sB; a.c = (const T*)c; a.sC = sC;
    a.Q = (const T*)Q; a.sQ = sQ; a.R = (const T*)R; a.sR = sR; a.Qf = (const T*)Qf; a.sQf = sQf;
    a.x0 = (const T*)x0; a.sX0 = sX0;
    a.xlo = (const T*)xlo; a.xhi = (const T*)xhi; a.sXb = sXb;
    a.lb = (const T*)lb; a.sLb = sLb; a.ub = (const T*)ub; a.sUb = sUb;
    a.U0 = (const T*)U0; a.sU0 = sU0;
    a.H2 = (const T*)H2; a.sH2 = sH2; a.q2 = (const T*)q2; a.sq2 = sq2;
    a.z = (T*)z; a.y = (T*)y; a.X = (T*)X; a.lam_u = (T*)lam_u; a.pi = (T*)pi; a.status = status;
    a.skip = skip; a.skip_mask = skip_mask;
    a.ws = (double*)ws;
    a.list = list; a.list_count = list_count; a.list_begin = list_begin;
  };
  if (dtype == MPCQP_F64) {
    ipm::Args<double> a;
    fill(a, 0.0);
    return ipm_launch(a, st);
  }
  ipm::Args<float> a;
  fill(a, 0.0f);
  return ipm_launch(a, st);
}

}  // namespace mpcqp

extern "C" size_t mpcqp_mpc_ipm_workspace(int dtype, int batch, int nx, int nu, int N) {
  if (dtype != MPCQP_F64 && dtype != MPCQP_F32) return 0;
  return mpcqp::ipm_ws_bytes(batch, nx, nu, N);
}

extern "C" int mpcqp_mpc_ipm(int dtype, int batch, int nx, int nu, int N, int flags,
                             const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                             const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                             const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                             const void* x0, int64_t strideX0, const void* xlo, const void* xhi,
                             int64_t strideXb, const void* lb, int64_t strideLb, const void* ub,
                             int64_t strideUb, const void* U0, int64_t strideU0, const void* H2,
                             int64_t strideH2, const void* q2, int64_t strideq2, void* z, void* y,
                             void* X, void* lam_u, void* pi, int32_t* status,
                             const int32_t* skip, int32_t skip_mask, int max_iter, double tol,
                             void* ws, size_t ws_bytes, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_mpc_ipm: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "mpcqp_mpc_ipm: bad sizes (batch=%d, N=%d)", batch, N);
  MPCQP_CHECK_ARG(nx >= 1 && nu >= 1, "mpcqp_mpc_ipm: nx=%d nu=%d", nx, nu);
  if (!ipm_supported(nx, nu)) {
    set_error("mpcqp_mpc_ipm: nx=%d nu=%d outside the compiled set (nx <= 4, nu <= 2)", nx, nu);
    return MPCQP_ENOTSUP;
  }
  MPCQP_CHECK_ARG(A && Bm && Q && R && Qf && x0 && z && status,
                  "mpcqp_mpc_ipm: A, B, Q, R, Qf, x0, z, status are required");
  MPCQP_CHECK_ARG(strideA >= 0 && strideB >= 0 && strideQ >= 0 && strideR >= 0 && strideQf >= 0 &&
                      strideC >= 0 && strideX0 >= 0 && strideXb >= 0 && strideLb >= 0 &&
                      strideUb >= 0 && strideU0 >= 0 && strideH2 >= 0 && strideq2 >= 0,
                  "mpcqp_mpc_ipm: negative stride");
  if (batch == 0) return MPCQP_OK;
  return mpc_ipm_impl(dtype, batch, nx, nu, N, flags, A, strideA, Bm, strideB, Q, strideQ, R,
                      strideR, Qf, strideQf, c, strideC, x0, strideX0, xlo, xhi, strideXb, lb,
                      strideLb, ub, strideUb, U0, strideU0, H2, strideH2, q2, strideq2, z, y, X,
                      lam_u, pi, status, skip, skip_mask, max_iter, tol, ws, ws_bytes,
                      (hipStream_t)stream, nullptr, nullptr, 0);
}
