// fallback64.hip -- the fp64 hand-off of mpcqp_mpc_qp's fp32 paths.
//
// The fp32 kernels (solve_zf.hip, solve_pf.hip) list the instances they
// could not certify as KKT points of the QP (and those with more active
// constraints than they hold).  Those are solved again here in fp64, from the
// caller's own data:
//   gather    the listed instances' A_k, B_k, c_k, x0, weights, bounds
//             (fp32 -> fp64) into compact slots 0..cnt-1
//   condense  condense_kernel<double> on the slots (workgroups past the
//             device count return at once)
//   rows      state-box rows xlo - xbar <= Gamma z <= xhi - xbar
//   solve     the fp64 workgroup active set (qp_wg_count_kernel): dual
//             Goldfarb-Idnani with its exact vertex solution
//   scatter   z, y back to the listed instances (fp32), status with
//             MPCQP_STATUS_POLISHED on an optimal solve
// Every step is a persistent launch over the device count, so the host
// never reads the count and the hand-off stays graph-capturable.  The
// latency is one workgroup QP (a few hundred microseconds at config 3)
// rather than the stage-wise interior point's serial sweeps (1.3 ms for a
// single instance there); the interior point keeps the list entries past
// the slot capacity.
#include <cstdlib>

#include "common.hpp"
#include "quad_api.hpp"

namespace mpcqp {

namespace {

struct Fb64Layout {
  int SA, SB, SC, SH, n, m, cap;
  size_t oA, oB, oC, oX0, oQ, oR, oQf, oH, of, oGam, oXbar, oHl, oHu, oLb, oUb, oZ, oY, oSt,
      total;
};

size_t al256(size_t b) { return (b + 255) / 256 * 256; }

Fb64Layout fb64_layout(int batch, int nx, int nu, int N, int tv, int sbox) {
  Fb64Layout L;
  const int S = tv ? N : 1;
  L.n = N * nu;
  L.m = sbox ? N * nx : 0;
  L.cap = fallback64_cap(batch);
  L.SA = S * nx * nx;
  L.SB = S * nx * nu;
  L.SC = N * nx;
  L.SH = L.n * (L.n + 1) / 2;
  const size_t c = (size_t)L.cap * sizeof(double);
  size_t o = 0;
  auto take = [&](size_t elems) {
    const size_t at = o;
    o += al256(elems * c);
    return at;
  };
  L.oA = take(L.SA);
  L.oB = take(L.SB);
  L.oC = take(L.SC);
  L.oX0 = take(nx);
  L.oQ = take(nx * nx);
  L.oR = take(nu * nu);
  L.oQf = take(nx * nx);
  L.oH = take(L.SH);
  L.of = take(L.n);
  L.oGam = take((size_t)L.m * L.n);
  L.oXbar = take(L.m);
  L.oHl = take(L.m);
  L.oHu = take(L.m);
  L.oLb = take(L.n);
  L.oUb = take(L.n);
  L.oZ = take(L.n);
  L.oY = take(L.m);
  L.oSt = o;
  o += al256((size_t)L.cap * sizeof(int32_t));
  L.total = o;
  return L;
}

__device__ __forceinline__ int fb_count(const int* count, int cap) {
  const int c = *count;
  return c < cap ? c : cap;
}

__global__ __launch_bounds__(256) void fb64_gather_kernel(Fallback64In in, Fb64Layout L, char* w,
                                                          const int* list, const int* count) {
  const int cnt = fb_count(count, L.cap);
  const int nx = in.nx, nu = in.nu;
  double* A = (double*)(w + L.oA);
  double* B = (double*)(w + L.oB);
  double* C = (double*)(w + L.oC);
  double* X0 = (double*)(w + L.oX0);
  double* Q = (double*)(w + L.oQ);
  double* R = (double*)(w + L.oR);
  double* Qf = (double*)(w + L.oQf);
  double* lb = (double*)(w + L.oLb);
  double* ub = (double*)(w + L.oUb);
  const double inf = Lim<double>::inf();
  for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
    const int64_t b = list[t];
    for (int i = threadIdx.x; i < L.SA; i += blockDim.x)
      A[(int64_t)t * L.SA + i] = in.A[b * in.sA + i];
    for (int i = threadIdx.x; i < L.SB; i += blockDim.x)
      B[(int64_t)t * L.SB + i] = in.B[b * in.sB + i];
    if (in.c)
      for (int i = threadIdx.x; i < L.SC; i += blockDim.x)
        C[(int64_t)t * L.SC + i] = in.c[b * in.sC + i];
    for (int i = threadIdx.x; i < nx; i += blockDim.x) X0[(int64_t)t * nx + i] = in.x0[b * in.sX0 + i];
    for (int i = threadIdx.x; i < nx * nx; i += blockDim.x) {
      Q[(int64_t)t * nx * nx + i] = in.Q[b * in.sQ + i];
      Qf[(int64_t)t * nx * nx + i] = in.Qf[b * in.sQf + i];
    }
    for (int i = threadIdx.x; i < nu * nu; i += blockDim.x)
      R[(int64_t)t * nu * nu + i] = in.R[b * in.sR + i];
    for (int i = threadIdx.x; i < L.n; i += blockDim.x) {
      lb[(int64_t)t * L.n + i] = in.lb ? (double)in.lb[b * in.sLb + i] : -inf;
      ub[(int64_t)t * L.n + i] = in.ub ? (double)in.ub[b * in.sUb + i] : inf;
    }
  }
}

// row bounds of the condensed state box: xlo - xbar <= Gamma z <= xhi - xbar
__global__ __launch_bounds__(256) void fb64_rows_kernel(Fallback64In in, Fb64Layout L, char* w,
                                                        const int* list, const int* count) {
  const int cnt = fb_count(count, L.cap);
  const double* xbar = (const double*)(w + L.oXbar);
  double* hl = (double*)(w + L.oHl);
  double* hu = (double*)(w + L.oHu);
  const double inf = Lim<double>::inf();
  for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
    const int64_t b = list[t];
    for (int i = threadIdx.x; i < L.m; i += blockDim.x) {
      const double xb = xbar[(int64_t)t * L.m + i];
      hl[(int64_t)t * L.m + i] = in.xlo ? (double)in.xlo[b * in.sXb + i] - xb : -inf;
      hu[(int64_t)t * L.m + i] = in.xhi ? (double)in.xhi[b * in.sXb + i] - xb : inf;
    }
  }
}

__global__ __launch_bounds__(256) void fb64_scatter_kernel(Fb64Layout L, const char* w,
                                                           const int* list, const int* count,
                                                           float* z, float* y, int32_t* status) {
  const int cnt = fb_count(count, L.cap);
  const double* Z = (const double*)(w + L.oZ);
  const double* Y = (const double*)(w + L.oY);
  const int32_t* S = (const int32_t*)(w + L.oSt);
  for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
    const int64_t b = list[t];
    for (int i = threadIdx.x; i < L.n; i += blockDim.x) z[b * L.n + i] = (float)Z[(int64_t)t * L.n + i];
    if (y)
      for (int i = threadIdx.x; i < L.m; i += blockDim.x)
        y[b * L.m + i] = (float)Y[(int64_t)t * L.m + i];
    if (threadIdx.x == 0) {
      const int32_t s = S[t];
      status[b] = (s & 0xFF) == MPCQP_STATUS_OPTIMAL ? (s | MPCQP_STATUS_POLISHED) : s;
    }
  }
}

}  // namespace

// slots of the fp64 hand-off: about 3 % of the batch (config 3 hands off
// ~1 %), at least 64 (or the batch), at most 4096.  MPCQP_FALLBACK64_CAP
// (tests) lowers it, so that the list's remainder takes the interior point.
// Which entries get the slots follows the list order (atomic appends): with
// more hand-offs than slots, the solver an instance gets varies from run to
// run, and so does its result at the level of the two fp64 solvers' rounding
// (both return the exact active-set vertex)
int fallback64_cap(int batch) {
  int c = batch / 32;
  if (c < 64) c = 64;
  if (c > 4096) c = 4096;
  if (const char* e = getenv("MPCQP_FALLBACK64_CAP")) {
    const int k = atoi(e);
    if (k >= 1 && k < c) c = k;
  }
  return c < batch ? c : batch;
}

size_t fallback64_bytes(int batch, int nx, int nu, int N, int sbox) {
  if (batch <= 0) return 0;
  return fb64_layout(batch, nx, nu, N, 1, sbox).total;
}

int fallback64(const Fallback64In& in, const int* list, const int* count, float* z, float* y,
               int32_t* status, void* ws, size_t ws_bytes, hipStream_t st) {
  const int sbox = (in.xlo || in.xhi) ? 1 : 0;
  const Fb64Layout L = fb64_layout(in.batch, in.nx, in.nu, in.N, in.tv, sbox);
  MPCQP_CHECK_ARG(ws && ws_bytes >= L.total, "mpcqp_mpc_qp: fp64 hand-off workspace %zu < %zu",
                  ws_bytes, L.total);
  char* w = (char*)ws;
  const unsigned grid = (unsigned)(L.cap < 1024 ? L.cap : 1024);
  hipLaunchKernelGGL(fb64_gather_kernel, dim3(grid), dim3(256), 0, st, in, L, w, list, count);
  MPCQP_CHECK_LAUNCH("fb64_gather_kernel");
  double* d = nullptr;
  auto P = [&](size_t o) { return (double*)(w + o); };
  int rc = condense_f64_count(L.cap, in.nx, in.nu, in.N, in.tv ? MPCQP_TV : 0, P(L.oA), L.SA,
                              P(L.oB), L.SB, P(L.oQ), in.nx * in.nx, P(L.oR), in.nu * in.nu,
                              P(L.oQf), in.nx * in.nx, in.c ? P(L.oC) : d, L.SC, P(L.oX0), in.nx,
                              P(L.oH), P(L.of), L.m ? P(L.oGam) : d, L.m ? P(L.oXbar) : d, count,
                              st);
  if (rc != MPCQP_OK) return rc;
  if (L.m) {
    hipLaunchKernelGGL(fb64_rows_kernel, dim3(grid), dim3(256), 0, st, in, L, w, list, count);
    MPCQP_CHECK_LAUNCH("fb64_rows_kernel");
  }
  rc = solve_qp_f64_count(L.cap, L.n, L.m, P(L.oH), L.SH, P(L.of), L.n, L.m ? P(L.oGam) : d,
                          (int64_t)L.m * L.n, L.m ? P(L.oHl) : d, L.m ? P(L.oHu) : d, L.m,
                          P(L.oLb), L.n, P(L.oUb), L.n, P(L.oZ), L.m ? P(L.oY) : d,
                          (int32_t*)(w + L.oSt), count, st);
  if (rc != MPCQP_OK) return rc;
  hipLaunchKernelGGL(fb64_scatter_kernel, dim3(grid), dim3(256), 0, st, L, w, list, count, z, y,
                     status);
  MPCQP_CHECK_LAUNCH("fb64_scatter_kernel");
  return MPCQP_OK;
}

}  // namespace mpcqp
