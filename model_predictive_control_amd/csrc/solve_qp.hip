// solve_qp.hip -- batched QPs with per-instance H and constraint rows, one
// instance per workgroup (wg.hpp):
//
//   min 1/2 z'Hz + f'z   s.t.  lb <= z <= ub,   hl <= G z <= hu
//
// This is the per-step QP of session_4/main.py:115-116 with BOTH the input box
// (lbx/ubx, main.py:68-69) and the state box (lbg/ubg, main.py:58-61) after
// condensing: G = Gamma (N*nx x N*nu), hl/hu = x_min/x_max - xbar per instance
// (BASELINE config 3), and the large input-box QPs of config 5 (n = 160,
// m = 0).  mpcqp_solve_box routes n > 64 here.
//
// Per instance: stage K = [[H, G'], [G, 0]] into registers, sweep every z
// index in (K -> [[-H^-1, H^-1 G'], [G H^-1, -G H^-1 G']], i.e. the dual
// matrix comes for free), then run the mixed primal/dual active set.
#include <cstdlib>

#include "wg.hpp"
#include "pf.hpp"
#include "quad_api.hpp"

namespace mpcqp {

int sweep_tiles(int dtype, int n, int m);
int sweep_launch(int batch, int n, int m, const void* H, int64_t sH, const void* G, int64_t sG,
                 void* M, int full, int32_t* status, hipStream_t st, const void* f, int64_t sf,
                 void* s0);
int hip_fail(hipError_t e, const char* where);

template <typename T>
struct QpArgs {
  int batch, n, m;
  const T* H; int64_t sH;  // packed lower n x n
  const T* f; int64_t sf;
  const T* G; int64_t sG;  // m x n row-major
  const T* hl; const T* hu; int64_t sh;
  const T* lb; int64_t sLb;
  const T* ub; int64_t sUb;
  T* z; T* y; int32_t* status;
  int max_iter;
  int refine;
  T tol;
  // pre-swept M (sweep.hip, full: dense (n+m) x (n+m) row-major per instance)
  // and its per-instance status in status[]; nullptr: sweep in the kernel
  const T* Ms;
  // retry mode (solve_pf.hip hand-off): solve only the instances listed
  const int* retry_count;
  const int* retry_list;
};

// Pivots per barrier in the initial sweep-in: the replicas cost BK*(BR+BC)
// registers, so large blocks (and fp64) use pairs.
template <typename T, class S>
struct QpBlock {
  static constexpr int e = S::BR * S::BC * (int)(sizeof(T) / 4);  // block VGPRs
  static constexpr int bk = e <= 32 ? 4 : (e <= 64 ? 2 : 1);
};

// Two waves per SIMD: a 512-thread workgroup fits once per CU, a 256-thread
// one twice (VGPR budget 256).
template <typename T, class S>
__device__ __forceinline__ void qp_wg_body(const QpArgs<T>& a, const int b) {
  using L = WLds<T, S>;
  constexpr int BR = S::BR, BC = S::BC;
  constexpr int NMAX = L::NMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  T* lo = sm + L::oLo;
  T* hi = sm + L::oHi;
  T* fs = sm + L::oF;
  const int tid = threadIdx.x;
  const int n = a.n, m = a.m, nt = n + m;
  const T inf = Lim<T>::inf();

#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  // status written by the pre-sweep (read before anyone writes it back)
  const int pre = (a.Ms && !a.retry_list) ? a.status[b] : 0;
  int bad = 0, nonfin = 0;
  for (int i = tid; i < NMAX; i += S::threads) {
    T l = -inf, u = inf, fi = T(0);
    if (i < n) {
      if (a.lb) l = a.lb[(int64_t)b * a.sLb + i];
      if (a.ub) u = a.ub[(int64_t)b * a.sUb + i];
      fi = a.f[(int64_t)b * a.sf + i];
      nonfin |= !finite(fi);
    } else if (i < nt) {
      if (a.hl) l = a.hl[(int64_t)b * a.sh + (i - n)];
      if (a.hu) u = a.hu[(int64_t)b * a.sh + (i - n)];
    }
    bad |= !(l <= u) || l == inf || u == -inf;
    lo[i] = l;
    hi[i] = u;
    fs[i] = fi;
    sm[L::oSl + i] = finite(l) ? T(1) / (T(1) + fabs(l)) : __builtin_nan("");
    sm[L::oSu + i] = finite(u) ? T(1) / (T(1) + fabs(u)) : __builtin_nan("");
  }
  WSym<T, S> M;
  M.init(tid);
  const T* Hb = a.H + (int64_t)b * a.sH;
  const T* Gb = a.G ? a.G + (int64_t)b * a.sG : nullptr;
  const T* Mb = a.Ms ? a.Ms + (int64_t)b * ((int64_t)nt * nt) : nullptr;
#pragma unroll
  for (int r = 0; r < BR; ++r)
#pragma unroll
    for (int c = 0; c < BC; ++c) {
      const int i = M.bi * BR + r, j = M.bj * BC + c;
      T v = T(0);
      if (Mb) {
        if (i < nt && j < nt) v = Mb[(int64_t)i * nt + j];
      } else if (i < n && j < n) {
        v = (j <= i) ? Hb[i * (i + 1) / 2 + j] : Hb[j * (j + 1) / 2 + i];
      } else if (i < nt && j < n) {
        v = Gb[(int64_t)(i - n) * n + j];
      } else if (j < nt && i < n) {
        v = Gb[(int64_t)(j - n) * n + i];
      }
      nonfin |= !finite(v);
      M.m[r][c] = v;
      if (c == BC - 1) asm volatile("" ::: "memory");  // one row of loads in flight
    }
  const int flags = __syncthreads_or((bad ? 1 : 0) | (nonfin ? 2 : 0));
  MPCQP_PHASE(0);
  int code = MPCQP_STATUS_OPTIMAL;
  int iters = 0;
  T val[BR], lam[BR];
#pragma unroll
  for (int r = 0; r < BR; ++r) {
    val[r] = __builtin_nan("");
    lam[r] = __builtin_nan("");
  }
  if (pre) {
    code = pre;
  } else if (flags & 2) {
    code = MPCQP_STATUS_NONFINITE;
  } else if (flags & 1) {
    code = MPCQP_STATUS_INFEASIBLE;
  } else {
    // sweep every z in: M = [[-H^-1, H^-1 G'], [G H^-1, -G H^-1 G']] --
    // BK pivots per publish/barrier (sweep_blk), the remainder one by one
    constexpr int BK = QpBlock<T, S>::bk;
    int k = Mb ? n : 0;  // pre-swept: every z is in already
    for (int blk = 0; BK > 1 && k + BK <= n; k += BK, ++blk) {
      T* cb = sm + L::oBlk + (blk & 1) * 8 * NMAX;
      T* rb = cb + 4 * NMAX;
#pragma unroll
      for (int t = 0; t < BK; ++t) M.put_col(k + t, cb + t * NMAX, rb + t * NMAX);
      __syncthreads();
      if (!M.template sweep_blk<BK>(k, T(1), true, cb, rb)) {
        code = MPCQP_STATUS_NOT_CONVEX;
        break;
      }
    }
    for (; code == MPCQP_STATUS_OPTIMAL && k < n; ++k) {
      T* cbuf = sm + ((k & 1) ? L::oCol1 : L::oCol0);
      T* rbuf = sm + ((k & 1) ? L::oRow1 : L::oRow0);
      M.put_col(k, cbuf, rbuf);
      __syncthreads();
      const T d = cbuf[k];
      if (!(d > T(0))) {
        code = MPCQP_STATUS_NOT_CONVEX;
        break;
      }
      M.sweep_buf(k, T(1), d, cbuf, rbuf);
    }
    MPCQP_PHASE(1);
    if (code == MPCQP_STATUS_OPTIMAL) {
      M.diag_abs(sm + L::oScale);
      __syncthreads();
      const T dep_tol = sizeof(T) == 8 ? T(1e-10) : T(2e-5);
      // original K_ij = [[H, G'], [G, 0]] for the refinement residual
      auto kel = [&](int i, int j) -> T {
        // opaque indices: stop the compiler from keeping the staging loads'
        // addresses alive across the whole solve (CSE with the K load above)
        asm volatile("" : "+v"(i), "+v"(j));
        if (i < n && j < n) return (j <= i) ? Hb[i * (i + 1) / 2 + j] : Hb[j * (j + 1) / 2 + i];
        if (i < nt && j < n) return Gb[(int64_t)(i - n) * n + j];
        if (j < nt && i < n) return Gb[(int64_t)(j - n) * n + i];
        return T(0);
      };
      code = gi_mixed<T, S>(M, sm, n, nt, a.max_iter, a.tol, dep_tol, val, lam, iters, kel,
                            a.refine MPCQP_CLK_ARG);
    }
  }
  const bool ok = code == MPCQP_STATUS_OPTIMAL || code == MPCQP_STATUS_MAXITER;
  if (M.bj == 0) {
#pragma unroll
    for (int r = 0; r < BR; ++r) {
      const int i = M.bi * BR + r;
      if (i < n) a.z[(int64_t)b * n + i] = ok ? val[r] : __builtin_nan("");
      if (a.y && i >= n && i < nt) a.y[(int64_t)b * m + (i - n)] = ok ? lam[r] : __builtin_nan("");
    }
  }
  if (tid == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

template <typename T, class S>
__global__ __launch_bounds__(S::threads) __attribute__((amdgpu_waves_per_eu(2)))
void qp_wg_kernel(QpArgs<T> a) {
  qp_wg_body<T, S>(a, blockIdx.x);
}

// hand-offs of solve_pf.hip: persistent workgroups walk the list
template <typename T, class S>
__global__ __launch_bounds__(S::threads) __attribute__((amdgpu_waves_per_eu(2)))
void qp_wg_retry_kernel(QpArgs<T> a) {
  const int cnt = *a.retry_count;
  for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
    qp_wg_body<T, S>(a, a.retry_list[t]);
    __syncthreads();
  }
}

// the first min(*retry_count, batch) instances, in place (the fp64 hand-off
// of mpcqp_mpc_qp: compact slots): persistent workgroups walk them
template <typename T, class S>
__global__ __launch_bounds__(S::threads) __attribute__((amdgpu_waves_per_eu(2)))
void qp_wg_count_kernel(QpArgs<T> a) {
  const int c = *a.retry_count;
  const int cnt = c < a.batch ? c : a.batch;
  for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
    qp_wg_body<T, S>(a, t);
    __syncthreads();
  }
}

template <typename T, class S>
static int launch_qp_bs(const QpArgs<T>& a, hipStream_t st) {
  const size_t bytes = (size_t)WLds<T, S>::total * sizeof(T);
  if (a.retry_count && !a.retry_list)  // count mode
    hipLaunchKernelGGL((qp_wg_count_kernel<T, S>), dim3(a.batch < 512 ? a.batch : 512),
                       dim3(S::threads), bytes, st, a);
  else if (a.retry_list)  // one persistent workgroup per CU walks the hand-off list
    hipLaunchKernelGGL((qp_wg_retry_kernel<T, S>), dim3(a.batch < 256 ? a.batch : 256),
                       dim3(S::threads), bytes, st, a);
  else
    hipLaunchKernelGGL((qp_wg_kernel<T, S>), dim3(a.batch), dim3(S::threads), bytes, st, a);
  MPCQP_CHECK_LAUNCH("qp_wg_kernel");
  return MPCQP_OK;
}

// Shapes: 256 threads (16 x 16 grid of 4 x 4 blocks) up to 64 indices, then
// 512 threads (32 x 16 grid of BR x 2BR blocks).
using Shape64 = WShape<16, 4, 16, 4>;
using Shape128 = WShape<32, 4, 16, 8>;
using Shape160 = WShape<32, 5, 16, 10>;
using Shape192 = WShape<32, 6, 16, 12>;

template <typename T>
int max_qp_size() {
  return 192;
}

template <typename T>
int launch_qp(const QpArgs<T>& a, hipStream_t st) {
  const int nt = a.n + a.m;
  if (nt <= 64) return launch_qp_bs<T, Shape64>(a, st);
  if (nt <= 128) return launch_qp_bs<T, Shape128>(a, st);
  if (nt <= 160) return launch_qp_bs<T, Shape160>(a, st);
  if (nt <= 192) return launch_qp_bs<T, Shape192>(a, st);
  set_error("qp_wg: n + m = %d exceeds %d", nt, max_qp_size<T>());
  return MPCQP_ENOTSUP;
}

template <typename T>
static int solve_qp_t(int batch, int n, int m, const void* H, int64_t sH, const void* f,
                      int64_t sf, const void* G, int64_t sG, const void* hl, const void* hu,
                      int64_t sh, const void* lb, int64_t sLb, const void* ub, int64_t sUb,
                      void* z, void* y, int32_t* status, int max_iter, double tol,
                      hipStream_t st, const void* Ms = nullptr,
                      const int* retry_count = nullptr, const int* retry_list = nullptr) {
  QpArgs<T> a;
  a.batch = batch; a.n = n; a.m = m;
  a.H = (const T*)H; a.sH = sH;
  a.f = (const T*)f; a.sf = sf;
  a.G = (const T*)G; a.sG = sG;
  a.hl = (const T*)hl; a.hu = (const T*)hu; a.sh = sh;
  a.lb = (const T*)lb; a.sLb = sLb;
  a.ub = (const T*)ub; a.sUb = sUb;
  a.z = (T*)z; a.y = (T*)y; a.status = status;
  a.max_iter = max_iter > 0 ? max_iter : 3 * (n + m) + 30;
  // fp32: two refinement steps against the original data; fp64: one
  a.refine = sizeof(T) == 4 ? 2 : 1;
  a.tol = tol > 0 ? (T)tol : (sizeof(T) == 8 ? (T)1e-12 : (T)1e-6);
  a.Ms = (const T*)Ms;
  a.retry_count = retry_count;
  a.retry_list = retry_list;
  return launch_qp<T>(a, st);
}

// fp64 solve of the first min(*count, batch) instances in place (fallback64.hip)
int solve_qp_f64_count(int batch, int n, int m, const double* H, int64_t sH, const double* f,
                       int64_t sf, const double* G, int64_t sG, const double* hl,
                       const double* hu, int64_t sh, const double* lb, int64_t sLb,
                       const double* ub, int64_t sUb, double* z, double* y, int32_t* status,
                       const int* count, hipStream_t st) {
  return solve_qp_t<double>(batch, n, m, H, sH, f, sf, G, sG, hl, hu, sh, lb, sLb, ub, sUb, z, y,
                            status, 0, 0.0, st, nullptr, count, nullptr);
}

// used by mpcqp_solve_box for n > 64
// (with Ms: the pre-swept -H^-1 of mpcqp_sweep, fp32 only)
int solve_box_wg(int dtype, int batch, int n, const void* H, int64_t sH, const void* f,
                 int64_t sf, const void* lb, int64_t sLb, const void* ub, int64_t sUb, void* z,
                 int32_t* status, int max_iter, double tol, hipStream_t st, const void* Ms) {
  if (dtype == MPCQP_F64)
    return solve_qp_t<double>(batch, n, 0, H, sH, f, sf, nullptr, 0, nullptr, nullptr, 0, lb,
                              sLb, ub, sUb, z, nullptr, status, max_iter, tol, st);
  return solve_qp_t<float>(batch, n, 0, H, sH, f, sf, nullptr, 0, nullptr, nullptr, 0, lb, sLb,
                           ub, sUb, z, nullptr, status, max_iter, tol, st, Ms);
}

// Workspace of the two-kernel path (MFMA pre-sweep -> product-form active
// set -> workgroup kernel for hand-offs): the dense swept matrix per
// instance, then the hand-off counter and list; 0 where that path does not
// apply (fp64, or n + m within the 256-thread kernel where the in-kernel
// sweep is cheap).
static size_t ws_m0_bytes(int batch, int n, int m) {
  const size_t nt = (size_t)(n + m);
  return ((size_t)batch * nt * nt * sizeof(float) + 255) / 256 * 256;
}

static size_t ws_s0_bytes(int batch, int n, int m) {
  return ((size_t)batch * (size_t)(n + m) * sizeof(float) + 255) / 256 * 256;
}

size_t qp_ws_bytes(int dtype, int batch, int n, int m) {
  if (batch <= 0 || n + m <= 64 || sweep_tiles(dtype, n, m) == 0) return 0;
  return ws_m0_bytes(batch, n, m) + ws_s0_bytes(batch, n, m) + 256 + (size_t)batch * sizeof(int);
}


// refinement steps of the product-form kernel (MPCQP_PF_REFINE overrides;
// a tuning knob, default 1: the fp64 residual against the original data
// brings z to the fp32 data floor in one step)
static int pf_refine() {
  const char* v = getenv("MPCQP_PF_REFINE");
  return v ? atoi(v) : 1;
}

// fp32, n + m > 64: sweep (MFMA) -> product-form active set, one instance per
// wavefront -> qp_wg_kernel for the instances with more than 64 active
// constraints (none at configs 3 and 5).
//
// With the dynamics refinement (mpcqp_mpc_qp), an instance handed off this
// way is solved on the fp32 condensed data without it: its status carries
// MPCQP_STATUS_UNREFINED so that the caller sees the fp32 condensing floor.
__global__ void flag_unrefined_kernel(const int* cnt, const int* list, int32_t* status) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < *cnt) {
    int32_t* s = status + list[j];
    *s = *s | MPCQP_STATUS_UNREFINED;
  }
}

QpWsParts qp_ws_parts(void* ws, int batch, int n, int m) {
  char* w = (char*)ws;
  QpWsParts p;
  p.m0 = w;
  p.m0_bytes = ws_m0_bytes(batch, n, m);
  p.s0 = w + p.m0_bytes;
  p.s0_bytes = ws_s0_bytes(batch, n, m);
  p.cnt = (int*)(w + p.m0_bytes + p.s0_bytes);
  p.list = p.cnt + 64;
  return p;
}

int solve_two_kernel(int batch, int n, int m, const void* H, int64_t sH, const void* f,
                     int64_t sf, const void* G, int64_t sG, const void* hl, const void* hu,
                     int64_t sh, const void* lb, int64_t sLb, const void* ub, int64_t sUb,
                     void* z, void* y, int32_t* status, int max_iter, double tol, void* ws,
                     hipStream_t st, const PfDyn* dyn, int refine, int wg_fallback) {
  const QpWsParts P = qp_ws_parts(ws, batch, n, m);
  float* M0 = (float*)P.m0;
  float* s0 = (float*)P.s0;
  int* cnt = P.cnt;
  int* list = P.list;
  hipError_t e = hipMemsetAsync(cnt, 0, sizeof(int), st);
  if (e != hipSuccess) return hip_fail(e, "mpcqp_solve_qp_ws: hipMemsetAsync");
  int rc = sweep_launch(batch, n, m, H, sH, G, sG, M0, 1, status, st, f, sf, s0);
  if (rc != MPCQP_OK) return rc;
  prof_mark(kProfSweep, st);
  const int mi = max_iter > 0 ? max_iter : 3 * (n + m) + 30;
  const float tl = tol > 0 ? (float)tol : 1e-6f;
  rc = launch_pf(batch, n, m, (const float*)H, sH, (const float*)f, sf, (const float*)G, sG,
                 (const float*)hl, (const float*)hu, sh, (const float*)lb, sLb, (const float*)ub,
                 sUb, M0, s0, (float*)z, (float*)y, status, cnt, list, mi,
                 refine >= 0 ? refine : pf_refine(), tl, st, dyn);
  if (rc != MPCQP_OK || !wg_fallback) return rc;
  rc = solve_qp_t<float>(batch, n, m, H, sH, f, sf, G, sG, hl, hu, sh, lb, sLb, ub, sUb, z, y,
                         status, max_iter, tol, st, M0, cnt, list);
  if (rc != MPCQP_OK || !dyn) return rc;
  hipLaunchKernelGGL(flag_unrefined_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0,
                     st, cnt, list, status);
  MPCQP_CHECK_LAUNCH("flag_unrefined_kernel");
  return MPCQP_OK;
}

int max_qp_size_dtype(int dtype) {
  return dtype == MPCQP_F64 ? max_qp_size<double>() : max_qp_size<float>();
}

}  // namespace mpcqp

extern "C" int mpcqp_max_qp_size(int dtype) { return mpcqp::max_qp_size_dtype(dtype); }

extern "C" int mpcqp_solve_qp(int dtype, int batch, int n, int m, const void* H, int64_t strideH,
                              const void* f, int64_t stridef, const void* G, int64_t strideG,
                              const void* hl, const void* hu, int64_t strideh, const void* lb,
                              int64_t strideLb, const void* ub, int64_t strideUb, void* z,
                              void* y, int32_t* status, int max_iter, double tol, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_solve_qp: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && n >= 1 && m >= 0, "mpcqp_solve_qp: bad sizes");
  MPCQP_CHECK_ARG(n + m <= max_qp_size_dtype(dtype), "mpcqp_solve_qp: n + m = %d exceeds %d",
                  n + m, max_qp_size_dtype(dtype));
  MPCQP_CHECK_ARG(H && f && z && status, "mpcqp_solve_qp: H, f, z, status are required");
  MPCQP_CHECK_ARG(m == 0 || G, "mpcqp_solve_qp: G required when m > 0");
  MPCQP_CHECK_ARG(strideH >= 0 && stridef >= 0 && strideG >= 0 && strideh >= 0 &&
                      strideLb >= 0 && strideUb >= 0,
                  "mpcqp_solve_qp: negative stride");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return solve_qp_t<double>(batch, n, m, H, strideH, f, stridef, G, strideG, hl, hu, strideh,
                              lb, strideLb, ub, strideUb, z, y, status, max_iter, tol, st);
  return solve_qp_t<float>(batch, n, m, H, strideH, f, stridef, G, strideG, hl, hu, strideh, lb,
                           strideLb, ub, strideUb, z, y, status, max_iter, tol, st);
}

extern "C" size_t mpcqp_solve_qp_workspace(int dtype, int batch, int n, int m) {
  return mpcqp::qp_ws_bytes(dtype, batch, n, m);
}

extern "C" int mpcqp_solve_qp_ws(int dtype, int batch, int n, int m, const void* H,
                                 int64_t strideH, const void* f, int64_t stridef, const void* G,
                                 int64_t strideG, const void* hl, const void* hu, int64_t strideh,
                                 const void* lb, int64_t strideLb, const void* ub,
                                 int64_t strideUb, void* z, void* y, int32_t* status,
                                 int max_iter, double tol, void* ws, size_t ws_bytes,
                                 void* stream) {
  using namespace mpcqp;
  const size_t need = qp_ws_bytes(dtype, batch, n, m);
  if (need == 0 || ws == nullptr)
    return mpcqp_solve_qp(dtype, batch, n, m, H, strideH, f, stridef, G, strideG, hl, hu, strideh,
                          lb, strideLb, ub, strideUb, z, y, status, max_iter, tol, stream);
  MPCQP_CHECK_ARG(ws_bytes >= need, "mpcqp_solve_qp_ws: workspace %zu bytes < %zu", ws_bytes, need);
  MPCQP_CHECK_ARG(n + m <= max_qp_size_dtype(dtype), "mpcqp_solve_qp_ws: n + m = %d exceeds %d",
                  n + m, max_qp_size_dtype(dtype));
  MPCQP_CHECK_ARG(H && f && z && status, "mpcqp_solve_qp_ws: H, f, z, status are required");
  MPCQP_CHECK_ARG(m == 0 || G, "mpcqp_solve_qp_ws: G required when m > 0");
  MPCQP_CHECK_ARG(strideH >= 0 && stridef >= 0 && strideG >= 0 && strideh >= 0 &&
                      strideLb >= 0 && strideUb >= 0,
                  "mpcqp_solve_qp_ws: negative stride");
  return solve_two_kernel(batch, n, m, H, strideH, f, stridef, G, strideG, hl, hu, strideh, lb,
                          strideLb, ub, strideUb, z, y, status, max_iter, tol, ws,
                          (hipStream_t)stream);
}

#ifdef MPCQP_PHASE_TIMING
MPCQP_DEBUG_PHASE_READER(mpcqp_debug_phase_cycles_qp)
#endif
