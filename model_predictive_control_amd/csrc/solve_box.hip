// solve_box.hip -- batched box-constrained QP, one instance per wavefront.
//
//   min 1/2 z'Hz + f'z   s.t.  lb <= z <= ub,   H symmetric positive definite
//
// Replaces the per-step IPOPT call of session_4/main.py:115-116 for the
// input-box OCP (lbx/ubx of main.py:68-69,97-98; session4_sol.py:176-181).
//
// Algorithm: Goldfarb-Idnani dual active set specialised to bound constraints
// (start at the unconstrained minimiser, repeatedly add the most violated
// bound, dropping bounds whose multiplier would turn negative).  It terminates
// finitely and its iteration count is close to the number of active bounds,
// which keeps the wavefront-latency tail short (no cycling, unlike plain
// primal-dual active set on non-M-matrix MPC Hessians).
//
// Linear algebra: the wavefront keeps M = SWEEP_F(H) -- H swept on the free
// set F --  as an 8x8 grid of register blocks (sym2d.hpp):
//     M_FF = -H_FF^{-1},  M_FA = H_FF^{-1} H_FA,  M_AA = Schur complement.
// Moving one index between F and the active set is one (reverse) sweep, a
// rank-1 update whose pivot column is broadcast through LDS; the dual step
// directions are column p of M; the subspace minimiser and the active-set
// gradient are one mat-vec  s = M w,  w = (f_F, -z_A).
#include "gi_box_core.hpp"
#include "quad_api.hpp"

namespace mpcqp {

template <typename T>
struct BoxArgs {
  int batch, n;
  const T* H; int64_t sH;
  const T* f; int64_t sf;
  const T* lb; int64_t slb;
  const T* ub; int64_t sub;
  T* z;
  int32_t* status;
  int max_iter;
  T tol;
};

template <typename T, int BS>
__global__ __launch_bounds__(64, BoxOcc<BS>::w) void box_gi_kernel(BoxArgs<T> a) {
  using L = BoxLds<T, BS>;
  constexpr int NMAX = L::NMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  T* buf = sm + L::oBuf;
  T* fs = sm + L::oF;
  T* lbs = sm + L::oLb;
  T* ubs = sm + L::oUb;
  T* Ps = sm + L::oEnd;  // packed H
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = a.n;
  const int P = n * (n + 1) / 2;

  stage_packed<T, NMAX*(NMAX + 1) / 2>(a.H + (int64_t)b * a.sH, Ps, P, lane);
  bool nonfinite = false, badbox = false;
  if (lane < NMAX) {
    const int i = lane;
    const bool v = i < n;
    const T fi = v ? a.f[(int64_t)b * a.sf + i] : T(0);
    const T li = (v && a.lb) ? a.lb[(int64_t)b * a.slb + i] : -Lim<T>::inf();
    const T ui = (v && a.ub) ? a.ub[(int64_t)b * a.sub + i] : Lim<T>::inf();
    fs[i] = fi;
    lbs[i] = li;
    ubs[i] = ui;
    nonfinite = v && !finite(fi);
    badbox = v && (!(li <= ui) || li == Lim<T>::inf() || ui == -Lim<T>::inf());
  }
  __syncthreads();

  Sym2D<T, BS> M;
  M.init(lane);
  M.load_packed(Ps, n, nonfinite);
  T zr[BS];
  int iters = 0;
  int code;
  if (__any(nonfinite)) {
    code = MPCQP_STATUS_NONFINITE;
  } else if (__any(badbox)) {
    code = MPCQP_STATUS_INFEASIBLE;
  } else {
    code = MPCQP_STATUS_OPTIMAL;
    // ---- M = SWEEP_all(H) = -H^{-1}
    for (int k = 0; k < n; ++k) {
      const T d = M.sweep(k, T(1), buf);
      if (!(d > T(0))) {
        code = MPCQP_STATUS_NOT_CONVEX;
        break;
      }
    }
    if (code == MPCQP_STATUS_OPTIMAL)
      code = gi_box_core<T, BS>(M, buf, fs, lbs, ubs, n, a.max_iter, a.tol, zr, iters);
  }
  if (code != MPCQP_STATUS_OPTIMAL && code != MPCQP_STATUS_MAXITER) {
#pragma unroll
    for (int r = 0; r < BS; ++r) zr[r] = __builtin_nan("");
  }
  if (M.bj == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      if (i < n) a.z[(int64_t)b * n + i] = zr[r];
    }
  }
  if (lane == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
}

template <typename T, int BS>
static int launch_box(const BoxArgs<T>& a, hipStream_t st) {
  const size_t bytes = (size_t)(BoxLds<T, BS>::oEnd + a.n * (a.n + 1) / 2) * sizeof(T);
  hipLaunchKernelGGL((box_gi_kernel<T, BS>), dim3(a.batch), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("box_gi_kernel");
  return MPCQP_OK;
}

template <typename T>
static int solve_box_t(int batch, int n, const void* H, int64_t sH, const void* f, int64_t sf,
                       const void* lb, int64_t slb, const void* ub, int64_t sub, void* z,
                       int32_t* status, int max_iter, double tol, hipStream_t st) {
  BoxArgs<T> a;
  a.batch = batch; a.n = n;
  a.H = (const T*)H; a.sH = sH; a.f = (const T*)f; a.sf = sf;
  a.lb = (const T*)lb; a.slb = slb; a.ub = (const T*)ub; a.sub = sub;
  a.z = (T*)z; a.status = status;
  a.max_iter = max_iter > 0 ? max_iter : 3 * n + 30;
  a.tol = tol > 0 ? (T)tol : (sizeof(T) == 8 ? (T)1e-12 : (T)1e-6);
  if (n <= 32 && !use_wave_kernels()) {
    BoxArgsQ<T> q{batch, n, a.H, sH, a.f, sf, a.lb, slb, a.ub, sub, a.z, status, a.max_iter, a.tol};
    return solve_box_quad<T>(q, st);
  }
  switch ((n + 7) / 8) {
    case 1: return launch_box<T, 1>(a, st);
    case 2: return launch_box<T, 2>(a, st);
    case 3: return launch_box<T, 3>(a, st);
    case 4: return launch_box<T, 4>(a, st);
    case 5: return launch_box<T, 5>(a, st);
    case 6: return launch_box<T, 6>(a, st);
    case 7: return launch_box<T, 7>(a, st);
    default: return launch_box<T, 8>(a, st);
  }
}

}  // namespace mpcqp

extern "C" int mpcqp_max_box_n(int dtype) { return mpcqp::max_qp_size_dtype(dtype); }

extern "C" int mpcqp_solve_box(int dtype, int batch, int n, const void* H, int64_t strideH,
                               const void* f, int64_t stridef, const void* lb, int64_t strideLb,
                               const void* ub, int64_t strideUb, void* z, int32_t* status,
                               int max_iter, double tol, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_solve_box: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_solve_box: batch < 0");
  MPCQP_CHECK_ARG(n >= 1 && n <= max_qp_size_dtype(dtype), "mpcqp_solve_box: n=%d outside [1,%d]",
                  n, max_qp_size_dtype(dtype));
  MPCQP_CHECK_ARG(H && f && z && status, "mpcqp_solve_box: H, f, z, status are required");
  MPCQP_CHECK_ARG(strideH >= 0 && stridef >= 0 && strideLb >= 0 && strideUb >= 0,
                  "mpcqp_solve_box: negative stride");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (n > 64 || use_block_kernels())
    return solve_box_wg(dtype, batch, n, H, strideH, f, stridef, lb, strideLb, ub, strideUb, z,
                        status, max_iter, tol, st);
  if (dtype == MPCQP_F64)
    return solve_box_t<double>(batch, n, H, strideH, f, stridef, lb, strideLb, ub, strideUb, z,
                               status, max_iter, tol, st);
  return solve_box_t<float>(batch, n, H, strideH, f, stridef, lb, strideLb, ub, strideUb, z,
                            status, max_iter, tol, st);
}

extern "C" int mpcqp_solve_box_ws(int dtype, int batch, int n, const void* H, int64_t strideH,
                                  const void* f, int64_t stridef, const void* lb,
                                  int64_t strideLb, const void* ub, int64_t strideUb, void* z,
                                  int32_t* status, int max_iter, double tol, void* ws,
                                  size_t ws_bytes, void* stream) {
  using namespace mpcqp;
  const size_t need = qp_ws_bytes(dtype, batch, n, 0);
  if (need == 0 || ws == nullptr || n <= 64)
    return mpcqp_solve_box(dtype, batch, n, H, strideH, f, stridef, lb, strideLb, ub, strideUb, z,
                           status, max_iter, tol, stream);
  MPCQP_CHECK_ARG(ws_bytes >= need, "mpcqp_solve_box_ws: workspace %zu bytes < %zu", ws_bytes, need);
  MPCQP_CHECK_ARG(n <= max_qp_size_dtype(dtype), "mpcqp_solve_box_ws: n=%d outside [1,%d]", n,
                  max_qp_size_dtype(dtype));
  MPCQP_CHECK_ARG(H && f && z && status, "mpcqp_solve_box_ws: H, f, z, status are required");
  MPCQP_CHECK_ARG(strideH >= 0 && stridef >= 0 && strideLb >= 0 && strideUb >= 0,
                  "mpcqp_solve_box_ws: negative stride");
  return solve_two_kernel(batch, n, 0, H, strideH, f, stridef, nullptr, 0, nullptr, nullptr, 0, lb,
                          strideLb, ub, strideUb, z, nullptr, status, max_iter, tol, ws,
                          (hipStream_t)stream);
}
