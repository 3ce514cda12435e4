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
// set F -- one row per lane in registers (lane i owns row i; n <= 64):
//     M_FF = -H_FF^{-1},  M_FA = H_FF^{-1} H_FA,  M_AA = Schur complement.
// Moving one index between F and the active set is one (reverse) sweep: a
// rank-1 update whose pivot row is broadcast with v_readlane (SGPR lane index,
// no LDS).  The step directions of the dual method are simply column p of M,
// and the subspace minimiser / active-set gradient is one mat-vec with M.
#include "common.hpp"

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

// st: 0 free, 1 at lower, 2 at upper, 3 padding lane (never free)
template <typename T, int NZ>
__device__ __forceinline__ T select_reg(const T (&m)[NZ], int k) {
  T r = T(0);
#pragma unroll
  for (int j = 0; j < NZ; ++j) r = (j == k) ? m[j] : r;
  return r;
}

// Goodnight sweep (sigma = +1: k joins F) / reverse sweep (sigma = -1: k
// leaves F) of the register-resident symmetric matrix, pivot k wave-uniform.
// Returns the pivot value (sign-checked by the caller).
template <typename T, int NZ>
__device__ __forceinline__ T sweep(T (&m)[NZ], int k, T sigma, int lane, int n) {
  const T mk = select_reg<T, NZ>(m, k);  // M_ik (own row, column k)
  const T d = readlane(mk, k);           // M_kk
  const T rd = T(1) / d;
  const T a = mk * rd;
  const T beta = (lane == k) ? (sigma * rd - T(1)) : -a;
#pragma unroll
  for (int j = 0; j < NZ; ++j) {
    if (j < n) m[j] = fma(beta, readlane(m[j], k), m[j]);
  }
  const T delta = (lane == k) ? (-rd - sigma) : sigma * a;
#pragma unroll
  for (int j = 0; j < NZ; ++j) m[j] = (j == k) ? m[j] + delta : m[j];
  return d;
}

template <typename T, int NZ>
__global__ __launch_bounds__(64) void box_gi_kernel(BoxArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Ps = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = a.n;
  const bool valid = lane < n;
  const int P = n * (n + 1) / 2;

  // ---- stage the packed lower triangle through LDS (coalesced HBM reads)
  {
    constexpr int MAXP = (NZ * (NZ + 1) / 2 + kWave - 1) / kWave;
    const T* Hb = a.H + (int64_t)b * a.sH;
    T tmp[MAXP];
#pragma unroll
    for (int t = 0; t < MAXP; ++t) {
      const int e = lane + t * kWave;
      tmp[t] = (e < P) ? Hb[e] : T(0);
    }
#pragma unroll
    for (int t = 0; t < MAXP; ++t) {
      const int e = lane + t * kWave;
      if (e < P) Ps[e] = tmp[t];
    }
  }
  T fi = T(0), lbi = -Lim<T>::inf(), ubi = Lim<T>::inf();
  if (valid) {
    fi = a.f[(int64_t)b * a.sf + lane];
    if (a.lb) lbi = a.lb[(int64_t)b * a.slb + lane];
    if (a.ub) ubi = a.ub[(int64_t)b * a.sub + lane];
  }
  __syncthreads();

  T m[NZ];
  bool nonfinite = valid && !finite(fi);
#pragma unroll
  for (int j = 0; j < NZ; ++j) {
    T v = T(0);
    if (valid && j < n) {
      const int idx = (j <= lane) ? lane * (lane + 1) / 2 + j : j * (j + 1) / 2 + lane;
      v = Ps[idx];
      nonfinite |= !finite(v);
    }
    m[j] = v;
  }
  const bool badbox = valid && (!(lbi <= ubi) || lbi == Lim<T>::inf() || ubi == -Lim<T>::inf());

  int code = MPCQP_STATUS_MAXITER;
  int iters = 0;
  T zi = T(0);
  int st = valid ? 0 : 3;
  const T tol = a.tol;

  if (__any(nonfinite)) {
    code = MPCQP_STATUS_NONFINITE;
    zi = __builtin_nan("");
    goto done;
  }
  if (__any(badbox)) {
    code = MPCQP_STATUS_INFEASIBLE;
    zi = __builtin_nan("");
    goto done;
  }

  // ---- M = SWEEP_all(H) = -H^{-1}
  for (int k = 0; k < n; ++k) {
    const T d = sweep<T, NZ>(m, k, T(1), lane, n);
    if (!(d > T(0))) {
      code = MPCQP_STATUS_NOT_CONVEX;
      zi = __builtin_nan("");
      goto done;
    }
  }

  {
    T gi = T(0);
    // subspace minimiser for the current (F, A): z_F = M_FF f_F - M_FA z_A,
    // g_A = f_A - M_AF f_F + M_AA z_A  ==  with w = (f_F, -z_A): s = M w.
    auto refresh = [&]() {
      const T zA = (st == 1) ? lbi : ((st == 2) ? ubi : T(0));
      const T w = (st == 0) ? fi : -zA;
      T s = T(0);
#pragma unroll
      for (int j = 0; j < NZ; ++j)
        if (j < n) s = fma(m[j], readlane(w, j), s);
      zi = (st == 0) ? s : zA;
      gi = (st == 0) ? T(0) : fi - s;
    };
    refresh();

    const int max_iter = a.max_iter;
    while (true) {
      // most violated free variable (relative to the bound's magnitude)
      T viol = -Lim<T>::inf();
      if (st == 0) {
        const T vl = (lbi - zi) / (T(1) + fabs(lbi));
        const T vu = (zi - ubi) / (T(1) + fabs(ubi));
        viol = fmax(vl, vu);
      }
      int p = lane;
      wave_argmax(viol, p);
      p = uniform(p);
      if (!(viol > tol)) {
        code = MPCQP_STATUS_OPTIMAL;
        break;
      }
      const T zp0 = readlane(zi, p);
      const T lbp = readlane(lbi, p), ubp = readlane(ubi, p);
      const int side = (zp0 < lbp) ? 1 : 2;
      const T tgt = (side == 1) ? lbp : ubp;
      T mu = (st == 1) ? gi : ((st == 2) ? -gi : T(0));
      bool added = false;
      while (!added) {
        if (++iters > max_iter) goto done;
        const T c = select_reg<T, NZ>(m, p);  // M_ip
        const T mpp = readlane(c, p);         // M_pp < 0 (p free)
        const T zp = readlane(zi, p);
        const T sgn = (tgt > zp) ? T(1) : T(-1);
        const T t2 = fabs(tgt - zp);
        const T cr = c / mpp;
        const T dmu = ((st == 1) ? -cr : ((st == 2) ? cr : T(0))) * sgn;
        T ti = ((st == 1 || st == 2) && dmu < T(0)) ? mu / (-dmu) : Lim<T>::inf();
        int k = lane;
        wave_argmin(ti, k);
        k = uniform(k);
        if (ti < t2) {
          // partial step: the multiplier of bound k reaches zero -> drop k
          if (st == 0) zi = fma(sgn * ti, cr, zi);
          mu = fma(ti, dmu, mu);
          if (lane == k) {
            mu = T(0);
            st = 0;
          }
          const T d = sweep<T, NZ>(m, k, T(1), lane, n);
          if (!(d > T(0))) {
            code = MPCQP_STATUS_NOT_CONVEX;
            goto done;
          }
        } else {
          // full step: bound p becomes active
          if (st == 0) zi = fma(sgn * t2, cr, zi);
          if (lane == p) {
            zi = tgt;
            st = side;
          }
          const T d = sweep<T, NZ>(m, p, T(-1), lane, n);
          if (!(d < T(0))) {
            code = MPCQP_STATUS_NOT_CONVEX;
            goto done;
          }
          refresh();
          added = true;
        }
      }
    }
    // project free variables that sit within tol outside their bounds
    zi = fmin(fmax(zi, lbi), ubi);
  }

done:
  if (valid) a.z[(int64_t)b * n + lane] = zi;
  if (lane == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
}

template <typename T, int NZ>
static int launch_box(const BoxArgs<T>& a, hipStream_t st) {
  const size_t bytes = (size_t)(a.n * (a.n + 1) / 2) * sizeof(T);
  hipLaunchKernelGGL((box_gi_kernel<T, NZ>), dim3(a.batch), dim3(kWave), bytes, st, a);
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
  if (n <= 8) return launch_box<T, 8>(a, st);
  if (n <= 16) return launch_box<T, 16>(a, st);
  if (n <= 24) return launch_box<T, 24>(a, st);
  if (n <= 32) return launch_box<T, 32>(a, st);
  if (n <= 48) return launch_box<T, 48>(a, st);
  return launch_box<T, 64>(a, st);
}

}  // namespace mpcqp

extern "C" int mpcqp_max_box_n(int dtype) {
  (void)dtype;
  return 64;
}

extern "C" int mpcqp_solve_box(int dtype, int batch, int n, const void* H, int64_t strideH,
                               const void* f, int64_t stridef, const void* lb, int64_t strideLb,
                               const void* ub, int64_t strideUb, void* z, int32_t* status,
                               int max_iter, double tol, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_solve_box: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_solve_box: batch < 0");
  MPCQP_CHECK_ARG(n >= 1 && n <= 64, "mpcqp_solve_box: n=%d outside [1,64]", n);
  MPCQP_CHECK_ARG(H && f && z && status, "mpcqp_solve_box: H, f, z, status are required");
  MPCQP_CHECK_ARG(strideH >= 0 && stridef >= 0 && strideLb >= 0 && strideUb >= 0,
                  "mpcqp_solve_box: negative stride");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return solve_box_t<double>(batch, n, H, strideH, f, stridef, lb, strideLb, ub, strideUb, z,
                               status, max_iter, tol, st);
  return solve_box_t<float>(batch, n, H, strideH, f, stridef, lb, strideLb, ub, strideUb, z,
                            status, max_iter, tol, st);
}
