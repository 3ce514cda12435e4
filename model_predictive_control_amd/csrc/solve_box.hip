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
#include "sym2d.hpp"

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

// st: 0 free, 1 at lower, 2 at upper, 3 padding row (never free)
// Occupancy target: 4 waves/SIMD (16 per CU) up to BS = 3 (n <= 24), which
// keeps a 4096-instance batch resident in one pass over the 256 CUs.
template <int BS>
struct BoxOcc {
  static constexpr int w = BS <= 3 ? 4 : (BS <= 5 ? 2 : 1);
};

template <typename T, int BS>
__global__ __launch_bounds__(64, BoxOcc<BS>::w) void box_gi_kernel(BoxArgs<T> a) {
  using S2 = Sym2D<T, BS>;
  constexpr int NMAX = S2::NMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = reinterpret_cast<T*>(smem_raw);  // Sym2D scratch
  T* fs = buf + S2::BUF;                    // per-row data by row index
  T* lbs = fs + NMAX;
  T* ubs = lbs + NMAX;
  T* zs = ubs + NMAX;
  T* Ps = zs + NMAX;                        // packed H
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
  T zr[BS], gr[BS];
  int st[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    st[r] = (M.bi * BS + r < n) ? 0 : 3;
    zr[r] = T(0);
    gr[r] = T(0);
  }

  int code = MPCQP_STATUS_MAXITER;
  int iters = 0;
  const T tol = a.tol;
  const int max_iter = a.max_iter;

  if (__any(nonfinite)) {
    code = MPCQP_STATUS_NONFINITE;
    goto done;
  }
  if (__any(badbox)) {
    code = MPCQP_STATUS_INFEASIBLE;
    goto done;
  }

  // ---- M = SWEEP_all(H) = -H^{-1}
  for (int k = 0; k < n; ++k) {
    const T d = M.sweep(k, T(1), buf);
    if (!(d > T(0))) {
      code = MPCQP_STATUS_NOT_CONVEX;
      goto done;
    }
  }

  {
    // subspace minimiser for (F, A): with w = (f_F, -z_A), s = M w gives
    // z_F = s_F and the active-set gradient g_A = f_A - s_A.
    auto refresh = [&]() {
      T w[BS], s[BS];
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const int i = M.bi * BS + r;
        const T zA = (st[r] == 1) ? lbs[i] : ((st[r] == 2) ? ubs[i] : T(0));
        w[r] = (st[r] == 0) ? fs[i] : -zA;
        zr[r] = zA;
      }
      M.matvec(w, buf, s);
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const int i = M.bi * BS + r;
        gr[r] = (st[r] == 0) ? T(0) : fs[i] - s[r];
        zr[r] = (st[r] == 0) ? s[r] : zr[r];
      }
    };
    refresh();

    while (true) {
      // most violated free variable (relative to the bound's magnitude)
      T viol = -Lim<T>::inf();
      int p = 0;
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        if (st[r] == 0) {
          const int i = M.bi * BS + r;
          const T li = lbs[i], ui = ubs[i];
          const T vl = finite(li) ? (li - zr[r]) / (T(1) + fabs(li)) : -Lim<T>::inf();
          const T vu = finite(ui) ? (zr[r] - ui) / (T(1) + fabs(ui)) : -Lim<T>::inf();
          const T v = fmax(vl, vu);
          if (v > viol) {
            viol = v;
            p = i;
          }
        }
      }
      blocks_argmax(viol, p);
      p = uniform(p);
      if (!(readlane(viol, 0) > tol)) {
        code = MPCQP_STATUS_OPTIMAL;
        break;
      }
      publish<T, BS>(zr, zs, M.bi, M.bj);
      __syncthreads();
      const T lbp = lbs[p], ubp = ubs[p];
      T zp = zs[p];
      __syncthreads();
      const int side = (zp < lbp) ? 1 : 2;
      const T tgt = (side == 1) ? lbp : ubp;
      T mu[BS];
#pragma unroll
      for (int r = 0; r < BS; ++r) mu[r] = (st[r] == 1) ? gr[r] : ((st[r] == 2) ? -gr[r] : T(0));
      bool added = false;
      while (!added) {
        if (++iters > max_iter) goto done;
        T c[BS], cc[BS];
        const T mpp = M.column(p, buf, c, cc);  // c[r] = M_ip; M_pp < 0 (p free)
        const T rm = T(1) / mpp;
        const T sgn = (tgt > zp) ? T(1) : T(-1);
        const T t2 = fabs(tgt - zp);
        T ti = Lim<T>::inf();
        int k = 0;
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          c[r] *= rm;  // c/M_pp: dz_F per unit step
          const T dmu = ((st[r] == 1) ? -c[r] : ((st[r] == 2) ? c[r] : T(0))) * sgn;
          const T t = ((st[r] == 1 || st[r] == 2) && dmu < T(0)) ? mu[r] / (-dmu)
                                                                  : Lim<T>::inf();
          if (t < ti) {
            ti = t;
            k = M.bi * BS + r;
          }
        }
        blocks_argmin(ti, k);
        k = uniform(k);
        ti = readlane(ti, 0);
        if (ti < t2) {
          // partial step: the multiplier of bound k reaches zero -> drop k
#pragma unroll
          for (int r = 0; r < BS; ++r) {
            const T dmu = ((st[r] == 1) ? -c[r] : ((st[r] == 2) ? c[r] : T(0))) * sgn;
            if (st[r] == 0) zr[r] = fma(sgn * ti, c[r], zr[r]);
            mu[r] = fma(ti, dmu, mu[r]);
            if (M.bi * BS + r == k) {
              mu[r] = T(0);
              st[r] = 0;
            }
          }
          const T d = M.sweep(k, T(1), buf);
          if (!(d > T(0))) {
            code = MPCQP_STATUS_NOT_CONVEX;
            goto done;
          }
          zp = fma(sgn, ti, zp);  // row p moves by sgn*ti*(M_pp/M_pp)
        } else {
          // full step: bound p becomes active
#pragma unroll
          for (int r = 0; r < BS; ++r) {
            if (M.bi * BS + r == p) st[r] = side;
          }
          const T d = M.sweep(p, T(-1), buf);
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
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      zr[r] = fmin(fmax(zr[r], lbs[i]), ubs[i]);
    }
  }

done:
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
  const size_t bytes = (size_t)(Sym2D<T, BS>::BUF + 4 * 8 * BS + a.n * (a.n + 1) / 2) * sizeof(T);
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
