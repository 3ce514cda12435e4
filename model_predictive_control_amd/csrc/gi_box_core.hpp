// gi_box_core.hpp -- the wavefront Goldfarb-Idnani dual active set for
//     min 1/2 z'Hz + f'z   s.t.  lb <= z <= ub
// shared by the stand-alone box solver (solve_box.hip) and the fused
// condense+solve kernel (mpc_box.hip).
//
// Entry state: M holds SWEEP_all(H) = -H^{-1} (all variables free), the LDS
// vectors fs/lbs/ubs hold f, lb, ub by row index (padding rows: f = 0,
// bounds = -/+inf), zs is scratch.  On exit zr holds the solution in the
// row-block layout and the status code is returned.
//
// One iteration of the method (bound p, the most violated free variable):
//   direction  dz_F = M_{F,p} / M_pp  per unit move of z_p          (column p)
//   multiplier rates of active bounds  dmu_A = -/+ M_{A,p} / M_pp
//   partial step (a multiplier hits 0): drop that bound  -> sweep(k, +1)
//   full step (z_p reaches its bound):  add bound p       -> sweep(p, -1)
// and after every full step the exact subspace minimiser / active gradient is
// recomputed by one mat-vec  s = M w,  w = (f_F, -z_A).
#pragma once
#include "sym2d.hpp"

namespace mpcqp {

// Occupancy target: 4 waves/SIMD (16 per CU) up to BS = 3 (n <= 24), which
// keeps a 4096-instance batch resident in one pass over the 256 CUs.
template <int BS>
struct BoxOcc {
  static constexpr int w = BS <= 3 ? 4 : (BS <= 5 ? 2 : 1);
};

// LDS layout shared by the box kernels (T elements)
template <typename T, int BS>
struct BoxLds {
  static constexpr int NMAX = 8 * BS;
  static constexpr int oBuf = 0;
  static constexpr int oF = Sym2D<T, BS>::BUF;
  static constexpr int oLb = oF + NMAX;
  static constexpr int oUb = oLb + NMAX;
  static constexpr int oZ = oUb + NMAX;
  static constexpr int oEnd = oZ + NMAX;  // kernels append their own staging
};


// st: 0 free, 1 at lower, 2 at upper, 3 padding row (never free)
template <typename T, int BS>
__device__ __forceinline__ int gi_box_core(Sym2D<T, BS>& M, T* buf, const T* fs, const T* lbs,
                                           const T* ubs, T* zs, int n, int max_iter, T tol,
                                           T (&zr)[BS], int& iters) {
  T gr[BS];
  int st[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    st[r] = (M.bi * BS + r < n) ? 0 : 3;
    zr[r] = T(0);
    gr[r] = T(0);
  }
  iters = 0;
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
        const T vl = finite(li) ? (li - zr[r]) * fast_rcp(T(1) + fabs(li)) : -Lim<T>::inf();
        const T vu = finite(ui) ? (zr[r] - ui) * fast_rcp(T(1) + fabs(ui)) : -Lim<T>::inf();
        const T v = fmax(vl, vu);
        if (v > viol) {
          viol = v;
          p = i;
        }
      }
    }
    blocks_argmax(viol, p);
    p = uniform(p);
    if (!(readlane(viol, 0) > tol)) break;
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
      if (++iters > max_iter) return MPCQP_STATUS_MAXITER;
      T c[BS], cc[BS];
      const T mpp = M.column(p, buf, c, cc);  // c[r] = M_ip; M_pp < 0 (p free)
      const T rm = fast_rcp(mpp);
      const T sgn = (tgt > zp) ? T(1) : T(-1);
      const T t2 = fabs(tgt - zp);
      T ti = Lim<T>::inf();
      int k = 0;
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        c[r] *= rm;  // dz per unit step of z_p
        const T dmu = ((st[r] == 1) ? -c[r] : ((st[r] == 2) ? c[r] : T(0))) * sgn;
        const T t = ((st[r] == 1 || st[r] == 2) && dmu < T(0)) ? -mu[r] * fast_rcp(dmu) : Lim<T>::inf();
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
        if (!(d > T(0))) return MPCQP_STATUS_NOT_CONVEX;
        zp = fma(sgn, ti, zp);  // row p moves by sgn*ti*(M_pp/M_pp)
      } else {
        // full step: bound p becomes active
#pragma unroll
        for (int r = 0; r < BS; ++r)
          if (M.bi * BS + r == p) st[r] = side;
        const T d = M.sweep(p, T(-1), buf);
        if (!(d < T(0))) return MPCQP_STATUS_NOT_CONVEX;
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
  return MPCQP_STATUS_OPTIMAL;
}

}  // namespace mpcqp
