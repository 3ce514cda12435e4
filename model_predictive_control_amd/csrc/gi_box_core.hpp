// gi_box_core.hpp -- the wavefront Goldfarb-Idnani dual active set for
//     min 1/2 z'Hz + f'z   s.t.  lb <= z <= ub
// shared by the stand-alone box solver (solve_box.hip) and the fused
// condense+solve kernel (mpc_box.hip).
//
// Entry state: M holds SWEEP_all(H) = -H^{-1} (all variables free), the LDS
// vectors fs/lbs/ubs hold f, lb, ub by row index (padding rows: f = 0,
// bounds = -/+inf).  On exit zr holds the solution in the row-block layout
// and the status code is returned.
//
// One iteration of the method (bound p, the most violated free variable):
//   direction  dz_F = M_{F,p} / M_pp  per unit move of z_p          (column p)
//   multiplier rates of active bounds  dmu_A = -/+ M_{A,p} / M_pp
//   partial step (a multiplier hits 0): drop that bound  -> sweep(k, +1)
//   full step (z_p reaches its bound):  add bound p       -> sweep(p, -1)
// with the primal/dual state tracked along the steps and one exact mat-vec
// refresh + re-check at the end (see gi_box in quad.hpp).
#pragma once
#include "quad.hpp"

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
  static constexpr int oEnd = oUb + NMAX;  // kernels append their own staging
};


// The wavefront kernels run the same Goldfarb-Idnani core as the four-QPs-
// per-wave kernels (gi_box in quad.hpp), on the 8 x 8 block layout.
template <typename T, int BS>
__device__ __forceinline__ int gi_box_core(Sym2D<T, BS>& M, T* buf, const T* fs, const T* lbs,
                                           const T* ubs, int n, int max_iter, T tol,
                                           T (&zr)[BS], int& iters) {
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  return gi_box<T, BS>(M, buf, fs, lbs, ubs, n, max_iter, tol, true, zr, iters MPCQP_CLK_ARG);
}

}  // namespace mpcqp
