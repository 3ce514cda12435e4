// wg.hpp -- one QP per workgroup of GR*GC threads: a symmetric n x n matrix
// (n <= GR*BR = GC*BC) held as a GR x GC grid of BR x BC register blocks, and the
// mixed primal/dual Goldfarb-Idnani active set that runs on it.
//
// Thread t owns block (bi, bj) with bi = t % GR and bj = t / GR, so the GR
// lanes of one (GR = 16) or two (GR = 32) DPP rows hold one block COLUMN.  Vectors
// indexed by matrix row ("row-block layout", T v[BR] for rows bi*BR..+BR-1)
// are replicated across bj, and every reduction over rows -- the arg-max of
// the violation scan, the ratio test -- is a row_ror butterfly inside a DPP
// row (plus one swizzle step for GR = 32).  Each of the 16 rows of the workgroup reduces identical data
// in the same total order, so every lane ends with the same scalar and the
// whole workgroup branches uniformly without a barrier.  Pivot columns travel
// through a double-buffered LDS vector (one barrier per column).
//
// Method.  The QP
//     min 1/2 z'Hz + f'z   s.t.  lz <= z <= uz,   lr <= C z <= ur
// is embedded in the augmented symmetric matrix K = [[H, C'], [C, 0]] over
// the index set {z_0..z_{n-1}, r_0..r_{m-1}}.  A swept set S holds the free
// z and the ACTIVE rows; M = SWEEP_S(K).  With w_q = c_q on S and -x_q off S
// (c = f on z, -bound on active rows; x = bound on fixed z, 0 = lambda on
// inactive rows), s = M w gives every primal/dual quantity:
//   free z: z = s;      fixed z: g = f - s;    active row: lambda = s;
//   inactive row: C_r z = -s.
// Adding constraint p (a violated bound of z_p or of row p) moves one scalar
// parameter tau in slot p (g_p for a z, lambda_p for a row); every quantity
// moves along column p of M.  A blocking multiplier is dropped by toggling
// its index (partial step); when p reaches its bound, p is toggled (full
// step).  Toggling = Goodnight sweep in (sigma = +1) or out (sigma = -1).
// A row (or z) that depends on the active set has M_pp ~ 0: the step is then
// a pure dual step that drops constraints until p becomes independent, or
// proves the QP infeasible.  Box-only problems (m = 0) reduce exactly to the
// box GI of gi_box_core.hpp.
#pragma once
#include "sym2d.hpp"

namespace mpcqp {

// (value, index[, payload]) reductions over the G lanes that hold one block
// column (G = 16: one DPP row; G = 32: two DPP rows, joined by a swizzle).
// NaN must be mapped to -inf / +inf by the caller (every lane must agree).
template <int G, typename T>
__device__ __forceinline__ void rowg_argmax(T& v, int& idx, T& pay) {
#define MPCQP_STEP(CTRL)                                         \
  {                                                              \
    const T ov = dpp<CTRL>(v);                                   \
    const int oi = dpp<CTRL>(idx);                               \
    const T op = dpp<CTRL>(pay);                                 \
    const bool take = (ov > v) || (ov == v && oi < idx);         \
    v = take ? ov : v;                                           \
    idx = take ? oi : idx;                                       \
    pay = take ? op : pay;                                       \
  }
  MPCQP_STEP(0x121)
  MPCQP_STEP(0x122)
  MPCQP_STEP(0x124)
  MPCQP_STEP(0x128)
#undef MPCQP_STEP
  if constexpr (G == 32) {
    const T ov = lane_step<16>(v);
    const int oi = lane_step<16>(idx);
    const T op = lane_step<16>(pay);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
    pay = take ? op : pay;
  }
}

template <int G, typename T>
__device__ __forceinline__ void rowg_argmin(T& v, int& idx) {
#define MPCQP_STEP(CTRL)                                         \
  {                                                              \
    const T ov = dpp<CTRL>(v);                                   \
    const int oi = dpp<CTRL>(idx);                               \
    const bool take = (ov < v) || (ov == v && oi < idx);         \
    v = take ? ov : v;                                           \
    idx = take ? oi : idx;                                       \
  }
  MPCQP_STEP(0x121)
  MPCQP_STEP(0x122)
  MPCQP_STEP(0x124)
  MPCQP_STEP(0x128)
#undef MPCQP_STEP
  if constexpr (G == 32) {
    const T ov = lane_step<16>(v);
    const int oi = lane_step<16>(idx);
    const bool take = (ov < v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
}

// Grid shape: GR x GC threads, BR x BC blocks, GR*BR == GC*BC.
template <int GR_, int BR_, int GC_, int BC_>
struct WShape {
  static constexpr int GR = GR_, BR = BR_, GC = GC_, BC = BC_;
  static constexpr int NMAX = GR * BR;
  static constexpr int threads = GR * GC;
  static_assert(GR * BR == GC * BC, "square matrix");
  static_assert(GR == 16 || GR == 32, "row reductions cover 16 or 32 lanes");
};

template <typename T, class S>
struct WSym {
  static constexpr int GR = S::GR, BR = S::BR, GC = S::GC, BC = S::BC;
  static constexpr int NMAX = S::NMAX;
  T m[BR][BC];
  int bi, bj;

  __device__ __forceinline__ void init(int tid) {
    bi = tid % GR;
    bj = tid / GR;
  }

  // Column kc / row kr (uniform) of this thread's block into an LDS vector.
  // Uniform compile-time switches that only READ registers; the asm marker
  // keeps the cases from being merged back into one dynamically indexed
  // access (which would live in scratch).
  template <int C>
  __device__ __forceinline__ void put_col_sel(int kc, T* buf) {
    if constexpr (C < BC) {
      if (kc == C) {
#pragma unroll
        for (int r = 0; r < BR; ++r) buf[bi * BR + r] = m[r][C];
        asm volatile("; col %0" ::"n"(C));
      } else {
        put_col_sel<C + 1>(kc, buf);
      }
    }
  }
  template <int R>
  __device__ __forceinline__ void put_row_sel(int kr, T* buf) {
    if constexpr (R < BR) {
      if (kr == R) {
#pragma unroll
        for (int c = 0; c < BC; ++c) buf[bj * BC + c] = m[R][c];
        asm volatile("; row %0" ::"n"(R));
      } else {
        put_row_sel<R + 1>(kr, buf);
      }
    }
  }
  // Publish column k into cbuf and row k into rbuf (the matrix is symmetric
  // up to rounding; the sweep needs both bit-exactly, see sweep_col).  k is
  // workgroup-uniform; readfirstlane keeps k and its block coordinates in
  // SGPRs so the case switches are scalar branches (otherwise the compiler
  // rewrites them through the lane-varying bi/bj into divergent searches).
  // The caller barriers before reading.
  __device__ __forceinline__ void put_col(int k, T* cbuf, T* rbuf) {
    k = uniform(k);
    const int kbc = k / BC, kbr = k / BR;
    const int kc = uniform(k - kbc * BC);  // convergent: not re-derived in the branch
    const int kr = uniform(k - kbr * BR);
    if (bj == kbc) put_col_sel<0>(kc, cbuf);
    if (bi == kbr) put_row_sel<0>(kr, rbuf);
  }
  // colr: column k at this thread's rows, colc: row k at its columns.
  __device__ __forceinline__ void get_col(const T* cbuf, const T* rbuf, T (&colr)[BR],
                                          T (&colc)[BC]) const {
#pragma unroll
    for (int r = 0; r < BR; ++r) colr[r] = cbuf[bi * BR + r];
#pragma unroll
    for (int c = 0; c < BC; ++c) colc[c] = rbuf[bj * BC + c];
  }

  // Goodnight sweep on pivot k (d = M_kk; colr = column k at this thread's
  // rows, colc = row k at its columns, both bit-exact register copies):
  //   M_ij -= M_ik M_kj / d;  row/col k := sigma M_.k / d;  M_kk := -1/d.
  // No branch writes matrix registers:
  //  * row k: with a_k = 1 exactly, the generic update leaves exactly
  //    m_kj - 1*m_kj = 0, and fma(ik, srow_j, .) installs the new row
  //    (ik in {0, 1}; elsewhere it adds an exact 0);
  //  * column k: selects, executed only by the wave that owns it.
  __device__ __forceinline__ void sweep_col(int k, T sigma, T d, const T (&colr)[BR],
                                            const T (&colc)[BC]) {
    k = uniform(k);
    const T rd = fast_rcp(d);
    const int kbc = k / BC, kbr = k / BR;
    const int kc = uniform(k - kbc * BC), kr = uniform(k - kbr * BR);
    T a[BR], ik[BR], srow[BC];
#pragma unroll
    for (int r = 0; r < BR; ++r) {
      const bool isk = (bi == kbr) && (r == kr);
      a[r] = isk ? T(1) : colr[r] * rd;
      ik[r] = isk ? T(1) : T(0);
    }
#pragma unroll
    for (int c = 0; c < BC; ++c) srow[c] = (bj * BC + c == k) ? -rd : sigma * colc[c] * rd;
#pragma unroll
    for (int r = 0; r < BR; ++r)
#pragma unroll
      for (int c = 0; c < BC; ++c) m[r][c] = fma(ik[r], srow[c], fma(-a[r], colc[c], m[r][c]));
    if (__any(bj == kbc)) {
      const bool own = bj == kbc;
#pragma unroll
      for (int r = 0; r < BR; ++r) {
        const T sc = (bi * BR + r == k) ? -rd : sigma * colr[r] * rd;
#pragma unroll
        for (int c = 0; c < BC; ++c) m[r][c] = (own && c == kc) ? sc : m[r][c];
      }
    }
  }

  // BK consecutive sweeps (pivots k0..k0+BK-1, sigma) from ONE publish of
  // their columns (cb[t*NMAX + i] = M[i][k0+t]) and rows (rb[t*NMAX + j] =
  // M[k0+t][j]).  Every thread replays the four sweeps on its block and on
  // local replicas of the fetched columns/rows and of the BK x BK pivot
  // block, with exactly the formulas of sweep_col, so every replica stays
  // bitwise equal to the register it mirrors; one barrier instead of BK.  Returns
  // false (uniformly) if a pivot fails the sign test (want > 0 when
  // positive, < 0 otherwise); the matrix is then left mid-block.
  template <int BK>
  __device__ __forceinline__ bool sweep_blk(int k0, T sigma, bool positive, const T* cb,
                                            const T* rb) {
    k0 = uniform(k0);
    T cr[BK][BR], cc[BK][BC], P[BK][BK];
#pragma unroll
    for (int t = 0; t < BK; ++t) {
#pragma unroll
      for (int r = 0; r < BR; ++r) cr[t][r] = cb[t * NMAX + bi * BR + r];
#pragma unroll
      for (int c = 0; c < BC; ++c) cc[t][c] = rb[t * NMAX + bj * BC + c];
#pragma unroll
      for (int q = 0; q < BK; ++q) P[q][t] = cb[t * NMAX + k0 + q];
    }
#pragma unroll
    for (int t = 0; t < BK; ++t) {
      const int k = k0 + t;
      const T d = P[t][t];
      if (positive ? !(d > T(0)) : !(d < T(0))) return false;
      const T rd = fast_rcp(d);
      const int kbc = k / BC, kbr = k / BR;
      const int kc = uniform(k - kbc * BC), kr = uniform(k - kbr * BR);
      // the register block (sweep_col)
      T a[BR], ik[BR], srow[BC];
#pragma unroll
      for (int r = 0; r < BR; ++r) {
        const bool isk = (bi == kbr) && (r == kr);
        a[r] = isk ? T(1) : cr[t][r] * rd;
        ik[r] = isk ? T(1) : T(0);
      }
#pragma unroll
      for (int c = 0; c < BC; ++c) srow[c] = (bj * BC + c == k) ? -rd : sigma * cc[t][c] * rd;
#pragma unroll
      for (int r = 0; r < BR; ++r)
#pragma unroll
        for (int c = 0; c < BC; ++c) m[r][c] = fma(ik[r], srow[c], fma(-a[r], cc[t][c], m[r][c]));
      if (__any(bj == kbc)) {
        const bool own = bj == kbc;
#pragma unroll
        for (int r = 0; r < BR; ++r) {
          const T sc = (bi * BR + r == k) ? -rd : sigma * cr[t][r] * rd;
#pragma unroll
          for (int c = 0; c < BC; ++c) m[r][c] = (own && c == kc) ? sc : m[r][c];
        }
      }
      // replicas of the later columns (my rows) and rows (my columns)
#pragma unroll
      for (int u = t + 1; u < BK; ++u) {
        const T pku = P[t][u], puk = P[u][t];  // M[k][k_u], M[k_u][k] before this sweep
#pragma unroll
        for (int r = 0; r < BR; ++r) {
          const bool isk = (bi == kbr) && (r == kr);
          cr[u][r] = isk ? sigma * pku * rd : fma(-(cr[t][r] * rd), pku, cr[u][r]);
        }
#pragma unroll
        for (int c = 0; c < BC; ++c) {
          const bool jk = bj * BC + c == k;
          cc[u][c] = jk ? sigma * puk * rd : fma(-(puk * rd), cc[t][c], cc[u][c]);
        }
      }
      // the pivot block, in place: entries off row/column t first (they read
      // row/column t), then row/column t; only the part later steps use
#pragma unroll
      for (int x = t + 1; x < BK; ++x)
#pragma unroll
        for (int y = t + 1; y < BK; ++y) P[x][y] = fma(-(P[x][t] * rd), P[t][y], P[x][y]);
    }
    return true;
  }

  // Same, reading column/row k from their LDS buffers (short live ranges).
  __device__ __forceinline__ void sweep_buf(int k, T sigma, T d, const T* cbuf, const T* rbuf) {
    T colr[BR], colc[BC];
    get_col(cbuf, rbuf, colr, colc);
    sweep_col(k, sigma, d, colr, colc);
  }

  // out[r] = sum_j M[bi*BR+r][j] w[j]; w in row-block layout.  wbuf: NMAX,
  // red: GC*NMAX.  Three barriers; every thread ends with its rows' sums.
  __device__ __forceinline__ void matvec(const T (&w)[BR], T* wbuf, T* red, T (&out)[BR]) {
    if (bj == 0) {
#pragma unroll
      for (int r = 0; r < BR; ++r) wbuf[bi * BR + r] = w[r];
    }
    __syncthreads();
    T wc[BC];
#pragma unroll
    for (int c = 0; c < BC; ++c) wc[c] = wbuf[bj * BC + c];
#pragma unroll
    for (int r = 0; r < BR; ++r) {
      T s = T(0);
#pragma unroll
      for (int c = 0; c < BC; ++c) s = fma(m[r][c], wc[c], s);
      red[bj * NMAX + bi * BR + r] = s;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < BR; ++r) {
      T s = T(0);
#pragma unroll 4
      for (int g = 0; g < GC; ++g) s += red[g * NMAX + bi * BR + r];
      out[r] = s;
    }
    __syncthreads();
  }

  // out[r] = sum_j K[bi*BR+r][j] x[j] in fp64 for an ORIGINAL matrix K given
  // element-wise by kel(i, j) (re-read from global memory), x in row-block
  // layout.  Used for the iterative-refinement residual.
  template <class KEl>
  __device__ __forceinline__ void matvec_orig(KEl&& kel, const T (&x)[BR], T* wbuf, double* redd,
                                              double (&out)[BR]) {
    if (bj == 0) {
#pragma unroll
      for (int r = 0; r < BR; ++r) wbuf[bi * BR + r] = x[r];
    }
    __syncthreads();
    T xc[BC];
#pragma unroll
    for (int c = 0; c < BC; ++c) xc[c] = wbuf[bj * BC + c];
#pragma unroll
    for (int r = 0; r < BR; ++r) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < BC; ++c) s = fma((double)kel(bi * BR + r, bj * BC + c), (double)xc[c], s);
      redd[bj * NMAX + bi * BR + r] = s;
      asm volatile("" ::: "memory");  // one row of loads in flight (register pressure)
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < BR; ++r) {
      double s = 0.0;
#pragma unroll 4
      for (int g = 0; g < GC; ++g) s += redd[g * NMAX + bi * BR + r];
      out[r] = s;
    }
    __syncthreads();
  }

  // |M_ii| for every i into out[i] (diagonal owners write).
  __device__ __forceinline__ void diag_abs(T* out) const {
#pragma unroll
    for (int r = 0; r < BR; ++r)
#pragma unroll
      for (int c = 0; c < BC; ++c)
        if (bi * BR + r == bj * BC + c) out[bi * BR + r] = fabs(m[r][c]);
  }
};

// LDS layout of the workgroup QP kernels (elements of T).
template <typename T, class S>
struct WLds {
  static constexpr int NMAX = S::NMAX;
  static constexpr int oCol0 = 0;
  static constexpr int oCol1 = oCol0 + NMAX;
  static constexpr int oRow0 = oCol1 + NMAX;
  static constexpr int oRow1 = oRow0 + NMAX;
  static constexpr int oBlk = oRow1 + NMAX;  // 2 x (4 columns + 4 rows) for sweep4
  static constexpr int oW = oBlk + 16 * NMAX;
  static constexpr int oLo = oW + NMAX;
  static constexpr int oHi = oLo + NMAX;
  static constexpr int oF = oHi + NMAX;
  static constexpr int oSl = oF + NMAX;     // 1/(1+|lo|), NaN for an infinite bound
  static constexpr int oSu = oSl + NMAX;    // 1/(1+|hi|)
  static constexpr int oScale = oSu + NMAX;
  static constexpr int oRed = oScale + NMAX;  // GC*NMAX doubles (8-byte aligned)
  static constexpr int total = oRed + S::GC * NMAX * (int)(sizeof(double) / sizeof(T));
};

// Mixed GI on M (entry: every z swept in, no row active).  nz = n, nt = n+m.
// lo/hi/f/scale live in LDS (f used for z indices only).  On exit val holds
// z (clamped to its box) / row values, lam the signed row multipliers
// (lambda > 0 at the upper bound) and the multipliers of fixed z (g).
// After convergence, `refine` steps of iterative refinement on the final
// active set S: e = (K x + c)_S from the ORIGINAL K (kel, fp64 accumulation),
// x_S -= K_SS^-1 e = x_S + M_SS e.  The swept matrix carries ~cond(H)*eps
// relative error (fp32: up to 1e-3); the residual from the original data
// brings z back to the accuracy of the data itself.
template <typename T, class S, class KEl>
__device__ __forceinline__ int gi_mixed(WSym<T, S>& M, T* sm, int nz, int nt, int max_iter,
                                        T tol, T dep_tol, T (&val)[S::BR], T (&lam)[S::BR],
                                        int& iters, KEl&& kel, int refine MPCQP_CLK_PARAM) {
  constexpr int BS = S::BR;  // row-block length
  using L = WLds<T, S>;
  T* lo = sm + L::oLo;
  T* hi = sm + L::oHi;
  T* fs = sm + L::oF;
  T* scale = sm + L::oScale;
  const T* sls = sm + L::oSl;
  const T* sus = sm + L::oSu;
  int st[BS];
  T mu[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    const int i = M.bi * BS + r;
    st[r] = (i < nt) ? 0 : 3;
    mu[r] = T(0);
    val[r] = T(0);
  }
  iters = 0;
  int code = MPCQP_STATUS_OPTIMAL;
  int cb = 0;  // column buffer parity

  // exact state from s = M w
  auto refresh = [&]() {
    T w[BS], s[BS];
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const bool isz = i < nz;
      const bool act = st[r] == 1 || st[r] == 2;
      const T bnd = (st[r] == 1) ? lo[i] : hi[i];
      const bool sw = isz ? (st[r] == 0) : act;
      const T fi = isz ? fs[i] : T(0);
      w[r] = (st[r] == 3) ? T(0) : (sw ? (isz ? fi : -bnd) : (isz ? -bnd : T(0)));
    }
    M.matvec(w, sm + L::oW, sm + L::oRed, s);
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const bool isz = i < nz;
      const bool act = st[r] == 1 || st[r] == 2;
      const T bnd = (st[r] == 1) ? lo[i] : hi[i];
      const T fi = isz ? fs[i] : T(0);
      const T mval = isz ? fi - s[r] : s[r];
      const T sside = ((st[r] == 1) ? T(1) : T(-1)) * (isz ? T(1) : T(-1));
      val[r] = act ? bnd : (isz ? s[r] : -s[r]);
      mu[r] = act ? sside * mval : T(0);
    }
  };

  auto scan = [&](T& viol, int& p, T& valp) {
    viol = -Lim<T>::inf();
    p = 0;
    valp = T(0);
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const T vl = (lo[i] - val[r]) * sls[i];  // NaN (never wins) for infinite bounds
      const T vu = (val[r] - hi[i]) * sus[i];
      T v = (st[r] == 0) ? fmax(vl, vu) : -Lim<T>::inf();
      v = (v == v) ? v : -Lim<T>::inf();
      const bool take = v > viol;
      viol = take ? v : viol;
      p = take ? i : p;
      valp = take ? val[r] : valp;
    }
    rowg_argmax<S::GR>(viol, p, valp);
  };

  refresh();
  bool active = true;
  for (int pass = 0; pass < 3 && active; ++pass) {
    while (true) {
      T viol, valp;
      int p;
      scan(viol, p, valp);
      p = uniform(p);
      viol = readlane(viol, 0);
      valp = readlane(valp, 0);
      if (!(viol > tol)) break;
      const T lop = lo[p], hip = hi[p];
      const int side = (valp < lop) ? 1 : 2;
      const T tgt = (side == 1) ? lop : hip;
      const bool pz = p < nz;
      const T epsp = pz ? T(-1) : T(1);
      const T sidesign = ((side == 1) ? T(1) : T(-1)) * (pz ? T(1) : T(-1));
      const T sgn = (tgt > valp) ? T(1) : T(-1);
      const T scp = scale[p];
      T tau = T(0);
      bool added = false;
      while (!added) {
        if (++iters > max_iter) {
          code = MPCQP_STATUS_MAXITER;
          goto out;
        }
        T* cbuf = sm + (cb ? L::oCol1 : L::oCol0);
        T* rbuf = sm + (cb ? L::oRow1 : L::oRow0);
        cb ^= 1;
        M.put_col(p, cbuf, rbuf);
        __syncthreads();
        const T* crb = cbuf + M.bi * BS;  // column p at this thread's rows
        const T mpp = cbuf[p];
        const bool dep = !(-mpp > dep_tol * scp);
        const T dtds = dep ? sidesign : sgn * epsp * fast_rcp(mpp);
        const T t2 = dep ? Lim<T>::inf() : fabs(tgt - valp);
        T ti = Lim<T>::inf();
        int k = 0;
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          const int i = M.bi * BS + r;
          const bool act = st[r] == 1 || st[r] == 2;
          const T dq = crb[r] * dtds;
          const T dmu = act ? ((st[r] == 1) ? dq : -dq) : T(0);
          T t = (act && dmu < T(0)) ? -mu[r] / dmu : Lim<T>::inf();
          t = (t == t) ? t : Lim<T>::inf();
          const bool take = t < ti;
          ti = take ? t : ti;
          k = take ? i : k;
        }
        rowg_argmin<S::GR>(ti, k);
        k = uniform(k);
        ti = readlane(ti, 0);
        if (!(ti < Lim<T>::inf()) && !(t2 < Lim<T>::inf())) {
          code = MPCQP_STATUS_INFEASIBLE;
          goto out;
        }
        const bool partial = ti < t2;
        const T s_eff = partial ? ti : t2;
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          const int i = M.bi * BS + r;
          const bool act = st[r] == 1 || st[r] == 2;
          const T dq = crb[r] * dtds;
          const T dmu = act ? ((st[r] == 1) ? dq : -dq) : T(0);
          const T dval = (st[r] == 0) ? ((i < nz) ? -dq : dq) : T(0);
          val[r] = fma(s_eff, dval, val[r]);
          mu[r] = fma(s_eff, dmu, mu[r]);
        }
        tau = fma(s_eff, dtds, tau);
        // the index whose state toggles: k leaves the active set (partial) or
        // p joins it (full); one sweep site keeps register pressure down
        int idx = p;
        T sigma = pz ? T(-1) : T(1);  // p inactive: swept if z, unswept if row
        T d = mpp;
        const T* sbuf = cbuf;
        const T* srbuf = rbuf;
        if (partial) {
          if (!dep) valp = fma(sgn, s_eff, valp);
          T* kbuf = sm + (cb ? L::oCol1 : L::oCol0);
          T* krbuf = sm + (cb ? L::oRow1 : L::oRow0);
          cb ^= 1;
          M.put_col(k, kbuf, krbuf);
          __syncthreads();
          idx = k;
          sigma = (k < nz) ? T(1) : T(-1);  // k active: unswept if z, swept if row
          d = kbuf[k];
          sbuf = kbuf;
          srbuf = krbuf;
        }
        if (partial ? !(d > T(0)) : !(d < T(0))) {
          code = MPCQP_STATUS_NOT_CONVEX;
          goto out;
        }
        M.sweep_buf(idx, sigma, d, sbuf, srbuf);
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          const bool me = M.bi * BS + r == idx;
          st[r] = me ? (partial ? 0 : side) : st[r];
          mu[r] = me ? (partial ? T(0) : sidesign * tau) : mu[r];
          val[r] = (me && !partial) ? tgt : val[r];
        }
        added = !partial;
      }
    }
    refresh();
    {
      T viol, valp;
      int p;
      scan(viol, p, valp);
      active = readlane(viol, 0) > tol;
    }
  }
  if (active) code = MPCQP_STATUS_MAXITER;
  MPCQP_PHASE(2);
  for (int it = 0; it < refine; ++it) {
    T x[BS];
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const bool isz = i < nz;
      const bool act = st[r] == 1 || st[r] == 2;
      const T sside = ((st[r] == 1) ? T(1) : T(-1)) * (isz ? T(1) : T(-1));
      x[r] = (st[r] == 3) ? T(0) : (isz ? val[r] : (act ? sside * mu[r] : T(0)));
    }
    double y[BS];
    M.matvec_orig(kel, x, sm + L::oW, reinterpret_cast<double*>(sm + L::oRed), y);
    T w[BS];
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const bool isz = i < nz;
      const bool act = st[r] == 1 || st[r] == 2;
      const double bnd = (st[r] == 1) ? (double)lo[i] : (double)hi[i];
      const bool inS = isz ? (st[r] == 0) : act;
      const double e = isz ? y[r] + (double)fs[i] : y[r] - bnd;
      w[r] = inS ? (T)e : T(0);
    }
    T sv[BS];
    M.matvec(w, sm + L::oW, sm + L::oRed, sv);
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const bool isz = i < nz;
      const bool act = st[r] == 1 || st[r] == 2;
      const T sside = ((st[r] == 1) ? T(1) : T(-1)) * (isz ? T(1) : T(-1));
      // free z: z += s;  active row: lambda += s  (mu = sside * lambda)
      val[r] = (isz && st[r] == 0) ? val[r] + sv[r] : val[r];
      mu[r] = (!isz && act) ? mu[r] + sside * sv[r] : mu[r];
    }
  }
out:
  MPCQP_PHASE(3);
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    const int i = M.bi * BS + r;
    const bool isz = i < nz;
    const T sside = ((st[r] == 1) ? T(1) : T(-1)) * (isz ? T(1) : T(-1));
    lam[r] = (st[r] == 1 || st[r] == 2) ? sside * mu[r] : T(0);
    if (isz && i < nt) val[r] = fmin(fmax(val[r], lo[i]), hi[i]);
  }
  return code;
}

}  // namespace mpcqp
