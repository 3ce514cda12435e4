// quad.hpp -- four QPs per wavefront, one per 16-lane DPP row ("group").
//
// Lane l: group g = l >> 4, and inside the group q = l & 15, bi = q >> 2,
// bj = q & 3.  A symmetric n x n matrix (n <= 4*BS) of group g is held as a
// 4 x 4 grid of BS x BS register blocks over the group's 16 lanes.  All
// per-QP scalars (pivot index, step lengths, ...) are group-uniform VGPR
// values; every reduction stays inside a DPP row (quad_perm for the 4 lanes
// of a row block, row_ror:4/8 across row blocks), so four independent QPs
// share each instruction and no cross-row traffic (bpermute) is needed.
//
// Compared with one QP per wavefront (sym2d.hpp) the per-iteration bookkeeping
// -- reductions, LDS publishes, waits, scalar control -- is paid once for four
// problems, which is what bounds the solve at the config-2 sizes (the SIMDs
// are instruction-issue bound, see profiles/).
#pragma once
#include "sym2d.hpp"

#ifndef MPCQP_SCAN_AHEAD
#define MPCQP_SCAN_AHEAD 1
#endif

namespace mpcqp {

// Max over the 4 row blocks of a group (lanes differing in bits 2..3),
// carrying an index and one payload value; ties to the smaller index.
template <typename T>
__device__ __forceinline__ void group_argmax(T& v, int& idx, T& pay) {
  {
    const T ov = dpp<0x124>(v);  // row_ror:4
    const int oi = dpp<0x124>(idx);
    const T op = dpp<0x124>(pay);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
    pay = take ? op : pay;
  }
  {
    const T ov = dpp<0x128>(v);  // row_ror:8
    const int oi = dpp<0x128>(idx);
    const T op = dpp<0x128>(pay);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
    pay = take ? op : pay;
  }
}

template <typename T>
__device__ __forceinline__ void group_argmin(T& v, int& idx) {
  {
    const T ov = dpp<0x124>(v);
    const int oi = dpp<0x124>(idx);
    const bool take = (ov < v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
  {
    const T ov = dpp<0x128>(v);
    const int oi = dpp<0x128>(idx);
    const bool take = (ov < v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
}

// Sum over the 4 lanes of a row block (bits 0..1).
template <typename T>
__device__ __forceinline__ T quad_sum(T v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  return v;
}

template <typename T, int BS>
struct QSym {
  static constexpr int NMAX = 4 * BS;
  static constexpr int NV = NMAX;  // row-indexed vectors
  static constexpr int NC = BS;    // columns per lane
  static constexpr int RPL = BS;   // rows per lane
  static constexpr int CBUF = NMAX * BS;  // column-publish tile (per group)
  static constexpr int BUF = CBUF + NMAX;  // + mat-vec vector
  T m[BS][BS];
  int bi, bj;

  __device__ __forceinline__ void init(int lane) {
    const int q = lane & 15;
    bi = q >> 2;
    bj = q & 3;
  }

  // From a dense row-major n x n matrix (leading dim ld) in LDS, symmetrised.
  __device__ __forceinline__ void load_dense_sym(const T* D, int ld, int n) {
#pragma unroll
    for (int r = 0; r < BS; ++r)
#pragma unroll
      for (int c = 0; c < BS; ++c) {
        const int i = bi * BS + r, j = bj * BS + c;
        m[r][c] = (i < n && j < n) ? T(0.5) * (D[i * ld + j] + D[j * ld + i]) : T(0);
      }
  }

  __device__ __forceinline__ void load_packed(const T* Ps, int n, bool& nonfinite) {
#pragma unroll
    for (int r = 0; r < BS; ++r)
#pragma unroll
      for (int c = 0; c < BS; ++c) {
        const int i = bi * BS + r, j = bj * BS + c;
        T v = T(0);
        if (i < n && j < n) {
          const int idx = (j <= i) ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i;
          v = Ps[idx];
          nonfinite |= !finite(v);
        }
        m[r][c] = v;
      }
  }

  // Column k (group-uniform) through the group's LDS tile; returns M_kk.
  __device__ __forceinline__ T column(int k, T* gb, T (&colr)[BS], T (&colc)[BS]) {
    const int kb = k / BS, kc = k - kb * BS;
    if (bj == kb) {
#pragma unroll
      for (int r = 0; r < BS; ++r)
#pragma unroll
        for (int c = 0; c < BS; ++c) gb[(bi * BS + r) * BS + c] = m[r][c];
    }
    lds_exchange();
#pragma unroll
    for (int r = 0; r < BS; ++r) colr[r] = gb[(bi * BS + r) * BS + kc];
#pragma unroll
    for (int c = 0; c < BS; ++c) colc[c] = gb[(bj * BS + c) * BS + kc];
    const T d = gb[k * BS + kc];
    lds_exchange();
    return d;
  }

  // Goodnight sweep (sigma = +1) / reverse sweep (sigma = -1) on pivot k with
  // its column already fetched:  M_ij - M_ik M_kj / d  off row/column k,
  // sigma M_kj / d on row k, sigma M_ik / d on column k, -1/d at (k, k).
  // Row/column k are selected, not produced by cancellation (their relative
  // error would otherwise grow like eps * |d|).
  __device__ __forceinline__ void sweep_col(int k, T sigma, T d, const T (&colr)[BS],
                                            const T (&colc)[BS]) {
    const T rd = fast_rcp(d);
    T a[BS], scol[BS], srow[BS];
    bool ik[BS], jk[BS];
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      a[r] = colr[r] * rd;
      scol[r] = sigma * a[r];
      ik[r] = (bi * BS + r == k);
    }
#pragma unroll
    for (int c = 0; c < BS; ++c) {
      jk[c] = (bj * BS + c == k);
      srow[c] = jk[c] ? -rd : sigma * colc[c] * rd;
    }
#pragma unroll
    for (int r = 0; r < BS; ++r)
#pragma unroll
      for (int c = 0; c < BS; ++c) {
        const T gen = fma(-a[r], colc[c], m[r][c]);
        m[r][c] = ik[r] ? srow[c] : (jk[c] ? scol[r] : gen);
      }
  }

  __device__ __forceinline__ T sweep(int k, T sigma, T* gb) {
    T colr[BS], colc[BS];
    const T d = column(k, gb, colr, colc);
    sweep_col(k, sigma, d, colr, colc);
    return d;
  }

  // out[r] = sum_j M[i][j] w[j] (w in the group's row-block layout).
  __device__ __forceinline__ void matvec(const T (&w)[BS], T* gb, T (&out)[BS]) {
    T* wb = gb + CBUF;
    if (bj == 0) {
#pragma unroll
      for (int r = 0; r < BS; ++r) wb[bi * BS + r] = w[r];
    }
    lds_exchange();
    T wc[BS];
#pragma unroll
    for (int c = 0; c < BS; ++c) wc[c] = wb[bj * BS + c];
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      T s = T(0);
#pragma unroll
      for (int c = 0; c < BS; ++c) s = fma(m[r][c], wc[c], s);
      out[r] = quad_sum(s);
    }
    lds_exchange();
  }
};

// Per-group LDS block for the box active set: [Mat::BUF | f | lb | ub], the
// vectors indexed by (padded) row.
template <class Mat>
struct GBoxLds {
  static constexpr int NMAX = Mat::NMAX;
  static constexpr int NV = Mat::NV;
  static constexpr int oBuf = 0;
  static constexpr int oF = Mat::BUF;
  static constexpr int oLb = oF + NV;
  static constexpr int oUb = oLb + NV;
  static constexpr int size = oUb + NV;
};
template <typename T, int BS>
using QBoxLds = GBoxLds<QSym<T, BS>>;

// Relative-violation scale of a bound: 1/(1+|b|) for a finite bound, NaN for
// an infinite one (a NaN violation never wins the arg-max and fmax skips it),
// so the per-iteration scan multiplies instead of dividing.
template <typename T>
__device__ __forceinline__ T bound_scale(T bnd) {
  return finite(bnd) ? T(1) / (T(1) + fabs(bnd)) : __builtin_nan("");
}

// Goldfarb-Idnani dual active set for one box QP per group / wave (see gi_box_core.hpp
// for the method); entry: M = -H^{-1}.  Primal and dual quantities are tracked
// incrementally along the steps (z_F, the active multipliers, and the
// multiplier of the bound being added); when every group has settled, one
// exact mat-vec refresh recomputes z and the multipliers and the bounds are
// re-checked, so accumulated drift can never hide a violated bound.
// live = this group holds a real instance.  Returns the status code.
// Bounds of this lane's rows and their violation scales, held in registers
// for the whole solve (loop-invariant; the scan runs every iteration).
template <typename T, int BS>
struct QBounds {
  T lo[BS], hi[BS], sl[BS], su[BS];
  template <class Mat>
  __device__ __forceinline__ void load(const Mat& M, const T* lbs, const T* ubs) {
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      lo[r] = lbs[i];
      hi[r] = ubs[i];
      sl[r] = bound_scale(lo[r]);
      su[r] = bound_scale(hi[r]);
    }
  }
};

// Reductions over the rows of one QP, per layout: four QPs per wave (DPP
// rows of 16 lanes) or one QP per wave (8 row blocks).
template <typename T, int BS>
__device__ __forceinline__ void rows_argmax(const QSym<T, BS>&, T& v, int& idx, T& pay) {
  group_argmax(v, idx, pay);
}
template <typename T, int BS>
__device__ __forceinline__ void rows_argmin(const QSym<T, BS>&, T& v, int& idx) {
  group_argmin(v, idx);
}
template <typename T, int BS>
__device__ __forceinline__ void rows_argmax(const Sym2D<T, BS>&, T& v, int& idx, T& pay) {
  blocks_argmax(v, idx, pay);
}
template <typename T, int BS>
__device__ __forceinline__ void rows_argmin(const Sym2D<T, BS>&, T& v, int& idx) {
  blocks_argmin(v, idx);
}

template <typename T, int BS, class Mat>
__device__ __forceinline__ void qscan(const Mat& M, const int (&st)[BS], const T (&zr)[BS],
                                      const QBounds<T, BS>& B, T& viol, int& pi, T& zv) {
  viol = -Lim<T>::inf();
  pi = 0;
  zv = T(0);
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    const int i = M.bi * BS + r;
    const T vl = (B.lo[r] - zr[r]) * B.sl[r];  // NaN for an infinite bound
    const T vu = (zr[r] - B.hi[r]) * B.su[r];
    const T v = (st[r] == 0) ? fmax(vl, vu) : -Lim<T>::inf();
    const bool take = v > viol;
    viol = take ? v : viol;
    pi = take ? i : pi;
    zv = take ? zr[r] : zv;
  }
  rows_argmax(M, viol, pi, zv);
}


// WARM: st (this lane's rows: 0 free, 1 at lb, 2 at ub, 3 padding) is the
// starting active set and M the matrix swept on its free rows (H swept on F
// equals -H^-1 swept back on the active rows); the active rows whose
// multipliers have the wrong sign are released first (one sweep each), then
// the active set runs as from a cold start.  st is returned either way.
template <typename T, int BS, bool WARM, class Mat>
__device__ __forceinline__ int gi_box_st(Mat& M, T* gb, const T* fs, const T* lbs,
                                         const T* ubs, int n, int max_iter, T tol, bool live,
                                         T (&zr)[BS], int& iters, int (&st)[BS] MPCQP_CLK_PARAM) {
  QBounds<T, BS> B;
  B.load(M, lbs, ubs);
  T mu[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    if constexpr (!WARM) st[r] = (M.bi * BS + r < n) ? 0 : 3;
    mu[r] = T(0);
    zr[r] = T(0);
  }
  iters = 0;
  int code = MPCQP_STATUS_OPTIMAL;
  auto refresh = [&]() {
    T w[BS], s[BS];
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const T zA = (st[r] == 1) ? B.lo[r] : ((st[r] == 2) ? B.hi[r] : T(0));
      w[r] = (st[r] == 0) ? fs[i] : -zA;
      zr[r] = zA;
    }
    M.matvec(w, gb, s);
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const T g = fs[i] - s[r];
      zr[r] = (st[r] == 0) ? s[r] : zr[r];
      mu[r] = (st[r] == 1) ? g : ((st[r] == 2) ? -g : T(0));
    }
  };
  refresh();
  bool active = live;
  if constexpr (WARM) {
    // release wrong-signed multipliers, the most negative first
    bool drop = live;
    while (true) {
      T mv = Lim<T>::inf();
      int k = 0;
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const bool a = (st[r] == 1 || st[r] == 2) && mu[r] < -tol;
        const bool take = a && mu[r] < mv;
        mv = take ? mu[r] : mv;
        k = take ? (M.bi * BS + r) : k;
      }
      rows_argmin(M, mv, k);
      drop = drop && mv < Lim<T>::inf();
      if (!__any(drop)) break;
      if (drop && ++iters > max_iter) {
        code = MPCQP_STATUS_MAXITER;
        drop = false;
        active = false;
      }
      T kr[BS], kc[Mat::NC];
      const T d = M.column(k, gb, kr, kc);
      if (drop && !(d > T(0))) {
        code = MPCQP_STATUS_NOT_CONVEX;
        drop = false;
        active = false;
      }
      if (drop) {
        M.sweep_col(k, T(1), d, kr, kc);
#pragma unroll
        for (int r = 0; r < BS; ++r)
          if (M.bi * BS + r == k) st[r] = 0;
      }
      refresh();
    }
  }
  for (int pass = 0; pass < 3; ++pass) {
    bool need_p = true;
    int p = 0, side = 1;
    T tgt = T(0), zp = T(0), gp = T(0);
#if MPCQP_SCAN_AHEAD
    T a_viol = T(0), a_zv = T(0);
    int a_pi = 0;
    bool have_scan = false;
#endif
    while (true) {
      if (__any(active && need_p)) {
        T viol, zv;
        int pi;
#if MPCQP_SCAN_AHEAD
        if (have_scan) {
          viol = a_viol;
          pi = a_pi;
          zv = a_zv;
        } else {
          qscan<T, BS>(M, st, zr, B, viol, pi, zv);
        }
#else
        qscan<T, BS>(M, st, zr, B, viol, pi, zv);
#endif
        if (active && need_p) {
          if (!(viol > tol)) {
            active = false;  // settled (pending the exact re-check)
          } else {
            p = pi;
            zp = zv;
            const T lbp = lbs[p], ubp = ubs[p];
            side = (zp < lbp) ? 1 : 2;
            tgt = (side == 1) ? lbp : ubp;
            gp = T(0);
            need_p = false;
          }
        }
      }
      MPCQP_PHASE(5);
      if (!__any(active)) break;
      bool stepping = active;
      if (stepping && ++iters > max_iter) {
        code = MPCQP_STATUS_MAXITER;
        active = false;
        stepping = false;
      }
      constexpr int NC = Mat::NC;  // columns per lane
      T c[BS], cc[NC];
      const T mpp = M.column(p, gb, c, cc);  // c[r] = M_ip, M_pp < 0
      const T rm = fast_rcp(mpp);
      const T sgn = (tgt > zp) ? T(1) : T(-1);
      const T t2 = fabs(tgt - zp);
      T ti = Lim<T>::inf();
      int k = 0;
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const T cs = c[r] * rm;  // dz per unit move of z_p (c stays raw for the sweep)
        const T dmu = ((st[r] == 1) ? -cs : ((st[r] == 2) ? cs : T(0))) * sgn;
        const bool cand = (st[r] == 1 || st[r] == 2) && dmu < T(0);
        const T t = cand ? -mu[r] * fast_rcp(dmu) : Lim<T>::inf();
        const bool take = t < ti;
        ti = take ? t : ti;
        k = take ? (M.bi * BS + r) : k;
      }
      rows_argmin(M, ti, k);
      const bool partial = ti < t2;
      const T s_eff = stepping ? (partial ? ti : t2) : T(0);
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const T cs = c[r] * rm;
        const T dmu = ((st[r] == 1) ? -cs : ((st[r] == 2) ? cs : T(0))) * sgn;
        zr[r] = (st[r] == 0) ? fma(sgn * s_eff, cs, zr[r]) : zr[r];
        mu[r] = fma(s_eff, dmu, mu[r]);
      }
      gp = fma(-sgn * s_eff, rm, gp);  // d g_p / d z_p = -1 / M_pp
      zp = fma(sgn, s_eff, zp);
      MPCQP_PHASE(6);
      // the index whose state changes: k joins F (partial) or p leaves it (full)
      const int idx = partial ? k : p;
      const T sigma = partial ? T(1) : T(-1);
      // full steps sweep on p, whose column is still in registers: publish
      // again only when some group of the wave drops a bound
      T kr[BS], kcol[NC];
      T d = mpp;
      if (__any(stepping && partial)) {
        d = M.column(idx, gb, kr, kcol);
      } else {
#pragma unroll
        for (int r = 0; r < BS; ++r) kr[r] = c[r];
#pragma unroll
        for (int r = 0; r < NC; ++r) kcol[r] = cc[r];
      }
      const bool bad = stepping && (partial ? !(d > T(0)) : !(d < T(0)));
#if MPCQP_SCAN_AHEAD
      // the state changes first, then the next pivot's scan: it reads only z
      // and the states, so its arg-max chain runs ahead of (and can overlap)
      // the sweep; used when the step was full (need_p)
      if (stepping && !bad) {
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          const int i = M.bi * BS + r;
          if (partial && i == k) {
            st[r] = 0;
            mu[r] = T(0);
          }
          if (!partial && i == p) {
            st[r] = side;
            zr[r] = tgt;
            mu[r] = (side == 1) ? gp : -gp;
          }
        }
        need_p = !partial;
      }
      if (bad) {
        code = MPCQP_STATUS_NOT_CONVEX;
        active = false;
      }
      qscan<T, BS>(M, st, zr, B, a_viol, a_pi, a_zv);
      have_scan = true;
      if (stepping && !bad) M.sweep_col(idx, sigma, d, kr, kcol);
      MPCQP_PHASE(7);
#else
      if (stepping && !bad) {
        M.sweep_col(idx, sigma, d, kr, kcol);
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          const int i = M.bi * BS + r;
          if (partial && i == k) {
            st[r] = 0;
            mu[r] = T(0);
          }
          if (!partial && i == p) {
            st[r] = side;
            zr[r] = tgt;
            mu[r] = (side == 1) ? gp : -gp;
          }
        }
        need_p = !partial;
      }
      MPCQP_PHASE(7);
      if (bad) {
        code = MPCQP_STATUS_NOT_CONVEX;
        active = false;
      }
#endif
    }
    // exact refresh for every group, then re-check the bounds
    refresh();
    T viol, zv;
    int pi;
    qscan<T, BS>(M, st, zr, B, viol, pi, zv);
    active = live && code == MPCQP_STATUS_OPTIMAL && viol > tol;
    if (!__any(active)) break;
  }
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    zr[r] = fmin(fmax(zr[r], B.lo[r]), B.hi[r]);
  }
  return code;
}

template <typename T, int BS, class Mat>
__device__ __forceinline__ int gi_box(Mat& M, T* gb, const T* fs, const T* lbs,
                                           const T* ubs, int n, int max_iter, T tol, bool live,
                                           T (&zr)[BS], int& iters MPCQP_CLK_PARAM) {
  int st[BS];
  return gi_box_st<T, BS, false>(M, gb, fs, lbs, ubs, n, max_iter, tol, live, zr, iters,
                                 st MPCQP_CLK_ARG);
}

}  // namespace mpcqp
