// sym2d.hpp -- a symmetric n x n matrix (n <= 8*BS) distributed over one
// wavefront as an 8 x 8 grid of BS x BS register blocks, plus the operations
// the active-set kernels need: Goodnight sweeps, column extraction and a
// mat-vec.  Lane l owns rows bi*BS..bi*BS+BS-1 and columns bj*BS..bj*BS+BS-1
// with bi = l >> 3, bj = l & 7; every lane works on every step (no idle
// lanes as in a row-per-lane layout), pivot columns travel through a 64-entry
// LDS buffer (broadcast reads) and row sums through DPP butterflies.
//
// Vectors indexed by matrix row ("row-block layout") live in T v[BS] on every
// lane, replicated across the 8 lanes of a row block (bj = 0..7).
#pragma once
#include "common.hpp"

#include <type_traits>

namespace mpcqp {

// ---------------------------------------------------------------- DPP
// dpp_ctrl codes (gfx9 encoding): quad_perm xor1 = 0xB1, xor2 = 0x4E,
// row_half_mirror = 0x141 (lane i <-> 7-i within 8), row_ror:8 = 0x128
// (i <-> i+8 within a 16-lane row, i.e. xor 8).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, MPCQP_DPP_BC));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xF, 0xF, MPCQP_DPP_BC);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, MPCQP_DPP_BC);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, MPCQP_DPP_BC);
}

// Sum over the 8 lanes of a row block (lanes bi*8 .. bi*8+7); every lane of
// the block receives the total.
template <typename T>
__device__ __forceinline__ T rowblock_sum(T v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  return v;
}

// Reduce a (value, index) pair across the 8 row blocks (lanes differing in
// bits 3..5).  Lanes within one row block hold identical candidates.
// Arg-max: larger value wins, ties to the smaller index.  NaN never wins.
template <typename T>
__device__ __forceinline__ void blocks_argmax(T& v, int& idx) {
  {
    const T ov = dpp<0x128>(v);
    const int oi = dpp<0x128>(idx);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
  argmax_step<16>(v, idx);
  argmax_step<32>(v, idx);
}

// Same with a payload value carried along with the winner.
template <typename T>
__device__ __forceinline__ void blocks_argmax(T& v, int& idx, T& pay) {
  {
    const T ov = dpp<0x128>(v);
    const int oi = dpp<0x128>(idx);
    const T op = dpp<0x128>(pay);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
    pay = take ? op : pay;
  }
  auto step = [&](auto x) __attribute__((always_inline)) {
    constexpr int X = decltype(x)::value;
    const T ov = lane_step<X>(v);
    const int oi = lane_step<X>(idx);
    const T op = lane_step<X>(pay);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
    pay = take ? op : pay;
  };
  step(std::integral_constant<int, 16>{});
  step(std::integral_constant<int, 32>{});
}

template <typename T>
__device__ __forceinline__ void blocks_argmin(T& v, int& idx) {
  {
    const T ov = dpp<0x128>(v);
    const int oi = dpp<0x128>(idx);
    const bool take = (ov < v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
  argmin_step<16>(v, idx);
  argmin_step<32>(v, idx);
}

// NOTE: no helper here indexes a register array with a runtime value --
// hipcc turns such selects into scratch-memory indexing (guide rule 20).
// Dynamic (wave-uniform) element access always goes through LDS instead.

template <typename T, int BS>
struct Sym2D {
  static constexpr int NMAX = 8 * BS;
  static constexpr int NV = NMAX;  // row-indexed vectors
  static constexpr int NC = BS;    // columns per lane
  static constexpr int RPL = BS;   // rows per lane
  // LDS scratch a kernel must provide: BUF elements (column buffer NMAX, the
  // mat-vec's vector at NMAX * BS)
  static constexpr int BUF = NMAX * BS + NMAX;
  T m[BS][BS];
  int bi, bj;

  __device__ __forceinline__ void init(int lane) {
    bi = lane >> 3;
    bj = lane & 7;
  }

  // Fill from a packed-lower matrix staged in LDS; entries outside n x n are 0.
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

  // Column k (wave-uniform) of M: colr[r] = M[bi*BS+r][k] for this lane's rows,
  // colc[c] = M[bj*BS+c][k] (= row k, by symmetry) for its columns; returns
  // M_kk.  The owning block column publishes only its column kc = k mod BS:
  // a uniform switch over kc (scalar branches; the asm marker keeps the cases
  // from being merged back into one runtime register index, which would live
  // in scratch), BS stores per owner lane instead of its whole tile.
  template <int C>
  __device__ __forceinline__ void put_col(int kc, T* buf) {
    if constexpr (C < BS) {
      if (kc == C) {
#pragma unroll
        for (int r = 0; r < BS; ++r) buf[bi * BS + r] = m[r][C];
        asm volatile("; s2col %0" ::"n"(C));
      } else {
        put_col<C + 1>(kc, buf);
      }
    }
  }
  __device__ __forceinline__ T column(int k, T* buf, T (&colr)[BS], T (&colc)[BS]) {
    T unused;
    return column<false>(k, buf, colr, colc, unused);
  }
  // The same, and with LANE: cl = M[lane][k] for the row-per-lane layout
  // (lanes past NMAX read row 0).
  template <bool LANE>
  __device__ __forceinline__ T column(int k, T* buf, T (&colr)[BS], T (&colc)[BS], T& cl) {
    k = __builtin_amdgcn_readfirstlane(k);
    const int kb = k / BS, kc = k - kb * BS;
    if (bj == kb) put_col<0>(kc, buf);
    lds_exchange();
#pragma unroll
    for (int r = 0; r < BS; ++r) colr[r] = buf[bi * BS + r];
#pragma unroll
    for (int c = 0; c < BS; ++c) colc[c] = buf[bj * BS + c];
    if constexpr (LANE) {
      const int l = (int)lane_id();
      cl = buf[l < NMAX ? l : 0];
    }
    const T d = buf[k];
    lds_exchange();
    return d;
  }

  // Goodnight sweep on pivot k with its column fetched (d = M_kk): sigma =
  // +1 moves k into the swept set, sigma = -1 (reverse sweep) moves it out.
  // Every element takes the rank-1 update; row and column k are then set
  // (selected, not produced by cancellation) by the lanes that hold them,
  // through uniform switches over k's in-block offset.
  // row k: sigma rd M[k][j] (-rd on the diagonal), on the lanes with bi == kb
  template <int R>
  __device__ __forceinline__ void patch_row(int kc, bool on, int k, T rd, T srd,
                                            const T (&colc)[BS]) {
    if constexpr (R < BS) {
      if (kc == R) {
#pragma unroll
        for (int c = 0; c < BS; ++c) {
          const T v = (bj * BS + c) == k ? -rd : srd * colc[c];
          m[R][c] = on ? v : m[R][c];
        }
        asm volatile("; s2row %0" ::"n"(R));
      } else {
        patch_row<R + 1>(kc, on, k, rd, srd, colc);
      }
    }
  }
  // column k: sigma rd M[i][k], on the lanes with bj == kb
  template <int C>
  __device__ __forceinline__ void patch_col(int kc, bool on, int k, T rd, T sigma,
                                            const T (&ar)[BS]) {
    if constexpr (C < BS) {
      if (kc == C) {
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          const T v = (bi * BS + r) == k ? -rd : sigma * ar[r];
          m[r][C] = on ? v : m[r][C];
        }
        asm volatile("; s2pc %0" ::"n"(C));
      } else {
        patch_col<C + 1>(kc, on, k, rd, sigma, ar);
      }
    }
  }
  __device__ __forceinline__ void sweep_col(int k, T sigma, T d, const T (&colr)[BS],
                                            const T (&colc)[BS]) {
    k = __builtin_amdgcn_readfirstlane(k);
    const int kb = k / BS, kc = k - kb * BS;
    const T rd = fast_rcp(d);
    T ar[BS];
#pragma unroll
    for (int r = 0; r < BS; ++r) ar[r] = colr[r] * rd;
#pragma unroll
    for (int r = 0; r < BS; ++r)
#pragma unroll
      for (int c = 0; c < BS; ++c) m[r][c] = fma(-ar[r], colc[c], m[r][c]);
    patch_row<0>(kc, bi == kb, k, rd, sigma * rd, colc);
    patch_col<0>(kc, bj == kb, k, rd, sigma, ar);
  }

  // Fetch column k and sweep on it.  Returns the pivot M_kk.
  __device__ __forceinline__ T sweep(int k, T sigma, T* buf) {
    T colr[BS], colc[BS];
    const T d = column(k, buf, colr, colc);
    sweep_col(k, sigma, d, colr, colc);
    return d;
  }

  // out[r] = sum_j M[i][j] w[j] for this lane's rows; w in row-block layout.
  __device__ __forceinline__ void matvec(const T (&w)[BS], T* buf, T (&out)[BS]) {
    T* wb = buf + NMAX * BS;
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
      out[r] = rowblock_sum(s);
    }
    lds_exchange();
  }
};

// out_l = sum_j M[l][j] w_j with both vectors one row per lane (lane l = row
// l; lanes past NMAX pass 0 and get row 0's value).  Uses the mat-vec's
// vector slot of buf and its column slot for the result.
template <typename T, int BS>
__device__ __forceinline__ T matvec_lane(const Sym2D<T, BS>& W, T w, T* buf) {
  constexpr int NMAX = Sym2D<T, BS>::NMAX;
  T* wb = buf + NMAX * BS;
  const int l = (int)lane_id();
  if (l < NMAX) wb[l] = w;
  lds_exchange();
  T wc[BS];
#pragma unroll
  for (int c = 0; c < BS; ++c) wc[c] = wb[W.bj * BS + c];
  T out[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    T s = T(0);
#pragma unroll
    for (int c = 0; c < BS; ++c) s = fma(W.m[r][c], wc[c], s);
    out[r] = rowblock_sum(s);
  }
  if (W.bj == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) buf[W.bi * BS + r] = out[r];
  }
  lds_exchange();
  const T v = buf[l < NMAX ? l : 0];
  lds_exchange();
  return v;
}

// The same with the row sums reduced through LDS instead of DPP butterflies:
// every lane stores its BS partial row sums (part: 8 * NMAX elements), and
// lane l adds the 8 partials of row l -- BS stores, 8 loads and 7 adds per
// lane instead of 3 DPP steps per row.
template <typename T, int BS>
__device__ __forceinline__ T matvec_lane_lds(const Sym2D<T, BS>& W, T w, T* buf, T* part) {
  constexpr int NMAX = Sym2D<T, BS>::NMAX;
  T* wb = buf + NMAX * BS;
  const int l = (int)lane_id();
  if (l < NMAX) wb[l] = w;
  lds_exchange();
  T wc[BS];
#pragma unroll
  for (int c = 0; c < BS; ++c) wc[c] = wb[W.bj * BS + c];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    T s = T(0);
#pragma unroll
    for (int c = 0; c < BS; ++c) s = fma(W.m[r][c], wc[c], s);
    part[(W.bi * BS + r) * 8 + W.bj] = s;
  }
  lds_exchange();
  const T* pr = part + (l < NMAX ? l : 0) * 8;
  T v = pr[0];
#pragma unroll
  for (int q = 1; q < 8; ++q) v += pr[q];
  lds_exchange();
  return v;
}

// Publish a row-block vector to LDS (vb[0..8*BS)) so that a wave-uniform
// element can be read back by address.
template <typename T, int BS>
__device__ __forceinline__ void publish(const T (&v)[BS], T* vb, int bi, int bj) {
  if (bj == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) vb[bi * BS + r] = v[r];
  }
}

// Stage a packed lower triangle of P elements into LDS with coalesced loads.
template <typename T, int MAXE>
__device__ __forceinline__ void stage_packed(const T* g, T* Ps, int P, int lane) {
  constexpr int MAXT = (MAXE + kWave - 1) / kWave;
  T tmp[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int e = lane + t * kWave;
    tmp[t] = (e < P) ? g[e] : T(0);
  }
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int e = lane + t * kWave;
    if (e < P) Ps[e] = tmp[t];
  }
}

}  // namespace mpcqp
