// condense.hip -- batched single-shooting condensing on gfx950.
//
// Restates the symbolic elimination of session_4/main.py:86-106 (and
// session4_sol.py:195-204) for linear(ised) dynamics
//     x_{k+1} = A_k x_k + B_k u_k + c_k,   z = [u_0; ...; u_{N-1}]
// with cost  sum_{k<N} x_k'Q x_k + u_k'R u_k + x_N'Qf x_N.
//
// Instead of forming Gamma and the dense product Gamma'QhatGamma, each
// instance runs a backward cost-to-go recursion
//     W_N = Qf,   W_k = Q + A_k' W_{k+1} A_k
// after which every entry of the condensed Hessian is a short forward sweep:
//     H_{(i,a),(j,b)} = B_i[:,a]' W_{i+1} s_{i+1},  s_{j+1} = B_j e_b,
//     s_{m+1} = A_m s_m                                       (i >= j)
//     F_{(i,a)}       = B_i[:,a]' W_{i+1} Phi_{i+1}
//     f_{(i,a)}       = B_i[:,a]' y_{i+1},   y_k = Q xbar_k + A_k' y_{k+1}
// (xbar = free response Phi x0 + w).  Cost O(N nx^2 (N nu + nx)) per
// instance; Gamma and Phi fall out of the forward sweep for free.
//
// Mapping: one instance per 64-lane workgroup (= one wavefront).  The
// per-instance matrices (A_k, B_k, Q, R, Qf, W_k, xbar, y_k) live in
// LDS; lane c owns column c of [H | F] (z-columns then Phi-columns), so each H
// row is written by consecutive lanes to consecutive packed addresses.  For
// nx <= 2 the recursions run redundantly in every lane's registers (no LDS
// round trips on the serial chain); wider states use an LDS-parallel W
// recursion with the xbar recursion on other lanes of the same phases.
#include "common.hpp"
#include "mfma.hpp"

#include <cstdlib>

// Recursions redundantly in every lane's registers up to this nx; wider
// states (already nx = 4) use the LDS-parallel recursion, one entry per lane.
#ifndef MPCQP_CONDENSE_REG_NX
#define MPCQP_CONDENSE_REG_NX 2
#endif

namespace mpcqp {

template <typename T>
struct CondenseArgs {
  int batch, nx, nu, N, tv;
  const T* A; int64_t sA;
  const T* B; int64_t sB;
  const T* Q; int64_t sQ;
  const T* R; int64_t sR;
  const T* Qf; int64_t sQf;
  const T* c; int64_t sC;
  const T* x0; int64_t sX0;
  T* H; T* F; T* f; T* Gam; T* Phi; T* xbar;
  int rh, rg;  // output rings (elements, powers of two) of the streamed sweep; rh = 0: direct stores
  int gpk = 0;     // Gam as its lower block triangle (MPCQP_GAM_PACKED)
  const int* count = nullptr;  // device count: instances b >= *count are skipped (list mode)
};

struct CLayout {
  int oA, oB, oQ, oQf, oR, oW, oT, oX, oY, oC, oX0, oWh, oRH, oRG, total;
};

// Streamed sweep (rh > 0): A, R and What_k = B_k' W_{k+1} persist; everything
// else is dead once What, f and xbar are out, and the two output rings
// overlay it.
__host__ __device__ inline CLayout clayout(int NX, int nu, int N, int tv, int rh, int rg) {
  CLayout L;
  const int S = tv ? N : 1;
  auto al4 = [](int o) { return (o + 3) & ~3; };  // 16-byte ring / vector alignment
  L.oA = 0;
  int o = S * NX * NX;
  L.oWh = L.oRH = L.oRG = 0;
  if (rh) {
    L.oR = o;
    o = al4(o + nu * nu);
    L.oWh = o;                         // What_k, k = 0..N-1 (nu x NX each)
    o = al4(o + N * nu * NX);
  }
  const int u = o;
  L.oB = o;
  L.oQ = L.oB + S * NX * nu;
  L.oQf = L.oQ + NX * NX;
  o = L.oQf + NX * NX;
  if (!rh) {
    L.oR = o;
    o += nu * nu;
  }
  L.oW = o;                            // W_k, k = 0..N  ((N+1) slots; slot 0 unused)
  L.oT = L.oW + (N + 1) * NX * NX;     // scratch NX x NX
  L.oX = L.oT + NX * NX;               // xbar_k, k = 0..N
  L.oY = L.oX + (N + 1) * NX;          // y_k, k = 0..N
  L.oC = L.oY + (N + 1) * NX;          // drift c_k, k = 0..N-1
  L.oX0 = L.oC + N * NX;               // x0
  L.total = L.oX0 + NX;
  if (rh) {
    L.oRH = u;
    L.oRG = u + rh;
    if (u + rh + rg > L.total) L.total = u + rh + rg;
  }
  return L;
}

// e / d for 0 <= e < 2^24 from a float estimate, corrected to exact
__device__ __forceinline__ int qdiv(int e, int d, float rd) {
  int s = (int)((float)e * rd);
  s -= (s * d > e) ? 1 : 0;
  s += ((s + 1) * d <= e) ? 1 : 0;
  return s;
}

// Stage-in of one instance into LDS.  A, B, c of one instance are dense runs
// in HBM.  All loads of a chunk (UA + UB + UC per lane, clamped addresses, no
// branches) are issued before its LDS stores, so a chunk costs one HBM round
// trip; config 3 (N = 30, nx = 4) is one chunk.  Padding (nx < NX) is zeroed
// first and the data scattered over it (LDS ops of one wave complete in order).
template <typename T, int NX>
__device__ __forceinline__ void stage_in(const CondenseArgs<T>& a, int b, int lane, bool need_aff,
                                         T* As, T* Bs, T* Cs, T* Qs, T* Qfs, T* Rs, T* X0s) {
  const int nx = a.nx, nu = a.nu, N = a.N;
  const int S = a.tv ? N : 1;
  const T* Ab = a.A + (int64_t)b * a.sA;
  const T* Bb = a.B + (int64_t)b * a.sB;
  const T* Cb = (need_aff && a.c) ? a.c + (int64_t)b * a.sC : nullptr;
  const T* Qb = a.Q + (int64_t)b * a.sQ;
  const T* Qfb = a.Qf + (int64_t)b * a.sQf;
  const T* Rb = a.R + (int64_t)b * a.sR;
  const T* X0b = (need_aff && a.x0) ? a.x0 + (int64_t)b * a.sX0 : nullptr;
  const int cA = S * nx * nx, cB = S * nx * nu, cC = Cb ? N * nx : 0, cR = nu * nu;
  // small operands: Q, Qf (QK padded entries per lane), R (<= 4 per lane), x0
  constexpr int QK = (NX * NX + kWave - 1) / kWave;
  T qv[QK], qfv[QK];
  bool qin[QK];
#pragma unroll
  for (int k = 0; k < QK; ++k) {
    const int e = k * kWave + lane, qr = e / NX, qq = e % NX;
    qin[k] = e < NX * NX && qr < nx && qq < nx;
    const int qo = qin[k] ? qr * nx + qq : 0;
    qv[k] = Qb[qo];
    qfv[k] = Qfb[qo];
  }
  T rv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = k * kWave + lane;
    rv[k] = Rb[e < cR ? e : 0];
  }
  const T x0v = X0b ? X0b[lane < nx ? lane : 0] : T(0);
  const bool pad = nx < NX;
  if (pad) {
    for (int e = lane; e < S * NX * NX; e += kWave) As[e] = T(0);
    for (int e = lane; e < S * NX * nu; e += kWave) Bs[e] = T(0);
  }
  if (need_aff && (pad || !Cb))
    for (int e = lane; e < N * NX; e += kWave) Cs[e] = T(0);
  const float rA = 1.f / (float)(nx * nx), rB = 1.f / (float)(nx * nu), rN = 1.f / (float)nx;
  constexpr int UA = 8, UB = 4, UC = 2;
  auto chunk = [&](int c) {
    T va[UA], vb[UB], vc[UC];
#pragma unroll
    for (int k = 0; k < UA; ++k) {
      const int e = (c * UA + k) * kWave + lane;
      va[k] = Ab[e < cA ? e : 0];
    }
#pragma unroll
    for (int k = 0; k < UB; ++k) {
      const int e = (c * UB + k) * kWave + lane;
      vb[k] = Bb[e < cB ? e : 0];
    }
#pragma unroll
    for (int k = 0; k < UC; ++k) {
      const int e = (c * UC + k) * kWave + lane;
      vc[k] = (e < cC) ? Cb[e] : T(0);
    }
#pragma unroll
    for (int k = 0; k < UA; ++k) {
      const int e = (c * UA + k) * kWave + lane;
      if (e < cA) {
        int o = e;
        if (pad) {
          const int s = qdiv(e, nx * nx, rA), rem = e - s * nx * nx;
          const int r = qdiv(rem, nx, rN);
          o = s * NX * NX + r * NX + (rem - r * nx);
        }
        As[o] = va[k];
      }
    }
#pragma unroll
    for (int k = 0; k < UB; ++k) {
      const int e = (c * UB + k) * kWave + lane;
      if (e < cB) Bs[pad ? e + qdiv(e, nx * nu, rB) * (NX - nx) * nu : e] = vb[k];
    }
#pragma unroll
    for (int k = 0; k < UC; ++k) {
      const int e = (c * UC + k) * kWave + lane;
      if (e < cC) Cs[pad ? e + qdiv(e, nx, rN) * (NX - nx) : e] = vc[k];
    }
  };
  // chunk 0 outside the loop: its loads share the round trip of the small
  // operands above (a loop header would wait for those first)
  chunk(0);
  for (int c = 1; c * kWave * UA < cA || c * kWave * UB < cB || c * kWave * UC < cC; ++c) chunk(c);
#pragma unroll
  for (int k = 0; k < QK; ++k) {
    const int e = k * kWave + lane;
    if (e < NX * NX) {
      Qs[e] = qin[k] ? qv[k] : T(0);
      Qfs[e] = qin[k] ? qfv[k] : T(0);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k * kWave + lane < cR) Rs[k * kWave + lane] = rv[k];
  if (need_aff && lane < NX) X0s[lane] = lane < nx ? x0v : T(0);
}

template <typename T, int NX>
__global__ __launch_bounds__(64) void condense_kernel(CondenseArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x;
  if (a.count && b >= *a.count) return;  // uniform per workgroup
  const int lane = threadIdx.x;
  const int nx = a.nx, nu = a.nu, N = a.N, n = N * nu;
  const int tv = a.tv;
  const CLayout L = clayout(NX, nu, N, tv, a.rh, a.rg);
  T* As = sm + L.oA;
  T* Bs = sm + L.oB;
  T* Qs = sm + L.oQ;
  T* Qfs = sm + L.oQf;
  T* Rs = sm + L.oR;
  T* Ws = sm + L.oW;
  T* Ts = sm + L.oT;
  T* Xs = sm + L.oX;
  T* Ys = sm + L.oY;
  T* Cs = sm + L.oC;
  T* X0s = sm + L.oX0;
  const bool need_aff = (a.f != nullptr) || (a.xbar != nullptr);
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif

  stage_in<T, NX>(a, b, lane, need_aff, As, Bs, Cs, Qs, Qfs, Rs, X0s);
  __syncthreads();
  MPCQP_PHASE(0);

  // ------------------------------------------------------------ recursions
  if constexpr (NX <= MPCQP_CONDENSE_REG_NX) {
    // Serial chains, computed redundantly by every lane in registers (the
    // wave issues one instruction stream either way); lane 0 publishes.
    T W[NX][NX], Qr[NX][NX], Ar[NX][NX];
#pragma unroll
    for (int r = 0; r < NX; ++r)
#pragma unroll
      for (int q = 0; q < NX; ++q) {
        W[r][q] = Qfs[r * NX + q];
        Qr[r][q] = Qs[r * NX + q];
        Ar[r][q] = As[r * NX + q];
      }
    if (lane == 0)
#pragma unroll
      for (int e = 0; e < NX * NX; ++e) Ws[N * NX * NX + e] = W[e / NX][e % NX];
    for (int k = N - 1; k >= 1; --k) {
      if (tv) {
#pragma unroll
        for (int r = 0; r < NX; ++r)
#pragma unroll
          for (int q = 0; q < NX; ++q) Ar[r][q] = As[k * NX * NX + r * NX + q];
      }
      T Tm[NX][NX];
#pragma unroll
      for (int p = 0; p < NX; ++p)
#pragma unroll
        for (int q = 0; q < NX; ++q) {
          T acc = T(0);
#pragma unroll
          for (int s = 0; s < NX; ++s) acc = fma(W[p][s], Ar[s][q], acc);
          Tm[p][q] = acc;
        }
#pragma unroll
      for (int r = 0; r < NX; ++r)
#pragma unroll
        for (int q = 0; q < NX; ++q) {
          T acc = Qr[r][q];
#pragma unroll
          for (int p = 0; p < NX; ++p) acc = fma(Ar[p][r], Tm[p][q], acc);
          W[r][q] = acc;
        }
      if (lane == 0)
#pragma unroll
        for (int e = 0; e < NX * NX; ++e) Ws[k * NX * NX + e] = W[e / NX][e % NX];
    }
    if (need_aff) {
      T xk[NX];
      T xs[NX];  // keep the whole trajectory in LDS; registers carry the chain
#pragma unroll
      for (int q = 0; q < NX; ++q) xk[q] = X0s[q];
      if (lane == 0)
#pragma unroll
        for (int q = 0; q < NX; ++q) Xs[q] = xk[q];
      if (!tv)
#pragma unroll
        for (int r = 0; r < NX; ++r)
#pragma unroll
          for (int q = 0; q < NX; ++q) Ar[r][q] = As[r * NX + q];
      for (int k = 0; k < N; ++k) {
        if (tv) {
#pragma unroll
          for (int r = 0; r < NX; ++r)
#pragma unroll
            for (int q = 0; q < NX; ++q) Ar[r][q] = As[k * NX * NX + r * NX + q];
        }
#pragma unroll
        for (int r = 0; r < NX; ++r) {
          T acc = Cs[k * NX + r];
#pragma unroll
          for (int q = 0; q < NX; ++q) acc = fma(Ar[r][q], xk[q], acc);
          xs[r] = acc;
        }
#pragma unroll
        for (int q = 0; q < NX; ++q) xk[q] = xs[q];
        if (lane == 0)
#pragma unroll
          for (int q = 0; q < NX; ++q) Xs[(k + 1) * NX + q] = xk[q];
      }
    }
  } else {
    // LDS-parallel recursions: entry (p,q) of each NX x NX product per lane;
    // the free-response recursion x_{k+1} = A_k x_k + c_k runs in the same
    // barrier phases on other lanes (it is independent of W).
    const int xoff = (NX * NX <= 32) ? 32 : 0;
    const int xl = lane - xoff;
    const bool xlane = need_aff && xl >= 0 && xl < NX;
    for (int e = lane; e < NX * NX; e += kWave) Ws[N * NX * NX + e] = Qfs[e];
    if (xlane) Xs[xl] = X0s[xl];
    __syncthreads();
    for (int t = 0; t < N; ++t) {
      const int k = N - 1 - t;  // W step (k >= 1)
      const T* Ak = As + (tv ? k : 0) * NX * NX;
      const T* W1 = Ws + (k + 1) * NX * NX;
      if (k >= 1) {
        for (int e = lane; e < NX * NX; e += kWave) {
          const int p = e / NX, q = e % NX;
          T acc = T(0);
#pragma unroll
          for (int s = 0; s < NX; ++s) acc = fma(W1[p * NX + s], Ak[s * NX + q], acc);
          Ts[e] = acc;
        }
      }
      if (xlane) {
        const T* At = As + (tv ? t : 0) * NX * NX;
        T acc = Cs[t * NX + xl];
#pragma unroll
        for (int q = 0; q < NX; ++q) acc = fma(At[xl * NX + q], Xs[t * NX + q], acc);
        Xs[(t + 1) * NX + xl] = acc;
      }
      __syncthreads();
      if (k >= 1) {
        for (int e = lane; e < NX * NX; e += kWave) {
          const int r = e / NX, q = e % NX;
          T acc = Qs[e];
#pragma unroll
          for (int p = 0; p < NX; ++p) acc = fma(Ak[p * NX + r], Ts[p * NX + q], acc);
          Ws[k * NX * NX + e] = acc;
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
  MPCQP_PHASE(1);
  // adjoint y_N = Qf xbar_N, y_k = Q xbar_k + A_k' y_{k+1}  (f = B_k' y_{k+1}).
  // Summing f along the columns instead (f_col = sum_k s_k' Q xbar_k) removes
  // this chain but loses ~10x accuracy in fp32 (cancellation), so it stays.
  if (need_aff) {
    if (lane < NX) {
      T acc = T(0);
#pragma unroll
      for (int q = 0; q < NX; ++q) acc = fma(Qfs[lane * NX + q], Xs[N * NX + q], acc);
      Ys[N * NX + lane] = acc;
    }
    __syncthreads();
    for (int k = N - 1; k >= 1; --k) {
      const T* Ak = As + (tv ? k : 0) * NX * NX;
      if (lane < NX) {
        T acc = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) acc = fma(Qs[lane * NX + q], Xs[k * NX + q], acc);
#pragma unroll
        for (int p = 0; p < NX; ++p) acc = fma(Ak[p * NX + lane], Ys[(k + 1) * NX + p], acc);
        Ys[k * NX + lane] = acc;
      }
      __syncthreads();
    }
  }
  MPCQP_PHASE(2);

  // ------------------------------------------------- linear term and xbar
  if (a.f) {
    T* fb = a.f + (int64_t)b * n;
    const float rNu = 1.f / (float)nu;
    for (int r = lane; r < n; r += kWave) {
      const int i = qdiv(r, nu, rNu), aa = r - i * nu;
      const T* Bi = Bs + (tv ? i : 0) * NX * nu;
      T acc = T(0);
#pragma unroll
      for (int q = 0; q < NX; ++q) acc = fma(Bi[q * nu + aa], Ys[(i + 1) * NX + q], acc);
      fb[r] = acc;
    }
  }
  if (a.xbar) {
    T* xb = a.xbar + (int64_t)b * N * nx;
    const float rN = 1.f / (float)nx;
    for (int e = lane; e < N * nx; e += kWave) {
      const int k = qdiv(e, nx, rN), q = e - k * nx;
      xb[e] = Xs[(k + 1) * NX + q];
    }
  }
  MPCQP_PHASE(3);

  // ------------------------------------------------------- column sweep
  // z columns (H, Gam), then -- only when F or Phi is requested -- the x0
  // columns
  const int ncol = n + ((a.F || a.Phi) ? nx : 0);
  T* Hb = a.H + (int64_t)b * ((int64_t)n * (n + 1) / 2);
  T* Fb = a.F ? a.F + (int64_t)b * n * nx : nullptr;
  // packed Gam: block row i (x_{i+1}) holds its (i+1) nu leading columns,
  // column by column (nx entries each), from nx nu i (i+1) / 2
  // (gam_packed_size / gam_packed_off)
  const int64_t gsz = a.gpk ? gam_packed_size(nx, nu, N) : (int64_t)N * nx * n;
  T* Gb = a.Gam ? a.Gam + (int64_t)b * gsz : nullptr;
  T* Pb = a.Phi ? a.Phi + (int64_t)b * ((int64_t)N * nx * nx) : nullptr;
  if (a.rh) {
    // Streamed sweep (ncol <= 64, one column per lane).  H row block i is
    // What_i s_{i+1} (nu x NX FMAs instead of W s then B' v), and both H
    // (packed rows, in order) and Gamma (block row i = rows i*nx..) are one
    // contiguous stream per instance in stage order: lanes scatter their
    // entries into an LDS ring, and every complete CH-element window leaves as
    // one 16-byte-per-lane store (a quarter of the store instructions of
    // per-row 4-byte stores, which bound the direct sweep).
    T* Whs = sm + L.oWh;
    {
      const int cnt = N * nu * NX;
      const float rW = 1.f / (float)(nu * NX);
      for (int e = lane; e < cnt; e += kWave) {
        const int k = qdiv(e, nu * NX, rW), rem = e - k * nu * NX;
        const int aa = rem / NX, q = rem % NX;
        const T* Bk = Bs + (tv ? k : 0) * NX * nu;
        const T* W1 = Ws + (k + 1) * NX * NX;
        T acc = T(0);
#pragma unroll
        for (int p = 0; p < NX; ++p) acc = fma(Bk[p * nu + aa], W1[p * NX + q], acc);
        Whs[e] = acc;
      }
    }
    const int col = lane;
    const bool act = col < ncol;
    const bool isz = col < n;
    const int j = isz ? col / nu : -1;
    const int bc = isz ? col - j * nu : col - n;
    T bcol[NX];  // B_j e_bc, injected at stage j
#pragma unroll
    for (int q = 0; q < NX; ++q) bcol[q] = isz ? Bs[(tv ? j : 0) * NX * nu + q * nu + bc] : T(0);
    __syncthreads();  // What visible; B, W, X, Y dead: the rings take over
    constexpr int VEC = 16 / (int)sizeof(T);
    constexpr int CH = kWave * VEC;
    typedef T VT __attribute__((ext_vector_type(VEC)));
    T* RH = sm + L.oRH;
    T* RG = sm + L.oRG;
    const int RHM = a.rh - 1, RGM = a.rg - 1;
    // ring position p <-> element g0 + p, g0 = VEC-aligned, d = offset of the stream
    const int dh = (int)(((uintptr_t)Hb / sizeof(T)) % VEC);
    const int dg = Gb ? (int)(((uintptr_t)Gb / sizeof(T)) % VEC) : 0;
    T* Hal = Hb - dh;
    T* Gal = Gb ? Gb - dg : nullptr;
    const int hiH = dh + n * (n + 1) / 2, hiG = dg + (int)gsz;
    auto flush = [&](const T* ring, int rmask, T* gal, int w, int lo, int hi) {
      const int p0 = w + lane * VEC;
      if (p0 < hi && p0 + VEC > lo) {
        const VT v = *reinterpret_cast<const VT*>(ring + (p0 & rmask));
        if (p0 >= lo && p0 + VEC <= hi) {
          __builtin_nontemporal_store(v, reinterpret_cast<VT*>(gal + p0));
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e)
            if (p0 + e >= lo && p0 + e < hi) gal[p0 + e] = v[e];
        }
      }
    };
    T s[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) s[q] = (!isz && q == bc) ? T(1) : T(0);
    int fh = 0, fg = 0;  // flushed ring positions (multiples of CH)
    for (int i = 0; i < N; ++i) {
      const T* Ai = As + (tv ? i : 0) * NX * NX;
      const T* Wh = Whs + i * nu * NX;
      const bool inj = isz && (i == j);
      T t[NX];
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        T acc = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) acc = fma(Ai[r * NX + q], s[q], acc);
        t[r] = acc;
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) s[q] = inj ? bcol[q] : t[q];
      if (Gb && isz) {
        if (a.gpk) {
          const int o = dg + gam_packed_off(nx, nu, i) + col * nx;
          if (col < (i + 1) * nu)
#pragma unroll
            for (int q = 0; q < NX; ++q)
              if (q < nx) RG[(o + q) & RGM] = s[q];
        } else {
#pragma unroll
          for (int q = 0; q < NX; ++q)
            if (q < nx) RG[(dg + (i * nx + q) * n + col) & RGM] = s[q];
        }
      }
      if (act && !isz && Pb) {
#pragma unroll
        for (int q = 0; q < NX; ++q)
          if (q < nx) Pb[(i * nx + q) * nx + bc] = s[q];
      }
      for (int aa = 0; aa < nu; ++aa) {
        T o = inj ? Rs[aa * nu + bc] : T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) o = fma(Wh[aa * NX + q], s[q], o);
        const int r = i * nu + aa;
        if (isz) {
          if (col <= r) RH[(dh + r * (r + 1) / 2 + col) & RHM] = o;
        } else if (act && Fb) {
          Fb[r * nx + bc] = o;
        }
      }
      const int rr = (i + 1) * nu;
      const int ph = dh + rr * (rr + 1) / 2,
                pg = Gb ? dg + (a.gpk ? gam_packed_off(nx, nu, i + 1) : (i + 1) * nx * n) : 0;
      if (ph - fh >= CH || pg - fg >= CH) {
        __syncthreads();
        for (; ph - fh >= CH; fh += CH) flush(RH, RHM, Hal, fh, dh, hiH);
        for (; pg - fg >= CH; fg += CH) flush(RG, RGM, Gal, fg, dg, hiG);
        asm volatile("" ::: "memory");
      }
    }
    __syncthreads();
    for (; fh < hiH; fh += CH) flush(RH, RHM, Hal, fh, dh, hiH);
    if (Gb)
      for (; fg < hiG; fg += CH) flush(RG, RGM, Gal, fg, dg, hiG);
  }
  for (int col0 = 0; col0 < (a.rh ? 0 : ncol); col0 += kWave) {
    const int col = col0 + lane;
    const bool act = col < ncol;
    const bool isz = col < n;
    const int j = isz ? col / nu : -1;
    const int bc = isz ? col - j * nu : col - n;
    T s[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) s[q] = (!isz && q == bc) ? T(1) : T(0);
    for (int i = 0; i < N; ++i) {
      const T* Ai = As + (tv ? i : 0) * NX * NX;
      const T* Bi = Bs + (tv ? i : 0) * NX * nu;
      const T* Wi = Ws + (i + 1) * NX * NX;
      const bool inj = isz && (i == j);
      if (inj) {
#pragma unroll
        for (int q = 0; q < NX; ++q) s[q] = Bi[q * nu + bc];
      } else {
        T t[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) {
          T acc = T(0);
#pragma unroll
          for (int q = 0; q < NX; ++q) acc = fma(Ai[r * NX + q], s[q], acc);
          t[r] = acc;
        }
#pragma unroll
        for (int q = 0; q < NX; ++q) s[q] = t[q];
      }
      if (act) {
        if (isz && Gb) {
          if (a.gpk) {
            if (col < (i + 1) * nu)
#pragma unroll
              for (int q = 0; q < NX; ++q)
                if (q < nx) __builtin_nontemporal_store(s[q], &Gb[gam_packed_off(nx, nu, i) + col * nx + q]);
          } else {
#pragma unroll
            for (int q = 0; q < NX; ++q)
              if (q < nx) __builtin_nontemporal_store(s[q], &Gb[((int64_t)(i * nx + q)) * n + col]);
          }
        }
        if (!isz && Pb) {
#pragma unroll
          for (int q = 0; q < NX; ++q)
            if (q < nx) Pb[(i * nx + q) * nx + bc] = s[q];
        }
      }
      if (isz && i < j) continue;  // strictly-upper block: nothing to emit
      T v[NX];
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        T acc = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) acc = fma(Wi[r * NX + q], s[q], acc);
        v[r] = acc;
      }
      for (int aa = 0; aa < nu; ++aa) {
        T o = inj ? Rs[aa * nu + bc] : T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) o = fma(Bi[q * nu + aa], v[q], o);
        const int r = i * nu + aa;
        if (act) {
          if (isz) {
            if (r >= col) __builtin_nontemporal_store(o, &Hb[(int64_t)r * (r + 1) / 2 + col]);
          } else if (Fb) {
            Fb[r * nx + bc] = o;
          }
        }
      }
    }
  }
  MPCQP_PHASE(4);
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

// ================================================================ streamed kernel
// condense_stream_kernel<T, NX, NU>: the wavefront kernel's streamed sweep
// (one column per lane, every column <= 64) with the affine part carried by
// a spare lane instead of the free-response and adjoint chains, and ONE LDS
// round trip per backward stage.  With the affine cost-to-go
//     y_k = W_k xbar_k + eta_k,  eta_N = 0,
//     eta_k = A_k' (W_{k+1} c_k + eta_{k+1})
// (y_k = Q xbar_k + A_k' y_{k+1} by induction), the linear term is
//     f_(i,a) = B_i[:,a]' y_{i+1} = What_i[a,:] xbar_{i+1} + ghat_i[a],
//     ghat_i = B_i' eta_{i+1},
// i.e. the H-row formula of one more column whose vector is xbar itself
// (s = A_i s + c_i from s = x0): the lane after the last column computes f
// and xbar inside the forward sweep.  Every backward quantity of stage k is a
// function of stage k+1's only,
//     out = base + sum_p L[p] (sum_s W_{k+1}[p][s] y[s] + e1 eta_{k+1}[p])
//   W_k(r,q):   L = A_k[:,r], y = A_k[:,q], base = Q[r][q]
//   eta_k(r):   L = A_k[:,r], y = c_k,      e1 = 1
//   What_k(a,q): L = B_k[:,a], y = e_q
//   ghat_k(a):  L = B_k[:,a], y = 0,        e1 = 1
// so each stage is one phase: every lane evaluates the same expression for
// its item (no divergence), W and eta double-buffered in LDS.
// Gamma is written packed (MPCQP_GAM_PACKED, block column by column): a
// lane's nx entries of its column are one contiguous vector, one 16-byte
// store per lane and stage (no ring).  H keeps the ring of packed rows,
// flushed in half-wave windows (a 256-element ring at config 3).
struct SLayout {
  int oA, oC, oWh, oGh, oR, oX0, oFo, oXo, oB, oQ, oQf, oW, oE, oI, oZ, oRH, total;
};
__host__ __device__ inline SLayout slayout(int NX, int nu, int N, int tv, int rh, int fo, int xo) {
  SLayout L;
  const int S = tv ? N : 1;
  auto al4 = [](int o) { return (o + 3) & ~3; };
  int o = 0;
  L.oA = o; o = al4(o + S * NX * NX);
  L.oC = o; o = al4(o + N * NX);
  L.oWh = o; o = al4(o + N * nu * NX);
  L.oGh = o; o = al4(o + N * nu);
  L.oR = o; o = al4(o + nu * nu);
  L.oX0 = o; o = al4(o + NX);
  L.oFo = o; o = al4(o + (fo ? N * nu : 0));
  L.oXo = o; o = al4(o + (xo ? N * NX : 0));
  // dead once the backward pass is done: the H ring overlays them
  int u = o;
  L.oB = u; u = al4(u + S * NX * nu);
  L.oQ = u; u = al4(u + NX * NX);
  L.oQf = u; u = al4(u + NX * NX);
  L.oW = u; u = al4(u + 2 * NX * NX);
  L.oE = u; u = al4(u + 2 * NX);
  L.oI = u; u = al4(u + NX * NX);
  L.oZ = u; u = al4(u + NX);
  L.oRH = o;
  L.total = u > o + rh ? u : o + rh;
  return L;
}

template <typename T, int NX, int NU>
__global__ __launch_bounds__(64) void condense_stream_kernel(CondenseArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x;
  if (a.count && b >= *a.count) return;  // uniform per workgroup
  const int lane = threadIdx.x;
  const int nx = a.nx, N = a.N, n = N * NU;
  const int tv = a.tv;
  const bool want_x0 = a.F || a.Phi;
  const bool want_aff = a.f || a.xbar;
  const SLayout L = slayout(NX, NU, N, tv, a.rh, a.f ? 1 : 0, a.xbar ? 1 : 0);
  T* As = sm + L.oA;
  T* Cs = sm + L.oC;
  T* Whs = sm + L.oWh;
  T* Ghs = sm + L.oGh;
  T* Rs = sm + L.oR;
  T* X0s = sm + L.oX0;
  T* Fo = sm + L.oFo;
  T* Xo = sm + L.oXo;
  T* Bs = sm + L.oB;
  T* Qs = sm + L.oQ;
  T* Qfs = sm + L.oQf;
  T* Ws = sm + L.oW;
  T* Es = sm + L.oE;
  T* Is = sm + L.oI;
  T* Zs = sm + L.oZ;
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  stage_in<T, NX>(a, b, lane, want_aff, As, Bs, Cs, Qs, Qfs, Rs, X0s);
  const int pN = N & 1;
  for (int e = lane; e < NX * NX; e += kWave) {
    Ws[pN * NX * NX + e] = Qfs[e];
    Is[e] = (e / NX == e % NX) ? T(1) : T(0);
  }
  if (lane < NX) {
    Es[pN * NX + lane] = T(0);
    Zs[lane] = T(0);
  }
  MPCQP_PHASE(0);

  // ------------------------------------------------------------ backward
  // per-lane item(s): L / y pointers (stage offsets added per stage), e1, base
  constexpr int nW = NX * NX, nE = NX, nH = NU * NX, nG = NU;
  constexpr int nItems = nW + nE + nH + nG;
  constexpr int IPL = (nItems + kWave - 1) / kWave;
  const int sAk = tv ? NX * NX : 0, sBk = tv ? NX * NU : 0;
  int lo[IPL], ls[IPL], lk[IPL], yo[IPL], ys[IPL], yk[IPL], dst[IPL], dpar[IPL], dk[IPL];
  T base[IPL];
  bool act[IPL], e1[IPL];  // e1: the item adds eta_{k+1} (a select, not a product: an
                           // unused eta may hold anything, e.g. without the drift)
#pragma unroll
  for (int it = 0; it < IPL; ++it) {
    const int e = it * kWave + lane;
    act[it] = e < nItems;
    e1[it] = false;
    base[it] = T(0);
    if (e < nW) {  // W_k(r,q)
      const int r = e / NX, q = e % NX;
      lo[it] = L.oA + r; ls[it] = NX; lk[it] = sAk;
      yo[it] = L.oA + q; ys[it] = NX; yk[it] = sAk;
      base[it] = Qs[e];
      dst[it] = L.oW + e; dpar[it] = NX * NX; dk[it] = 0;
    } else if (e < nW + nE) {  // eta_k(r)
      const int r = e - nW;
      lo[it] = L.oA + r; ls[it] = NX; lk[it] = sAk;
      yo[it] = L.oC; ys[it] = 1; yk[it] = NX;
      e1[it] = true;
      dst[it] = L.oE + r; dpar[it] = NX; dk[it] = 0;
    } else if (e < nW + nE + nH) {  // What_k(a,q)
      const int h = e - nW - nE, aa = h / NX, q = h % NX;
      lo[it] = L.oB + aa; ls[it] = NU; lk[it] = sBk;
      yo[it] = L.oI + q * NX; ys[it] = 1; yk[it] = 0;
      dst[it] = L.oWh + h; dpar[it] = 0; dk[it] = NU * NX;
    } else {  // ghat_k(a) (and idle lanes: harmless reads of B, the zeros)
      const int aa = act[it] ? e - nW - nE - nH : 0;
      lo[it] = L.oB + aa; ls[it] = NU; lk[it] = sBk;
      yo[it] = L.oZ; ys[it] = 1; yk[it] = 0;
      e1[it] = true;
      dst[it] = L.oGh + aa; dpar[it] = 0; dk[it] = NU;
    }
  }
  wave_lds_sync();
  for (int k = N - 1; k >= 0; --k) {
    const int p1 = (k + 1) & 1, p0 = k & 1;
    const T* W1 = Ws + p1 * NX * NX;
    const T* E1 = Es + p1 * NX;
#pragma unroll
    for (int it = 0; it < IPL; ++it) {
      const T* Lp = sm + lo[it] + k * lk[it];
      const T* Yp = sm + yo[it] + k * yk[it];
      T y[NX], x[NX];
#pragma unroll
      for (int s2 = 0; s2 < NX; ++s2) y[s2] = Yp[s2 * ys[it]];
#pragma unroll
      for (int p = 0; p < NX; ++p) {
        T acc = e1[it] ? E1[p] : T(0);
#pragma unroll
        for (int s2 = 0; s2 < NX; ++s2) acc = fma(W1[p * NX + s2], y[s2], acc);
        x[p] = acc;
      }
      T out = base[it];
#pragma unroll
      for (int p = 0; p < NX; ++p) out = fma(Lp[p * ls[it]], x[p], out);
      if (act[it]) sm[dst[it] + p0 * dpar[it] + k * dk[it]] = out;
    }
    wave_lds_sync();
  }
  MPCQP_PHASE(1);

  // ------------------------------------------------------------ forward sweep
  const int ncx = n + (want_x0 ? nx : 0);  // z columns, then the x0 columns
  const int col = lane;
  const bool isz = col < n;
  const bool isx0 = !isz && col < ncx;
  const bool isxl = want_aff && col == ncx;  // the affine lane: s = xbar
  const int j = isz ? col / NU : -1;
  const int bc = isz ? col - j * NU : (isx0 ? col - n : 0);
  T bcol[NX];
#pragma unroll
  for (int q = 0; q < NX; ++q) bcol[q] = isz ? Bs[(tv ? j : 0) * NX * NU + q * NU + bc] : T(0);
  T s[NX];
#pragma unroll
  for (int q = 0; q < NX; ++q) s[q] = isx0 ? (q == bc ? T(1) : T(0)) : (isxl ? X0s[q] : T(0));
  T rcol[NU];
#pragma unroll
  for (int aa = 0; aa < NU; ++aa) rcol[aa] = isz ? Rs[aa * NU + bc] : T(0);
  wave_lds_sync();  // B, W, ... dead: the H ring takes over

  T* Hb = a.H + (int64_t)b * ((int64_t)n * (n + 1) / 2);
  T* Fb = a.F ? a.F + (int64_t)b * n * nx : nullptr;
  T* Pb = a.Phi ? a.Phi + (int64_t)b * ((int64_t)N * nx * nx) : nullptr;
  T* Gb = a.Gam ? a.Gam + (int64_t)b * gam_packed_size(nx, NU, N) : nullptr;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int FW = (kWave / 2) * VEC;  // flush window: half a wave of 16-byte stores
  typedef T VT __attribute__((ext_vector_type(VEC)));
  T* RH = sm + L.oRH;
  const int RHM = a.rh - 1;
  const int dh = (int)(((uintptr_t)Hb / sizeof(T)) % VEC);
  T* Hal = Hb - dh;
  const int hiH = dh + n * (n + 1) / 2;
  auto flush = [&](int w) {
    const int p0 = w + lane * VEC;
    if (lane < kWave / 2 && p0 < hiH && p0 + VEC > dh) {
      const VT v = *reinterpret_cast<const VT*>(RH + (p0 & RHM));
      if (p0 >= dh && p0 + VEC <= hiH) {
        __builtin_nontemporal_store(v, reinterpret_cast<VT*>(Hal + p0));
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          if (p0 + e >= dh && p0 + e < hiH) Hal[p0 + e] = v[e];
      }
    }
  };
  // Gamma column vectors: one or more 16-byte stores when nx == NX and the
  // instance's packed block is 16-byte aligned, element stores otherwise
  constexpr int GV = NX * (int)sizeof(T) / 16;
  const bool gvec = Gb && nx == NX && GV >= 1 && (NX * (int)sizeof(T)) % 16 == 0 &&
                    ((uintptr_t)Gb % 16) == 0;
  int fh = 0;
  for (int i = 0; i < N; ++i) {
    const T* Ai = As + (tv ? i : 0) * NX * NX;
    const T* Wh = Whs + i * NU * NX;
    const bool inj = isz && (i == j);
    T t[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      T acc = isxl ? Cs[i * NX + r] : T(0);
#pragma unroll
      for (int q = 0; q < NX; ++q) acc = fma(Ai[r * NX + q], s[q], acc);
      t[r] = acc;
    }
#pragma unroll
    for (int q = 0; q < NX; ++q) s[q] = inj ? bcol[q] : t[q];
    if (Gb && isz && col < (i + 1) * NU) {
      T* g = Gb + gam_packed_off(nx, NU, i) + col * nx;
      if (gvec) {
        typedef T GT __attribute__((ext_vector_type(VEC)));
#pragma unroll
        for (int v = 0; v < GV; ++v) {
          GT gv;
#pragma unroll
          for (int e = 0; e < VEC; ++e) gv[e] = s[v * VEC + e];
          __builtin_nontemporal_store(gv, reinterpret_cast<GT*>(g) + v);
        }
      } else {
#pragma unroll
        for (int q = 0; q < NX; ++q)
          if (q < nx) __builtin_nontemporal_store(s[q], g + q);
      }
    }
    if (Pb && isx0) {
#pragma unroll
      for (int q = 0; q < NX; ++q)
        if (q < nx) Pb[(i * nx + q) * nx + bc] = s[q];
    }
    if (a.xbar && isxl) {
#pragma unroll
      for (int q = 0; q < NX; ++q) Xo[i * NX + q] = s[q];
    }
#pragma unroll
    for (int aa = 0; aa < NU; ++aa) {
      T o = inj ? rcol[aa] : (isxl ? Ghs[i * NU + aa] : T(0));
#pragma unroll
      for (int q = 0; q < NX; ++q) o = fma(Wh[aa * NX + q], s[q], o);
      const int r = i * NU + aa;
      if (isz) {
        if (col <= r) RH[(dh + r * (r + 1) / 2 + col) & RHM] = o;
      } else if (isx0) {
        if (Fb) Fb[r * nx + bc] = o;
      } else if (isxl && a.f) {
        Fo[r] = o;
      }
    }
    const int rr = (i + 1) * NU;
    const int ph = dh + rr * (rr + 1) / 2;
    if (ph - fh >= FW) {
      wave_lds_sync();
      for (; ph - fh >= FW; fh += FW) flush(fh);
      wave_lds_sync();
    }
  }
  wave_lds_sync();
  for (; fh < hiH; fh += FW) flush(fh);
  if (a.f) {
    T* fb = a.f + (int64_t)b * n;
    if (lane < n) fb[lane] = Fo[lane];
  }
  if (a.xbar) {
    T* xb = a.xbar + (int64_t)b * N * nx;
    const float rN = 1.f / (float)nx;
    for (int e = lane; e < N * nx; e += kWave) {
      const int k = qdiv(e, nx, rN), q = e - k * nx;
      xb[e] = Xo[k * NX + q];
    }
  }
  MPCQP_PHASE(2);
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

template <typename T, int NX, int NU>
static int launch_condense_stream(CondenseArgs<T> a, hipStream_t st) {
  constexpr int VEC = 16 / (int)sizeof(T), FW = (kWave / 2) * VEC;
  const int n = a.N * NU;
  int rh = 1;
  while (rh < FW + NU * n + VEC) rh <<= 1;
  a.rh = rh;
  a.rg = 0;
  const size_t bytes =
      (size_t)slayout(NX, NU, a.N, a.tv, rh, a.f ? 1 : 0, a.xbar ? 1 : 0).total * sizeof(T);
  if (bytes > 160 * 1024) return 1;
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)condense_stream_kernel<T, NX, NU>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(condense_stream)");
  }
  hipLaunchKernelGGL((condense_stream_kernel<T, NX, NU>), dim3(a.batch), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("condense_stream_kernel");
  return MPCQP_OK;
}

// The streamed kernel takes every shape whose columns (z, the x0 columns,
// and the affine lane when f or xbar is requested) fit one wavefront, for
// nu in {1, 2, 4} and nx <= 8, Gamma packed or not requested; 1 = not
// applicable (MPCQP_CONDENSE_STREAM=0
// keeps everything on condense_kernel, for A/B checks)
template <typename T, int NX>
static int condense_stream(const CondenseArgs<T>& a, hipStream_t st) {
  static const int enabled = [] {
    const char* e = getenv("MPCQP_CONDENSE_STREAM");
    return e ? atoi(e) : 1;
  }();
  const int n = a.N * a.nu;
  const int lanes = n + ((a.F || a.Phi) ? a.nx : 0) + ((a.f || a.xbar) ? 1 : 0);
  // (a dense Gamma, structural zeros included, stays on condense_kernel's ring)
  if (!enabled || NX > 8 || lanes > kWave || (a.Gam && !a.gpk)) return 1;
  if (a.nu == 1) return launch_condense_stream<T, NX, 1>(a, st);
  if (a.nu == 2) return launch_condense_stream<T, NX, 2>(a, st);
  if (a.nu == 4) return launch_condense_stream<T, NX, 4>(a, st);
  return 1;
}

template <typename T, int NX>
static int launch_condense(CondenseArgs<T> a, hipStream_t st) {
  if constexpr (NX <= 8) {
    const int rc = condense_stream<T, NX>(a, st);
    if (rc != 1) return rc;
  }
  // streamed sweep when every column fits one wavefront (MPCQP_CONDENSE_RING=0: direct stores)
  static const int ring_on = [] {
    const char* e = getenv("MPCQP_CONDENSE_RING");
    return e ? atoi(e) : 1;
  }();
  const int n = a.N * a.nu, ncol = n + ((a.F || a.Phi) ? a.nx : 0);
  a.rh = a.rg = 0;
  if (ring_on && ncol <= kWave) {
    constexpr int VEC = 16 / (int)sizeof(T), CH = kWave * VEC;
    auto pow2 = [](int v) {
      int p = 1;
      while (p < v) p <<= 1;
      return p;
    };
    a.rh = pow2(CH + a.nu * n + VEC);
    a.rg = a.Gam ? pow2(CH + a.nx * n + VEC) : 0;
    if ((size_t)clayout(NX, a.nu, a.N, a.tv, a.rh, a.rg).total * sizeof(T) > 160 * 1024) a.rh = a.rg = 0;
  }
  const CLayout L = clayout(NX, a.nu, a.N, a.tv, a.rh, a.rg);
  const size_t bytes = (size_t)L.total * sizeof(T);
  if (bytes > 160 * 1024) {
    set_error("mpcqp_condense: per-instance LDS footprint %zu B exceeds 160 KiB (N too large)", bytes);
    return MPCQP_ENOTSUP;
  }
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)condense_kernel<T, NX>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(condense)");
  }
  hipLaunchKernelGGL((condense_kernel<T, NX>), dim3(a.batch), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("condense_kernel");
  return MPCQP_OK;
}

// ===================================================================== MFMA path
// condense_mfma_kernel (fp32, 5 <= nx <= 15): the same recursions as
// condense_kernel, on v_mfma_f32_16x16x4_f32 with the state padded to 16 and
// slot 15 carrying the affine part (augmented state x~ = [x; 1]):
//     A~_k = [[A_k, c_k], [0, 1]],  Q~ = diag(Q, 0),  B~_k = [B_k; 0]
//     W~_N = Qf~,  W~_k = Q~ + A~_k' W~_{k+1} A~_k = [[W_k, eta_k], [eta_k', *]]
//     What_k = B~_k' W~_{k+1}                      (nu x 16, kept in LDS)
// so that the forward sweep over Gamma~_{k+1} = A~_k Gamma~_k (+ B_k in block
// k) and E_{k+1} = A~_k E_k, E_0 = [[I, x0], [0, 1]] (E = [Phi, xbar]) yields
//     H row block k   = What_k Gamma~_{k+1}   (+ R on the diagonal block)
//     [F | f] block k = What_k E_{k+1}        (column 15: f = B_k'(W x + eta) = B_k' y)
// i.e. f, F, Phi and xbar come out of one extra 16-column tile, drift
// included, with no separate adjoint chain.
//
// Layout: one instance per wavefront.  Every 16 x 16 operand is an MFMA tile
// held in C layout (lane (g, c): rows 4g..4g+3 of column c), and every
// product is written as mfma4(P, Y) = P'Y (mfma.hpp: the K index of chunk s
// in lane group g is 4g + s): W~A~ = W~'A~ (W~ symmetric), A~'X, B~'W~, and
// A~ Gamma~ with A~' loaded in C layout.  An MFMA result is then the next
// product's operand as it stands -- no transpose on the recursion (round 3
// moved every C tile to a B layout by a 4 x 4 permlane transpose: two per
// backward stage, one per Gamma tile and stage).  The Gamma block row lives
// in registers as NT C-layout tiles.  The What_k Gamma~ product (nu <= 16
// rows) runs on the VALU from the C tile: 16 FMAs per 4 output rows plus the
// same transpose as a cross-group reduction, which leaves output row g of
// column c in lane (g, c), so each H row segment is one 64-lane store.
// NT: Gamma tiles (n <= 16 NT); NU4: What rows held per lane (nu <= NU4);
// DRIFT: per-stage c_k present (its loads get their own queue)
//
// State slots: tile position pos = 4g + s holds state cm_state(pos) -- states
// 0..11 in registers s = 0..2, states 12..14 and the affine slot in register
// s = 3 of the four lane groups.  For nx <= 12 the K chunk s = 3 of Gamma~
// (states 12..14 and the affine row, all zero in Gamma~) is then empty, and
// the forward product A~ Gamma~ -- three quarters of the kernel's MFMA work --
// runs three of the four 16x16x4 instructions.
__device__ __forceinline__ int cm_state(int pos) {
  const int g = pos >> 2, s = pos & 3;
  return s < 3 ? 3 * g + s : (g < 3 ? 12 + g : 15);
}
template <int NT, int NU4, bool DRIFT, bool P12>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
void condense_mfma_kernel(CondenseArgs<float> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* wh = reinterpret_cast<float*>(smem_raw);  // What_k: N x NU4 x 16
  float* Rs = wh + a.N * NU4 * 16;                 // R: nu x nu
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  const int b = blockIdx.x;
  const int l = threadIdx.x, g = l >> 4, cl = l & 15;
  const int nx = a.nx, nu = a.nu, N = a.N, n = N * nu;
  const int64_t sa = a.tv ? (int64_t)nx * nx : 0, sbk = a.tv ? (int64_t)nx * nu : 0;
  const float* Ab = a.A + (int64_t)b * a.sA;
  const float* Bb = a.B + (int64_t)b * a.sB;
  const float* Cb = DRIFT ? a.c + (int64_t)b * a.sC : nullptr;
  {
    const float* Rb = a.R + (int64_t)b * a.sR;
    for (int e = l; e < nu * nu; e += kWave) Rs[e] = Rb[e];
  }
  // Operand loads run PF stages ahead through a register queue (shifted by
  // one slot per stage): one stage of the serial chain is a few hundred
  // cycles, an HBM miss several thousand.
  constexpr int PF = 4;
  // A~[p][q] = A[p][q] (p,q < nx) | c[p] (q = 15) | 1 (p = q = 15) | 0: the A and
  // c loads return 0 outside their masks, so A~ = rawA + rawC + one.
  int oAb[4], oCb[4], oBb[4], oAf[4], oCf[4];
  float one_b[4], one_f[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int p = 4 * g + s;  // C layout: register s of lane (g, cl) is row 4g+s, column cl
    const int sp = cm_state(p), sc = cm_state(cl);
    oAb[s] = (sp < nx && sc < nx) ? 4 * (sp * nx + sc) : kOOB;
    oCb[s] = (sp < nx && cl == 15) ? 4 * sp : kOOB;
    oBb[s] = (sp < nx && cl < nu) ? 4 * (sp * nu + cl) : kOOB;
    one_b[s] = (p == 15 && cl == 15) ? 1.f : 0.f;
    oAf[s] = (sc < nx && sp < nx) ? 4 * (sc * nx + sp) : kOOB;  // forward: row cl, column p
    oCf[s] = (sc < nx && p == 15) ? 4 * sc : kOOB;
    one_f[s] = (cl == 15 && p == 15) ? 1.f : 0.f;
  }
  auto stage_rsrc = [&](int k, rsrc_t& ra, rsrc_t& rb, rsrc_t& rc) {
    ra = mk_rsrc(Ab + k * sa, (int64_t)nx * nx * 4);
    rb = mk_rsrc(Bb + k * sbk, (int64_t)nx * nu * 4);
    rc = mk_rsrc(Cb ? Cb + (int64_t)k * nx : Ab, Cb ? (int64_t)nx * 4 : 0);
  };

  // ------------------------------------------------ backward: W~, What
  float wB[4], qC[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int sp = cm_state(4 * g + s), sc = cm_state(cl);
    wB[s] = (sp < nx && sc < nx) ? a.Qf[(int64_t)b * a.sQf + sp * nx + sc] : 0.f;
    qC[s] = (sp < nx && sc < nx) ? a.Q[(int64_t)b * a.sQ + sp * nx + sc] : 0.f;
  }
  auto load_bw = [&](int k, float (&ao)[4], float (&co)[4], float (&bo)[4]) {
    (void)co;
    rsrc_t ra, rb, rc;
    stage_rsrc(k, ra, rb, rc);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ao[s] = bld(ra, oAb[s]);
      if constexpr (DRIFT) co[s] = bld(rc, oCb[s]);
      bo[s] = bld(rb, oBb[s]);
    }
  };
  // stage body: consume slot (loaded PF stages earlier), refill it with
  // stage k - PF, run the stage.  The loop is unrolled by PF so every slot
  // is a fixed register set (moving a slot would wait on its load).
  auto bw_stage = [&](int k, float (&sa_)[4], float (&sc_)[4], float (&sb_)[4]) {
    float aT[4], bT[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      aT[s] = sa_[s] + one_b[s];
      if constexpr (DRIFT) aT[s] += sc_[s];
      bT[s] = sb_[s];
    }
    // unconditional refill (clamped stage): no phi ever touches a slot
    load_bw(k - PF >= 0 ? (k - PF < N ? k - PF : N - 1) : 0, sa_, sc_, sb_);
    if (k >= N) return;  // alignment padding
    // What_k = B~_k' W~_{k+1}: rows 4g+j < nu of lane (g, cl)
    const mf4 w = mfma4(bT, wB, mf4{0.f, 0.f, 0.f, 0.f});
    if (k >= 1) {
      const mf4 x = mfma4(wB, aT, mf4{0.f, 0.f, 0.f, 0.f});  // X = W~' A~ = W~ A~
      const float xv[4] = {x[0], x[1], x[2], x[3]};
      const mf4 w2 = mfma4(aT, xv, mf4{qC[0], qC[1], qC[2], qC[3]});  // Q~ + A~' X
#pragma unroll
      for (int s = 0; s < 4; ++s) wB[s] = w2[s];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * g + j;
      if (i < NU4) wh[(k * NU4 + i) * 16 + cl] = (i < nu) ? w[j] : 0.f;
    }
  };
  float qa[PF][4], qb[PF][4], qc[PF][4];
  // stages kt = N-1+pad .. 0 with pad so that the count is a multiple of PF
  const int ktop = N - 1 + (PF - N % PF) % PF;
#pragma unroll
  for (int d = 0; d < PF; ++d) {
    const int k = ktop - d;
    load_bw(k < N ? (k >= 0 ? k : 0) : N - 1, qa[d], qc[d], qb[d]);
  }
  for (int k0 = ktop; k0 >= 0; k0 -= PF) {
#pragma unroll
    for (int d = 0; d < PF; ++d) bw_stage(k0 - d, qa[d], qc[d], qb[d]);
  }
  __syncthreads();
  MPCQP_PHASE(0);

  // ------------------------------------------------ forward: Gamma~, E
  const bool wantE = a.f || a.F || a.Phi || a.xbar;
  const bool wantFf = a.f || a.F;
  const rsrc_t rH = mk_rsrc(a.H + (int64_t)b * ((int64_t)n * (n + 1) / 2), (int64_t)n * (n + 1) / 2 * 4);
  const rsrc_t rG = mk_rsrc(a.Gam ? a.Gam + (int64_t)b * ((int64_t)N * nx * n) : a.H,
                            a.Gam ? (int64_t)N * nx * n * 4 : 0);
  const rsrc_t rF = mk_rsrc(a.F ? a.F + (int64_t)b * n * nx : a.H, a.F ? (int64_t)n * nx * 4 : 0);
  const rsrc_t rf = mk_rsrc(a.f ? a.f + (int64_t)b * n : a.H, a.f ? (int64_t)n * 4 : 0);
  const rsrc_t rP = mk_rsrc(a.Phi ? a.Phi + (int64_t)b * N * nx * nx : a.H, a.Phi ? (int64_t)N * nx * nx * 4 : 0);
  const rsrc_t rX = mk_rsrc(a.xbar ? a.xbar + (int64_t)b * N * nx : a.H, a.xbar ? (int64_t)N * nx * 4 : 0);
  float gB[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) gB[t][s] = 0.f;
  float eB[4];
  {
    const float* X0b = a.x0 ? a.x0 + (int64_t)b * a.sX0 : nullptr;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int p = 4 * g + s, sp = cm_state(p), sc = cm_state(cl);
      float v = 0.f;
      if (sp < nx && sc < nx) v = (p == cl) ? 1.f : 0.f;
      else if (cl == 15) v = (sp < nx) ? (X0b ? X0b[sp] : 0.f) : (p == 15 ? 1.f : 0.f);
      eB[s] = v;
    }
  }
  // A~_r as A operand (lane: row cl, column 4s+g); B_r rows 4g+j at this
  // lane's column of block r
  auto load_fw = [&](int r, float (&ao)[4], float (&co)[4], float (&bo)[4]) {
    (void)co;
    rsrc_t ra, rb, rc;
    stage_rsrc(r, ra, rb, rc);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ao[s] = bld(ra, oAf[s]);
      if constexpr (DRIFT) co[s] = bld(rc, oCf[s]);
    }
    const int q = (cl - r * nu) & 15;  // this lane's column offset in block r (mod 16)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sp = cm_state(4 * g + j);
      bo[j] = bld(rb, (sp < nx && q < nu) ? 4 * (sp * nu + q) : kOOB);
    }
  };
  constexpr int PFF = 3;  // forward prefetch depth (1: +6 %, 2: +1.6 % time at config 5)
  auto fw_stage = [&](int r, float (&sa_)[4], float (&sc_)[4], float (&sb_)[4]) {
    float aA[4], bI[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      aA[s] = sa_[s] + one_f[s];
      if constexpr (DRIFT) aA[s] += sc_[s];
      bI[s] = sb_[s];
    }
    load_fw(r + PFF < N ? r + PFF : N - 1, sa_, sc_, sb_);
    if (r >= N) return;  // alignment padding
    float wv[NU4][4];
#pragma unroll
    for (int i = 0; i < NU4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) wv[i][j] = wh[(r * NU4 + i) * 16 + 4 * g + j];
    const int blk0 = r * nu;
    const int ntact = ((r + 1) * nu + 15) >> 4;
    MPCQP_PHASE(1);
    // all MFMA chains first (independent tiles overlap in the matrix pipe),
    // then the VALU epilogue per tile
    if constexpr (P12) {  // nx <= 12: K chunk 3 of Gamma~ is empty (cm_state)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (t < ntact) {
          mf4 dd = mf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 3; ++s) dd = __builtin_amdgcn_mfma_f32_16x16x4f32(aA[s], gB[t][s], dd, 0, 0, 0);
#pragma unroll
          for (int s = 0; s < 4; ++s) gB[t][s] = dd[s];
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (t < ntact) {
          const mf4 dd = mfma4(aA, gB[t], mf4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int s = 0; s < 4; ++s) gB[t][s] = dd[s];
        }
      }
    }
    float eC[4];
    if (wantE) {
      const mf4 dd = mfma4(aA, eB, mf4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int s = 0; s < 4; ++s) eC[s] = dd[s];
    }
#ifdef MPCQP_PHASE_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n v_mov_b32 %0, %0" : "+v"(gB[0][0]));
#endif
    MPCQP_PHASE(2);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = 16 * t + cl;
      if (t < ntact) {
        float(&d)[4] = gB[t];  // Gamma~_{r+1} tile, C layout
        const bool inblk = col >= blk0 && col < blk0 + nu;
#pragma unroll
        for (int j = 0; j < (P12 ? 3 : 4); ++j) d[j] = inblk ? bI[j] : d[j];
        if (a.Gam) {
#pragma unroll
          for (int j = 0; j < (P12 ? 3 : 4); ++j) {
            const int sp = cm_state(4 * g + j);
            bst(d[j], rG, (sp < nx && col < n) ? 4 * ((r * nx + sp) * n + col) : kOOB);
          }
        }
#pragma unroll
        for (int ic = 0; ic < NU4 / 4; ++ic) {
          float P[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float acc = 0.f;
#pragma unroll
            for (int j = 0; j < (P12 ? 3 : 4); ++j) acc = fmaf(wv[4 * ic + i][j], d[j], acc);
            P[i] = acc;
          }
          xpose4(P);
          float h = (P[0] + P[1]) + (P[2] + P[3]);
          const int i = 4 * ic + g;
          const int R = blk0 + i;
          const bool st = i < nu && col <= R;
          if (inblk && i < nu) h += Rs[i * nu + (col - blk0)];
          bst(h, rH, st ? 4 * (R * (R + 1) / 2 + col) : kOOB);
        }
      } else if (a.Gam && 16 * t < n) {  // structural zeros of the block row
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sp = cm_state(4 * g + j);
          bst(0.f, rG, (sp < nx && col < n) ? 4 * ((r * nx + sp) * n + col) : kOOB);
        }
      }
    }
    MPCQP_PHASE(3);
    if (wantE) {
      float(&d)[4] = eC;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int sp = cm_state(4 * g + j), sc = cm_state(cl);
        if (a.xbar) bst(d[j], rX, (sp < nx && cl == 15) ? 4 * (r * nx + sp) : kOOB);
        if (a.Phi) bst(d[j], rP, (sp < nx && sc < nx) ? 4 * ((r * nx + sp) * nx + sc) : kOOB);
      }
      if (wantFf) {
#pragma unroll
        for (int ic = 0; ic < NU4 / 4; ++ic) {
          float P[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float acc = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) acc = fmaf(wv[4 * ic + i][j], d[j], acc);
            P[i] = acc;
          }
          xpose4(P);
          const float h = (P[0] + P[1]) + (P[2] + P[3]);
          const int i = 4 * ic + g;
          const int R = blk0 + i;
          if (a.F) bst(h, rF, (i < nu && cm_state(cl) < nx) ? 4 * (R * nx + cm_state(cl)) : kOOB);
          if (a.f) bst(h, rf, (i < nu && cl == 15) ? 4 * R : kOOB);
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) eB[s] = d[s];
    }
    MPCQP_PHASE(4);
  };
#pragma unroll
  for (int d = 0; d < PFF; ++d) load_fw(d < N ? d : N - 1, qa[d], qc[d], qb[d]);
  for (int r0 = 0; r0 < N; r0 += PFF) {
#pragma unroll
    for (int d = 0; d < PFF; ++d) fw_stage(r0 + d, qa[d], qc[d], qb[d]);
  }
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

// ------------------------------------------------------- fused-H MFMA path
// condense_mfma_fh_kernel<NT> (fp32, 5 <= nx <= 12, nu <= 4, no drift, no
// F / Phi): the
// H rows come out of the forward MFMA itself.  With nx <= 12 the state slots
// 12..14 and the affine slot (tile positions 3, 7, 11, 15 = register 3 of
// every lane group, cm_state) carry nothing in Gamma~ or Phi, so the four
// output rows at those positions are free: the forward A operand gets
// (What_r A_r)[a, :] in the lanes of output row 4a + 3, and
//     D = [A_r; What_r A_r] Gamma~_r
// gives Gamma~_{r+1} (registers 0..2, before the injection of B_r) AND the
// H rows of block r (register 3: What_r A_r Gamma~_r = What_r Gamma~_{r+1}
// off the diagonal block) in the same three 16x16x4 MFMAs; f and xbar come
// from a VALU mat-vec of the same A operand.  No VALU epilogue, no What_k in
// LDS.
// The backward pass gets What_k A_k and the diagonal block What_k B_k from
// its own recursion: with Z_k = A~_k whose unused columns (positions 4b + 3)
// hold B_k[:, b],
//     X = W~_{k+1} Z_k,   Y = Q~ + Z_k' X,
// Y's state block is W~_k, its row 4b + 3 is (B_k' W~_{k+1} A_k)[b, :] =
// (What_k A_k)[b, :] and its entry (4b + 3, 4c + 3) is (What_k B_k)[b, c] --
// six MFMAs per stage (three K chunks each: state slots only) for what took
// twelve (X, W~, What).  LDS per instance: (What A)_k (4 x 12) and
// What_k B_k + R (4 x 4) per stage, the footprint What had.
#ifndef MPCQP_FH_PF
#define MPCQP_FH_PF 4   // backward prefetch depth (stages; 8 measured 0.6 % slower, 10 and 20 slower still)
#endif
#ifndef MPCQP_FH_PFF
#define MPCQP_FH_PFF 4  // forward prefetch depth (stages)
#endif
__device__ __forceinline__ mf4 mfma3(const float* a, const float* b, mf4 acc) {
#pragma unroll
  for (int s = 0; s < 3; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
  return acc;
}
template <int NT, bool EXACT, bool X3, bool GAM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void condense_mfma_fh_kernel(CondenseArgs<float> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* whA = reinterpret_cast<float*>(smem_raw);  // (What_k A_k)[b][state]: N x 4 x 12
  float* dgs = whA + a.N * 48;                      // What_k B_k + R: N x 4 x 4
  // (exactly 256 floats per stage: 10 KB at N = 40, four waves per SIMD)
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  const int b = blockIdx.x;
  const int l = threadIdx.x, g = l >> 4, cl = l & 15;
  const int nx = a.nx, nu = a.nu, N = a.N, n = N * nu;
  const int64_t sa = a.tv ? (int64_t)nx * nx : 0, sbk = a.tv ? (int64_t)nx * nu : 0;
  const float* Ab = a.A + (int64_t)b * a.sA;
  const float* Bb = a.B + (int64_t)b * a.sB;
  // position cl: a state column (zc false, state sc) or input column zb of
  // Z (backward) / H row zb of the forward A operand (zc true)
  const bool zc = (cl & 3) == 3;
  const int zb = cl >> 2;
  const int sc = cm_state(cl);
  // R[g][zb]: what this lane adds to its entry of What_k B_k
  const float rgz = (zc && g < nu && zb < nu) ? a.R[(int64_t)b * a.sR + g * nu + zb] : 0.f;
  // backward prefetch depth (stages): a stage is a few hundred cycles of
  // MFMA chain, an HBM miss under load several thousand
  constexpr int PF = MPCQP_FH_PF;
  // Memory instructions, not bytes, bound this kernel's loads (dword gathers
  // of 64 lanes): one load per operand register and stage.  Backward: Z's
  // column of this lane comes from A (state column sc, stride nx) or from B
  // (input column zb, stride nu) through a per-lane pointer; a lane outside
  // both reads A's first element and is masked to 0.
  const bool zv = (zc ? (zb < nu) : (sc < nx)) && 3 * g < nx;  // (rows past nx: never read)
  const float* zp = !zv ? Ab : (zc ? Bb + zb + 3 * g * nu : Ab + sc + 3 * g * nx);
  const int zstep = !zv ? 0 : (zc ? nu : nx);
  const int zstage = !zv ? 0 : (int)(zc ? sbk : sa);  // in-instance offsets: 32-bit
  float zm[3];
  int zo[3];  // element offsets (a row past nx re-reads row 3g: never out of bounds)
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    zm[s] = (zv && 3 * g + s < nx) ? 1.f : 0.f;
    zo[s] = (zv && 3 * g + s < nx) ? s * zstep : 0;
  }

  // ------------------------------------------------ backward
  float wB[3], qC[4];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int sp = 3 * g + s;
    wB[s] = (sp < nx && sc < nx) ? a.Qf[(int64_t)b * a.sQf + sp * nx + sc] : 0.f;
    qC[s] = (sp < nx && sc < nx) ? a.Q[(int64_t)b * a.sQ + sp * nx + sc] : 0.f;
  }
  qC[3] = 0.f;
  auto load_bw = [&](int k, float (&za)[3]) {
    const float* p = zp + k * zstage;
#pragma unroll
    for (int s = 0; s < 3; ++s) za[s] = p[zo[s]];
  };
  auto bw_stage = [&](int k, float (&za)[3]) {
    const float z[3] = {za[0] * zm[0], za[1] * zm[1], za[2] * zm[2]};
    // the slot is consumed before its refill is issued: otherwise the
    // scheduler hoists the refill above the consumption, the refill needs
    // fresh registers and the loop's back edge copies them into the slot --
    // a wait on every outstanding load once per PF stages
    __builtin_amdgcn_sched_barrier(0);
    load_bw(k - PF >= 0 ? (k - PF < N ? k - PF : N - 1) : 0, za);
    // alignment padding (k >= N, the first stages when N % PF != 0) runs
    // without effect instead of branching around: a branch here makes the
    // queue slots loop-carried through copies again
    const bool live = EXACT || k < N;
    const mf4 X = mfma3(wB, z, mf4{0.f, 0.f, 0.f, 0.f});  // W~ Z (W~ symmetric)
    const float xv[3] = {X[0], X[1], X[2]};
    const mf4 Y = mfma3(z, xv, mf4{qC[0], qC[1], qC[2], qC[3]});  // Q~ + Z' W~ Z
    if (live && g < nu) {
      if (!zc) whA[(k * 4 + g) * 12 + sc] = Y[3];
      else if (zb < nu) dgs[(k * 4 + g) * 4 + zb] = Y[3] + rgz;
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) wB[s] = live ? (zc ? 0.f : Y[s]) : wB[s];
  };
  float qz[PF][3];
  const int ktop = N - 1 + (PF - N % PF) % PF;
#pragma unroll
  for (int d = 0; d < PF; ++d) {
    const int k = ktop - d;
    load_bw(k < N ? (k >= 0 ? k : 0) : N - 1, qz[d]);
  }
  for (int k0 = ktop; k0 >= 0; k0 -= PF) {
#pragma unroll
    for (int d = 0; d < PF; ++d) bw_stage(k0 - d, qz[d]);
  }
  wave_lds_sync();
  MPCQP_PHASE(0);
#ifdef MPCQP_FH_NOFW  // (timing probe: the backward pass alone)
  if (whA[0] == 12345.f) a.H[b] = whA[l];
  return;
#endif

  // ------------------------------------------------ forward
  // f and xbar (no F, no Phi: those calls take condense_mfma_kernel) need
  // one x0 column, not an E tile of three more MFMAs per stage:
  // xbar_{r+1} = A_r xbar_r and f_r = (What A)_r xbar_r are the same mat-vec
  // of this lane's A operand (state rows / H rows), done on the VALU (three
  // FMAs, a sum over the four lane groups, a within-row gather for the next
  // stage), off the MFMA chain.
#ifndef MPCQP_FH_NOE
  const bool wantX = a.f || a.xbar;
#else  // (timing probe: no x0 column at all)
  const bool wantX = false;
#endif
  const rsrc_t rH = mk_rsrc(a.H + (int64_t)b * ((int64_t)n * (n + 1) / 2), (int64_t)n * (n + 1) / 2 * 4);
  // dense Gamma (GAM: tests and callers that ask for it; mpcqp_mpc_qp does not)
  auto rG = [&]() {
    return mk_rsrc(a.Gam + (int64_t)b * ((int64_t)N * nx * n), (int64_t)N * nx * n * 4);
  };
  // (an output not asked for gets a zero-size descriptor: its stores drop)
  const rsrc_t rf = mk_rsrc(a.f ? a.f + (int64_t)b * n : a.H, a.f ? (int64_t)n * 4 : 0);
  const rsrc_t rX = mk_rsrc(a.xbar ? a.xbar + (int64_t)b * N * nx : a.H, a.xbar ? (int64_t)N * nx * 4 : 0);
  float gB[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) gB[t][s] = 0.f;
  // xbar_r, states 3g..3g+2 (xbar_0 = x0), and the ds_bpermute address of
  // tile position 4g (state 3g) in this lane's row (+4 s: state 3g + s)
  float xv[3];
  const int xsrc = 4 * (16 * g + 4 * g);
  // f_r[zb] (H-row lanes of group 0) at blk0 + zb: the per-lane byte base
  // (kOOB elsewhere); xbar_{r+1}[sc] (state lanes of group 0) at r nx + sc
  const int fo = (g == 0 && zc && zb < nu) ? 4 * zb : kOOB;
  {
    const float* X0b = a.x0 ? a.x0 + (int64_t)b * a.sX0 : nullptr;
#pragma unroll
    for (int s = 0; s < 3; ++s) xv[s] = (3 * g + s < nx && X0b) ? X0b[3 * g + s] : 0.f;
  }
  // Forward: the A operand of a state lane is row sc of A_r, columns 3g..3g+2
  // -- contiguous, one 12-byte load when nx % 3 == 0 (X3) -- and, in K chunk
  // 3 (the input selectors, below), B_r[sc][g]: two loads per stage.  The H
  // lanes (zc) take (What A)_r and What_r B_r + R from LDS.  Invalid lanes
  // read A's first element and are masked.
  const bool av = !zc && sc < nx && 3 * g < nx;
  const float* ap = av ? Ab + sc * nx + 3 * g : Ab;
  const int astage = av ? (int)sa : 0;
  float am[3];
  int ao_[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    am[s] = (av && 3 * g + s < nx) ? 1.f : 0.f;
    ao_[s] = (av && 3 * g + s < nx) ? s : 0;
  }
  const bool bv = !zc && sc < nx && g < nu;
  const float* bp = bv ? Bb + sc * nu + g : Ab;
  const int bstage = bv ? (int)sbk : 0;
  const float bm = bv ? 1.f : 0.f;
  const int zbr = zb < nu ? zb : 0, gr = g < nu ? g : 0;  // clamped LDS rows (written ones)
  const float wm = (zc && zb < nu) ? 1.f : 0.f;
  const float dm = (zc && zb < nu && g < nu) ? 1.f : 0.f;
  auto load_fw = [&](int r, float (&ao)[3], float& bo) {
    const float* p = ap + r * astage;
    if constexpr (X3) {
      // exactly 12 bytes (global_load_dwordx3, 4-byte aligned): a vec3 type
      // would be a 16-byte vector in the IR, one float past A's last row
      struct F3 { float v[3]; } t;
      __builtin_memcpy(&t, p, sizeof(F3));
      ao[0] = t.v[0];
      ao[1] = t.v[1];
      ao[2] = t.v[2];
    } else {
#pragma unroll
      for (int s = 0; s < 3; ++s) ao[s] = p[ao_[s]];
    }
    bo = bp[r * bstage];
  };
  constexpr int PFF = MPCQP_FH_PFF;  // forward prefetch depth
  auto fw_stage = [&](int r, float (&qa_)[3], float& qb_) {
    float aA[4];
    const int rr = r < N ? r : 0;
    const float* wa = whA + (rr * 4 + zbr) * 12 + 3 * g;
    const float dv = dgs[(rr * 4 + zbr) * 4 + gr];
    // zc lanes: (What A)_r and What_r B_r + R from LDS; the others: A_r and
    // B_r from their queue slot.  Masked arithmetic, not selects: a select on
    // a load is turned into a masked load INTO the queue slot, whose refill
    // then needs fresh registers (copies and a wait at the loop's back edge)
#pragma unroll
    for (int s = 0; s < 3; ++s) aA[s] = fmaf(wa[s], wm, qa_[s] * am[s]);
    aA[3] = fmaf(dv, dm, qb_ * bm);
    // the slot is refilled at the END of the stage, once aA (its values) is
    // dead: a refill issued while they are live needs fresh
    // registers, which the loop's back edge copies back into the slot -- a
    // wait on every outstanding load once per PFF stages
    const int rnext = r + PFF < N ? r + PFF : N - 1;
    if (!EXACT && r >= N) {  // alignment padding (EXACT: N % PFF == 0)
      load_fw(rnext, qa_, qb_);
      return;
    }
    const int blk0 = r * nu;
    const int ntact = ((r + 1) * nu + 15) >> 4;
    const int tlo = blk0 >> 4;  // tiles holding block r's columns: tlo..ntact-1
    auto xchain = [&]() __attribute__((always_inline)) {
      if (wantX) {
        // position cl of the sum: xbar_{r+1}[sc] (state lanes), f_r[zb] (H rows)
        float px = fmaf(aA[2], xv[2], fmaf(aA[1], xv[1], aA[0] * xv[0]));
        // sum over the four lane groups: permlane16_swap of (v, v) leaves rows
        // (0, 1) and (2, 3) of the two results holding (v.r0, v.r1) and
        // (v.r2, v.r3) in some order, so their sum is the pair sum in every
        // lane without a select; permlane32_swap then pairs the row pairs
        {
          const auto s1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(px), __float_as_uint(px), false, false);
          px = __uint_as_float(s1[0]) + __uint_as_float(s1[1]);
          const auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(px), __float_as_uint(px), false, false);
          px = __uint_as_float(s2[0]) + __uint_as_float(s2[1]);
        }
        bst(px, rf, fo, 4 * blk0);
        if (a.xbar)  // (mpcqp_mpc_qp asks for none)
          bst(px, rX, (g == 0 && !zc && sc < nx) ? 4 * sc : kOOB, 4 * r * nx);
        int xs = xsrc;
        asm volatile("" : "+v"(xs));  // (the three addresses are formed here, not held)
#pragma unroll
        for (int s = 0; s < 3; ++s)
          xv[s] = __int_as_float(__builtin_amdgcn_ds_bpermute(xs + 4 * s, __float_as_int(px)));
      }
    };
#ifdef MPCQP_FH_XFIRST
    xchain();
#endif
    MPCQP_PHASE(1);
    // K chunk 3 carries the input selectors on the tiles of block r: row
    // 4b + 3 of Gamma~_r is 1 in block r's column b, and the A operand's
    // chunk 3 is B_r (state rows) / What_r B_r + R (H rows), so the MFMA
    // injects B_r into Gamma~_{r+1} and writes the diagonal block of H
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t < ntact) {
        mf4 dd;
        if (t >= tlo) {
          const int col = 16 * t + cl;
          gB[t][3] = (g < nu && col == blk0 + g) ? 1.f : 0.f;
          dd = mfma4(aA, gB[t], mf4{0.f, 0.f, 0.f, 0.f});
        } else {
          dd = mfma3(aA, gB[t], mf4{0.f, 0.f, 0.f, 0.f});
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) gB[t][s] = dd[s];
      }
    }
#ifndef MPCQP_FH_XFIRST
    xchain();
#endif
    MPCQP_PHASE(2);
    const int R = blk0 + g;  // the H row of this lane's register 3
    // packed row R from column cl; tile t adds the immediate 64 t.  Tiles
    // before tlo lie below the diagonal block (every column valid)
    const int rowb = g < nu ? 4 * ((R * (R + 1) >> 1) + cl) : kOOB;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = 16 * t + cl;
      if (t < ntact) {
        const float(&d)[4] = gB[t];
        if constexpr (GAM) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const int sp = 3 * g + j;
            bst(d[j], rG(), (sp < nx && col < n) ? 4 * ((r * nx + sp) * n + col) : kOOB);
          }
        }
#ifndef MPCQP_FH_NOSTORE
        // the tile's displacement 64 t rides in the store's SGPR offset
        if (t < tlo)  // (a uniform branch: no per-lane test below the diagonal)
          bst(d[3], rH, rowb, 64 * t);
        else
          bst(d[3], rH, col <= R ? rowb : kOOB, 64 * t);
#else
        if (d[3] == 12345.f) bst(d[3], rH, 0);
#endif
      } else if (GAM && 16 * t < n) {  // structural zeros of the block row
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int sp = 3 * g + j;
          bst(0.f, rG(), (sp < nx && col < n) ? 4 * ((r * nx + sp) * n + col) : kOOB);
        }
      }
    }
    MPCQP_PHASE(3);
    __builtin_amdgcn_sched_barrier(0);
    load_fw(rnext, qa_, qb_);
    MPCQP_PHASE(4);
  };
  float qa[PFF][3], qb[PFF];
#pragma unroll
  for (int d = 0; d < PFF; ++d) load_fw(d < N ? d : N - 1, qa[d], qb[d]);
  for (int r0 = 0; r0 < N; r0 += PFF) {
#pragma unroll
    for (int d = 0; d < PFF; ++d) fw_stage(r0 + d, qa[d], qb[d]);
  }
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

template <int NT, bool EXACT, bool X3, bool GAM = false>
static int launch_condense_mfma_fh3(const CondenseArgs<float>& a, hipStream_t st) {
  const size_t bytes = (size_t)a.N * 64 * sizeof(float);
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)condense_mfma_fh_kernel<NT, EXACT, X3, GAM>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(condense_mfma_fh)");
  }
  hipLaunchKernelGGL((condense_mfma_fh_kernel<NT, EXACT, X3, GAM>), dim3(a.batch), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("condense_mfma_fh_kernel");
  return MPCQP_OK;
}
template <int NT, bool EXACT>
static int launch_condense_mfma_fh2(const CondenseArgs<float>& a, hipStream_t st) {
  return a.nx % 3 == 0 ? launch_condense_mfma_fh3<NT, EXACT, true>(a, st)
                       : launch_condense_mfma_fh3<NT, EXACT, false>(a, st);
}
template <int NT>
static int launch_condense_mfma_fh(const CondenseArgs<float>& a, hipStream_t st) {
  if (a.Gam) return launch_condense_mfma_fh3<NT, false, false, true>(a, st);  // (generic)
  return (a.N % MPCQP_FH_PF == 0 && a.N % MPCQP_FH_PFF == 0) ? launch_condense_mfma_fh2<NT, true>(a, st)
                                                             : launch_condense_mfma_fh2<NT, false>(a, st);
}

template <int NT, int NU4, bool DRIFT, bool P12>
static int launch_condense_mfma4(const CondenseArgs<float>& a, hipStream_t st) {
  const size_t bytes = ((size_t)a.N * NU4 * 16 + (size_t)a.nu * a.nu) * sizeof(float);
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)condense_mfma_kernel<NT, NU4, DRIFT, P12>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(condense_mfma)");
  }
  hipLaunchKernelGGL((condense_mfma_kernel<NT, NU4, DRIFT, P12>), dim3(a.batch), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("condense_mfma_kernel");
  return MPCQP_OK;
}
template <int NT, int NU4, bool DRIFT>
static int launch_condense_mfma3(const CondenseArgs<float>& a, hipStream_t st) {
  return a.nx <= 12 ? launch_condense_mfma4<NT, NU4, DRIFT, true>(a, st)
                    : launch_condense_mfma4<NT, NU4, DRIFT, false>(a, st);
}
template <int NT, int NU4>
static int launch_condense_mfma(const CondenseArgs<float>& a, hipStream_t st) {
  return a.c ? launch_condense_mfma3<NT, NU4, true>(a, st) : launch_condense_mfma3<NT, NU4, false>(a, st);
}

// fp32 with 5 <= nx <= 15 and N*nu <= 256 (MPCQP_CONDENSE_MFMA=0 forces the
// wavefront kernel, for A/B checks).  Returns 1 if not applicable.
static int condense_mfma(const CondenseArgs<float>& a, hipStream_t st) {
  static const int enabled = [] {
    const char* e = getenv("MPCQP_CONDENSE_MFMA");
    return e ? atoi(e) : 1;
  }();
  const int n = a.N * a.nu;
  // (packed Gamma only on the wavefront kernel: its one consumer, the
  // z-space QP, has nx <= 4)
  if (!enabled || a.gpk || a.nx < 5 || a.nx > 15 || a.nu > 16 || n > 256 ||
      (size_t)a.N * 16 * 16 * sizeof(float) > 160 * 1024)
    return 1;
  const int nt = (n + 15) / 16;
  // no drift, nx <= 12, nu <= 4: the fused-H kernel (MPCQP_CONDENSE_FH=0: the
  // VALU-epilogue kernel, A/B)
  static const int fh = [] {
    const char* e = getenv("MPCQP_CONDENSE_FH");
    return e ? atoi(e) : 1;
  }();
  if (fh && !a.c && !a.F && !a.Phi && a.nx <= 12 && (a.nu == 1 || a.nu == 2 || a.nu == 4)) {
    if (nt <= 4) return launch_condense_mfma_fh<4>(a, st);
    if (nt <= 8) return launch_condense_mfma_fh<8>(a, st);
    if (nt <= 10) return launch_condense_mfma_fh<10>(a, st);
    if (nt <= 12) return launch_condense_mfma_fh<12>(a, st);
    return launch_condense_mfma_fh<16>(a, st);
  }
  if (a.nu <= 4) {
    if (nt <= 4) return launch_condense_mfma<4, 4>(a, st);
    if (nt <= 8) return launch_condense_mfma<8, 4>(a, st);
    if (nt <= 10) return launch_condense_mfma<10, 4>(a, st);
    if (nt <= 12) return launch_condense_mfma<12, 4>(a, st);
    return launch_condense_mfma<16, 4>(a, st);
  }
  if (a.nu <= 8) {
    if (nt <= 8) return launch_condense_mfma<8, 8>(a, st);
    return launch_condense_mfma<16, 8>(a, st);
  }
  return launch_condense_mfma<16, 16>(a, st);
}

template <typename T>
static int condense_t(int batch, int nx, int nu, int N, int flags, const void* A, int64_t sA,
                      const void* Bm, int64_t sB, const void* Q, int64_t sQ, const void* R,
                      int64_t sR, const void* Qf, int64_t sQf, const void* c, int64_t sC,
                      const void* x0, int64_t sX0, void* H, void* F, void* f, void* Gam,
                      void* Phi, void* xbar, hipStream_t st, const int* count = nullptr) {
  CondenseArgs<T> a;
  a.count = count;
  a.batch = batch; a.nx = nx; a.nu = nu; a.N = N; a.tv = (flags & MPCQP_TV) ? 1 : 0;
  a.A = (const T*)A; a.sA = sA; a.B = (const T*)Bm; a.sB = sB;
  a.Q = (const T*)Q; a.sQ = sQ; a.R = (const T*)R; a.sR = sR;
  a.Qf = (const T*)Qf; a.sQf = sQf; a.c = (const T*)c; a.sC = sC;
  a.x0 = (const T*)x0; a.sX0 = sX0;
  a.H = (T*)H; a.F = (T*)F; a.f = (T*)f; a.Gam = (T*)Gam; a.Phi = (T*)Phi; a.xbar = (T*)xbar;
  a.gpk = (flags & MPCQP_GAM_PACKED) ? 1 : 0;
  if constexpr (sizeof(T) == 4) {
    const int rc = condense_mfma(a, st);
    if (rc != 1) return rc;
  }
  if (nx <= 2) return launch_condense<T, 2>(a, st);
  if (nx <= 4) return launch_condense<T, 4>(a, st);
  if (nx <= 8) return launch_condense<T, 8>(a, st);
  if (nx <= 12) return launch_condense<T, 12>(a, st);
  return launch_condense<T, 16>(a, st);
}

// fp64 condensing of the first min(*count, batch) instances (the fp64
// hand-off of mpcqp_mpc_qp, fallback64.hip): the per-instance kernel, the
// workgroups past the device count return at once
int condense_f64_count(int batch, int nx, int nu, int N, int flags, const double* A, int64_t sA,
                       const double* Bm, int64_t sB, const double* Q, int64_t sQ, const double* R,
                       int64_t sR, const double* Qf, int64_t sQf, const double* c, int64_t sC,
                       const double* x0, int64_t sX0, double* H, double* f, double* Gam,
                       double* xbar, const int* count, hipStream_t st) {
  return condense_t<double>(batch, nx, nu, N, flags, A, sA, Bm, sB, Q, sQ, R, sR, Qf, sQf, c, sC,
                            x0, sX0, H, nullptr, f, Gam, nullptr, xbar, st, count);
}

}  // namespace mpcqp

extern "C" int mpcqp_condense(int dtype, int batch, int nx, int nu, int N, int flags,
                              const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                              const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                              const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                              const void* x0, int64_t strideX0, void* H, void* F, void* f,
                              void* Gam, void* Phi, void* xbar, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_condense: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_condense: batch < 0");
  MPCQP_CHECK_ARG(nx >= 1 && nx <= 16, "mpcqp_condense: nx=%d outside [1,16]", nx);
  MPCQP_CHECK_ARG(nu >= 1 && nu <= 16, "mpcqp_condense: nu=%d outside [1,16]", nu);
  MPCQP_CHECK_ARG(N >= 1 && (int64_t)N * nu <= 4096, "mpcqp_condense: N=%d out of range", N);
  MPCQP_CHECK_ARG(A && Bm && Q && R && Qf && H, "mpcqp_condense: A, B, Q, R, Qf, H are required");
  MPCQP_CHECK_ARG(strideA >= 0 && strideB >= 0 && strideQ >= 0 && strideR >= 0 && strideQf >= 0 &&
                      strideC >= 0 && strideX0 >= 0,
                  "mpcqp_condense: negative stride");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return condense_t<double>(batch, nx, nu, N, flags, A, strideA, Bm, strideB, Q, strideQ, R,
                              strideR, Qf, strideQf, c, strideC, x0, strideX0, H, F, f, Gam, Phi,
                              xbar, st);
  return condense_t<float>(batch, nx, nu, N, flags, A, strideA, Bm, strideB, Q, strideQ, R,
                           strideR, Qf, strideQf, c, strideC, x0, strideX0, H, F, f, Gam, Phi,
                           xbar, st);
}

#ifdef MPCQP_PHASE_TIMING
MPCQP_DEBUG_PHASE_READER(mpcqp_debug_phase_cycles_condense)
#endif
