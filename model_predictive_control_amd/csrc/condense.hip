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
};

struct CLayout {
  int oA, oB, oQ, oQf, oR, oW, oT, oX, oY, oC, oX0, total;
};

__host__ __device__ inline CLayout clayout(int NX, int nu, int N, int tv) {
  CLayout L;
  const int S = tv ? N : 1;
  L.oA = 0;
  L.oB = L.oA + S * NX * NX;
  L.oQ = L.oB + S * NX * nu;
  L.oQf = L.oQ + NX * NX;
  L.oR = L.oQf + NX * NX;
  L.oW = L.oR + nu * nu;               // W_k, k = 0..N  ((N+1) slots; slot 0 unused)
  L.oT = L.oW + (N + 1) * NX * NX;     // scratch NX x NX
  L.oX = L.oT + NX * NX;               // xbar_k, k = 0..N
  L.oY = L.oX + (N + 1) * NX;          // y_k, k = 0..N
  L.oC = L.oY + (N + 1) * NX;          // drift c_k, k = 0..N-1
  L.oX0 = L.oC + N * NX;               // x0
  L.total = L.oX0 + NX;
  return L;
}

template <typename T, int NX>
__global__ __launch_bounds__(64) void condense_kernel(CondenseArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int nx = a.nx, nu = a.nu, N = a.N, n = N * nu;
  const int tv = a.tv;
  const int S = tv ? N : 1;
  const CLayout L = clayout(NX, nu, N, tv);
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

  // ---------------------------------------------------------------- stage in
  {
    const T* Ab = a.A + (int64_t)b * a.sA;
    for (int e = lane; e < S * NX * NX; e += kWave) {
      const int s = e / (NX * NX), r = (e / NX) % NX, q = e % NX;
      As[e] = (r < nx && q < nx) ? Ab[(int64_t)s * nx * nx + r * nx + q] : T(0);
    }
    const T* Bb = a.B + (int64_t)b * a.sB;
    for (int e = lane; e < S * NX * nu; e += kWave) {
      const int s = e / (NX * nu), rem = e - s * NX * nu, r = rem / nu, q = rem - r * nu;
      Bs[e] = (r < nx) ? Bb[(int64_t)s * nx * nu + r * nu + q] : T(0);
    }
    const T* Qb = a.Q + (int64_t)b * a.sQ;
    const T* Qfb = a.Qf + (int64_t)b * a.sQf;
    for (int e = lane; e < NX * NX; e += kWave) {
      const int r = e / NX, q = e % NX;
      const bool in = r < nx && q < nx;
      Qs[e] = in ? Qb[r * nx + q] : T(0);
      Qfs[e] = in ? Qfb[r * nx + q] : T(0);
    }
    const T* Rb = a.R + (int64_t)b * a.sR;
    for (int e = lane; e < nu * nu; e += kWave) Rs[e] = Rb[e];
    if (need_aff) {
      const T* Cb = a.c ? a.c + (int64_t)b * a.sC : nullptr;
      for (int e = lane; e < N * NX; e += kWave) {
        const int k = e / NX, q = e % NX;
        Cs[e] = (Cb && q < nx) ? Cb[k * nx + q] : T(0);
      }
      const T* X0b = a.x0 ? a.x0 + (int64_t)b * a.sX0 : nullptr;
      if (lane < NX) X0s[lane] = (X0b && lane < nx) ? X0b[lane] : T(0);
    }
  }
  __syncthreads();

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

  // ------------------------------------------------------- column sweep
  // z columns (H, Gam), then -- only when F or Phi is requested -- the x0
  // columns
  const int ncol = n + ((a.F || a.Phi) ? nx : 0);
  T* Hb = a.H + (int64_t)b * ((int64_t)n * (n + 1) / 2);
  T* Fb = a.F ? a.F + (int64_t)b * n * nx : nullptr;
  T* Gb = a.Gam ? a.Gam + (int64_t)b * ((int64_t)N * nx * n) : nullptr;
  T* Pb = a.Phi ? a.Phi + (int64_t)b * ((int64_t)N * nx * nx) : nullptr;
  for (int col0 = 0; col0 < ncol; col0 += kWave) {
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
#pragma unroll
          for (int q = 0; q < NX; ++q)
            if (q < nx) __builtin_nontemporal_store(s[q], &Gb[((int64_t)(i * nx + q)) * n + col]);
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

  // ------------------------------------------------- linear term and xbar
  if (a.f) {
    T* fb = a.f + (int64_t)b * n;
    for (int r = lane; r < n; r += kWave) {
      const int i = r / nu, aa = r - i * nu;
      const T* Bi = Bs + (tv ? i : 0) * NX * nu;
      T acc = T(0);
#pragma unroll
      for (int q = 0; q < NX; ++q) acc = fma(Bi[q * nu + aa], Ys[(i + 1) * NX + q], acc);
      fb[r] = acc;
    }
  }
  if (a.xbar) {
    T* xb = a.xbar + (int64_t)b * N * nx;
    for (int e = lane; e < N * nx; e += kWave) {
      const int k = e / nx, q = e - k * nx;
      xb[e] = Xs[(k + 1) * NX + q];
    }
  }
}

template <typename T, int NX>
static int launch_condense(const CondenseArgs<T>& a, hipStream_t st) {
  const CLayout L = clayout(NX, a.nu, a.N, a.tv);
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

template <typename T>
static int condense_t(int batch, int nx, int nu, int N, int flags, const void* A, int64_t sA,
                      const void* Bm, int64_t sB, const void* Q, int64_t sQ, const void* R,
                      int64_t sR, const void* Qf, int64_t sQf, const void* c, int64_t sC,
                      const void* x0, int64_t sX0, void* H, void* F, void* f, void* Gam,
                      void* Phi, void* xbar, hipStream_t st) {
  CondenseArgs<T> a;
  a.batch = batch; a.nx = nx; a.nu = nu; a.N = N; a.tv = (flags & MPCQP_TV) ? 1 : 0;
  a.A = (const T*)A; a.sA = sA; a.B = (const T*)Bm; a.sB = sB;
  a.Q = (const T*)Q; a.sQ = sQ; a.R = (const T*)R; a.sR = sR;
  a.Qf = (const T*)Qf; a.sQf = sQf; a.c = (const T*)c; a.sC = sC;
  a.x0 = (const T*)x0; a.sX0 = sX0;
  a.H = (T*)H; a.F = (T*)F; a.f = (T*)f; a.Gam = (T*)Gam; a.Phi = (T*)Phi; a.xbar = (T*)xbar;
  if (nx <= 2) return launch_condense<T, 2>(a, st);
  if (nx <= 4) return launch_condense<T, 4>(a, st);
  if (nx <= 8) return launch_condense<T, 8>(a, st);
  if (nx <= 12) return launch_condense<T, 12>(a, st);
  return launch_condense<T, 16>(a, st);
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
