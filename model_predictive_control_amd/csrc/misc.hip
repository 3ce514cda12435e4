// misc.hip -- the small batched kernels around condense/solve:
//   mpcqp_riccati  : ricatti_recursion (session_1/FHC.py:51-61), batched
//   mpcqp_gemv     : y = alpha M x + beta y, batched (f = F x0, primal recovery)
//   mpcqp_rollout  : LinearSystem.simulate (LinearSystem.py:20-26) under
//                    u = K x (AutoCruising.control_law, FHC.py:25-26), batched
#include "common.hpp"

namespace mpcqp {

// ------------------------------------------------------------- Riccati
// One instance per lane; matrices in registers (fixed 4x4 / 4x4 tiles with
// runtime guards so every index is compile-time).
constexpr int RX = 4;  // max nx
constexpr int RU = 4;  // max nu

template <typename T>
struct RiccatiArgs {
  int batch, nx, nu, N;
  const T* A; int64_t sA;
  const T* B; int64_t sB;
  const T* Q; int64_t sQ;
  const T* R; int64_t sR;
  const T* Pf; int64_t sPf;
  T* P; T* K;
};

template <typename T>
__global__ __launch_bounds__(256) void riccati_kernel(RiccatiArgs<T> a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.batch) return;
  const int nx = a.nx, nu = a.nu, N = a.N;
  T A[RX][RX], B[RX][RU], Q[RX][RX], R[RU][RU], P[RX][RX];
#pragma unroll
  for (int i = 0; i < RX; ++i)
#pragma unroll
    for (int j = 0; j < RX; ++j) {
      const bool in = i < nx && j < nx;
      A[i][j] = in ? a.A[(int64_t)b * a.sA + i * nx + j] : T(0);
      Q[i][j] = in ? a.Q[(int64_t)b * a.sQ + i * nx + j] : T(0);
      P[i][j] = in ? a.Pf[(int64_t)b * a.sPf + i * nx + j] : T(0);
    }
#pragma unroll
  for (int i = 0; i < RX; ++i)
#pragma unroll
    for (int j = 0; j < RU; ++j)
      B[i][j] = (i < nx && j < nu) ? a.B[(int64_t)b * a.sB + i * nu + j] : T(0);
#pragma unroll
  for (int i = 0; i < RU; ++i)
#pragma unroll
    for (int j = 0; j < RU; ++j)
      R[i][j] = (i < nu && j < nu) ? a.R[(int64_t)b * a.sR + i * nu + j] : T(0);

  T* Pout = a.P + (int64_t)b * (N + 1) * nx * nx;
  T* Kout = a.K + (int64_t)b * N * nu * nx;
#pragma unroll
  for (int i = 0; i < RX; ++i)
#pragma unroll
    for (int j = 0; j < RX; ++j)
      if (i < nx && j < nx) Pout[(int64_t)N * nx * nx + i * nx + j] = P[i][j];

  for (int t = 0; t < N; ++t) {
    // PA = P A, PB = P B
    T PA[RX][RX], PB[RX][RU];
#pragma unroll
    for (int i = 0; i < RX; ++i) {
#pragma unroll
      for (int j = 0; j < RX; ++j) {
        T s = T(0);
#pragma unroll
        for (int k = 0; k < RX; ++k) s = fma(P[i][k], A[k][j], s);
        PA[i][j] = s;
      }
#pragma unroll
      for (int j = 0; j < RU; ++j) {
        T s = T(0);
#pragma unroll
        for (int k = 0; k < RX; ++k) s = fma(P[i][k], B[k][j], s);
        PB[i][j] = s;
      }
    }
    // S = R + B'PB (nu x nu), Y = B'PA (nu x nx); pad S with identity
    T S[RU][RU], Y[RU][RX];
#pragma unroll
    for (int i = 0; i < RU; ++i) {
#pragma unroll
      for (int j = 0; j < RU; ++j) {
        T s = R[i][j];
#pragma unroll
        for (int k = 0; k < RX; ++k) s = fma(B[k][i], PB[k][j], s);
        S[i][j] = (i < nu && j < nu) ? s : (i == j ? T(1) : T(0));
      }
#pragma unroll
      for (int j = 0; j < RX; ++j) {
        T s = T(0);
#pragma unroll
        for (int k = 0; k < RX; ++k) s = fma(B[k][i], PA[k][j], s);
        Y[i][j] = s;
      }
    }
    // K = -S^{-1} Y  (Gauss-Jordan with partial pivoting, like numpy inv)
#pragma unroll
    for (int c = 0; c < RU; ++c) {
      int piv = c;
      T best = fabs(S[c][c]);
#pragma unroll
      for (int r = c + 1; r < RU; ++r)
        if (fabs(S[r][c]) > best) { best = fabs(S[r][c]); piv = r; }
#pragma unroll
      for (int r = c + 1; r < RU; ++r) {
        if (r == piv) {
#pragma unroll
          for (int j = 0; j < RU; ++j) { T t0 = S[c][j]; S[c][j] = S[r][j]; S[r][j] = t0; }
#pragma unroll
          for (int j = 0; j < RX; ++j) { T t0 = Y[c][j]; Y[c][j] = Y[r][j]; Y[r][j] = t0; }
        }
      }
      const T inv = T(1) / S[c][c];
#pragma unroll
      for (int j = 0; j < RU; ++j) S[c][j] *= inv;
#pragma unroll
      for (int j = 0; j < RX; ++j) Y[c][j] *= inv;
#pragma unroll
      for (int r = 0; r < RU; ++r) {
        if (r == c) continue;
        const T fct = S[r][c];
#pragma unroll
        for (int j = 0; j < RU; ++j) S[r][j] = fma(-fct, S[c][j], S[r][j]);
#pragma unroll
        for (int j = 0; j < RX; ++j) Y[r][j] = fma(-fct, Y[c][j], Y[r][j]);
      }
    }
    T Kk[RU][RX];
#pragma unroll
    for (int i = 0; i < RU; ++i)
#pragma unroll
      for (int j = 0; j < RX; ++j) Kk[i][j] = -Y[i][j];
    // P' = Q + A'PA + A'PB K   (FHC.py:57, same association)
    T Pn[RX][RX];
#pragma unroll
    for (int i = 0; i < RX; ++i)
#pragma unroll
      for (int j = 0; j < RX; ++j) {
        T s1 = T(0), s2 = T(0);
#pragma unroll
        for (int k = 0; k < RX; ++k) s1 = fma(A[k][i], PA[k][j], s1);
        T BK[RX];
#pragma unroll
        for (int k = 0; k < RX; ++k) {
          T s = T(0);
#pragma unroll
          for (int l = 0; l < RU; ++l) s = fma(PB[k][l], Kk[l][j], s);
          BK[k] = s;
        }
#pragma unroll
        for (int k = 0; k < RX; ++k) s2 = fma(A[k][i], BK[k], s2);
        Pn[i][j] = Q[i][j] + s1 + s2;
      }
#pragma unroll
    for (int i = 0; i < RX; ++i)
#pragma unroll
      for (int j = 0; j < RX; ++j) P[i][j] = Pn[i][j];
    const int slot = N - 1 - t;  // reference returns the lists reversed
#pragma unroll
    for (int i = 0; i < RX; ++i)
#pragma unroll
      for (int j = 0; j < RX; ++j)
        if (i < nx && j < nx) Pout[(int64_t)slot * nx * nx + i * nx + j] = P[i][j];
#pragma unroll
    for (int i = 0; i < RU; ++i)
#pragma unroll
      for (int j = 0; j < RX; ++j)
        if (i < nu && j < nx) Kout[(int64_t)slot * nu * nx + i * nx + j] = Kk[i][j];
  }
}

// --------------------------------------------------------------- GEMV
// One wavefront per instance; lanes over rows, x staged through LDS.
template <typename T>
struct GemvArgs {
  int batch, rows, cols;
  T alpha, beta;
  const T* M; int64_t sM;
  const T* x; int64_t sX;
  T* y; int64_t sY;
};

template <typename T>
__global__ __launch_bounds__(64) void gemv_kernel(GemvArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* xs = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x, lane = threadIdx.x;
  const T* xb = a.x + (int64_t)b * a.sX;
  for (int j = lane; j < a.cols; j += kWave) xs[j] = xb[j];
  __syncthreads();
  const T* Mb = a.M + (int64_t)b * a.sM;
  T* yb = a.y + (int64_t)b * a.sY;
  for (int r = lane; r < a.rows; r += kWave) {
    const T* row = Mb + (int64_t)r * a.cols;
    T s = T(0);
    for (int j = 0; j < a.cols; ++j) s = fma(row[j], xs[j], s);
    yb[r] = (a.beta == T(0)) ? a.alpha * s : fma(a.beta, yb[r], a.alpha * s);
  }
}

// ------------------------------------------------------------- rollout
// One instance per lane.  xs layout: time-major (steps, batch, nx); the
// Python mirror returns the reference's (nx, batch, steps) view of it.
constexpr int LX = 16;

template <typename T>
struct RolloutArgs {
  int batch, nx, nu, steps;
  const T* A; const T* B; const T* K; const T* x0; T* xs;
};

template <typename T>
__global__ __launch_bounds__(256) void rollout_kernel(RolloutArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Acl = reinterpret_cast<T*>(smem_raw);  // A + B K, nx x nx
  const int nx = a.nx, nu = a.nu;
  for (int e = threadIdx.x; e < nx * nx; e += blockDim.x) {
    const int i = e / nx, j = e % nx;
    T s = a.A[e];
    for (int l = 0; l < nu; ++l) s = fma(a.B[i * nu + l], a.K[l * nx + j], s);
    Acl[e] = s;
  }
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.batch) return;
  T x[LX];
#pragma unroll
  for (int q = 0; q < LX; ++q) x[q] = (q < nx) ? a.x0[(int64_t)b * nx + q] : T(0);
  T* out = a.xs + (int64_t)b * nx;
  const int64_t tstride = (int64_t)a.batch * nx;
#pragma unroll
  for (int q = 0; q < LX; ++q)
    if (q < nx) out[q] = x[q];
  for (int t = 1; t < a.steps; ++t) {
    T y[LX];
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      T s = T(0);
#pragma unroll
      for (int j = 0; j < LX; ++j)
        if (i < nx && j < nx) s = fma(Acl[i * nx + j], x[j], s);
      y[i] = s;
    }
#pragma unroll
    for (int q = 0; q < LX; ++q) {
      x[q] = y[q];
      if (q < nx) out[t * tstride + q] = x[q];
    }
  }
}

}  // namespace mpcqp

using namespace mpcqp;

extern "C" int mpcqp_riccati(int dtype, int batch, int nx, int nu, int N, const void* A,
                             int64_t strideA, const void* Bm, int64_t strideB, const void* Q,
                             int64_t strideQ, const void* R, int64_t strideR, const void* Pf,
                             int64_t stridePf, void* P, void* K, void* stream) {
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_riccati: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "mpcqp_riccati: batch < 0 or N < 1");
  MPCQP_CHECK_ARG(nx >= 1 && nx <= RX && nu >= 1 && nu <= RU,
                  "mpcqp_riccati: nx=%d nu=%d outside the compiled 4x4 tile", nx, nu);
  MPCQP_CHECK_ARG(A && Bm && Q && R && Pf && P && K, "mpcqp_riccati: null pointer");
  if (batch == 0) return MPCQP_OK;
  const int threads = 256, blocks = (batch + threads - 1) / threads;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64) {
    RiccatiArgs<double> a{batch, nx, nu, N, (const double*)A, strideA, (const double*)Bm, strideB,
                          (const double*)Q, strideQ, (const double*)R, strideR,
                          (const double*)Pf, stridePf, (double*)P, (double*)K};
    hipLaunchKernelGGL(riccati_kernel<double>, dim3(blocks), dim3(threads), 0, st, a);
  } else {
    RiccatiArgs<float> a{batch, nx, nu, N, (const float*)A, strideA, (const float*)Bm, strideB,
                         (const float*)Q, strideQ, (const float*)R, strideR, (const float*)Pf,
                         stridePf, (float*)P, (float*)K};
    hipLaunchKernelGGL(riccati_kernel<float>, dim3(blocks), dim3(threads), 0, st, a);
  }
  MPCQP_CHECK_LAUNCH("riccati_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_gemv(int dtype, int batch, int rows, int cols, double alpha, const void* M,
                          int64_t strideM, const void* x, int64_t strideX, double beta, void* y,
                          int64_t strideY, void* stream) {
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_gemv: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && rows >= 0 && cols >= 0, "mpcqp_gemv: negative size");
  MPCQP_CHECK_ARG(M && x && y, "mpcqp_gemv: null pointer");
  MPCQP_CHECK_ARG(cols <= 8192, "mpcqp_gemv: cols=%d > 8192", cols);
  if (batch == 0 || rows == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64) {
    GemvArgs<double> a{batch, rows, cols, alpha, beta, (const double*)M, strideM,
                       (const double*)x, strideX, (double*)y, strideY};
    hipLaunchKernelGGL(gemv_kernel<double>, dim3(batch), dim3(kWave), (size_t)cols * 8, st, a);
  } else {
    GemvArgs<float> a{batch, rows, cols, (float)alpha, (float)beta, (const float*)M, strideM,
                      (const float*)x, strideX, (float*)y, strideY};
    hipLaunchKernelGGL(gemv_kernel<float>, dim3(batch), dim3(kWave), (size_t)cols * 4, st, a);
  }
  MPCQP_CHECK_LAUNCH("gemv_kernel");
  return MPCQP_OK;
}

extern "C" int mpcqp_rollout(int dtype, int batch, int nx, int nu, int steps, const void* A,
                             const void* Bm, const void* K, const void* x0, void* xs,
                             void* stream) {
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_rollout: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && steps >= 1, "mpcqp_rollout: batch < 0 or steps < 1");
  MPCQP_CHECK_ARG(nx >= 1 && nx <= LX && nu >= 1 && nu <= LX, "mpcqp_rollout: nx/nu outside [1,16]");
  MPCQP_CHECK_ARG(A && Bm && K && x0 && xs, "mpcqp_rollout: null pointer");
  if (batch == 0) return MPCQP_OK;
  const int threads = 256, blocks = (batch + threads - 1) / threads;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64) {
    RolloutArgs<double> a{batch, nx, nu, steps, (const double*)A, (const double*)Bm,
                          (const double*)K, (const double*)x0, (double*)xs};
    hipLaunchKernelGGL(rollout_kernel<double>, dim3(blocks), dim3(threads), (size_t)nx * nx * 8,
                       st, a);
  } else {
    RolloutArgs<float> a{batch, nx, nu, steps, (const float*)A, (const float*)Bm,
                         (const float*)K, (const float*)x0, (float*)xs};
    hipLaunchKernelGGL(rollout_kernel<float>, dim3(blocks), dim3(threads), (size_t)nx * nx * 4,
                       st, a);
  }
  MPCQP_CHECK_LAUNCH("rollout_kernel");
  return MPCQP_OK;
}
