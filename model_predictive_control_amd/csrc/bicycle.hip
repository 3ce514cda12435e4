// bicycle.hip -- batched re-linearisation of the kinematic bicycle for the
// real-time-iteration MPC of session_4 (main.py:41-113 builds the OCP on
// fwd_euler(KinematicBicycle), main.py:132-135, 250-251).
//
// For each instance: roll the forward-Euler model out from x0 under the
// warm-start inputs U (the linearisation points x_0..x_{N-1}) and emit
//     A_k = I + ts df/dx,  B_k = ts df/du,  c_k = fd(x_k, u_k) - A_k x_k - B_k u_k
// so that x_{k+1} ~= A_k x_k + B_k u_k + c_k -- exactly the per-stage
// (A_k, B_k, c_k) that mpcqp_condense(MPCQP_TV) consumes (BASELINE config 3,
// and the config-5 style re-linearisation each step).  ODE (parity unpinned:
// rcracers is absent; restated from parameters.py:7-8,47-48):
//     beta = atan(lr/(lf+lr) tan delta)
//     px' = v cos(psi+beta), py' = v sin(psi+beta), psi' = v/lr sin(beta),
//     v' = acc * a - fric * v.
//
// Mapping: G <= 64 instances per workgroup (within 64 KiB of LDS).  Phase 1
// (lane = instance) runs the serial rollout and stages x_k in LDS; phase 2
// (lane = (instance, stage))
// evaluates the trig terms once per point; phase 3 writes A, B, c element-
// wise over the workgroup's contiguous output block, so every store
// instruction is coalesced across lanes.
#include <algorithm>

#include "common.hpp"

namespace mpcqp {

template <typename T>
struct BikeArgs {
  int batch, N, G;  // G instances per workgroup (<= 64, sized to the LDS budget)
  T ts, lf, lr, acc, fric;
  const T* x0; int64_t sX0;
  const T* U; int64_t sU;  // N x 2 per instance
  T* X;                    // (N+1) x 4 per instance, optional
  T* A; T* B; T* c;        // N x 16, N x 8, N x 4 per instance
};

constexpr int kBikeP = 5;  // per-point terms: sin th, cos th, sin beta, cos beta, dbeta

template <typename T>
__global__ __launch_bounds__(64) void bicycle_rti_kernel(BikeArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Xs = reinterpret_cast<T*>(smem_raw);  // G x (N+1) x 4 states
  T* Ps = Xs + a.G * (a.N + 1) * 4;        // G x N x kBikeP per-point terms
  const int lane = threadIdx.x;
  const int N = a.N;
  const int i0 = blockIdx.x * a.G;
  const int G = min(a.G, a.batch - i0);
  const T kk = a.lr / (a.lf + a.lr);

  // -------------------------------------------------- phase 1: rollout
  if (lane < G) {
    const int b = i0 + lane;
    const T* x0 = a.x0 + (int64_t)b * a.sX0;
    const T* U = a.U + (int64_t)b * a.sU;
    T x[4] = {x0[0], x0[1], x0[2], x0[3]};
    T* xs = Xs + lane * (N + 1) * 4;
    for (int k = 0; k <= N; ++k) {
#pragma unroll
      for (int r = 0; r < 4; ++r) xs[k * 4 + r] = x[r];
      if (k == N) break;
      const T ua = U[2 * k], ud = U[2 * k + 1];
      const T beta = atan(kk * tan(ud));
      const T th = x[2] + beta;
      const T v = x[3];
      const T dx0 = v * cos(th), dx1 = v * sin(th), dx2 = v / a.lr * sin(beta);
      const T dx3 = a.acc * ua - a.fric * v;
      x[0] += a.ts * dx0;
      x[1] += a.ts * dx1;
      x[2] += a.ts * dx2;
      x[3] += a.ts * dx3;
    }
  }
  __syncthreads();

  // ------------------------------------ phase 2: per-point trig terms
  for (int e = lane; e < G * N; e += 64) {
    const int g = e / N, k = e - g * N;
    const int b = i0 + g;
    const T* U = a.U + (int64_t)b * a.sU;
    const T ud = U[2 * k + 1];
    const T td = tan(ud);
    const T beta = atan(kk * td);
    const T* x = Xs + (g * (N + 1) + k) * 4;
    const T th = x[2] + beta;
    const T cd = cos(ud);
    const T dbeta = kk / (cd * cd) / (T(1) + (kk * td) * (kk * td));
    T* P = Ps + e * kBikeP;
    P[0] = sin(th);
    P[1] = cos(th);
    P[2] = sin(beta);
    P[3] = cos(beta);
    P[4] = dbeta;
  }
  __syncthreads();

  // ------------------------------------------------ phase 3: A, B, c
  // A_k = I + ts J: J rows [0,0,-v s,c], [0,0,v c,s], [0,0,0,sb/lr], [0,0,0,-fric]
  {
    T* Ab = a.A + (int64_t)i0 * N * 16;
    for (int e = lane; e < G * N * 16; e += 64) {
      const int gk = e >> 4, rc = e & 15, r = rc >> 2, q = rc & 3;
      const int g = gk / N, k = gk - g * N;
      const T* x = Xs + (g * (N + 1) + k) * 4;
      const T* P = Ps + gk * kBikeP;
      const T v = x[3];
      T j = T(0);
      if (q == 2) j = (r == 0) ? -v * P[0] : ((r == 1) ? v * P[1] : T(0));
      if (q == 3) j = (r == 0) ? P[1] : ((r == 1) ? P[0] : ((r == 2) ? P[2] / a.lr : -a.fric));
      Ab[e] = ((r == q) ? T(1) : T(0)) + a.ts * j;
    }
  }
  // B_k = ts Ju: Ju rows [0,-v s db], [0, v c db], [0, v cb db/lr], [acc, 0]
  {
    T* Bb = a.B + (int64_t)i0 * N * 8;
    for (int e = lane; e < G * N * 8; e += 64) {
      const int gk = e >> 3, rc = e & 7, r = rc >> 1, q = rc & 1;
      const int g = gk / N, k = gk - g * N;
      const T* x = Xs + (g * (N + 1) + k) * 4;
      const T* P = Ps + gk * kBikeP;
      const T v = x[3];
      T j;
      if (q == 0) {
        j = (r == 3) ? a.acc : T(0);
      } else {
        j = (r == 0) ? -v * P[0] * P[4]
                     : ((r == 1) ? v * P[1] * P[4] : ((r == 2) ? v * P[3] * P[4] / a.lr : T(0)));
      }
      Bb[e] = a.ts * j;
    }
  }
  // c_k = x_{k+1} - A_k x_k - B_k u_k  (x_{k+1} = fd(x_k, u_k) from phase 1)
  {
    T* Cb = a.c + (int64_t)i0 * N * 4;
    for (int e = lane; e < G * N * 4; e += 64) {
      const int gk = e >> 2, r = e & 3;
      const int g = gk / N, k = gk - g * N;
      const T* x = Xs + (g * (N + 1) + k) * 4;
      const T* xn = x + 4;
      const T* P = Ps + gk * kBikeP;
      const T* U = a.U + (int64_t)(i0 + g) * a.sU + 2 * k;
      const T v = x[3], ts = a.ts;
      T ax, bu;  // (A x)_r, (B u)_r
      if (r == 0) {
        ax = x[0] + ts * (-v * P[0] * x[2] + P[1] * x[3]);
        bu = ts * (-v * P[0] * P[4]) * U[1];
      } else if (r == 1) {
        ax = x[1] + ts * (v * P[1] * x[2] + P[0] * x[3]);
        bu = ts * (v * P[1] * P[4]) * U[1];
      } else if (r == 2) {
        ax = x[2] + ts * (P[2] / a.lr) * x[3];
        bu = ts * (v * P[3] * P[4] / a.lr) * U[1];
      } else {
        ax = x[3] - ts * a.fric * x[3];
        bu = ts * a.acc * U[0];
      }
      Cb[e] = xn[r] - ax - bu;
    }
  }
  if (a.X) {
    T* Xb = a.X + (int64_t)i0 * (N + 1) * 4;
    for (int e = lane; e < G * (N + 1) * 4; e += 64) Xb[e] = Xs[e];
  }
}

template <typename T>
static int bicycle_t(int batch, int N, double ts, const double* prm, const void* x0, int64_t sX0,
                     const void* U, int64_t sU, void* X, void* A, void* B, void* c,
                     hipStream_t st) {
  BikeArgs<T> a;
  a.batch = batch; a.N = N; a.ts = (T)ts;
  a.lf = (T)prm[0]; a.lr = (T)prm[1]; a.acc = (T)prm[2]; a.fric = (T)prm[3];
  a.x0 = (const T*)x0; a.sX0 = sX0; a.U = (const T*)U; a.sU = sU;
  a.X = (T*)X; a.A = (T*)A; a.B = (T*)B; a.c = (T*)c;
  // instances per workgroup: up to 64, within a 64 KiB LDS budget
  const size_t per = (size_t)((N + 1) * 4 + N * kBikeP) * sizeof(T);
  a.G = (int)std::min<size_t>(64, (64 * 1024) / per);
  if (a.G < 1) {
    set_error("mpcqp_bicycle_rti: N=%d too large (%zu B of LDS per instance)", N, per);
    return MPCQP_ENOTSUP;
  }
  const size_t bytes = (size_t)a.G * per;
  hipLaunchKernelGGL(bicycle_rti_kernel<T>, dim3((batch + a.G - 1) / a.G), dim3(64), bytes, st, a);
  MPCQP_CHECK_LAUNCH("bicycle_rti_kernel");
  return MPCQP_OK;
}

}  // namespace mpcqp

extern "C" int mpcqp_bicycle_rti(int dtype, int batch, int N, double ts, const double* params,
                                 const void* x0, int64_t strideX0, const void* U,
                                 int64_t strideU, void* X, void* A, void* B, void* c,
                                 void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_bicycle_rti: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1, "mpcqp_bicycle_rti: bad sizes");
  MPCQP_CHECK_ARG(params && x0 && U && A && B && c, "mpcqp_bicycle_rti: null pointer");
  MPCQP_CHECK_ARG(params[1] > 0 && params[0] + params[1] > 0, "mpcqp_bicycle_rti: bad axle lengths");
  MPCQP_CHECK_ARG(strideX0 >= 4 && strideU >= 2 * N, "mpcqp_bicycle_rti: bad strides");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return bicycle_t<double>(batch, N, ts, params, x0, strideX0, U, strideU, X, A, B, c, st);
  return bicycle_t<float>(batch, N, ts, params, x0, strideX0, U, strideU, X, A, B, c, st);
}
