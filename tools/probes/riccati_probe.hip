// Per-stage cycle counts of the wave interior point's recursions
// (ipm_wave.hpp) on one wave, stage data random but well-posed (SPD weights):
// clock64 (core clock) around riccati_mfma, forward_mfma, rhs_mfma at N = 30.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define MPCQP_HD __host__ __device__
#include "../../model_predictive_control_amd/csrc/common.hpp"
#include "../../model_predictive_control_amd/csrc/ipm_lane.hpp"
#include "../../model_predictive_control_amd/csrc/ipm_quad.hpp"
#include "../../model_predictive_control_amd/csrc/ipm_wave.hpp"
using namespace mpcqp;
using L = ipmq::L;
constexpr int N = 30;
__global__ __launch_bounds__(64, 1) void probe(const double* init, long long* t, double* out) {
  __shared__ double W[N * L::F];
  for (int e = threadIdx.x; e < N * L::F; e += 64) W[e] = init[e];
  wave_lds_sync();
  long long t0 = clock64();
  bool ok = ipmw::riccati_mfma<L::GA + 2, L::GA, L::DXA, L::DUA>(W, N, 0.0);
  wave_lds_sync();
  long long t1 = clock64();
  ipmw::forward_mfma<L::DX>(W, N);
  wave_lds_sync();
  long long t2 = clock64();
  ipmw::rhs_mfma<L::GA + 2, L::GA>(W, N);
  wave_lds_sync();
  long long t3 = clock64();
  if (threadIdx.x == 0) { t[0] = t1 - t0; t[1] = t2 - t1; t[2] = t3 - t2; t[3] = ok; }
  for (int e = threadIdx.x; e < N * L::F; e += 64) out[e] = W[e];
}
int main() {
  const int n = N * L::F;
  double* h = (double*)malloc(n * 8);
  srand(1);
  for (int e = 0; e < n; ++e) h[e] = 0.1 * ((double)rand() / RAND_MAX - 0.5);
  for (int k = 0; k < N; ++k) {  // diagonal weights and Sigma positive
    double* S = h + k * L::F;
    for (int i = 0; i < 4; ++i) { S[L::WXX + ipm::pk(i, i)] = 1.0; S[L::DXA + i] = 0.5; S[L::DA + i * 4 + i] += 1.0; }
    for (int i = 0; i < 2; ++i) { S[L::WUU + ipm::pk(i, i)] = 1.0; S[L::DUA + i] = 0.5; }
  }
  double *d, *o; long long* t; long long ht[4];
  hipMalloc(&d, n * 8); hipMalloc(&o, n * 8); hipMalloc(&t, 32);
  hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, t, o);
  hipMemcpy(ht, t, 32, hipMemcpyDeviceToHost);
  printf("N=%d cycles/stage: riccati %.0f forward %.0f rhs %.0f (ok=%lld)\n", N, ht[0] / (double)N,
         ht[1] / (double)N, ht[2] / (double)N, ht[3]);
  return 0;
}
