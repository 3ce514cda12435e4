// Latency / issue probes of v_mfma_f64_4x4x4_4b_f64 and fp64 VALU on one wave
// (clock64 = core cycles): dependent chains through the B and C operands,
// independent products back to back, and an MFMA result read by the VALU.
#include <hip/hip_runtime.h>
#include <cstdio>
#define MF(a, b, c) __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0)
__global__ void kmfma(double* out, long long* t, double a0) {
  int l = threadIdx.x;
  double a = a0 * (l + 1), d = 1.0;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) d = MF(a, d, 0.0);
  long long t1 = clock64();
  out[l] = d; if (l == 0) t[0] = t1 - t0;
}
__global__ void kmfmac(double* out, long long* t, double a0) {
  int l = threadIdx.x;
  double a = a0 * (l + 1), b = 0.5, d = 1.0;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) d = MF(a, b, d);
  long long t1 = clock64();
  out[l] = d; if (l == 0) t[0] = t1 - t0;
}
__global__ void kmfma4(double* out, long long* t, double a0) {  // 4 independent chains
  int l = threadIdx.x;
  double a = a0 * (l + 1), d0 = 1, d1 = 2, d2 = 3, d3 = 4;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) { d0 = MF(a, d0, 0.0); d1 = MF(a, d1, 0.0); d2 = MF(a, d2, 0.0); d3 = MF(a, d3, 0.0); }
  long long t1 = clock64();
  out[l] = d0 + d1 + d2 + d3; if (l == 0) t[0] = t1 - t0;
}
__global__ void kmfmav(double* out, long long* t, double a0) {  // MFMA -> VALU -> MFMA
  int l = threadIdx.x;
  double a = a0 * (l + 1), d = 1.0;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) { d = MF(a, d, 0.0); d = d * 0.5 + 0.25; }
  long long t1 = clock64();
  out[l] = d; if (l == 0) t[0] = t1 - t0;
}
__global__ void kfma(double* out, long long* t, double a0) {
  int l = threadIdx.x;
  double a = a0 * (l + 1), d = 1.0;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) d = fma(d, a, 0.5);
  long long t1 = clock64();
  out[l] = d; if (l == 0) t[0] = t1 - t0;
}
__global__ void kfma4(double* out, long long* t, double a0) {
  int l = threadIdx.x;
  double a = a0 * (l + 1), d0 = 1.0, d1 = 2, d2 = 3, d3 = 4;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) { d0 = fma(d0, a, 0.5); d1 = fma(d1, a, 0.5); d2 = fma(d2, a, 0.5); d3 = fma(d3, a, 0.5); }
  long long t1 = clock64();
  out[l] = d0 + d1 + d2 + d3; if (l == 0) t[0] = t1 - t0;
}
__global__ void klds(double* out, long long* t, double a0) {  // LDS store -> load round trip
  __shared__ double s[64];
  int l = threadIdx.x;
  double d = a0 * l;
  long long t0 = clock64();
  for (int i = 0; i < 1000; ++i) { s[l] = d; __builtin_amdgcn_wave_barrier(); d = s[l ^ 1] + 1.0; }
  long long t1 = clock64();
  out[l] = d; if (l == 0) t[0] = t1 - t0;
}
int main() {
  double* o; long long* t; long long ht;
  hipMalloc(&o, 512); hipMalloc(&t, 8);
  auto run = [&](auto kern, const char* name, int ops) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, o, t, 1e-3);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, o, t, 1e-3);
    hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    printf("%-48s %.2f cycles per op\n", name, (double)ht / ops);
  };
  run(kmfma, "mfma_f64_4x4x4 chained via B", 1000);
  run(kmfmac, "mfma_f64_4x4x4 chained via C", 1000);
  run(kmfma4, "mfma_f64_4x4x4 4 independent chains (per op)", 4000);
  run(kmfmav, "mfma -> v_fma -> mfma (per pair)", 1000);
  run(kfma, "v_fma_f64 dependent chain", 1000);
  run(kfma4, "v_fma_f64 4 independent chains (per fma)", 4000);
  run(klds, "LDS store + dependent load round trip", 1000);
  return 0;
}
