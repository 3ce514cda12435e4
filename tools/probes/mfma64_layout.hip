#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out, const double* a, const double* b) {
  int l = threadIdx.x;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}
int main() {
  double *a, *b, *o;
  hipMalloc(&a, 64 * 8); hipMalloc(&b, 64 * 8); hipMalloc(&o, 64 * 8);
  double ha[64], hb[64], ho[64];
  // probe A: one-hot a at lane p, b = l+1
  for (int p : {0, 1, 2, 3, 4, 5, 8, 12, 15, 16, 17, 20, 33, 63}) {
    for (int l = 0; l < 64; ++l) { ha[l] = (l == p); hb[l] = l + 1; }
    hipMemcpy(a, ha, 512, hipMemcpyHostToDevice); hipMemcpy(b, hb, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, a, b);
    hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
    printf("A one-hot lane %2d ->", p);
    for (int l = 0; l < 64; ++l) if (ho[l] != 0) printf(" D[%d]=b[%d]", l, (int)ho[l] - 1);
    printf("\n");
  }
  // probe B: a = 1 everywhere in block, b one-hot at lane p -> which D lanes get it
  for (int p : {0, 1, 2, 3, 4, 5, 8, 12, 15, 16, 17, 33}) {
    for (int l = 0; l < 64; ++l) { ha[l] = l + 1; hb[l] = (l == p); }
    hipMemcpy(a, ha, 512, hipMemcpyHostToDevice); hipMemcpy(b, hb, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, a, b);
    hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
    printf("B one-hot lane %2d ->", p);
    for (int l = 0; l < 64; ++l) if (ho[l] != 0) printf(" D[%d]=a[%d]", l, (int)ho[l] - 1);
    printf("\n");
  }
  return 0;
}
