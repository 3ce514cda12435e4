// quad_api.hpp -- host-side entry points of the 4-QPs-per-wavefront kernels
// (quad_box.hip), used by the C ABI dispatchers for n <= 32.
#pragma once
#include <stdlib.h>

#include "common.hpp"

namespace mpcqp {

template <typename T>
struct BoxArgsQ {
  int batch, n;
  const T* H; int64_t sH;
  const T* f; int64_t sf;
  const T* lb; int64_t slb;
  const T* ub; int64_t sub;
  T* z;
  int32_t* status;
  int max_iter;
  T tol;
};

template <typename T>
struct MpcArgsQ {
  int batch, nx, nu, N, tv;
  const T* A; int64_t sA;
  const T* B; int64_t sB;
  const T* Q; int64_t sQ;
  const T* R; int64_t sR;
  const T* Qf; int64_t sQf;
  const T* c; int64_t sC;
  const T* x0; int64_t sX0;
  const T* lb; int64_t slb;
  const T* ub; int64_t sub;
  T* z;
  int32_t* status;
  int max_iter;
  T tol;
};

template <typename T>
int solve_box_quad(const BoxArgsQ<T>& a, hipStream_t st);
template <typename T>
int mpc_box_quad(const MpcArgsQ<T>& a, hipStream_t st);

// MPCQP_KERNEL=wave forces the one-QP-per-wavefront kernels (A/B runs).
inline bool use_wave_kernels() {
  const char* v = getenv("MPCQP_KERNEL");
  return v && v[0] == 'w';
}
// MPCQP_KERNEL=block forces the one-QP-per-workgroup kernel (solve_qp.hip).
inline bool use_block_kernels() {
  const char* v = getenv("MPCQP_KERNEL");
  return v && v[0] == 'b';
}

// solve_qp.hip
int solve_box_wg(int dtype, int batch, int n, const void* H, int64_t sH, const void* f,
                 int64_t sf, const void* lb, int64_t sLb, const void* ub, int64_t sUb, void* z,
                 int32_t* status, int max_iter, double tol, hipStream_t st,
                 const void* Ms = nullptr);
int max_qp_size_dtype(int dtype);

// ipm.hip: stage-wise interior point (any horizon; nx <= 4, nu <= 2)
bool ipm_supported(int nx, int nu);
size_t ipm_ws_bytes(int batch, int nx, int nu, int N);
int mpc_ipm_impl(int dtype, int batch, int nx, int nu, int N, int flags, const void* A,
                 int64_t sA, const void* Bm, int64_t sB, const void* Q, int64_t sQ, const void* R,
                 int64_t sR, const void* Qf, int64_t sQf, const void* c, int64_t sC,
                 const void* x0, int64_t sX0, const void* xlo, const void* xhi, int64_t sXb,
                 const void* lb, int64_t sLb, const void* ub, int64_t sUb, const void* U0,
                 int64_t sU0, const void* H2, int64_t sH2, const void* q2, int64_t sq2, void* z,
                 void* y, void* X, void* lam_u, void* pi, int32_t* status,
                 const int32_t* skip, int32_t skip_mask, int max_iter, double tol, void* ws,
                 size_t ws_bytes, hipStream_t st, const int* list = nullptr,
                 const int* list_count = nullptr, int list_begin = 0);
size_t qp_ws_bytes(int dtype, int batch, int n, int m);
struct PfDyn;
// dyn != NULL: refine from the dynamics (pf.hpp); refine < 0: default steps;
// wg_fallback = 0: the hand-off list is left to the caller (see qp_ws_parts)
// condense.hip / solve_qp.hip: the fp64 kernels over the first
// min(*count, batch) instances (compact slots of fallback64.hip)
int condense_f64_count(int batch, int nx, int nu, int N, int flags, const double* A, int64_t sA,
                       const double* Bm, int64_t sB, const double* Q, int64_t sQ, const double* R,
                       int64_t sR, const double* Qf, int64_t sQf, const double* c, int64_t sC,
                       const double* x0, int64_t sX0, double* H, double* f, double* Gam,
                       double* xbar, const int* count, hipStream_t st);
int solve_qp_f64_count(int batch, int n, int m, const double* H, int64_t sH, const double* f,
                       int64_t sf, const double* G, int64_t sG, const double* hl,
                       const double* hu, int64_t sh, const double* lb, int64_t sLb,
                       const double* ub, int64_t sUb, double* z, double* y, int32_t* status,
                       const int* count, hipStream_t st);

// fallback64.hip: the fp64 hand-off of mpcqp_mpc_qp's fp32 paths -- the
// first min(*count, cap) listed instances re-condensed in fp64 and solved by
// the fp64 workgroup active set, results scattered back (status bit
// MPCQP_STATUS_POLISHED); the rest of the list is left to the caller
struct Fallback64In {
  int batch, nx, nu, N, tv;
  const float *A, *B, *c, *x0, *Q, *R, *Qf, *xlo, *xhi, *lb, *ub;
  int64_t sA, sB, sC, sX0, sQ, sR, sQf, sXb, sLb, sUb;
};
int fallback64_cap(int batch);
size_t fallback64_bytes(int batch, int nx, int nu, int N, int sbox);
int fallback64(const Fallback64In& in, const int* list, const int* count, float* z, float* y,
               int32_t* status, void* ws, size_t ws_bytes, hipStream_t st);

// stage marks of mpcqp_mpc_qp's profiler (mpc_qp.hip; no-ops unless enabled)
enum { kProfStart, kProfCondense, kProfSweep, kProfSolve, kProfFallback, kProfStates, kProfN };
void prof_mark(int stage, hipStream_t st);

int solve_two_kernel(int batch, int n, int m, const void* H, int64_t sH, const void* f,
                     int64_t sf, const void* G, int64_t sG, const void* hl, const void* hu,
                     int64_t sh, const void* lb, int64_t sLb, const void* ub, int64_t sUb,
                     void* z, void* y, int32_t* status, int max_iter, double tol, void* ws,
                     hipStream_t st, const PfDyn* dyn = nullptr, int refine = -1,
                     int wg_fallback = 1);
// the two-kernel workspace's parts: the dense M0 region and the s0 region
// (both free once the product-form kernel has run), the hand-off count and list
struct QpWsParts {
  void* m0; size_t m0_bytes;
  void* s0; size_t s0_bytes;
  int* cnt; int* list;
};
QpWsParts qp_ws_parts(void* ws, int batch, int n, int m);

}  // namespace mpcqp
