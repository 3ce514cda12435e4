// pf.hpp -- interface between the product-form active-set kernel
// (solve_pf.hip) and its callers (solve_qp.hip, mpc_qp.hip).
#pragma once
#include "common.hpp"

namespace mpcqp {

constexpr int kSlots = 64;
constexpr int kKChunk = 1536;  // floats of K rows per refinement chunk (6 KB of LDS)
constexpr int kStatusRetry = 0x7f;  // internal: hand the instance to qp_wg_kernel
// refinement scratch (doubles): K-pass = red (8*64) + rsum (3*64) + kbuf
constexpr int kPool = 8 * kWave + 3 * kWave + kKChunk / 2;
// doubles added to the pool for the M0 row cache of qp_pf_kernel (NXP <= 4):
// 20 rows at n + m = 180, within the LDS of 8 waves per CU (2 per SIMD, the
// occupancy the kernel is latency-bound at: 47 rows at 4 waves per CU cut
// the traffic by 3x and doubled the time)
constexpr int kPoolCacheExtra = 400;
// DYN layout inside the pool (doubles): xd (3*64: u, then mu of the state
// rows; g overwrites u) | lam (2 x 16) | X ((N+1) nx) | Q, Qf, R (floats) |
// stage chunk (floats): [A_s | B_s | c_s] for a run of stages
constexpr int kDynXd = 0, kDynLam = 3 * kWave, kDynX = kDynLam + 32;
// DYN refinement: converged once a correction is below this (relative to
// 1 + |value|); the residual after it is the certificate's
constexpr float kDynStop = 1e-7f;
// certificate, primal: relative violation of an inactive row or free z (the
// scan's scales), from the exact values
constexpr float kDynTol = 1e-7f;
// certificate, dual: a fixed z whose exact Lagrangian gradient has the wrong
// sign by more than kDualTol (1 + |f_i|), or an active row whose multiplier is
// below -kDualTol, is released.  A wrong-signed weakly active bound moves z by
// about its multiplier over the reduced curvature (>= 1e-2 at config 3), so
// this keeps such a bound's effect below the 1e-5 bar.
constexpr float kDualTol = 2e-8f;
// DYN: active-set + refinement + certificate rounds before an uncertified
// instance goes to the fp64 fallback
constexpr int kDynRounds = 4;

// Dynamics of the condensed QP (mpcqp_mpc_qp): z = [u_0..u_{N-1}], rows (m =
// N nx, or 0) = the state box on x_1..x_N with the ORIGINAL bounds xlo/xhi.
struct PfDyn {
  int nx, nu, N, tv;
  const float* A; int64_t sA;   // nx*nx (or N*nx*nx with tv) per instance
  const float* B; int64_t sB;   // nx*nu (or N*nx*nu)
  const float* c; int64_t sC;   // N*nx, optional
  const float* x0; int64_t sX0; // nx
  const float* Q; int64_t sQ;
  const float* R; int64_t sR;
  const float* Qf; int64_t sQf;
  const float* xlo; const float* xhi; int64_t sXb;  // N*nx (m > 0)
};

// stages per run of the DYN stage stream (what fits the pool); 0 = the DYN
// path does not apply
__host__ __device__ inline int dyn_chunk_stages(int nx, int nu, int N) {
  const int qr = (2 * nx * nx + nu * nu + 1) / 2;
  const int free_d = kPool - kDynX - (N + 1) * nx - qr;
  const int sf = nx * nx + nx * nu + nx;
  return free_d <= 0 ? 0 : (2 * free_d) / sf;
}

// compiled DYN widths (padded max(nx, nu)); 0 = none
__host__ __device__ inline int dyn_nxp(int nx, int nu) {
  const int w = nx > nu ? nx : nu;
  return w <= 4 ? 4 : (w <= 8 ? 8 : (w <= 12 ? 12 : (w <= 16 ? 16 : 0)));
}

// solve_zf.hip: the z-space product form with H^-1 on chip (fp32, DYN only)
bool zf_supported(int n, int m, int nx, int nu, int N);
int launch_zf(int batch, int n, int m, const float* M, const float* s0, const float* Gam,
              const float* f, int64_t sf, const float* lb, int64_t sLb, const float* ub,
              int64_t sUb, float* z, float* y, int32_t* status, int* retry_count, int* retry_list,
              int max_iter, int refine, float tol, const PfDyn& dyn, hipStream_t st);
// sweep.hip: -H^-1 (n x n full) and s0 = -H^-1 f for 48 < n <= 64
int sweep_hinv(int batch, int n, const void* H, int64_t sH, const void* f, int64_t sf, void* M,
               void* s0, int32_t* status, hipStream_t st);

int launch_pf(int batch, int n, int m, const float* H, int64_t sH, const float* f, int64_t sf,
              const float* G, int64_t sG, const float* hl, const float* hu, int64_t sh,
              const float* lb, int64_t sLb, const float* ub, int64_t sUb, const float* M0,
              const float* s0, float* z, float* y, int32_t* status, int* retry_count,
              int* retry_list, int max_iter, int refine, float tol, hipStream_t st,
              const PfDyn* dyn = nullptr);

}  // namespace mpcqp
