// loop_box.hip -- mpcqp_mpc_box_loop: the receding-horizon loop of an
// input-box MPC on a linear plant, T steps in ONE launch, four instances per
// wavefront (quad.hpp layout, one per 16-lane DPP row).
//
// Reference: the closed loop of session_1 (LinearSystem.simulate under a
// policy, LinearSystem.py:20-26; FHC.py:20-29) with the box-constrained MPC
// step of session_4 (MPCController.solve, main.py:115-116, input box
// main.py:68-69) as the policy, and simulate(x0, dynamics, n, policy)
// (main.py:270-271) as the loop.  Per step t and instance b:
//   f_t = F x_t                          (the condensed gradient; H, F of the
//                                          instance's LTI plant, mpcqp_condense)
//   z_t = argmin 1/2 z'Hz + f_t'z, lb <= z <= ub
//   x_{t+1} = A x_t + B u_0(z_t)
//
// Everything of an instance stays on chip for the whole episode: packed H and
// F in the group's LDS block, x_t in LDS, the active set in registers.  Each
// step is warm-started from the previous step's active set shifted one stage
// (row i takes the state of row i + nu; the last stage repeats): the matrix of
// the active set is H swept on its FREE rows only (H swept on F equals -H^-1
// swept back on the active rows), so a mostly saturated problem (config 2:
// ~80 % of the bounds active) starts from a handful of sweeps instead of n,
// and the Goldfarb-Idnani iterations only correct the guess (gi_box_st).  No
// Riccati, no -H^-1, no HBM traffic per step but x, u, the status and the
// (optional) input plan.
#include "quad.hpp"
#include "quad_api.hpp"

namespace mpcqp {

template <typename T>
struct LoopArgs {
  int batch, nx, nu, N, n, steps;
  const T* H; int64_t sH;      // packed lower n(n+1)/2 per instance
  const T* F; int64_t sF;      // n x nx per instance (f = F x)
  const T* A; int64_t sA;      // plant nx x nx
  const T* B; int64_t sB;      // plant nx x nu
  const T* x0; int64_t sX0;
  const T* lb; int64_t slb;
  const T* ub; int64_t sub;
  T* xs;                       // (steps + 1) x batch x nx
  T* us;                       // steps x batch x nu
  T* zs;                       // optional steps x batch x n: the input plans
  int32_t* status;             // steps x batch
  int max_iter;
  T tol;
};

template <typename T, int NX, int NU, int BS>
struct LoopLds {
  using Box = QBoxLds<T, BS>;
  static constexpr int NMAX = 4 * BS;
  static constexpr int PMAX = NMAX * (NMAX + 1) / 2;
  static constexpr int oP = Box::size;          // packed H
  static constexpr int oF = oP + PMAX;          // F, NMAX x NX
  static constexpr int oA = oF + NMAX * NX;     // A, NX x NX
  static constexpr int oB = oA + NX * NX;       // B, NX x NU
  static constexpr int oX = oB + NX * NU;       // x_t
  static constexpr int oU = oX + NX;            // u_0
  static constexpr int oS = oU + NU;            // active-set flags (as T) for the shift
  static constexpr int size = oS + NMAX;
};

// Waves per SIMD the registers must allow.  A batch of 4096 is 1024 waves,
// one per SIMD: above BS = 2 the loop takes the whole register file (at 2
// waves per SIMD it spilled 176 B per lane at BS = 5).
template <typename T, int BS>
struct LoopOcc {
  static constexpr int w = BS <= 2 ? 4 : 1;
};

template <typename T, int NX, int NU, int BS>
__global__ __launch_bounds__(64, (LoopOcc<T, BS>::w)) void box_loop_kernel(LoopArgs<T> a) {
  using Lq = LoopLds<T, NX, NU, BS>;
  using Box = QBoxLds<T, BS>;
  constexpr int NMAX = Lq::NMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int lane = threadIdx.x, g = lane >> 4, q = lane & 15;
  const int b = blockIdx.x * 4 + g;
  const bool live = b < a.batch;
  const int bl = live ? b : 0;
  const int n = a.n, nx = a.nx, nu = a.nu, P = n * (n + 1) / 2;
  T* gs = reinterpret_cast<T*>(smem_raw) + g * Lq::size;
  T* gb = gs + Box::oBuf;
  T* fs = gs + Box::oF;
  T* lbs = gs + Box::oLb;
  T* ubs = gs + Box::oUb;
  T* Ps = gs + Lq::oP;
  T* Fs = gs + Lq::oF;
  T* As = gs + Lq::oA;
  T* Bs = gs + Lq::oB;
  T* xg = gs + Lq::oX;
  T* ug = gs + Lq::oU;
  T* sg = gs + Lq::oS;

  // ------------------------------------------------------------- stage in
  {
    const T* Hb = a.H + (int64_t)bl * a.sH;
    for (int e = q; e < Lq::PMAX; e += 16) Ps[e] = e < P ? Hb[e] : T(0);
    const T* Fb = a.F + (int64_t)bl * a.sF;
    for (int e = q; e < NMAX * NX; e += 16) {
      const int i = e / NX, j = e - i * NX;
      Fs[e] = (i < n && j < nx) ? Fb[i * nx + j] : T(0);
    }
    for (int e = q; e < NX * NX; e += 16) {
      const int i = e / NX, j = e - i * NX;
      As[e] = (i < nx && j < nx) ? a.A[(int64_t)bl * a.sA + i * nx + j] : T(0);
    }
    for (int e = q; e < NX * NU; e += 16) {
      const int i = e / NU, j = e - i * NU;
      Bs[e] = (i < nx && j < nu) ? a.B[(int64_t)bl * a.sB + i * nu + j] : T(0);
    }
    if (q < NX) xg[q] = q < nx ? a.x0[(int64_t)bl * a.sX0 + q] : T(0);
  }
  bool nonfinite = false, badbox = false;
  for (int i = q; i < NMAX; i += 16) {
    const bool v = live && i < n;
    const T li = (v && a.lb) ? a.lb[(int64_t)b * a.slb + i] : -Lim<T>::inf();
    const T ui = (v && a.ub) ? a.ub[(int64_t)b * a.sub + i] : Lim<T>::inf();
    lbs[i] = li;
    ubs[i] = ui;
    badbox |= v && (!(li <= ui) || li == Lim<T>::inf() || ui == -Lim<T>::inf());
  }
  __syncthreads();
  for (int e = q; e < P; e += 16) nonfinite |= live && !finite(Ps[e]);
  const unsigned long long gmask = 0xFFFFull << (16 * g);
  const int code0 = ((__ballot(nonfinite) & gmask) != 0)
                        ? MPCQP_STATUS_NONFINITE
                        : (((__ballot(badbox) & gmask) != 0) ? MPCQP_STATUS_INFEASIBLE
                                                              : MPCQP_STATUS_OPTIMAL);

#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  QSym<T, BS> M;
  M.init(lane);
  int st[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) st[r] = (M.bi * BS + r < n) ? 0 : 3;  // cold first step

  for (int t = 0; t < a.steps; ++t) {
    // record x_t; f = F x_t (rows q, q + 16 of the group)
    if (live && q < nx) a.xs[((int64_t)t * a.batch + b) * nx + q] = xg[q];
    for (int i = q; i < NMAX; i += 16) {
      T s = T(0);
#pragma unroll
      for (int j = 0; j < NX; ++j) s = fma(Fs[i * NX + j], xg[j], s);
      fs[i] = s;
    }
    lds_exchange();
    bool nf = false;
    M.load_packed(Ps, n, nf);
    // sweep H on the free rows of the warm-start set: free-row mask of the
    // group (rows bi*BS + r from the bj == 0 lanes)
    unsigned fmask = 0;
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const unsigned long long bal = __ballot(M.bj == 0 && st[r] == 0);
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
        if ((bal >> (16 * g + 4 * bb)) & 1ull) fmask |= 1u << (bb * BS + r);
    }
    int code = code0;
    int sweeps = 0;
    bool okp = true;
    while (__any(fmask != 0)) {
      const bool has = fmask != 0;
      const int k = has ? __builtin_ctz(fmask) : 0;
      fmask = has ? fmask & (fmask - 1) : 0u;
      T colr[BS], colc[BS];
      const T d = M.column(k, gb, colr, colc);
      if (has) {
        okp = okp && d > T(0);
        M.sweep_col(k, T(1), d, colr, colc);
        ++sweeps;
      }
    }
    if (code == MPCQP_STATUS_OPTIMAL && !okp) code = MPCQP_STATUS_NOT_CONVEX;
    T zr[BS];
    int iters = 0;
    const int c2 = gi_box_st<T, BS, true>(M, gb, fs, lbs, ubs, n, a.max_iter, a.tol,
                                          live && code == MPCQP_STATUS_OPTIMAL, zr, iters, st
                                          MPCQP_CLK_ARG);
    if (code == MPCQP_STATUS_OPTIMAL) code = c2;
    const bool okc = code == MPCQP_STATUS_OPTIMAL || code == MPCQP_STATUS_MAXITER;
    if (!okc) {
#pragma unroll
      for (int r = 0; r < BS; ++r) zr[r] = __builtin_nan("");
    }
    // outputs of the step; u_0 and the active set through LDS
    if (M.bj == 0) {
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const int i = M.bi * BS + r;
        if (i < NU) ug[i] = zr[r];
        if (i < NMAX) sg[i] = (T)st[r];
        if (live && a.zs && i < n) a.zs[((int64_t)t * a.batch + b) * n + i] = zr[r];
      }
    }
    if (live && q == 0)
      a.status[(int64_t)t * a.batch + b] = (code & 0xff) | (((iters + sweeps) & 0xffff) << 8);
    lds_exchange();
    if (live && q < nu) a.us[((int64_t)t * a.batch + b) * nu + q] = ug[q];
    // plant: x_{t+1} = A x_t + B u_0
    T xn = T(0);
    if (q < NX) {
#pragma unroll
      for (int j = 0; j < NX; ++j) xn = fma(As[q * NX + j], xg[j], xn);
#pragma unroll
      for (int j = 0; j < NU; ++j) xn = fma(Bs[q * NU + j], ug[j], xn);
    }
    // warm start of the next step: row i takes row i + nu's state (the last
    // stage keeps its own); a failed step restarts cold
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      const int src = i + nu < n ? i + nu : i;
      st[r] = i < n ? (okc ? (int)sg[src] : 0) : 3;
    }
    lds_exchange();
    if (q < NX) xg[q] = xn;
    lds_exchange();
  }
  if (live && q < nx) a.xs[((int64_t)a.steps * a.batch + b) * nx + q] = xg[q];
}

template <typename T, int NX, int NU, int BS>
static int launch_loop(const LoopArgs<T>& a, hipStream_t st) {
  using Lq = LoopLds<T, NX, NU, BS>;
  const size_t bytes = (size_t)4 * Lq::size * sizeof(T);
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)box_loop_kernel<T, NX, NU, BS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(box_loop)");
  }
  hipLaunchKernelGGL((box_loop_kernel<T, NX, NU, BS>), dim3((unsigned)((a.batch + 3) / 4)),
                     dim3(64), bytes, st, a);
  MPCQP_CHECK_LAUNCH("box_loop_kernel");
  return MPCQP_OK;
}

template <typename T, int NX, int NU>
static int loop_bs(const LoopArgs<T>& a, hipStream_t st) {
  switch ((a.n + 3) / 4) {
    case 1: return launch_loop<T, NX, NU, 1>(a, st);
    case 2: return launch_loop<T, NX, NU, 2>(a, st);
    case 3: return launch_loop<T, NX, NU, 3>(a, st);
    case 4: return launch_loop<T, NX, NU, 4>(a, st);
    case 5: return launch_loop<T, NX, NU, 5>(a, st);
    case 6: return launch_loop<T, NX, NU, 6>(a, st);
    case 7: return launch_loop<T, NX, NU, 7>(a, st);
    default: return launch_loop<T, NX, NU, 8>(a, st);
  }
}

template <typename T>
static int loop_t(const LoopArgs<T>& a, hipStream_t st) {
  if (a.nx <= 2 && a.nu <= 1) return loop_bs<T, 2, 1>(a, st);
  if (a.nx <= 2 && a.nu <= 2) return loop_bs<T, 2, 2>(a, st);
  return loop_bs<T, 4, 2>(a, st);
}

}  // namespace mpcqp

extern "C" int mpcqp_mpc_box_loop(int dtype, int batch, int nx, int nu, int N, int steps,
                                  const void* H, int64_t strideH, const void* F, int64_t strideF,
                                  const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                                  const void* x0, int64_t strideX0, const void* lb,
                                  int64_t strideLb, const void* ub, int64_t strideUb, void* xs,
                                  void* us, void* zs, int32_t* status, int max_iter, double tol,
                                  void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_mpc_box_loop: bad dtype %d",
                  dtype);
  MPCQP_CHECK_ARG(batch >= 0 && N >= 1 && steps >= 0, "mpcqp_mpc_box_loop: bad sizes");
  MPCQP_CHECK_ARG(nx >= 1 && nx <= 4 && nu >= 1 && nu <= 2 && N * nu <= 32,
                  "mpcqp_mpc_box_loop: nx=%d nu=%d N=%d outside nx <= 4, nu <= 2, N*nu <= 32",
                  nx, nu, N);
  MPCQP_CHECK_ARG(H && F && A && Bm && x0 && xs && (steps == 0 || (us && status)),
                  "mpcqp_mpc_box_loop: H, F, A, B, x0, xs (and us, status for steps > 0) "
                  "are required");
  MPCQP_CHECK_ARG(strideH >= 0 && strideF >= 0 && strideA >= 0 && strideB >= 0 &&
                      strideX0 >= 0 && strideLb >= 0 && strideUb >= 0,
                  "mpcqp_mpc_box_loop: negative stride");
  if (batch == 0) return MPCQP_OK;
  auto fill = [&](auto& a, auto tp) {
    using T = decltype(tp);
    a.batch = batch; a.nx = nx; a.nu = nu; a.N = N; a.n = N * nu; a.steps = steps;
    a.H = (const T*)H; a.sH = strideH; a.F = (const T*)F; a.sF = strideF;
    a.A = (const T*)A; a.sA = strideA; a.B = (const T*)Bm; a.sB = strideB;
    a.x0 = (const T*)x0; a.sX0 = strideX0;
    a.lb = (const T*)lb; a.slb = strideLb; a.ub = (const T*)ub; a.sub = strideUb;
    a.xs = (T*)xs; a.us = (T*)us; a.zs = (T*)zs; a.status = status;
    a.max_iter = max_iter > 0 ? max_iter : 3 * N * nu + 30;
    a.tol = tol > 0 ? (T)tol : (dtype == MPCQP_F64 ? (T)1e-12 : (T)1e-6);
  };
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64) {
    LoopArgs<double> a;
    fill(a, 0.0);
    return loop_t(a, st);
  }
  LoopArgs<float> a;
  fill(a, 0.0f);
  return loop_t(a, st);
}
