// pfdyn.hpp -- shared by the product-form kernels (solve_pf.hip,
// solve_zf.hip): single-wave LDS helpers and the KKT residual of the MPC QP
// computed from the DYNAMICS in fp64 (dyn_residual).
#pragma once
#include "pf.hpp"

// tools/phase_timing.py dyn3|dyn5 builds with MPCQP_PHASE_DYN: the phase
// clock then times the DYN refinement (PHASE_D) instead of the active set
#ifdef MPCQP_PHASE_DYN
#define MPCQP_PHASE_K(i) \
  do {               \
  } while (0)
#define MPCQP_PHASE_D(i) MPCQP_PHASE(i)
#else
#define MPCQP_PHASE_K(i) MPCQP_PHASE(i)
#define MPCQP_PHASE_D(i) \
  do {               \
  } while (0)
#endif

namespace mpcqp {

// cnt floats from up to three contiguous global segments into LDS, every
// load of a 1024-float group issued before its first LDS store
template <int BATCH = 16>
__device__ __forceinline__ void lds_copy3(float* dst, const float* s1, int n1, const float* s2,
                                          int n2, const float* s3, int n3, int l) {
  const int cnt = n1 + n2 + n3;
  for (int e0 = 0; e0 < cnt; e0 += BATCH * kWave) {
    float t[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int e = e0 + l + kWave * k;
      const float* p = e < n1 ? s1 + e : (e < n1 + n2 ? s2 + (e - n1) : s3 + (e - n1 - n2));
      t[k] = e < cnt ? *p : 0.f;
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int e = e0 + l + kWave * k;
      if (e < cnt) dst[e] = t[k];
    }
  }
}

// The same copy by LDS DMA (global_load_lds_dword: global memory straight
// into LDS at M0 + 4 lane, no VGPR staging): every load of the whole copy is
// in flight at once -- one HBM round trip per copy instead of one per
// register batch -- then vmcnt(0).  The caller syncs before the LDS reads.
__device__ __forceinline__ void lds_copy3_dma(float* dst, const float* s1, int n1, const float* s2,
                                              int n2, const float* s3, int n3, int l) {
  typedef __attribute__((address_space(3))) void* lptr_t;
  typedef __attribute__((address_space(1))) void* gptr_t;
  const int cnt = n1 + n2 + n3;
  for (int e0 = 0; e0 < cnt; e0 += kWave) {
    const int e = e0 + l;
    if (e < cnt) {
      const float* p = e < n1 ? s1 + e : (e < n1 + n2 ? s2 + (e - n1) : s3 + (e - n1 - n2));
      __builtin_amdgcn_global_load_lds((gptr_t)p, (lptr_t)(dst + e0), 4, 0, 0);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt untouched
}

__device__ __forceinline__ float bperm(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(lane << 2, __float_as_int(v)));
}


template <int NR, typename V>
__device__ __forceinline__ V pick(const V (&x)[NR], int i) {
  // value at index i (uniform) from lane i % 64, register i / 64: read every
  // register's lane, then select on the (scalar) results -- a select over
  // x[r] first gets folded into a dynamically indexed private array (scratch)
  V v = readlane(x[0], i & 63);
#pragma unroll
  for (int r = 1; r < NR; ++r) {
    const V w = readlane(x[r], i & 63);
    v = ((i >> 6) == r) ? w : v;
  }
  return v;
}

template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffffll), CTRL, 0xF, 0xF, MPCQP_DPP_BC);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xF, 0xF, MPCQP_DPP_BC);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Sum over groups of P lanes (P = 2 or 4, wave-uniform), result in every lane.
__device__ __forceinline__ double group_sum(double v, int P) {
  v += dppd<0xB1>(v);             // quad_perm [1,0,3,2]
  if (P == 4) v += dppd<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}

// KKT residual of the condensed QP from the dynamics, in fp64 (DYN pf
// kernels).  x + xl (a float pair): z (i < n) and the signed row multipliers
// (rows i >= n, the state box on x_1..x_N in stage-major order).  Out: w_i = (H z + f + G'mu)_i
// on free z, (G z - h)_i = x_k(z)_c - xlo/xhi on active rows, 0 elsewhere.
//   forward   x_{s+1} = A_s x_s + B_s u_s + c_s
//   backward  lam_N = Qf x_N + mu_N,  g_s = R u_s + B_s' lam_{s+1},
//             lam_s = Q x_s + mu_s + A_s' lam_{s+1}
// Every matrix-vector row is a dot product over 4 lanes (row r = lane / 4)
// whose NXP/2 terms per lane are unrolled at compile time (NXP >= nx, nu,
// the padded terms are masked), so a stage costs one LDS round trip.
// Stage data (A_s, B_s, c_s) streams through the pool in runs of `cap`
// stages, visited forward 0..K-1 then backward K-1..0 (`loaded` = the
// resident run; a horizon that fits one run is loaded once per kernel).
// Measured: register prefetching of the next run (8-16 VGPRs) cost more in
// spills and short runs than the round trips it hid; a run is now copied by
// LDS DMA, all of it in flight at once (lds_copy3_dma).
// FWD: the forward rollout only (X = x_1..x_N of z into the pool; w untouched)
// RESIDENT: the whole horizon and the weights are already in the pool (an
// earlier call loaded them, one run): no load code at all (register pressure)
template <int NR, int NXP, bool FWD = false, bool RESIDENT = false>
__device__ __forceinline__ void dyn_residual(const PfDyn& d, int b, int n, int m, int l,
                                             const float (&x)[NR], const float* xl,
                                             const int (&st)[NR],
                                             double* pool, int& loaded,
                                             float (&w)[NR] MPCQP_CLK_PARAM) {
  static_assert(NXP % 4 == 0 && NXP <= 16, "4 lanes per row, at most 16 rows");
  // an opaque copy of the lane id: the per-lane LDS addresses below are then
  // computed where they are used instead of being hoisted out of the caller's
  // loops (where they would stay live across the caller's whole loop body)
  asm volatile("" : "+v"(l));
  constexpr int TT = NXP / 2;  // terms per lane: 2*NXP padded terms over 4 lanes
  const int nx = d.nx, nu = d.nu, N = d.N, tv = d.tv;
  double* xd = pool + kDynXd;
  double* lam = pool + kDynLam;
  double* X = pool + kDynX;
  float* Qs = reinterpret_cast<float*>(X + (N + 1) * nx);
  float* Qfs = Qs + nx * nx;
  float* Rs = Qfs + nx * nx;
  float* ch = reinterpret_cast<float*>(X + (N + 1) * nx + (2 * nx * nx + nu * nu + 1) / 2);
  const int cap = dyn_chunk_stages(nx, nu, N);
  const int K = (N + cap - 1) / cap;
  const int sfA = nx * nx, sfB = nx * nu;
  const float* Ab = d.A + (int64_t)b * d.sA;
  const float* Bb = d.B + (int64_t)b * d.sB;
  const float* cb = d.c ? d.c + (int64_t)b * d.sC : nullptr;
  const int i4 = l >> 2, q = l & 3;

  // run r: stages [r cap, r cap + S); LDS image A_c (S or 1) | B_c | c_c (S)
  auto run_len = [&](int r) { return N - r * cap < cap ? N - r * cap : cap; };
  auto chA = [&](int S, int t) { return ch + (tv ? t * sfA : 0); };
  auto chB = [&](int S, int t) { return ch + (tv ? S * sfA : sfA) + (tv ? t * sfB : 0); };
  auto chC = [&](int S, int t) { return ch + (tv ? S * (sfA + sfB) : sfA + sfB) + t * nx; };
  // run r into LDS: every load of a 16-register batch issued before its
  // first LDS store
  auto load_run = [&](int r) __attribute__((always_inline)) {
    const int s0 = r * cap, S = run_len(r);
#ifndef MPCQP_DYN_VGPR_COPY
    lds_copy3_dma(ch, Ab + (tv ? (int64_t)s0 * sfA : 0), tv ? S * sfA : sfA,
                  Bb + (tv ? (int64_t)s0 * sfB : 0), tv ? S * sfB : sfB,
                  cb ? cb + (int64_t)s0 * nx : nullptr, cb ? S * nx : 0, l);
#else  // (A/B: through VGPRs in register batches)
    lds_copy3<NXP >= 8 ? 8 : 16>(ch, Ab + (tv ? (int64_t)s0 * sfA : 0), tv ? S * sfA : sfA,
              Bb + (tv ? (int64_t)s0 * sfB : 0), tv ? S * sfB : sfB,
              cb ? cb + (int64_t)s0 * nx : nullptr, cb ? S * nx : 0, l);
#endif
    loaded = r;
  };
  if (!RESIDENT && loaded < 0)
    lds_copy3(Qs, d.Q + (int64_t)b * d.sQ, sfA, d.Qf + (int64_t)b * d.sQf, sfA,
              d.R + (int64_t)b * d.sR, nu * nu, l);

  // x0, u and the row multipliers into LDS
  if (l < nx) X[l] = (double)d.x0[(int64_t)b * d.sX0 + l];
#pragma unroll
  for (int r = 0; r < NR; ++r) xd[l + kWave * r] = (double)x[r] + (double)xl[l + kWave * r];

  auto fwd_run = [&](int r) __attribute__((always_inline)) {
    const int s0 = r * cap, S = run_len(r);
    const bool row = i4 < nx;
    for (int t = 0; t < S; ++t) {
      const int s = s0 + t;
      const float* As = chA(S, t);
      const float* Bs = chB(S, t);
      const float cs = (cb && row) ? chC(S, t)[i4] : 0.f;
      double acc = 0.0;
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const int k = q + 4 * tt;
        bool ok;
        float cf;
        double v;
        if (4 * tt < NXP) {  // A_s row i4 . x_s
          ok = row && k < nx;
          cf = As[ok ? i4 * nx + k : 0];
          v = X[s * nx + (ok ? k : 0)];
        } else {             // B_s row i4 . u_s
          const int k2 = k - NXP;
          ok = row && k2 < nu;
          cf = Bs[ok ? i4 * nu + k2 : 0];
          v = xd[s * nu + (ok ? k2 : 0)];
        }
        acc = fma(ok ? (double)cf : 0.0, v, acc);
      }
      acc = group_sum(acc, 4);
      if (row && q == 0) X[(s + 1) * nx + i4] = acc + (double)cs;
      wave_lds_sync();
    }
  };
  // one backward sub-step for rows of one kind: g rows (a = row) or lam rows
  auto bwd_rows = [&](int s, int S, int t, const double* ln, bool isg, bool isl, int rr)
      __attribute__((always_inline)) {
    const float* As = chA(S, t);
    const float* Bs = chB(S, t);
    double acc = 0.0;
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const int k = q + 4 * tt;
      bool ok;
      float cf;
      double v;
      if (4 * tt < NXP) {  // A_s col / B_s col . lam_{s+1}
        ok = (isl || isg) && k < nx;
        cf = isl ? As[ok ? k * nx + rr : 0] : Bs[ok ? k * nu + rr : 0];
        v = ln[ok ? k : 0];
      } else {             // Q x_s / R u_s
        const int k2 = k - NXP;
        ok = isl ? k2 < nx : (isg && k2 < nu);
        cf = isl ? Qs[ok ? rr * nx + k2 : 0] : Rs[ok ? rr * nu + k2 : 0];
        v = isl ? X[s * nx + (ok ? k2 : 0)] : xd[s * nu + (ok ? k2 : 0)];
      }
      acc = fma(ok ? (double)cf : 0.0, v, acc);
    }
    return group_sum(acc, 4);
  };
  auto bwd_run = [&](int r) __attribute__((always_inline)) {
    const int s0 = r * cap, S = run_len(r);
    const bool one = nx + nu <= 16;  // lam and g rows side by side
    for (int t = S - 1; t >= 0; --t) {
      const int s = s0 + t;
      const double* ln = lam + ((s + 1) & 1) * 16;  // lam_{s+1}
      if (one) {
        const bool isl = i4 < nx && s >= 1, isg = i4 >= nx && i4 < nx + nu;
        const int rr = isl || i4 < nx ? i4 : i4 - nx;
        const double acc = bwd_rows(s, S, t, ln, isg, isl, rr);
        if (q == 0) {
          if (isl) lam[(s & 1) * 16 + rr] = acc + (m ? xd[n + (s - 1) * nx + rr] : 0.0);
          if (isg) xd[s * nu + rr] = acc;
        }
      } else {
        const bool isg = i4 < nu, isl = i4 < nx && s >= 1;
        const double ag = bwd_rows(s, S, t, ln, isg, false, i4);
        const double al = bwd_rows(s, S, t, ln, false, isl, i4);
        if (q == 0) {
          if (isl) lam[(s & 1) * 16 + i4] = al + (m ? xd[n + (s - 1) * nx + i4] : 0.0);
          if (isg) xd[s * nu + i4] = ag;
        }
      }
      wave_lds_sync();
    }
  };

  for (int p = 0; p < (FWD ? K : 2 * K); ++p) {
    const bool fw = p < K;
    const int r = fw ? p : 2 * K - 1 - p;
    if (!RESIDENT && loaded != r) {
      wave_lds_sync();  // the previous run's readers are done
      load_run(r);
    }
    wave_lds_sync();
    MPCQP_PHASE_D(1);
    if (p == K) {  // lam_N = Qf x_N + mu_N
      double acc = 0.0;
#pragma unroll
      for (int tt = 0; tt < NXP / 4; ++tt) {
        const int k = q + 4 * tt;
        const bool ok = i4 < nx && k < nx;
        acc = fma(ok ? (double)Qfs[ok ? i4 * nx + k : 0] : 0.0, X[N * nx + (ok ? k : 0)], acc);
      }
      acc = group_sum(acc, 4);
      if (i4 < nx && q == 0) lam[(N & 1) * 16 + i4] = acc + (m ? xd[n + (N - 1) * nx + i4] : 0.0);
      wave_lds_sync();
    }
    if (fw) {
      fwd_run(r);
      MPCQP_PHASE_D(2);
    } else {
      bwd_run(r);
      MPCQP_PHASE_D(3);
    }
  }
  if constexpr (FWD) {
    wave_lds_sync();
    return;
  }
  // ---- residual on the working set
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int i = l + kWave * r;
    const bool isz = i < n;
    const bool act = st[r] == 1 || st[r] == 2;
    double e = 0.0;
    if (isz) {
      e = xd[i];
    } else if (act && i < n + m) {
      const int j = i - n;
      const float* bp = (st[r] == 1) ? d.xlo : d.xhi;
      e = X[nx + j] - (double)bp[(int64_t)b * d.sXb + j];
    }
    const bool inS = isz ? (st[r] == 0) : act;
    w[r] = (inS && i < n + m) ? (float)e : 0.f;
  }
  wave_lds_sync();
  MPCQP_PHASE_D(4);
}


// The resident stage run of the DYN pool layout when the whole horizon fits
// one run (dyn_chunk_stages >= N): A_s, B_s as floats in LDS.
struct DynChunk {
  const float* ch;
  int N, sfA, sfB, tv;
  __device__ __forceinline__ const float* A(int t) const { return ch + (tv ? t * sfA : 0); }
  __device__ __forceinline__ const float* B(int t) const {
    return ch + (tv ? N * sfA : sfA) + (tv ? t * sfB : 0);
  }
};
__device__ __forceinline__ DynChunk dyn_chunk(const PfDyn& d, double* pool) {
  const int nx = d.nx, nu = d.nu, N = d.N;
  const double* X = pool + kDynX;
  DynChunk c;
  c.ch = reinterpret_cast<const float*>(X + (N + 1) * nx + (2 * nx * nx + nu * nu + 1) / 2);
  c.N = N;
  c.sfA = nx * nx;
  c.sfB = nx * nu;
  c.tv = d.tv;
  return c;
}

}  // namespace mpcqp
