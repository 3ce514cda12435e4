// quad_box.hip -- the box-QP kernels for n <= 32 with FOUR instances per
// wavefront (quad.hpp): one QP per 16-lane DPP row on a 4 x 4 grid of register
// blocks.  Two kernels:
//   box_quad_kernel  -- mpcqp_solve_box: packed H in, n sweeps form -H^{-1},
//                       then the group-wise Goldfarb-Idnani active set;
//   mpc_quad_kernel  -- mpcqp_mpc_box: per-instance plant in, Riccati-built
//                       -H^{-1} (see mpc_box.hip for the derivation), same
//                       active set; nothing but (A, B, x0, bounds) and z cross HBM.
#include "quad.hpp"
#include "quad_api.hpp"

namespace mpcqp {

template <typename T, int BS>
struct QuadOcc {
  // fp64 BS = 5 (n = 17..20, BASELINE config 2) needs ~190 VGPRs
  static constexpr int w = sizeof(T) == 8 ? (BS <= 3 ? 4 : (BS == 4 ? 3 : (BS == 5 ? 2 : 1)))
                                           : (BS <= 3 ? 4 : (BS <= 5 ? 3 : 2));
};

template <typename T, int BS>
__global__ __launch_bounds__(64, (QuadOcc<T, BS>::w)) void box_quad_kernel(BoxArgsQ<T> a) {
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  using L = QBoxLds<T, BS>;
  constexpr int NMAX = L::NMAX;
  constexpr int PMAX = NMAX * (NMAX + 1) / 2;
  constexpr int GSZ = L::size + PMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int lane = threadIdx.x, g = lane >> 4, q = lane & 15;
  const int b = blockIdx.x * 4 + g;
  const bool live = b < a.batch;
  const int bl = live ? b : 0;
  const int n = a.n, P = n * (n + 1) / 2;
  T* gs = reinterpret_cast<T*>(smem_raw) + g * GSZ;
  T* gb = gs + L::oBuf;
  T* fs = gs + L::oF;
  T* lbs = gs + L::oLb;
  T* ubs = gs + L::oUb;
  T* Ps = gs + L::size;
  {
    constexpr int MAXT = (PMAX + 15) / 16;
    const T* Hb = a.H + (int64_t)bl * a.sH;
    T tmp[MAXT];
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const int e = q + 16 * t;
      tmp[t] = (e < P) ? Hb[e] : T(0);
    }
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const int e = q + 16 * t;
      if (e < P) Ps[e] = tmp[t];
    }
  }
  bool nonfinite = false, badbox = false;
  for (int i = q; i < NMAX; i += 16) {
    const bool v = live && i < n;
    const T fi = v ? a.f[(int64_t)b * a.sf + i] : T(0);
    const T li = (v && a.lb) ? a.lb[(int64_t)b * a.slb + i] : -Lim<T>::inf();
    const T ui = (v && a.ub) ? a.ub[(int64_t)b * a.sub + i] : Lim<T>::inf();
    fs[i] = fi;
    lbs[i] = li;
    ubs[i] = ui;
    nonfinite |= v && !finite(fi);
    badbox |= v && (!(li <= ui) || li == Lim<T>::inf() || ui == -Lim<T>::inf());
  }
  __syncthreads();
  QSym<T, BS> M;
  M.init(lane);
  M.load_packed(Ps, n, nonfinite);
  // group-wide flags (OR over the 16 lanes of the row)
  const unsigned long long gmask = 0xFFFFull << (16 * g);
  const bool g_nonfinite = (__ballot(nonfinite) & gmask) != 0;
  const bool g_badbox = (__ballot(badbox) & gmask) != 0;
  int code = MPCQP_STATUS_OPTIMAL;
  if (g_nonfinite) code = MPCQP_STATUS_NONFINITE;
  else if (g_badbox) code = MPCQP_STATUS_INFEASIBLE;
  bool ok = true;
  for (int k = 0; k < n; ++k) {
    const T d = M.sweep(k, T(1), gb);
    ok &= d > T(0);
  }
  if (code == MPCQP_STATUS_OPTIMAL && !ok) code = MPCQP_STATUS_NOT_CONVEX;
  T zr[BS];
  int iters = 0;
  const int c2 = gi_box<T, BS>(M, gb, fs, lbs, ubs, n, a.max_iter, a.tol,
                                    live && code == MPCQP_STATUS_OPTIMAL, zr, iters MPCQP_CLK_ARG);
  if (code == MPCQP_STATUS_OPTIMAL) code = c2;
  if (code != MPCQP_STATUS_OPTIMAL && code != MPCQP_STATUS_MAXITER) {
#pragma unroll
    for (int r = 0; r < BS; ++r) zr[r] = __builtin_nan("");
  }
  if (live && M.bj == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      if (i < n) a.z[(int64_t)b * n + i] = zr[r];
    }
  }
  if (live && q == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
}

// ----------------------------------------------------------- fused kernel
template <typename T, int NX, int NU, class Mat>
struct QMpcLds {
  int oA, oB, oQ, oQf, oR, oC, oX0, oK, oSi, oAcl, oX, oKf, oMinv, total, ld;
  __host__ __device__ QMpcLds(int N, int n, int tv) {
    const int S = tv ? N : 1;
    oA = GBoxLds<Mat>::size;
    oB = oA + S * NX * NX;
    oQ = oB + S * NX * NU;
    oQf = oQ + NX * NX;
    oR = oQf + NX * NX;
    oC = oR + NU * NU;
    oX0 = oC + N * NX;
    oK = oX0 + NX;
    oSi = oK + N * NU * NX;
    oAcl = oSi + N * NU * NU;
    oX = oAcl + N * NX * NX;
    oKf = oX + (N + 1) * NX;
    oMinv = oKf + N * n * NU;
    ld = n + 1;
    total = (oMinv + n * ld + 1) & ~1;  // keep every group's base 16-byte aligned
  }
};

template <typename T, int NX, int NU>
__device__ __forceinline__ void load_sq(const T* s, T (&m)[NX][NU], int ld) {
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NU; ++j) m[i][j] = s[i * ld + j];
}

template <typename T, int NX, int BS>
struct QMpcOcc {
  static constexpr int w = NX <= 2 ? QuadOcc<T, BS>::w : (QuadOcc<T, BS>::w < 2 ? 1 : 2);
};

// GL lanes per QP (16 with QSym: four QPs per wave); OCC: minimum waves per
// SIMD the register allocation must allow.  Measured and rejected: two QPs
// per wave (32-lane groups, 3 x 5 blocks at n = 20, row-block reductions
// through v_permlane16_swap): 73.1 vs 70.6 us at config 2 -- the per-wave
// fixed work (Riccati, x-bar/adjoint chains, reductions) doubles per QP, so
// VALU instructions per QP rose 47 % (PMC SQ_INSTS_VALU) while the two waves
// per SIMD hid only part of it.
#ifdef MPCQP_WAVE_CLOCK
// Debug library only (tools/wave_clock.py): per wave of mpc_group_kernel, the
// s_memrealtime (100 MHz, chip-wide) at entry and at exit and the largest GI
// iteration count of the wave's QPs -- the distribution of wave end times
// against the kernel's slowest wave.
constexpr int kWaveClockMax = 16384;
__device__ unsigned long long mpcqp_wave_clock[3 * kWaveClockMax];
#endif

template <typename T, int NX, int NU, class Mat, int GL, int OCC>
__global__ __launch_bounds__(64, OCC) void mpc_group_kernel(MpcArgsQ<T> a) {
#ifdef MPCQP_WAVE_CLOCK
  const unsigned long long wclk0 = __builtin_amdgcn_s_memrealtime();
#endif
  using BL = GBoxLds<Mat>;
  constexpr int NV = BL::NV;
  constexpr int RPL = Mat::RPL;
  constexpr int GPW = kWave / GL;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int lane = threadIdx.x, g = lane / GL, q = lane % GL;
  const int b = blockIdx.x * GPW + g;
  const bool live = b < a.batch;
  const int bl = live ? b : 0;
  const int nx = a.nx, nu = a.nu, N = a.N, n = N * nu, tv = a.tv;
  const int S = tv ? N : 1;
  const QMpcLds<T, NX, NU, Mat> L(N, n, tv);
  T* sm = reinterpret_cast<T*>(smem_raw) + g * L.total;
  T* gb = sm + BL::oBuf;
  T* fs = sm + BL::oF;
  T* lbs = sm + BL::oLb;
  T* ubs = sm + BL::oUb;
  T* As = sm + L.oA;
  T* Bs = sm + L.oB;
  T* Qs = sm + L.oQ;
  T* Qfs = sm + L.oQf;
  T* Rs = sm + L.oR;
  T* Cs = sm + L.oC;
  T* X0s = sm + L.oX0;
  T* Ks = sm + L.oK;
  T* Sis = sm + L.oSi;
  T* Acls = sm + L.oAcl;
  T* Xs = sm + L.oX;
  T* Kfs = sm + L.oKf;
  T* Mv = sm + L.oMinv;
  const int ld = L.ld;

#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  // ------------------------------------------------------------- stage in
  bool nonfinite = false, badbox = false;
  {
    const T* Ab = a.A + (int64_t)bl * a.sA;
    for (int e = q; e < S * NX * NX; e += GL) {
      const int s = e / (NX * NX), r = (e / NX) % NX, cc = e % NX;
      const T v = (r < nx && cc < nx) ? Ab[(int64_t)s * nx * nx + r * nx + cc] : T(0);
      As[e] = v;
      nonfinite |= !finite(v);
    }
    const T* Bb = a.B + (int64_t)bl * a.sB;
    for (int e = q; e < S * NX * NU; e += GL) {
      const int s = e / (NX * NU), r = (e / NU) % NX, cc = e % NU;
      const T v = (r < nx && cc < nu) ? Bb[(int64_t)s * nx * nu + r * nu + cc] : T(0);
      Bs[e] = v;
      nonfinite |= !finite(v);
    }
    for (int e = q; e < NX * NX; e += GL) {
      const int r = e / NX, cc = e % NX;
      const bool in = live && r < nx && cc < nx;
      Qs[e] = in ? a.Q[(int64_t)b * a.sQ + r * nx + cc] : T(0);
      Qfs[e] = in ? a.Qf[(int64_t)b * a.sQf + r * nx + cc] : T(0);
    }
    for (int e = q; e < NU * NU; e += GL) {
      const int r = e / NU, cc = e % NU;
      // padded inputs get R = I so that S_k stays invertible (their B cols are 0)
      Rs[e] = (live && r < nu && cc < nu) ? a.R[(int64_t)b * a.sR + r * nu + cc] : (r == cc ? T(1) : T(0));
    }
    const T* Cb = (live && a.c) ? a.c + (int64_t)b * a.sC : nullptr;
    for (int e = q; e < N * NX; e += GL) {
      const int k = e / NX, cc = e % NX;
      Cs[e] = (Cb && cc < nx) ? Cb[k * nx + cc] : T(0);
    }
    if (q < NX) X0s[q] = (live && a.x0 && q < nx) ? a.x0[(int64_t)b * a.sX0 + q] : T(0);
    for (int i = q; i < NV; i += GL) {
      const bool v = live && i < n;
      const T li = (v && a.lb) ? a.lb[(int64_t)b * a.slb + i] : -Lim<T>::inf();
      const T ui = (v && a.ub) ? a.ub[(int64_t)b * a.sub + i] : Lim<T>::inf();
      lbs[i] = li;
      ubs[i] = ui;
      fs[i] = T(0);
      badbox |= v && (!(li <= ui) || li == Lim<T>::inf() || ui == -Lim<T>::inf());
    }
  }
  __syncthreads();

  int code = MPCQP_STATUS_OPTIMAL;
  MPCQP_PHASE(0);
  // -------------- Riccati backward + free response forward (all lanes, regs)
  // The two recursions are independent serial chains; one loop runs Riccati
  // stage N-1-t next to x-bar stage t so that their latencies overlap (at one
  // wave per SIMD nothing else hides them).
  {
    T P[NX][NX], Qr[NX][NX], Rr[NU][NU], Ar[NX][NX], Br[NX][NU], Ax[NX][NX];
    load_sq<T, NX, NX>(Qfs, P, NX);
    load_sq<T, NX, NX>(Qs, Qr, NX);
    load_sq<T, NU, NU>(Rs, Rr, NU);
    load_sq<T, NX, NX>(As, Ar, NX);
    load_sq<T, NX, NU>(Bs, Br, NU);
    load_sq<T, NX, NX>(As, Ax, NX);
    T xk[NX];
#pragma unroll
    for (int qq = 0; qq < NX; ++qq) xk[qq] = X0s[qq];
    bool ok = true;
    for (int t = 0; t < N; ++t) {
      {  // x-bar stage t: x_{t+1} = A_t x_t + c_t
        if (tv) load_sq<T, NX, NX>(As + t * NX * NX, Ax, NX);
        T xn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          T s = Cs[t * NX + i];
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) s = fma(Ax[i][qq], xk[qq], s);
          xn[i] = s;
        }
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) xk[qq] = xn[qq];
        if (q == 0)
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) Xs[(t + 1) * NX + qq] = xk[qq];
      }
      const int k = N - 1 - t;
      if (tv) {
        load_sq<T, NX, NX>(As + k * NX * NX, Ar, NX);
        load_sq<T, NX, NU>(Bs + k * NX * NU, Br, NU);
      }
      T PA[NX][NX], PB[NX][NU];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          T s = T(0);
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) s = fma(P[i][qq], Ar[qq][j], s);
          PA[i][j] = s;
        }
#pragma unroll
        for (int j = 0; j < NU; ++j) {
          T s = T(0);
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) s = fma(P[i][qq], Br[qq][j], s);
          PB[i][j] = s;
        }
      }
      T Sm[NU][NU], Y[NU][NX];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
#pragma unroll
        for (int j = 0; j < NU; ++j) {
          T s = Rr[i][j];
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) s = fma(Br[qq][i], PB[qq][j], s);
          Sm[i][j] = s;
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          T s = T(0);
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) s = fma(Br[qq][i], PA[qq][j], s);
          Y[i][j] = s;
        }
      }
      // S^{-1} by Gauss-Jordan (S symmetric positive definite)
      T Si[NU][NU];
#pragma unroll
      for (int i = 0; i < NU; ++i)
#pragma unroll
        for (int j = 0; j < NU; ++j) Si[i][j] = (i == j) ? T(1) : T(0);
#pragma unroll
      for (int p = 0; p < NU; ++p) {
        ok &= Sm[p][p] > T(0);
        const T rp = T(1) / Sm[p][p];
#pragma unroll
        for (int j = 0; j < NU; ++j) {
          Sm[p][j] *= rp;
          Si[p][j] *= rp;
        }
#pragma unroll
        for (int i = 0; i < NU; ++i) {
          if (i == p) continue;
          const T fct = Sm[i][p];
#pragma unroll
          for (int j = 0; j < NU; ++j) {
            Sm[i][j] = fma(-fct, Sm[p][j], Sm[i][j]);
            Si[i][j] = fma(-fct, Si[p][j], Si[i][j]);
          }
        }
      }
      T K[NU][NX];
#pragma unroll
      for (int i = 0; i < NU; ++i)
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          T s = T(0);
#pragma unroll
          for (int qq = 0; qq < NU; ++qq) s = fma(Si[i][qq], Y[qq][j], s);
          K[i][j] = -s;
        }
      if (q == 0) {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
#pragma unroll
          for (int j = 0; j < NX; ++j) Ks[(k * NU + i) * NX + j] = K[i][j];
#pragma unroll
          for (int j = 0; j < NU; ++j) Sis[(k * NU + i) * NU + j] = Si[i][j];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            T s = Ar[i][j];
#pragma unroll
            for (int qq = 0; qq < NU; ++qq) s = fma(Br[i][qq], K[qq][j], s);
            Acls[(k * NX + i) * NX + j] = s;
          }
      }
      if (k > 0) {
        // P <- Q + A'PA + (A'PB) K
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
          for (int j = 0; j < NX; ++j) {
            T s = Qr[i][j];
#pragma unroll
            for (int qq = 0; qq < NX; ++qq) s = fma(Ar[qq][i], PA[qq][j], s);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
              T apb = T(0);
#pragma unroll
              for (int qq = 0; qq < NX; ++qq) apb = fma(Ar[qq][i], PB[qq][u], apb);
              s = fma(apb, K[u][j], s);
            }
            P[i][j] = s;
          }
      }
    }
    if (!ok) code = MPCQP_STATUS_NOT_CONVEX;

    MPCQP_PHASE(1);
    // ---- adjoint y -> f (backward); x_k of the next stage is read from LDS
    // one iteration ahead so the read overlaps this stage's FMA chain
    __syncthreads();
    T yk[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      T s = T(0);
#pragma unroll
      for (int qq = 0; qq < NX; ++qq) s = fma(Qfs[i * NX + qq], xk[qq], s);
      yk[i] = s;
    }
    T xnext[NX];
#pragma unroll
    for (int qq = 0; qq < NX; ++qq) xnext[qq] = Xs[(N - 1) * NX + qq];
    for (int k = N - 1; k >= 0; --k) {
      // f_(k,u) = B_k[:,u]' y_{k+1}
      const T* Bk = Bs + (tv ? k : 0) * NX * NU;
      if (q == 0) {
        for (int u = 0; u < nu; ++u) {
          T s = T(0);
#pragma unroll
          for (int qq = 0; qq < NX; ++qq) s = fma(Bk[qq * NU + u], yk[qq], s);
          fs[k * nu + u] = s;
        }
      }
      if (k == 0) break;
      T xc[NX];
#pragma unroll
      for (int qq = 0; qq < NX; ++qq) {
        xc[qq] = xnext[qq];
        xnext[qq] = Xs[(k > 1 ? k - 1 : 1) * NX + qq];
      }
      if (tv) load_sq<T, NX, NX>(As + k * NX * NX, Ar, NX);
      T yn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T s = T(0);
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) s = fma(Qr[i][qq], xc[qq], s);
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) s = fma(Ar[qq][i], yk[qq], s);
        yn[i] = s;
      }
#pragma unroll
      for (int qq = 0; qq < NX; ++qq) yk[qq] = yn[qq];
    }
  }
  __syncthreads();

  MPCQP_PHASE(2);
  // ------------------------------ columns of -H^{-1}, one lane per column
  for (int c = q; c < n; c += GL) {
    const int jj = c / nu, bb = c - jj * nu;
    T s[NX], kf[NU];
    // k = jj: kff = S^{-1} e_b, s = -K' e_b
#pragma unroll
    for (int u = 0; u < NU; ++u) kf[u] = Sis[(jj * NU + u) * NU + bb];
#pragma unroll
    for (int qq = 0; qq < NX; ++qq) s[qq] = -Ks[(jj * NU + bb) * NX + qq];
#pragma unroll
    for (int u = 0; u < NU; ++u) Kfs[(jj * n + c) * NU + u] = kf[u];
    for (int k = jj - 1; k >= 0; --k) {
      const T* Bk = Bs + (tv ? k : 0) * NX * NU;
      T t[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        T v = T(0);
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) v = fma(Bk[qq * NU + u], s[qq], v);
        t[u] = v;
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        T v = T(0);
#pragma unroll
        for (int qq = 0; qq < NU; ++qq) v = fma(Sis[(k * NU + u) * NU + qq], t[qq], v);
        kf[u] = -v;
        Kfs[(k * n + c) * NU + u] = kf[u];
      }
      T sn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T v = T(0);
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) v = fma(Acls[(k * NX + qq) * NX + i], s[qq], v);
        sn[i] = v;
      }
#pragma unroll
      for (int qq = 0; qq < NX; ++qq) s[qq] = sn[qq];
    }
    // forward rollout from x_0 = 0
    T x[NX];
#pragma unroll
    for (int qq = 0; qq < NX; ++qq) x[qq] = T(0);
    for (int k = 0; k < N; ++k) {
      const T* Ak = As + (tv ? k : 0) * NX * NX;
      const T* Bk = Bs + (tv ? k : 0) * NX * NU;
      T u[NU];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        T v = (k <= jj) ? Kfs[(k * n + c) * NU + i] : T(0);
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) v = fma(Ks[(k * NU + i) * NX + qq], x[qq], v);
        u[i] = v;
      }
      for (int i = 0; i < nu; ++i) Mv[(k * nu + i) * ld + c] = -u[i];
      T xn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T v = T(0);
#pragma unroll
        for (int qq = 0; qq < NX; ++qq) v = fma(Ak[i * NX + qq], x[qq], v);
#pragma unroll
        for (int qq = 0; qq < NU; ++qq) v = fma(Bk[i * NU + qq], u[qq], v);
        xn[i] = v;
      }
#pragma unroll
      for (int qq = 0; qq < NX; ++qq) x[qq] = xn[qq];
    }
  }
  __syncthreads();

  MPCQP_PHASE(3);
  // ------------------------------------------------ box QP on M = -H^{-1}
  Mat M;
  M.init(lane);
  M.load_dense_sym(Mv, ld, n);
  for (int i = q; i < n; i += GL) nonfinite |= !finite(fs[i]);
  const unsigned long long gmask = (GL == 64 ? ~0ull : ((1ull << GL) - 1)) << (GL * g);
  if ((__ballot(nonfinite) & gmask) != 0) code = MPCQP_STATUS_NONFINITE;
  else if ((__ballot(badbox) & gmask) != 0) code = MPCQP_STATUS_INFEASIBLE;
  T zr[RPL];
  int iters = 0;
  const int c2 = gi_box<T, RPL>(M, gb, fs, lbs, ubs, n, a.max_iter, a.tol,
                                     live && code == MPCQP_STATUS_OPTIMAL, zr, iters MPCQP_CLK_ARG);
  if (code == MPCQP_STATUS_OPTIMAL) code = c2;
  MPCQP_PHASE(4);
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
  if (code != MPCQP_STATUS_OPTIMAL && code != MPCQP_STATUS_MAXITER) {
#pragma unroll
    for (int r = 0; r < RPL; ++r) zr[r] = __builtin_nan("");
  }
  if (live && M.bj == 0) {
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = M.bi * RPL + r;
      if (i < n) a.z[(int64_t)b * n + i] = zr[r];
    }
  }
  if (live && q == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
#ifdef MPCQP_WAVE_CLOCK
  {
    int itmax = 0;
#pragma unroll
    for (int gg = 0; gg < GPW; ++gg) {
      const int v = __builtin_amdgcn_readlane(iters, gg * GL);
      itmax = v > itmax ? v : itmax;
    }
    const unsigned long long wclk1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && blockIdx.x < kWaveClockMax) {
      mpcqp_wave_clock[3 * blockIdx.x] = wclk0;
      mpcqp_wave_clock[3 * blockIdx.x + 1] = wclk1;
      mpcqp_wave_clock[3 * blockIdx.x + 2] = (unsigned long long)itmax;
    }
  }
#endif
}

// ------------------------------------------------------------- launchers
template <typename T, int BS>
int launch_box_quad(const BoxArgsQ<T>& a, hipStream_t st) {
  using L = QBoxLds<T, BS>;
  constexpr int NMAX = L::NMAX;
  const size_t bytes = (size_t)4 * (L::size + NMAX * (NMAX + 1) / 2) * sizeof(T);
  hipLaunchKernelGGL((box_quad_kernel<T, BS>), dim3((a.batch + 3) / 4), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("box_quad_kernel");
  return MPCQP_OK;
}

template <typename T>
int solve_box_quad(const BoxArgsQ<T>& a, hipStream_t st) {
  switch ((a.n + 3) / 4) {
    case 1: return launch_box_quad<T, 1>(a, st);
    case 2: return launch_box_quad<T, 2>(a, st);
    case 3: return launch_box_quad<T, 3>(a, st);
    case 4: return launch_box_quad<T, 4>(a, st);
    case 5: return launch_box_quad<T, 5>(a, st);
    case 6: return launch_box_quad<T, 6>(a, st);
    case 7: return launch_box_quad<T, 7>(a, st);
    default: return launch_box_quad<T, 8>(a, st);
  }
}

template <typename T, int NX, int NU, class Mat, int GL, int OCC>
int launch_mpc_group(const MpcArgsQ<T>& a, hipStream_t st) {
  constexpr int GPW = kWave / GL;
  const int n = a.N * a.nu;
  const QMpcLds<T, NX, NU, Mat> L(a.N, n, a.tv);
  const size_t bytes = (size_t)GPW * L.total * sizeof(T);
  if (bytes > 160 * 1024) {
    set_error("mpcqp_mpc_box: LDS footprint %zu B > 160 KiB", bytes);
    return MPCQP_ENOTSUP;
  }
  auto kern = mpc_group_kernel<T, NX, NU, Mat, GL, OCC>;
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(mpc_group)");
  }
  hipLaunchKernelGGL(kern, dim3((a.batch + GPW - 1) / GPW), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("mpc_group_kernel");
  return MPCQP_OK;
}

// four QPs per wave (QSym, 16 lanes each)
template <typename T, int NX, int NU, int BS>
int launch_mpc_quad(const MpcArgsQ<T>& a, hipStream_t st) {
  return launch_mpc_group<T, NX, NU, QSym<T, BS>, 16, QMpcOcc<T, NX, BS>::w>(a, st);
}

template <typename T, int NX, int NU>
int mpc_quad_bs(const MpcArgsQ<T>& a, hipStream_t st) {
  switch ((a.N * a.nu + 3) / 4) {
    case 1: return launch_mpc_quad<T, NX, NU, 1>(a, st);
    case 2: return launch_mpc_quad<T, NX, NU, 2>(a, st);
    case 3: return launch_mpc_quad<T, NX, NU, 3>(a, st);
    case 4: return launch_mpc_quad<T, NX, NU, 4>(a, st);
    case 5: return launch_mpc_quad<T, NX, NU, 5>(a, st);
    case 6: return launch_mpc_quad<T, NX, NU, 6>(a, st);
    case 7: return launch_mpc_quad<T, NX, NU, 7>(a, st);
    default: return launch_mpc_quad<T, NX, NU, 8>(a, st);
  }
}

template <typename T>
int mpc_box_quad(const MpcArgsQ<T>& a, hipStream_t st) {
  if (a.nx <= 2 && a.nu == 1) return mpc_quad_bs<T, 2, 1>(a, st);
  if (a.nx <= 2) return mpc_quad_bs<T, 2, 2>(a, st);
  if (a.nu == 1) return mpc_quad_bs<T, 4, 1>(a, st);
  return mpc_quad_bs<T, 4, 2>(a, st);
}

template int solve_box_quad<double>(const BoxArgsQ<double>&, hipStream_t);
template int solve_box_quad<float>(const BoxArgsQ<float>&, hipStream_t);
template int mpc_box_quad<double>(const MpcArgsQ<double>&, hipStream_t);
template int mpc_box_quad<float>(const MpcArgsQ<float>&, hipStream_t);

}  // namespace mpcqp

#ifdef MPCQP_WAVE_CLOCK
extern "C" int mpcqp_debug_wave_clock(unsigned long long* out, int waves) {
  const int w = waves < mpcqp::kWaveClockMax ? waves : mpcqp::kWaveClockMax;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcqp::mpcqp_wave_clock),
                             3 * (size_t)w * sizeof(unsigned long long)) == hipSuccess ? 0 : -2;
}
#endif

#ifdef MPCQP_PHASE_TIMING
// Debug library only: read (and optionally reset) the phase counters.
MPCQP_DEBUG_PHASE_READER(mpcqp_debug_phase_cycles)
#endif
