// mpc_box.hip -- fused per-instance condense + input-box QP solve:
//
//   x_{k+1} = A_k x_k + B_k u_k + c_k,   lb <= u <= ub,
//   min  sum_{k<N} x_k'Q x_k + u_k'R u_k + x_N'Qf x_N        (main.py:86-106)
//
// i.e. MPCController.solve (session_4/main.py:115-116 / session4_sol.py:
// 128-129) for the input-box OCP, one instance per wavefront, nothing but the
// plant, x0 and the bounds read from HBM and only z written back.
//
// The box active set (gi_box_core.hpp) starts from M = -H^{-1}.  Instead of
// forming H and inverting it with n Gauss-Jordan sweeps, the kernel uses the
// problem's dynamic-programming structure: one backward Riccati pass
//     S_k = R + B_k'P_{k+1}B_k,  K_k = -S_k^{-1} B_k'P_{k+1}A_k,
//     P_k = Q + A_k'P_{k+1}A_k + A_k'P_{k+1}B_k K_k,   P_N = Qf
// (FHC.py:51-61 with time-varying A_k, B_k), after which column (j, b) of H^{-1}
// is the minimiser of the same LQ problem from x_0 = 0 with a unit linear
// cost on u_{j,b}:  a short backward affine pass from stage j
//     kff_j = S_j^{-1} e_b,  s_j = -K_j' e_b;  kff_k = -S_k^{-1} B_k' s_{k+1},
//     s_k = (A_k + B_k K_k)' s_{k+1}   (k < j)
// and one forward rollout  u_k = K_k x_k + kff_k,  x_{k+1} = A_k x_k + B_k u_k.
// One lane per column: O(N nx^2) per lane instead of O(n^3) sweeps.  The
// linear term f = Gam'Qhat xbar comes from the free response xbar and the
// adjoint y_k = Q xbar_k + A_k'y_{k+1} (as in condense.hip).
#include "gi_box_core.hpp"
#include "quad_api.hpp"

namespace mpcqp {

template <typename T>
struct MpcBoxArgs {
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

template <int NX, int BS>
struct MpcOcc {
  static constexpr int w = (NX <= 2 && BS <= 3) ? 4 : 2;
};

// LDS layout (T elements); the box-solver block comes first.
template <typename T, int NX, int NU, int BS>
struct MpcLds {
  int oA, oB, oQ, oQf, oR, oC, oX0, oK, oSi, oAcl, oX, oKf, oMinv, total, ld;
  __host__ __device__ MpcLds(int N, int n, int tv) {
    const int S = tv ? N : 1;
    oA = BoxLds<T, BS>::oEnd;
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
    total = oMinv + n * ld;
  }
};

template <typename T, int NX, int NU>
__device__ __forceinline__ void load_sq(const T* s, T (&m)[NX][NU], int ld) {
#pragma unroll
  for (int i = 0; i < NX; ++i)
#pragma unroll
    for (int j = 0; j < NU; ++j) m[i][j] = s[i * ld + j];
}

template <typename T, int NX, int NU, int BS>
__global__ __launch_bounds__(64, (MpcOcc<NX, BS>::w)) void mpc_box_kernel(MpcBoxArgs<T> a) {
  using BL = BoxLds<T, BS>;
  constexpr int NMAX = BL::NMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* sm = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int nx = a.nx, nu = a.nu, N = a.N, n = N * nu, tv = a.tv;
  const int S = tv ? N : 1;
  const MpcLds<T, NX, NU, BS> L(N, n, tv);
  T* buf = sm + BL::oBuf;
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

  // ------------------------------------------------------------- stage in
  bool nonfinite = false, badbox = false;
  {
    const T* Ab = a.A + (int64_t)b * a.sA;
    for (int e = lane; e < S * NX * NX; e += kWave) {
      const int s = e / (NX * NX), r = (e / NX) % NX, q = e % NX;
      const T v = (r < nx && q < nx) ? Ab[(int64_t)s * nx * nx + r * nx + q] : T(0);
      As[e] = v;
      nonfinite |= !finite(v);
    }
    const T* Bb = a.B + (int64_t)b * a.sB;
    for (int e = lane; e < S * NX * NU; e += kWave) {
      const int s = e / (NX * NU), r = (e / NU) % NX, q = e % NU;
      const T v = (r < nx && q < nu) ? Bb[(int64_t)s * nx * nu + r * nu + q] : T(0);
      Bs[e] = v;
      nonfinite |= !finite(v);
    }
    if (lane < NX * NX) {
      const int r = lane / NX, q = lane % NX;
      const bool in = r < nx && q < nx;
      Qs[lane] = in ? a.Q[(int64_t)b * a.sQ + r * nx + q] : T(0);
      Qfs[lane] = in ? a.Qf[(int64_t)b * a.sQf + r * nx + q] : T(0);
    }
    if (lane < NU * NU) {
      const int r = lane / NU, q = lane % NU;
      // padded inputs get R = I so that S_k stays invertible (their B cols are 0)
      Rs[lane] = (r < nu && q < nu) ? a.R[(int64_t)b * a.sR + r * nu + q] : (r == q ? T(1) : T(0));
    }
    const T* Cb = a.c ? a.c + (int64_t)b * a.sC : nullptr;
    for (int e = lane; e < N * NX; e += kWave) {
      const int k = e / NX, q = e % NX;
      Cs[e] = (Cb && q < nx) ? Cb[k * nx + q] : T(0);
    }
    if (lane < NX) X0s[lane] = (a.x0 && lane < nx) ? a.x0[(int64_t)b * a.sX0 + lane] : T(0);
    if (lane < NMAX) {
      const bool v = lane < n;
      const T li = (v && a.lb) ? a.lb[(int64_t)b * a.slb + lane] : -Lim<T>::inf();
      const T ui = (v && a.ub) ? a.ub[(int64_t)b * a.sub + lane] : Lim<T>::inf();
      lbs[lane] = li;
      ubs[lane] = ui;
      fs[lane] = T(0);
      badbox = v && (!(li <= ui) || li == Lim<T>::inf() || ui == -Lim<T>::inf());
    }
  }
  __syncthreads();

  int code = MPCQP_STATUS_OPTIMAL;
  // ------------------------------------- Riccati backward (all lanes, regs)
  {
    T P[NX][NX], Qr[NX][NX], Rr[NU][NU], Ar[NX][NX], Br[NX][NU];
    load_sq<T, NX, NX>(Qfs, P, NX);
    load_sq<T, NX, NX>(Qs, Qr, NX);
    load_sq<T, NU, NU>(Rs, Rr, NU);
    load_sq<T, NX, NX>(As, Ar, NX);
    load_sq<T, NX, NU>(Bs, Br, NU);
    bool ok = true;
    for (int k = N - 1; k >= 0; --k) {
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
          for (int q = 0; q < NX; ++q) s = fma(P[i][q], Ar[q][j], s);
          PA[i][j] = s;
        }
#pragma unroll
        for (int j = 0; j < NU; ++j) {
          T s = T(0);
#pragma unroll
          for (int q = 0; q < NX; ++q) s = fma(P[i][q], Br[q][j], s);
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
          for (int q = 0; q < NX; ++q) s = fma(Br[q][i], PB[q][j], s);
          Sm[i][j] = s;
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) {
          T s = T(0);
#pragma unroll
          for (int q = 0; q < NX; ++q) s = fma(Br[q][i], PA[q][j], s);
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
          for (int q = 0; q < NU; ++q) s = fma(Si[i][q], Y[q][j], s);
          K[i][j] = -s;
        }
      if (lane == 0) {
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
            for (int q = 0; q < NU; ++q) s = fma(Br[i][q], K[q][j], s);
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
            for (int q = 0; q < NX; ++q) s = fma(Ar[q][i], PA[q][j], s);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
              T apb = T(0);
#pragma unroll
              for (int q = 0; q < NX; ++q) apb = fma(Ar[q][i], PB[q][u], apb);
              s = fma(apb, K[u][j], s);
            }
            P[i][j] = s;
          }
      }
    }
    if (!ok) code = MPCQP_STATUS_NOT_CONVEX;

    // ---- free response xbar (forward) and adjoint y -> f (backward)
    if (tv == 0) load_sq<T, NX, NX>(As, Ar, NX);
    T xk[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) xk[q] = X0s[q];
    for (int k = 0; k < N; ++k) {
      if (tv) load_sq<T, NX, NX>(As + k * NX * NX, Ar, NX);
      T xn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T s = Cs[k * NX + i];
#pragma unroll
        for (int q = 0; q < NX; ++q) s = fma(Ar[i][q], xk[q], s);
        xn[i] = s;
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) xk[q] = xn[q];
      if (lane == 0)
#pragma unroll
        for (int q = 0; q < NX; ++q) Xs[(k + 1) * NX + q] = xk[q];
    }
    __syncthreads();
    T yk[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      T s = T(0);
#pragma unroll
      for (int q = 0; q < NX; ++q) s = fma(Qfs[i * NX + q], xk[q], s);
      yk[i] = s;
    }
    for (int k = N - 1; k >= 0; --k) {
      // f_(k,u) = B_k[:,u]' y_{k+1}
      const T* Bk = Bs + (tv ? k : 0) * NX * NU;
      if (lane == 0) {
        for (int u = 0; u < nu; ++u) {
          T s = T(0);
#pragma unroll
          for (int q = 0; q < NX; ++q) s = fma(Bk[q * NU + u], yk[q], s);
          fs[k * nu + u] = s;
        }
      }
      if (k == 0) break;
      if (tv) load_sq<T, NX, NX>(As + k * NX * NX, Ar, NX);
      T yn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T s = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) s = fma(Qr[i][q], Xs[k * NX + q], s);
#pragma unroll
        for (int q = 0; q < NX; ++q) s = fma(Ar[q][i], yk[q], s);
        yn[i] = s;
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) yk[q] = yn[q];
    }
  }
  __syncthreads();

  // ------------------------------ columns of -H^{-1}, one lane per column
  if (lane < n) {
    const int c = lane;
    const int jj = c / nu, bb = c - jj * nu;
    T s[NX], kf[NU];
    // k = jj: kff = S^{-1} e_b, s = -K' e_b
#pragma unroll
    for (int u = 0; u < NU; ++u) kf[u] = Sis[(jj * NU + u) * NU + bb];
#pragma unroll
    for (int q = 0; q < NX; ++q) s[q] = -Ks[(jj * NU + bb) * NX + q];
#pragma unroll
    for (int u = 0; u < NU; ++u) Kfs[(jj * n + c) * NU + u] = kf[u];
    for (int k = jj - 1; k >= 0; --k) {
      const T* Bk = Bs + (tv ? k : 0) * NX * NU;
      T t[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        T v = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) v = fma(Bk[q * NU + u], s[q], v);
        t[u] = v;
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        T v = T(0);
#pragma unroll
        for (int q = 0; q < NU; ++q) v = fma(Sis[(k * NU + u) * NU + q], t[q], v);
        kf[u] = -v;
        Kfs[(k * n + c) * NU + u] = kf[u];
      }
      T sn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T v = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) v = fma(Acls[(k * NX + q) * NX + i], s[q], v);
        sn[i] = v;
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) s[q] = sn[q];
    }
    // forward rollout from x_0 = 0
    T x[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) x[q] = T(0);
    for (int k = 0; k < N; ++k) {
      const T* Ak = As + (tv ? k : 0) * NX * NX;
      const T* Bk = Bs + (tv ? k : 0) * NX * NU;
      T u[NU];
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        T v = (k <= jj) ? Kfs[(k * n + c) * NU + i] : T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) v = fma(Ks[(k * NU + i) * NX + q], x[q], v);
        u[i] = v;
      }
      for (int i = 0; i < nu; ++i) Mv[(k * nu + i) * ld + c] = -u[i];
      T xn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        T v = T(0);
#pragma unroll
        for (int q = 0; q < NX; ++q) v = fma(Ak[i * NX + q], x[q], v);
#pragma unroll
        for (int q = 0; q < NU; ++q) v = fma(Bk[i * NU + q], u[q], v);
        xn[i] = v;
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) x[q] = xn[q];
    }
  }
  __syncthreads();

  // ------------------------------------------------ box QP on M = -H^{-1}
  Sym2D<T, BS> M;
  M.init(lane);
#pragma unroll
  for (int r = 0; r < BS; ++r)
#pragma unroll
    for (int cc = 0; cc < BS; ++cc) {
      const int i = M.bi * BS + r, j = M.bj * BS + cc;
      M.m[r][cc] = (i < n && j < n) ? T(0.5) * (Mv[i * ld + j] + Mv[j * ld + i]) : T(0);
    }
  if (lane < n) nonfinite |= !finite(fs[lane]);
  T zr[BS];
  int iters = 0;
  if (__any(nonfinite)) code = MPCQP_STATUS_NONFINITE;
  else if (__any(badbox)) code = MPCQP_STATUS_INFEASIBLE;
  if (code == MPCQP_STATUS_OPTIMAL)
    code = gi_box_core<T, BS>(M, buf, fs, lbs, ubs, n, a.max_iter, a.tol, zr, iters);
  if (code != MPCQP_STATUS_OPTIMAL && code != MPCQP_STATUS_MAXITER) {
#pragma unroll
    for (int r = 0; r < BS; ++r) zr[r] = __builtin_nan("");
  }
  if (M.bj == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = M.bi * BS + r;
      if (i < n) a.z[(int64_t)b * n + i] = zr[r];
    }
  }
  if (lane == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
}

template <typename T, int NX, int NU, int BS>
static int launch_mpc(const MpcBoxArgs<T>& a, hipStream_t st) {
  const int n = a.N * a.nu;
  const MpcLds<T, NX, NU, BS> L(a.N, n, a.tv);
  const size_t bytes = (size_t)L.total * sizeof(T);
  if (bytes > 160 * 1024) {
    set_error("mpcqp_mpc_box: LDS footprint %zu B > 160 KiB", bytes);
    return MPCQP_ENOTSUP;
  }
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)mpc_box_kernel<T, NX, NU, BS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(mpc_box)");
  }
  hipLaunchKernelGGL((mpc_box_kernel<T, NX, NU, BS>), dim3(a.batch), dim3(kWave), bytes, st, a);
  MPCQP_CHECK_LAUNCH("mpc_box_kernel");
  return MPCQP_OK;
}

template <typename T, int NX, int NU>
static int mpc_bs(const MpcBoxArgs<T>& a, hipStream_t st) {
  switch ((a.N * a.nu + 7) / 8) {
    case 1: return launch_mpc<T, NX, NU, 1>(a, st);
    case 2: return launch_mpc<T, NX, NU, 2>(a, st);
    case 3: return launch_mpc<T, NX, NU, 3>(a, st);
    default: return launch_mpc<T, NX, NU, 4>(a, st);
  }
}

template <typename T>
static int mpc_box_t(MpcBoxArgs<T>& a, hipStream_t st) {
  if (!use_wave_kernels()) {
    MpcArgsQ<T> q{a.batch, a.nx, a.nu, a.N, a.tv, a.A, a.sA, a.B, a.sB, a.Q, a.sQ, a.R, a.sR,
                  a.Qf, a.sQf, a.c, a.sC, a.x0, a.sX0, a.lb, a.slb, a.ub, a.sub, a.z, a.status,
                  a.max_iter, a.tol};
    return mpc_box_quad<T>(q, st);
  }
  if (a.nx <= 2 && a.nu == 1) return mpc_bs<T, 2, 1>(a, st);
  if (a.nx <= 2) return mpc_bs<T, 2, 2>(a, st);
  if (a.nu == 1) return mpc_bs<T, 4, 1>(a, st);
  return mpc_bs<T, 4, 2>(a, st);
}

}  // namespace mpcqp

extern "C" int mpcqp_mpc_box(int dtype, int batch, int nx, int nu, int N, int flags,
                             const void* A, int64_t strideA, const void* Bm, int64_t strideB,
                             const void* Q, int64_t strideQ, const void* R, int64_t strideR,
                             const void* Qf, int64_t strideQf, const void* c, int64_t strideC,
                             const void* x0, int64_t strideX0, const void* lb, int64_t strideLb,
                             const void* ub, int64_t strideUb, void* z, int32_t* status,
                             int max_iter, double tol, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_mpc_box: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_mpc_box: batch < 0");
  MPCQP_CHECK_ARG(nx >= 1 && nx <= 4 && nu >= 1 && nu <= 2,
                  "mpcqp_mpc_box: nx=%d nu=%d outside the fused kernel set (nx<=4, nu<=2); "
                  "use mpcqp_condense + mpcqp_solve_box", nx, nu);
  MPCQP_CHECK_ARG(N >= 1 && N * nu <= 32, "mpcqp_mpc_box: n = N*nu = %d outside [1,32]", N * nu);
  MPCQP_CHECK_ARG(A && Bm && Q && R && Qf && z && status, "mpcqp_mpc_box: null pointer");
  MPCQP_CHECK_ARG(strideA >= 0 && strideB >= 0 && strideQ >= 0 && strideR >= 0 && strideQf >= 0 &&
                      strideC >= 0 && strideX0 >= 0 && strideLb >= 0 && strideUb >= 0,
                  "mpcqp_mpc_box: negative stride");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64) {
    MpcBoxArgs<double> a{batch, nx, nu, N, (flags & MPCQP_TV) ? 1 : 0,
                         (const double*)A, strideA, (const double*)Bm, strideB,
                         (const double*)Q, strideQ, (const double*)R, strideR,
                         (const double*)Qf, strideQf, (const double*)c, strideC,
                         (const double*)x0, strideX0, (const double*)lb, strideLb,
                         (const double*)ub, strideUb, (double*)z, status,
                         max_iter > 0 ? max_iter : 3 * N * nu + 30, tol > 0 ? tol : 1e-12};
    return mpc_box_t<double>(a, st);
  }
  MpcBoxArgs<float> a{batch, nx, nu, N, (flags & MPCQP_TV) ? 1 : 0,
                      (const float*)A, strideA, (const float*)Bm, strideB,
                      (const float*)Q, strideQ, (const float*)R, strideR,
                      (const float*)Qf, strideQf, (const float*)c, strideC,
                      (const float*)x0, strideX0, (const float*)lb, strideLb,
                      (const float*)ub, strideUb, (float*)z, status,
                      max_iter > 0 ? max_iter : 3 * N * nu + 30, tol > 0 ? (float)tol : 1e-6f};
  return mpc_box_t<float>(a, st);
}
