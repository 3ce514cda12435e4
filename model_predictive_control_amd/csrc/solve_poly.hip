// solve_poly.hip -- batched polytope QP through its dual, one instance per
// wavefront:
//
//   min 1/2 z'Hz + f'z   s.t.  l <= C z <= u,   C = [G; I] (box rows optional)
//
// Replaces the IPOPT call of session_4/main.py:115-116 for constraint rows
// g(z) with bounds lbg/ubg (main.py:58-61,99-100: after condensing, the state
// box is the row block Gam with bounds shifted by the free response), and the
// BASELINE config-4 polytope (40 random rows over N*nu = 200 inputs).
//
// Shared phase (once per call, H and G shared by the batch):
//   Hinv = H^{-1}   (single-workgroup Gauss-Jordan on device)
//   Ut   = C Hinv   (mt x n),  M = C Hinv C'  (mt x mt, packed lower)
// Per instance:
//   s0 = -Ut f,  z0 = -Hinv f                     (gemv)
//   dual range active set on M  -> y (y_r > 0: row r at its upper bound,
//                                     y_r < 0: at its lower bound)
//   z  = z0 - Ut' y                               (gemv, transposed)
//
// Dual range active set (Goldfarb-Idnani written in the row space): the
// wavefront keeps W = SWEEP_A(M), M swept on the active rows, as an 8x8
// grid of register blocks (sym2d.hpp).  With w = (s0 - b on A, 0 elsewhere), v = W w gives y_A = -v_A and
// the inactive row values s_I = s0_I - v_I.  Adding row p is a sweep with
// pivot W_pp (its Schur complement -- zero when p depends on the active rows,
// in which case a pure dual step drops rows first), dropping row k is a
// reverse sweep.  Same register-resident sweep machinery as solve_box.hip.
#include "sym2d.hpp"

namespace mpcqp {

template <typename T>
struct DualArgs {
  int batch, mt, m1;           // rows; the first m1 use (l1,u1) with stride s1
  const T* M; int64_t sM;      // packed lower mt x mt
  const T* s0; int64_t sS0;
  const T* l1; const T* u1; int64_t s1;
  const T* l2; const T* u2;    // rows m1..mt-1, shared
  T* y;
  int32_t* status;
  int max_iter;
  T tol;
};

// st: 0 inactive, 1 at lower, 2 at upper, 3 padding row
template <typename T, int BS>
__global__ __launch_bounds__(64) void dual_range_kernel(DualArgs<T> a) {
  using S2 = Sym2D<T, BS>;
  constexpr int NMAX = S2::NMAX;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = reinterpret_cast<T*>(smem_raw);
  T* lis = buf + S2::BUF;
  T* uis = lis + NMAX;
  T* mds = uis + NMAX;
  T* ss = mds + NMAX;
  T* Ps = ss + NMAX;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = a.mt;
  const int P = n * (n + 1) / 2;
  stage_packed<T, NMAX*(NMAX + 1) / 2>(a.M + (int64_t)b * a.sM, Ps, P, lane);

  Sym2D<T, BS> W;
  W.init(lane);
  T s0[BS], li[BS], ui[BS], yi[BS], si[BS];
  int st[BS];
  bool nonfinite = false, badbox = false;
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    const int i = W.bi * BS + r;
    const bool v = i < n;
    s0[r] = v ? a.s0[(int64_t)b * a.sS0 + i] : T(0);
    li[r] = -Lim<T>::inf();
    ui[r] = Lim<T>::inf();
    if (v) {
      if (i < a.m1) {
        if (a.l1) li[r] = a.l1[(int64_t)b * a.s1 + i];
        if (a.u1) ui[r] = a.u1[(int64_t)b * a.s1 + i];
      } else {
        if (a.l2) li[r] = a.l2[i - a.m1];
        if (a.u2) ui[r] = a.u2[i - a.m1];
      }
    }
    st[r] = v ? 0 : 3;
    yi[r] = T(0);
    si[r] = s0[r];
    nonfinite |= v && !finite(s0[r]);
    badbox |= v && (!(li[r] <= ui[r]) || li[r] == Lim<T>::inf() || ui[r] == -Lim<T>::inf());
  }
  publish<T, BS>(li, lis, W.bi, W.bj);
  publish<T, BS>(ui, uis, W.bi, W.bj);
  __syncthreads();
  W.load_packed(Ps, n, nonfinite);
  // diagonal of M by row (dependency test scale)
  for (int i = lane; i < n; i += kWave) mds[i] = Ps[i * (i + 1) / 2 + i];
  __syncthreads();
  int code = MPCQP_STATUS_MAXITER;
  int iters = 0;
  const T tol = a.tol;
  const T dep_tol = sizeof(T) == 8 ? T(1e-10) : T(1e-5);
  const int max_iter = a.max_iter;
  if (__any(nonfinite)) {
    code = MPCQP_STATUS_NONFINITE;
    goto done;
  }
  if (__any(badbox)) {
    code = MPCQP_STATUS_INFEASIBLE;
    goto done;
  }
  {
    // w = (s0 - b on active rows, 0 elsewhere);  v = W w;
    // active: y = -v, s = bound;  inactive: s = s0 - v
    auto refresh = [&]() {
      T w[BS], v[BS];
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const bool act = st[r] == 1 || st[r] == 2;
        const T bnd = (st[r] == 1) ? li[r] : ui[r];
        w[r] = act ? s0[r] - bnd : T(0);
      }
      W.matvec(w, buf, v);
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const bool act = st[r] == 1 || st[r] == 2;
        const T bnd = (st[r] == 1) ? li[r] : ui[r];
        yi[r] = act ? -v[r] : T(0);
        si[r] = act ? bnd : s0[r] - v[r];
      }
    };
    while (true) {
      T viol = -Lim<T>::inf();
      int p = 0;
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        if (st[r] == 0) {
          const T vl = finite(li[r]) ? (li[r] - si[r]) / (T(1) + fabs(li[r])) : -Lim<T>::inf();
          const T vu = finite(ui[r]) ? (si[r] - ui[r]) / (T(1) + fabs(ui[r])) : -Lim<T>::inf();
          const T vv = fmax(vl, vu);
          if (vv > viol) {
            viol = vv;
            p = W.bi * BS + r;
          }
        }
      }
      blocks_argmax(viol, p);
      p = uniform(p);
      if (!(readlane(viol, 0) > tol)) {
        code = MPCQP_STATUS_OPTIMAL;
        break;
      }
      publish<T, BS>(si, ss, W.bi, W.bj);
      __syncthreads();
      const T sp0 = ss[p];
      const T lp = lis[p], up = uis[p];
      const T mpp = mds[p];
      __syncthreads();
      const int side = (sp0 < lp) ? 1 : 2;
      const T tgt = (side == 1) ? lp : up;
      const T ysgn = (side == 1) ? T(-1) : T(1);
      T sp = sp0;
      bool added = false;
      while (!added) {
        if (++iters > max_iter) goto done;
        T c[BS], cc[BS];
        const T wpp = W.column(p, buf, c, cc);  // c[r] = W_ip
        const bool dep = !(wpp > dep_tol * fmax(mpp, T(1e-300)));
        T ti = Lim<T>::inf();
        int k = 0;
        T dy[BS];
#pragma unroll
        for (int r = 0; r < BS; ++r) {
          dy[r] = -c[r] * ysgn;
          T t = Lim<T>::inf();
          if (st[r] == 2 && dy[r] < T(0)) t = yi[r] / (-dy[r]);
          if (st[r] == 1 && dy[r] > T(0)) t = (-yi[r]) / dy[r];
          if (t < ti) {
            ti = t;
            k = W.bi * BS + r;
          }
        }
        blocks_argmin(ti, k);
        k = uniform(k);
        ti = readlane(ti, 0);
        const T t2 = dep ? Lim<T>::inf() : fabs(sp - tgt) / wpp;
        if (!(ti < Lim<T>::inf()) && !(t2 < Lim<T>::inf())) {
          code = MPCQP_STATUS_INFEASIBLE;
          goto done;
        }
        if (ti < t2) {
#pragma unroll
          for (int r = 0; r < BS; ++r) {
            if (st[r] == 1 || st[r] == 2) yi[r] = fma(ti, dy[r], yi[r]);
            if (W.bi * BS + r == k) {
              yi[r] = T(0);
              st[r] = 0;
            }
          }
          if (!dep) sp = sp - wpp * ysgn * ti;
          W.sweep(k, T(-1), buf);
        } else {
          const T d = W.sweep(p, T(1), buf);
          if (!(d > T(0))) {
            code = MPCQP_STATUS_NOT_CONVEX;
            goto done;
          }
#pragma unroll
          for (int r = 0; r < BS; ++r)
            if (W.bi * BS + r == p) st[r] = side;
          refresh();
          added = true;
        }
      }
    }
  }
done:
  if (code != MPCQP_STATUS_OPTIMAL && code != MPCQP_STATUS_MAXITER) {
#pragma unroll
    for (int r = 0; r < BS; ++r) yi[r] = __builtin_nan("");
  }
  if (a.y && W.bj == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) {
      const int i = W.bi * BS + r;
      if (i < n) a.y[(int64_t)b * n + i] = yi[r];
    }
  }
  if (lane == 0) a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
}

// ------------------------------------------------------- shared phase
// Gauss-Jordan inverse of the shared SPD H (packed lower -> dense Hinv) by one
// workgroup; the pivot row is staged in LDS each step.
template <typename T>
__global__ __launch_bounds__(1024) void gj_inverse_kernel(const T* Hp, int n, T* W, T* Hinv,
                                                          int32_t* flag) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* prow = reinterpret_cast<T*>(smem_raw);  // 2n: pivot row of [W | Hinv]
  T* pcol = prow + 2 * n;                    // n : pivot column
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < n * n; e += nt) {
    const int i = e / n, j = e % n;
    W[e] = (j <= i) ? Hp[i * (i + 1) / 2 + j] : Hp[j * (j + 1) / 2 + i];
    Hinv[e] = (i == j) ? T(1) : T(0);
  }
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    const T piv = W[k * n + k];
    if (!(piv > T(0))) {
      if (tid == 0) *flag = 1;
      return;
    }
    const T rp = T(1) / piv;
    for (int j = tid; j < n; j += nt) {
      prow[j] = W[k * n + j] * rp;
      prow[n + j] = Hinv[k * n + j] * rp;
      pcol[j] = W[j * n + k];
    }
    __syncthreads();
    for (int e = tid; e < n * n; e += nt) {
      const int i = e / n, j = e % n;
      if (i == k) {
        W[e] = prow[j];
        Hinv[e] = prow[n + j];
      } else {
        const T fct = pcol[i];
        W[e] = fma(-fct, prow[j], W[e]);
        Hinv[e] = fma(-fct, prow[n + j], Hinv[e]);
      }
    }
    __syncthreads();
  }
}

// Ut[r][j] = sum_k C[r][k] Hinv[k][j],  C = [G; I]
template <typename T>
__global__ void form_ut_kernel(const T* G, int m, int n, int mt, const T* Hinv, T* Ut) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= mt * n) return;
  const int r = e / n, j = e % n;
  T s = T(0);
  if (r < m) {
    for (int k = 0; k < n; ++k) s = fma(G[(int64_t)r * n + k], Hinv[(int64_t)k * n + j], s);
  } else {
    s = Hinv[(int64_t)(r - m) * n + j];
  }
  Ut[e] = s;
}

// M[r][s] (packed lower) = sum_j Ut[r][j] C[s][j]
template <typename T>
__global__ void form_m_kernel(const T* G, int m, int n, int mt, const T* Ut, T* Mp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= mt * mt) return;
  const int r = e / mt, s = e % mt;
  if (s > r) return;
  T acc = T(0);
  if (s < m) {
    for (int j = 0; j < n; ++j) acc = fma(Ut[(int64_t)r * n + j], G[(int64_t)s * n + j], acc);
  } else {
    acc = Ut[(int64_t)r * n + (s - m)];
  }
  Mp[(int64_t)r * (r + 1) / 2 + s] = acc;
}

// y_b = alpha * op(Mat) x_b + beta * y_b with op = transpose when trans.
template <typename T>
__global__ __launch_bounds__(64) void gemv_t_kernel(int rows, int cols, T alpha, const T* Mat,
                                                    const T* x, int64_t sX, T beta, T* y,
                                                    int64_t sY, int trans) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* xs = reinterpret_cast<T*>(smem_raw);
  const int b = blockIdx.x, lane = threadIdx.x;
  const int outn = trans ? cols : rows, inn = trans ? rows : cols;
  for (int j = lane; j < inn; j += kWave) xs[j] = x[(int64_t)b * sX + j];
  __syncthreads();
  for (int o = lane; o < outn; o += kWave) {
    T s = T(0);
    if (trans) {
      for (int j = 0; j < inn; ++j) s = fma(Mat[(int64_t)j * cols + o], xs[j], s);
    } else {
      for (int j = 0; j < inn; ++j) s = fma(Mat[(int64_t)o * cols + j], xs[j], s);
    }
    T* yo = y + (int64_t)b * sY + o;
    *yo = (beta == T(0)) ? alpha * s : fma(beta, *yo, alpha * s);
  }
}

static inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

struct PolyWs {
  int64_t oW, oHinv, oUt, oM, oS0, oFlag, total;
};

static PolyWs poly_ws(size_t es, int batch, int n, int mt) {
  PolyWs w;
  w.oW = 0;
  w.oHinv = align256(w.oW + (int64_t)n * n * es);
  w.oUt = align256(w.oHinv + (int64_t)n * n * es);
  w.oM = align256(w.oUt + (int64_t)mt * n * es);
  w.oS0 = align256(w.oM + (int64_t)mt * (mt + 1) / 2 * es);
  w.oFlag = align256(w.oS0 + (int64_t)batch * mt * es);
  w.total = align256(w.oFlag + 16);
  return w;
}

template <typename T, int BS>
static void launch_dual(const DualArgs<T>& a, hipStream_t st) {
  const size_t bytes = (size_t)(Sym2D<T, BS>::BUF + 4 * 8 * BS + a.mt * (a.mt + 1) / 2) * sizeof(T);
  hipLaunchKernelGGL((dual_range_kernel<T, BS>), dim3(a.batch), dim3(kWave), bytes, st, a);
}

template <typename T>
static int solve_poly_t(int batch, int n, int m, const void* H, const void* f, int64_t sf,
                        const void* G, const void* hl, const void* hu, int64_t sh,
                        const void* lbz, const void* ubz, void* z, void* y, int32_t* status,
                        int max_iter, double tol, void* ws, int64_t wsb, hipStream_t st) {
  const int mt = m + ((lbz || ubz) ? n : 0);
  const PolyWs L = poly_ws(sizeof(T), batch, n, mt);
  if (wsb < L.total) {
    set_error("mpcqp_solve_poly: workspace %lld B < required %lld B", (long long)wsb,
              (long long)L.total);
    return MPCQP_EINVAL;
  }
  char* base = (char*)ws;
  T* W = (T*)(base + L.oW);
  T* Hinv = (T*)(base + L.oHinv);
  T* Ut = (T*)(base + L.oUt);
  T* Mp = (T*)(base + L.oM);
  T* S0 = (T*)(base + L.oS0);
  int32_t* flag = (int32_t*)(base + L.oFlag);
  hipError_t e = hipMemsetAsync(flag, 0, 16, st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(poly flag)");
  const size_t gj_lds = (size_t)3 * n * sizeof(T);
  if (gj_lds > 64 * 1024) {
    set_error("mpcqp_solve_poly: n=%d too large for the shared inverse", n);
    return MPCQP_ENOTSUP;
  }
  hipLaunchKernelGGL(gj_inverse_kernel<T>, dim3(1), dim3(1024), gj_lds, st, (const T*)H, n, W,
                     Hinv, flag);
  MPCQP_CHECK_LAUNCH("gj_inverse_kernel");
  const int thr = 256;
  hipLaunchKernelGGL(form_ut_kernel<T>, dim3((mt * n + thr - 1) / thr), dim3(thr), 0, st,
                     (const T*)G, m, n, mt, (const T*)Hinv, Ut);
  MPCQP_CHECK_LAUNCH("form_ut_kernel");
  hipLaunchKernelGGL(form_m_kernel<T>, dim3((mt * mt + thr - 1) / thr), dim3(thr), 0, st,
                     (const T*)G, m, n, mt, (const T*)Ut, Mp);
  MPCQP_CHECK_LAUNCH("form_m_kernel");
  // s0 = -Ut f ; z0 = -Hinv f
  hipLaunchKernelGGL(gemv_t_kernel<T>, dim3(batch), dim3(kWave), (size_t)n * sizeof(T), st, mt,
                     n, T(-1), (const T*)Ut, (const T*)f, sf, T(0), S0, (int64_t)mt, 0);
  MPCQP_CHECK_LAUNCH("gemv_t_kernel(s0)");
  hipLaunchKernelGGL(gemv_t_kernel<T>, dim3(batch), dim3(kWave), (size_t)n * sizeof(T), st, n, n,
                     T(-1), (const T*)Hinv, (const T*)f, sf, T(0), (T*)z, (int64_t)n, 0);
  MPCQP_CHECK_LAUNCH("gemv_t_kernel(z0)");
  DualArgs<T> a;
  a.batch = batch; a.mt = mt; a.m1 = m;
  a.M = Mp; a.sM = 0; a.s0 = S0; a.sS0 = mt;
  a.l1 = (const T*)hl; a.u1 = (const T*)hu; a.s1 = sh;
  a.l2 = (const T*)lbz; a.u2 = (const T*)ubz;
  a.y = (T*)y; a.status = status;
  a.max_iter = max_iter > 0 ? max_iter : 4 * mt + 40;
  a.tol = tol > 0 ? (T)tol : (sizeof(T) == 8 ? (T)1e-12 : (T)1e-6);
  switch ((mt + 7) / 8) {
    case 1: launch_dual<T, 1>(a, st); break;
    case 2: launch_dual<T, 2>(a, st); break;
    case 3: launch_dual<T, 3>(a, st); break;
    case 4: launch_dual<T, 4>(a, st); break;
    case 5: launch_dual<T, 5>(a, st); break;
    case 6: launch_dual<T, 6>(a, st); break;
    case 7: launch_dual<T, 7>(a, st); break;
    default: launch_dual<T, 8>(a, st); break;
  }
  MPCQP_CHECK_LAUNCH("dual_range_kernel");
  // z = z0 - Ut' y
  hipLaunchKernelGGL(gemv_t_kernel<T>, dim3(batch), dim3(kWave), (size_t)mt * sizeof(T), st, mt,
                     n, T(-1), (const T*)Ut, (const T*)y, (int64_t)mt, T(1), (T*)z, (int64_t)n, 1);
  MPCQP_CHECK_LAUNCH("gemv_t_kernel(z)");
  return MPCQP_OK;
}

}  // namespace mpcqp

extern "C" int64_t mpcqp_solve_poly_workspace(int dtype, int batch, int n, int m, int nbox) {
  const int mt = m + (nbox ? n : 0);
  return mpcqp::poly_ws(mpcqp::dtype_size(dtype), batch, n, mt).total;
}

extern "C" int mpcqp_solve_poly(int dtype, int batch, int n, int m, const void* H, const void* f,
                                int64_t stridef, const void* G, const void* hl, const void* hu,
                                int64_t strideh, const void* lbz, const void* ubz, void* z,
                                void* y, int32_t* status, int max_iter, double tol,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, "mpcqp_solve_poly: bad dtype %d", dtype);
  MPCQP_CHECK_ARG(batch >= 0 && n >= 1 && m >= 0, "mpcqp_solve_poly: bad sizes");
  const int mt = m + ((lbz || ubz) ? n : 0);
  MPCQP_CHECK_ARG(mt >= 1 && mt <= 64, "mpcqp_solve_poly: rows m_total=%d outside [1,64]", mt);
  MPCQP_CHECK_ARG(H && f && z && y && status && workspace, "mpcqp_solve_poly: null pointer");
  MPCQP_CHECK_ARG(m == 0 || G, "mpcqp_solve_poly: G required when m > 0");
  MPCQP_CHECK_ARG(stridef >= 0 && strideh >= 0, "mpcqp_solve_poly: negative stride");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return solve_poly_t<double>(batch, n, m, H, f, stridef, G, hl, hu, strideh, lbz, ubz, z, y,
                                status, max_iter, tol, workspace, workspace_bytes, st);
  return solve_poly_t<float>(batch, n, m, H, f, stridef, G, hl, hu, strideh, lbz, ubz, z, y,
                             status, max_iter, tol, workspace, workspace_bytes, st);
}
