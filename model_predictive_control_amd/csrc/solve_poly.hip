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
// Shared phase (mpcqp_poly_setup, once per (H, G, F); H and G shared by the
// batch, F = the condensed x0 -> gradient map, optional):
//   Hinv = H^{-1}   (single-workgroup Gauss-Jordan on device)
//   Ut   = C Hinv   (mt x n),  M = C Hinv C'  (mt x mt, packed lower)
//   Kt   = (-Hinv F)'  (nx x n),  L = -Ut F  (mt x nx)
// Per instance, one wavefront (mpcqp_poly_solve), gradient f = F x0 + f1:
//   prologue  s0 = L x0 - Ut f1                     (unconstrained row values)
//   dual range active set on M  -> y (y_r > 0: row r at its upper bound,
//                                     y_r < 0: at its lower bound)
//   epilogue  z  = Kt' x0 - Hinv f1 - Ut' y
// With x0 given, the per-instance work is O(mt*(nx + n) + n*nx) instead of
// the O(n^2) of forming f and -Hinv f (BASELINE config 4: n = 200, mt = 40).
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
  const T* l1; const T* u1; int64_t s1;
  const T* l2; const T* u2;    // rows m1..mt-1, shared
  // prologue / epilogue operands (shared factors from the setup phase)
  int n, nx;
  const T* Ut;                 // mt x n
  const T* Hinv;               // n x n   (used when f1 is given)
  const T* Kt;                 // nx x n  (used when x0 is given)
  const T* L;                  // mt x nx (used when x0 is given)
  const T* x0; int64_t sX0;
  const T* f1; int64_t sF1;
  const int32_t* flag;         // set by the shared inverse when H is not PD
  T* z;
  T* y;
  int32_t* status;
  int max_iter;
  T tol;
};

// st: 0 inactive, 1 at lower, 2 at upper, 3 padding row.
// Layout: the swept matrix W on the 8 x 8 block grid (Sym2D); every
// row-indexed vector (s0, bounds, scales, y, s, st) one row per lane (lane i =
// row i, mt <= 64), so the scan and the ratio test run once per row instead
// of once per row-block replica, with full-wave DPP arg-max / arg-min.
// (152 VGPRs, 3 waves per SIMD, since the drop and the add share one sweep
// call: with two sweep sites W lived in two register sets, 220 VGPRs and 2
// waves per SIMD; config 4 poly_solve 2.72 -> 1.99 ms.)
template <typename T, int BS>
__global__ __launch_bounds__(64) void dual_range_kernel(DualArgs<T> a) {
  using S2 = Sym2D<T, BS>;
  constexpr int NMAX = S2::NMAX;
  static_assert(NMAX <= kWave, "one row per lane");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = reinterpret_cast<T*>(smem_raw);
  T* xs = buf + S2::BUF;       // 16: x0
  T* part = xs + 16;           // 8 * NMAX: partial row sums of the mat-vec
  T* Ps = part + 8 * NMAX;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = a.mt;
  const int P = n * (n + 1) / 2;
  const int nz = a.n, nx = a.nx;
  const T* x0 = a.x0 ? a.x0 + (int64_t)b * a.sX0 : nullptr;
  const T* f1 = a.f1 ? a.f1 + (int64_t)b * a.sF1 : nullptr;
  stage_packed<T, NMAX*(NMAX + 1) / 2>(a.M + (int64_t)b * a.sM, Ps, P, lane);
  if (x0 && lane < nx) xs[lane] = x0[lane];
  __syncthreads();
  // row `lane`: unconstrained value s0 = L x0 - Ut f1, bounds, scales, M_ii
  const bool row = lane < n;
  T s0 = T(0), li = -Lim<T>::inf(), ui = Lim<T>::inf(), md = T(1);
  if (row) {
    T acc = T(0);
    if (x0)
      for (int k = 0; k < nx; ++k) acc = fma(a.L[lane * nx + k], xs[k], acc);
    if (f1)
      for (int j = 0; j < nz; ++j) acc = fma(-a.Ut[(int64_t)lane * nz + j], f1[j], acc);
    s0 = acc;
    if (lane < a.m1) {
      if (a.l1) li = a.l1[(int64_t)b * a.s1 + lane];
      if (a.u1) ui = a.u1[(int64_t)b * a.s1 + lane];
    } else {
      if (a.l2) li = a.l2[lane - a.m1];
      if (a.u2) ui = a.u2[lane - a.m1];
    }
    md = Ps[lane * (lane + 1) / 2 + lane];
  }
  int st = row ? 0 : 3;
  T yi = T(0), si = s0;
  bool nonfinite = row && !finite(s0);
  const bool badbox =
      row && (!(li <= ui) || li == Lim<T>::inf() || ui == -Lim<T>::inf());
  // relative-violation scales 1/(1+|bound|), NaN for an infinite bound (a NaN
  // violation never wins the arg-max): the per-iteration scan only multiplies
  const T sl = finite(li) ? T(1) / (T(1) + fabs(li)) : T(__builtin_nan(""));
  const T su = finite(ui) ? T(1) / (T(1) + fabs(ui)) : T(__builtin_nan(""));

  S2 W;
  W.init(lane);
  W.load_packed(Ps, n, nonfinite);
  int code = MPCQP_STATUS_MAXITER;
  int iters = 0;
  const T tol = a.tol;
  const T dep_tol = sizeof(T) == 8 ? T(1e-10) : T(1e-5);
  const int max_iter = a.max_iter;
  if (*a.flag) {
    code = MPCQP_STATUS_NOT_CONVEX;
    goto done;
  }
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
      const bool act = st == 1 || st == 2;
      const T bnd = (st == 1) ? li : ui;
      const T v = matvec_lane_lds<T, BS>(W, act ? s0 - bnd : T(0), buf, part);
      yi = act ? -v : T(0);
      si = act ? bnd : s0 - v;
    };
    while (true) {
      const T vl = (li - si) * sl;
      const T vu = (si - ui) * su;
      // arg-max as a wave max (3 VALU per step) and a ballot of the lanes
      // holding it: the smallest such lane wins, as in an (value, index) reduction
      const T viol = (st == 0) ? fmax(vl, vu) : -Lim<T>::inf();
      const T vmax = wave_max(viol);
      if (!(readlane(vmax, 0) > tol)) {
        code = MPCQP_STATUS_OPTIMAL;
        break;
      }
      const int p = uniform(__builtin_ctzll(__builtin_amdgcn_ballot_w64(viol == vmax)));
      const T sp0 = readlane(si, p);
      const T lp = readlane(li, p), up = readlane(ui, p);
      const T mpp = readlane(md, p);
      const int side = (sp0 < lp) ? 1 : 2;
      const T tgt = (side == 1) ? lp : up;
      const T ysgn = (side == 1) ? T(-1) : T(1);
      T sp = sp0;
      bool added = false;
      while (!added) {
        if (++iters > max_iter) goto done;
        T c[BS], cc[BS], cl;
        const T wpp = W.template column<true>(p, buf, c, cc, cl);  // cl = W_lane,p
        const bool dep = !(wpp > dep_tol * fmax(mpp, T(1e-300)));
        // an active row's multiplier moves toward 0: t = -y / dy (>= 0)
        const T dy = -cl * ysgn;
        const bool cand = (st == 2 && dy < T(0)) || (st == 1 && dy > T(0));
        const T tl = cand ? -yi * fast_rcp(dy) : Lim<T>::inf();
        const T ti = readlane(wave_min(tl), 0);
        const uint64_t kb = __builtin_amdgcn_ballot_w64(tl == ti);
        const int k = kb ? uniform(__builtin_ctzll(kb)) : 0;
        const T t2 = dep ? Lim<T>::inf() : fabs(sp - tgt) / wpp;
        if (!(ti < Lim<T>::inf()) && !(t2 < Lim<T>::inf())) {
          code = MPCQP_STATUS_INFEASIBLE;
          goto done;
        }
        // one sweep call for both steps (its pivot column fetched for a
        // drop, still in registers for an add): W stays in one register set
        // across the loop (two sweep sites had the compiler copy all of W
        // between two sets at the back edge)
        const bool part = ti < t2;  // wave-uniform
        int idx = p;
        T sig = T(1), d = wpp;
        if (part) {
          if (st == 1 || st == 2) yi = fma(ti, dy, yi);
          if (lane == k) {
            yi = T(0);
            st = 0;
          }
          if (!dep) sp = sp - wpp * ysgn * ti;
          idx = k;
          sig = T(-1);
          d = W.column(k, buf, c, cc);
        }
        W.sweep_col(idx, sig, d, c, cc);
        if (!part) {
          if (!(wpp > T(0))) {
            code = MPCQP_STATUS_NOT_CONVEX;
            goto done;
          }
          if (lane == p) st = side;
          refresh();
          added = true;
        }
      }
    }
  }
done:
  const bool okc = code == MPCQP_STATUS_OPTIMAL || code == MPCQP_STATUS_MAXITER;
  if (!okc) yi = __builtin_nan("");
  if (a.y && row) a.y[(int64_t)b * n + lane] = yi;
  // epilogue: z = Kt' x0 - Hinv f1 - Ut' y   (lanes over z, coalesced rows;
  // only the rows with y != 0 -- the active ones -- contribute)
  const uint64_t yact = __builtin_amdgcn_ballot_w64(row && yi != T(0));
  for (int j = lane; j < nz; j += kWave) {
    T acc = T(0);
    if (x0)
      for (int k = 0; k < nx; ++k) acc = fma(a.Kt[(int64_t)k * nz + j], xs[k], acc);
    if (f1)
      for (int i = 0; i < nz; ++i) acc = fma(-a.Hinv[(int64_t)i * nz + j], f1[i], acc);
    for (uint64_t mk = yact; mk; mk &= mk - 1) {
      const int r = uniform(__builtin_ctzll(mk));
      acc = fma(-a.Ut[(int64_t)r * nz + j], readlane(yi, r), acc);
    }
    a.z[(int64_t)b * nz + j] = okc ? acc : __builtin_nan("");
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

// Kt[k][j] = -(Hinv F)[j][k]   (nx x n)
template <typename T>
__global__ void form_kt_kernel(const T* F, int n, int nx, const T* Hinv, T* Kt) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nx * n) return;
  const int k = e / n, j = e % n;
  T acc = T(0);
  for (int i = 0; i < n; ++i) acc = fma(Hinv[(int64_t)j * n + i], F[(int64_t)i * nx + k], acc);
  Kt[e] = -acc;
}

// L[r][k] = sum_j C[r][j] Kt[k][j]  (= -C Hinv F = -Ut F, mt x nx)
template <typename T>
__global__ void form_l_kernel(const T* G, int m, int n, int mt, int nx, const T* Kt, T* L) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= mt * nx) return;
  const int r = e / nx, k = e % nx;
  T acc = T(0);
  if (r < m) {
    for (int j = 0; j < n; ++j) acc = fma(G[(int64_t)r * n + j], Kt[(int64_t)k * n + j], acc);
  } else {
    acc = Kt[(int64_t)k * n + (r - m)];
  }
  L[e] = acc;
}

static inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// Shared factors; independent of the batch size.
struct PolyWs {
  int64_t oW, oHinv, oUt, oM, oKt, oL, oFlag, total;
};

static PolyWs poly_ws(size_t es, int n, int mt, int nx) {
  PolyWs w;
  w.oW = 0;
  w.oHinv = align256(w.oW + (int64_t)n * n * es);
  w.oUt = align256(w.oHinv + (int64_t)n * n * es);
  w.oM = align256(w.oUt + (int64_t)mt * n * es);
  w.oKt = align256(w.oM + (int64_t)mt * (mt + 1) / 2 * es);
  w.oL = align256(w.oKt + (int64_t)nx * n * es);
  w.oFlag = align256(w.oL + (int64_t)mt * nx * es);
  w.total = align256(w.oFlag + 16);
  return w;
}

template <typename T, int BS>
static void launch_dual(const DualArgs<T>& a, hipStream_t st) {
  const size_t bytes =
      (size_t)(Sym2D<T, BS>::BUF + 16 + 8 * Sym2D<T, BS>::NMAX + a.mt * (a.mt + 1) / 2) * sizeof(T);
  hipLaunchKernelGGL((dual_range_kernel<T, BS>), dim3(a.batch), dim3(kWave), bytes, st, a);
}

template <typename T>
static int poly_setup_t(int n, int m, int nbox, int nx, const void* H, const void* G,
                        const void* F, void* ws, int64_t wsb, hipStream_t st) {
  const int mt = m + (nbox ? n : 0);
  const PolyWs L = poly_ws(sizeof(T), n, mt, nx);
  if (wsb < L.total) {
    set_error("mpcqp_poly_setup: workspace %lld B < required %lld B", (long long)wsb,
              (long long)L.total);
    return MPCQP_EINVAL;
  }
  char* base = (char*)ws;
  T* W = (T*)(base + L.oW);
  T* Hinv = (T*)(base + L.oHinv);
  T* Ut = (T*)(base + L.oUt);
  T* Mp = (T*)(base + L.oM);
  int32_t* flag = (int32_t*)(base + L.oFlag);
  hipError_t e = hipMemsetAsync(flag, 0, 16, st);
  if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(poly flag)");
  const size_t gj_lds = (size_t)3 * n * sizeof(T);
  if (gj_lds > 64 * 1024) {
    set_error("mpcqp_poly_setup: n=%d too large for the shared inverse", n);
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
  if (nx > 0 && F) {
    T* Kt = (T*)(base + L.oKt);
    T* Lm = (T*)(base + L.oL);
    hipLaunchKernelGGL(form_kt_kernel<T>, dim3((nx * n + thr - 1) / thr), dim3(thr), 0, st,
                       (const T*)F, n, nx, (const T*)Hinv, Kt);
    MPCQP_CHECK_LAUNCH("form_kt_kernel");
    hipLaunchKernelGGL(form_l_kernel<T>, dim3((mt * nx + thr - 1) / thr), dim3(thr), 0, st,
                       (const T*)G, m, n, mt, nx, (const T*)Kt, Lm);
    MPCQP_CHECK_LAUNCH("form_l_kernel");
  }
  return MPCQP_OK;
}

template <typename T>
static int poly_solve_t(int batch, int n, int m, int nbox, int nx, const void* ws,
                        const void* x0, int64_t sX0, const void* f1, int64_t sF1, const void* hl,
                        const void* hu, int64_t sh, const void* lbz, const void* ubz, void* z,
                        void* y, int32_t* status, int max_iter, double tol, hipStream_t st) {
  const int mt = m + (nbox ? n : 0);
  const PolyWs L = poly_ws(sizeof(T), n, mt, nx);
  const char* base = (const char*)ws;
  DualArgs<T> a;
  a.batch = batch; a.mt = mt; a.m1 = m;
  a.M = (const T*)(base + L.oM); a.sM = 0;
  a.l1 = (const T*)hl; a.u1 = (const T*)hu; a.s1 = sh;
  a.l2 = (const T*)lbz; a.u2 = (const T*)ubz;
  a.n = n; a.nx = x0 ? nx : 0;
  a.Ut = (const T*)(base + L.oUt);
  a.Hinv = (const T*)(base + L.oHinv);
  a.Kt = (const T*)(base + L.oKt);
  a.L = (const T*)(base + L.oL);
  a.x0 = x0 ? (const T*)x0 : nullptr; a.sX0 = sX0;
  a.f1 = (const T*)f1; a.sF1 = sF1;
  a.flag = (const int32_t*)(base + L.oFlag);
  a.z = (T*)z; a.y = (T*)y; a.status = status;
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
  return MPCQP_OK;
}

}  // namespace mpcqp

extern "C" int64_t mpcqp_solve_poly_workspace(int dtype, int batch, int n, int m, int nbox) {
  (void)batch;
  const int mt = m + (nbox ? n : 0);
  return mpcqp::poly_ws(mpcqp::dtype_size(dtype), n, mt, 0).total;
}

extern "C" int64_t mpcqp_poly_workspace(int dtype, int n, int m, int nbox, int nx) {
  const int mt = m + (nbox ? n : 0);
  return mpcqp::poly_ws(mpcqp::dtype_size(dtype), n, mt, nx).total;
}

#define MPCQP_POLY_SIZES(fn)                                                                  \
  MPCQP_CHECK_ARG(dtype == MPCQP_F64 || dtype == MPCQP_F32, fn ": bad dtype %d", dtype);       \
  MPCQP_CHECK_ARG(n >= 1 && m >= 0 && nx >= 0 && nx <= 16, fn ": bad sizes");                  \
  MPCQP_CHECK_ARG(m + (nbox ? n : 0) >= 1 && m + (nbox ? n : 0) <= 64,                         \
                  fn ": rows m_total=%d outside [1,64]", m + (nbox ? n : 0));

extern "C" int mpcqp_poly_setup(int dtype, int n, int m, int nbox, int nx, const void* H,
                                const void* G, const void* F, void* workspace,
                                int64_t workspace_bytes, void* stream) {
  using namespace mpcqp;
  MPCQP_POLY_SIZES("mpcqp_poly_setup")
  MPCQP_CHECK_ARG(H && workspace, "mpcqp_poly_setup: H and workspace are required");
  MPCQP_CHECK_ARG(m == 0 || G, "mpcqp_poly_setup: G required when m > 0");
  MPCQP_CHECK_ARG(nx == 0 || F, "mpcqp_poly_setup: F required when nx > 0");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return poly_setup_t<double>(n, m, nbox, nx, H, G, F, workspace, workspace_bytes, st);
  return poly_setup_t<float>(n, m, nbox, nx, H, G, F, workspace, workspace_bytes, st);
}

extern "C" int mpcqp_poly_solve(int dtype, int batch, int n, int m, int nbox, int nx,
                                const void* workspace, const void* x0, int64_t strideX0,
                                const void* f, int64_t stridef, const void* hl, const void* hu,
                                int64_t strideh, const void* lbz, const void* ubz, void* z,
                                void* y, int32_t* status, int max_iter, double tol,
                                void* stream) {
  using namespace mpcqp;
  MPCQP_POLY_SIZES("mpcqp_poly_solve")
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_poly_solve: batch < 0");
  MPCQP_CHECK_ARG(workspace && z && status, "mpcqp_poly_solve: workspace, z, status are required");
  MPCQP_CHECK_ARG(x0 == nullptr || nx > 0, "mpcqp_poly_solve: x0 given but nx = 0");
  MPCQP_CHECK_ARG(strideX0 >= 0 && stridef >= 0 && strideh >= 0, "mpcqp_poly_solve: negative stride");
  MPCQP_CHECK_ARG(!nbox || lbz || ubz, "mpcqp_poly_solve: nbox set without lbz/ubz");
  if (batch == 0) return MPCQP_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MPCQP_F64)
    return poly_solve_t<double>(batch, n, m, nbox, nx, workspace, x0, strideX0, f, stridef, hl,
                                hu, strideh, lbz, ubz, z, y, status, max_iter, tol, st);
  return poly_solve_t<float>(batch, n, m, nbox, nx, workspace, x0, strideX0, f, stridef, hl, hu,
                             strideh, lbz, ubz, z, y, status, max_iter, tol, st);
}

extern "C" int mpcqp_solve_poly(int dtype, int batch, int n, int m, const void* H, const void* f,
                                int64_t stridef, const void* G, const void* hl, const void* hu,
                                int64_t strideh, const void* lbz, const void* ubz, void* z,
                                void* y, int32_t* status, int max_iter, double tol,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace mpcqp;
  const int nbox = (lbz || ubz) ? 1 : 0, nx = 0;
  MPCQP_POLY_SIZES("mpcqp_solve_poly")
  MPCQP_CHECK_ARG(batch >= 0, "mpcqp_solve_poly: batch < 0");
  MPCQP_CHECK_ARG(H && f && z && y && status && workspace, "mpcqp_solve_poly: null pointer");
  MPCQP_CHECK_ARG(m == 0 || G, "mpcqp_solve_poly: G required when m > 0");
  MPCQP_CHECK_ARG(stridef >= 0 && strideh >= 0, "mpcqp_solve_poly: negative stride");
  if (batch == 0) return MPCQP_OK;
  int rc = mpcqp_poly_setup(dtype, n, m, nbox, nx, H, G, nullptr, workspace, workspace_bytes,
                            stream);
  if (rc != MPCQP_OK) return rc;
  return mpcqp_poly_solve(dtype, batch, n, m, nbox, nx, workspace, nullptr, 0, f, stridef, hl,
                          hu, strideh, lbz, ubz, z, y, status, max_iter, tol, stream);
}
