// sweep.hip -- batched blocked Goodnight sweep on MFMA (fp32): the "sweep every
// z in" phase of the workgroup QP kernel (solve_qp.hip) as its own kernel.
//
// For the condensed QP of session_4/main.py:115-116 the dual active set needs
//     M = SWEEP_z(K),  K = [[H, G'], [G, 0]]
//       = [[-H^-1, H^-1 G'], [G H^-1, -G H^-1 G']]
// before its first iteration.  In qp_wg_kernel this is n rank-1 updates of
// the (n+m)^2 matrix, each behind a barrier (65 % of config 5's solve time).
// Here it is the same sweep in 16-pivot blocks: per block k, with
// D = M_kk = L L' (Cholesky), R_i = M_ki (the block row), W_i = L^-1 R_i,
//     M_ij -= W_i' W_j             (i >= j, both != k)   -- MFMA
//     M_ki  = L^-T W_i  (i < k),   M_ik = W_i' L^-1 (i > k),   M_kk = -L^-T L^-1
// which is Goodnight's a_ij - a_ik a_kj / a_kk with a_kk -> D, in the
// symmetric square-root form (as accurate as the unblocked sweep; the
// explicit-D^-1 form is not).  Sweeping every z block leaves M above (L^-1 of
// each 16 x 16 block runs on the VALU with DPP row_newbcast / ds_bpermute
// broadcasts).
//
// Layout: one instance per wavefront, the lower block triangle of the padded
// matrix held as T(T+1)/2 MFMA C-layout tiles in registers (mfma.hpp: lane
// (g, c) holds rows 4g..4g+3 of column c), so every product above is of the
// form P' Y that v_mfma_f32_16x16x4f32 takes from C-layout operands directly;
// the transposed block rows R_i = M_ik' (i > k) come from one MFMA against the
// identity (exact).  Index space: z indices at 0..n-1, padded to np = 16 KP
// with identity pivots (sweeping a decoupled unit pivot changes nothing
// else), rows at np..np+m-1.  T = ceil((np + m) / 16) <= 12.
//
// Input H packed lower (n(n+1)/2), G (m x n) row-major; output M over the
// original n + m indices, packed lower or (full) dense row-major.  status[b]: 0, MPCQP_STATUS_NOT_CONVEX (a
// pivot <= 0: H not positive definite) or MPCQP_STATUS_NONFINITE;
// mpcqp_solve_qp_ws / mpcqp_solve_box_ws consume M and that status.
#include "common.hpp"
#include "mfma.hpp"

namespace mpcqp {

struct SweepArgs {
  int batch, n, m, np, kp, full;
  const float* H; int64_t sH;
  const float* G; int64_t sG;
  float* M;
  int32_t* status;
  // optional (full only): s0 = M[:, z] f per instance (n + m), the free
  // response the product-form solver starts from
  const float* f; int64_t sf;
  float* s0;
};

__device__ __forceinline__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

__device__ __forceinline__ mf4 mm(const mf4& p, const mf4& y, mf4 acc) {
  // acc + P' Y (both C layout)
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(p[s], y[s], acc, 0, 0, 0);
  return acc;
}

template <int P>
__device__ __forceinline__ float row_bcast(float v) {
  // lane P of each 16-lane row to the whole row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + P, 0xf, 0xf, MPCQP_DPP_BC));
}

// Inverse Cholesky factor of a symmetric positive definite 16 x 16 C-layout
// tile: row operations that reduce A to L' (scale pivot row p by 1/sqrt(a_pp),
// eliminate below it) applied to X = I leave X = L^-1 (A = L L').  bad |= a
// pivot that is not > 0.  The blocked sweep below applies D^-1 = L^-T L^-1
// as W' W with W = L^-1 R: forming D^-1 explicitly and multiplying by it
// loses ~100x accuracy on ill-conditioned pivot blocks (config-3 Hessians).
__device__ __forceinline__ void chol_inv16(mf4 a, mf4& x, int g, int c, bool& bad) {
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int gp = p >> 2, ip = p & 3;
    const float piv = readlane(a[ip], 16 * gp + p);
    bad |= !(piv > 0.f);
    const float r = 1.f / __builtin_sqrtf(piv);
    float col[4];
    switch (p) {  // row_newbcast needs an immediate lane
#define MPCQP_RB(P_)                                               \
  case P_:                                                         \
    for (int i = 0; i < 4; ++i) col[i] = row_bcast<P_>(a[i]);      \
    break;
      MPCQP_RB(0) MPCQP_RB(1) MPCQP_RB(2) MPCQP_RB(3) MPCQP_RB(4) MPCQP_RB(5) MPCQP_RB(6)
      MPCQP_RB(7) MPCQP_RB(8) MPCQP_RB(9) MPCQP_RB(10) MPCQP_RB(11) MPCQP_RB(12) MPCQP_RB(13)
      MPCQP_RB(14) MPCQP_RB(15)
#undef MPCQP_RB
    }
    // scaled pivot rows: lane (gp, c), register ip
    const float ra = r * __int_as_float(
        __builtin_amdgcn_ds_bpermute(4 * (16 * gp + c), __float_as_int(a[ip])));
    const float rx = r * __int_as_float(
        __builtin_amdgcn_ds_bpermute(4 * (16 * gp + c), __float_as_int(x[ip])));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int R = 4 * g + i;
      const float mlt = col[i] * r;
      a[i] = (R == p) ? ra : (R > p ? fmaf(-mlt, ra, a[i]) : a[i]);
      x[i] = (R == p) ? rx : (R > p ? fmaf(-mlt, rx, x[i]) : x[i]);
    }
  }
}

// offsets are 32-bit bytes from a range-checked descriptor: a masked lane
// adds kOOB and reads 0 / drops its store (cols of tile column tj go in the
// instruction's immediate offset)
// (masked offsets are kOOB | x <= 0x7fffffff, so adding imm <= 4095 never wraps)
__device__ __forceinline__ float bld_i(rsrc_t r, unsigned voff, int imm) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(voff + (unsigned)imm), 0, 0));
}
__device__ __forceinline__ void bst_i(float v, rsrc_t r, unsigned voff, int imm) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(voff + (unsigned)imm), 0, 0);
}

template <int T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1)))
void sweep_mfma_kernel(SweepArgs a) {
  constexpr int NT = T * (T + 1) / 2;
  const int b = blockIdx.x;
  const int l = threadIdx.x, g = l >> 4, c = l & 15;
  const int n = a.n, m = a.m, np = a.np, kp = a.kp, nt = n + m;
  const rsrc_t rH = mk_rsrc(a.H + (int64_t)b * a.sH, (int64_t)n * (n + 1) / 2 * 4);
  const rsrc_t rG = mk_rsrc(m ? a.G + (int64_t)b * a.sG : a.H, (int64_t)m * n * 4);

  // ---- load K into the lower block triangle (z at 0..n-1, pad, rows at np..)
  mf4 t[NT];
  bool nonfin = false;
  // pad columns of the last z tile column read nothing
  const unsigned cmask = (16 * (kp - 1) + c < n) ? 0u : (unsigned)kOOB;
#pragma unroll
  for (int ti = 0; ti < T; ++ti) {
    unsigned base[4];
    if (ti < kp) {  // H rows: packed row offset
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * ti + 4 * g + i;
        base[i] = r < n ? 4 * (r * (r + 1) / 2 + c) : kOOB;
      }
    } else {  // G rows
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * ti + 4 * g + i - np;
        base[i] = r < m ? 4 * (r * n + c) : kOOB;
      }
    }
#pragma unroll
    for (int tj = 0; tj < ti; ++tj) {
      if (tj < kp) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = bld_i(ti < kp ? rH : rG, base[i] | (tj == kp - 1 ? cmask : 0u), 64 * tj);
          nonfin |= !finite(v);
          t[tri(ti, tj)][i] = v;
        }
      } else {
        t[tri(ti, tj)] = mf4{0.f, 0.f, 0.f, 0.f};
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (ti < kp) {  // diagonal z tile: mirror the upper half, unit pad pivots
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * ti + 4 * g + i, cc = 16 * ti + c;
        const int hi = r > cc ? r : cc, lo = r > cc ? cc : r;
        const float v = bld(rH, hi < n ? 4 * (hi * (hi + 1) / 2 + lo) : kOOB) +
                        ((r == cc && r >= n) ? 1.f : 0.f);
        nonfin |= !finite(v);
        t[tri(ti, ti)][i] = v;
      }
    } else {
      t[tri(ti, ti)] = mf4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  bool bad = false;
  mf4 eye;
#pragma unroll
  for (int i = 0; i < 4; ++i) eye[i] = (4 * g + i == c) ? 1.f : 0.f;
  const mf4 zero = {0.f, 0.f, 0.f, 0.f};

  // ---- blocked sweep over the z blocks: with D = M_kk = L L', R_j = M_kj,
  // W_j = L^-1 R_j:  M_ij -= W_i' W_j,  M_kj = L^-T W_j,  M_kk = -L^-T L^-1
#pragma unroll
  for (int k = 0; k < T; ++k) {
    if (k < kp) {  // uniform
      mf4 li = eye;
      chol_inv16(t[tri(k, k)], li, g, c, bad);  // L^-1
      __builtin_amdgcn_sched_barrier(0);
      const mf4 lit = mm(li, eye, zero);  // L^-T (exact transpose)
      mf4 W[T];
#pragma unroll
      for (int i = 0; i < T; ++i) {
        if (i == k) continue;
        const mf4 r = (i < k) ? t[tri(k, i)] : mm(t[tri(i, k)], eye, zero);  // M_ki
        W[i] = mm(lit, r, zero);  // L^-1 M_ki
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < T; ++j) {
        if (j == k) continue;
        const mf4 wn = -W[j];
#pragma unroll
        for (int i = j; i < T; ++i)
          if (i != k) t[tri(i, j)] = mm(W[i], wn, t[tri(i, j)]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < T; ++i) {
        if (i < k) t[tri(k, i)] = mm(li, W[i], zero);        // L^-T W_i = D^-1 M_ki
        else if (i > k) t[tri(i, k)] = mm(W[i], li, zero);   // W_i' L^-1 = M_ik D^-1
      }
      t[tri(k, k)] = mm(li, -li, zero);  // -L^-T L^-1 = -D^-1
    }
  }

  // ---- store M over the original n + m indices: packed lower, or full
  // row-major (a.full: the product-form solver reads columns as rows)
  const bool fin_bad = __builtin_amdgcn_ballot_w64(nonfin) != 0;
  const bool piv_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
  const int64_t msz = a.full ? (int64_t)nt * nt : (int64_t)nt * (nt + 1) / 2;
  const rsrc_t rM = mk_rsrc(a.M + (int64_t)b * msz, msz * 4);
  // opaque lane id: keeps the load phase's index math from being CSE'd into
  // (and kept live until) the stores
  int ls = l;
  asm volatile("" : "+v"(ls));
  const int gs = ls >> 4, cs = ls & 15;
  auto orig = [&](int X) { return X < n ? X : (X < np ? -1 : (X - np < m ? n + X - np : -1)); };
  if (!a.full) {
    // tile-space column -> original column (pad: masked)
    const unsigned czmask = (16 * (kp - 1) + cs < n) ? 0u : (unsigned)kOOB;     // last z tile column
    const unsigned crmask = (16 * (T - 1) + cs - np < m) ? 0u : (unsigned)kOOB;  // last row tile column
#pragma unroll
    for (int ti = 0; ti < T; ++ti) {
      unsigned base[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = orig(16 * ti + 4 * gs + i);
        base[i] = r >= 0 ? 4 * (r * (r + 1) / 2 + cs) : kOOB;
      }
#pragma unroll
      for (int tj = 0; tj <= ti; ++tj) {
        // column orig = C (z) or C - np + n (rows); diagonal tiles keep r >= c
        const int shift = tj < kp ? 0 : 4 * (n - np);
        const unsigned msk = (tj == kp - 1 ? czmask : 0u) | (tj == T - 1 && tj >= kp ? crmask : 0u);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned dm = (tj == ti && cs > 4 * gs + i) ? (unsigned)kOOB : 0u;
          bst_i(t[tri(ti, tj)][i], rM, (base[i] + (unsigned)shift) | msk | dm, 64 * tj);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    // tile (rb, cb) in C layout -> rows of block rb, columns of block cb;
    // part: 0 all, 1 only c <= r (diagonal, from the lower tile), 2 only c > r
    auto put = [&](const mf4& v, int rb, int cb, int part) {
      const int cc = orig(16 * cb + cs);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = 4 * gs + i, r = orig(16 * rb + rr);
        const bool keep = r >= 0 && cc >= 0 && (part == 0 || (part == 1 ? cs <= rr : cs > rr));
        bst(v[i], rM, keep ? 4 * (r * nt + cc) : kOOB);
      }
    };
    // s0 = M F with F_j = f of z block j in every column (MFMA, from the
    // tiles and their transposes on their way out)
    const bool want_s0 = a.s0 != nullptr;
    mf4 F[T], acc[T];
#pragma unroll
    for (int tj = 0; tj < T; ++tj) {
      acc[tj] = zero;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int z = 16 * tj + 4 * gs + i;
        F[tj][i] = (want_s0 && tj < kp && z < n) ? a.f[(int64_t)b * a.sf + z] : 0.f;
      }
    }
#pragma unroll
    for (int ti = 0; ti < T; ++ti)
#pragma unroll
      for (int tj = 0; tj <= ti; ++tj) {
        const mf4 tt = mm(t[tri(ti, tj)], eye, zero);  // transpose (exact)
        if (ti == tj) {
          put(t[tri(ti, tj)], ti, tj, 1);
          put(tt, ti, tj, 2);
        } else {
          put(t[tri(ti, tj)], ti, tj, 0);
          put(tt, tj, ti, 0);
        }
        if (want_s0) {
          if (tj < kp) acc[ti] = mm(tt, F[tj], acc[ti]);                       // M_ij f_j
          if (ti != tj && ti < kp) acc[tj] = mm(t[tri(ti, tj)], F[ti], acc[tj]);  // M_ji f_i
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    if (want_s0 && cs == 0) {
#pragma unroll
      for (int ti = 0; ti < T; ++ti)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = orig(16 * ti + 4 * gs + i);
          if (r >= 0) a.s0[(int64_t)b * nt + r] = acc[ti][i];
        }
    }
  }
  if (l == 0)
    a.status[b] = fin_bad ? MPCQP_STATUS_NONFINITE : (piv_bad ? MPCQP_STATUS_NOT_CONVEX : 0);
}

// ------------------------------------------------------------ rows variant
// m > 0, dense output (the product-form solver's input): only the z columns
// of the lower block triangle live in registers -- zz (KP(KP+1)/2 tiles) and
// G z (TR x KP tiles, row tile ir, z tile k) -- and the row-row block, which
// the sweep only ever subtracts into, is formed at the end as
//     M_GG = -G H^-1 G' = -M_Gz G'       (MFMA against G' re-read from HBM)
// so the register file holds 42 instead of 78 tiles at config 3 (KP = 4,
// TR = 8) and the kernel runs without spills.  G is staged in LDS once (m n
// floats, <= 36 KB; one wave per SIMD): the M_GG products read each G tile
// (jr, k) once per row tile ir >= jr, which from HBM was ~5x the bytes of G.
template <int KP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1)))
void sweep_rows_kernel(SweepArgs a) {
  constexpr int TRM = 12 - KP;  // row tiles held at most (np + m <= 192)
  constexpr int NZ = KP * (KP + 1) / 2;
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif
  const int b = blockIdx.x;
  const int l = threadIdx.x, g = l >> 4, c = l & 15;
  const int n = a.n, m = a.m, nt = n + m;
  const int tr = (m + 15) / 16;
  const float* Hb = a.H + (int64_t)b * a.sH;
  const float* Gb = a.G + (int64_t)b * a.sG;
  const rsrc_t rH = mk_rsrc(Hb, (int64_t)n * (n + 1) / 2 * 4);
  const rsrc_t rG = mk_rsrc(Gb, (int64_t)m * n * 4);
  mf4 Z[NZ], Gt[TRM][KP];
  bool nonfin = false;
  // The zz tiles (packed H, mirrored on the diagonal tiles, unit pad pivots)
  // and the G z tiles (G[rho][z], rho = 16 ir + 4g + i, z = 16 k + c) come
  // straight from HBM, every load issued before the first use (one round
  // trip); G is then kept in LDS (zero-padded to 16 tr x ldg, ldg = 16 KP +
  // 4 so that the float4 reads of the M_GG phase are bank-conflict free) for
  // the G' operands at the end.
  extern __shared__ float Gs[];
  const int ldg = 16 * KP + 4;
#pragma unroll
  for (int ti = 0; ti < KP; ++ti)
#pragma unroll
    for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * ti + 4 * g + i, cc = 16 * tj + c;
        const int hi = r > cc ? r : cc, lo = r > cc ? cc : r;
        Z[tri(ti, tj)][i] = bld(rH, hi < n ? 4 * (hi * (hi + 1) / 2 + lo) : kOOB);
      }
#pragma unroll
  for (int ir = 0; ir < TRM; ++ir)
#pragma unroll
    for (int k = 0; k < KP; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rho = 16 * ir + 4 * g + i, z = 16 * k + c;
        Gt[ir][k][i] = bld(rG, (ir < tr && rho < m && z < n) ? 4 * (rho * n + z) : kOOB);
      }
#pragma unroll
  for (int ti = 0; ti < KP; ++ti)
#pragma unroll
    for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * ti + 4 * g + i, cc = 16 * tj + c;
        nonfin |= !finite(Z[tri(ti, tj)][i]);
        Z[tri(ti, tj)][i] += (r == cc && r >= n) ? 1.f : 0.f;
      }
#pragma unroll
  for (int ir = 0; ir < TRM; ++ir) {
    if (ir < tr) {  // uniform
#pragma unroll
      for (int k = 0; k < KP; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          nonfin |= !finite(Gt[ir][k][i]);
          Gs[(16 * ir + 4 * g + i) * ldg + 16 * k + c] = Gt[ir][k][i];
        }
    }
  }
  bool bad = false;
  mf4 eye;
#pragma unroll
  for (int i = 0; i < 4; ++i) eye[i] = (4 * g + i == c) ? 1.f : 0.f;
  const mf4 zero = {0.f, 0.f, 0.f, 0.f};
  MPCQP_PHASE(0);

#pragma unroll
  for (int k = 0; k < KP; ++k) {
    mf4 li = eye;
    chol_inv16(Z[tri(k, k)], li, g, c, bad);  // L^-1
    __builtin_amdgcn_sched_barrier(0);
    MPCQP_PHASE(1);
    const mf4 lit = mm(li, eye, zero);
    mf4 Wz[KP];
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i == k) continue;
      const mf4 r = (i < k) ? Z[tri(k, i)] : mm(Z[tri(i, k)], eye, zero);
      Wz[i] = mm(lit, r, zero);
    }
    // zz block
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      if (j == k) continue;
      const mf4 wn = -Wz[j];
#pragma unroll
      for (int i = j; i < KP; ++i)
        if (i != k) Z[tri(i, j)] = mm(Wz[i], wn, Z[tri(i, j)]);
    }
    __builtin_amdgcn_sched_barrier(0);
    MPCQP_PHASE(2);
    // row tiles, one W at a time: M_rho,j -= W_rho' W_j, M_rho,k = W_rho' L^-1
#pragma unroll
    for (int ir = 0; ir < TRM; ++ir) {
      if (ir < tr) {  // uniform
        const mf4 wr = mm(lit, mm(Gt[ir][k], eye, zero), zero);  // L^-1 M_k,rho
#pragma unroll
        for (int j = 0; j < KP; ++j)
          if (j != k) Gt[ir][j] = mm(wr, -Wz[j], Gt[ir][j]);
        Gt[ir][k] = mm(wr, li, zero);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    MPCQP_PHASE(3);
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      if (i < k) Z[tri(k, i)] = mm(li, Wz[i], zero);
      else if (i > k) Z[tri(i, k)] = mm(Wz[i], li, zero);
    }
    Z[tri(k, k)] = mm(li, -li, zero);
    __builtin_amdgcn_sched_barrier(0);
    MPCQP_PHASE(4);
  }

  const bool fin_bad = __builtin_amdgcn_ballot_w64(nonfin) != 0;
  const bool piv_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
  const rsrc_t rM = mk_rsrc(a.M + (int64_t)b * nt * nt, (int64_t)nt * nt * 4);
  int ls = l;
  asm volatile("" : "+v"(ls));
  const int gs = ls >> 4, cs = ls & 15;
  // dense store of a C-layout tile: rows rb / columns cb of the ORIGINAL
  // index space (z tile k -> 16k, row tile ir -> n + 16 ir); part as in the
  // generic kernel (1: c <= r only, 2: c > r only)
  auto put = [&](const mf4& v, int rb, bool rrow, int cb, bool crow, int part) {
    const int c0 = crow ? 16 * cb + cs : 16 * cb + cs;
    const int cc = crow ? (c0 < m ? n + c0 : -1) : (c0 < n ? c0 : -1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = 4 * gs + i, r0 = 16 * rb + rr;
      const int r = rrow ? (r0 < m ? n + r0 : -1) : (r0 < n ? r0 : -1);
      const bool keep = r >= 0 && cc >= 0 && (part == 0 || (part == 1 ? cs <= rr : cs > rr));
      bst(v[i], rM, keep ? 4 * (r * nt + cc) : kOOB);
    }
  };
  const bool want_s0 = a.s0 != nullptr;
  mf4 F[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int z = 16 * k + 4 * gs + i;
      F[k][i] = (want_s0 && z < n) ? a.f[(int64_t)b * a.sf + z] : 0.f;
    }
  // zz tiles and the z part of s0
  {
    mf4 acc[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) acc[k] = zero;
#pragma unroll
    for (int ti = 0; ti < KP; ++ti)
#pragma unroll
      for (int tj = 0; tj <= ti; ++tj) {
        const mf4 tt = mm(Z[tri(ti, tj)], eye, zero);
        if (ti == tj) {
          put(Z[tri(ti, tj)], ti, false, tj, false, 1);
          put(tt, ti, false, tj, false, 2);
        } else {
          put(Z[tri(ti, tj)], ti, false, tj, false, 0);
          put(tt, tj, false, ti, false, 0);
        }
        if (want_s0) {
          acc[ti] = mm(tt, F[tj], acc[ti]);
          if (ti != tj) acc[tj] = mm(Z[tri(ti, tj)], F[ti], acc[tj]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    if (want_s0 && cs == 0) {
#pragma unroll
      for (int k = 0; k < KP; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * k + 4 * gs + i;
          if (r < n) a.s0[(int64_t)b * nt + r] = acc[k][i];
        }
    }
  }
  MPCQP_PHASE(5);
  // G z tiles (and their transposes, the z-row block), the row part of s0,
  // then the row-row block -M_Gz G'
#pragma unroll
  for (int ir = 0; ir < TRM; ++ir) {
    if (ir < tr) {
      mf4 acc = zero;
      mf4 tts[KP];
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        tts[k] = mm(Gt[ir][k], eye, zero);
        put(Gt[ir][k], ir, true, k, false, 0);
        put(tts[k], k, false, ir, true, 0);
        if (want_s0) acc = mm(tts[k], F[k], acc);
      }
      if (want_s0 && cs == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rho = 16 * ir + 4 * gs + i;
          if (rho < m) a.s0[(int64_t)b * nt + n + rho] = acc[i];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // G(jr, k)' in C layout: lane (g, c) holds G[16 jr + c][16 k + 4g + e],
      // one float4 of the padded LDS copy (zero outside m x n)
      auto gtile = [&](int jr, int k) __attribute__((always_inline)) {
        const float4 v = *reinterpret_cast<const float4*>(&Gs[(16 * jr + cs) * ldg + 16 * k + 4 * gs]);
        return mf4{v.x, v.y, v.z, v.w};
      };
      auto emit = [&](mf4 gg, int jr) __attribute__((always_inline)) {
        gg = -gg;
        const mf4 ggt = mm(gg, eye, zero);
        if (jr == ir) {
          put(gg, ir, true, jr, true, 1);
          put(ggt, ir, true, jr, true, 2);
        } else {
          put(gg, ir, true, jr, true, 0);
          put(ggt, jr, true, ir, true, 0);
        }
      };
      // two independent accumulation chains at a time (MFMA dependent
      // latency, one wave per SIMD)
      int jr = 0;
      for (; jr + 1 <= ir; jr += 2) {
        mf4 g0 = zero, g1 = zero;
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          g0 = mm(tts[k], gtile(jr, k), g0);  // M_Gz(ir, k) G(jr, k)'
          g1 = mm(tts[k], gtile(jr + 1, k), g1);
        }
        emit(g0, jr);
        emit(g1, jr + 1);
      }
      if (jr <= ir) {
        mf4 g0 = zero;
#pragma unroll
        for (int k = 0; k < KP; ++k) g0 = mm(tts[k], gtile(jr, k), g0);
        emit(g0, jr);
      }
    }
  }
  if (l == 0)
    a.status[b] = fin_bad ? MPCQP_STATUS_NONFINITE : (piv_bad ? MPCQP_STATUS_NOT_CONVEX : 0);
  MPCQP_PHASE(6);
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

template <int KP>
static int launch_sweep_rows(const SweepArgs& a, hipStream_t st) {
  const size_t lds = (size_t)((a.m + 15) / 16 * 16) * (16 * KP + 4) * sizeof(float);  // G staged per wave
  hipLaunchKernelGGL((sweep_rows_kernel<KP>), dim3(a.batch), dim3(64), lds, st, a);
  MPCQP_CHECK_LAUNCH("sweep_rows_kernel");
  return MPCQP_OK;
}

template <int T>
static int launch_sweep_t(const SweepArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((sweep_mfma_kernel<T>), dim3(a.batch), dim3(64), 0, st, a);
  MPCQP_CHECK_LAUNCH("sweep_mfma_kernel");
  return MPCQP_OK;
}

// tiles of the padded index space, or 0 when the MFMA sweep does not apply
int sweep_tiles(int dtype, int n, int m) {
  if (dtype != MPCQP_F32 || n < 1 || m < 0) return 0;
  const int np = (n + 15) / 16 * 16;
  const int T = (np + m + 15) / 16;
  return (T >= 5 && T <= 12) ? T : 0;
}

// -H^-1 (n x n, row-major full) and s0 = -H^-1 f for 48 < n <= 64 (four
// z tiles, no rows): the inverse the z-space kernel (solve_zf.hip) iterates
// with, on MFMA in square-root form
int sweep_hinv(int batch, int n, const void* H, int64_t sH, const void* f, int64_t sf, void* M,
               void* s0, int32_t* status, hipStream_t st) {
  if (n <= 48 || n > 64) {
    set_error("sweep_hinv: n = %d outside 49..64", n);
    return MPCQP_ENOTSUP;
  }
  SweepArgs a;
  a.batch = batch; a.n = n; a.m = 0; a.full = 1;
  a.f = (const float*)f; a.sf = sf; a.s0 = (float*)s0;
  a.np = 64;
  a.kp = 4;
  a.H = (const float*)H; a.sH = sH;
  a.G = nullptr; a.sG = 0;
  a.M = (float*)M;
  a.status = status;
  return launch_sweep_t<4>(a, st);
}

int sweep_launch(int batch, int n, int m, const void* H, int64_t sH, const void* G, int64_t sG,
                 void* M, int full, int32_t* status, hipStream_t st, const void* f, int64_t sf,
                 void* s0) {
  SweepArgs a;
  a.batch = batch; a.n = n; a.m = m; a.full = full ? 1 : 0;
  a.f = (const float*)f; a.sf = sf; a.s0 = full ? (float*)s0 : nullptr;
  a.np = (n + 15) / 16 * 16;
  a.kp = a.np / 16;
  a.H = (const float*)H; a.sH = sH;
  a.G = (const float*)G; a.sG = sG;
  a.M = (float*)M;
  a.status = status;
  if (full && m > 0) {
    switch (a.kp) {
      case 1: return launch_sweep_rows<1>(a, st);
      case 2: return launch_sweep_rows<2>(a, st);
      case 3: return launch_sweep_rows<3>(a, st);
      case 4: return launch_sweep_rows<4>(a, st);
      case 5: return launch_sweep_rows<5>(a, st);
      case 6: return launch_sweep_rows<6>(a, st);
      default: break;  // wider z blocks: the generic kernel
    }
  }
  switch (sweep_tiles(MPCQP_F32, n, m)) {
    case 5: return launch_sweep_t<5>(a, st);
    case 6: return launch_sweep_t<6>(a, st);
    case 7: return launch_sweep_t<7>(a, st);
    case 8: return launch_sweep_t<8>(a, st);
    case 9: return launch_sweep_t<9>(a, st);
    case 10: return launch_sweep_t<10>(a, st);
    case 11: return launch_sweep_t<11>(a, st);
    case 12: return launch_sweep_t<12>(a, st);
    default:
      set_error("mpcqp_sweep: padded n + m = %d outside the MFMA sweep's 65..192", (n + 15) / 16 * 16 + m);
      return MPCQP_ENOTSUP;
  }
}

}  // namespace mpcqp

extern "C" int mpcqp_sweep(int dtype, int batch, int n, int m, const void* H, int64_t strideH,
                           const void* G, int64_t strideG, void* M, int full,
                           int32_t* status, void* stream) {
  using namespace mpcqp;
  MPCQP_CHECK_ARG(dtype == MPCQP_F32, "mpcqp_sweep: only MPCQP_F32 runs on the MFMA sweep");
  MPCQP_CHECK_ARG(batch >= 0 && n >= 1 && m >= 0, "mpcqp_sweep: bad sizes");
  MPCQP_CHECK_ARG(H && M && status && (m == 0 || G), "mpcqp_sweep: H, M, status (and G) required");
  MPCQP_CHECK_ARG(strideH >= 0 && strideG >= 0, "mpcqp_sweep: negative stride");
  MPCQP_CHECK_ARG(sweep_tiles(dtype, n, m) > 0, "mpcqp_sweep: padded n + m = %d outside 65..192",
                  (n + 15) / 16 * 16 + m);
  if (batch == 0) return MPCQP_OK;
  return sweep_launch(batch, n, m, H, strideH, G, strideG, M, full, status, (hipStream_t)stream,
                      nullptr, 0, nullptr);
}

#ifdef MPCQP_PHASE_TIMING
MPCQP_DEBUG_PHASE_READER(mpcqp_debug_phase_cycles_sweep)
#endif
