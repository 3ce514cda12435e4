// solve_pf.hip -- the mixed primal/dual active set of solve_qp.hip (wg.hpp
// gi_mixed) in PRODUCT FORM on the pre-swept matrix of sweep.hip, one QP
// instance per wavefront.  This is the fp32 path of mpcqp_solve_qp_ws /
// mpcqp_solve_box_ws (BASELINE configs 3 and 5: the per-step QP of
// session_4/main.py:115-116 with the input box main.py:68-69 and the state
// box main.py:58-61).
//
// gi_mixed keeps the current swept matrix M = SWEEP_P(M0) (P = fixed z and
// active rows, M0 = SWEEP_z(K) from sweep.hip) in registers and applies one
// rank-1 sweep of the whole (n+m)^2 matrix per iteration, behind workgroup
// barriers.  With S = -M0[P,P] (positive definite while the active
// constraints are independent) every entry that iteration needs follows from
// M0 and S^-1 alone:
//     M[i,p] = M0[i,p] + M0[i,P] v,      v = S^-1 M0[P,p]        (i, p not in P)
//     M[a,p] = -s_a v_a                  (a in P; s_a = -1 fixed z, +1 active row)
//     M[a,b] = s_a s_b S^-1[a,b]
// so an iteration reads column p and the |P| active columns of M0 (rows of
// the symmetric dense M0, coalesced), and updates S^-1 by a bordered-inverse
// rank-1 step (add) or a Schur rank-1 step (drop): O((n+m)|P| + |P|^2)
// instead of O((n+m)^2), with no barrier and with register state small
// enough for several instances per SIMD.
//
// Layout: index i = lane + 64 r (r < NR); slot j of the active set = lane j,
// which holds row j of S^-1 in 64 registers (unused slots are zero rows and
// columns), the index a_j and its bound.  More than 64 active constraints
// (n > 64 only) hands the instance to the workgroup kernel (kStatusRetry).
// The refinement (iterative refinement of the final active set with an fp64
// KKT residual) follows gi_mixed.  The residual comes from one of:
//   * the ORIGINAL H, G (fp32 data, fp64 accumulation): K x streamed through
//     LDS -- the generic QP of mpcqp_solve_qp_ws;
//   * the DYNAMICS (DYN = true, mpcqp_mpc_qp): H z + f + G'lam and G z - h
//     from an fp64 forward rollout x_{k+1} = A_k x_k + B_k u_k + c_k and the
//     adjoint lam_k = Qhat x_k + mu_k + A_k' lam_{k+1}, g_k = R u_k +
//     B_k' lam_{k+1}.  This is the residual of the QP the fp32 inputs define
//     exactly (no fp32 rounding of the condensed H, Gam, xbar), so refinement
//     converges past the fp32 condensing floor, and it costs O(N nx (nx+nu))
//     instead of O((n+m)^2) reads.
#include <cstdlib>

// DPP moves keep the old encoding here (bound_ctrl clear, common.hpp): A/B on
// config 5 (tools/ab_run.sh 5 dppold, 200-step lines): the new encoding made
// qp_pf_kernel 3.97 -> 4.14 ms, while every other kernel gained 0.5-5 %
#define MPCQP_DPP_BC false

#include "mfma.hpp"
#include "pfdyn.hpp"

namespace mpcqp {

struct PfArgs {
  int batch, n, m;
  const float* H; int64_t sH;  // packed lower n x n (refinement)
  const float* f; int64_t sf;
  const float* G; int64_t sG;  // m x n row-major (refinement)
  const float* hl; const float* hu; int64_t sh;
  const float* lb; int64_t sLb;
  const float* ub; int64_t sUb;
  const float* M0;             // sweep.hip full output, (n+m)^2 per instance
  const float* s0;             // sweep.hip: M0[:, z] f, (n+m) per instance
  float* z; float* y; int32_t* status;
  int* retry_count; int* retry_list;
  int max_iter, refine;
  float tol;
  PfDyn d;                     // DYN kernels only
  float dyn_stop;              // DYN: refinement stop (kDynStop; MPCQP_DYN_STOP)
};
template <int NR, int NXP>
__global__ __launch_bounds__(64, 2) void qp_pf_kernel(PfArgs a) {
  __shared__ float xb[NR * kWave];
  // per-index bounds and scales live in LDS (read by the scan and the
  // output only): keeps them out of the register budget
  __shared__ float s_lo[NR * kWave], s_hi[NR * kWave], s_sl[NR * kWave], s_su[NR * kWave],
      s_scl[NR * kWave];
  __shared__ __attribute__((aligned(16))) float sx[kSlots];  // slot-vector broadcast
  // refinement scratch (K-pass or DYN layout); during the active set, the
  // M0 row cache (below), extended past the refinement's needs where the row
  // cache is on: 34 KB of LDS per wave, 4 waves per CU
  constexpr bool kCache = NXP <= 4;
  // past kPool: the row cache's extra rows (active set) or, in the DYN
  // refinement, the low parts of the refined values (NR * 64 floats)
  constexpr int kExtD = NR * kWave / 2;
  static_assert(kExtD <= kPoolCacheExtra, "the refinement's low parts fit the cache extension");
  constexpr int kPoolX = kCache ? kPool + kPoolCacheExtra : (NXP > 0 ? kPool + kExtD : kPool);
  __shared__ double pool[kPoolX];
  double* red = pool;
  double* rsum = pool + 8 * kWave;
  float* kbuf = reinterpret_cast<float*>(pool + 11 * kWave);  // rows of K staged per chunk
  static_assert(NR <= 3, "rsum holds 3 * 64 doubles");
  static_assert(kKChunk >= 8 * NR * kWave, "8 rows of K (<= NR*64 floats each) must fit one chunk");
  static_assert(kKChunk % kWave == 0, "chunk is whole wave loads");
  const int b = blockIdx.x, l = threadIdx.x;
  const int n = a.n, m = a.m, nt = n + m;
  const float* M0 = a.M0 + (int64_t)b * nt * nt;
  // M0 rows through a range-checked descriptor: a masked lane (past nt, or an
  // empty slot) loads 0 with no exec-mask branch around the load
  const rsrc_t rM0 = mk_rsrc(M0, (int64_t)nt * nt * 4);
  const float* fb = a.f + (int64_t)b * a.sf;
  const float inf = Lim<float>::inf();
  const int pre = a.status[b];  // sweep status
#ifdef MPCQP_PHASE_TIMING
  PhaseClock mpcqp_clk;
#endif

  float fz[NR], val[NR], mu[NR], s0[NR];
  int st[NR], slot[NR];
  bool bad = false, nonfin = false;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int i = l + kWave * r;
    float lv = -inf, uv = inf, fi = 0.f;
    if (i < n) {
      if (a.lb) lv = a.lb[(int64_t)b * a.sLb + i];
      if (a.ub) uv = a.ub[(int64_t)b * a.sUb + i];
      fi = fb[i];
    } else if (i < nt) {
      if (a.hl) lv = a.hl[(int64_t)b * a.sh + (i - n)];
      if (a.hu) uv = a.hu[(int64_t)b * a.sh + (i - n)];
    }
    bad |= i < nt && (!(lv <= uv) || lv == inf || uv == -inf);
    nonfin |= !finite(fi);
    s_lo[i] = lv;
    s_hi[i] = uv;
    fz[r] = fi;
    s_sl[i] = finite(lv) ? 1.f / (1.f + fabsf(lv)) : __builtin_nanf("");
    s_su[i] = finite(uv) ? 1.f / (1.f + fabsf(uv)) : __builtin_nanf("");
    st[r] = i < nt ? 0 : 3;
    slot[r] = -1;
    val[r] = 0.f;
    mu[r] = 0.f;
    s_scl[i] = i < nt ? fabsf(M0[(int64_t)i * nt + i]) : 0.f;
    s0[r] = i < nt ? a.s0[(int64_t)b * nt + i] : 0.f;
  }
  // active-set slots: lane j = slot j
  int aidx = -1, sisz = 0;
  float sbnd = 0.f;
  float S[kSlots];
#pragma unroll
  for (int j = 0; j < kSlots; ++j) S[j] = 0.f;
  uint64_t used = 0;
  // Row cache: during the active set the refinement pool is free, and holds
  // the M0 rows of the first ncache slots (written when a constraint joins,
  // from the raw column p already in registers), so the per-iteration
  // M0[:, P] v reads those from LDS instead of HBM.  cmask = cached slots;
  // the refinement's residual reuses the pool and clears it.
  // (measured: pays at config 3; with the wide-state DYN residual (NXP >= 8,
  // config 5) the extra registers spill and it costs more than it saves)
  float* cache = reinterpret_cast<float*>(pool);
  const int ncache = !kCache ? 0 : ((2 * kPoolX) / nt < kSlots ? (2 * kPoolX) / nt : kSlots);
  uint64_t cmask = 0;

  int code = MPCQP_STATUS_OPTIMAL, iters = 0;
  if (pre) {
    code = pre;
  } else if (__builtin_amdgcn_ballot_w64(nonfin)) {
    code = MPCQP_STATUS_NONFINITE;
  } else if (__builtin_amdgcn_ballot_w64(bad)) {
    code = MPCQP_STATUS_INFEASIBLE;
  }
  if (code != MPCQP_STATUS_OPTIMAL) goto out;

  {
    const float dep_tol = 2e-5f;
    // ---------------------------------------------------------- helpers
    // value at index a_j in lane j (0 in unused slots)
    auto gather = [&](const float (&x)[NR]) -> float {
#pragma unroll
      for (int r = 0; r < NR; ++r) xb[l + kWave * r] = x[r];
      wave_lds_sync();
      const float v = aidx >= 0 ? xb[aidx] : 0.f;
      wave_lds_sync();
      return v;
    };
    // slot vector t (lane j) to every lane through LDS: 16 broadcast b128
    // reads instead of 64 v_readlane (which pile up in SGPRs and spill)
    auto bcast_slots = [&](float t) __attribute__((always_inline)) {
      wave_lds_sync();
      sx[l] = t;
      wave_lds_sync();
    };
    auto slot4 = [&](int j4) __attribute__((always_inline)) { return *reinterpret_cast<const float4*>(&sx[4 * j4]); };
    // lane i: (S^-1 t)_i
    auto smul = [&](float t) __attribute__((always_inline)) -> float {
      bcast_slots(t);
      float q = 0.f;
#pragma unroll
      for (int j4 = 0; j4 < kSlots / 4; ++j4) {
        const float4 tv = slot4(j4);
        q = fmaf(S[4 * j4 + 0], tv.x, q);
        q = fmaf(S[4 * j4 + 1], tv.y, q);
        q = fmaf(S[4 * j4 + 2], tv.z, q);
        q = fmaf(S[4 * j4 + 3], tv.w, q);
      }
      return q;
    };
    // out += sum_t c_t M0[row_t, :] for kB rows at a time: every row's loads
    // are issued before the first FMA (one memory round trip per batch)
#ifndef MPCQP_PF_KB
#define MPCQP_PF_KB 8
#endif
    constexpr int kB = MPCQP_PF_KB;  // active rows per memory round trip
    constexpr int kZB = 8;           // z rows per batch in zcols (double-buffered)
    auto axpy_rows = [&](const int (&row)[kB], const float (&c)[kB], float (&out)[NR]) {
      float v[kB][NR];
#pragma unroll
      for (int t = 0; t < kB; ++t) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int i = l + kWave * r;
          v[t][r] = bld(rM0, (row[t] >= 0 && i < nt) ? 4 * (row[t] * nt + i) : kOOB);  // row -1: empty
        }
      }
#pragma unroll
      for (int t = 0; t < kB; ++t)
#pragma unroll
        for (int r = 0; r < NR; ++r) out[r] = fmaf(c[t], v[t][r], out[r]);
    };
    // out += sign * M0[:, P] q  (rows a_j of the symmetric M0); fixed_z_f:
    // coefficient -f_a on the fixed z instead (rows contribute nothing)
    // cached slots: the row from LDS, no memory round trip
    // (kCB slots per LDS round trip: all their reads issued before the FMAs)
    auto ccols = [&](float q, float (&out)[NR], float sign, bool fixed_z_f, uint64_t mm) {
      if constexpr (!kCache) return;
      constexpr int kCB = 4;
      while (mm) {
        float c[kCB], v[kCB][NR];
        // an empty entry of the last batch re-reads the previous entry's row
        // with coefficient 0: the pool outside the cached slots holds the
        // refinement's doubles, whose bits can be NaN (and 0 * NaN = NaN)
        int j = 0;
#pragma unroll
        for (int t = 0; t < kCB; ++t) {
          c[t] = 0.f;
          if (mm) {
            j = __builtin_ctzll(mm);
            mm &= mm - 1;
            const int aj = readlane(aidx, j);
            c[t] = fixed_z_f ? (aj < n ? -fb[aj] : 0.f) : sign * readlane(q, j);
          }
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            v[t][r] = cache[j * nt + (i < nt ? i : 0)];
          }
        }
#pragma unroll
        for (int t = 0; t < kCB; ++t)
#pragma unroll
          for (int r = 0; r < NR; ++r) out[r] = fmaf(c[t], l + kWave * r < nt ? v[t][r] : 0.f, out[r]);
      }
    };
    auto pcols = [&](float q, float (&out)[NR], float sign, bool fixed_z_f, uint64_t mm) {
      if constexpr (kCache) {
        ccols(q, out, sign, fixed_z_f, mm & cmask);
        mm &= ~cmask;
      }
      while (mm) {
        int row[kB];
        float c[kB];
#pragma unroll
        for (int t = 0; t < kB; ++t) {
          row[t] = -1;
          c[t] = 0.f;
          if (mm) {
            const int j = __builtin_ctzll(mm);
            mm &= mm - 1;
            const int aj = readlane(aidx, j);
            row[t] = aj;
            c[t] = fixed_z_f ? (aj < n ? -fb[aj] : 0.f) : sign * readlane(q, j);
          }
        }
        axpy_rows(row, c, out);
      }
    };
    // out += M0[:, F] w_F over the FREE z only (w is zero on fixed z, whose
    // rows are skipped); kZB rows per memory round trip, the next batch in
    // flight while the current one is accumulated
    auto zcols_free = [&](const float (&wv)[NR], float (&out)[NR]) {
      uint64_t mk0 = __builtin_amdgcn_ballot_w64(st[0] == 0 && l < n);
      uint64_t mk1 = NR > 1 ? __builtin_amdgcn_ballot_w64(st[NR > 1 ? 1 : 0] == 0 && l + kWave < n) : 0;
      uint64_t mk2 = NR > 2 ? __builtin_amdgcn_ballot_w64(st[NR > 2 ? 2 : 0] == 0 && l + 2 * kWave < n) : 0;
      auto take = [&](int& j, float& c) __attribute__((always_inline)) {
        j = -1;
        c = 0.f;
        if (mk0) {
          const int bit = __builtin_ctzll(mk0);
          mk0 &= mk0 - 1;
          j = bit;
          c = readlane(wv[0], bit);
        } else if (mk1) {
          const int bit = __builtin_ctzll(mk1);
          mk1 &= mk1 - 1;
          j = kWave + bit;
          c = readlane(wv[NR > 1 ? 1 : 0], bit);
        } else if (mk2) {
          const int bit = __builtin_ctzll(mk2);
          mk2 &= mk2 - 1;
          j = 2 * kWave + bit;
          c = readlane(wv[NR > 2 ? 2 : 0], bit);
        }
      };
      auto load = [&](float (&v)[kZB][NR], float (&c)[kZB]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < kZB; ++t) {
          int j;
          take(j, c[t]);
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            v[t][r] = bld(rM0, (j >= 0 && i < nt) ? 4 * (j * nt + i) : kOOB);  // exhausted slots: 0
          }
        }
      };
      float v[kZB][NR], c[kZB];
      load(v, c);
      while (true) {
        const bool more = (mk0 | mk1 | mk2) != 0;
        float vn[kZB][NR], cn[kZB];
        if (more) load(vn, cn);
#pragma unroll
        for (int t = 0; t < kZB; ++t)
#pragma unroll
          for (int r = 0; r < NR; ++r) out[r] = fmaf(c[t], v[t][r], out[r]);
        if (!more) break;
#pragma unroll
        for (int t = 0; t < kZB; ++t) {
          c[t] = cn[t];
#pragma unroll
          for (int r = 0; r < NR; ++r) v[t][r] = vn[t][r];
        }
      }
    };
    // out += M0[:, z] c_z with c_z = coef(j) for j < n; the next batch's
    // rows are in flight while the current one is accumulated
    auto zcols = [&](auto&& coef, float (&out)[NR]) {
      auto load = [&](int j0, float (&v)[kZB][NR], float (&c)[kZB]) {
#pragma unroll
        for (int t = 0; t < kZB; ++t) {
          const int j = j0 + t < n ? j0 + t : 0;
          c[t] = j0 + t < n ? coef(j0 + t) : 0.f;
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            v[t][r] = bld(rM0, i < nt ? 4 * (j * nt + i) : kOOB);
          }
        }
      };
      float v[kZB][NR], c[kZB];
      load(0, v, c);
      for (int j0 = 0; j0 < n; j0 += kZB) {
        float vn[kZB][NR], cn[kZB];
        load(j0 + kZB < n ? j0 + kZB : 0, vn, cn);
#pragma unroll
        for (int t = 0; t < kZB; ++t)
#pragma unroll
          for (int r = 0; r < NR; ++r) out[r] = fmaf(c[t], v[t][r], out[r]);
#pragma unroll
        for (int t = 0; t < kZB; ++t) {
          c[t] = cn[t];
#pragma unroll
          for (int r = 0; r < NR; ++r) v[t][r] = vn[t][r];
        }
      }
    };
    // exact state from s = M w (gi_mixed refresh) in product form:
    //   y = M0[:, Pc] w_Pc = s0 - M0[:, fixed z] f,  q = S^-1 (y_P - w'_P),
    //   (Ms w')_i = y_i + M0[i, P] q (i not in P), -q_i (i in P);  s = J_R Ms w'
    auto refresh = [&]() __attribute__((always_inline)) {
      float yv[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) yv[r] = s0[r];
      pcols(0.f, yv, 1.f, true, used);
      const float ys = gather(yv);
      const float t = aidx >= 0 ? ys - (sisz ? sbnd : -sbnd) : 0.f;
      const float q = smul(t);
      pcols(q, yv, 1.f, false, used);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int i = l + kWave * r;
        const bool isz = i < n;
        const bool act = st[r] == 1 || st[r] == 2;
        const float qi = bperm(q, slot[r] < 0 ? 0 : slot[r]);
        const float msw = act ? -qi : yv[r];
        const float s = (act && isz) ? -msw : msw;
        const float bnd = (st[r] == 1) ? s_lo[i] : s_hi[i];
        const float mval = isz ? fz[r] - s : s;
        const float sside = ((st[r] == 1) ? 1.f : -1.f) * (isz ? 1.f : -1.f);
        val[r] = act ? bnd : (isz ? s : -s);
        mu[r] = act ? sside * mval : 0.f;
      }
    };
    auto scan = [&](float& viol, int& p) __attribute__((always_inline)) {
      viol = -inf;
      p = 0;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int i = l + kWave * r;
        const float vl = (s_lo[i] - val[r]) * s_sl[i];  // NaN (never wins) for infinite bounds
        const float vu = (val[r] - s_hi[i]) * s_su[i];
        float v = (st[r] == 0) ? fmaxf(vl, vu) : -inf;
        v = (v == v) ? v : -inf;
        const bool take = v > viol;
        viol = take ? v : viol;
        p = take ? i : p;
      }
      wave_argmax(viol, p);
      p = uniform(p);
      viol = readlane(viol, 0);
    };
    // S^-1 of P + {p}: bordered inverse, S^-1 += w w' / sigma with w = v
    // and w_snew = 1 (row/column snew were zero)
    auto s_add = [&](float v, int snew, float sigma) __attribute__((always_inline)) {
      const float w = (l == snew) ? 1.f : v;
      const float wi = w / sigma;
      bcast_slots(w);
#pragma unroll
      for (int j4 = 0; j4 < kSlots / 4; ++j4) {
        const float4 wv = slot4(j4);
        S[4 * j4 + 0] = fmaf(wi, wv.x, S[4 * j4 + 0]);
        S[4 * j4 + 1] = fmaf(wi, wv.y, S[4 * j4 + 1]);
        S[4 * j4 + 2] = fmaf(wi, wv.z, S[4 * j4 + 2]);
        S[4 * j4 + 3] = fmaf(wi, wv.w, S[4 * j4 + 3]);
      }
    };
    // row q of S^-1 (lane q's registers) to LDS
    auto s_row = [&](int q) __attribute__((always_inline)) {
      wave_lds_sync();
      if (l == q) {
#pragma unroll
        for (int j4 = 0; j4 < kSlots / 4; ++j4)
          *reinterpret_cast<float4*>(&sx[4 * j4]) =
              float4{S[4 * j4], S[4 * j4 + 1], S[4 * j4 + 2], S[4 * j4 + 3]};
      }
      wave_lds_sync();
    };
    // S^-1 of P - {slot q} (row q already in sx): Schur step, then row and
    // column q exactly zero
    auto s_drop = [&](int q, float dqq) __attribute__((always_inline)) {
      const float c = -sx[l] / dqq;  // -S[l][q] / S[q][q]  (symmetric)
#pragma unroll
      for (int j4 = 0; j4 < kSlots / 4; ++j4) {
        const float4 rv = slot4(j4);
        const float r4[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * j4 + e;
          S[j] = (l == q || j == q) ? 0.f : fmaf(c, r4[e], S[j]);
        }
      }
    };

    MPCQP_PHASE_K(0);
    refresh();
    MPCQP_PHASE_K(1);
    // DYN: after the refinement, the exact values are re-scanned with a tight
    // tolerance; a bound the fp32 active set left within a.tol of violation
    // (invisible to it, but amplified by ill-conditioning) re-enters the
    // active set, and the refinement runs again
    // Only the first scan of a round >= 1 sees refined values; every later
    // scan follows refresh() or fp32 active-set steps and keeps a.tol (the
    // fp32 floor would show as spurious violations of kDynTol)
    bool gi_skip = false;  // after a dual release: refine before the next scan
    for (int round = 0; round < (NXP > 0 ? kDynRounds : 1); ++round) {
    bool active = !gi_skip;
    gi_skip = false;
    bool tight = round > 0;
    for (int pass = 0; pass < 3 && active; ++pass) {
      while (true) {
        float viol;
        int p;
        scan(viol, p);
        const float tolc = tight ? kDynTol : a.tol;
        tight = false;
        if (!(viol > tolc)) break;
        const float valp0 = pick<NR>(val, p);
        float valp = valp0;
        const float lop = s_lo[p], hip = s_hi[p];
        const int side = (valp < lop) ? 1 : 2;
        const float tgt = (side == 1) ? lop : hip;
        const bool pz = p < n;
        const float epsp = pz ? -1.f : 1.f;
        const float sidesign = ((side == 1) ? 1.f : -1.f) * (pz ? 1.f : -1.f);
        const float sgn = (tgt > valp) ? 1.f : -1.f;
        const float scp = s_scl[p];
        float tau = 0.f;
        bool added = false;
        while (!added) {
          if (++iters > a.max_iter) {
            code = MPCQP_STATUS_MAXITER;
            goto out;
          }
          // column p of the current M.  The first kB active rows of M0 are
          // loaded in the same memory round trip as column p (their indices
          // are known; only their coefficients v wait for the column)
          float col[NR], v0[kB][NR], rawc[NR];
          int j0[kB];
          uint64_t mrest = kCache ? used & ~cmask : used;
          {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              const int i = l + kWave * r;
              col[r] = bld(rM0, i < nt ? 4 * (p * nt + i) : kOOB);
              if constexpr (kCache) rawc[r] = col[r];
            }
#pragma unroll
            for (int t = 0; t < kB; ++t) {
              j0[t] = -1;
              int aj = 0;
              if (mrest) {
                j0[t] = __builtin_ctzll(mrest);
                mrest &= mrest - 1;
                aj = readlane(aidx, j0[t]);
              }
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                const int i = l + kWave * r;
                v0[t][r] = bld(rM0, (j0[t] >= 0 && i < nt) ? 4 * (aj * nt + i) : kOOB);  // empty: 0
              }
            }
          }
          MPCQP_PHASE_K(2);
          const float u = gather(col);
          const float v = smul(u);
          MPCQP_PHASE_K(3);
#pragma unroll
          for (int t = 0; t < kB; ++t) {
            const float c = j0[t] >= 0 ? readlane(v, j0[t]) : 0.f;
#pragma unroll
            for (int r = 0; r < NR; ++r) col[r] = fmaf(c, v0[t][r], col[r]);
          }
          if constexpr (kCache) ccols(v, col, 1.f, false, used & cmask);
          pcols(v, col, 1.f, false, mrest);
          MPCQP_PHASE_K(4);
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            const bool act = st[r] == 1 || st[r] == 2;
            const float vs = bperm(v, slot[r] < 0 ? 0 : slot[r]);
            col[r] = act ? ((i < n) ? vs : -vs) : col[r];
          }
          const float mpp = pick<NR>(col, p);
          const bool dep = !(-mpp > dep_tol * scp);
          const float dtds = dep ? sidesign : sgn * epsp * fast_rcp(mpp);
          const float t2 = dep ? inf : fabsf(tgt - valp);
          float ti = inf;
          int k = 0;
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            const bool act = st[r] == 1 || st[r] == 2;
            const float dq = col[r] * dtds;
            const float dmu = act ? ((st[r] == 1) ? dq : -dq) : 0.f;
            float t = (act && dmu < 0.f) ? -mu[r] / dmu : inf;
            t = (t == t) ? t : inf;
            const bool take = t < ti;
            ti = take ? t : ti;
            k = take ? i : k;
          }
          wave_argmin(ti, k);
          k = uniform(k);
          ti = readlane(ti, 0);
          if (!(ti < inf) && !(t2 < inf)) {
            code = MPCQP_STATUS_INFEASIBLE;
            goto out;
          }
          const bool partial = ti < t2;
          const float s_eff = partial ? ti : t2;
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            const bool act = st[r] == 1 || st[r] == 2;
            const float dq = col[r] * dtds;
            const float dmu = act ? ((st[r] == 1) ? dq : -dq) : 0.f;
            const float dval = (st[r] == 0) ? ((i < n) ? -dq : dq) : 0.f;
            val[r] = fmaf(s_eff, dval, val[r]);
            mu[r] = fmaf(s_eff, dmu, mu[r]);
          }
          tau = fmaf(s_eff, dtds, tau);
          MPCQP_PHASE_K(5);
          if (partial) {
            // k leaves the active set
            if (!dep) valp = fmaf(sgn, s_eff, valp);
            const int q = uniform(pick<NR>(slot, k));
            s_row(q);
            const float d = sx[q];
            if (!(d > 0.f)) {
              code = MPCQP_STATUS_NOT_CONVEX;
              goto out;
            }
            s_drop(q, d);
            used &= ~(1ull << q);
            cmask &= ~(1ull << q);
            if (l == q) aidx = -1;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              const bool me = l + kWave * r == k;
              st[r] = me ? 0 : st[r];
              mu[r] = me ? 0.f : mu[r];
              slot[r] = me ? -1 : slot[r];
            }
          } else {
            // p joins the active set
            if (!(mpp < 0.f)) {
              code = MPCQP_STATUS_NOT_CONVEX;
              goto out;
            }
            if (~used == 0) {
              code = kStatusRetry;
              goto out;
            }
            const int snew = __builtin_ctzll(~used);
            s_add(v, snew, -mpp);
            used |= 1ull << snew;
            if (kCache && snew < ncache) {
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                const int i = l + kWave * r;
                if (i < nt) cache[snew * nt + i] = rawc[r];
              }
              cmask |= 1ull << snew;
            }
            if (l == snew) {
              aidx = p;
              sbnd = tgt;
              sisz = pz ? 1 : 0;
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              const bool me = l + kWave * r == p;
              st[r] = me ? side : st[r];
              mu[r] = me ? sidesign * tau : mu[r];
              val[r] = me ? tgt : val[r];
              slot[r] = me ? snew : slot[r];
            }
          }
          added = !partial;
          MPCQP_PHASE_K(6);
        }
      }
      MPCQP_PHASE_K(2);
      refresh();
      MPCQP_PHASE_K(1);
      {
        float viol;
        int p;
        scan(viol, p);
        active = viol > a.tol;
      }
    }
    if (active) code = MPCQP_STATUS_MAXITER;
    MPCQP_PHASE_K(2);

    // ------------------------------------------- iterative refinement
    const float* Hb = a.H + (int64_t)b * a.sH;
    const float* Gb = m ? a.G + (int64_t)b * a.sG : nullptr;
    // DYN: the horizon's stage data stays in LDS across refinement steps
    // when it fits one chunk
    int dyn_loaded = -1;
    cmask = 0;  // the residual below reuses the pool
    // correction sv = M w for a residual w on free z and active rows, in
    // product form: y2 = M0[:, free z] w, q = S^-1 (y2_P - w_P),
    // sv_i = y2_i + M0[i, P] q (i not in P), -q_i (i in P)
    auto correction = [&](const float (&w)[NR], float (&sv)[NR]) __attribute__((always_inline)) {
      float y2[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) y2[r] = 0.f;
      // (measured: skipping the fixed z rows pays in the DYN kernels, the
      // plain sweep over every z row is faster in the others)
      if constexpr (NXP > 0)
        zcols_free(w, y2);
      else
        zcols([&](int j) __attribute__((always_inline)) { return pick<NR>(w, j); }, y2);
      const float ys = gather(y2);
      const float wsl = gather(w);
      const float q = smul(aidx >= 0 ? ys - wsl : 0.f);
      pcols(q, y2, 1.f, false, used);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const bool act = st[r] == 1 || st[r] == 2;
        const float qi = bperm(q, slot[r] < 0 ? 0 : slot[r]);
        sv[r] = act ? -qi : y2[r];
      }
    };
    // the refinement variable: z on free z, the signed multiplier on active
    // rows (0 elsewhere; fixed z sit on their bound)
    auto refvar = [&](float (&x)[NR]) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int i = l + kWave * r;
        const bool isz = i < n;
        const bool act = st[r] == 1 || st[r] == 2;
        const float sside = ((st[r] == 1) ? 1.f : -1.f) * (isz ? 1.f : -1.f);
        x[r] = (st[r] == 3) ? 0.f : (isz ? val[r] : (act ? sside * mu[r] : 0.f));
      }
    };
    if constexpr (NXP == 0) {
      // K-pass: the residual from the fp32 condensed data (H, G), fp64
      // accumulation; converges to the fp32 data floor
      for (int it = 0; it < a.refine; ++it) {
        float x[NR], w[NR];
        refvar(x);
      // yk = K x in fp64, K = [[H, G'], [G, 0]]: row sweeps over packed H
      // and over G; the row-direction sums reduce 8 rows at a time in LDS
      double yk[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) yk[r] = 0.0;
      for (int r = l; r < NR * kWave; r += kWave) rsum[r] = 0.0;
      wave_lds_sync();
      // Rows of K stream through LDS in chunks of up to kKChunk floats:
      // packed H rows (row j = lanes i <= j, contiguous) then G rows (n each,
      // contiguous).  A chunk is a whole number of 8-row groups; its loads are
      // all issued before the first LDS store (one memory round trip per
      // chunk instead of one per 4 rows).  Per 8-row group the row-direction
      // sums reduce in LDS as before.
      auto kpass = [&](const float* base, int jb, int je, bool isH) __attribute__((always_inline)) {
        auto rstart = [&](int j) -> int64_t {
          return isH ? (int64_t)j * (j + 1) / 2 : (int64_t)(j - jb) * n;
        };
        for (int j0 = jb; j0 < je;) {
          const int64_t c0 = rstart(j0);
          int j1 = j0;
          while (j1 < je) {
            const int jn = j1 + 8 < je ? j1 + 8 : je;
            if (rstart(jn) - c0 > kKChunk) break;
            j1 = jn;
          }
          const int cnt = (int)(rstart(j1) - c0);
          {
            float tmp[kKChunk / kWave];
#pragma unroll
            for (int k = 0; k < kKChunk / kWave; ++k) {
              const int e = l + kWave * k;
              tmp[k] = e < cnt ? base[c0 + e] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < kKChunk / kWave; ++k) kbuf[l + kWave * k] = tmp[k];
          }
          wave_lds_sync();
          for (int g = j0; g < j1; g += 8) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const int j = g + t;
              const int lim = j < j1 ? (isH ? j : n - 1) : -1;
              const int ro = (int)(rstart(j < j1 ? j : j0) - c0);
              const double xj = j < j1 ? (double)xb[j] : 0.0;  // LDS broadcast
              double part = 0.0;
#pragma unroll
              for (int r = 0; r < NR; ++r) {
                const int i = l + kWave * r;
                const double hh = i <= lim ? kbuf[ro + i] : 0.f;
                // H row: the diagonal counts once (through yk); G row: all z
                part = (!isH || i < j) ? fma(hh, (double)x[r], part) : part;
                yk[r] = fma(hh, xj, yk[r]);
              }
              red[t * kWave + l] = part;
            }
            wave_lds_sync();
            {
              const int rr = l & 7, qq = l >> 3;
              double sm = 0.0;
#pragma unroll
              for (int t = 0; t < 8; ++t) sm += red[rr * kWave + qq * 8 + t];
              sm += lane_step<8>(sm);  // row_ror:8 = lane ^ 8 inside a 16-lane row
              sm += lane_step<16>(sm);
              sm += lane_step<32>(sm);
              if (qq == 0 && g + rr < j1) rsum[g + rr] += sm;
            }
            wave_lds_sync();
          }
          j0 = j1;
        }
      };
      // x_j of each row comes from an LDS broadcast (xb is free until the
      // gathers below)
#pragma unroll
      for (int r = 0; r < NR; ++r) xb[l + kWave * r] = x[r];
      wave_lds_sync();
      kpass(Hb, 0, n, true);
      if (m) kpass(Gb, n, nt, false);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int i = l + kWave * r;
        const bool isz = i < n;
        const bool act = st[r] == 1 || st[r] == 2;
        const double yi = yk[r] + rsum[i < NR * kWave ? i : 0];
        const double bnd = (st[r] == 1) ? (double)s_lo[i] : (double)s_hi[i];
        const bool inS = isz ? (st[r] == 0) : act;
        const double e = isz ? yi + (double)fz[r] : yi - bnd;
        w[r] = (inS && i < nt) ? (float)e : 0.f;
      }
        wave_lds_sync();
        float sv[NR];
        correction(w, sv);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int i = l + kWave * r;
          const bool isz = i < n;
          const bool act = st[r] == 1 || st[r] == 2;
          const float sside = ((st[r] == 1) ? 1.f : -1.f) * (isz ? 1.f : -1.f);
          val[r] = (isz && st[r] == 0) ? val[r] + sv[r] : val[r];
          val[r] = (!isz && st[r] == 0) ? val[r] - sv[r] : val[r];  // row values G z
          mu[r] = (!isz && act) ? mu[r] + sside * sv[r] : mu[r];
        }
      }
      break;
    } else {
      if (a.refine <= 0) break;  // (A/B knob: no refinement, no certificate)
      // DYN: refine from the exact (fp64) residual of the dynamics.  The
      // refinement variable is carried as a float pair (val or mu, and its
      // low part ext), so the fixed point is the fp64 solution on this
      // active set, not its fp32 rounding.
      //
      // Certificate of a refined point (at the residual just computed):
      //   primal: every inactive state row from the fp64 rollout X, every
      //           free z, within kDynTol (relative, the scan's scales);
      //   dual:   the exact Lagrangian gradient g of every fixed z has the
      //           bound's sign, every active row multiplier is >= 0, both
      //           within kDualTol.
      // It is decided as soon as it is unambiguous: after a contracting
      // correction (the residual fell 1000x), every checked quantity whose
      // margin to its threshold exceeds the point's error -- taken as 10x the
      // residual norm r (the residual is the error of the point as seen
      // through the KKT matrix) -- decides the same way at the exact
      // solution, so one correction usually suffices.  Otherwise the point
      // is refined until a correction is below dyn_stop, and the
      // certificate is decided on that converged point.  A refinement that
      // neither contracts nor converges within a.refine corrections hands
      // the instance to the fp64 fallback.
      float* ext = reinterpret_cast<float*>(pool + kPool);  // low parts, in LDS
#pragma unroll
      for (int r = 0; r < NR; ++r) ext[l + kWave * r] = 0.f;
      const double* gx = pool + kDynXd;
      const double* Xr = pool + kDynX + a.d.nx;  // x_1..x_N, stage-major = row order
      const float* xlo = a.d.xlo ? a.d.xlo + (int64_t)b * a.d.sXb : nullptr;
      const float* xhi = a.d.xhi ? a.d.xhi + (int64_t)b * a.d.sXb : nullptr;
      bool decided = false;
      float prev = inf, r_prev = inf;
      float pv = -inf, dv = -inf;
      int dk = 0;
      for (int it = 0;; ++it) {
        MPCQP_PHASE_D(0);
        float x[NR], w[NR];
        refvar(x);
        dyn_residual<NR, NXP>(a.d, b, n, m, l, x, ext, st, pool, dyn_loaded, w MPCQP_CLK_ARG);
        MPCQP_PHASE_K(0);  // phase timing: the residual is charged with the setup
        float rn = 0.f;
#pragma unroll
        for (int r = 0; r < NR; ++r) rn = fmaxf(rn, fabsf(w[r]));
        rn = wave_max(rn);
        if (it > 0) {
          // the certificate at this point, with margins tau = 10 r
          const float tau = 10.f * rn;
          float pvm = -inf, dvm = -inf;
          pv = -inf;
          dv = -inf;
          dk = 0;
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = l + kWave * r;
            float p = -inf, dd = -inf, pm = -inf, dm = -inf;
            if (i < n) {
              if (st[r] == 0) {
                const float vl = (s_lo[i] - val[r]) * s_sl[i], vu = (val[r] - s_hi[i]) * s_su[i];
                p = fmaxf(vl, vu);
                pm = fmaxf(vl + tau * s_sl[i], vu + tau * s_su[i]);
              } else {
                const float g = (float)gx[i];
                const float wg = (st[r] == 1) ? -g : g;  // > 0: wrong sign
                dd = wg - kDualTol * (1.f + fabsf(fz[r]));
                dm = wg + tau;
              }
            } else if (i < nt) {
              const int j = i - n;
              if (st[r] == 0) {
                const double xv = Xr[j];
                const bool hl = xlo && finite(s_lo[i]);
                const bool hh = xhi && finite(s_hi[i]);
                const float el = hl ? (float)((double)xlo[j] - xv) : -inf;  // > 0: below xlo
                const float eh = hh ? (float)(xv - (double)xhi[j]) : -inf;  // > 0: above xhi
                p = fmaxf(el * (hl ? s_sl[i] : 0.f), eh * (hh ? s_su[i] : 0.f));
                pm = fmaxf((el + tau) * (hl ? s_sl[i] : 0.f), (eh + tau) * (hh ? s_su[i] : 0.f));
                // the exact row value on the condensed rows' scale
                val[r] = hl ? s_lo[i] - el : (hh ? s_hi[i] + eh : val[r]);
              } else if (st[r] == 1 || st[r] == 2) {
                dd = -mu[r] - kDualTol;
                dm = -mu[r] + tau;
              }
            }
            pv = fmaxf(pv, p == p ? p : -inf);
            pvm = fmaxf(pvm, pm == pm ? pm : -inf);
            dvm = fmaxf(dvm, dm);
            const bool take = dd > dv;
            dv = take ? dd : dv;
            dk = take ? i : dk;
          }
          pv = wave_max(pv);
          pvm = wave_max(pvm);
          dvm = wave_max(dvm);
          wave_argmax(dv, dk);
          dk = uniform(dk);
          dv = readlane(dv, 0);
          // unambiguous: all clear by the margin, or a violation beyond it
          const bool clear = !(pvm > kDynTol) && !(dvm > 0.f);
          const bool fails = pv > kDynTol + tau || dv > tau;
          const bool contracting = !(rn > 1e-3f * r_prev);
          const bool converged = !(prev > a.dyn_stop);
          if ((contracting && (clear || fails)) || converged) {
            decided = true;
            break;
          }
        }
        if (it >= a.refine) break;
        float sv[NR];
        correction(w, sv);
        float dmax = 0.f;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int i = l + kWave * r;
          const bool isz = i < n;
          const bool act = st[r] == 1 || st[r] == 2;
          const bool ref = isz ? st[r] == 0 : act;
          const float sside = ((st[r] == 1) ? 1.f : -1.f) * (isz ? 1.f : -1.f);
          // x + ext + sv in fp64, split back into the float pair
          const double xf = (double)x[r] + (double)ext[i] + (double)sv[r];
          const float xh = (float)xf;
          ext[i] = ref ? (float)(xf - (double)xh) : 0.f;
          val[r] = (isz && st[r] == 0) ? xh : val[r];
          val[r] = (!isz && st[r] == 0) ? val[r] - sv[r] : val[r];  // row values G z (re-set above)
          mu[r] = (!isz && act) ? sside * xh : mu[r];
          dmax = ref ? fmaxf(dmax, fabsf(sv[r]) / (1.f + fabsf(xh))) : dmax;
        }
        prev = wave_max(dmax);
        r_prev = rn;
#ifdef MPCQP_PF_DEBUG
        if (l == 0)
          printf("pf b=%d round=%d it=%d |r|=%.3e dmax=%.3e nP=%d\n", b, round, it, rn, prev,
                 __builtin_popcountll(used));
#endif
        MPCQP_PHASE_D(5);
      }
      MPCQP_PHASE_D(6);
#ifdef MPCQP_PF_DEBUG
      if (l == 0)
        printf("pf b=%d round=%d cert decided=%d pv=%.3e dv=%.3e (at %d) code=%d\n", b, round,
               (int)decided, pv, dv, dk, code);
#endif
      const bool conv = decided;
      if (code != MPCQP_STATUS_OPTIMAL) break;
      if (conv && !(pv > kDynTol) && !(dv > 0.f)) break;  // certified optimal
      // not certified: a refinement that does not contract, or no round
      // left, hands the instance to the fp64 fallback (never OPTIMAL)
      if (!conv || round + 1 >= kDynRounds) {
        code = kStatusRetry;
        break;
      }
      if (dv > 0.f) {
        // release the worst wrong-signed constraint (a Schur drop, as a
        // partial step does); the next round refines first and certifies
        // again (re-scanning fp32 values would re-add it: the fp32 floor)
        const int q = uniform(pick<NR>(slot, dk));
        s_row(q);
        const float d = sx[q];
        if (!(d > 0.f)) {
          code = kStatusRetry;
          break;
        }
        s_drop(q, d);
        used &= ~(1ull << q);
        if (l == q) aidx = -1;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const bool me = l + kWave * r == dk;
          st[r] = me ? 0 : st[r];
          mu[r] = me ? 0.f : mu[r];
          slot[r] = me ? -1 : slot[r];
        }
        wave_lds_sync();
        refresh();
        gi_skip = true;
      }
      // else: a primal violation; the next round's active set adds it from
      // the exact values (first scan with the tight tolerance)
    }
    }
  }
  // a non-finite value in the final state (never expected; the scan skips
  // NaN violations, so it would otherwise pass as optimal): hand the
  // instance to the workgroup kernel, which solves it from scratch
  if (code == MPCQP_STATUS_OPTIMAL || code == MPCQP_STATUS_MAXITER) {
    bool nf = false;
#pragma unroll
    for (int r = 0; r < NR; ++r) nf |= (l + kWave * r < nt) && !(finite(val[r]) && finite(mu[r]));
    if (__builtin_amdgcn_ballot_w64(nf)) code = kStatusRetry;
  }
out:
  MPCQP_PHASE_K(7);
  MPCQP_PHASE_D(7);
  {
    const bool ok = code == MPCQP_STATUS_OPTIMAL || code == MPCQP_STATUS_MAXITER;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int i = l + kWave * r;
      const bool isz = i < n;
      const float sside = ((st[r] == 1) ? 1.f : -1.f) * (isz ? 1.f : -1.f);
      const float lam = (st[r] == 1 || st[r] == 2) ? sside * mu[r] : 0.f;
      if (code == kStatusRetry) continue;
      if (isz) a.z[(int64_t)b * n + i] = ok ? fminf(fmaxf(val[r], s_lo[i]), s_hi[i]) : __builtin_nanf("");
      else if (a.y && i < nt) a.y[(int64_t)b * m + (i - n)] = ok ? lam : __builtin_nanf("");
    }
    if (l == 0) {
      a.status[b] = (code & 0xff) | ((iters & 0xffff) << 8);
      if (code == kStatusRetry) a.retry_list[atomicAdd(a.retry_count, 1)] = b;
    }
  }
#ifdef MPCQP_PHASE_TIMING
  mpcqp_clk.flush();
#endif
}

int launch_pf(int batch, int n, int m, const float* H, int64_t sH, const float* f, int64_t sf,
              const float* G, int64_t sG, const float* hl, const float* hu, int64_t sh,
              const float* lb, int64_t sLb, const float* ub, int64_t sUb, const float* M0,
              const float* s0, float* z, float* y, int32_t* status, int* retry_count,
              int* retry_list, int max_iter, int refine, float tol, hipStream_t st,
              const PfDyn* dyn) {
  PfArgs a{batch, n, m, H, sH, f, sf, G, sG, hl, hu, sh, lb, sLb, ub, sUb, M0, s0, z, y, status,
           retry_count, retry_list, max_iter, refine, tol, PfDyn{}, kDynStop};
  if (dyn) a.d = *dyn;
  if (const char* e = getenv("MPCQP_DYN_STOP")) a.dyn_stop = (float)atof(e);
  const bool two = n + m <= 2 * kWave;
  const int nxp = dyn ? dyn_nxp(dyn->nx, dyn->nu) : 0;
#define MPCQP_PF(NRV, NXPV) \
  hipLaunchKernelGGL((qp_pf_kernel<NRV, NXPV>), dim3(batch), dim3(kWave), 0, st, a)
  switch (nxp) {
    case 4: if (two) MPCQP_PF(2, 4); else MPCQP_PF(3, 4); break;
    case 8: if (two) MPCQP_PF(2, 8); else MPCQP_PF(3, 8); break;
    case 12: if (two) MPCQP_PF(2, 12); else MPCQP_PF(3, 12); break;
    case 16: if (two) MPCQP_PF(2, 16); else MPCQP_PF(3, 16); break;
    default: if (two) MPCQP_PF(2, 0); else MPCQP_PF(3, 0); break;
  }
#undef MPCQP_PF
  MPCQP_CHECK_LAUNCH("qp_pf_kernel");
  return MPCQP_OK;
}

}  // namespace mpcqp

#ifdef MPCQP_PHASE_TIMING
MPCQP_DEBUG_PHASE_READER(mpcqp_debug_phase_cycles_pf)
#endif
