// common.hpp -- shared device helpers for libmpcqp (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <limits>

#include "../../include/mpcqp.h"

namespace mpcqp {

// Optional phase timing (tools/phase_timing.py builds a separate library
// with -DMPCQP_PHASE_TIMING): every wave accumulates the s_memtime cycles of
// each phase in registers and lane 0 adds them to this translation unit's
// mpcqp_phase_cycles[] once, at the end of the kernel; each instrumented
// unit exports its own mpcqp_debug_phase_cycles_* reader.
#ifdef MPCQP_PHASE_TIMING
static __device__ unsigned long long mpcqp_phase_cycles[8];  // one copy per translation unit
struct PhaseClock {
  unsigned long long t, acc[8];
  __device__ PhaseClock() : t(__builtin_readcyclecounter()) {
    for (int i = 0; i < 8; ++i) acc[i] = 0;
  }
  __device__ __forceinline__ void mark(int i) {
    const unsigned long long n = __builtin_readcyclecounter();
    acc[i] += n - t;
    t = n;
  }
  __device__ __forceinline__ void flush() {
    if (threadIdx.x % 64 == 0)
      for (int i = 0; i < 8; ++i) atomicAdd(&mpcqp_phase_cycles[i], acc[i]);
  }
};
#define MPCQP_PHASE(i) mpcqp_clk.mark(i)
#define MPCQP_DEBUG_PHASE_READER(NAME)                                                        \
  extern "C" int NAME(unsigned long long* out, int reset) {                                   \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcqp::mpcqp_phase_cycles),                       \
                            8 * sizeof(unsigned long long)) != hipSuccess)                    \
      return -2;                                                                              \
    if (reset) {                                                                              \
      unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                     \
      if (hipMemcpyToSymbol(HIP_SYMBOL(mpcqp::mpcqp_phase_cycles), z, sizeof(z)) != hipSuccess) \
        return -2;                                                                            \
    }                                                                                         \
    return 0;                                                                                 \
  }
#define MPCQP_CLK_PARAM , PhaseClock& mpcqp_clk
#define MPCQP_CLK_ARG , mpcqp_clk
#else
#define MPCQP_CLK_PARAM
#define MPCQP_CLK_ARG
#define MPCQP_PHASE(i) \
  do {                 \
  } while (0)
#endif


constexpr int kWave = 64;  // CDNA wavefront width (hard-coded, never warpSize)

// DPP moves: old value 0 with bound_ctrl set.  A lane whose source is out of
// range (or disabled) gets 0 either way, but with bound_ctrl clear the
// compiler must first materialise the old value 0 in the destination -- one
// v_mov per DPP move (60 of the 462 instructions of the SQP kernel's serial
// Riccati step).  -DMPCQP_DPP_BC=false restores the old encoding (A/B builds).
#ifndef MPCQP_DPP_BC
#define MPCQP_DPP_BC true
#endif

// LDS exchange inside the single-wave workgroup: a wave's LDS operations
// execute in issue order, so only the compiler must not move them (no
// s_barrier, and no fence that would drain the outstanding global loads)
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Gamma as its lower block triangle (MPCQP_GAM_PACKED): block row k (the
// state x_{k+1}, nx rows) keeps its (k+1) nu leading columns, column by
// column, from element nx nu k (k+1) / 2 -- entry (k nx + q, col) at
// gam_packed_off(k) + col nx + q, so the nx entries one lane of the
// condensing sweep holds for its column are one contiguous vector
__host__ __device__ __forceinline__ int gam_packed_off(int nx, int nu, int k) {
  return nx * nu * (k * (k + 1) / 2);
}
__host__ __device__ __forceinline__ int64_t gam_packed_size(int nx, int nu, int N) {
  return (int64_t)nx * nu * ((int64_t)N * (N + 1) / 2);
}

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* where);

#define MPCQP_CHECK_ARG(cond, ...)          \
  do {                                      \
    if (!(cond)) {                          \
      ::mpcqp::set_error(__VA_ARGS__);      \
      return MPCQP_EINVAL;                  \
    }                                       \
  } while (0)

#define MPCQP_CHECK_LAUNCH(where)                                  \
  do {                                                             \
    hipError_t _e = hipGetLastError();                             \
    if (_e != hipSuccess) return ::mpcqp::hip_fail(_e, where);     \
  } while (0)

// ------------------------------------------------ wave-uniform broadcasts
// v_readlane with an SGPR (wave-uniform) lane index: a scalar broadcast of one
// lane's value, no LDS traffic.  fp64 travels as two 32-bit halves.
__device__ __forceinline__ float readlane(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ double readlane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int readlane(int v, int lane) {
  return __builtin_amdgcn_readlane(v, lane);
}

// Make a value provably wave-uniform for the compiler (lives in an SGPR).
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------ wave reductions
// Cross-lane steps without LDS: quad_perm DPP (lane ^ 1, ^ 2), row_ror:4 and
// row_ror:8 DPP (within a 16-lane row: after the quad steps every quad holds
// its best, so rotating by 4 then 8 combines all four quads), and
// v_permlane16_swap / v_permlane32_swap (lane ^ 16, ^ 32).  Every step is a
// VALU op (ds_bpermute, what __shfl_xor compiles to, is an LDS round trip per
// step); the result of a commutative reduction is the same in every lane.
__device__ __forceinline__ unsigned lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
template <int X>
__device__ __forceinline__ int lane_step(int v) {
  if constexpr (X == 1) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, MPCQP_DPP_BC);
  } else if constexpr (X == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, MPCQP_DPP_BC);
  } else if constexpr (X == 4) {
    return __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, MPCQP_DPP_BC);
  } else if constexpr (X == 8) {
    return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, MPCQP_DPP_BC);
  } else if constexpr (X == 16) {
    const auto s = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((lane_id() & 16) ? s[0] : s[1]);
  } else {
    static_assert(X == 32, "lane_step: 1, 2, 4, 8, 16 or 32");
    const auto s = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)((lane_id() & 32) ? s[0] : s[1]);
  }
}
template <int X>
__device__ __forceinline__ float lane_step(float v) {
  return __int_as_float(lane_step<X>(__float_as_int(v)));
}
template <int X>
__device__ __forceinline__ double lane_step(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = lane_step<X>((int)(b & 0xffffffffll));
  const int hi = lane_step<X>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Arg-max over the wave: returns the largest value; ties resolve to the
// smallest lane index.  Lanes that should not compete pass -inf.
template <int X, typename T>
__device__ __forceinline__ void argmax_step(T& v, int& idx) {
  const T ov = lane_step<X>(v);
  const int oi = lane_step<X>(idx);
  const bool take = (ov > v) || (ov == v && oi < idx);
  v = take ? ov : v;
  idx = take ? oi : idx;
}
template <int X, typename T>
__device__ __forceinline__ void argmin_step(T& v, int& idx) {
  const T ov = lane_step<X>(v);
  const int oi = lane_step<X>(idx);
  const bool take = (ov < v) || (ov == v && oi < idx);
  v = take ? ov : v;
  idx = take ? oi : idx;
}
template <typename T>
__device__ __forceinline__ void wave_argmax(T& v, int& idx) {
  argmax_step<1>(v, idx);
  argmax_step<2>(v, idx);
  argmax_step<4>(v, idx);
  argmax_step<8>(v, idx);
  argmax_step<16>(v, idx);
  argmax_step<32>(v, idx);
}

template <typename T>
__device__ __forceinline__ void wave_argmin(T& v, int& idx) {
  argmin_step<1>(v, idx);
  argmin_step<2>(v, idx);
  argmin_step<4>(v, idx);
  argmin_step<8>(v, idx);
  argmin_step<16>(v, idx);
  argmin_step<32>(v, idx);
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
  v = fmax(v, lane_step<1>(v));
  v = fmax(v, lane_step<2>(v));
  v = fmax(v, lane_step<4>(v));
  v = fmax(v, lane_step<8>(v));
  v = fmax(v, lane_step<16>(v));
  v = fmax(v, lane_step<32>(v));
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
  v = fmin(v, lane_step<1>(v));
  v = fmin(v, lane_step<2>(v));
  v = fmin(v, lane_step<4>(v));
  v = fmin(v, lane_step<8>(v));
  v = fmin(v, lane_step<16>(v));
  v = fmin(v, lane_step<32>(v));
  return v;
}

template <typename T>
struct Lim {
  static __device__ __forceinline__ T inf() { return __builtin_huge_val(); }
};
template <>
struct Lim<float> {
  static __device__ __forceinline__ float inf() { return __builtin_huge_valf(); }
};

// Reciprocal from the hardware estimate plus Newton steps (~1 ulp), instead of
// the ~12-instruction IEEE division sequence on the serial pivot chain.
__device__ __forceinline__ double fast_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ float fast_rcp(float d) {
  float r = __builtin_amdgcn_rcpf(d);
  return fmaf(r, fmaf(-d, r, 1.0f), r);
}

template <typename T>
__device__ __forceinline__ bool finite(T v) {
  return __builtin_isfinite(v);
}

// LDS exchange inside a single-wave workgroup (every kernel on the Sym2D /
// QSym register layouts launches 64 threads): a wave's LDS operations execute
// in issue order, so only the compiler must be kept from moving them across
// the exchange -- no s_barrier and no fence
__device__ __forceinline__ void lds_exchange() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

inline size_t dtype_size(int dtype) { return dtype == MPCQP_F64 ? 8 : 4; }

}  // namespace mpcqp
