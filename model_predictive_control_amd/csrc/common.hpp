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
// Arg-max over the wave: returns the largest value; ties resolve to the
// smallest lane index.  Lanes that should not compete pass -inf.
template <typename T>
__device__ __forceinline__ void wave_argmax(T& v, int& idx) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const T ov = __shfl_xor(v, off, kWave);
    const int oi = __shfl_xor(idx, off, kWave);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
}

template <typename T>
__device__ __forceinline__ void wave_argmin(T& v, int& idx) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const T ov = __shfl_xor(v, off, kWave);
    const int oi = __shfl_xor(idx, off, kWave);
    const bool take = (ov < v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
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

inline size_t dtype_size(int dtype) { return dtype == MPCQP_F64 ? 8 : 4; }

}  // namespace mpcqp
