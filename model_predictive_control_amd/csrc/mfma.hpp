// mfma.hpp -- gfx950 MFMA tile helpers shared by the MFMA kernels
// (condense.hip, sweep.hip).
//
// A 16 x 16 fp32 tile in "C layout" (the v_mfma_f32_16x16x4f32 accumulator
// layout) is 4 registers per lane: lane (g, c) = (l / 16, l % 16) holds rows
// 4g..4g+3 of column c.  mfma4(P, Y, acc) runs four 16x16x4 MFMAs with the
// K index of chunk s in lane group g taken as k = 4g + s, so with P and Y
// both in C layout it returns acc + P' Y -- no transposes are needed for
// products of the form P' Y.
#pragma once
#include "common.hpp"

namespace mpcqp {

typedef float mf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void xpose4(float (&v)[4]) {
  // lane group g, register r  ->  lane group r, register g
  auto s0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[0]), __float_as_uint(v[2]), false, false);
  auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[1]), __float_as_uint(v[3]), false, false);
  auto t0 = __builtin_amdgcn_permlane16_swap(s0[0], s1[0], false, false);
  auto t1 = __builtin_amdgcn_permlane16_swap(s0[1], s1[1], false, false);
  v[0] = __uint_as_float(t0[0]);
  v[1] = __uint_as_float(t0[1]);
  v[2] = __uint_as_float(t1[0]);
  v[3] = __uint_as_float(t1[1]);
}

__device__ __forceinline__ mf4 mfma4(const float (&a)[4], const float (&b)[4], mf4 acc) {
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
  return acc;
}

// Buffer descriptors (raw, stride 0, range-checked): every per-lane memory
// access is base (SGPR) + 32-bit byte offset, and a masked-out lane uses an
// offset past num_records -- its load returns 0 and its store is dropped, so
// the loads and stores carry no exec-mask branches and no selects.
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kOOB = 0x7ffffff0;
__device__ __forceinline__ rsrc_t mk_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld(rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void bst(float v, rsrc_t r, int off) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
// per-lane byte offset + a wave-uniform one (the instruction's SGPR soffset:
// a compile-time or uniform displacement costs no VALU address arithmetic)
__device__ __forceinline__ void bst(float v, rsrc_t r, int off, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, soff, 0);
}

}  // namespace mpcqp
