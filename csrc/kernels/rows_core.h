// Wave-level helpers of the row-streaming GEMVs (gemv_rows.hip, decode_persist.hip): a
// DPP wave sum and the v_dot2c_f32_bf16 dot products over 16-byte chunks.
#pragma once
#include "common.h"

namespace rfq {

// one DPP move (row_mask / bank_mask all, bound_ctrl off)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL,
                                                            0xf, 0xf, false));
}

// full 64-lane sum, result in every lane: xor 1 / xor 2 (quad_perm), 8-lane and 16-lane
// mirrors (each lane then holds its 16-lane row's sum), then two cross-row swizzles
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);    // row_half_mirror
  v += dpp_f<0x140>(v);    // row_mirror
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// x . w over 8 bf16 pairs.  Each dword is copied to a scalar before the bit_cast:
// hipcc (ROCm 7.2) lowers __builtin_bit_cast of a vector-element lvalue (w.y, w[i]) as a
// read of the vector's FIRST element, so bit-casting elements in place silently computes
// x0 . w0 four times.
__device__ __forceinline__ float dot2(uint32_t w, uint32_t x, float acc) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, w),
                                         __builtin_bit_cast(bf16x2, x), acc, false);
}
__device__ __forceinline__ float dot8(const u32x4& w, const u32x4& x, float acc) {
  const uint32_t w0 = w.x, w1 = w.y, w2 = w.z, w3 = w.w;
  const uint32_t x0 = x.x, x1 = x.y, x2 = x.z, x3 = x.w;
  acc = dot2(w0, x0, acc);
  acc = dot2(w1, x1, acc);
  acc = dot2(w2, x2, acc);
  acc = dot2(w3, x3, acc);
  return acc;
}

}  // namespace rfq
