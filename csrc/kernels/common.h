// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Everything here is written for wave64 and the gfx950 MFMA/LDS instruction set;
// there is no portability layer.  bf16 tensors are carried as raw uint16 bits and
// moved in 16-byte vectors (8 x bf16) — scalar bf16 traffic is ~2x slower on CDNA
// (cdna_hip_programming.md, Guideline 13).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace rfq {

constexpr int kWave = 64;

typedef uint16_t bf16_t;                                            // raw bf16 bits
typedef short s16x8 __attribute__((ext_vector_type(8)));            // 8 x bf16 bits (16 B)
typedef short s16x4 __attribute__((ext_vector_type(4)));            // 4 x bf16 bits (8 B)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));          // MFMA operand
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t x) {
  return __uint_as_float(((uint32_t)x) << 16);
}
__device__ __forceinline__ float bf2f_s(short x) { return bf2f((bf16_t)x); }

// Round-to-nearest-even f32 -> bf16 (lowers to v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  // fptrunc <2 x float> -> <2 x bfloat>: a single v_cvt_pk_bf16_f32 (RNE)
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}

__device__ __forceinline__ void unpack8(const s16x8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f_s(v[i]);
}

__device__ __forceinline__ s16x8 pack8(const float* f) {
  u32x4 w;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return __builtin_bit_cast(s16x8, w);
}

__device__ __forceinline__ bf16x8 as_bf16x8(const s16x8& v) {
  return __builtin_bit_cast(bf16x8, v);
}

// Wave64 reductions via cross-lane shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64).  `scratch` >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = (lane < nw) ? scratch[lane] : 0.f;
  t = wave_sum(t);
  __syncthreads();
  return t;
}

// Fast exp2 (v_exp_f32).
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Transposed LDS read: per 16-lane group, 4 rows x 16 cols of 16-bit data, lane i
// receives column i (row q in element q).  Lane 4q+p supplies &tile[row q][col 4p].
__device__ __forceinline__ s16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_ptr));
}

typedef __attribute__((address_space(3))) void lds_void_t;

// 16-byte global -> LDS DMA (global_load_lds_dwordx4): no VGPR round trip.  The LDS
// destination is lane-linear: wave-uniform base + lane * 16 B, so any swizzle of
// the LDS image is applied to the per-lane *source* address.  Completion is
// tracked by vmcnt like any other vector load.
__device__ __forceinline__ void glds16(const bf16_t* g, bf16_t* l) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
#endif
}

// Error words of the bounded in-launch waits (kerr.hip): slot kErrStreamK counts stream-K
// slab waits that gave up, kErrPersist the persistent decode layer's stage waits,
// kErrPersistInfo keeps the first failing (layer, stage) of the latter.
enum { kErrStreamK = 0, kErrPersist = 1, kErrPersistInfo = 2, kKernelErrorWords = 16 };
uint32_t* kernel_error_words(hipStream_t s);
uint32_t kernel_error_read(int slot);

// Bounded waits are timed on the 100 MHz s_memrealtime clock: 1 s.
constexpr uint64_t kSpinTicks = 100000000ull;

__device__ __forceinline__ void report_error(uint32_t* words, int slot) {
  if (words != nullptr)
    __hip_atomic_fetch_add(words + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// MoE grouped GEMM enumeration (gemm_w4.hip GROUPED): 256-row chunks over the experts'
// 128-row-padded segments.
__device__ __forceinline__ int moe_live_chunks(const int32_t* offs, int E) {
  int n = 0;
  for (int e = 0; e < E; ++e) n += ((offs[e + 1] - offs[e]) / 128 + 1) >> 1;
  return n;
}

// Split-K rule of the grouped w2 (gemm_w4.hip KS = 2, moe.hip moe_combine_w2_kernel):
// two K slices when `tiles` 256x256 tiles leave the last round on `cus` CUs at most half
// full within the first three rounds (measured: profiles/r6_mixtral_window.md).  Both
// kernels evaluate it on the same offsets, so the combine reads what the GEMM wrote.
__device__ __forceinline__ int moe_w2_ksplit(int tiles, int cus) {
  if (cus <= 0) return 1;
  const int full = tiles / cus, part = tiles - full * cus;
  return (part > 0 && 2 * part <= cus && full <= 2) ? 2 : 1;
}

// Counter-based RNG (splitmix/murmur style finaliser) — deterministic per
// (seed, row, column), identical on every TP rank for the same global column.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint32_t a, uint32_t b) {
  uint64_t x = seed ^ (((uint64_t)a << 32) | b);
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

}  // namespace rfq
