// Custom all-reduce core of the all-reduce kernels (custom_ar.hip): the signal region
// layout, the bounded flag protocol and the push form's fixed slots and per-row sum +
// residual-add RMSNorm.
#pragma once
#include <hip/hip_runtime.h>

#include "../kernels/common.h"

namespace rfq {

constexpr int kCarMaxRanks = 8;
constexpr int kCarMaxBlocks = 64;
constexpr int kCarThreads = 512;

struct CarSignal {
  uint32_t start[kCarMaxBlocks][kCarMaxRanks];
  uint32_t mid[kCarMaxBlocks][kCarMaxRanks];     // two-shot: reduced slices published
  uint32_t end[kCarMaxBlocks][kCarMaxRanks];
  uint32_t push[2][kCarMaxBlocks][kCarMaxRanks]; // push one-shot: row published, by parity
  uint32_t counter[kCarMaxBlocks];
  uint32_t error;
  uint32_t info;             // first timeout: 0x80000000 | phase << 24 | block << 8 | peer
  uint32_t pad[62];
};

constexpr int64_t kCarDataOffset = (sizeof(CarSignal) + 4095) / 4096 * 4096;

struct CarPeers {
  char* base[kCarMaxRanks];  // region base of every rank (own included)
};

__device__ __forceinline__ void car_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Spins are bounded in wall time (the 100 MHz s_memrealtime clock), not in
// iterations: a peer whose queue the hardware scheduler has not mapped yet (more GPU
// processes than concurrent process slots, e.g. 8 ranks + a launcher sharing one
// device) is waited for the same 2 s however slow each poll is.  A timeout records
// the first failing (phase, block, peer) in `info` for the host's diagnostics.
constexpr uint64_t kCarSpinTicks = 200000000ull;           // 2 s at 100 MHz
enum : uint32_t { kCarStart = 1, kCarMid = 2, kCarEnd = 3, kCarPush = 4 };

// A region whose error counter is set (a peer went silent before) fails every wait at
// once: after the first timeout a lost peer costs no further 2 s spins -- the runner
// sees the error behind that step and the replica restarts on RCCL (router.py).
__device__ __forceinline__ bool car_wait(CarSignal* self, uint32_t* p, uint32_t v,
                                         uint32_t phase, int b, int peer) {
  if (__hip_atomic_load(&self->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
    return false;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == v) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > kCarSpinTicks) {
      atomicCAS(&self->info, 0u, 0x80000000u | (phase << 24) | ((uint32_t)b << 8) | (uint32_t)peer);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

constexpr int kCarPushRows = 16;      // decode rows of the push form
constexpr int kCarPushD = 8192;       // max row width of the push form (bf16)

// slot (parity par, source rank src, row b) of the push form in the region at `base`:
// a fixed home whatever the call's shape, so a call of another shape on a faster rank
// never writes into slots a slower rank is still reading (parity alternates per row)
__device__ __forceinline__ s16x8* car_push_slot(char* base, int par, int src, int b) {
  return reinterpret_cast<s16x8*>(base + kCarDataOffset) +
         (((int64_t)par * kCarMaxRanks + src) * kCarPushRows + b) * (kCarPushD / 8);
}

// The residual and norm-weight chunks a thread of car_push_sum_norm_row owns, loaded
// before the flag wait so their latency overlaps it.
template <int NCH>
__device__ __forceinline__ void car_push_preload(int b, const bf16_t* residual,
                                                 int64_t res_stride, const bf16_t* w, int d,
                                                 s16x8 (&rv)[NCH], s16x8 (&wv)[NCH]) {
  const int tid = threadIdx.x, nchunk = d >> 3;
  const s16x8* rr = reinterpret_cast<const s16x8*>(residual + b * res_stride);
  const s16x8* wr = reinterpret_cast<const s16x8*>(w);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + k * 256;
    if (tid < 256 && ch < nchunk) {
      rv[k] = rr[ch];
      wv[k] = wr[ch];
    }
  }
}

// Row b's all-reduce result from the world rows in this rank's own staging (rank order,
// fp32, rounded to bf16 = the all-reduce output), residual <- bf16(sum + residual),
// out <- rmsnorm(residual) * w (rv / wv: car_push_preload).  Threads [0, 256) own chunks
// tid + 256 k (k < NCH); any further threads of the block only join block_sum with 0
// (the same float sum order).
template <int NCH>
__device__ __forceinline__ void car_push_sum_norm_row(
    char* self_base, int par, int world, int b, bf16_t* __restrict__ residual,
    int64_t res_stride, const s16x8 (&rv)[NCH], const s16x8 (&wv)[NCH], bf16_t* out,
    int64_t out_stride, int d, float eps, float* scratch) {
  const int tid = threadIdx.x;
  const int nchunk = d >> 3;
  s16x8* rr = reinterpret_cast<s16x8*>(residual + b * res_stride);
  float v[NCH][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + k * 256;
    if (tid < 256 && ch < nchunk) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < world; ++p) {
        const s16x8 pv = car_push_slot(self_base, par, p, b)[ch];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f_s(pv[j]);
      }
      float a[8], r[8];
      unpack8(pack8(acc), a);
      unpack8(rv[k], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += r[j];
      const s16x8 packed = pack8(a);
      rr[ch] = packed;
      unpack8(packed, v[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float rs = rsqrtf(ss / (float)d + eps);
  s16x8* orow = reinterpret_cast<s16x8*>(out + b * out_stride);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + k * 256;
    if (tid < 256 && ch < nchunk) {
      float wf[8], o[8];
      unpack8(wv[k], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * rs * wf[j];
      orow[ch] = pack8(o);
    }
  }
}

}  // namespace rfq
