// SwiGLU activation (silu(gate) * up) and the token-embedding row gather.
//
// SURVEY.md §2.4 K10 / K1.  Both are pure streaming ops: 16-byte vector loads,
// grid-stride loops capped near 8 blocks/CU (Guideline 11).
#include "common.h"

namespace rfq {

// gate_up: [rows, 2F] (gate | up), out: [rows, F]
__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16_t* __restrict__ gate_up,
                                                       int64_t in_stride,
                                                       bf16_t* __restrict__ out,
                                                       int64_t out_stride, int rows, int F) {
  const int cpr = F >> 3;  // chunks per row
  const int64_t total = (int64_t)rows * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr);
    const s16x8 g = reinterpret_cast<const s16x8*>(gate_up + r * in_stride)[c];
    const s16x8 u = reinterpret_cast<const s16x8*>(gate_up + r * in_stride + F)[c];
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gf = bf2f_s(g[k]);
      // silu in f32 then round once; matches torch's bf16 silu(g) * u within 1 ulp
      const float sg = gf / (1.f + __expf(-gf));
      o[k] = bf2f(f2bf(sg)) * bf2f_s(u[k]);
    }
    reinterpret_cast<s16x8*>(out + r * out_stride)[c] = pack8(o);
  }
}

__global__ __launch_bounds__(256) void embed_kernel(const int32_t* __restrict__ ids,
                                                    const bf16_t* __restrict__ table,
                                                    bf16_t* __restrict__ out, int rows,
                                                    int d, int vocab_start, int vocab_end) {
  const int cpr = d >> 3;
  const int64_t total = (int64_t)rows * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr);
    const int id = ids[r];
    s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    // vocab-parallel embedding: rows outside this rank's shard contribute zeros
    if (id >= vocab_start && id < vocab_end)
      v = reinterpret_cast<const s16x8*>(table + (int64_t)(id - vocab_start) * d)[c];
    reinterpret_cast<s16x8*>(out + r * d)[c] = v;
  }
}

static inline int stream_grid(int64_t work, int block) {
  int64_t g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

void launch_silu_mul(const bf16_t* gate_up, int64_t in_stride, bf16_t* out, int64_t out_stride,
                     int rows, int F, hipStream_t s) {
  if (rows == 0) return;
  const int64_t work = (int64_t)rows * (F >> 3);
  silu_mul_kernel<<<stream_grid(work, 256), 256, 0, s>>>(gate_up, in_stride, out, out_stride,
                                                        rows, F);
}

void launch_embed(const int32_t* ids, const bf16_t* table, bf16_t* out, int rows, int d,
                  int vocab_start, int vocab_end, hipStream_t s) {
  if (rows == 0) return;
  const int64_t work = (int64_t)rows * (d >> 3);
  embed_kernel<<<stream_grid(work, 256), 256, 0, s>>>(ids, table, out, rows, d, vocab_start,
                                                     vocab_end);
}

}  // namespace rfq
