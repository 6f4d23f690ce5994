// JSON-schema-constrained sampler: grammar bitmask + temperature + Gumbel-max
// argmax over the (possibly vocab-sharded) logits.  SURVEY.md §2.4 K13/K14.
//
// The reference decodes at temperature 0.1 (rfq_agent.py:66) and must emit JSON
// only (rfq_agent.py:103,114).  The grammar runtime on the host reduces every
// sequence's automaton state to an index into a small table of precomputed
// vocabulary bitmasks (one u32 per 32 token ids, global ids), so a step uploads
// only B int32s.  Sampling is Gumbel-max — argmax(logit/T + G), G ~ Gumbel(0,1)
// from a counter-based hash of (per-row seed, global token id) — which is exactly
// categorical sampling at temperature T and reduces to a plain (val, idx) argmax.
// That makes the tensor-parallel form trivial: each rank reduces its vocab shard,
// the (val, idx) partials are all-gathered, and the same second stage picks the
// winner.  Every rank draws identical noise for a given global id.
#include "common.h"

namespace rfq {

constexpr int kSampleBlock = 256;

__global__ __launch_bounds__(kSampleBlock) void sample_partial_kernel(
    const bf16_t* __restrict__ logits, int64_t row_stride, int Vl, int v0,
    const uint32_t* __restrict__ mask_table, int mask_words, const int32_t* __restrict__ mask_idx,
    const float* __restrict__ temps, const uint64_t* __restrict__ seeds,
    float* __restrict__ part_val, int32_t* __restrict__ part_idx, int chunk) {
  __shared__ float sv[kSampleBlock / 64];
  __shared__ int si[kSampleBlock / 64];
  const int split = blockIdx.x, b = blockIdx.y, nsplit = gridDim.x;
  const int c0 = split * chunk, c1 = min(Vl, c0 + chunk);
  const int mi = mask_idx[b];
  const uint32_t* mrow = mi >= 0 ? mask_table + (int64_t)mi * mask_words : nullptr;
  const float t = temps[b];
  const float invT = t > 0.f ? 1.f / t : 0.f;
  const uint64_t seed = seeds[b];
  const bf16_t* row = logits + (int64_t)b * row_stride;

  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int c = c0 + threadIdx.x * 8; c < c1; c += kSampleBlock * 8) {
    const int gcol = v0 + c;
    uint32_t bits = 0xffu;
    if (mrow) bits = (mrow[gcol >> 5] >> (gcol & 31)) & 0xffu;
    if (bits == 0) continue;
    const s16x8 v = reinterpret_cast<const s16x8*>(row + c)[0];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (!((bits >> k) & 1u) || c + k >= c1) continue;
      float sc = bf2f_s(v[k]);
      if (t > 0.f) {
        const uint32_t hsh = hash_u32(seed, 0x9e3779b9u, (uint32_t)(gcol + k));
        const float u = ((float)(hsh >> 8) + 0.5f) * (1.f / 16777216.f);
        sc = sc * invT - __logf(-__logf(u));
      }
      if (sc > best || (sc == best && gcol + k < besti)) {
        best = sc;
        besti = gcol + k;
      }
    }
  }
  // wave argmax, then across the block's waves
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ov > best || (ov == best && oi < besti)) { best = ov; besti = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = best; si[wid] = besti; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kSampleBlock / 64; ++w)
      if (sv[w] > best || (sv[w] == best && si[w] < besti)) { best = sv[w]; besti = si[w]; }
    part_val[(int64_t)b * nsplit + split] = sv[0] > best ? sv[0] : best;
    part_idx[(int64_t)b * nsplit + split] = besti;
  }
}

// Final argmax over n partials per row (n = splits, or ranks*splits after the
// tensor-parallel all-gather).  One wave per row.
__global__ __launch_bounds__(64) void sample_final_kernel(const float* __restrict__ part_val,
                                                          const int32_t* __restrict__ part_idx,
                                                          int n, int64_t row_stride,
                                                          int64_t group_stride, int groups,
                                                          int32_t* __restrict__ out_tokens) {
  const int b = blockIdx.x;
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int gr = 0; gr < groups; ++gr)
    for (int i = threadIdx.x; i < n; i += 64) {
      const int64_t o = gr * group_stride + b * row_stride + i;
      const float v = part_val[o];
      const int id = part_idx[o];
      if (v > best || (v == best && id < besti)) { best = v; besti = id; }
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ov > best || (ov == best && oi < besti)) { best = ov; besti = oi; }
  }
  if (threadIdx.x == 0) out_tokens[b] = besti == 0x7fffffff ? 0 : besti;
}

void launch_sample_partial(const bf16_t* logits, int64_t row_stride, int B, int Vl, int v0,
                           const uint32_t* mask_table, int mask_words, const int32_t* mask_idx,
                           const float* temps, const uint64_t* seeds, float* part_val,
                           int32_t* part_idx, int nsplit, hipStream_t s) {
  if (B == 0) return;
  int chunk = (Vl + nsplit - 1) / nsplit;
  chunk = (chunk + 7) / 8 * 8;
  dim3 grid(nsplit, B);
  sample_partial_kernel<<<grid, kSampleBlock, 0, s>>>(logits, row_stride, Vl, v0, mask_table,
                                                      mask_words, mask_idx, temps, seeds,
                                                      part_val, part_idx, chunk);
}

void launch_sample_final(const float* part_val, const int32_t* part_idx, int B, int n,
                         int groups, int32_t* out_tokens, hipStream_t s) {
  if (B == 0) return;
  sample_final_kernel<<<B, 64, 0, s>>>(part_val, part_idx, n, n, (int64_t)B * n, groups,
                                       out_tokens);
}

}  // namespace rfq
