// Paged attention for decode and short extend rows (q_len small), GQA, split-K.
// SURVEY.md §2.4 K7 — the bandwidth-critical kernel of a large-batch decode step,
// also used for grammar jump-forward extends (a sampled token + the forced schema
// tokens after it, q_len = 1 + k, k ~ 3-8).
//
// Design (gfx950, wave64):
//   * one wave per (split, kv_head, work item); a work item is (sequence, column
//     tile).  The 16 MFMA columns of mfma_f32_16x16x32_bf16 are (query, head)
//     pairs c = query * G + head of one kv head: a decode row uses G columns, an
//     extend row q_len * G (several column tiles if > 16).  Each K/V byte is read
//     once per column tile, i.e. once per kv head for decode.
//   * QK^T is computed swapped, S^T = K * Q^T: K fragments are 16-byte rows loaded
//     straight from the page into VGPRs (no LDS round trip; "GEMV / M<=16" row
//     of the staging table).  The result has one column per lane, so the online
//     softmax state (running max, partial sum) is lane-local; each column carries
//     its own causal limit (key < kv_len - q_len + query + 1).
//   * P*V is computed as O^T = V^T * P^T: the S^T accumulators are converted in
//     place into the bf16 B operand (accumulator-as-operand, §3), V goes through
//     LDS once and is read back with ds_read_b64_tr_b16 (T10) in the permuted key
//     order the accumulator layout implies.  O^T keeps the column on the lane, so
//     the softmax rescale needs no cross-lane traffic.
//   * V's LDS image is XOR-swizzled (chunk ^ ((row&7)<<1)) so every transposed read
//     of a 32-lane half touches 16 distinct 16-byte slots (conflict-free).
//   * split-K partials (unnormalised O, running max, sum) are merged by
//     attn_decode_reduce; with one split the kernel writes bf16 output directly.
//   The split size is derived per sequence from its context length on device, so a
//   hipGraph captured with a fixed split count stays balanced as contexts grow.
//
// Shared-prefix (cascade) mode, large decode batches: every RFQ request starts with the
// same system prompt + template, whose KV pages the prefix cache shares.  Reading those
// pages once per sequence is ~half of the decode KV traffic.  attn_prefix_meta finds on
// device the longest run of leading pages that decode sequence 0 shares with the other
// sequences (P pages; sequences sharing fewer than kMinPrefixPages opt out), then
//   * MODE 2 (prefix): the MFMA columns are (q row, head) pairs of EIGHT different
//     sequences (NT = 2, G = 4), so each prefix K/V page is read once per 8 rows;
//     writes the unnormalised O, running max and sum per (row, head);
//   * MODE 1 (suffix): the normal per-sequence kernel over keys [P*32, kv_len) that
//     merges the prefix partial into its registers before the bf16 store.
// Everything is derived on device, so captured decode graphs stay valid.
#include "attn_decode_core.h"

namespace rfq {

// Single workgroup: P = min over participating sequences of the shared leading page run.
__global__ __launch_bounds__(1024) void attn_prefix_meta_kernel(
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ seq_q_start,
    const int32_t* __restrict__ seq_q_len, const int32_t* __restrict__ seq_kv_len, int nseq,
    int32_t* __restrict__ meta, int32_t* __restrict__ pflag, int32_t* __restrict__ rowlist) {
  __shared__ int32_t ref[256];
  __shared__ int32_t s_min, s_cnt, s_cand;
  const int tid = threadIdx.x;
  const int ref_len = nseq > 0 ? min(min((seq_kv_len[0] - seq_q_len[0]) / kPage, bt_stride), 256) : 0;
  if (tid < ref_len) ref[tid] = block_tables[tid];
  if (tid == 0) { s_min = 1 << 30; s_cnt = 0; s_cand = 0; }
  __syncthreads();
  for (int s = tid; s < nseq; s += blockDim.x) {
    const int cap = min(ref_len, (seq_kv_len[s] - seq_q_len[s]) / kPage);
    const int32_t* bt = block_tables + (int64_t)s * bt_stride;
    int m = 0;
    while (m < cap && bt[m] == ref[m]) ++m;
    pflag[s] = m;
    if (m >= kMinPrefixPages) {
      atomicMin(&s_min, m);
      atomicAdd(&s_cand, 1);
    }
  }
  __syncthreads();
  const int P = s_cand < 2 ? 0 : s_min;     // sequence 0 alone shares nothing
  for (int s = tid; s < nseq; s += blockDim.x) {
    const int on = P > 0 && pflag[s] >= P;   // each thread rereads only what it wrote
    pflag[s] = on;
    if (on) {
      const int ql = seq_q_len[s], q0 = seq_q_start[s];
      const int base = atomicAdd(&s_cnt, ql);
      for (int i = 0; i < ql; ++i) rowlist[base + i] = q0 + i;
    }
  }
  __syncthreads();
  if (tid == 0) { meta[0] = P * kPage; meta[1] = s_cnt; }
}

template <int NT, int MODE = 0, bool NTK = false>
__global__ __launch_bounds__(64, 2) void attn_decode_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    int bt_stride, const int32_t* __restrict__ seq_q_start, const int32_t* __restrict__ seq_q_len,
    const int32_t* __restrict__ seq_kv_len, const int32_t* __restrict__ work_seq,
    const int32_t* __restrict__ work_ct, bf16_t* __restrict__ out, int64_t out_stride,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hq, int Hkv, float scale_log2,
    int num_splits, PrefixArgs px = PrefixArgs{}, int32_t* __restrict__ tickets = nullptr) {
  __shared__ __attribute__((aligned(16))) bf16_t v_lds[kPage * kD];
  attn_decode_body<NT, MODE, NTK>(
      q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_q_start, seq_q_len, seq_kv_len,
      work_seq, work_ct, out, out_stride, part_o, part_ml, Hq, Hkv, scale_log2, num_splits, px,
      tickets, blockIdx.x, blockIdx.y, blockIdx.z, v_lds);
}

// Merge split-K partials: one workgroup of 128 lanes (one per dh) per (row, head).
__global__ __launch_bounds__(128) void attn_decode_reduce_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_ml,
    bf16_t* __restrict__ out, int64_t out_stride, int Hq, int num_splits) {
  const int bh = blockIdx.x;
  const int b = bh / Hq, h = bh % Hq;
  const int d = threadIdx.x;
  __shared__ float ml_s[2 * 32];
  const float* ml = part_ml + (int64_t)bh * num_splits * 2;
  if (d < 2 * num_splits) ml_s[d] = ml[d];     // num_splits <= 32: one load per lane
  // issue every split's partial load before the LDS round trip
  float po[32];
#pragma unroll
  for (int s = 0; s < 32; ++s)
    po[s] = s < num_splits ? part_o[((int64_t)bh * num_splits + s) * kD + d] : 0.f;
  __syncthreads();
  float gm = -INFINITY;
  for (int s = 0; s < num_splits; ++s) gm = fmaxf(gm, ml_s[2 * s]);
  float num = 0.f, den = 0.f;
  if (gm != -INFINITY) {
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (s >= num_splits) break;
      const float ms = ml_s[2 * s];
      if (ms == -INFINITY) continue;
      const float wgt = fast_exp2(ms - gm);
      num += wgt * po[s];
      den += wgt * ml_s[2 * s + 1];
    }
  }
  out[(int64_t)b * out_stride + (int64_t)h * kD + d] = f2bf(den > 0.f ? num / den : 0.f);
}

// Merge split-K partials of `rows` q rows (also exposed as ops.attn_decode_merge for a
// decode attention launched with reduce = false).
void launch_attn_decode_reduce(const float* part_o, const float* part_ml, bf16_t* out,
                               int64_t out_stride, int rows, int Hq, int num_splits,
                               hipStream_t s) {
  if (rows == 0 || num_splits <= 1) return;
  attn_decode_reduce_kernel<<<rows * Hq, 128, 0, s>>>(part_o, part_ml, out, out_stride, Hq,
                                                      num_splits);
}

// rows = number of q rows covered (for the split-K reduce), W = work items;
// reduce = false leaves split partials for the consumer to merge (attn_decode_merge)
void launch_attn_decode(const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                        const bf16_t* v_cache, const int32_t* block_tables, int bt_stride,
                        const int32_t* seq_q_start, const int32_t* seq_q_len,
                        const int32_t* seq_kv_len, const int32_t* work_seq,
                        const int32_t* work_ct, int W, int rows, bf16_t* out, int64_t out_stride,
                        float* part_o, float* part_ml, int Hq, int Hkv, float scale,
                        int num_splits, int tiles_per_item, int32_t* tickets, hipStream_t s,
                        bool reduce) {
  if (W == 0 || rows == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_splits, Hkv, W);
  int32_t* tk = num_splits > 1 ? tickets : nullptr;
  // RFQ_ATTN_NT=1: non-temporal loads for the per-sequence KV pages (NTK above)
  static const bool ntk = [] {
    const char* v = getenv("RFQ_ATTN_NT");
    return v != nullptr && v[0] == '1';
  }();
#define RFQ_AD_LAUNCH(T, N)                                                                     \
  attn_decode_kernel<T, 0, N><<<grid, 64, 0, s>>>(                                            \
      q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_q_start, seq_q_len,            \
      seq_kv_len, work_seq, work_ct, out, out_stride, part_o, part_ml, Hq, Hkv, scale_log2,      \
      num_splits, PrefixArgs{}, tk)
  if (tiles_per_item == 2) {
    if (ntk) RFQ_AD_LAUNCH(2, true); else RFQ_AD_LAUNCH(2, false);
  } else {
    if (ntk) RFQ_AD_LAUNCH(1, true); else RFQ_AD_LAUNCH(1, false);
  }
#undef RFQ_AD_LAUNCH
  // without a ticket buffer the split partials are merged by a second launch
  if (num_splits > 1 && tk == nullptr && reduce)
    attn_decode_reduce_kernel<<<rows * Hq, 128, 0, s>>>(part_o, part_ml, out, out_stride, Hq,
                                                        num_splits);
}

// Shared-prefix decode attention (num_splits == 1): meta pass, prefix pass over the rows
// of the participating sequences (8 rows per wave), suffix pass per sequence + merge.
// ws_i32: [2 + nseq + rows] int32; pre_o: rows*Hq*128 fp32; pre_ml: rows*Hq*2 fp32.
void launch_attn_decode_shared(const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                               const bf16_t* v_cache, const int32_t* block_tables, int bt_stride,
                               const int32_t* seq_q_start, const int32_t* seq_q_len,
                               const int32_t* seq_kv_len, int nseq, const int32_t* work_seq,
                               const int32_t* work_ct, int W, int rows, bf16_t* out,
                               int64_t out_stride, int32_t* ws_i32, float* pre_o, float* pre_ml,
                               int Hq, int Hkv, float scale, int tiles_per_item, bool run_meta,
                               hipStream_t s) {
  if (W == 0 || rows == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  PrefixArgs px{ws_i32, ws_i32 + 2, ws_i32 + 2 + nseq, pre_o, pre_ml};
  if (run_meta)
    attn_prefix_meta_kernel<<<1, 1024, 0, s>>>(block_tables, bt_stride, seq_q_start, seq_q_len,
                                                seq_kv_len, nseq, ws_i32, ws_i32 + 2,
                                                ws_i32 + 2 + nseq);
  const int G = Hq / Hkv;
  const dim3 gp(1, Hkv, (rows * G + 31) / 32);
  attn_decode_kernel<2, 2><<<gp, 64, 0, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                             bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                             work_seq, work_ct, out, out_stride, nullptr, nullptr,
                                             Hq, Hkv, scale_log2, 1, px);
  const dim3 grid(1, Hkv, W);
  if (tiles_per_item == 2)
    attn_decode_kernel<2, 1><<<grid, 64, 0, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                 bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                 work_seq, work_ct, out, out_stride, nullptr,
                                                 nullptr, Hq, Hkv, scale_log2, 1, px);
  else
    attn_decode_kernel<1, 1><<<grid, 64, 0, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                 bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                 work_seq, work_ct, out, out_stride, nullptr,
                                                 nullptr, Hq, Hkv, scale_log2, 1, px);
}

}  // namespace rfq
