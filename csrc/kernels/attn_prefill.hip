// Paged, causal, variable-length prefill / extend attention with GQA.
// prompts of 262-958 tokens, q_len <= kv_len whenever the
// prefix cache already holds the shared system+template prefix (or for chunked
// prefill / grammar jump-forward extends).
//
// Structure (gfx950):
//   * workgroup = 4 waves = 4 query heads of ONE kv head x one 32-query block, so
//     the K/V tiles staged in LDS are shared by the whole GQA group;
//   * 64-key tiles (two 32-token pages) are staged through registers into LDS:
//       K image  [64][128] bf16, 16-B chunk ch of row r at ch ^ (r & 15)
//                (ds_read_b128 row reads conflict-free, T2),
//       V image  [64][128] bf16, chunk ch of row r at ch ^ ((r & 3) << 2)
//                (ds_read_b64_tr_b16 transposed reads conflict-free, T10);
//   * S^T = K Q^T on mfma_f32_32x32x16_bf16 with Q^T held in registers, so each
//     lane owns one query column and the online softmax is lane-local (+1 xor-32
//     shuffle per row statistic);
//   * O^T = V^T P^T with the S^T accumulators reused as the bf16 B operand
//     (accumulator-as-operand, §3) — O keeps the query on the lane, so the
//     rescale by exp2(m_old - m_new) needs no data movement.
#include "common.h"

namespace rfq {

constexpr int kPD = 128;
constexpr int kPPage = 32;
constexpr int kKT = 64;  // keys per tile
constexpr int kQB = 32;  // queries per wave

__global__ __launch_bounds__(256) void attn_prefill_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_q_start, const int32_t* __restrict__ seq_q_len,
    const int32_t* __restrict__ seq_kv_len, const int32_t* __restrict__ work_seq,
    const int32_t* __restrict__ work_qblk, bf16_t* __restrict__ out, int64_t out_stride, int Hq,
    int Hkv, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* k_lds = reinterpret_cast<bf16_t*>(smem);
  bf16_t* v_lds = k_lds + kKT * kPD;

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h2 = lane >> 5;
  const int seq = work_seq[blockIdx.x];
  const int qs = work_qblk[blockIdx.x] * kQB;
  const int G = Hq / Hkv;
  const int head = blockIdx.y * 4 + wid;
  const int kvh = head / G;
  const int q_len = seq_q_len[seq], kv_len = seq_kv_len[seq];
  const int ctx0 = kv_len - q_len;  // absolute position of query 0
  const int tok0 = seq_q_start[seq];
  const int32_t* bt = block_tables + (int64_t)seq * bt_stride;

  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[query r][16ks + 8h2 .. +7]
  const int qi = qs + r;
  const bool qvalid = qi < q_len;
  s16x8 qf[8];
  {
    const bf16_t* qrow = q + (int64_t)(tok0 + (qvalid ? qi : 0)) * q_stride + (int64_t)head * kPD;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = reinterpret_cast<const s16x8*>(qrow + 16 * ks + 8 * h2)[0];
  }
  const int qpos = ctx0 + qi;
  const int last_q = min(qs + kQB, q_len) - 1;
  const int kv_end = min(kv_len, ctx0 + last_q + 1);  // keys this workgroup needs

  float m_run = -INFINITY, l_run = 0.f;
  f32x16 o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[m][i] = 0.f;

  for (int kt = 0; kt < kv_end; kt += kKT) {
    // ---- stage K/V tile (64 rows x 16 chunks each) : thread -> 4 chunks of K and V
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (threadIdx.x >> 4) + 16 * i, ch = threadIdx.x & 15;
      const int key = kt + row;
      s16x8 kv = (s16x8){0, 0, 0, 0, 0, 0, 0, 0}, vv = kv;
      if (key < kv_end) {
        const int64_t page = bt[key / kPPage];
        const int64_t off = ((page * Hkv + kvh) * kPPage + (key % kPPage)) * kPD;
        kv = reinterpret_cast<const s16x8*>(k_cache + off)[ch];
        vv = reinterpret_cast<const s16x8*>(v_cache + off)[ch];
      }
      reinterpret_cast<s16x8*>(k_lds + row * kPD)[ch ^ (row & 15)] = kv;
      reinterpret_cast<s16x8*>(v_lds + row * kPD)[ch ^ ((row & 3) << 2)] = vv;
    }
    __syncthreads();

    // ---- S^T for two 32-key subtiles ----
    f32x16 s[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[st][i] = 0.f;
      const int row = 32 * st + r;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int ch = 2 * ks + h2;
        const s16x8 a = reinterpret_cast<const s16x8*>(k_lds + row * kPD)[ch ^ (row & 15)];
        s[st] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(qf[ks]), s[st], 0, 0, 0);
      }
    }
    // lane: S^T[key 32st + (i&3) + 8(i>>2) + 4h2][query r]
    float mx = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kt + 32 * st + (i & 3) + 8 * (i >> 2) + 4 * h2;
        float v = s[st][i] * scale_log2;
        if (key > qpos || key >= kv_end) v = -INFINITY;
        s[st][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = fast_exp2(m_run - m_use);
    float psum = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fast_exp2(s[st][i] - m_use);
        s[st][i] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] *= alpha;

    // ---- O^T += V^T P^T ----
    const int gi = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int ksub = 0; ksub < 2; ++ksub) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = s[st][8 * ksub + j];
        const s16x8 pb = pack8(pv);
        const int r0 = 32 * st + 16 * ksub + 4 * h2 + qq;
        const int r1 = r0 + 8;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int col = 32 * m + 16 * (gi & 1) + 4 * pp;
          const int ch = col >> 3, sub = col & 7;
          const s16x4 a0 = ds_read_tr16(v_lds + r0 * kPD + ((ch ^ ((r0 & 3) << 2)) << 3) + sub);
          const s16x4 a1 = ds_read_tr16(v_lds + r1 * kPD + ((ch ^ ((r1 & 3) << 2)) << 3) + sub);
          const s16x8 a = (s16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          o[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(pb), o[m], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  if (!qvalid) return;
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  bf16_t* orow = out + (int64_t)(tok0 + qi) * out_stride + (int64_t)head * kPD;
  // O^T lane: dh rows (i&3) + 8(i>>2) + 4h2 of each 32-row tile m
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint2 w;
      w.x = pack_bf16x2(o[m][4 * k + 0] * inv, o[m][4 * k + 1] * inv);
      w.y = pack_bf16x2(o[m][4 * k + 2] * inv, o[m][4 * k + 3] * inv);
      *reinterpret_cast<uint2*>(orow + 32 * m + 8 * k + 4 * h2) = w;
    }
}

void launch_attn_prefill(const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                         const bf16_t* v_cache, const int32_t* block_tables, int bt_stride,
                         const int32_t* seq_q_start, const int32_t* seq_q_len,
                         const int32_t* seq_kv_len, const int32_t* work_seq,
                         const int32_t* work_qblk, int num_work, bf16_t* out, int64_t out_stride,
                         int Hq, int Hkv, float scale, hipStream_t s) {
  if (num_work == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_work, Hq / 4);
  const size_t lds = 2 * kKT * kPD * sizeof(bf16_t);
  attn_prefill_kernel<<<grid, 256, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                             bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                             work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                             scale_log2);
}

}  // namespace rfq
