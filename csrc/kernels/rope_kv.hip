// Rotary embedding (rotate-half / NeoX form used by Llama-3 and Mixtral) fused with
// the paged KV-cache append.  SURVEY.md §2.4 K4+K5.
//
// One workgroup per token.  q heads are rotated in place inside the fused QKV GEMM
// output (so attention reads q straight from it), k heads are rotated and
// scattered into the paged cache together with v.  cos/sin come from a host-built
// table (no on-device trig — Appendix B, element-wise ops).
//
// Cache layout (per layer): [num_blocks][Hkv][BS][D] bf16 — one (block, head) is a
// contiguous BS*D*2-byte page, which is what the attention kernels stream.
#include "common.h"

namespace rfq {

constexpr int kHeadDim = 128;

__global__ __launch_bounds__(256) void rope_kv_kernel(
    bf16_t* __restrict__ qkv, int64_t qkv_stride, const int32_t* __restrict__ positions,
    const float* __restrict__ cos_sin, const int32_t* __restrict__ slot_mapping,
    bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache, int Hq, int Hkv, int BS) {
  constexpr int D = kHeadDim, HALF = D / 2, PC = HALF / 8;  // 8 pair-chunks per head
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int slot = slot_mapping[t];
  bf16_t* row = qkv + (int64_t)t * qkv_stride;
  const float* cs = cos_sin + (int64_t)pos * D;
  const int rot_items = (Hq + Hkv) * PC;
  const int v_items = Hkv * (D / 8);
  const int64_t blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  for (int it = threadIdx.x; it < rot_items + v_items; it += blockDim.x) {
    if (it < rot_items) {
      const int h = it / PC, pc = it % PC;
      bf16_t* hp = row + h * D;
      const s16x8 x1v = reinterpret_cast<const s16x8*>(hp)[pc];
      const s16x8 x2v = reinterpret_cast<const s16x8*>(hp + HALF)[pc];
      const float4* c4 = reinterpret_cast<const float4*>(cs + pc * 8);
      const float4* s4 = reinterpret_cast<const float4*>(cs + HALF + pc * 8);
      float c[8], s[8];
      *reinterpret_cast<float4*>(c) = c4[0];
      *reinterpret_cast<float4*>(c + 4) = c4[1];
      *reinterpret_cast<float4*>(s) = s4[0];
      *reinterpret_cast<float4*>(s + 4) = s4[1];
      float o1[8], o2[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float a = bf2f_s(x1v[i]), b = bf2f_s(x2v[i]);
        o1[i] = a * c[i] - b * s[i];
        o2[i] = b * c[i] + a * s[i];
      }
      const s16x8 p1 = pack8(o1), p2 = pack8(o2);
      if (h < Hq) {
        reinterpret_cast<s16x8*>(hp)[pc] = p1;
        reinterpret_cast<s16x8*>(hp + HALF)[pc] = p2;
      } else if (slot >= 0) {
        const int kh = h - Hq;
        bf16_t* dst = k_cache + ((blk * Hkv + kh) * BS + off) * D;
        reinterpret_cast<s16x8*>(dst)[pc] = p1;
        reinterpret_cast<s16x8*>(dst + HALF)[pc] = p2;
      }
    } else if (slot >= 0) {
      const int j = it - rot_items;
      const int vh = j / (D / 8), c = j % (D / 8);
      const s16x8 v = reinterpret_cast<const s16x8*>(row + (Hq + Hkv + vh) * D)[c];
      bf16_t* dst = v_cache + ((blk * Hkv + vh) * BS + off) * D;
      reinterpret_cast<s16x8*>(dst)[c] = v;
    }
  }
}

void launch_rope_kv(bf16_t* qkv, int64_t qkv_stride, const int32_t* positions,
                    const float* cos_sin, const int32_t* slot_mapping, bf16_t* k_cache,
                    bf16_t* v_cache, int T, int Hq, int Hkv, int BS, hipStream_t s) {
  if (T == 0) return;
  rope_kv_kernel<<<T, 256, 0, s>>>(qkv, qkv_stride, positions, cos_sin, slot_mapping, k_cache,
                                  v_cache, Hq, Hkv, BS);
}

}  // namespace rfq
