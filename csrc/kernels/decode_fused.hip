// Fused QKV projection + RoPE + KV append + decode attention: ONE launch per layer on
// the latency path (M <= 16 decode / jump-forward rows, no prefill rows in the step).
//
// Why: at batch 1 the QKV GEMV (split-K weight stream, gemm_skinny.hip) and the split-K
// decode attention are two dependent launches.  The attention launch cannot start its
// KV-page loads -- a metadata -> block table -> page chain of three memory round trips
// -- until the QKV launch has drained, and it then runs latency-bound on a handful of
// waves (7.7 us per layer for the 8B model, profiles/r3_latency_8b_kernel_stats_
// session2.md) while 250 CUs idle.  Here the attention waves are extra workgroups at
// the END of the QKV GEMV's grid: they walk that chain and load every KV page that
// holds only earlier tokens while the weight stream runs, then wait on a per-kv-head
// counter for the QKV tiles of their group (gemv_core.h PUB: write-through results +
// one relaxed agent-scope count per tile), read q and this step's new KV rows with sc1
// loads, and finish with the pages already in registers (attn_decode_core.h FUSED).
//
// Grid: [units QKV work units (NW waves each)] + [ceil(n_att / NW) workgroups of NW
// independent attention waves].  Dispatch is in blockIdx order in practice, so the
// spinning attention waves never hold slots the QKV units still need (a few dozen waves
// on a 256-CU chip); correctness never depends on it: every spin is bounded in wall
// time and a timeout is counted in err (the runner fails such a step).
// The split-K partials of the attention are merged by attn_decode_reduce afterwards.
#include "gemv_core.h"
#include "attn_decode_core.h"

namespace rfq {

struct FusedAttnArgs {
  const int32_t* block_tables;
  int bt_stride;
  const int32_t* seq_q_start;
  const int32_t* seq_q_len;
  const int32_t* seq_kv_len;
  const int32_t* work_seq;
  const int32_t* work_ct;
  const bf16_t* k_cache;
  const bf16_t* v_cache;
  bf16_t* out;
  int64_t out_stride;
  float* part_o;
  float* part_ml;
  float scale_log2;
  int num_splits;
  int list_tpi;   // column tiles per work item of the work list
  int run_tiles;  // of those, how many can hold columns (1 when every row is a decode row)
  int n_att;      // attention waves: num_splits * Hkv * work items * run_tiles
  int att_wgs;    // workgroups of attention waves
  int att_last;   // 0: attention workgroups first in the grid, 1: after the QKV units
  unsigned* zero_slot;   // the previous layer's counter slot, zeroed here (Hkv words)
};

// NW = 8: the attention waves need ~240 VGPRs (two KV pages in flight), so the kernel
// runs one 8-wave workgroup per CU -- what the QKV GEMV's 8-wave cfgs already run at.
template <int U, bool TL, bool NTL>
__global__ __launch_bounds__(512) void qkv_attn_kernel(
    const bf16_t* __restrict__ X, int64_t ldx, const bf16_t* __restrict__ W, int K,
    bf16_t* __restrict__ Y, int64_t ldy, int M, int KS, float* __restrict__ part, int Nn,
    unsigned* __restrict__ tile_cnt, RopeEpi re, int units, FusedAttnArgs aa, FuseWait fw) {
  constexpr int NW = 8;
  __shared__ __attribute__((aligned(16))) bf16_t att_lds[NW * kPage * kD];
  const int b = (int)blockIdx.x;
  const int ub = aa.att_last ? b : b - aa.att_wgs;        // QKV work unit of this block
  if (ub >= 0 && ub < units) {
    // QKV work unit; the first one zeroes the previous layer's counters (its launch
    // drained before this one started, so nothing reads them any more)
    if (ub == 0 && threadIdx.x < (unsigned)re.Hkv && aa.zero_slot != nullptr)
      __hip_atomic_store((gu32*)(aa.zero_slot + kFuseStride * threadIdx.x), 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    gemv_splitk_unit<NW, U, kGvRope, TL, NTL, true>(ub, units / KS, X, ldx, W, K, Y, ldy, M, KS,
                                                    part, Nn, tile_cnt, NormEpi{}, re, 0, fw.done);
    return;
  }
  // attention waves: first in the grid (att_last 0) they walk the metadata -> block
  // table -> KV page chain while the QKV units stream their weights; last, they take
  // the CUs the first finished QKV units free
  const int wv = (int)(threadIdx.x >> 6);
  const int idx = (aa.att_last ? b - units : b) * NW + wv;
  if (idx >= aa.n_att) return;             // wave-uniform; no workgroup barrier below
  const int S = aa.num_splits;
  const int split = idx % S;
  int rest = idx / S;
  const int kvh = rest % re.Hkv;
  rest /= re.Hkv;
  const int n_work = aa.n_att / (S * re.Hkv * aa.run_tiles);
  const int w = rest % n_work, t = rest / n_work;   // tile-major: active tile-0 waves first
  FuseWait f = fw;
  f.ct_mult = aa.list_tpi;
  f.ct_add = t;
  attn_decode_body<1, 0, 1, false, true>(
      Y, ldy, aa.k_cache, aa.v_cache, aa.block_tables, aa.bt_stride, aa.seq_q_start, aa.seq_q_len,
      aa.seq_kv_len, aa.work_seq, aa.work_ct, aa.out, aa.out_stride, aa.part_o, aa.part_ml, re.Hq,
      re.Hkv, aa.scale_log2, S, PrefixArgs{}, nullptr, split, kvh, w, 0, att_lds + wv * kPage * kD,
      f);
}

// cfg: the split-K GEMV cfg bits of launch_gemv_splitk_epi (KS = 2 << (cfg & 3); bit 3
// = U 2; bit 4 = tiled weights; bit 5 = non-temporal); always 8 waves; bit 6: the
// attention workgroups after the QKV units instead of before them.  done: this
// layer's counter slot (Hkv uint32, zero at launch); zero_slot: the previous layer's
// slot (zeroed here, may be null); err: uint32 timeout counter.
void launch_qkv_attn(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K, bf16_t* Y,
                     int64_t ldy, int M, int cfg, float* part, unsigned* tile_cnt,
                     const int32_t* positions, const float* cos_sin, const int32_t* slots,
                     bf16_t* k_cache, bf16_t* v_cache, int Hq, int Hkv, int BS,
                     const int32_t* block_tables, int bt_stride, const int32_t* seq_q_start,
                     const int32_t* seq_q_len, const int32_t* seq_kv_len,
                     const int32_t* work_seq, const int32_t* work_ct, int n_work, int list_tpi,
                     int run_tiles, bf16_t* out, int64_t out_stride, float* part_o,
                     float* part_ml, float scale, int num_splits, unsigned* done,
                     unsigned* zero_slot, unsigned* err, hipStream_t s) {
  constexpr int NW = 8;
  const int KS = 2 << (cfg & 3);
  const int units = (N / 32) * KS;
  const RopeEpi re{positions, cos_sin, slots, k_cache, v_cache, Hq, Hkv, BS};
  const int n_att = num_splits * Hkv * n_work * run_tiles;
  FusedAttnArgs aa{block_tables, bt_stride, seq_q_start, seq_q_len, seq_kv_len, work_seq,
                   work_ct, k_cache, v_cache, out, out_stride, part_o, part_ml,
                   scale * 1.4426950408889634f, num_splits, list_tpi, run_tiles, n_att,
                   (n_att + NW - 1) / NW, (cfg >> 6) & 1, zero_slot};
  const int G = Hq / Hkv;
  const FuseWait fw{done, (unsigned)((G + 2) * 4), err, 1, 0};
  const dim3 grid(aa.att_wgs + units);
#define QA_LAUNCH(Uv)                                                                          \
  switch ((cfg >> 4) & 3) {                                                                    \
    case 0: hipLaunchKernelGGL((qkv_attn_kernel<Uv, false, false>), grid, dim3(512), 0, s,       \
                               X, ldx, W, K, Y, ldy, M, KS, part, N, tile_cnt, re, units, aa, fw); \
            break;                                                                             \
    case 1: hipLaunchKernelGGL((qkv_attn_kernel<Uv, true, false>), grid, dim3(512), 0, s,        \
                               X, ldx, W, K, Y, ldy, M, KS, part, N, tile_cnt, re, units, aa, fw); \
            break;                                                                             \
    case 2: hipLaunchKernelGGL((qkv_attn_kernel<Uv, false, true>), grid, dim3(512), 0, s,        \
                               X, ldx, W, K, Y, ldy, M, KS, part, N, tile_cnt, re, units, aa, fw); \
            break;                                                                             \
    default: hipLaunchKernelGGL((qkv_attn_kernel<Uv, true, true>), grid, dim3(512), 0, s,        \
                                X, ldx, W, K, Y, ldy, M, KS, part, N, tile_cnt, re, units, aa, fw);\
  }
  if (cfg & 8) { QA_LAUNCH(2); } else { QA_LAUNCH(4); }
#undef QA_LAUNCH
}

}  // namespace rfq
