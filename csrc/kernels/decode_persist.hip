// Persistent decode layers for small steps (M <= 4 rows, every row a decode / short
// extend row): one launch runs the whole chain
//
//   qkv + RoPE + KV append (folded attn norm) -> paged attention + split merge
//   -> o (+= residual) -> gate|up + SwiGLU (folded mlp norm) -> down (+= residual)
//
// for a range of layers (the whole step), or any sub-range of those stages (e.g. only
// attention -> o per layer, with the projections on their own launches).  SURVEY.md §3.4
// / §7.2 step 7; VERDICT r5 item 1.
//
// Why.  At batch 1 a decode layer is five weight-streaming launches.  Every launch pays a
// boundary (~1.2-1.9 µs), its own fill and drain, and every dependent latency chain in it
// (the attention: metadata -> q -> K/V -> split partials -> ticket -> merge, ~10 µs for a
// few MB) runs with the weight stream stopped.  The weight loads of a stage never depend
// on the previous stage's output, so here they are issued BEFORE the stage's input is
// ready: while the attention chain runs on a few waves, every other wave already holds
// its slice of the o projection in registers (8B: the whole 33.5 MB o weight is in
// flight during the attention), and at every other seam the next stage's first 16 KB
// per wave are in flight while the seam settles (cdna_hip_programming.md §5.6,
// MI355X_MICROARCH.md 'prefetch-credit').
//
// Geometry: one workgroup of 4 waves per CU (grid = CUs, all resident), one wave per SIMD
// with the whole 512-register file: three 16 KB weight groups in flight per wave (192 KB
// per CU) and the attention body without spills.
// Work of a stage is dealt to the 4 x CUs waves with consecutive units on different CUs:
// wave slot gw = wave * CUs + workgroup; unit U goes to slot U % slots.
//
// GEMV stages (the row-streaming scheme of gemv_rows.hip): a unit is one weight row
// (o, down: residual add) or a pair of rows (qkv: the rotate-half partners of one head,
// RoPE + KV append; gate|up: gate row q and up row F + q, SwiGLU); each lane reads 16 B
// of every 1 KB chunk of the row (non-temporal), the stage's input rows come from LDS
// (staged once per workgroup per stage), v_dot2c_f32_bf16 accumulates, a DPP wave sum
// reduces.  A wave streams its (unit, chunk) items in groups of 16 loads (16 KB),
// three groups in flight; the first three groups of a stage are prefetched across the seam.
// Per-lane accumulation order = gemv_rows.hip's, so each projection is bit-identical to
// its row-streaming launch.
//
// Attention stage: one wave per (work item, kv head, split), the MODE-0 / one-column-
// tile body of attn_decode_core.h with the in-launch loads made sc1 (q and the new
// token's K / V were written by this launch) and a wave-local V-tile sync; split
// partials merge in-kernel (the last split of a (work item, kv head) merges, ticket
// protocol of attn_decode_core.h).
//
// Seams (cdna_hip_programming.md §6 Guideline 16, counter form, sc1 everywhere): every
// store another CU reads in this launch is an sc1 store (write-through); each wave drains
// its stores (vmcnt(0)), the workgroup meets at a barrier, one lane adds 1 to its shard
// (workgroup % 8) of the seam's counter; wave 0 polls the 8 shards with sc1 loads until
// they sum to the grid, then a barrier releases the workgroup; every load of handed-off
// bytes is an sc1 load.  Waves issue the next stage's first three weight groups before they
// wait, so the stream keeps going through the seam; wave 0 polls first, except behind the
// attention (its poll would wait behind its own prefetch: loads retire in order, and only
// the attention seam is long enough to hide that).
// Every wait is bounded (1 s on s_memrealtime): a timeout counts kErrPersist (kerr.hip),
// records the first failing (layer, stage) and raises the launch's abort word, and every
// wave then skips the remaining work -- the runner sees the error after the step and fails
// it.  The last workgroup to leave zeroes the launch's counters (they start zeroed:
// allocated with zeros), so graph replays need no memset.
#include "attn_decode_core.h"
#include "rows_core.h"

namespace rfq {

enum { kDpQkv = 0, kDpAttn = 1, kDpO = 2, kDpGu = 3, kDpDown = 4, kDpStages = 5 };
enum { kEpRope = 0, kEpSwi = 1, kEpRes = 2 };
constexpr int kDpWaves = 4;               // one wave per SIMD: 512 registers each
constexpr int kDpThreads = kDpWaves * 64;
constexpr int kDpLoads = 16;              // 16-byte weight loads per wave per group
constexpr int kDpShards = 8;              // seam counter shards
constexpr int kDpShardWords = 32;         // 128 B between shards
constexpr int kDpMaxM = 4;
constexpr int kDpCsBytes = kDpMaxM * 128 * 4;     // cos / sin rows of the step's tokens
constexpr int kDpCtlBytes = 64;
constexpr int kDpVTile = kPage * kD * 2;          // 8 KB V tile per attention wave
constexpr int kSc1 = 16;                          // buffer aux: sc1 (device scope)
constexpr int kNt = 2;                            // buffer aux: nt

struct DpLayer {                 // one layer's pointers (device table, 8 x 8 bytes)
  const bf16_t* wqkv;            // [(Hq + 2 Hkv) * 128, d], attention norm folded in
  const bf16_t* wo;              // [d, Hq * 128]
  const bf16_t* wgu;             // [2F, d], MLP norm folded in
  const bf16_t* wd;              // [d, F]
  bf16_t* kc;                    // [blocks, Hkv, 32, 128]
  bf16_t* vc;
  const void* pad0;
  const void* pad1;
};

struct DpArgs {
  const DpLayer* layers;
  int l0, l1, stages;            // layers [l0, l1), stage bit mask (1 << kDp*)
  int M, d, Hq, Hkv, F;
  bf16_t* residual;              // [M, d]
  bf16_t* qbuf;                  // q rows (RoPE applied), row stride ldq
  int ldq;
  bf16_t* attn;                  // [M, Hq * 128]
  bf16_t* act;                   // [M, F]
  const int32_t* positions;
  const float* cos_sin;          // [max_pos, 128]
  const int32_t* slots;
  int BS;
  const int32_t* block_tables;
  int bt_stride;
  const int32_t* q_start;
  const int32_t* q_len;
  const int32_t* kv_len;
  const int32_t* work_seq;
  const int32_t* work_ct;
  int W, splits;
  float* part_o;
  float* part_ml;
  int32_t* tickets;
  float scale_log2;
  uint32_t* cnt;                 // seam counters (see dp_cnt), abort and exit words
  uint32_t* err;                 // kernel_error_words (may be null)
  float eps;
  int flags;                     // A/B and timing bits: 1 wave 0 prefetches too, 2 no
                                 // cross-seam prefetch, 4 attention units skipped (timing),
                                 // 8 rotated chunk start per wave, 16 the engine form;
                                 // engine timing bits (WRONG results): 32 slots released
                                 // unread, 64 no weight stream
  int eg_ring, eg_parts, eg_area, eg_ring_off;   // engine form: ring slots, LDS offsets
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dp_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 dp_ld16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}
// a pointer the compiler must treat as wave-uniform (buffer descriptors need SGPRs; a
// VGPR-held base would make every buffer access a waterfall loop)
template <typename T>
__device__ __forceinline__ T* dp_uni(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t* dp_cnt(uint32_t* cnt, int seam, int shard) {
  return cnt + (seam * kDpShards + shard) * kDpShardWords;
}

// ------------------------------------------------------------------ GEMV stages
struct DpStage {
  const bf16_t* W;
  int K, nunits, rstride, bytes;      // bytes: the whole weight (buffer range)
};

template <int EPI>
__device__ __forceinline__ int dp_row0(int U) {
  if constexpr (EPI == kEpRope) return (U >> 6) * 128 + (U & 63);
  else return U;
}

// A wave's items are (unit i, chunk c), units U = gw + i * nwt, walked in order by two
// cursors (issue, consume).  Weight loads are buffer loads over the whole weight (uniform
// descriptor and byte offset, lane * 16 in the VGPR): a group is always 16 load
// instructions -- past the wave's last item the offset leaves the buffer's range, the
// load returns zeros and moves no bytes -- so the compiler's wait counts stay static.
struct DpCur {
  int i, c;
};

constexpr int kDpOob = 0x7ffffff0;      // byte offset past every weight's range

template <int EPI>
__device__ __forceinline__ void dp_issue(u32x4 (&b)[kDpLoads], const DpStage& s, int gw, int nwt,
                                         DpCur& cur, int nu, int nch, int rot, int lane) {
  constexpr int NR = EPI == kEpRes ? 1 : 2;
  constexpr int CU = kDpLoads / NR;
  const __amdgpu_buffer_rsrc_t wr = dp_rsrc(dp_uni(s.W), s.bytes);
  const int rsb = s.rstride * s.K * 2;
#pragma unroll
  for (int t = 0; t < CU; ++t) {
    const bool live = cur.i < nu;
    const int row = dp_row0<EPI>(gw + cur.i * nwt);
    const int ch = cur.c + rot < nch ? cur.c + rot : cur.c + rot - nch;
    // the item's offset rides in the VGPR offset (no per-load SGPR), past the end out of range
    const int off = live ? row * s.K * 2 + ch * 1024 + lane * 16 : kDpOob;
#pragma unroll
    for (int r = 0; r < NR; ++r)
      b[t * NR + r] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, live ? off + r * rsb : kDpOob, 0, kNt));
    if (++cur.c == nch) {
      cur.c = 0;
      ++cur.i;
    }
  }
}

struct DpEpi {
  const DpArgs* a;
  const bf16_t* res_l;      // LDS residual copy [MM][d] (o / down: the add's old value)
  const float* cs_l;        // LDS cos / sin [MM][128]
  bf16_t* kc;
  bf16_t* vc;
  int my_slot;              // lane m < M: token m's KV slot
};

// epilogue of unit U: lanes m < M finish token m (all lanes hold the wave sums)
template <int MM, int EPI>
__device__ __forceinline__ void dp_epilogue(float (&acc)[2][MM], const float (&rs)[MM], int U,
                                            const DpEpi& e, int lane) {
  constexpr int NR = EPI == kEpRes ? 1 : 2;
  const DpArgs& a = *e.a;
  float s[NR][MM];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int m = 0; m < MM; ++m) s[r][m] = wave_sum_dpp(acc[r][m]) * (EPI == kEpRes ? 1.f : rs[m]);
  if (lane >= a.M) return;
  float va = 0.f, vb = 0.f;
#pragma unroll
  for (int m = 0; m < MM; ++m)
    if (lane == m) {
      va = s[0][m];
      vb = s[NR - 1][m];
    }
  const int m = lane;
  if constexpr (EPI == kEpRes) {
    // residual <- bf16(bf16(x . w) + residual)  (gemv_rows.hip kRwResAdd)
    const float old = bf2f(e.res_l[m * a.d + U]);
    const bf16_t nv = f2bf(bf2f(f2bf(va)) + old);
    __builtin_amdgcn_raw_buffer_store_b16(nv, dp_rsrc(a.residual, a.M * a.d * 2),
                                          (m * a.d + U) * 2, 0, kSc1);
  } else if constexpr (EPI == kEpSwi) {
    const float gf = bf2f(f2bf(va));                 // = the gate_up GEMM's bf16 output
    const float sg = gf / (1.f + __expf(-gf));
    const bf16_t o = f2bf(bf2f(f2bf(sg)) * bf2f(f2bf(vb)));
    __builtin_amdgcn_raw_buffer_store_b16(o, dp_rsrc(a.act, a.M * a.F * 2), (m * a.F + U) * 2, 0,
                                          kSc1);
  } else {
    const int h = U >> 6, dd = U & 63;
    float o1 = va, o2 = vb;
    if (h < a.Hq + a.Hkv) {
      const float cc = e.cs_l[m * 128 + dd], ss = e.cs_l[m * 128 + 64 + dd];
      o1 = va * cc - vb * ss;
      o2 = vb * cc + va * ss;
    }
    if (h < a.Hq) {
      const __amdgpu_buffer_rsrc_t qr = dp_rsrc(a.qbuf, a.M * a.ldq * 2);
      const int off = (m * a.ldq + h * 128 + dd) * 2;
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(o1), qr, off, 0, kSc1);
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(o2), qr, off + 128, 0, kSc1);
    } else if (e.my_slot >= 0) {
      const bool is_k = h < a.Hq + a.Hkv;
      const int kvh = is_k ? h - a.Hq : h - a.Hq - a.Hkv;
      // the row differs per lane (token): global sc1 stores with a per-lane address.  A
      // buffer store would need a per-lane descriptor, i.e. a waterfall loop -- and hipcc
      // (ROCm 7.2) reloads the loop's address registers from AGPR spill slots inside it
      // and overwrote the address after the first lane group (illegal access at M >= 2)
      bf16_t* dst = (is_k ? e.kc : e.vc) +
                    (((int64_t)(e.my_slot / a.BS) * a.Hkv + kvh) * a.BS + e.my_slot % a.BS) * 128;
      __hip_atomic_store(dst + dd, f2bf(o1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + 64 + dd, f2bf(o2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// consume one group (held in b): dot products against the LDS input rows, epilogue at
// the end of every unit; `left` = items not yet consumed
template <int MM, int EPI>
__device__ __forceinline__ void dp_consume(const u32x4 (&b)[kDpLoads], float (&acc)[2][MM],
                                           const float (&rs)[MM], const bf16_t* x_l, int K,
                                           int gw, int nwt, DpCur& cur, int& left, int nch,
                                           int rot, const DpEpi& e, int lane) {
  constexpr int NR = EPI == kEpRes ? 1 : 2;
  constexpr int CU = kDpLoads / NR;
#pragma unroll
  for (int t = 0; t < CU; ++t) {
    if (left <= 0) break;                         // wave-uniform
    --left;
    u32x4 x[MM];
    const int ch = cur.c + rot < nch ? cur.c + rot : cur.c + rot - nch;
#pragma unroll
    for (int m = 0; m < MM; ++m)
      x[m] = *reinterpret_cast<const u32x4*>(x_l + m * K + ch * 512 + lane * 8);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int m = 0; m < MM; ++m) acc[r][m] = dot8(b[t * NR + r], x[m], acc[r][m]);
    if (cur.c == nch - 1) {
      dp_epilogue<MM, EPI>(acc, rs, gw + cur.i * nwt, e, lane);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int m = 0; m < MM; ++m) acc[r][m] = 0.f;
      cur.c = 0;
      ++cur.i;
    } else {
      ++cur.c;
    }
  }
}

// units of this wave in a stage of nunits units
__device__ __forceinline__ int dp_units(int nunits, int gw, int nwt) {
  return gw < nunits ? (nunits - gw + nwt - 1) / nwt : 0;
}

// The body of one GEMV stage for this wave, after its input rows are in LDS.  Groups
// rotate through a ring of three 16 KB register buffers: every consume has the two
// younger groups in flight (48 KB per wave, 192 KB per CU), and the consumed buffer is
// refilled with the group three ahead right away.  Every group is 16 loads (out-of-range
// past the end), so the loop is one static body and the compiler's wait counts are exact.
// With `prefetched` the first three groups are already in flight (issued across the
// seam; the issue cursor `ic` then points past them).  normx: scale by
// rsqrt(mean(x^2) + eps) per token (folded RMSNorm, gemv_rows.hip kRwNormX).
template <int MM, int EPI>
__device__ __forceinline__ void dp_gemv(u32x4 (&bA)[kDpLoads], u32x4 (&bB)[kDpLoads],
                                        u32x4 (&bC)[kDpLoads], bool prefetched, DpCur ic,
                                        const DpStage& s, const bf16_t* x_l, bool normx,
                                        float eps, int gw, int nwt, int rot, const DpEpi& e,
                                        int lane) {
  const int nu = dp_units(s.nunits, gw, nwt);
  if (nu == 0) return;
  const int K = s.K, nch = K >> 9;
  constexpr int NR = EPI == kEpRes ? 1 : 2;
  constexpr int CU = kDpLoads / NR;
  const int nitems = nu * nch;
  const int ngroups = (nitems + CU - 1) / CU;
  if (!prefetched) {
    ic = DpCur{0, 0};
    dp_issue<EPI>(bA, s, gw, nwt, ic, nu, nch, rot, lane);
    dp_issue<EPI>(bB, s, gw, nwt, ic, nu, nch, rot, lane);
    dp_issue<EPI>(bC, s, gw, nwt, ic, nu, nch, rot, lane);
  }
  float rs[MM];
#pragma unroll
  for (int m = 0; m < MM; ++m) rs[m] = 1.f;
  if (normx) {
    float ssq[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) ssq[m] = 0.f;
    for (int c = 0; c < nch; ++c)
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const u32x4 x = *reinterpret_cast<const u32x4*>(x_l + m * K + c * 512 + lane * 8);
        ssq[m] = dot8(x, x, ssq[m]);
      }
#pragma unroll
    for (int m = 0; m < MM; ++m) rs[m] = rsqrtf(wave_sum_dpp(ssq[m]) / (float)K + eps);
  }
  float acc[2][MM];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int m = 0; m < MM; ++m) acc[r][m] = 0.f;
  DpCur cc{0, 0};
  int left = nitems;
  for (int g = 0; g < ngroups; g += 3) {
    dp_consume<MM, EPI>(bA, acc, rs, x_l, K, gw, nwt, cc, left, nch, rot, e, lane);
    dp_issue<EPI>(bA, s, gw, nwt, ic, nu, nch, rot, lane);
    dp_consume<MM, EPI>(bB, acc, rs, x_l, K, gw, nwt, cc, left, nch, rot, e, lane);
    dp_issue<EPI>(bB, s, gw, nwt, ic, nu, nch, rot, lane);
    dp_consume<MM, EPI>(bC, acc, rs, x_l, K, gw, nwt, cc, left, nch, rot, e, lane);
    dp_issue<EPI>(bC, s, gw, nwt, ic, nu, nch, rot, lane);
  }
}

// stage the step's rows of up to two sources ([M, n] bf16, row stride ld) into LDS
// [MM][n] with sc1 loads (bytes of this launch), rows past M zero: every load of both is
// issued before the LDS stores, so the staging costs one memory round trip
template <int MM>
__device__ __forceinline__ void dp_stage_rows(bf16_t* dst0, const bf16_t* src0, int ld0, int n0,
                                              bf16_t* dst1, const bf16_t* src1, int ld1, int n1,
                                              int M) {
  constexpr int U = 8;                  // loads in flight per thread before the LDS stores
  const int per0 = n0 >> 3, tot0 = MM * per0;
  const int per1 = n1 >> 3, total = tot0 + MM * per1;
  const __amdgpu_buffer_rsrc_t r0 = dp_rsrc(src0, M * ld0 * 2);
  const __amdgpu_buffer_rsrc_t r1 = dp_rsrc(src1 != nullptr ? src1 : src0,
                                            src1 != nullptr ? M * ld1 * 2 : 0);
  for (int base = threadIdx.x; base < total; base += U * kDpThreads) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * kDpThreads;
      v[u] = (u32x4){0u, 0u, 0u, 0u};
      if (i < tot0) {
        const int m = i / per0, c = i - m * per0;
        if (m < M) v[u] = dp_ld16(r0, (m * ld0 + c * 8) * 2);
      } else if (i < total) {
        const int j = i - tot0, m = j / per1, c = j - m * per1;
        if (m < M) v[u] = dp_ld16(r1, (m * ld1 + c * 8) * 2);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * kDpThreads;
      if (i < tot0) {
        const int m = i / per0, c = i - m * per0;
        *reinterpret_cast<u32x4*>(dst0 + m * n0 + c * 8) = v[u];
      } else if (i < total) {
        const int j = i - tot0, m = j / per1, c = j - m * per1;
        *reinterpret_cast<u32x4*>(dst1 + m * n1 + c * 8) = v[u];
      }
    }
  }
}

// ------------------------------------------------------------------ attention stage
// One (work item w, kv head, split) unit: attn_decode_core.h MODE 0 with one column tile,
// sc1 loads of q / K / V (this launch wrote the new token's q, k, v), a wave-local V tile
// sync, sc1 stores of the partials and of the output (read by the o stage).
__device__ __forceinline__ void dp_wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void dp_attn_unit(const DpArgs& a, const DpLayer& L, int w, int kvh,
                                          int split, bf16_t* __restrict__ v_lds, int lane) {
  const int g = lane >> 4, c = lane & 15;
  const int Hq = a.Hq, Hkv = a.Hkv, G = Hq / Hkv, S = a.splits;
  const int seq = a.work_seq[w];
  if (seq < 0) return;                               // padding work item
  const int ql = a.q_len[seq], kvl = a.kv_len[seq];
  const int tile = a.work_ct[w];
  if (tile * 16 >= ql * G) return;                   // wave-uniform: the whole item is empty
  const int col = tile * 16 + c;
  const bool cvalid = col < ql * G;
  const int qi = cvalid ? col / G : 0;
  const int h = kvh * G + (cvalid ? col % G : 0);
  const int qrow = a.q_start[seq] + qi;
  const int lim = kvl - ql + qi + 1;                 // keys [0, lim) visible
  // pages split, split + S, ... (interleaved, as attn_decode_core.h MODE 0)
  const int32_t* bt = a.block_tables + (int64_t)seq * a.bt_stride;
  int pg_next = bt[__builtin_amdgcn_readfirstlane(min(split, a.bt_stride - 1))];
  const int npg_all = (kvl + kPage - 1) / kPage;
  const int start = split * kPage;
  const int end = kvl;

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) o[m] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (start < end) {
    s16x8 qf[4];
    const __amdgpu_buffer_rsrc_t qr = dp_rsrc(a.qbuf, a.M * a.ldq * 2);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[ks] = __builtin_bit_cast(
          s16x8, dp_ld16(qr, (qrow * a.ldq + h * kD + 32 * ks + 8 * g) * 2));
      if (!cvalid) qf[ks] = (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
    const int pg0 = split;
    const int np = (npg_all - split + S - 1) / S;
    const int pg_last = pg0 + (np - 1) * S;
    bf16_t* const kc = dp_uni(L.kc);
    bf16_t* const vc = dp_uni(L.vc);
    auto fetch = [&](int j, s16x8 (&kf)[2][4], s16x8 (&vr)[8]) {
      const int64_t page = __builtin_amdgcn_readfirstlane(pg_next);
      pg_next = bt[__builtin_amdgcn_readfirstlane(min(pg0 + (j + 1) * S, pg_last))];
      const __amdgpu_buffer_rsrc_t kr = dp_rsrc(kc + ((page * Hkv + kvh) * kPage) * kD, kDpVTile);
      const __amdgpu_buffer_rsrc_t vr_ = dp_rsrc(vc + ((page * Hkv + kvh) * kPage) * kD, kDpVTile);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          kf[mt][ks] = __builtin_bit_cast(
              s16x8, dp_ld16(kr, ((16 * mt + c) * kD + 32 * ks + 8 * g) * 2));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        vr[i] = __builtin_bit_cast(s16x8, dp_ld16(vr_, ((g + 4 * i) * kD + 8 * c) * 2));
    };
    auto process = [&](int j, const s16x8 (&kf)[2][4], const s16x8 (&vr)[8]) {
      const int kt = start + j * S * kPage;
      const int nvalid = end - kt;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = g + 4 * i, ch = c;
        const s16x8 v = row >= nvalid ? (s16x8){0, 0, 0, 0, 0, 0, 0, 0} : vr[i];
        const int pch = ch ^ ((row & 7) << 1);
        reinterpret_cast<s16x8*>(v_lds + row * kD)[pch] = v;
      }
      f32x4 s[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        s[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(kf[mt][ks]), as_bf16x8(qf[ks]),
                                                          s[mt], 0, 0, 0);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = 16 * mt + 4 * g + i;
          float v = s[mt][i] * a.scale_log2;
          if (key >= nvalid || kt + key >= lim) v = -INFINITY;
          s[mt][i] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = fast_exp2(m_run - m_use);
      float psum = 0.f;
      float p[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        p[jj] = fast_exp2(s[jj >> 2][jj & 3] - m_use);
        psum += p[jj];
      }
      l_run = l_run * alpha + psum;
      m_run = m_new;
#pragma unroll
      for (int m = 0; m < 8; ++m) o[m] *= alpha;
      const s16x8 pb = pack8(p);
      dp_wave_lds_sync();                              // V tile visible to the wave
      const int q4 = c >> 2, p4 = c & 3;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int r0 = 4 * g + q4, r1 = 16 + 4 * g + q4;
        const int ch = 2 * m + (p4 >> 1), sub = (p4 & 1) * 4;
        const s16x4 a0 = ds_read_tr16(v_lds + r0 * kD + ((ch ^ ((r0 & 7) << 1)) * 8) + sub);
        const s16x4 a1 = ds_read_tr16(v_lds + r1 * kD + ((ch ^ ((r1 & 7) << 1)) * 8) + sub);
        const s16x8 av = (s16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        o[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(av), as_bf16x8(pb), o[m], 0, 0, 0);
      }
      dp_wave_lds_sync();                              // before the next tile overwrites it
    };
    // page j + 1's K / V loads are issued before page j is processed (two register sets):
    // a split walking several pages pays one memory round trip, not one per page
    constexpr int kVmcnt0 = 0x0F70;          // vmcnt(0), expcnt / lgkmcnt untouched
    s16x8 kA[2][4], vA[8], kB[2][4], vB[8];
    fetch(0, kA, vA);
    for (int j = 0; j < np; j += 2) {
      __builtin_amdgcn_s_waitcnt(kVmcnt0);
      if (j + 1 < np) fetch(j + 1, kB, vB);
      process(j, kA, vA);
      if (j + 1 >= np) break;
      __builtin_amdgcn_s_waitcnt(kVmcnt0);
      if (j + 2 < np) fetch(j + 2, kA, vA);
      process(j + 1, kB, vB);
    }
  }

  float l_tot = l_run;
  l_tot += __shfl_xor(l_tot, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  const int ldo = Hq * kD;
  const __amdgpu_buffer_rsrc_t outr = dp_rsrc(a.attn, a.M * ldo * 2);
  if (S == 1) {
    if (!cvalid) return;
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const uint32_t w0 = pack_bf16x2(o[m][0] * inv, o[m][1] * inv);
      const uint32_t w1 = pack_bf16x2(o[m][2] * inv, o[m][3] * inv);
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(
          (u32x2){w0, w1}, outr, (qrow * ldo + h * kD + 16 * m + 4 * g) * 2, 0, kSc1);
    }
    return;
  }
  if (cvalid) {
    const int64_t pidx = ((int64_t)qrow * Hq + h) * S + split;
    float* po = a.part_o + pidx * kD;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      gu64* dq = (gu64*)(po + 16 * m + 4 * g);
      __hip_atomic_store(dq, pack_f2(o[m][0], o[m][1]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dq + 1, pack_f2(o[m][2], o[m][3]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (g == 0)
      __hip_atomic_store((gu64*)(a.part_ml + pidx * 2), pack_f2(m_run, l_tot), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // single-pass merge: the last split of (w, kvh) merges (attn_decode_core.h protocol)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  gu32* tk = (gu32*)(a.tickets + (int64_t)w * Hkv + kvh);
  unsigned prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __builtin_amdgcn_readfirstlane(prev);   // uniform: the merge branch is scalar
  if (prev != (unsigned)S - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every handed-off load is sc1
  if (lane == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int mj = lane & 15, mq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int cc = 4 * r + mq;
    const int v_cc = __shfl((int)cvalid, cc, 64);
    const int q_cc = __shfl(qrow, cc, 64), h_cc = __shfl(h, cc, 64);
    if (!__builtin_amdgcn_ballot_w64(v_cc != 0)) continue;
    const int64_t pbase = ((int64_t)q_cc * Hq + h_cc) * S;
    const bool live = v_cc != 0;
    unsigned long long mlx = 0xff800000ull;
    if (live && mj < S)
      mlx = __hip_atomic_load((const gu64*)(a.part_ml + (pbase + mj) * 2), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    const float m_j = __uint_as_float((unsigned)mlx), l_j = __uint_as_float((unsigned)(mlx >> 32));
    float gm = m_j;
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) gm = fmaxf(gm, __shfl_xor(gm, o2, 64));
    const float w_j = (gm == -INFINITY || m_j == -INFINITY) ? 0.f : fast_exp2(m_j - gm);
    float den = w_j * l_j;
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) den += __shfl_xor(den, o2, 64);
    f32x4 num[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
    // the splits' partial rows in two batches of 8 (every load of a batch in flight)
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      f32x4 pv[8][2];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int sp = hb * 8 + q;
        if (live && sp < S) {
          const gu64* dq = (const gu64*)(a.part_o + (pbase + sp) * kD + 8 * mj);
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const unsigned long long x0 =
                __hip_atomic_load(dq + 2 * u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long x1 =
                __hip_atomic_load(dq + 2 * u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pv[q][u] = (f32x4){__uint_as_float((unsigned)x0), __uint_as_float((unsigned)(x0 >> 32)),
                               __uint_as_float((unsigned)x1), __uint_as_float((unsigned)(x1 >> 32))};
          }
        } else {
          pv[q][0] = pv[q][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float wsp = __shfl(w_j, (lane & 48) | (hb * 8 + q), 64);
#pragma unroll
        for (int u = 0; u < 2; ++u) num[u] += wsp * pv[q][u];
      }
    }
    if (!live) continue;
    const float inv = den > 0.f ? 1.f / den : 0.f;
    u32x4 ov;
    ov[0] = pack_bf16x2(num[0][0] * inv, num[0][1] * inv);
    ov[1] = pack_bf16x2(num[0][2] * inv, num[0][3] * inv);
    ov[2] = pack_bf16x2(num[1][0] * inv, num[1][1] * inv);
    ov[3] = pack_bf16x2(num[1][2] * inv, num[1][3] * inv);
    __builtin_amdgcn_raw_buffer_store_b128(ov, outr, (q_cc * ldo + h_cc * kD + 8 * mj) * 2, 0,
                                           kSc1);
  }
}

// ------------------------------------------------------------------ the kernel
__device__ __forceinline__ DpStage dp_desc(const DpArgs& a, const DpLayer& L, int st) {
  const int nq = (a.Hq + 2 * a.Hkv) * 128;
  switch (st) {
    case kDpQkv: return DpStage{L.wqkv, a.d, nq / 2, 64, nq * a.d * 2};
    case kDpO: return DpStage{L.wo, a.Hq * kD, a.d, 0, a.d * a.Hq * kD * 2};
    case kDpGu: return DpStage{L.wgu, a.d, a.F, a.F, 2 * a.F * a.d * 2};
    default: return DpStage{L.wd, a.F, a.d, 0, a.d * a.F * 2};
  }
}

// seam k, arrive: every wave drains its stores, adds 1 to the workgroup's LDS count of
// the seam (parity slot), and the wave whose add completes the count adds 1 to the
// workgroup's shard of the seam's global counter (Guideline 16: each wave's own vmcnt(0)
// wait precedes its LDS add; the signalling wave's add follows all of them).  No barrier:
// a wave goes straight on to its next stage's prefetch.
__device__ __forceinline__ void dp_arrive(const DpArgs& a, int k, int* ctl, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    const int prev = atomicAdd(&ctl[2 + (k & 1)], 1);
    if (prev == kDpWaves - 1) {
      ctl[2 + (k & 1)] = 0;      // reused at seam k + 2, after every wave passed wait(k + 1)
      __hip_atomic_fetch_add(dp_cnt(a.cnt, k, blockIdx.x & (kDpShards - 1)), 1u,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// seam k, wait: wave 0 polls the 8 shards (sc1) until they sum to the grid, bounded; a
// barrier releases the workgroup.  Returns the launch's abort state.
__device__ __forceinline__ bool dp_wait(const DpArgs& a, int k, int l, int st, int* ctl,
                                     uint32_t* abort_w, int wave, int lane) {
  if (wave == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t nwg = gridDim.x;
    for (;;) {
      uint32_t v = 0;
      if (lane < kDpShards)
        v = __hip_atomic_load(dp_cnt(a.cnt, k, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (lane == kDpShards)
        v = __hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t ab = __builtin_amdgcn_readfirstlane(__shfl(v, kDpShards, 64));
      uint32_t tot = lane < kDpShards ? v : 0u;
#pragma unroll
      for (int o2 = 1; o2 < kDpShards; o2 <<= 1) tot += __shfl_xor(tot, o2, 64);
      tot = __builtin_amdgcn_readfirstlane(tot);
      if (ab != 0) {
        if (lane == 0) ctl[0] = 1;
        break;
      }
      if (tot >= nwg) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
        if (lane == 0) {
          report_error(a.err, kErrPersist);
          uint32_t zero = 0;
          if (a.err != nullptr)
            __hip_atomic_compare_exchange_strong(a.err + kErrPersistInfo, &zero,
                                                 (uint32_t)((l << 8) | st) + 1u, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ctl[0] = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(ctl[0]) != 0;
}

template <int MM, int EPI>
__device__ __forceinline__ bool dp_gemv_stage(const DpArgs& a, const DpLayer& L, int st, int k,
                                              int l, bool aborted, bool after_attn, int* ctl,
                                              uint32_t* abort_w,
                                              bf16_t* res_l, bf16_t* x_l, const DpEpi& e,
                                              int wave, int gw, int nwt, int lane) {
  const DpStage s = dp_desc(a, L, st);
  u32x4 bA[kDpLoads], bB[kDpLoads], bC[kDpLoads];
  bool pre = false;
  DpCur ic{0, 0};
  const int nu = dp_units(s.nunits, gw, nwt);
  // flags bit 3: each wave starts its rows at chunk gw % nch (rotating), so the waves of a
  // stage do not all read the same 1 KB column of their rows at once after a seam
  const int rot = (a.flags & 8) ? gw % (s.K >> 9) : 0;
  // the first three groups' weight loads go out before the seam settles (wave 0 polls
  // first, except behind the attention or with flags bit 0)
  if (!aborted && nu > 0 && !(a.flags & 2) && (wave != 0 || after_attn || (a.flags & 1))) {
    const int nch = s.K >> 9;
    dp_issue<EPI>(bA, s, gw, nwt, ic, nu, nch, rot, lane);
    dp_issue<EPI>(bB, s, gw, nwt, ic, nu, nch, rot, lane);
    dp_issue<EPI>(bC, s, gw, nwt, ic, nu, nch, rot, lane);
    pre = true;
  }
  if (k > 0) aborted = dp_wait(a, k - 1, l, st, ctl, abort_w, wave, lane);
  if (aborted) return true;
  // the input rows (and, for o / down, the residual the epilogue adds to) into LDS
  if (st == kDpO)
    dp_stage_rows<MM>(res_l, a.residual, a.d, a.d, x_l, a.attn, a.Hq * kD, a.Hq * kD, a.M);
  else if (st == kDpDown)
    dp_stage_rows<MM>(res_l, a.residual, a.d, a.d, x_l, a.act, a.F, a.F, a.M);
  else
    dp_stage_rows<MM>(res_l, a.residual, a.d, a.d, nullptr, nullptr, 0, 0, a.M);
  __syncthreads();
  const bool nx = EPI != kEpRes;
  dp_gemv<MM, EPI>(bA, bB, bC, pre, ic, s, nx ? res_l : x_l, nx, a.eps, gw, nwt, rot, e, lane);
  return false;
}

template <int MM>
__global__ __launch_bounds__(kDpThreads, 1) void decode_persist_kernel(DpArgs a) {
  extern __shared__ __attribute__((aligned(16))) char dp_smem[];
  float* cs_l = reinterpret_cast<float*>(dp_smem);
  int* ctl = reinterpret_cast<int*>(dp_smem + kDpCsBytes);
  bf16_t* res_l = reinterpret_cast<bf16_t*>(dp_smem + kDpCsBytes + kDpCtlBytes);
  bf16_t* x_l = res_l + MM * a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, nwt = kDpWaves * nwg;
  const int gw = wave * nwg + blockIdx.x;

  // per-launch constants: cos / sin rows of the step's tokens, each lane's token slot
  for (int i = tid; i < MM * 128; i += kDpThreads) {
    const int m = i >> 7;
    cs_l[i] = m < a.M ? a.cos_sin[(int64_t)a.positions[m] * 128 + (i & 127)] : 0.f;
  }
  if (tid < 4) ctl[tid] = 0;
  const int my_slot = lane < a.M ? a.slots[lane] : -1;
  int nper = 0;
  for (int st = 0; st < kDpStages; ++st) nper += (a.stages >> st) & 1;
  const int nst = (a.l1 - a.l0) * nper;          // executed stages; seams = nst - 1
  uint32_t* abort_w = a.cnt + (nst > 1 ? nst - 1 : 0) * kDpShards * kDpShardWords;
  uint32_t* exit_w = abort_w + kDpShardWords;
  __syncthreads();

  bool aborted = false, prev_attn = false;
  int k = 0;
  for (int l = a.l0; l < a.l1; ++l) {
    const DpLayer L = a.layers[l];
    const DpEpi e{&a, res_l, cs_l, L.kc, L.vc, my_slot};
    for (int st = 0; st < kDpStages; ++st) {
      if (!((a.stages >> st) & 1)) continue;
      if (st == kDpAttn) {
        if (k > 0) aborted = dp_wait(a, k - 1, l, st, ctl, abort_w, wave, lane);
        if (!aborted && !(a.flags & 4)) {
          // units (w, kvh, split) on wave slots; the V tiles reuse the LDS rows
          const int nu = a.W * a.Hkv * a.splits;
          bf16_t* v_lds = res_l + wave * (kDpVTile / 2);
          for (int u = gw; u < nu; u += nwt) {
            const int split = u % a.splits, rest = u / a.splits;
            dp_attn_unit(a, L, rest / a.Hkv, rest % a.Hkv, split, v_lds, lane);
          }
        }
      } else if (st == kDpQkv) {
        aborted = dp_gemv_stage<MM, kEpRope>(a, L, st, k, l, aborted, prev_attn, ctl, abort_w, res_l, x_l, e,
                                             wave, gw, nwt, lane);
      } else if (st == kDpGu) {
        aborted = dp_gemv_stage<MM, kEpSwi>(a, L, st, k, l, aborted, prev_attn, ctl, abort_w, res_l, x_l, e,
                                            wave, gw, nwt, lane);
      } else {
        aborted = dp_gemv_stage<MM, kEpRes>(a, L, st, k, l, aborted, prev_attn, ctl, abort_w, res_l, x_l, e,
                                            wave, gw, nwt, lane);
      }
      if (k + 1 < nst) dp_arrive(a, k, ctl, lane);
      prev_attn = st == kDpAttn;
      ++k;
    }
  }

  // ---- exit: the last workgroup out zeroes this launch's counters for the next launch
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(exit_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ctl[1] = prev == (unsigned)nwg - 1;
  }
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(ctl[1])) {
    const int nseam = nst > 1 ? nst - 1 : 0;
    for (int i = tid; i < nseam * kDpShards; i += kDpThreads)
      __hip_atomic_store(a.cnt + i * kDpShardWords, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) {
      __hip_atomic_store(abort_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(exit_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ================================================================== engine form
// flags bit 4 (RFQ_PERSIST=engine), M <= 2.  The same chain and seams, with the weight
// stream moved off the computing waves (MI355X_MICROARCH.md 'engine-vs-launches',
// 'ldsdma-fill', 'prefetch-credit'): per CU wave 0 is a LOADER that only issues LDS-DMA
// (buffer_load ... lds, nt) of the CU's weight pieces into a ring of 16 KB slots, and
// waves 1-3 are CONSUMERS that take the slots round-robin, run the attention units and
// the stage epilogues.  The loader never waits on a seam: it walks the launch's weight
// sequence (every layer's qkv, o, gate|up, down rows of this CU, in stage order) and
// stalls only on a full ring, so during every seam and during the attention the ring
// fills with the next stage's weights (o's whole 33.5 MB at 8B fits the chip's rings).
//
// Stream of a stage: the CU's units U = cu + i * CUs (qkv: a rotate-half row pair, gate|up:
// gate row U and up row F + U, o / down: row U), each row as K / 512 pieces of 1 KB
// (64 lanes x 16 B, a piece never straddles rows since K % 512 == 0); slot j holds pieces
// 16 j .. 16 j + 15 of the CU's stage stream.  Hand-offs inside the CU are LDS words:
// FULL[slot] = sequence number (loader, after the counted vmcnt that lands it; at most
// kEgDepth slots in flight), DONE[slot] = sequence number (consumer, once the slot is in
// its registers).  A consumer reduces each row segment of a slot (DPP wave sum) into
// parts[row][segment] (deterministic: no float atomics); the consumer that takes the
// stage's last slot (an LDS count) sums the segments in order, runs the epilogue (RoPE +
// q / KV stores, SwiGLU, residual add) for all of the CU's units and arrives at the seam.
// Seams: consumer 1 polls the global shards (the GEMV form's protocol) and releases the
// others through an LDS word; the loader is not part of any barrier.
constexpr int kEgFlag = 16;
constexpr int kEgCons = 3;                // consumer waves (1..3); wave 0 loads
constexpr int kEgSlot = 16384;            // ring slot: 16 pieces of 1 KB
constexpr int kEgDepth = 4;               // slots in flight per loader
constexpr int kEgSegs = 3;                // ring slots one row can span (K <= 16.5 K)
constexpr int kEgCtlBytes = 256;
enum { kEgFull = 0, kEgDone = 8, kEgRel = 16, kEgAb = 17, kEgCons_ = 18, kEgStg = 19,
       kEgAtt = 20, kEgExit = 21 };

typedef __attribute__((address_space(3))) char eg_lds_c;
typedef volatile __attribute__((address_space(3))) int eg_ctl_t;   // LDS control words
typedef const __attribute__((address_space(3))) u32x4 eg_lds_v4;

struct EgStage {
  const bf16_t* W;
  int K, ppr, rpu, n_cu, u0, P, S, bytes, Kin;
};

__device__ __forceinline__ EgStage eg_stage(const DpArgs& a, const DpLayer& L, int st, int cu,
                                            int nwg) {
  EgStage s;
  const int nq = (a.Hq + 2 * a.Hkv) * 128;
  int nunits;
  switch (st) {
    case kDpQkv: s.W = L.wqkv; s.K = a.d; nunits = nq / 2; s.rpu = 2; s.bytes = nq * a.d * 2; break;
    case kDpO: s.W = L.wo; s.K = a.Hq * kD; nunits = a.d; s.rpu = 1; s.bytes = a.d * s.K * 2; break;
    case kDpGu: s.W = L.wgu; s.K = a.d; nunits = a.F; s.rpu = 2; s.bytes = 2 * a.F * a.d * 2; break;
    default: s.W = L.wd; s.K = a.F; nunits = a.d; s.rpu = 1; s.bytes = a.d * a.F * 2; break;
  }
  s.Kin = s.K;
  // a contiguous block of units per CU (units u0 .. u0 + n_cu - 1): the CU's rows share
  // pages, where a unit stride of CUs put every row of a CU 2 MB from the last (one TLB
  // walk per row; the stream measured ~18 GB/s per CU)
  const int base = nunits / nwg, rem = nunits - base * nwg;
  s.n_cu = base + (cu < rem ? 1 : 0);
  s.u0 = cu * base + (cu < rem ? cu : rem);
  s.ppr = s.K >> 9;
  s.P = s.n_cu * s.rpu * s.ppr;
  s.S = (s.P + 15) >> 4;
  return s;
}

// weight row of the CU's unit U, row r of the unit
__device__ __forceinline__ int eg_row(const DpArgs& a, int st, int U, int r) {
  if (st == kDpQkv) return (U >> 6) * 128 + (U & 63) + r * 64;
  if (st == kDpGu) return U + r * a.F;
  return U;
}

__device__ __forceinline__ eg_ctl_t* eg_ctl(char* smem) {
  return (eg_ctl_t*)(smem + kDpCsBytes);
}
// a control word read as a wave-uniform value: without the readfirstlane the compiler
// treats every branch on an LDS-loaded word as divergent, and everything after it (loop
// cursors, slot indices, the LDS-DMA destination in M0) moves to VGPRs with exec-masked
// control flow -- the loader then took ~1 µs per slot with no loads at all
__device__ __forceinline__ int eg_ld(eg_ctl_t* ctl, int i) {
  return __builtin_amdgcn_readfirstlane(ctl[i]);
}
__device__ __forceinline__ int eg_lds_add(eg_ctl_t* ctl, int i) {
  return __atomic_fetch_add((__attribute__((address_space(3))) int*)(ctl + i), 1,
                            __ATOMIC_RELAXED);
}

// bounded LDS spin: true once `ok()` holds, false on the abort word or after 1 s (which
// raises the abort word and counts kErrPersist).  A tight LDS poll: the clock (an SMEM
// round trip) and the abort word are read every 256 polls only -- a sleep or a clock read
// per poll made every ring hand-off cost ~0.3 µs.
template <typename F>
__device__ __forceinline__ bool eg_spin(const DpArgs& a, eg_ctl_t* ctl, F ok) {
  if (ok()) return true;
  uint64_t t0 = 0;
  for (int it = 1;; ++it) {
    if (ok()) return true;
    if (a.flags & 512) __builtin_amdgcn_s_sleep(1);   // A/B: sleeping pollers
    if ((it & 255) == 0) {
      if (eg_ld(ctl, kEgAb)) return false;
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      if (t0 == 0) {
        t0 = t;
      } else if (t - t0 > kSpinTicks) {
        report_error(a.err, kErrPersist);
        ctl[kEgAb] = 1;
        return false;
      }
    }
  }
}

// flags bit 8 (diagnostic): CU 0 writes s_memrealtime stamps (100 MHz) into part_ml viewed
// as uint64 [512]: 0-3 wave start, 4-7 wave end, 8-10 consumer after staging, 12-14 after
// rs, 16 epilogue start, 17 epilogue end, 64 + n loader starts issuing slot n (n < 64),
// 256 + n its 16 loads issued, 128 + n slot n published, 192 + n consumer saw it full
__device__ __forceinline__ void eg_stamp(const DpArgs& a, int i, int lane) {
  if ((a.flags & 256) && blockIdx.x == 0 && lane == 0 && i < 512)
    reinterpret_cast<uint64_t*>(a.part_ml)[i] = __builtin_amdgcn_s_memrealtime();
}
// the shader clock counter next to the real-time one (clock = d memtime / d realtime)
__device__ __forceinline__ void eg_stamp_clk(const DpArgs& a, int i, int lane) {
  if ((a.flags & 256) && blockIdx.x == 0 && lane == 0) {
    reinterpret_cast<uint64_t*>(a.part_ml)[i] = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<uint64_t*>(a.part_ml)[i + 1] = __builtin_amdgcn_s_memtime();
  }
}

// ---- loaders (waves 0 .. NL-1): loader li issues the slots n with n % NL == li and
// publishes them; every loader walks the whole piece sequence to keep its cursor
template <int NL>
__device__ void eg_loader(const DpArgs& a, char* smem, int li, int lane) {
  eg_ctl_t* ctl = eg_ctl(smem);
  eg_lds_c* const ring = (eg_lds_c*)(smem + a.eg_ring_off);
  const int R = a.eg_ring, cu = blockIdx.x, nwg = gridDim.x;
  const int vl = lane * 16;
  int n = 0, idx = 0;                   // global slot sequence, n % R
  int pub = li, pidx = li, last = li - NL;   // next own slot to publish (and % R), last issued
  auto publish_upto = [&](int upto) {
    for (; pub <= upto; pub += NL) {
      ctl[kEgFull + pidx] = pub;
      if (pub < 64) eg_stamp(a, 128 + pub, lane);
      pidx += NL;
      if (pidx >= R) pidx -= R;
    }
  };
  for (int l = a.l0; l < a.l1; ++l) {
    const DpLayer L = a.layers[l];
    for (int st = 0; st < kDpStages; ++st) {
      if (!((a.stages >> st) & 1) || st == kDpAttn) continue;
      const EgStage s = eg_stage(a, L, st, cu, nwg);
      const __amdgpu_buffer_rsrc_t wr = dp_rsrc(dp_uni(s.W), s.bytes);
      const int nrows = s.n_cu * s.rpu, rsb = s.K * 2;
      // piece cursor: byte offset of the next piece and pieces left in its row; past the
      // stage's rows the offset is 0 (the weight's first KB, loaded and never consumed)
      int ri = 0;
      int so = nrows > 0 ? eg_row(a, st, s.u0, 0) * rsb : 0;
      int left = nrows > 0 ? s.ppr : 1 << 30;
      auto next_row = [&]() {
        ++ri;
        if (ri < nrows) {
          so = (s.rpu == 2 ? eg_row(a, st, s.u0 + (ri >> 1), ri & 1)
                           : eg_row(a, st, s.u0 + ri, 0)) * rsb;
          left = s.ppr;
        } else {
          so = 0;
          left = 1 << 30;
        }
      };
      for (int j = 0; j < s.S; ++j) {
        const bool own = NL == 1 || (n % NL) == li;
        if (own && !(a.flags & 64)) {   // 64: timing, no weight stream
          if (n >= R && eg_ld(ctl, kEgDone + idx) < n - R) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            publish_upto(last);         // consumers may be waiting on landed slots
            const int need = n - R, ix = idx;
            if (!eg_spin(a, ctl, [&]() { return eg_ld(ctl, kEgDone + ix) >= need; })) return;
          }
          eg_lds_c* const dst = ring + idx * kEgSlot;
          if (n < 64) eg_stamp(a, 64 + n, lane);
#pragma unroll
          for (int p = 0; p < 16; ++p) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)(dst + p * 1024), 16, vl,
                                                     so, 0, kNt);
            so += 1024;
            if (--left == 0) next_row();
          }
          if (n < 64) eg_stamp(a, 256 + n, lane);
        } else {
          if (own && n >= R && eg_ld(ctl, kEgDone + idx) < n - R) {
            publish_upto(last);
            const int need = n - R, ix = idx;
            if (!eg_spin(a, ctl, [&]() { return eg_ld(ctl, kEgDone + ix) >= need; })) return;
          }
          for (int adv = 16; adv > 0;) {     // another loader's slot: move the cursor only
            const int t = adv < left ? adv : left;
            so += t * 1024;
            left -= t;
            adv -= t;
            if (left == 0) next_row();
          }
        }
        if (own) {
          last = n;
          if (last - pub >= (kEgDepth - 1) * NL) {
            // all but this loader's youngest kEgDepth - 1 slots (16 loads each) have landed
            asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
            publish_upto(last - (kEgDepth - 1) * NL);
          }
        }
        ++n;
        if (++idx == R) idx = 0;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  publish_upto(last);
}

// ---- consumers (waves 1..3): seam wait.  Consumer 0 polls the global shards (bounded, as
// dp_wait) and releases the others through ctl[kEgRel]; returns the abort state.
__device__ bool eg_wait(const DpArgs& a, int k, int l, int st, eg_ctl_t* ctl,
                        uint32_t* abort_w, int c, int lane) {
  if (c == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t nwg = gridDim.x;
    for (;;) {
      uint32_t v = 0;
      if (lane < kDpShards)
        v = __hip_atomic_load(dp_cnt(a.cnt, k, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (lane == kDpShards)
        v = __hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t ab = __builtin_amdgcn_readfirstlane(__shfl(v, kDpShards, 64));
      uint32_t tot = lane < kDpShards ? v : 0u;
#pragma unroll
      for (int o2 = 1; o2 < kDpShards; o2 <<= 1) tot += __shfl_xor(tot, o2, 64);
      tot = __builtin_amdgcn_readfirstlane(tot);
      if (ab != 0 || eg_ld(ctl, kEgAb)) {
        if (lane == 0) ctl[kEgAb] = 1;
        break;
      }
      if (tot >= nwg) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
        if (lane == 0) {
          report_error(a.err, kErrPersist);
          uint32_t zero = 0;
          if (a.err != nullptr)
            __hip_atomic_compare_exchange_strong(a.err + kErrPersistInfo, &zero,
                                                 (uint32_t)((l << 8) | st) + 1u, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ctl[kEgAb] = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) ctl[kEgRel] = k + 1;
    return eg_ld(ctl, kEgAb) != 0;
  }
  eg_spin(a, ctl, [&]() { return eg_ld(ctl, kEgRel) >= k + 1; });
  return eg_ld(ctl, kEgAb) != 0;
}

// the arriving wave's stores are drained (vmcnt(0)) before its add: Guideline 16
__device__ __forceinline__ void eg_arrive_global(const DpArgs& a, int k, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    __hip_atomic_fetch_add(dp_cnt(a.cnt, k, blockIdx.x & (kDpShards - 1)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// the stage's input rows (and the residual the o / down epilogue adds to) into LDS by the
// three consumers (every load of a thread in flight before its LDS stores), then an LDS
// count over the consumers (monotonic: stage ordinal sn)
template <int MM, int NC>
__device__ void eg_stage_inputs(const DpArgs& a, int st, bf16_t* res_l, bf16_t* x_l, int c,
                                int lane, eg_ctl_t* ctl, int sn) {
  const bf16_t* src1 = st == kDpO ? a.attn : st == kDpDown ? a.act : nullptr;
  const int n1 = st == kDpO ? a.Hq * kD : a.F;
  const int per0 = a.d >> 3, tot0 = MM * per0;
  const int per1 = n1 >> 3, total = tot0 + (src1 != nullptr ? MM * per1 : 0);
  const __amdgpu_buffer_rsrc_t r0 = dp_rsrc(a.residual, a.M * a.d * 2);
  const __amdgpu_buffer_rsrc_t r1 = dp_rsrc(src1 != nullptr ? src1 : a.residual,
                                            src1 != nullptr ? a.M * n1 * 2 : 0);
  constexpr int U = 8, NT = NC * 64;
  for (int base = c * 64 + lane; base < total; base += U * NT) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * NT;
      v[u] = (u32x4){0u, 0u, 0u, 0u};
      if (i < tot0) {
        const int m = i / per0, cc = i - m * per0;
        if (m < a.M) v[u] = dp_ld16(r0, (m * a.d + cc * 8) * 2);
      } else if (i < total) {
        const int jj = i - tot0, m = jj / per1, cc = jj - m * per1;
        if (m < a.M) v[u] = dp_ld16(r1, (m * n1 + cc * 8) * 2);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * NT;
      if (i < tot0) {
        const int m = i / per0, cc = i - m * per0;
        *reinterpret_cast<u32x4*>(res_l + m * a.d + cc * 8) = v[u];
      } else if (i < total) {
        const int jj = i - tot0, m = jj / per1, cc = jj - m * per1;
        *reinterpret_cast<u32x4*>(x_l + m * n1 + cc * 8) = v[u];
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) eg_lds_add(ctl, kEgStg);
  eg_spin(a, ctl, [&]() { return eg_ld(ctl, kEgStg) >= NC * (sn + 1); });
}

// epilogue of the CU's units of a GEMV stage (one consumer wave; lanes over (unit, token))
template <int MM>
__device__ void eg_epilogue(const DpArgs& a, const DpLayer& L, int st, const EgStage& s,
                            const float* parts_l, const bf16_t* res_l, const float* cs_l,
                            const float (&rs)[MM], int lane) {
  const int cu = blockIdx.x, nwg = gridDim.x;
  for (int t = lane; t < s.n_cu * MM; t += 64) {
    const int i = t / MM, m = t - i * MM;
    if (m >= a.M) continue;
    float v[2] = {0.f, 0.f};
    for (int r = 0; r < s.rpu; ++r) {
      const int ri = i * s.rpu + r;
      const int f = (ri * s.ppr) >> 4, e = (ri * s.ppr + s.ppr - 1) >> 4;
      float sum = 0.f;
      for (int sg = 0; sg <= e - f; ++sg) sum += parts_l[(ri * kEgSegs + sg) * MM + m];
      v[r] = sum;
    }
    float rsm = 1.f;
#pragma unroll
    for (int q = 0; q < MM; ++q)
      if (q == m) rsm = rs[q];
    const int U = s.u0 + i;
    if (st == kDpO || st == kDpDown) {
      // residual <- bf16(bf16(x . w) + residual)  (gemv_rows.hip kRwResAdd)
      const float old = bf2f(res_l[m * a.d + U]);
      const bf16_t nv = f2bf(bf2f(f2bf(v[0])) + old);
      __builtin_amdgcn_raw_buffer_store_b16(nv, dp_rsrc(a.residual, a.M * a.d * 2),
                                            (m * a.d + U) * 2, 0, kSc1);
    } else if (st == kDpGu) {
      const float gf = bf2f(f2bf(v[0] * rsm));
      const float sg = gf / (1.f + __expf(-gf));
      const bf16_t o = f2bf(bf2f(f2bf(sg)) * bf2f(f2bf(v[1] * rsm)));
      __builtin_amdgcn_raw_buffer_store_b16(o, dp_rsrc(a.act, a.M * a.F * 2), (m * a.F + U) * 2, 0,
                                            kSc1);
    } else {
      const float va = v[0] * rsm, vb = v[1] * rsm;
      const int h = U >> 6, dd = U & 63;
      float o1 = va, o2 = vb;
      if (h < a.Hq + a.Hkv) {
        const float cc = cs_l[m * 128 + dd], ss = cs_l[m * 128 + 64 + dd];
        o1 = va * cc - vb * ss;
        o2 = vb * cc + va * ss;
      }
      if (h < a.Hq) {
        const __amdgpu_buffer_rsrc_t qr = dp_rsrc(a.qbuf, a.M * a.ldq * 2);
        const int off = (m * a.ldq + h * 128 + dd) * 2;
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(o1), qr, off, 0, kSc1);
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(o2), qr, off + 128, 0, kSc1);
      } else {
        const int slot = a.slots[m];
        if (slot >= 0) {
          const bool is_k = h < a.Hq + a.Hkv;
          const int kvh = is_k ? h - a.Hq : h - a.Hq - a.Hkv;
          // per-lane global sc1 stores (see dp_epilogue: no per-lane buffer descriptor)
          bf16_t* dst = (is_k ? L.kc : L.vc) +
                        (((int64_t)(slot / a.BS) * a.Hkv + kvh) * a.BS + slot % a.BS) * 128;
          __hip_atomic_store(dst + dd, f2bf(o1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(dst + 64 + dd, f2bf(o2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

// one slot: 16 pieces, partial dot products per row segment into parts_l
template <int MM>
__device__ __forceinline__ void eg_consume_slot(const eg_lds_c* sl, const EgStage& s, int j,
                                                const bf16_t* x_in, float* parts_l,
                                                eg_ctl_t* ctl, int idx, int seq, int lane) {
  u32x4 w[16];
#pragma unroll
  for (int p = 0; p < 16; ++p)
    w[p] = *(eg_lds_v4*)(sl + p * 1024 + lane * 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) ctl[kEgDone + idx] = seq;       // the slot's bytes are in registers
  const int q0 = j * 16;
  int row = q0 / s.ppr, kp = q0 - row * s.ppr;
  int seg = j - ((row * s.ppr) >> 4);
  float acc[MM];
#pragma unroll
  for (int m = 0; m < MM; ++m) acc[m] = 0.f;
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    if (q0 + p < s.P) {                          // wave-uniform
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const u32x4 x = *reinterpret_cast<const u32x4*>(x_in + m * s.Kin + kp * 512 + lane * 8);
        acc[m] = dot8(w[p], x, acc[m]);
      }
      const bool row_end = kp == s.ppr - 1;
      if (row_end || p == 15 || q0 + p + 1 == s.P) {
#pragma unroll
        for (int m = 0; m < MM; ++m) {
          const float t = wave_sum_dpp(acc[m]);
          if (lane == 0) parts_l[(row * kEgSegs + seg) * MM + m] = t;
          acc[m] = 0.f;
        }
      }
      if (row_end) {
        kp = 0;
        ++row;
        seg = j - ((row * s.ppr) >> 4);
      } else {
        ++kp;
      }
    }
  }
}

template <int MM, int NL>
__global__ __launch_bounds__(kDpThreads, 1) void decode_engine_kernel(DpArgs a) {
  constexpr int NC = kDpWaves - NL;       // consumer waves
  extern __shared__ __attribute__((aligned(1024))) char eg_smem[];
  float* cs_l = reinterpret_cast<float*>(eg_smem);
  eg_ctl_t* ctl = eg_ctl(eg_smem);
  float* parts_l = reinterpret_cast<float*>(eg_smem + a.eg_parts);
  bf16_t* res_l = reinterpret_cast<bf16_t*>(eg_smem + a.eg_area);
  bf16_t* x_l = res_l + MM * a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, cu = blockIdx.x;

  for (int i = tid; i < MM * 128; i += kDpThreads) {
    const int m = i >> 7;
    cs_l[i] = m < a.M ? a.cos_sin[(int64_t)a.positions[m] * 128 + (i & 127)] : 0.f;
  }
  for (int i = tid; i < kEgCtlBytes / 4; i += kDpThreads) ctl[i] = i < 16 ? -1 : 0;
  int nper = 0;
  for (int st = 0; st < kDpStages; ++st) nper += (a.stages >> st) & 1;
  const int nst = (a.l1 - a.l0) * nper;
  uint32_t* abort_w = a.cnt + (nst > 1 ? nst - 1 : 0) * kDpShards * kDpShardWords;
  uint32_t* exit_w = abort_w + kDpShardWords;
  __syncthreads();

  if (wave < NL) {
    eg_stamp(a, wave, lane);
    if (wave == 0) eg_stamp_clk(a, 24, lane);
    eg_loader<NL>(a, eg_smem, wave, lane);
    if (wave == 0) eg_stamp_clk(a, 26, lane);
    eg_stamp(a, 4 + wave, lane);
  } else {
    const int c = wave - NL;
    eg_stamp(a, wave, lane);
    const int gw = c * nwg + cu, nwt = NC * nwg;
    const eg_lds_c* const ring = (const eg_lds_c*)(eg_smem + a.eg_ring_off);
    const int R = a.eg_ring;
    bool aborted = false;
    int n = 0, cbase = 0, sn = 0, an = 0, k = 0;
    for (int l = a.l0; l < a.l1 && !aborted; ++l) {
      const DpLayer L = a.layers[l];
      for (int st = 0; st < kDpStages && !aborted; ++st) {
        if (!((a.stages >> st) & 1)) continue;
        if (k > 0) aborted = eg_wait(a, k - 1, l, st, ctl, abort_w, c, lane);
        if (aborted) break;
        if (st == kDpAttn) {
          if (!(a.flags & 4)) {
            const int nu = a.W * a.Hkv * a.splits;
            bf16_t* v_lds = res_l + c * (kDpVTile / 2);
            for (int u = gw; u < nu; u += nwt) {
              const int split = u % a.splits, rest = u / a.splits;
              dp_attn_unit(a, L, rest / a.Hkv, rest % a.Hkv, split, v_lds, lane);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          int prev = 0;
          if (lane == 0) prev = eg_lds_add(ctl, kEgAtt);
          prev = __builtin_amdgcn_readfirstlane(prev);
          if (prev == NC * an + NC - 1 && k + 1 < nst) eg_arrive_global(a, k, lane);
          ++an;
        } else {
          const EgStage s = eg_stage(a, L, st, cu, nwg);
          eg_stage_inputs<MM, NC>(a, st, res_l, x_l, c, lane, ctl, sn);
          if (sn == 0) eg_stamp(a, 8 + c, lane);
          const bool normx = st == kDpQkv || st == kDpGu;
          const bf16_t* x_in = normx ? res_l : x_l;
          float rs[MM];
#pragma unroll
          for (int m = 0; m < MM; ++m) rs[m] = 1.f;
          if (normx) {
            float ssq[MM];
#pragma unroll
            for (int m = 0; m < MM; ++m) ssq[m] = 0.f;
            for (int ch = 0; ch < (a.d >> 9); ++ch)
#pragma unroll
              for (int m = 0; m < MM; ++m) {
                const u32x4 x = *reinterpret_cast<const u32x4*>(res_l + m * a.d + ch * 512 + lane * 8);
                ssq[m] = dot8(x, x, ssq[m]);
              }
#pragma unroll
            for (int m = 0; m < MM; ++m) rs[m] = rsqrtf(wave_sum_dpp(ssq[m]) / (float)a.d + a.eps);
          }
          if (sn == 0) eg_stamp(a, 12 + c, lane);
          int idx = (n + c) % R;
          for (int j = c; j < s.S; j += NC, idx = idx + NC >= R ? idx + NC - R : idx + NC) {
            const int seq = n + j;
            if (!eg_spin(a, ctl, [&]() { return eg_ld(ctl, kEgFull + idx) >= seq; })) {
              aborted = true;
              break;
            }
            if (seq < 64) eg_stamp(a, 192 + seq, lane);
            if (a.flags & 32) {         // timing: slots released unread (WRONG results)
              if (lane == 0) ctl[kEgDone + idx] = seq;
            } else {
              eg_consume_slot<MM>(ring + idx * kEgSlot, s, j, x_in, parts_l, ctl, idx, seq, lane);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            int prev = 0;
            if (lane == 0) prev = eg_lds_add(ctl, kEgCons_);
            prev = __builtin_amdgcn_readfirstlane(prev);
            if (prev == cbase + s.S - 1) {            // the stage's last slot: epilogue
              if (sn == 0) eg_stamp(a, 16, lane);
              eg_epilogue<MM>(a, L, st, s, parts_l, res_l, cs_l, rs, lane);
              if (sn == 0) eg_stamp(a, 17, lane);
              if (k + 1 < nst) eg_arrive_global(a, k, lane);
            }
          }
          if (s.S == 0 && c == 0 && k + 1 < nst) eg_arrive_global(a, k, lane);
          n += s.S;
          cbase += s.S;
          ++sn;
        }
        ++k;
      }
    }
    if (aborted && lane == 0) ctl[kEgAb] = 1;
    eg_stamp(a, 4 + wave, lane);
  }

  // ---- exit (as decode_persist_kernel)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(exit_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ctl[kEgExit] = prev == (unsigned)nwg - 1;
  }
  __syncthreads();
  if (eg_ld(ctl, kEgExit)) {
    const int nseam = nst > 1 ? nst - 1 : 0;
    for (int i = tid; i < nseam * kDpShards; i += kDpThreads)
      __hip_atomic_store(a.cnt + i * kDpShardWords, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) {
      __hip_atomic_store(abort_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(exit_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// engine LDS layout for (M, d, Hq, Hkv, F) on `grid` CUs: cs | ctl | parts | area | ring;
// returns the total bytes (0 when fewer than 5 ring slots fit in 160 KB)
int decode_engine_layout(int M, int d, int Hq, int Hkv, int F, int grid, int* ring, int* parts,
                         int* area, int* ring_off) {
  const int mm = M <= 1 ? 1 : 2;
  const int nq = (Hq + 2 * Hkv) * 128, qd = Hq * kD;
  auto cdiv = [](int x, int y) { return (x + y - 1) / y; };
  int rows = cdiv(nq / 2, grid) * 2;
  rows = rows > cdiv(d, grid) ? rows : cdiv(d, grid);
  rows = rows > cdiv(F, grid) * 2 ? rows : cdiv(F, grid) * 2;
  const int kx = qd > F ? qd : F;
  int ar = mm * (d + kx) * 2;
  if (ar < kEgCons * kDpVTile) ar = kEgCons * kDpVTile;
  const int p0 = kDpCsBytes + kEgCtlBytes;
  const int a0 = (p0 + rows * kEgSegs * mm * 4 + 15) & ~15;
  const int r0 = (a0 + ar + 1023) & ~1023;
  int R = (160 * 1024 - r0) / kEgSlot;
  if (R > 8) R = 8;
  if (R < 5) return 0;
  *ring = R;
  *parts = p0;
  *area = a0;
  *ring_off = r0;
  return r0 + R * kEgSlot;
}

// counter words a launch of `nst` stages needs: (nst - 1) seams x 8 shards x 32 words,
// then the abort and exit words (32 words apart)
int decode_persist_counter_words(int nst) {
  return ((nst > 1 ? nst - 1 : 0) * kDpShards + 2) * kDpShardWords;
}

int decode_persist_lds_bytes(int M, int d, int Kx) {
  const int mm = M <= 1 ? 1 : M <= 2 ? 2 : 4;
  const int rows = mm * (d + Kx) * 2;
  const int vt = kDpWaves * kDpVTile;
  return kDpCsBytes + kDpCtlBytes + (rows > vt ? rows : vt);
}

int decode_persist_grid() {
  static const int ncu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return ncu;
}

void launch_decode_persist(const DpArgs& a, hipStream_t s) {
  const int Kx = a.Hq * kD > a.F ? a.Hq * kD : a.F;
  const int lds = decode_persist_lds_bytes(a.M, a.d, Kx);
  const int grid = decode_persist_grid();
  DpArgs b = a;
  b.err = kernel_error_words(s);
  if (a.flags & kEgFlag) {
    // shapes (M <= 2, K / 512 <= 33, the layout fits) are checked by the binding
    const int bytes = decode_engine_layout(a.M, a.d, a.Hq, a.Hkv, a.F, grid, &b.eg_ring,
                                           &b.eg_parts, &b.eg_area, &b.eg_ring_off);
    // flags bit 7: two loader waves (two consumers)
    if (a.flags & 128) {
      if (a.M <= 1)
        decode_engine_kernel<1, 2><<<grid, kDpThreads, bytes, s>>>(b);
      else
        decode_engine_kernel<2, 2><<<grid, kDpThreads, bytes, s>>>(b);
    } else if (a.M <= 1) {
      decode_engine_kernel<1, 1><<<grid, kDpThreads, bytes, s>>>(b);
    } else {
      decode_engine_kernel<2, 1><<<grid, kDpThreads, bytes, s>>>(b);
    }
    return;
  }
  if (a.M <= 1)
    decode_persist_kernel<1><<<grid, kDpThreads, lds, s>>>(b);
  else if (a.M <= 2)
    decode_persist_kernel<2><<<grid, kDpThreads, lds, s>>>(b);
  else
    decode_persist_kernel<4><<<grid, kDpThreads, lds, s>>>(b);
}

// host entry of the torch binding (shapes checked there)
void launch_decode_persist_op(const int64_t* layers, int l0, int l1, int stages, int M, int d,
                              int Hq, int Hkv, int F, bf16_t* residual, bf16_t* qbuf, int ldq,
                              bf16_t* attn, bf16_t* act, const int32_t* positions,
                              const float* cos_sin, const int32_t* slots, int BS,
                              const int32_t* block_tables, int bt_stride, const int32_t* q_start,
                              const int32_t* q_len, const int32_t* kv_len,
                              const int32_t* work_seq, const int32_t* work_ct, int W, int splits,
                              float* part_o, float* part_ml, int32_t* tickets, float scale,
                              uint32_t* cnt, float eps, int flags, hipStream_t s) {
  DpArgs a{};
  a.layers = reinterpret_cast<const DpLayer*>(layers);
  a.l0 = l0; a.l1 = l1; a.stages = stages;
  a.M = M; a.d = d; a.Hq = Hq; a.Hkv = Hkv; a.F = F;
  a.residual = residual; a.qbuf = qbuf; a.ldq = ldq; a.attn = attn; a.act = act;
  a.positions = positions; a.cos_sin = cos_sin; a.slots = slots; a.BS = BS;
  a.block_tables = block_tables; a.bt_stride = bt_stride;
  a.q_start = q_start; a.q_len = q_len; a.kv_len = kv_len;
  a.work_seq = work_seq; a.work_ct = work_ct; a.W = W; a.splits = splits;
  a.part_o = part_o; a.part_ml = part_ml; a.tickets = tickets;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.cnt = cnt; a.eps = eps; a.flags = flags;
  launch_decode_persist(a, s);
}

}  // namespace rfq
