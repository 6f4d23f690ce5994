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
                                 // 8 rotated chunk start per wave
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
  prev = __shfl(prev, 0, 64);
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
      const uint32_t ab = __shfl(v, kDpShards, 64);
      uint32_t tot = lane < kDpShards ? v : 0u;
#pragma unroll
      for (int o2 = 1; o2 < kDpShards; o2 <<= 1) tot += __shfl_xor(tot, o2, 64);
      tot = __shfl(tot, 0, 64);
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
  return ctl[0] != 0;
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
  if (ctl[1]) {
    const int nseam = nst > 1 ? nst - 1 : 0;
    for (int i = tid; i < nseam * kDpShards; i += kDpThreads)
      __hip_atomic_store(a.cnt + i * kDpShardWords, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) {
      __hip_atomic_store(abort_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(exit_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
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
