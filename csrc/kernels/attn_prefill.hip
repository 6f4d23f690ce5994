// Paged, causal, variable-length prefill / extend attention with GQA.
// prompts of 262-958 tokens, q_len <= kv_len whenever the
// prefix cache already holds the shared system+template prefix (or for chunked
// prefill / grammar jump-forward extends).
//
// Structure (gfx950):
//   * workgroup = NW waves = the G query heads of ONE kv head x QB queries (QB = 64
//     for Llama-3-8B / Mixtral, G = 4, NW = 8; 32 for Llama-3-70B at TP = 8, G = 8),
//     so every K/V tile staged in LDS feeds 256 (query, head) rows; each wave owns
//     32 queries of one head (cdna_hip_programming.md "Fused attention prefill");
//   * 1-D grid with kv head = blockIdx % Hkv: at Hkv = 8 every workgroup of one kv
//     head lands on one XCD, whose L2 holds that head's K/V (T1); the work list runs
//     back to front so the heaviest (latest) causal blocks start first;
//   * 64-key tiles (two 32-token pages) arrive by LDS-DMA into a 4-slot ring, two
//     tiles ahead, behind counted vmcnt waits, one barrier per tile (T14);
//       K image  [64][128] bf16, 16-B chunk ch of row r at ch ^ (r & 15)
//                (ds_read_b128 row reads conflict-free, T2),
//       V image  [64][128] bf16, chunk ch of row r at ch ^ ((r & 3) << 2)
//                (ds_read_b64_tr_b16 transposed reads conflict-free, T10);
//   * S^T = K Q^T on mfma_f32_32x32x16_bf16 with Q^T held in registers, so each
//     lane owns one query column and the online softmax is lane-local (+1
//     permlane32 swap per row statistic);
//   * O^T = V^T P^T with the S^T accumulators packed to bf16 as the B operand
//     (accumulator-as-operand, §3); O keeps the query on the lane, so the rescale by
//     exp2(m_old - m_new) needs no data movement, and it is deferred (T13);
//   * per tile every wave runs QK^T(t+1), then PV(t) with softmax(t+1) sliced
//     between its MFMAs (intra-wave overlap);
//   * causal: a wave skips the MFMAs of tiles past its last query.
// Measured in profiles/r2_prefill_attention.md.
#include "common.h"

namespace rfq {

constexpr int kPD = 128;
constexpr int kPPage = 32;
constexpr int kKT = 64;  // keys per tile
constexpr int kQB = 32;  // queries per wave
constexpr int kStage = 2 * kKT * kPD;   // K + V elements per LDS stage
constexpr float kRescale = 8.f;         // defer-max threshold (log2 units)

// Per 64-key tile t every wave runs:
//   S = K(t+1) Q^T            16 MFMAs (K fragments a subtile ahead)
//   O^T += V(t)^T P(t)^T      16 MFMAs, with softmax(S) -> P(t+1) issued between them
// so the exp / max / sum chain of tile t+1 fills the issue slots the PV MFMAs leave
// (an MFMA holds the SIMD's vector issue for 8 of its 32 cycles) instead of running
// serially behind its own QK^T.  K/V sit in a 4-slot LDS ring: tile t+3 is written
// by LDS-DMA into the slot tile t-1 vacated, so ONE barrier per tile suffices and
// each tile's DMA has two tiles of latency cover.
constexpr int kSlots = 4;
constexpr int kMinSplitTiles = 3;       // key tiles per split workgroup, at least
constexpr int kMaxKvSplit = 4;          // split workgroups per work item, at most
typedef __attribute__((address_space(3))) char lds_c;
typedef __attribute__((address_space(3))) const s16x8 lds_s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_prefill_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_q_start, const int32_t* __restrict__ seq_q_len,
    const int32_t* __restrict__ seq_kv_len, const int32_t* __restrict__ work_seq,
    const int32_t* __restrict__ work_qblk, bf16_t* __restrict__ out, int64_t out_stride, int Hq,
    int Hkv, float scale_log2, int hgroups, int kvsplit = 1, float* __restrict__ ws = nullptr,
    int32_t* __restrict__ tickets = nullptr, uint64_t* __restrict__ ts = nullptr,
    int bal_work = 0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // ts (diagnostics, attn_prefill_timing): per workgroup 8 words of s_memrealtime
  // (100 MHz) stamps written by thread 0 -- entry, metadata, first tiles landed, key
  // loop done, split hand-off done, end; word 6 = tiles | split << 16 | merger << 17
  const bool stamp = ts != nullptr && threadIdx.x == 0;
  uint64_t* const tsw = ts != nullptr ? ts + (int64_t)blockIdx.x * 8 : nullptr;
  if (stamp) tsw[0] = __builtin_amdgcn_s_memrealtime();
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);
  constexpr int NT = NW * 64;
  constexpr int NCH = kKT * 16 / NT;

  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h2 = lane >> 5;
  const int G = Hq / Hkv;
  // hgroups > 1 (small grids, e.g. one sequence at the TP = 8 rank shape Hq 8 / Hkv 1):
  // the G query heads of a kv head are split over hgroups workgroups of HPW heads, so
  // twice the workgroups share the causal critical path and each SIMD runs one wave
  const int HPW = G / hgroups;
  const int QB = NW / HPW * kQB;
  // kvsplit = 2: the two workgroups of a (work item, kv head, head group) take the two
  // halves of its key tiles and merge (below); adjacent in the grid, heaviest first
  //
  // Balanced form (bal_work = work items <= 128, kvsplit = 4, hgroups = 1, one workgroup
  // per CU): the grid is an exact task list, not (item, split) slots.  A grid with idle
  // slots does not help: the dispatcher does not back-fill a CU freed by a workgroup
  // that leaves at once (r6 phase stamps: the 257th workgroup started after ~24 µs with
  // 220 of 384 slots active), so here every workgroup derives the same list from the
  // work items' key-tile counts (two items per lane, wave reductions): tiles per split
  // = the smallest value >= max(kMinSplitTiles, ceil(tmax / 4)) whose task count fits
  // the grid, items heaviest first, each item's Hkv x nact tasks contiguous.
  int kvs, bid, num_work;
  int split_tiles = kMinSplitTiles;
  if (bal_work > 0) {
    num_work = bal_work;
    auto item_tiles = [&](int w) {
      const int sq = work_seq[w];
      const int ql = seq_q_len[sq], kl = seq_kv_len[sq];
      const int last = min(work_qblk[w] * QB + QB, ql) - 1;
      return (min(kl, kl - ql + last + 1) + kKT - 1) / kKT;
    };
    const int ta = lane < num_work ? item_tiles(lane) : 0;             // item lane
    const int tb = lane + 64 < num_work ? item_tiles(lane + 64) : 0;   // item lane + 64
    int tmax = max(ta, tb);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) tmax = max(tmax, __shfl_xor(tmax, o, 64));
    tmax = __builtin_amdgcn_readfirstlane(tmax);
    int tgt = max(kMinSplitTiles, (tmax + kvsplit - 1) / kvsplit);
    auto nsp = [&](int t) { return t == 0 ? 0 : max(1, min(kvsplit, (t + tgt - 1) / tgt)); };
    // ends: tgt = tmax gives every item one task, num_work * Hkv <= 128 <= gridDim.x
    for (;;) {
      int c = nsp(ta) + nsp(tb);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
      c = __builtin_amdgcn_readfirstlane(c) * Hkv;
      if (c <= (int)gridDim.x || tgt >= tmax) break;
      ++tgt;
    }
    split_tiles = tgt;
    // heavy first = descending item index: items 64..127 (tb) before 0..63 (ta)
    const int cb = nsp(tb) * Hkv, ca = nsp(ta) * Hkv;
    int pb = cb, pa = ca;                                 // inclusive prefix over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int xb = __shfl_up(pb, o, 64), xa = __shfl_up(pa, o, 64);
      if (lane >= o) { pb += xb; pa += xa; }
    }
    const int totb = __builtin_amdgcn_readfirstlane(__shfl(pb, 63, 64));
    const int tot = totb + __builtin_amdgcn_readfirstlane(__shfl(pa, 63, 64));
    const int task = blockIdx.x;
    if (task >= tot) return;                              // more CUs than tasks
    const int sb = totb - pb, sa = tot - pa;              // tasks before the item
    const uint64_t mb = __builtin_amdgcn_ballot_w64(cb > 0 && task >= sb && task < sb + cb);
    const uint64_t ma = __builtin_amdgcn_ballot_w64(ca > 0 && task >= sa && task < sa + ca);
    const int l = mb ? __builtin_ctzll(mb) : __builtin_ctzll(ma);
    const int item = mb ? l + 64 : l;
    const int base = __builtin_amdgcn_readfirstlane(mb ? __shfl(sb, l, 64) : __shfl(sa, l, 64));
    const int ns = nsp(__builtin_amdgcn_readfirstlane(mb ? __shfl(tb, l, 64)
                                                         : __shfl(ta, l, 64)));
    const int rank_in_item = task - base;                 // kv head major, split minor
    kvs = rank_in_item % ns;
    bid = (num_work - 1 - item) * Hkv + rank_in_item / ns;
  } else {
    kvs = blockIdx.x % kvsplit;
    bid = blockIdx.x / kvsplit;
    num_work = gridDim.x / (Hkv * hgroups * kvsplit);
  }
  const int kvh = bid % Hkv;
  const int hg = (bid / Hkv) % hgroups;
  const int wi = num_work - 1 - bid / (Hkv * hgroups);
  const int seq = work_seq[wi];
  const int head = kvh * G + hg * HPW + wid % HPW;
  const int qs = work_qblk[wi] * QB + (wid / HPW) * kQB;
  const int q_len = seq_q_len[seq], kv_len = seq_kv_len[seq];
  const int ctx0 = kv_len - q_len;
  const int tok0 = seq_q_start[seq];
  const int32_t* bt = block_tables + (int64_t)seq * bt_stride;

  const int qi = qs + r;
  const bool qvalid = qi < q_len;
  s16x8 qf[8];
  {
    const bf16_t* qrow = q + (int64_t)(tok0 + (qvalid ? qi : 0)) * q_stride + (int64_t)head * kPD;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = reinterpret_cast<const s16x8*>(qrow + 16 * ks + 8 * h2)[0];
  }
  const int qpos = ctx0 + qi;
  const int wg_last_q = min(work_qblk[wi] * QB + QB, q_len) - 1;
  const int kv_end = min(kv_len, ctx0 + wg_last_q + 1);
  const int w_last_q = min(qs + kQB, q_len) - 1;
  const int w_kv_end = w_last_q < qs ? 0 : min(kv_len, ctx0 + w_last_q + 1);
  const int ntiles = (kv_end + kKT - 1) / kKT;
  const int wt = (w_kv_end + kKT - 1) / kKT;   // tiles this wave computes
  // key tiles [t0, t1) of this workgroup: an item's tiles go to nact <= kvsplit
  // workgroups of >= kMinSplitTiles tiles each; the others leave at once, and an
  // unsplit item's first workgroup writes the output directly
  const int nact = bal_work > 0
                       ? max(1, min(kvsplit, (ntiles + split_tiles - 1) / split_tiles))
                       : max(1, min(kvsplit, ntiles / kMinSplitTiles));
  if (kvs >= nact) return;
  const bool split = nact > 1;
  const int t0 = kvs * ntiles / nact;
  const int t1 = (kvs + 1) * ntiles / nact;
  if (stamp) {
    tsw[1] = __builtin_amdgcn_s_memrealtime();
    tsw[6] = (uint64_t)(t1 - t0) | ((uint64_t)split << 16);
  }
  const int wend = min(wt, t1);

  lds_c* const lbase = (lds_c*)smem;
  // K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction,
  // lane-linear destination): wave instruction g of a tile fills rows 4g..4g+3, and the
  // lane filling slot (row, chunk c') fetches the global chunk that the row's XOR
  // swizzle puts there.  Keys past kv_end are clamped to the last valid key (finite
  // data; those scores are masked, so their P is exactly 0).
  constexpr int NPT = 2 * NCH;                 // DMA instructions per wave per tile
  auto load = [&](int t) {
    const int kt = t * kKT, pg0 = kt / kPPage;
    const int64_t page_a = bt[pg0];
    const int64_t page_b = kt + kPPage < kv_end ? bt[pg0 + 1] : page_a;
    lds_c* const sl = lbase + (t % kSlots) * (kStage * 2);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int g = wid * NCH + i;
      const int row = 4 * g + (lane >> 4), cp = lane & 15;
      const int key = min(kt + row, kv_end - 1);
      const int64_t page = key - kt < kPPage ? page_a : page_b;
      const int64_t off = ((page * Hkv + kvh) * kPPage + (key % kPPage)) * kPD;
      __builtin_amdgcn_global_load_lds(k_cache + off + 8 * (cp ^ (row & 15)),
                                       (lds_void_t*)(sl + g * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(v_cache + off + 8 * (cp ^ ((row & 3) << 2)),
                                       (lds_void_t*)(sl + kKT * kPD * 2 + g * 1024), 16, 0, 0);
    }
  };
  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                         0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16 s[2];
  // LDS addressing, two invariant registers each for K and V:
  //   K: chunk (2ks + h2) ^ (r & 15) of row r = krow + (kx ^ 32 ks), kx = (h2 ^ (r & 15)) << 4
  //   V: chunk ((m ^ qq) << 2) + low of row 4h2 + qq = vrow + (vx ^ 64 m), vx = qq << 6
  // Each tile rebuilds the per-read-group pointers (one v_xad each) from an opaque
  // copy of kx / vx plus the slot base, so the subtile / key-chunk steps fold into the
  // ds_read immediates; otherwise the compiler hoists every (offset + constant)
  // combination into its own VGPR and the kernel spills.
  const int gi = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
  const uint32_t krow = r * 256, kx = (uint32_t)(h2 ^ (r & 15)) << 4;
  const uint32_t vrow = kKT * kPD * 2 + (4 * h2 + qq) * 256 +
                        ((2 * (gi & 1) + (pp >> 1)) << 4) + (4 * (pp & 1)) * 2;
  const uint32_t vx = (uint32_t)qq << 6;
  auto slot = [&](int t) { return lbase + (t % kSlots) * (kStage * 2); };
  // S^T of tile t (lane: S^T[key 32st + (i&3) + 8(i>>2) + 4h2][query r]), masked
  auto qk = [&](int t) {
    lds_c* const sl = slot(t);
    uint32_t x = kx;
    asm volatile("" : "+v"(x));
    lds_c* kp[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      kp[ks] = sl + krow + (x ^ (32 * ks));
      asm volatile("" : "+v"(kp[ks]));
    }
    // K fragments by inline-asm ds_read_b128 with counted waits tied to each fragment:
    // every MFMA waits only for its own read (LDS returns in order), not lgkmcnt(0)
    // for all eight as the compiler's waits did
    s16x8 ka[8];
#define RFQ_KREAD(KS, OFF) \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ka[KS]) : "v"(kp[KS]), "i"(OFF))
#define RFQ_KWAIT(KS, N) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(ka[KS]))
    RFQ_KREAD(0, 0); RFQ_KREAD(1, 0); RFQ_KREAD(2, 0); RFQ_KREAD(3, 0);
    RFQ_KREAD(4, 0); RFQ_KREAD(5, 0); RFQ_KREAD(6, 0); RFQ_KREAD(7, 0);
#define RFQ_QK0(KS)                                                                        \
    RFQ_KWAIT(KS, 7);                                                                      \
    s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[KS]), as_bf16x8(qf[KS]),   \
                                                   (KS) == 0 ? zero16 : s[0], 0, 0, 0);    \
    RFQ_KREAD(KS, 32 * 256);                                                               \
    __builtin_amdgcn_sched_barrier(0);
    RFQ_QK0(0) RFQ_QK0(1) RFQ_QK0(2) RFQ_QK0(3) RFQ_QK0(4) RFQ_QK0(5) RFQ_QK0(6) RFQ_QK0(7)
#define RFQ_QK1(KS, N)                                                                     \
    RFQ_KWAIT(KS, N);                                                                      \
    s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[KS]), as_bf16x8(qf[KS]),   \
                                                   (KS) == 0 ? zero16 : s[1], 0, 0, 0);    \
    __builtin_amdgcn_sched_barrier(0);
    RFQ_QK1(0, 7) RFQ_QK1(1, 6) RFQ_QK1(2, 5) RFQ_QK1(3, 4)
    RFQ_QK1(4, 3) RFQ_QK1(5, 2) RFQ_QK1(6, 1) RFQ_QK1(7, 0)
#undef RFQ_QK0
#undef RFQ_QK1
#undef RFQ_KREAD
#undef RFQ_KWAIT
    const int kt = t * kKT;
    if (kt + kKT > ctx0 + qs || kt + kKT > kv_end) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kt + 32 * st + (i & 3) + 8 * (i >> 2) + 4 * h2;
          if (key > qpos || key >= kv_end) s[st][i] = -INFINITY;
        }
    }
  };

  float m_run = -INFINITY, l_run = 0.f;
  const float rescale_raw = kRescale / scale_log2;
  s16x8 pb[4];                                 // P^T of the pending tile, bf16, per 16-key chunk
  // softmax of s in slices (so PV's key chunks can carry one each): sm_max sets the
  // row max, the wave-uniform defer-max decision (T13) and the O/l rescale factor;
  // sm_exp(c) turns key chunk c into bf16 P and adds its row sum.
  float alpha = 1.f, nb = 0.f, psum = 0.f;
  bool resc = false;
  auto sm_max = [&]() {
    float mx = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[st][i]);
    {   // other half of the row: v_permlane32_swap (VALU), not an LDS bpermute
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx),
                                                       false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    resc = __any(mx > m_run + rescale_raw);
    const float m_new = resc ? fmaxf(m_run, mx) : m_run;
    alpha = (!resc || m_new == -INFINITY) ? 1.f : fast_exp2((m_run - m_new) * scale_log2);
    m_run = m_new;
    nb = m_new == -INFINITY ? 0.f : -m_new * scale_log2;
    psum = 0.f;
  };
  auto sm_exp = [&](int c, s16x8* pn) {
    float pv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pv[j] = fast_exp2(fmaf(s[c >> 1][8 * (c & 1) + j], scale_log2, nb));
      psum += pv[j];
    }
    pn[c] = pack8(pv);
  };
  auto sm_done = [&]() { l_run = l_run * alpha + psum; };
  f32x16 o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) o[m] = zero16;
  // V^T fragments by inline-asm ds_read_b64_tr_b16 with counted lgkmcnt waits tied
  // to the destination registers: through the builtin the compiler guards every such
  // read with vmcnt(0) against the in-flight LDS-DMA (it cannot tell the slots apart),
  // which would drain the next tiles' DMA in every PV phase.
  auto pv_mfma = [&](int t, const bool sm, s16x8* pn) {
    lds_c* const sl = slot(t);
    uint32_t x = vx;
    asm volatile("" : "+v"(x));
    lds_c* vp[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      vp[m] = sl + vrow + (x ^ (64 * m));
      asm volatile("" : "+v"(vp[m]));
    }
    s16x4 va[2][4][2];
#define RFQ_VREAD(C)                                                                   \
    _Pragma("unroll") for (int m = 0; m < 4; ++m)                                      \
      asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4" \
                   : "=v"(va[(C) & 1][m][0]), "=v"(va[(C) & 1][m][1])                  \
                   : "v"(vp[m]), "i"((C) * 4096), "i"((C) * 4096 + 2048));
#define RFQ_VWAIT(C, N)                                                                \
    asm volatile("s_waitcnt lgkmcnt(" #N ")"                                           \
                 : "+v"(va[(C) & 1][0][0]), "+v"(va[(C) & 1][0][1]), "+v"(va[(C) & 1][1][0]), \
                   "+v"(va[(C) & 1][1][1]), "+v"(va[(C) & 1][2][0]), "+v"(va[(C) & 1][2][1]), \
                   "+v"(va[(C) & 1][3][0]), "+v"(va[(C) & 1][3][1]));
#define RFQ_VMFMA(C)                                                                   \
    _Pragma("unroll") for (int m = 0; m < 4; ++m) {                                    \
      const s16x4 a0 = va[(C) & 1][m][0], a1 = va[(C) & 1][m][1];                      \
      const s16x8 a = (s16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]}; \
      o[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a), as_bf16x8(pb[C]), o[m], 0, 0, 0); \
    }
    // four regions fenced by sched_barrier(0): [next chunk's reads, this chunk's
    // counted wait, its 4 MFMAs + one softmax slice] -- the slice's VALU issues in
    // the MFMAs' shadow (guide: "sm-split across d0-blocks")
    RFQ_VREAD(0)
    RFQ_VREAD(1)
    RFQ_VWAIT(0, 8)
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VMFMA(0)
    if (sm) { sm_max(); sm_exp(0, pn); }
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VREAD(2)
    RFQ_VWAIT(1, 8)
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VMFMA(1)
    if (sm) sm_exp(1, pn);
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VREAD(3)
    RFQ_VWAIT(2, 8)
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VMFMA(2)
    if (sm) sm_exp(2, pn);
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VWAIT(3, 0)
    __builtin_amdgcn_sched_barrier(0);
    RFQ_VMFMA(3)
    if (sm) { sm_exp(3, pn); sm_done(); }
    __builtin_amdgcn_sched_barrier(0);
#undef RFQ_VREAD
#undef RFQ_VWAIT
#undef RFQ_VMFMA
  };

  // prologue: tiles 0 and 1 landed, tile 2 in flight.  Tile t+3 is issued at the
  // start of iteration t into the slot tile t-1 vacated (kSlots = 4) and must have
  // landed by the end of iteration t+1: two tiles of DMA latency cover, and the
  // counted vmcnt(NPT) leaves the newest tile in flight across the barrier.
  auto wait_dma = [&](bool newest_pending) {
    if (newest_pending) {
      if constexpr (NPT == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  load(t0);
  if (t0 + 1 < t1) load(t0 + 1);
  if (t0 + 2 < t1) load(t0 + 2);
  wait_dma(t0 + 2 < t1);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (stamp) tsw[2] = __builtin_amdgcn_s_memrealtime();
  if (wend > t0) {
    qk(t0);
    sm_max();
#pragma unroll
    for (int c = 0; c < 4; ++c) sm_exp(c, pb);
    sm_done();
  }
  for (int t = t0; t < t1; ++t) {
    if (t + 3 < t1) load(t + 3);
    if (t < wend) {
      if (t + 1 < wend) {
        qk(t + 1);
        s16x8 pn[4];
        pv_mfma(t, true, pn);
        // pin P(t+1) inside the PV block: otherwise the exp chain is sunk past the
        // rescale branch and runs after the MFMAs instead of between them
        asm volatile("" ::"v"(pn[0]), "v"(pn[1]), "v"(pn[2]), "v"(pn[3]));
        if (resc) {
#pragma unroll
          for (int m = 0; m < 4; ++m) o[m] *= alpha;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) pb[c] = pn[c];
      } else {
        pv_mfma(t, false, nullptr);
      }
    }
    wait_dma(t + 3 < t1);                       // tile t+2 landed (tile t+3 may fly)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  if (stamp) tsw[3] = __builtin_amdgcn_s_memrealtime();
  float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  if (split) {
    // Hand-off of the unnormalised O, running max (raw score units) and row sum between
    // the two halves (cdna_hip_programming.md §6 Guideline 16, "every load sc1"): sc1
    // 8-byte stores drained by vmcnt(0) + barrier, a relaxed agent-scope ticket, sc1
    // loads of the partner's partial by the second arriver, which merges and writes the
    // output; it resets the ticket for the next launch.  No fences, no L2 writeback.
    // Memory-model note: the ordering rests on the gfx950 ISA, not on a C++ release /
    // acquire pair -- every handed-off store and load is an sc1 (device-coherent)
    // access, the stores are retired by vmcnt(0) before the barrier that precedes the
    // ticket, and the ticket is an L2 atomic.  An acq_rel agent-scope ticket would
    // compile to an L2 writeback + invalidate (buffer_wbl2 / buffer_inv), several µs
    // per split; gemv_core.h's split-K ticket relies on the same three facts.  The
    // GPU tests exercise every split form four times per case.
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    constexpr int kPart = 64 * 64 + 64 * 2;               // floats per wave
    float* mine = ws + (((int64_t)bid * kMaxKvSplit + kvs) * NW + wid) * kPart;
#pragma unroll
    for (int j = 0; j < 32; ++j) {                        // o[m][2jj..2jj+1], j = 8m + jj
      const float a = o[j >> 3][2 * (j & 7)], b = o[j >> 3][2 * (j & 7) + 1];
      __hip_atomic_store((gu64*)(mine + (j * 64 + lane) * 2),
                         (unsigned long long)__float_as_uint(a) |
                             ((unsigned long long)__float_as_uint(b) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store((gu64*)(mine + 4096 + lane * 2),
                       (unsigned long long)__float_as_uint(m_run) |
                           ((unsigned long long)__float_as_uint(l_tot) << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int s_second;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(tickets + bid, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      s_second = prev == nact - 1;
      if (prev == nact - 1)
        __hip_atomic_store(tickets + bid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (stamp) {
      tsw[4] = __builtin_amdgcn_s_memrealtime();
      tsw[6] |= (uint64_t)s_second << 17;
    }
    if (!s_second) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every handed-off load is sc1
    // The np = nact - 1 partners p(i) (ascending split index, skipping this one) are
    // merged in ascending order, as one rescale per partial.  Their loads are
    // pipelined: every (max, sum) and the first partial's O go out together; with 4
    // waves (512 VGPRs per lane) the second's too, and the third's once the first has
    // been consumed (two load round trips instead of one per partner plus one for the
    // (max, sum)); the 8-wave form (256 VGPRs, a second 64-register buffer spills)
    // loads each further partial after the previous one is absorbed.
    const int np = nact - 1;
    auto pidx = [&](int i) { return i < kvs ? i : i + 1; };
    auto part = [&](int i) {
      return ws + (((int64_t)bid * kMaxKvSplit + pidx(i)) * NW + wid) * kPart;
    };
    auto ld8 = [&](const float* p) {
      return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    unsigned long long mlv[kMaxKvSplit - 1];
#pragma unroll
    for (int i = 0; i < kMaxKvSplit - 1; ++i)
      mlv[i] = i < np ? ld8(part(i) + 4096 + lane * 2) : 0ull;
    unsigned long long ua[32], ub[NW == 4 ? 32 : 1];
#pragma unroll
    for (int i = 0; i < 32; ++i) ua[i] = ld8(part(0) + (i * 64 + lane) * 2);
    if constexpr (NW == 4) {
      if (np > 1) {
#pragma unroll
        for (int i = 0; i < 32; ++i) ub[i] = ld8(part(1) + (i * 64 + lane) * 2);
      }
    }
    float m_p[kMaxKvSplit - 1], l_p[kMaxKvSplit - 1];
    float m_n = m_run;
#pragma unroll
    for (int i = 0; i < kMaxKvSplit - 1; ++i) {
      m_p[i] = i < np ? __uint_as_float((unsigned)mlv[i]) : -INFINITY;
      l_p[i] = i < np ? __uint_as_float((unsigned)(mlv[i] >> 32)) : 0.f;
      m_n = fmaxf(m_n, m_p[i]);
    }
    const float a_s = m_run == -INFINITY ? 0.f : fast_exp2((m_run - m_n) * scale_log2);
    l_tot *= a_s;
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] *= a_s;
    auto absorb = [&](const unsigned long long* u, int i) {
      const float a_o = m_p[i] == -INFINITY ? 0.f : fast_exp2((m_p[i] - m_n) * scale_log2);
      l_tot += l_p[i] * a_o;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const int m = k >> 3, e = 2 * (k & 7);
        o[m][e] += __uint_as_float((unsigned)u[k]) * a_o;
        o[m][e + 1] += __uint_as_float((unsigned)(u[k] >> 32)) * a_o;
      }
    };
    absorb(ua, 0);
    if constexpr (NW == 4) {
      if (np > 2) {
#pragma unroll
        for (int i = 0; i < 32; ++i) ua[i] = ld8(part(2) + (i * 64 + lane) * 2);
      }
      if (np > 1) absorb(ub, 1);
      if (np > 2) absorb(ua, 2);
    } else {
      for (int i2 = 1; i2 < np; ++i2) {
#pragma unroll
        for (int i = 0; i < 32; ++i) ua[i] = ld8(part(i2) + (i * 64 + lane) * 2);
        absorb(ua, i2);
      }
    }
  }
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  bf16_t* ol = lds + wid * (kQB * kPD);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint2 w;
      w.x = pack_bf16x2(o[m][4 * k + 0] * inv, o[m][4 * k + 1] * inv);
      w.y = pack_bf16x2(o[m][4 * k + 2] * inv, o[m][4 * k + 3] * inv);
      *reinterpret_cast<uint2*>(ol + r * kPD + (((4 * m + k) ^ (r & 15)) << 3) + 4 * h2) = w;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int cc = lane & 15;
#pragma unroll
  for (int j = 0; j < kQB / 4; ++j) {
    const int row = (lane >> 4) + 4 * j;
    const u32x4 v = *reinterpret_cast<const u32x4*>(ol + row * kPD + ((cc ^ (row & 15)) << 3));
    if (qs + row < q_len)
      *reinterpret_cast<u32x4*>(out + (int64_t)(tok0 + qs + row) * out_stride +
                                (int64_t)head * kPD + 8 * cc) = v;
  }
  if (stamp) tsw[5] = __builtin_amdgcn_s_memrealtime();
}

// Split-KV workspace (ws, tickets): per (work item, kv head, head group) up to 4 splits
// x up to 8 waves x (64 x 64 + 128) floats and one zeroed ticket; kPrefillSplitMaxWg bounds the
// split grid (ops.prefill_split_ws allocates for it).
constexpr int kPrefillSplitMaxWg = 256;
int prefill_split_ws_floats() {
  return (kPrefillSplitMaxWg / 2) * kMaxKvSplit * 8 * (64 * 64 + 64 * 2);   // <= 8 waves
}
int prefill_split_tickets() { return kPrefillSplitMaxWg / 2; }

// qblk: queries per work item (the packer's prefill block): NW = qblk * G / 32 waves.
// hsplit_below: when num_work * Hkv is below this many workgroups (the grid cannot
// fill the CUs) and the 8 waves are one query block of 8 heads (G = 8, qblk 32), the
// heads are split over 2 workgroups of 4 waves (0 = never).
// Diagnostics: while set, every attn_prefill launch stamps its workgroups' phases into
// this buffer (>= 8 words per workgroup; attn_prefill_kernel ts).
static uint64_t* g_prefill_ts = nullptr;
void set_attn_prefill_timing(uint64_t* buf) { g_prefill_ts = buf; }

void launch_attn_prefill(const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                         const bf16_t* v_cache, const int32_t* block_tables, int bt_stride,
                         const int32_t* seq_q_start, const int32_t* seq_q_len,
                         const int32_t* seq_kv_len, const int32_t* work_seq,
                         const int32_t* work_qblk, int num_work, bf16_t* out, int64_t out_stride,
                         int Hq, int Hkv, float scale, int qblk, int hsplit_below,
                         float* ws, int32_t* tickets, int small_mode, hipStream_t s) {
  if (num_work == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  const int nw = qblk * G / kQB;
  const size_t lds = kSlots * kStage * sizeof(bf16_t);    // 128 KB ring
  // Small grids (num_work * Hkv < hsplit_below), two forms:
  //   head split (small_mode 1): G = 8 heads over two 4-wave workgroups, split-KV 2-4 on
  //     top while the grid fits the CUs once;
  //   8-wave split-KV (small_mode 2): all G heads in one 8-wave workgroup (two waves per
  //     SIMD), the key tiles split 2-4 ways.
  // small_mode 0 (auto) takes the head split while it can also split the keys 4 ways
  // (grids below 64 workgroups) and the 8-wave split-KV from 64 on: B1 S4096 Hq8/Hkv1
  // 98 -> 76 us, B2 S2048 54 -> 46 us, B1 S1024 17 vs 22 us (profiles/r3_prefill_kv8.md);
  // B1 S2048 (64 items) 32.8 -> 31.0 us kernel time (profiles/r4_prefill_small_grid.md).
  const int wg0 = num_work * Hkv;
  const bool small = nw == 8 && wg0 < hsplit_below && ws != nullptr && tickets != nullptr;
  // small_mode 3 (balanced split-KV): the 8-wave form over an exact task list of up to 4
  // splits per item, one workgroup per CU (attn_prefill_kernel bal_work; <= 128 items).
  // Auto takes it for 65-128 items (it replaced the uniform 2-way split there, r6 rank
  // shape Hq 8 / Hkv 1: S 2,912 with a 416-key prefix 57.5 -> 44.0 µs, S 4,096 75 -> 63 µs,
  // B2 S2048 45 -> 41 µs, profiles/r6_prefill_balanced.md); at <= 64 items the uniform
  // 4-way split is faster (the task list costs 2-4 µs of metadata before the first tile),
  // and so is the 2-way split for few, short items over several kv heads (70B TP=1, 8 kv
  // heads x 10-16 items: 21-30 µs vs 24-35 µs balanced), hence the rule on items.
  const bool bal = small && wg0 * 2 <= kPrefillSplitMaxWg &&
                   (small_mode == 3 || (small_mode == 0 && num_work * 4 > kPrefillSplitMaxWg));
  if (bal) {
    const dim3 grid8(kPrefillSplitMaxWg);
    attn_prefill_kernel<8><<<grid8, 512, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                   bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                   work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                   scale_log2, 1, kMaxKvSplit, ws, tickets,
                                                   g_prefill_ts, num_work);
    return;
  }
  const bool kv8 = small && (small_mode == 2 ||
                             (small_mode == 0 && wg0 * 4 >= kPrefillSplitMaxWg &&
                              wg0 * 2 <= kPrefillSplitMaxWg));
  if (kv8) {
    const int wg = wg0;
    const int kvsplit = wg * 4 <= kPrefillSplitMaxWg ? 4 : (wg * 2 <= kPrefillSplitMaxWg ? 2 : 1);
    const dim3 grid8(wg * kvsplit);
    attn_prefill_kernel<8><<<grid8, 512, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                   bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                   work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                   scale_log2, 1, kvsplit, ws, tickets,
                                                   g_prefill_ts);
    return;
  }
  if (nw == 8 && G == 8 && num_work * Hkv < hsplit_below) {
    // kv split on top when the workspace is given and the doubled grid still fits the
    // CUs once (one 128 KB-LDS workgroup per CU)
    // the most splits (4 or 2; items with fewer tiles activate fewer) whose grid still
    // fits the CUs in one round: a second round of workgroups costs more than the
    // shorter critical path saves (B1 S2048 Hq8/Hkv1: 4 splits over 512 workgroups
    // 38-40 us vs 2 splits over 256: 34 us; profiles/r3_prefill_head_split.md)
    const int wg2 = num_work * Hkv * 2;
    const int kvsplit = (ws == nullptr || tickets == nullptr) ? 1
                        : (wg2 * 4 <= kPrefillSplitMaxWg ? 4
                           : (wg2 * 2 <= kPrefillSplitMaxWg ? 2 : 1));
    const dim3 grid2(num_work * Hkv * 2 * kvsplit);
    attn_prefill_kernel<4><<<grid2, 256, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                   bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                   work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                   scale_log2, 2, kvsplit, ws, tickets,
                                                   g_prefill_ts);
    return;
  }
  dim3 grid(num_work * Hkv);
  if (nw == 8)
    attn_prefill_kernel<8><<<grid, 512, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                  bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                  work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                  scale_log2, 1, 1, nullptr, nullptr,
                                                  g_prefill_ts);
  else
    attn_prefill_kernel<4><<<grid, 256, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                  bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                  work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                  scale_log2, 1, 1, nullptr, nullptr,
                                                  g_prefill_ts);
}

}  // namespace rfq
