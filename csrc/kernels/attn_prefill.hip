// Paged, causal, variable-length prefill / extend attention with GQA.
// prompts of 262-958 tokens, q_len <= kv_len whenever the
// prefix cache already holds the shared system+template prefix (or for chunked
// prefill / grammar jump-forward extends).
//
// Structure (gfx950):
//   * workgroup = 8 waves = the G query heads of ONE kv head x QB queries
//     (QB = 256 / G: 64 queries for Llama-3-8B / Mixtral, G = 4; 32 for Llama-3-70B,
//     G = 8), so every K/V tile staged in LDS feeds 256 (query, head) rows; each
//     wave owns 32 queries of one head (cdna_hip_programming.md Appendix B "Fused
//     attention prefill": 8 waves x 32 rows, KVBLK 64);
//   * 64-key tiles (two 32-token pages), double-buffered in LDS with the
//     async-STAGE split (T14): a tile's global loads are issued two phases before
//     they are written to the other buffer; raw s_barrier + lgkmcnt(0) only, so the
//     loads stay in flight across barriers;
//   * ping-pong: the two halves of the workgroup run half a tile apart (QK^T +
//     softmax of one group beside the PV MFMAs of the other on every SIMD);
//       K image  [64][128] bf16, 16-B chunk ch of row r at ch ^ (r & 15)
//                (ds_read_b128 row reads conflict-free, T2),
//       V image  [64][128] bf16, chunk ch of row r at ch ^ ((r & 3) << 2)
//                (ds_read_b64_tr_b16 transposed reads conflict-free, T10);
//   * S^T = K Q^T on mfma_f32_32x32x16_bf16 with Q^T held in registers, so each
//     lane owns one query column and the online softmax is lane-local (+1 xor-32
//     shuffle per row statistic);
//   * O^T = V^T P^T with the S^T accumulators reused as the bf16 B operand
//     (accumulator-as-operand, §3) — O keeps the query on the lane, so the
//     rescale by exp2(m_old - m_new) needs no data movement;
//   * causal: a wave skips the MFMAs of tiles past its last query; the grid runs
//     the work list back to front so the heaviest (latest) query blocks start first.
#include "common.h"

namespace rfq {

constexpr int kPD = 128;
constexpr int kPPage = 32;
constexpr int kKT = 64;  // keys per tile
constexpr int kQB = 32;  // queries per wave
constexpr int kStage = 2 * kKT * kPD;   // K + V elements per LDS stage
constexpr float kRescale = 8.f;         // defer-max threshold (log2 units)

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_prefill_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_q_start, const int32_t* __restrict__ seq_q_len,
    const int32_t* __restrict__ seq_kv_len, const int32_t* __restrict__ work_seq,
    const int32_t* __restrict__ work_qblk, bf16_t* __restrict__ out, int64_t out_stride, int Hq,
    int Hkv, float scale_log2, int hsplit) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);
  constexpr int NT = NW * 64;
  constexpr int NCH = kKT * 16 / NT;          // 16-B chunks of K (and of V) per thread per tile

  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h2 = lane >> 5;
  const int G = Hq / Hkv;
  const int Gw = G / hsplit;                  // query heads per workgroup
  const int QB = NW * kQB / Gw;               // queries per work item
  // 1-D grid of num_work x hsplit x Hkv: consecutive workgroups land on consecutive
  // XCDs, so kv head = id % Hkv keeps every workgroup of one kv head on one XCD (its
  // L2 holds that head's K/V; T1), and the work list runs heaviest (latest) blocks
  // first.  hsplit = 2 halves the heads per workgroup when the grid is small.
  const int num_work = gridDim.x / (Hkv * hsplit);
  const int kvh = blockIdx.x % Hkv;
  const int rest = blockIdx.x / Hkv;
  const int wi = num_work - 1 - rest / hsplit;
  const int seq = work_seq[wi];
  const int head = kvh * G + (rest % hsplit) * Gw + wid % Gw;
  const int qs = work_qblk[wi] * QB + (wid / Gw) * kQB;   // this wave's first query
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
  // keys the workgroup needs (its last query) and this wave needs
  const int wg_last_q = min(work_qblk[wi] * QB + QB, q_len) - 1;
  const int kv_end = min(kv_len, ctx0 + wg_last_q + 1);
  const int w_last_q = min(qs + kQB, q_len) - 1;
  const int w_kv_end = w_last_q < qs ? 0 : min(kv_len, ctx0 + w_last_q + 1);

  auto load = [&](int kt, s16x8* kr, s16x8* vr) {
    // the tile's two pages: wave-uniform block-table reads (scalar loads)
    const int pg0 = kt / kPPage;
    const int64_t page_a = bt[pg0];
    const int64_t page_b = kt + kPPage < kv_end ? bt[pg0 + 1] : page_a;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = threadIdx.x + NT * i, row = idx >> 4, ch = idx & 15;
      const int key = kt + row;
      kr[i] = vr[i] = (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
      if (key < kv_end) {
        const int64_t page = row < kPPage ? page_a : page_b;
        const int64_t off = ((page * Hkv + kvh) * kPPage + (key % kPPage)) * kPD;
        kr[i] = reinterpret_cast<const s16x8*>(k_cache + off)[ch];
        vr[i] = reinterpret_cast<const s16x8*>(v_cache + off)[ch];
      }
    }
  };
  auto store = [&](int buf, const s16x8* kr, const s16x8* vr) {
    bf16_t* kl = lds + buf * kStage;
    bf16_t* vl = kl + kKT * kPD;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = threadIdx.x + NT * i, row = idx >> 4, ch = idx & 15;
      reinterpret_cast<s16x8*>(kl + row * kPD)[ch ^ (row & 15)] = kr[i];
      reinterpret_cast<s16x8*>(vl + row * kPD)[ch ^ ((row & 3) << 2)] = vr[i];
    }
  };

  // online softmax state in raw score units (scale applied inside the exp2's FMA)
  float m_run = -INFINITY, l_run = 0.f;
  const float rescale_raw = kRescale / scale_log2;
  f32x16 o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[m][i] = 0.f;
  f32x16 s[2];                                 // S^T, then P^T, of the current tile

  // Ping-pong phases: the waves of group 1 run half a tile behind group 0, so in
  // every barrier interval one group's QK^T + softmax (VALU / transcendental) runs
  // beside the other group's PV MFMAs on the same SIMD instead of both groups
  // queueing for the same unit.  Phase p: group g works on half-tile p - g (stage 0 =
  // QK^T + softmax, stage 1 = PV).  Tile T+1 is loaded at phase 2T and written to the
  // other LDS buffer at the end of phase 2T+1, after both groups left tile T-1.
  const int grp = wid >= NW / 2 ? 1 : 0;
  const int ntiles = (kv_end + kKT - 1) / kKT;
  s16x8 kr[NCH], vr[NCH];
  // the second-dispatched half loses every VALU arbitration at equal priority: one
  // static s_setprio for it, no per-phase flips (MI355X_MICROARCH "Two waves per SIMD" 4)
  if (grp) __builtin_amdgcn_s_setprio(1);
  load(0, kr, vr);
  store(0, kr, vr);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int p = 0; p <= 2 * ntiles; ++p) {
    const int T = p >> 1;
    if (!(p & 1) && T + 1 < ntiles) load((T + 1) * kKT, kr, vr);   // in flight 2 phases
    const int tp = p - grp;
    const int t = tp >> 1, kt = t * kKT;
    if (tp >= 0 && t < ntiles && kt < w_kv_end) {
      const bf16_t* k_lds = lds + (t & 1) * kStage;
      const bf16_t* v_lds = k_lds + kKT * kPD;
      if (!(tp & 1)) {
        // ---- S^T for two 32-key subtiles ----
        // K fragments are read a whole subtile ahead of the MFMAs that use them: the
        // 8 reads of subtile 1 issue between subtile 0's MFMAs (each waits only for its
        // own fragment), so no MFMA waits out a full LDS round trip
        const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                               0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        auto kfrag = [&](int st, int ks) {
          const int row = 32 * st + r, ch = 2 * ks + h2;
          return reinterpret_cast<const s16x8*>(k_lds + row * kPD)[ch ^ (row & 15)];
        };
        s16x8 ka[8];
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) ka[ks] = kfrag(0, ks);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[ks]), as_bf16x8(qf[ks]),
                                                         ks == 0 ? zero16 : s[0], 0, 0, 0);
          ka[ks] = kfrag(1, ks);
        }
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
          s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[ks]), as_bf16x8(qf[ks]),
                                                         ks == 0 ? zero16 : s[1], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);   // 8 DS reads
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA ks of subtile 0
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // read ks of subtile 1
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);   // subtile 1
        // lane: S^T[key 32st + (i&3) + 8(i>>2) + 4h2][query r]
        if (kt + kKT > ctx0 + qs || kt + kKT > kv_end) {
#pragma unroll
          for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int key = kt + 32 * st + (i & 3) + 8 * (i >> 2) + 4 * h2;
              if (key > qpos || key >= kv_end) s[st][i] = -INFINITY;
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[st][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        // defer-max (T13): keep the running max -- and skip rescaling O -- unless a
        // row's max grew by more than kRescale (log2 units); p <= 2^kRescale meanwhile
        if (__any(mx > m_run + rescale_raw)) {
          const float m_new = fmaxf(m_run, mx);
          const float alpha = m_new == -INFINITY ? 1.f : fast_exp2((m_run - m_new) * scale_log2);
          l_run *= alpha;
#pragma unroll
          for (int m = 0; m < 4; ++m) o[m] *= alpha;
          m_run = m_new;
        }
        const float nb = m_run == -INFINITY ? 0.f : -m_run * scale_log2;
        float psum = 0.f;
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float pr = fast_exp2(fmaf(s[st][i], scale_log2, nb));
            s[st][i] = pr;
            psum += pr;
          }
        l_run += psum;
      } else {
        // ---- O^T += V^T P^T ----
        // 4 key chunks x 4 dh tiles; the V^T fragments of chunk c + 1 (8 transposing
        // reads) are in flight while chunk c's 4 MFMAs run
        const int gi = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
        auto vfrag = [&](int c, int m) {
          const int r0 = 16 * c + 4 * h2 + qq, r1 = r0 + 8;
          const int col = 32 * m + 16 * (gi & 1) + 4 * pp;
          const int ch = col >> 3, sub = col & 7;
          const s16x4 a0 = ds_read_tr16(v_lds + r0 * kPD + ((ch ^ ((r0 & 3) << 2)) << 3) + sub);
          const s16x4 a1 = ds_read_tr16(v_lds + r1 * kPD + ((ch ^ ((r1 & 3) << 2)) << 3) + sub);
          return (s16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        };
        s16x8 va[2][4];
#pragma unroll
        for (int m = 0; m < 4; ++m) va[0][m] = vfrag(0, m);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c < 3) {
#pragma unroll
            for (int m = 0; m < 4; ++m) va[(c + 1) & 1][m] = vfrag(c + 1, m);
          }
          float pv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) pv[j] = s[c >> 1][8 * (c & 1) + j];
          const s16x8 pb = pack8(pv);
#pragma unroll
          for (int m = 0; m < 4; ++m)
            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(va[c & 1][m]), as_bf16x8(pb),
                                                           o[m], 0, 0, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // chunks 0 and 1
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // chunk c
          if (c < 2) __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // chunk c + 2
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }
    if ((p & 1) && T + 1 < ntiles) store((T + 1) & 1, kr, vr);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS stores done; loads stay in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  // Epilogue (T21): the loop's last barrier has retired every K/V read, so each wave
  // stages its 32 x 128 O tile in its own 8 KB of LDS (16-B chunks XOR-swizzled by
  // row) and stores whole rows, 16 B per lane -- 8 dwordx4 row stores instead of 16
  // dwordx2 stores that each touch 32 rows.
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
}

// ---------------------------------------------------------------------------------
// v3: intra-wave overlap.  Every wave runs the same stream per 64-key tile t:
//   S = K(t+1) Q^T            16 MFMAs (K fragments a subtile ahead)
//   O^T += V(t)^T P(t)^T      16 MFMAs, with softmax(S) -> P(t+1) issued between them
// so the exp / max / sum chain of tile t+1 fills the issue slots the PV MFMAs leave
// (an MFMA holds the SIMD's vector issue for 8 of its 32 cycles) instead of running
// serially behind its own QK^T.  K/V sit in a 3-slot LDS ring: tile t+2 is written
// to the slot tile t-1 vacated, so ONE barrier per tile suffices; its global loads
// are issued a whole tile earlier (T14).
constexpr int kSlots = 4;
typedef __attribute__((address_space(3))) char lds_c;
typedef __attribute__((address_space(3))) const s16x8 lds_s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_prefill_v3_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_q_start, const int32_t* __restrict__ seq_q_len,
    const int32_t* __restrict__ seq_kv_len, const int32_t* __restrict__ work_seq,
    const int32_t* __restrict__ work_qblk, bf16_t* __restrict__ out, int64_t out_stride, int Hq,
    int Hkv, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);
  constexpr int NT = NW * 64;
  constexpr int NCH = kKT * 16 / NT;

  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h2 = lane >> 5;
  const int G = Hq / Hkv;
  const int QB = NW * kQB / G;
  const int num_work = gridDim.x / Hkv;
  const int kvh = blockIdx.x % Hkv;
  const int wi = num_work - 1 - blockIdx.x / Hkv;
  const int seq = work_seq[wi];
  const int head = kvh * G + wid % G;
  const int qs = work_qblk[wi] * QB + (wid / G) * kQB;
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
  // S^T of tile t (lane: S^T[key 32st + (i&3) + 8(i>>2) + 4h2][query r]), masked
  // LDS addressing: per-lane byte offsets are loop-invariant (8 for K, 4 for V); each
  // tile adds its slot base once per offset behind an opaque asm, so the subtile /
  // key-chunk steps fold into the ds_read immediates instead of the compiler hoisting
  // every (offset + constant) combination into its own VGPR
  uint32_t koff[8], voff[4];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) koff[ks] = r * 256 + ((((2 * ks + h2) ^ (r & 15))) << 4);
  const int gi = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int col = 32 * m + 16 * (gi & 1) + 4 * pp;
    voff[m] = kKT * kPD * 2 + (4 * h2 + qq) * 256 + ((((col >> 3) ^ (qq << 2)) << 3) + (col & 7)) * 2;
  }
  auto slot = [&](int t) { return lbase + (t % kSlots) * (kStage * 2); };
  auto qk = [&](int t) {
    lds_c* const sl = slot(t);
    lds_c* kp[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      kp[ks] = sl + koff[ks];
      asm volatile("" : "+v"(kp[ks]));
    }
    s16x8 ka[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) ka[ks] = *(const lds_s16x8*)(kp[ks]);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[ks]), as_bf16x8(qf[ks]),
                                                     ks == 0 ? zero16 : s[0], 0, 0, 0);
      ka[ks] = *(const lds_s16x8*)(kp[ks] + 32 * 256);
    }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ka[ks]), as_bf16x8(qf[ks]),
                                                     ks == 0 ? zero16 : s[1], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
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
    lds_c* vp[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      vp[m] = sl + voff[m];
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
  load(0);
  if (ntiles > 1) load(1);
  if (ntiles > 2) load(2);
  wait_dma(ntiles > 2);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wt > 0) {
    qk(0);
    sm_max();
#pragma unroll
    for (int c = 0; c < 4; ++c) sm_exp(c, pb);
    sm_done();
  }
  for (int t = 0; t < ntiles; ++t) {
    if (t + 3 < ntiles) load(t + 3);
    if (t < wt) {
      if (t + 1 < wt) {
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
    wait_dma(t + 3 < ntiles);                   // tile t+2 landed (tile t+3 may fly)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  float l_tot = l_run + __shfl_xor(l_run, 32, 64);
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
}

// qblk: queries per work item (the packer's prefill block): NW = qblk * G / 32 waves.
void launch_attn_prefill(const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                         const bf16_t* v_cache, const int32_t* block_tables, int bt_stride,
                         const int32_t* seq_q_start, const int32_t* seq_q_len,
                         const int32_t* seq_kv_len, const int32_t* work_seq,
                         const int32_t* work_qblk, int num_work, bf16_t* out, int64_t out_stride,
                         int Hq, int Hkv, float scale, int qblk, hipStream_t s) {
  if (num_work == 0) return;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  // hsplit = 2 (half the query heads per workgroup, twice the workgroups) measured
  // slower at B = 1 (S 2048: 104 vs 89 us; profiles/r2_prefill_attention.md): a small
  // grid here is bound by its heaviest causal block's latency, not by idle CUs
  const int hsplit = 1;
  const int nw = qblk * G / (kQB * hsplit);
  dim3 grid(num_work * Hkv * hsplit);
  const size_t lds = 2 * kStage * sizeof(bf16_t);
  static const int variant = [] {
    const char* e = getenv("RFQ_PREFILL_V");
    return e ? atoi(e) : 3;
  }();

  if (variant == 3) {
    const size_t lds3 = kSlots * kStage * sizeof(bf16_t);
    if (nw == 8)
      attn_prefill_v3_kernel<8><<<grid, 512, lds3, s>>>(
          q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_q_start, seq_q_len,
          seq_kv_len, work_seq, work_qblk, out, out_stride, Hq, Hkv, scale_log2);
    else
      attn_prefill_v3_kernel<4><<<grid, 256, lds3, s>>>(
          q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_q_start, seq_q_len,
          seq_kv_len, work_seq, work_qblk, out, out_stride, Hq, Hkv, scale_log2);
    return;
  }
  if (nw == 8)
    attn_prefill_kernel<8><<<grid, 512, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                  bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                  work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                  scale_log2, hsplit);
  else
    attn_prefill_kernel<4><<<grid, 256, lds, s>>>(q, q_stride, k_cache, v_cache, block_tables,
                                                  bt_stride, seq_q_start, seq_q_len, seq_kv_len,
                                                  work_seq, work_qblk, out, out_stride, Hq, Hkv,
                                                  scale_log2, hsplit);
}

}  // namespace rfq
