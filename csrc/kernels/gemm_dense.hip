// Dense large-M projection GEMM for the throughput path (SURVEY.md §2.4 K3/K8/K9/K11,
// with K10 SwiGLU fused into K9's epilogue):
//
//   out[M, N]  = x[M, K] . w[N, K]^T                      (EPI_STORE)
//   act[M, F]  = silu(x . Wg^T) * (x . Wu^T),  w = [Wg; Wu] [2F, K]   (EPI_SWIGLU)
//
// Both operands are K-contiguous (torch Linear layout), bf16 in, fp32 accumulate,
// bf16 out.  This is the implied compute behind /root/reference/app/rfq_agent.py:163
// for every engine step of more than ~64 tokens (prefill chunks, batched decode +
// jump-forward extends).
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", re-derived for
// mfma_f32_32x32x16_bf16 and a 2-stage LDS ring):
//  * tile 256 (x rows) x 256 (w rows) x 64 (k); 512 threads = 8 waves.  Wave
//    (g = wid >> 2, wn = wid & 3) owns x rows [128 g, +128) and w rows [64 wn, +64):
//    8 accumulators of 32 x 32 (128 AGPR/VGPR per lane).  Operands are swapped
//    (C^T = W X^T) so a lane holds 4 consecutive output columns (8-byte stores), and
//    with SWIGLU the gate and up values of the same output element.
//  * Each K-tile is 4 "quadrant" phases per wave: (x 64 rows) x (w 32 rows) x k64 =
//    8 MFMAs; fragments: x(m0)+w(n0), w(n1), x(m1), - (24 ds_read_b128 per tile).
//  * Every phase is a read segment R (ds_reads + 2 LDS-DMA pieces) and a matrix
//    segment M (lgkmcnt(0), 8 MFMAs at s_setprio 1), each closed by a raw s_barrier.
//    Waves 4-7 start one segment late (one extra barrier), so on every SIMD one wave
//    multiplies while its partner reads and stages -- the ping-pong of the template.
//  * LDS: 2 stages x {XA, XB, W0, W1} half-tiles of [128 rows][64 k] (16 KB each,
//    128 KB total, one dynamic __shared__ array).  Chunk ch of row r is stored at
//    ch ^ ((r >> 1) & 7) (conflict-free ds_read_b128 for the 32x32x16 operand lane
//    groups); LDS-DMA writes lane-linearly, so the swizzle is applied on the source.
//  * The 64 one-KB DMA pieces of a K-tile are spread two per wave per R segment; each
//    piece is issued at least two segments after the last read of the buffer it
//    overwrites and retired by the issuing wave's counted vmcnt before the barrier
//    that precedes its first reader (the schedule and the counts are derived in
//    docs/GEMM_DENSE.md; the last two K-tiles wait vmcnt(0)).
//  * Block order: bijective XCD remap, then groups of 16 row-tiles swept w-tile by
//    w-tile, so the blocks that share a weight panel run together on one XCD's L2.
// Shapes: K % 64 == 0, N % 256 == 0 (F % 128 with SWIGLU), any M >= 1 (rows past M
// read row M-1 and are not stored), 16-byte aligned rows.
#include <type_traits>

#include "common.h"

namespace rfq {

constexpr int kGM = 256, kGN = 256, kGK = 64;
constexpr int kGHalf = 128 * kGK;                 // bf16 elements per half-tile image
constexpr int kGStage = 4 * kGHalf;               // XA, XB, W0, W1
constexpr int kGLds = 2 * kGStage * 2;            // bytes (2 stages)
constexpr int kGroupM = 16;                       // row-tiles per L2 group

enum : int { EPI_STORE = 0, EPI_SWIGLU = 1 };

__device__ __forceinline__ void gbar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// Grouped form (GROUPED, Mixtral's routed experts): x = the
// expert-sorted, 128-row-padded gathered rows (moe_align / moe_gather), w = [E, N, K],
// expert_offsets[E+1] = padded row offsets.  A tile is two consecutive 128-row blocks
// of ONE expert (the second absent when the expert has an odd block count: its rows
// are neither loaded past the buffer nor stored); live tiles are enumerated
// expert-major from the device-side offsets, so no host sync and a fixed grid.
// TLW: w is stored in the decode-tiled layout of the split-K GEMVs (ops.tile_weight;
// gemm_skinny.hip TL), for models that keep only that copy of a projection.  A 16-byte
// chunk (row, k0 + 8 gch) of a 64-deep K-tile then sits at
//   (row >> 4) K/128 2048 + (row & 15) 8 + (gch >> 2) 512 + (gch & 3) 128
//   + (k0 >> 7) 2048 + ((k0 >> 6) & 1) 1024,
// i.e. a per-lane base plus a K-tile term; the LDS image and everything after the DMA
// are unchanged, so the result is bit-identical to the row-major kernel.
template <int EPI, int MF, int PH, int ABL = 0, bool GROUPED = false, bool TLW = false>
__global__ __launch_bounds__(512) void gemm_dense_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ w, int64_t ldw,
    bf16_t* __restrict__ out, int64_t ldo, int M, int K, int up_off, int tiles_m, int tiles_n,
    const int32_t* __restrict__ expert_offsets, int E, int64_t w_estride) {
  extern __shared__ __attribute__((aligned(16))) char smem_g[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem_g);

  // ---- block -> (row tile, weight tile)
  int row0, tn, m_load, m_store;           // first row, w tile, rows readable / stored
  const bf16_t* xt;
  const bf16_t* wt = w;
  if constexpr (GROUPED) {
    constexpr int kB = 128;
    int nchunks = 0;
    for (int e = 0; e < E; ++e)
      nchunks += ((expert_offsets[e + 1] - expert_offsets[e]) / kB + 1) >> 1;
    const int nlive = nchunks * tiles_n;
    const int bid = blockIdx.x;
    if (bid >= nlive) return;                // before any barrier: the whole block leaves
    const int q8 = nlive >> 3, r8 = nlive & 7, xg = bid & 7;
    const int wg = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + (bid >> 3);
    // expert-major, then weight tile, then 256-row chunk: the chunks sharing a weight
    // tile run back to back on one XCD (the remap above) and hit its L2
    int e = 0, p0 = 0, s0 = 0, nbe = 0, che = 0;
    for (; e < E; ++e) {
      s0 = expert_offsets[e] / kB;
      nbe = expert_offsets[e + 1] / kB - s0;
      che = (nbe + 1) >> 1;
      if (wg < (p0 + che) * tiles_n) break;
      p0 += che;
    }
    if (e >= E) return;
    const int local = wg - p0 * tiles_n;
    tn = local / che;
    const int chunk = local % che;
    row0 = (s0 + 2 * chunk) * kB;
    const bool two = 2 * chunk + 1 < nbe;
    m_store = two ? 256 : 128;
    m_load = min(expert_offsets[E] - row0, 256);
    xt = x + (int64_t)row0 * ldx;
    wt = w + (int64_t)e * w_estride;
  } else {
    const int nwg = tiles_m * tiles_n;
    const int bid = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xg = bid & 7;
    const int wg = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + (bid >> 3);
    const int per_group = kGroupM * tiles_n;
    const int gid = wg / per_group, first_m = gid * kGroupM;
    const int gm = min(tiles_m - first_m, kGroupM);
    const int rin = wg - gid * per_group;
    const int tm = first_m + rin % gm;
    tn = rin / gm;
    row0 = tm * kGM;
    m_load = m_store = min(M - row0, 256);
    xt = x + (int64_t)row0 * ldx;
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, wn = wid & 3;
  const int r = lane & 31, h2 = lane >> 5;

  // ---- LDS-DMA pieces of this wave (per K-tile): 8 pieces of 8 rows x 128 B, issued
  // PH = 4: two per R segment (slot = segment);  PH = 2: four per R segment.
  //   PH 4  g0: R1 W[24+2wn..]  R2 XA[8+2wn..]  R3 XB[8+2wn..]  R4 W[8+2wn..]
  //         g1: R1 XA[2wn..]    R2 XB[2wn..]    R3 W[2wn..]     R4 W[16+2wn..]
  //   PH 2  g0: R1 W[16+4wn..]  R2 XB[4wn..]
  //         g1: R1 XA[4wn..]    R2 W[4wn..]
  // W pieces 0..15 are half W0 (tile rows 0..127), 16..31 half W1.
  constexpr int PPS = 8 / PH;                      // pieces per R segment per wave
  const int prow = lane >> 3, pch = lane & 7;
  int src_off[8];             // element offset from the x / w tile base (+ k0)
  int dst_off[8];             // bf16 element offset inside a stage (wave-uniform)
  bool src_is_w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int seg = i / PPS, pp = i % PPS;
    int half, piece;          // half: 0 XA, 1 XB, 2 W (piece 0..31 over W0|W1)
    if constexpr (PH == 4) {
      if (g == 0) {
        if (seg == 0) { half = 2; piece = 24 + 2 * wn + pp; }
        else if (seg == 1) { half = 0; piece = 8 + 2 * wn + pp; }
        else if (seg == 2) { half = 1; piece = 8 + 2 * wn + pp; }
        else { half = 2; piece = 8 + 2 * wn + pp; }
      } else {
        if (seg == 0) { half = 0; piece = 2 * wn + pp; }
        else if (seg == 1) { half = 1; piece = 2 * wn + pp; }
        else if (seg == 2) { half = 2; piece = 2 * wn + pp; }
        else { half = 2; piece = 16 + 2 * wn + pp; }
      }
    } else {
      if (g == 0) {
        if (seg == 0) { half = 2; piece = 16 + 4 * wn + pp; }
        else { half = 1; piece = 4 * wn + pp; }
      } else {
        if (seg == 0) { half = 0; piece = 4 * wn + pp; }
        else { half = 2; piece = 4 * wn + pp; }
      }
    }
    const int prow_in_half = (piece & 15) * 8 + prow;          // row inside its half
    const int gch = pch ^ ((prow_in_half >> 1) & 7);            // source chunk
    if (half < 2) {
      int row = half * 128 + prow_in_half;                      // inside the tile
      row = row < m_load ? row : m_load - 1;
      src_off[i] = row * (int)ldx + 8 * gch;                    // from the x tile base
      dst_off[i] = half * kGHalf + (piece & 15) * 512;
      src_is_w[i] = false;
    } else {
      const int j = piece * 8 + prow;                           // w tile row 0..255
      int wrow;
      if constexpr (EPI == EPI_SWIGLU) {
        const int v = j >> 6, hh = (j >> 5) & 1, c = j & 31;   // wave v: 32 gate + 32 up
        wrow = (hh ? up_off : 0) + tn * 128 + 32 * v + c;
      } else {
        wrow = tn * kGN + j;
      }
      src_off[i] = TLW ? (wrow >> 4) * (K >> 7) * 2048 + (wrow & 15) * 8 + (gch >> 2) * 512 +
                             (gch & 3) * 128
                       : wrow * (int)ldw + 8 * gch;             // from w (this expert's)
      dst_off[i] = (2 + (piece >> 4)) * kGHalf + (piece & 15) * 512;
      src_is_w[i] = true;
    }
  }

  auto issue = [&](int slot, int stage, int k0) {
    bf16_t* st = lds + stage * kGStage;
#pragma unroll
    for (int pp = 0; pp < PPS; ++pp) {
      const int i = PPS * slot + pp;
      const int kk = (TLW && src_is_w[i]) ? (k0 >> 7) * 2048 + ((k0 >> 6) & 1) * 1024 : k0;
      const bf16_t* src = (src_is_w[i] ? wt : xt) + src_off[i] + kk;
      __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(st + dst_off[i]), 16, 0, 0);
    }
  };

  // ---- fragments.  MF = 32: mfma_f32_32x32x16_bf16, lane (r = l & 31, h2 = l >> 5) holds
  // row r, chunk 2 ks + h2 of a 32-row subtile; MF = 16: mfma_f32_16x16x32_bf16, lane
  // (rr = l & 15, q = l >> 4) holds row rr, chunk 4 ks + q of a 16-row subtile.  Either
  // way the chunk lives at chunk ^ ((row >> 1) & 7) and the subtile base row is a
  // multiple of 16, so the per-lane offset of each k-step is a constant.
  constexpr int KS = MF == 32 ? 4 : 2;             // k-steps per 64-deep tile
  constexpr int XS = 64 / MF;                      // x subtiles per 64-row quadrant
  constexpr int WS = 32 / MF;                      // w subtiles per 32-row quadrant
  typedef typename std::conditional<MF == 32, f32x16, f32x4>::type acc_t;
  int frag_off[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if constexpr (MF == 32)
      frag_off[ks] = r * kGK + 8 * ((2 * ks + h2) ^ ((r >> 1) & 7));
    else
      frag_off[ks] = (lane & 15) * kGK + 8 * ((4 * ks + (lane >> 4)) ^ (((lane & 15) >> 1) & 7));
  }
  const int xa_base = g * kGHalf;                                    // x half of this wave
  const int wa_base = (2 + (wn >> 1)) * kGHalf + (wn & 1) * 64 * kGK; // w rows of this wave

  acc_t acc[2 * WS][2 * XS];          // [w subtile][x subtile] of the wave's 64 x 128
#pragma unroll
  for (int i = 0; i < 2 * WS; ++i)
#pragma unroll
    for (int j = 0; j < 2 * XS; ++j)
#pragma unroll
      for (int q = 0; q < (MF == 32 ? 16 : 4); ++q) acc[i][j][q] = 0.f;

  s16x8 xf[XS][KS];           // x fragments of the current m-quadrant: [subtile][k-step]
  s16x8 wf[2][WS][KS];        // w fragments: [n-quadrant][subtile][k-step]

  auto read_x = [&](const bf16_t* st, int mq) {
#pragma unroll
    for (int j = 0; j < XS; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        xf[j][ks] = *reinterpret_cast<const s16x8*>(st + xa_base + (mq * 64 + MF * j) * kGK +
                                                    frag_off[ks]);
  };
  auto read_w = [&](const bf16_t* st, int nq) {
#pragma unroll
    for (int i = 0; i < WS; ++i)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        wf[nq][i][ks] = *reinterpret_cast<const s16x8*>(st + wa_base + (nq * 32 + MF * i) * kGK +
                                                        frag_off[ks]);
  };
  auto mma = [&](int nq, int mq) {      // (the compiler waits for the fragments' lgkmcnt)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < WS; ++i)
#pragma unroll
        for (int j = 0; j < XS; ++j) {
          acc_t& c = acc[nq * WS + i][mq * XS + j];
          if constexpr (MF == 32)
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wf[nq][i][ks]),
                                                        as_bf16x8(xf[j][ks]), c, 0, 0, 0);
          else
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wf[nq][i][ks]),
                                                        as_bf16x8(xf[j][ks]), c, 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  // (diagnostic ablations only: keep the fragments live without reading LDS)
  auto opaque_frags = [&]() {
#pragma unroll
    for (int j = 0; j < XS; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(xf[j][ks]));
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < WS; ++i)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(wf[n][i][ks]));
  };

  const int nk = K / kGK;
  if constexpr (PH == 4) {
  // ---- prologue: tile 0 whole (every wave its 8 pieces), then the W pieces of tile 1
  // that the steady state issues in period -1 (g1: R3 and R4 slots, g0: R4 slot)
#pragma unroll
  for (int s = 0; s < 4; ++s) issue(s, 0, 0);
  if (nk > 1) {
    if (g == 1) { issue(2, 1, kGK); issue(3, 1, kGK); }
    else issue(3, 1, kGK);
    if (g == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  gbar();
  if (g == 1) gbar();                               // stagger waves 4-7 by one segment

  for (int t = 0; t < nk; ++t) {
    const bf16_t* cur = lds + (t & 1) * kGStage;
    const int nxt = (t + 1) & 1;
    const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
    const bool steady = has2;
    const int k1 = (t + 1) * kGK, k2 = (t + 2) * kGK;
    // R1: x(m0) + w(n0); DMA slot 0 (tile t+1)
    read_x(cur, 0);
    read_w(cur, 0);
    if (has1) issue(0, nxt, k1);
    if (g == 0) {
      if (steady) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gbar();
    mma(0, 0);                                      // M1
    gbar();
    read_w(cur, 1);                                 // R2; slot 1 (tile t+1)
    if (has1) issue(1, nxt, k1);
    gbar();
    mma(1, 0);                                      // M2
    gbar();
    read_x(cur, 1);                                 // R3; slot 2 (g0: tile t+1, g1: t+2)
    if (g == 0) { if (has1) issue(2, nxt, k1); }
    else { if (has2) issue(2, t & 1, k2); }
    gbar();
    mma(1, 1);                                      // M3
    gbar();
    if (has2) issue(3, t & 1, k2);                  // R4: slot 3 (tile t+2)
    if (g == 1) {
      if (steady) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gbar();
    mma(0, 1);                                      // M4
    if (steady) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    gbar();
  }
  if (g == 0) gbar();                               // balance the stagger barrier
  } else {
  // ---- PH = 2: R1 = x(m0) + w(n0, n1), M1 = (n0, m0), (n1, m0); R2 = x(m1), M2 = (n*, m1).
  // Per period t: g0 R1 issues W[16..31] of tile t+1, R2 XB of t+1; g1 R1 XA of t+1,
  // R2 W[0..15] of t+2.  Waits: g0 end of R1 and end of M2 vmcnt(4), g1 end of R2
  // vmcnt(4) (docs/GEMM_DENSE.md).  Prologue: tile 0 whole, then g1's period -1 slot.
  issue(0, 0, 0);
  issue(1, 0, 0);
  if (nk > 1 && g == 1) {
    issue(1, 1, kGK);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  gbar();
  if (g == 1) gbar();                               // stagger waves 4-7 by one segment
  for (int t = 0; t < nk; ++t) {
    const bf16_t* cur = lds + (t & 1) * kGStage;
    const int nxt = (t + 1) & 1;
    const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
    const bool steady = has2;
    const int k1 = (t + 1) * kGK, k2 = (t + 2) * kGK;
    if constexpr (!(ABL & 4)) {                     // R1
      read_x(cur, 0);
      read_w(cur, 0);
      read_w(cur, 1);
    } else {
      opaque_frags();
    }
    if (has1 && !(ABL & 2)) issue(0, nxt, k1);
    if (g == 0) {
      if (steady) { if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gbar();
    mma(0, 0);                                      // M1
    mma(1, 0);
    gbar();
    if constexpr (!(ABL & 4)) read_x(cur, 1);       // R2
    else opaque_frags();
    if (g == 0) { if (has1 && !(ABL & 2)) issue(1, nxt, k1); }
    else {
      if (has2 && !(ABL & 2)) issue(1, t & 1, k2);
      if (steady) { if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gbar();
    mma(1, 1);                                      // M2 (n1 first: w(n1) is the newest)
    mma(0, 1);
    if (g == 0) {
      if (steady) { if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gbar();
  }
  if (g == 0) gbar();                               // balance the stagger barrier
  }

  // ---- epilogue.  C^T lane layout -- MF 32: w row (q&3) + 8(q>>2) + 4 h2 of the
  // subtile, x row r; MF 16: w row 4 (l >> 4) + q, x row l & 15.  Either way each
  // group of 4 registers is 4 consecutive output columns of one row (8-byte store).
  constexpr int NG = MF == 32 ? 4 : 1;             // 4-register groups per accumulator
#pragma unroll
  for (int j = 0; j < 2 * XS; ++j) {
    const int trow = g * 128 + MF * j + (MF == 32 ? r : (lane & 15));
    if (trow >= m_store) continue;
    const int row = row0 + trow;
    const int lane_col = MF == 32 ? 4 * h2 : 4 * (lane >> 4);
    if constexpr (EPI == EPI_SWIGLU) {
      bf16_t* orow = out + (int64_t)row * ldo + tn * 128 + 32 * wn + lane_col;
#pragma unroll
      for (int i = 0; i < WS; ++i)                 // gate subtile i, up subtile WS + i
#pragma unroll
        for (int q4 = 0; q4 < NG; ++q4) {
          float o[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float gf = bf2f(f2bf(acc[i][j][4 * q4 + u]));    // = the gate GEMM's bf16
            const float sg = gf / (1.f + __expf(-gf));
            o[u] = bf2f(f2bf(sg)) * bf2f(f2bf(acc[WS + i][j][4 * q4 + u]));
          }
          uint2 v;
          v.x = pack_bf16x2(o[0], o[1]);
          v.y = pack_bf16x2(o[2], o[3]);
          *reinterpret_cast<uint2*>(orow + MF * i + 8 * q4) = v;
        }
    } else {
      bf16_t* orow = out + (int64_t)row * ldo + tn * kGN + 64 * wn + lane_col;
#pragma unroll
      for (int i = 0; i < 2 * WS; ++i)
#pragma unroll
        for (int q4 = 0; q4 < NG; ++q4) {
          uint2 v;
          v.x = pack_bf16x2(acc[i][j][4 * q4 + 0], acc[i][j][4 * q4 + 1]);
          v.y = pack_bf16x2(acc[i][j][4 * q4 + 2], acc[i][j][4 * q4 + 3]);
          *reinterpret_cast<uint2*>(orow + MF * i + 8 * q4) = v;
        }
    }
  }
}

void launch_gemm_w4(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, int, int,
                    int, int, bool, int, hipStream_t);

// out = x w^T ([M, N]) or, swiglu, act = silu(x Wg^T) * (x Wu^T) ([M, F], w = [2F, K],
// up rows at up_off = F).  n_out = N or F.
void launch_gemm_dense(const bf16_t* x, int64_t ldx, const bf16_t* w, int64_t ldw, bf16_t* out,
                       int64_t ldo, int M, int n_out, int K, int up_off, bool swiglu, int cfg,
                       hipStream_t s) {
  if (M <= 0) return;
  const int tiles_m = (M + kGM - 1) / kGM;
  const int tiles_n = swiglu ? n_out / 128 : n_out / kGN;
  const int grid = tiles_m * tiles_n;
  // cfg bit 3: the one-wave-per-SIMD kernel (gemm_w4.hip; K % 128 == 0); with bits 4-6
  // its diagnostic timing builds (WRONG results): 16 no DMA, 32 no fragment reads, 64 no
  // waits / barriers in the K loop; 128: the DMA pieces spread over all 16 MFMA groups;
  // bits 8-9: row tiles per L2 group (16, 8, 4, 32); bit 10 (with 128): fragment reads
  // early in each half; bit 11 (with 128 | 1024): the 32x32x16 MFMA form; bit 12 (with
  // 128 | 1024, not 2048): the weight image in three LDS slots, the activations in two;
  // bit 13 (with 4096, K % 256 == 0): the persistent form (gemm_w4p_kernel); bit 14 (with
  // 8192): stream-K over its last rounds (30344 = 13960 | 16384)
  if (cfg & 8) {
    launch_gemm_w4(x, ldx, w, ldw, out, ldo, M, n_out, K, up_off, swiglu, (cfg >> 4) & 2047, s);
    return;
  }
  // cfg bit 0: the 32x32x16 MFMA variant (else 16x16x32); bit 1: 2 phases per K-tile;
  // bit 2: w in the decode-tiled layout (16x16x32, 2 phases)
#define RFQ_GD_LAUNCH(E, F, P) \
  gemm_dense_kernel<E, F, P><<<grid, 512, kGLds, s>>>(x, ldx, w, ldw, out, ldo, M, K, up_off, \
                                                      tiles_m, tiles_n, nullptr, 0, 0)
#define RFQ_GD_EPI(E)                                                  \
  switch (cfg & 3) {                                                   \
    case 0: RFQ_GD_LAUNCH(E, 16, 4); break;                            \
    case 1: RFQ_GD_LAUNCH(E, 32, 4); break;                            \
    case 2: RFQ_GD_LAUNCH(E, 16, 2); break;                            \
    default: RFQ_GD_LAUNCH(E, 32, 2); break;                           \
  }
  // cfg bits 4-6 (diagnostic timing builds, WRONG results): 16 = no counted vmcnt
  // waits, 32 = no DMA in the loop, 64 = no fragment reads (16x16x32, 2 phases only)
  const int abl = (cfg >> 4) & 7;
  if (abl && !swiglu) {
#define RFQ_GD_ABL(A) \
    gemm_dense_kernel<EPI_STORE, 16, 2, A><<<grid, 512, kGLds, s>>>(x, ldx, w, ldw, out, ldo, M, \
                                                                  K, up_off, tiles_m, tiles_n, \
                                                                  nullptr, 0, 0)
    switch (abl) {
      case 1: RFQ_GD_ABL(1); break;
      case 2: RFQ_GD_ABL(2); break;
      case 3: RFQ_GD_ABL(3); break;
      case 4: RFQ_GD_ABL(4); break;
      default: RFQ_GD_ABL(6); break;
    }
#undef RFQ_GD_ABL
    return;
  }
  if (cfg & 4) {   // w in the decode-tiled layout (16x32 MFMA, 2 phases per K-tile)
    if (swiglu)
      gemm_dense_kernel<EPI_SWIGLU, 16, 2, 0, false, true><<<grid, 512, kGLds, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, nullptr, 0, 0);
    else
      gemm_dense_kernel<EPI_STORE, 16, 2, 0, false, true><<<grid, 512, kGLds, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, nullptr, 0, 0);
    return;
  }
  if (swiglu) { RFQ_GD_EPI(EPI_SWIGLU) } else { RFQ_GD_EPI(EPI_STORE) }
#undef RFQ_GD_EPI
#undef RFQ_GD_LAUNCH
}

// Grouped (MoE) form: x = [rows, K] expert-sorted 128-row-padded rows, w = [E, N, K],
// expert_offsets [E+1] (device, padded row offsets), max_blocks = rows / 128.  swiglu:
// N = 2F (gate | up per expert), out [rows, F].  Fixed grid for graph capture.
void launch_gemm_grouped(const bf16_t* x, const bf16_t* w, bf16_t* out,
                         const int32_t* expert_offsets, int max_blocks, int n_out, int K, int E,
                         int64_t w_rows, bool swiglu, hipStream_t s) {
  if (max_blocks <= 0) return;
  const int tiles_n = swiglu ? n_out / 128 : n_out / kGN;
  const int chunks = (max_blocks + E) / 2 + 1;    // live 256-row tiles <= this
  const int grid = chunks * tiles_n;
  const int64_t estride = w_rows * K;
  if (swiglu)
    gemm_dense_kernel<EPI_SWIGLU, 16, 2, 0, true><<<grid, 512, kGLds, s>>>(
        x, K, w, K, out, n_out, max_blocks * 128, K, n_out, 0, tiles_n, expert_offsets, E, estride);
  else
    gemm_dense_kernel<EPI_STORE, 16, 2, 0, true><<<grid, 512, kGLds, s>>>(
        x, K, w, K, out, n_out, max_blocks * 128, K, n_out, 0, tiles_n, expert_offsets, E, estride);
}

}  // namespace rfq
