// Dense large-M projection GEMM, one wave per SIMD (the throughput path's hipBLASLt
// replacement candidate; SURVEY.md §2.4 K3/K8/K9/K11, K10 SwiGLU in the epilogue):
//
//   out[M, N] = x[M, K] . w[N, K]^T                         (kW4Store)
//   act[M, F] = silu(x . Wg^T) * (x . Wu^T), w = [Wg; Wu]    (kW4Swiglu, up rows at up_off)
//
// gemm_dense.hip's 8-wave ping-pong parks a quarter of its wave cycles at barriers and
// tops out at 1.67 PF/s with no memory traffic at all (profiles/r3_gemm_dense.md).  This
// kernel is the other structure: 4 waves per 256 x 256 tile, each wave alone on its SIMD
// with a 128 x 128 quadrant of the output in 64 16x16 fp32 accumulators (256 registers,
// AGPRs), so nothing but its own instruction stream competes for the SIMD, and one
// barrier per 32-deep K-step.
//
//  * K-step = 32.  LDS: 4 stages x {W image, X image} of [256 rows][32 k] bf16 (16 KB
//    each, 128 KB).  Row rho's 16-byte chunk c sits at chunk c ^ ((rho >> 2) & 3): the 16
//    lanes of a ds_read_b128 quarter (16 rows, one chunk) hit 16 distinct 4-bank groups.
//    LDS-DMA (global_load_lds_dwordx4) writes lane-linearly, so the swizzle is applied
//    to the per-lane source column.
//  * Step t: wait for stage t+1's DMA (own pieces: vmcnt leaving step t+2's 8 pieces in
//    flight), one barrier (every wave's pieces landed; every wave has consumed the
//    stage that step t+3's DMA overwrites), then 16 groups of [one ds_read_b128 of step
//    t+1's fragments, one DMA piece of step t+3 (first 8 groups), four MFMAs of step t on
//    the fragments read during step t-1].  The DMA runs 2 steps (128 MFMAs per wave)
//    ahead of its first reader; the fragment reads one step.
//  * Fragment reads are inline-asm ds_read_b128 with an lgkmcnt(0) at the top of the
//    next step tied to the destination registers (through the builtin the compiler
//    guards LDS reads with vmcnt(0) against the in-flight DMA: it cannot tell the
//    stages apart, and that would drain the prefetch every step).
//  * MFMA operands are swapped (C^T = W X^T, as gemm_dense): a lane holds 4 consecutive
//    output columns of one row (8-byte stores), and with SwiGLU the wave's W rows are 64
//    gate + the matching 64 up rows, so gate and up of an output meet in one lane.
//  * Block order: bijective XCD remap, then groups of 16 row-tiles swept w-tile by
//    w-tile (blocks sharing a weight panel run together on one XCD's L2).
// Shapes: K % 128 == 0, N % 256 == 0 (F % 128 with SwiGLU), any M >= 1 (rows past M read
// row M-1 and are not stored), 16-byte aligned rows.
#include <mutex>
#include <type_traits>

#include "common.h"

namespace rfq {

constexpr int kW4M = 256, kW4N = 256, kW4K = 64;
constexpr int kW4Stages = 2;
constexpr int kW4Img = 256 * kW4K;                 // bf16 elements per operand image
constexpr int kW4StageB = 2 * kW4Img * 2;          // bytes per stage (W then X)
constexpr int kW4Lds = kW4Stages * kW4StageB;      // 128 KB

enum : int { kW4Store = 0, kW4Swiglu = 1 };

typedef __attribute__((address_space(3))) char w4_lds_c;

#define W4_READ(DST, ADDR, OFF) \
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(DST) : "v"(ADDR), "i"(OFF))

// ABL (diagnostic timing builds, WRONG results): 1 = no DMA in the K loop, 2 = no
// fragment reads in the K loop (registers kept live), 4 = no vmcnt wait / barrier.
// SPREAD: the 16 DMA pieces of half 1 go out one per MFMA group over all 16 groups (the
// texture path takes ~16-23 cycles per 1 KB piece; two per group in the first 8 groups
// back the wave's issue up behind it), at the cost of a shorter landing window for the
// last pieces.
// EARLY: the 16 fragment reads of a half go out two per group in its first 8 groups (the
// last one then has 8 groups = 32 MFMAs to land before the next half's lgkmcnt(0));
// otherwise one per group over all 16.
// MF: 16 = mfma_f32_16x16x32_bf16 (a wave's quadrant = 8 x 8 accumulators of 16 x 16),
// 32 = mfma_f32_32x32x16_bf16 (4 x 4 of 32 x 32).  A 32x32x16 MFMA holds the SIMD for 32
// cycles, twice the 16x16x32's 16, so a DMA piece's issue (~16-23 cycles) hides behind
// one MFMA instead of stalling the pipe.
// W3 (MF 16 with SPREAD + EARLY): the W image gets three LDS slots and the X image two
// (160 KB): W pieces go out two K-tiles ahead of their first reader instead of one
// (the weights are the operand that misses L2; a panel of activations is shared by
// every weight tile of its row group).
// GROUPED (Mixtral's routed experts, the gemm_dense.hip grouped form's contract): x =
// the expert-sorted, 128-row-padded gathered rows (moe_align / moe_gather), w = [E, N,
// K] (expert stride w_estride elements), expert_offsets[E + 1] = padded row offsets on
// the device.  A tile is two consecutive 128-row blocks of ONE expert (the second absent
// when the expert has an odd block count: its rows are read clamped and not stored);
// live tiles are enumerated expert-major -> weight tile -> 256-row chunk from the
// offsets, so no host sync and a grid fixed by the capacity (blocks past the live
// tiles leave before any barrier).
// KS = 2 (grouped store form only): split-K decided on the device.  From the live tile
// count (expert offsets) every workgroup evaluates moe_w2_ksplit (common.h); with two
// slices each tile's K range is cut in half, run by two adjacent workgroups, and slice s
// writes its fp32 partial to slab s of outf ([2][M][ldo], M = the slab's rows); with one,
// the bf16 store to `out` as KS = 1.  The top-k combine evaluates the same rule and reads
// whichever was written (moe.hip moe_combine_w2_kernel).  For Mixtral's w2 at ~2,600-token
// steps the grouped store has 1.5 rounds of 256x256 tiles on 256 CUs, a half-empty second
// round; two K slices make it 3 half-length rounds (profiles/r6_mixtral_window.md).
template <int EPI, int ABL = 0, bool SPREAD = false, bool EARLY = false, int MF = 16,
          bool W3 = false, bool GROUPED = false, int KS = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm_w4_kernel(const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ w,
                    int64_t ldw, bf16_t* __restrict__ out, int64_t ldo, int M, int K, int up_off,
                    int tiles_m, int tiles_n, int group_m,
                    const int32_t* __restrict__ expert_offsets = nullptr, int E = 0,
                    int64_t w_estride = 0, float* __restrict__ outf = nullptr, int split_cus = 0) {
  static_assert(KS == 1 || (KS == 2 && GROUPED && EPI == kW4Store && MF == 16),
                "split-K: grouped fp32-partial store form only");
  extern __shared__ __attribute__((aligned(16))) char smem_w4[];
  w4_lds_c* const lds = (w4_lds_c*)smem_w4;

  // ---- block -> (row tile, weight tile): bijective XCD remap, then L2 groups
  int row0, tn, m_valid, m_store;         // first row, weight tile, rows readable / stored
  int kslice = 0, nslice = 1;             // KS > 1: this workgroup's K slice, slices
  if constexpr (GROUPED) {
    constexpr int kB = 128;
    const int nchunks = moe_live_chunks(expert_offsets, E);
    if constexpr (KS > 1) nslice = moe_w2_ksplit(nchunks * tiles_n, split_cus);
    const int nlive = nchunks * tiles_n * nslice;
    const int bid = blockIdx.x;
    if (bid >= nlive) return;               // before any barrier: the whole block leaves
    const int q8 = nlive >> 3, r8 = nlive & 7, xg = bid & 7;
    int wg = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + (bid >> 3);
    if (KS > 1 && nslice > 1) {
      kslice = wg & 1;
      wg >>= 1;
    }
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
    m_store = 2 * chunk + 1 < nbe ? 256 : 128;
    m_valid = min(expert_offsets[E] - row0, kW4M);
    w += (int64_t)e * w_estride;
    if (KS > 1 && nslice > 1) {
      K >>= 1;                              // rows keep their full strides ldx / ldw
      x += (int64_t)kslice * K;
      w += (int64_t)kslice * K;
    }
  } else {
    const int nwg = tiles_m * tiles_n;
    const int bid = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xg = bid & 7;
    const int wg = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + (bid >> 3);
    const int per_group = group_m * tiles_n;
    const int gid = wg / per_group, first_m = gid * group_m;
    const int gm = min(tiles_m - first_m, group_m);
    const int rin = wg - gid * per_group;
    const int tm = first_m + rin % gm;
    tn = rin / gm;
    row0 = tm * kW4M;
    m_valid = m_store = min(M - row0, kW4M);
  }

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int rr = lane & 15, kq = lane >> 4;

  // ---- DMA: per 64-deep K-tile a stage holds the W image (256 rows x 128 B, 32 pieces
  // of 8 rows) and the X image (32 pieces); wave wid issues W pieces 8 wid + q and X
  // pieces 8 wid + q (q = 0..7).  Lane -> image row 8 p + lane / 8, physical chunk lane & 7,
  // source chunk (lane & 7) ^ ((row >> 1) & 7).  buffer_load ... lds with the per-piece
  // row offset and the K-tile offset in SGPRs: one VGPR offset per lane for W, one per
  // X piece (rows past M are clamped to row M-1).
  const int lrow = lane >> 3, lch = lane & 7;
  // source chunk of image row 8p + lrow: lch ^ (((8p + lrow) >> 1) & 7), i.e. it depends on
  // the piece's parity (4p & 7): one W lane offset per parity
  auto src_chunk = [&](int p) { return lch ^ (((8 * p + lrow) >> 1) & 7); };
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + (int64_t)row0 * ldx), (short)0, 0x7fffffff, 0x00020000);
  const int w_voff[2] = {(lrow * (int)ldw + 8 * src_chunk(0)) * 2,
                         (lrow * (int)ldw + 8 * src_chunk(1)) * 2};
  int x_voff[8], w_soff[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = 8 * wid + q;                      // piece 0..31 of each image
    x_voff[q] = (min(8 * p + lrow, m_valid - 1) * (int)ldx + 8 * src_chunk(p)) * 2;
    int n0;                                         // W row of the piece's first image row
    if constexpr (EPI == kW4Swiglu) {
      const int i = (p >> 1) & 7, wc = p >> 4;      // image row 8p = 128 wc + 16 i + 8 (p & 1)
      n0 = (i < 4 ? 0 : up_off) + tn * 128 + 64 * wc + 16 * (i & 3) + 8 * (p & 1);
    } else {
      n0 = tn * kW4N + 8 * p;
    }
    w_soff[q] = __builtin_amdgcn_readfirstlane(n0 * (int)ldw * 2);
  }
  // operand image bases: W3: W slots 0..2 then X slots 0..1; else stage s = {W, X}
  auto wbase = [&](int slot) { return W3 ? lds + slot * (kW4Img * 2) : lds + slot * kW4StageB; };
  auto xbase = [&](int slot) {
    return W3 ? lds + 3 * (kW4Img * 2) + slot * (kW4Img * 2) : lds + slot * kW4StageB + kW4Img * 2;
  };
  auto dma_w = [&](int q, int stage, int k0) {      // k0: element offset of the K-tile
    w4_lds_c* const st = wbase(stage);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)(st + (8 * wid + q) * 1024), 16,
                                             w_voff[q & 1], w_soff[q] + 2 * k0, 0, 0);
  };
  auto dma_x = [&](int q, int stage, int k0) {
    w4_lds_c* const st = xbase(stage);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(st + (8 * wid + q) * 1024), 16,
                                             x_voff[q], 2 * k0, 0, 0);
  };
  auto dma = [&](int q, int stage, int k0) {
    dma_w(q, stage, k0);
    dma_x(q, stage, k0);
  };

  // ---- fragment addresses: W subtile i = image rows 128 wn + 16 i + rr, X subtile j =
  // rows 128 wm + 16 j + rr; k-half h reads chunk 4 h + kq at (4 h + kq) ^ ((rr >> 1) & 7);
  // subtile steps of 2 KB are ds_read immediates
  // MF 32: 32-row subtiles (4 KB apart), lane l reads row l & 31, chunk 4 h + 2 ks + (l >> 5)
  // of k-half h, k-step ks
  const int sw = (rr >> 1) & 7;
  const int r32 = lane & 31, k32 = lane >> 5, sw32 = (r32 >> 1) & 7;
  const int lo[2][2] = {
      {MF == 16 ? rr * 128 + 16 * (kq ^ sw) : r32 * 128 + 16 * (k32 ^ sw32),
       MF == 16 ? 0 : r32 * 128 + 16 * ((2 + k32) ^ sw32)},
      {MF == 16 ? rr * 128 + 16 * ((4 + kq) ^ sw) : r32 * 128 + 16 * ((4 + k32) ^ sw32),
       MF == 16 ? 0 : r32 * 128 + 16 * ((6 + k32) ^ sw32)}};
  const int wo = 16384 * wn, xo = 16384 * wm;
  constexpr int SUB = MF == 16 ? 2048 : 4096;       // bytes between subtiles

  f32x4 acc[MF == 16 ? 8 : 1][MF == 16 ? 8 : 1];   // MF 16: [W subtile i][X subtile j]
  f32x16 acc32[MF == 32 ? 4 : 1][MF == 32 ? 4 : 1];  // MF 32: [W subtile i][X subtile j]
#pragma unroll
  for (int i = 0; i < (MF == 16 ? 8 : 1); ++i)
#pragma unroll
    for (int j = 0; j < (MF == 16 ? 8 : 1); ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < (MF == 32 ? 4 : 1); ++i)
#pragma unroll
    for (int j = 0; j < (MF == 32 ? 4 : 1); ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc32[i][j][q] = 0.f;

  s16x8 f0[16], f1[16];      // fragments of k-half 0 / 1 of a K-tile: [0..7] W_i, [8..15] X_j

  // every fragment read issued so far has landed; the operands tie the registers to the
  // wait so no MFMA reading them is scheduled above it
  auto wait_frags = [&](s16x8 (&f)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]),
                   "+v"(f[6]), "+v"(f[7]), "+v"(f[8]), "+v"(f[9]), "+v"(f[10]), "+v"(f[11]),
                   "+v"(f[12]), "+v"(f[13]), "+v"(f[14]), "+v"(f[15]));
    __builtin_amdgcn_sched_barrier(0);
  };

  // One k-half: 64 MFMAs on `cur`, 16 fragment reads into `nxt` (k-half NH of the K-tile
  // in stage RS), and (DM) the 16 DMA pieces of K-tile k3 into stage S3, two per group in
  // the first 8 groups.
  // W3: rs = W slot, rx = X slot, s3 / k3 the X DMA's slot / K-tile, DW / sw / kw the
  // W DMA's; otherwise rs = rx = the stage and one DMA (s3, k3) covers both images.
  auto half = [&](s16x8 (&cur)[16], s16x8 (&nxt)[16], auto RD, auto NH, int rs, auto DM,
                  int s3, int k3, int rx, auto DW, int sw, int kw) {
    constexpr bool rd = decltype(RD)::value, dm = decltype(DM)::value;
    constexpr bool dw = decltype(DW)::value;
    constexpr int nh = decltype(NH)::value;
    w4_lds_c* const pw = wbase(rs) + wo + lo[nh][0];
    w4_lds_c* const px = xbase(rx) + xo + lo[nh][0];
    w4_lds_c* const pw1 = wbase(rs) + wo + lo[nh][1];   // MF 32, k-step 1
    w4_lds_c* const px1 = xbase(rx) + xo + lo[nh][1];
#define W4_MFMA(G, JJ)                                                                     \
    {                                                                                     \
      if constexpr (MF == 16) {                                                           \
        const int i = (G) >> 1, j = ((G) & 1) * 4 + (JJ);                                 \
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(cur[i]),            \
                                                            as_bf16x8(cur[8 + j]),        \
                                                            acc[i][j], 0, 0, 0);          \
      } else if constexpr ((JJ) < 2) {          /* (i, j) = (G / 4, G % 4), k-step JJ */ \
        const int i = (G) >> 2, j = (G) & 3;                                              \
        acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                            \
            as_bf16x8(cur[2 * i + (JJ)]), as_bf16x8(cur[8 + 2 * j + (JJ)]), acc32[i][j],   \
            0, 0, 0);                                                                     \
      }                                                                                   \
    }
    /* [MFMA, DMA piece, MFMA, fragment read, MFMA, MFMA]: a DMA piece's issue (~16-23   \
       cycles of the texture path) starts right behind an MFMA, so it overlaps that      \
       MFMA's execution instead of an idle pipe */                                        \
#define W4_FRAG(F)                                                                        \
    {                                                                                     \
      if constexpr (rd && !(ABL & 2)) {                                                   \
        if constexpr (MF == 16) {                                                         \
          if constexpr ((F) < 8) W4_READ(nxt[F], pw, SUB * ((F) & 7));                    \
          else W4_READ(nxt[F], px, SUB * ((F) & 7));                                      \
        } else {                    /* F = 2 subtile + k-step (W 0..7, X 8..15) */       \
          if constexpr ((F) < 8) W4_READ(nxt[F], ((F) & 1) ? pw1 : pw, SUB * ((F) >> 1)); \
          else W4_READ(nxt[F], ((F) & 1) ? px1 : px, SUB * (((F) & 7) >> 1));             \
        }                                                                                 \
      }                                                                                   \
      if constexpr (rd && (ABL & 2)) asm volatile("" : "+v"(nxt[F]));                     \
    }
#define W4_GROUP(G)                                                                       \
    {                                                                                     \
      W4_MFMA(G, 0)                                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr (dm && !(ABL & 1)) {                                                   \
        if constexpr (SPREAD) {                 /* X first: fewer blocks share it */     \
          if constexpr ((G) < 8) dma_x(G, s3, k3);                                        \
          else if constexpr (!W3) dma_w((G) & 7, s3, k3);                                 \
          else if constexpr (dw) dma_w((G) & 7, sw, kw);                                  \
        } else if constexpr ((G) < 8) {                                                   \
          dma(G, s3, k3);                                                                 \
        }                                                                                 \
      }                                                                                   \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      W4_MFMA(G, 1)                                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr (EARLY) {                                                              \
        if constexpr ((G) < 8) W4_FRAG(2 * (G));                                          \
      } else {                                                                            \
        W4_FRAG(G);                                                                       \
      }                                                                                   \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      W4_MFMA(G, 2)                                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr (EARLY && (G) < 8) W4_FRAG(2 * (G) + 1);                               \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      W4_MFMA(G, 3)                                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                  \
    }
    W4_GROUP(0) W4_GROUP(1) W4_GROUP(2) W4_GROUP(3) W4_GROUP(4) W4_GROUP(5) W4_GROUP(6)
    W4_GROUP(7) W4_GROUP(8) W4_GROUP(9) W4_GROUP(10) W4_GROUP(11) W4_GROUP(12) W4_GROUP(13)
    W4_GROUP(14) W4_GROUP(15)
#undef W4_GROUP
#undef W4_MFMA
#undef W4_FRAG
  };
  // the boundary inside K-tile t: K-tile t+1's DMA (own pieces) landed, k-half 1's
  // fragments landed, one barrier (every wave: the same, and done reading stage t's
  // image, which K-tile t+2's DMA overwrites next)
  auto mid = [&](auto VM8) {
    if constexpr (!(ABL & 4)) {
      // W3: the 8 youngest pieces are the W DMA two K-tiles ahead: leave them in flight
      if constexpr (decltype(VM8)::value) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wait_frags(f1);
      __builtin_amdgcn_s_barrier();
    } else {
      wait_frags(f1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  using T_ = std::true_type;
  using F_ = std::false_type;
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;
  const int nk = K / 64;
  // ---- prologue: K-tiles 0 and 1 in flight, tile 0 landed, its k-half 0 read
  // (W3: W tiles 0-2 and X tiles 0-1, issued W0 X0 X1 W1 W2 for the counted waits)
  if constexpr (W3) {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(q, 0, 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma_x(q, 1, 64);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma_w(q, 1, 64);
    if (nk > 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) dma_w(q, 2, 128);
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    }
  } else {
#pragma unroll
  for (int q = 0; q < 8; ++q) dma(q, 0, 0);
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(q, 1, 64);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (MF == 16) {
    w4_lds_c* const pw = wbase(0) + wo + lo[0][0];
    w4_lds_c* const px = xbase(0) + xo + lo[0][0];
    W4_READ(f0[0], pw, 0);     W4_READ(f0[1], pw, 2048);  W4_READ(f0[2], pw, 4096);
    W4_READ(f0[3], pw, 6144);  W4_READ(f0[4], pw, 8192);  W4_READ(f0[5], pw, 10240);
    W4_READ(f0[6], pw, 12288); W4_READ(f0[7], pw, 14336);
    W4_READ(f0[8], px, 0);     W4_READ(f0[9], px, 2048);  W4_READ(f0[10], px, 4096);
    W4_READ(f0[11], px, 6144); W4_READ(f0[12], px, 8192); W4_READ(f0[13], px, 10240);
    W4_READ(f0[14], px, 12288); W4_READ(f0[15], px, 14336);
  } else {
    w4_lds_c* const pw = wbase(0) + wo + lo[0][0];
    w4_lds_c* const px = xbase(0) + xo + lo[0][0];
    w4_lds_c* const pw1 = wbase(0) + wo + lo[0][1];
    w4_lds_c* const px1 = xbase(0) + xo + lo[0][1];
    W4_READ(f0[0], pw, 0);      W4_READ(f0[1], pw1, 0);     W4_READ(f0[2], pw, 4096);
    W4_READ(f0[3], pw1, 4096);  W4_READ(f0[4], pw, 8192);   W4_READ(f0[5], pw1, 8192);
    W4_READ(f0[6], pw, 12288);  W4_READ(f0[7], pw1, 12288);
    W4_READ(f0[8], px, 0);      W4_READ(f0[9], px1, 0);     W4_READ(f0[10], px, 4096);
    W4_READ(f0[11], px1, 4096); W4_READ(f0[12], px, 8192);  W4_READ(f0[13], px1, 8192);
    W4_READ(f0[14], px, 12288); W4_READ(f0[15], px1, 12288);
  }

  // ---- K-tile t: half 0 (MFMAs on f0, reads of half 1 into f1, same stage), the
  // boundary, half 1 (MFMAs on f1, reads of K-tile t+1's half 0 into f0, DMA of t+2
  // into this stage)
  int t = 0;
  using V8 = std::true_type;
  if constexpr (W3) {
    // K-tile t: half 0 on slot t % 3 / t % 2; mid leaves W(t+2) in flight; half 1 reads
    // tile t+1 and issues X(t+2) into X slot t % 2 and W(t+3) into W slot t % 3
    for (; t + 3 < nk; ++t) {
      wait_frags(f0);
      half(f0, f1, T_{}, H1{}, t % 3, F_{}, 0, 0, t & 1, F_{}, 0, 0);
      mid(V8{});
      half(f1, f0, T_{}, H0{}, (t + 1) % 3, T_{}, t & 1, (t + 2) * 64, (t + 1) & 1, T_{},
           t % 3, (t + 3) * 64);
    }
    if (t + 2 < nk) {          // nk >= 4: X(t+2) still to come, no W
      wait_frags(f0);
      half(f0, f1, T_{}, H1{}, t % 3, F_{}, 0, 0, t & 1, F_{}, 0, 0);
      mid(V8{});
      half(f1, f0, T_{}, H0{}, (t + 1) % 3, T_{}, t & 1, (t + 2) * 64, (t + 1) & 1, F_{}, 0, 0);
      ++t;
    }
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, t % 3, F_{}, 0, 0, t & 1, F_{}, 0, 0);
    mid(F_{});
    half(f1, f0, T_{}, H0{}, (t + 1) % 3, F_{}, 0, 0, (t + 1) & 1, F_{}, 0, 0);
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, (t + 1) % 3, F_{}, 0, 0, (t + 1) & 1, F_{}, 0, 0);
    mid(F_{});
    half(f1, f0, F_{}, H0{}, 0, F_{}, 0, 0, 0, F_{}, 0, 0);
  } else {
  for (; t + 2 < nk; ++t) {
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, t & 1, F_{}, 0, 0, t & 1, F_{}, 0, 0);
    mid(F_{});
    half(f1, f0, T_{}, H0{}, (t + 1) & 1, T_{}, t & 1, (t + 2) * 64, (t + 1) & 1, F_{}, 0, 0);
  }
  // the last two K-tiles (nk is even): no more DMA
  wait_frags(f0);
  half(f0, f1, T_{}, H1{}, t & 1, F_{}, 0, 0, t & 1, F_{}, 0, 0);
  mid(F_{});
  half(f1, f0, T_{}, H0{}, (t + 1) & 1, F_{}, 0, 0, (t + 1) & 1, F_{}, 0, 0);
  wait_frags(f0);
  half(f0, f1, T_{}, H1{}, (t + 1) & 1, F_{}, 0, 0, (t + 1) & 1, F_{}, 0, 0);
  mid(F_{});
  half(f1, f0, F_{}, H0{}, 0, F_{}, 0, 0, 0, F_{}, 0, 0);
  }

  // ---- epilogue.  MF 16: lane holds out[row0 + 128 wm + 16 j + rr][n0 + 16 i + 4 kq + 0..3];
  // MF 32: out[row0 + 128 wm + 32 j + (l & 31)][n0 + 32 i + 4 (l >> 5) + 8 vq + 0..3]
  if constexpr (MF == 16) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int trow = 128 * wm + 16 * j + rr;
    if (trow >= m_store) continue;
    bf16_t* orow = out + (int64_t)(row0 + trow) * ldo;
    if (KS > 1 && nslice > 1) {
      float* frow = outf + ((int64_t)kslice * M + row0 + trow) * ldo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float4 v;
        v.x = acc[i][j][0];
        v.y = acc[i][j][1];
        v.z = acc[i][j][2];
        v.w = acc[i][j][3];
        *reinterpret_cast<float4*>(frow + tn * kW4N + 128 * wn + 16 * i + 4 * kq) = v;
      }
    } else if constexpr (EPI == kW4Swiglu) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float gf = bf2f(f2bf(acc[i][j][u]));          // = the gate GEMM's bf16
          const float sg = gf / (1.f + __expf(-gf));
          o[u] = bf2f(f2bf(sg)) * bf2f(f2bf(acc[4 + i][j][u]));
        }
        uint2 v;
        v.x = pack_bf16x2(o[0], o[1]);
        v.y = pack_bf16x2(o[2], o[3]);
        *reinterpret_cast<uint2*>(orow + tn * 128 + 64 * wn + 16 * i + 4 * kq) = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint2 v;
        v.x = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
        v.y = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(orow + tn * kW4N + 128 * wn + 16 * i + 4 * kq) = v;
      }
    }
  }
  } else {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int trow = 128 * wm + 32 * j + r32;
    if (trow >= m_store) continue;
    bf16_t* orow = out + (int64_t)(row0 + trow) * ldo;
    if constexpr (EPI == kW4Swiglu) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int vq = 0; vq < 4; ++vq) {
          float o[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float gf = bf2f(f2bf(acc32[i][j][4 * vq + u]));
            const float sg = gf / (1.f + __expf(-gf));
            o[u] = bf2f(f2bf(sg)) * bf2f(f2bf(acc32[2 + i][j][4 * vq + u]));
          }
          uint2 v;
          v.x = pack_bf16x2(o[0], o[1]);
          v.y = pack_bf16x2(o[2], o[3]);
          *reinterpret_cast<uint2*>(orow + tn * 128 + 64 * wn + 32 * i + 4 * k32 + 8 * vq) = v;
        }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int vq = 0; vq < 4; ++vq) {
          uint2 v;
          v.x = pack_bf16x2(acc32[i][j][4 * vq + 0], acc32[i][j][4 * vq + 1]);
          v.y = pack_bf16x2(acc32[i][j][4 * vq + 2], acc32[i][j][4 * vq + 3]);
          *reinterpret_cast<uint2*>(orow + tn * kW4N + 128 * wn + 32 * i + 4 * k32 + 8 * vq) = v;
        }
    }
  }
  }
}

// Persistent form of the tuned kernel (cfg 5768 + bit 13; K % 256 == 0): one workgroup
// per CU walks output tiles id, id + G, ... (G = grid), with one K-tile pipeline running
// straight across tile boundaries: during the last three K-tiles of a tile the weight /
// activation pieces of the NEXT tile's K-tiles 0-2 are issued into the slots that free
// up, and the last half reads the next tile's first fragments, so the next tile's
// prologue latency and this tile's epilogue stores overlap instead of adding up.  (The
// non-persistent kernel pays ~80 µs of per-tile prologue + epilogue per launch on the
// gate|up shape: the intercept of its time-vs-K line, where hipBLASLt's is ~0;
// profiles/r4_gemm_w4.md.)  The last tile's "next" pieces re-read its own K-tiles 0-2
// (harmless; drained before exit).  Slots: W 3 (g % 3, g = K-tile counter over all the
// workgroup's tiles), X 2 (g % 2), 160 KB.
//
// SK (stream-K for the last rounds): the first nwg - sk_tiles tiles go round-robin as
// above (whole rounds); the last sk_tiles tiles are cut into chunks of 4 K-tiles and
// every workgroup takes an equal run of consecutive chunks, so no CU idles through a
// partly filled last round.  A run is a sequence of units (tile, K-tile range); a unit
// that is not a whole tile is a partial sum:
//   * the unit that starts a tile's K range (its "owner": the lowest workgroup on it) is
//     the LAST unit of its workgroup's run;
//   * the others ("partners": higher workgroups, whose runs START inside that tile) are
//     the FIRST unit of their runs: each publishes its fp32 accumulators (sc1 stores,
//     drained, then one lane's agent-scope flag; cdna_hip_programming.md §6 Guideline 16
//     recipe) and goes on to its next unit;
//   * the owner polls each partner's flag (resetting it for the next launch), adds the
//     partner's slab with sc1 loads and runs the ordinary epilogue.
// A partner publishes before it waits for anything and all G <= CUs workgroups are
// resident (one per CU, 160 KB LDS), so every wait ends; the spin is bounded anyway.
template <int EPI, bool SK = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm_w4p_kernel(const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ w,
                     int64_t ldw, bf16_t* __restrict__ out, int64_t ldo, int M, int K, int up_off,
                     int tiles_m, int tiles_n, int group_m, int sk_tiles = 0,
                     float* __restrict__ sk_ws = nullptr, int* __restrict__ sk_flag = nullptr,
                     uint32_t* __restrict__ sk_err = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem_w4[];
  w4_lds_c* const lds = (w4_lds_c*)smem_w4;
  const int nwg = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int rr = lane & 15, kq = lane >> 4;
  const int lrow = lane >> 3, lch = lane & 7;
  auto src_chunk = [&](int p) { return lch ^ (((8 * p + lrow) >> 1) & 7); };
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
  // output: num_records = M rows, so a store to a row past M is dropped
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, M * (int)ldo * 2, 0x00020000);
  const int w_voff[2] = {(lrow * (int)ldw + 8 * src_chunk(0)) * 2,
                         (lrow * (int)ldw + 8 * src_chunk(1)) * 2};
  // tile id -> (row tile, weight tile): the same XCD remap and L2 groups as the
  // one-tile kernel (G % 8 == 0, so id & 7 is this workgroup's XCD for every id)
  auto tile_of = [&](int id, int& tm, int& tn) {
    const int q8 = nwg >> 3, r8 = nwg & 7, xg = id & 7;
    const int wg = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + (id >> 3);
    const int per_group = group_m * tiles_n;
    const int gid = wg / per_group, first_m = gid * group_m;
    const int gm = min(tiles_m - first_m, group_m);
    const int rin = wg - gid * per_group;
    tm = first_m + rin % gm;
    tn = rin / gm;
  };
  // a tile's DMA offsets: X rows (clamped to M - 1) with the tile's row offset folded in,
  // W piece rows in SGPRs
  // kb: the unit's first K-tile (stream-K partial units), folded into both offsets
  auto addrs = [&](int id, int kb, int (&xv)[8], int (&ws)[8]) {
    int tm, tn;
    tile_of(id, tm, tn);
    const int row0 = tm * kW4M, mv = min(M - row0, kW4M);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int p = 8 * wid + q;
      xv[q] = ((row0 + min(8 * p + lrow, mv - 1)) * (int)ldx + 8 * src_chunk(p) + kb * 64) * 2;
      int n0;
      if constexpr (EPI == kW4Swiglu) {
        const int i = (p >> 1) & 7, wc = p >> 4;
        n0 = (i < 4 ? 0 : up_off) + tn * 128 + 64 * wc + 16 * (i & 3) + 8 * (p & 1);
      } else {
        n0 = tn * kW4N + 8 * p;
      }
      ws[q] = __builtin_amdgcn_readfirstlane((n0 * (int)ldw + kb * 64) * 2);
    }
  };
  auto wbase = [&](int slot) { return lds + slot * (kW4Img * 2); };
  auto xbase = [&](int slot) { return lds + 3 * (kW4Img * 2) + slot * (kW4Img * 2); };
  int xv_c[8], ws_c[8], xv_n[8], ws_n[8];
  auto dma_w = [&](int q, int slot, int k0, const int (&ws)[8]) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_void_t*)(wbase(slot) + (8 * wid + q) * 1024),
                                             16, w_voff[q & 1], ws[q] + 2 * k0, 0, 0);
  };
  auto dma_x = [&](int q, int slot, int k0, const int (&xv)[8]) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(xbase(slot) + (8 * wid + q) * 1024),
                                             16, xv[q], 2 * k0, 0, 0);
  };

  const int sw = (rr >> 1) & 7;
  const int lo0 = rr * 128 + 16 * (kq ^ sw), lo1 = rr * 128 + 16 * ((4 + kq) ^ sw);
  const int wo = 16384 * wn, xo = 16384 * wm;
  constexpr int SUB = 2048;
  f32x4 acc[8][8];
  s16x8 f0[16], f1[16];
  auto wait_frags = [&](s16x8 (&f)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]),
                   "+v"(f[6]), "+v"(f[7]), "+v"(f[8]), "+v"(f[9]), "+v"(f[10]), "+v"(f[11]),
                   "+v"(f[12]), "+v"(f[13]), "+v"(f[14]), "+v"(f[15]));
    __builtin_amdgcn_sched_barrier(0);
  };
  // One k-half: 64 MFMAs on `cur`; RD: 16 fragment reads of k-half NH from W slot rs / X
  // slot rx into `nxt`; DX: X pieces of K-tile kx into X slot sx (NX: the next tile's),
  // DW: W pieces of K-tile kw into W slot sw (NW: the next tile's).
  auto half = [&](s16x8 (&cur)[16], s16x8 (&nxt)[16], auto RD, auto NH, int rs, int rx,
                  auto DX, auto NXX, int sx, int kx, auto DW, auto NXW, int swl, int kw) {
    constexpr bool rd = decltype(RD)::value, dx = decltype(DX)::value;
    constexpr bool dw = decltype(DW)::value, nxx = decltype(NXX)::value;
    constexpr bool nxw = decltype(NXW)::value;
    constexpr int nh = decltype(NH)::value;
    w4_lds_c* const pw = wbase(rs) + wo + (nh ? lo1 : lo0);
    w4_lds_c* const px = xbase(rx) + xo + (nh ? lo1 : lo0);
#define W4P_MFMA(G_, JJ)                                                                   \
    {                                                                                     \
      const int i = (G_) >> 1, j = ((G_) & 1) * 4 + (JJ);                                \
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(cur[i]),              \
                                                          as_bf16x8(cur[8 + j]), acc[i][j], \
                                                          0, 0, 0);                        \
    }
#define W4P_FRAG(F)                                                                       \
    {                                                                                     \
      if constexpr (rd) {                                                                 \
        if constexpr ((F) < 8) W4_READ(nxt[F], pw, SUB * ((F) & 7));                      \
        else W4_READ(nxt[F], px, SUB * ((F) & 7));                                        \
      }                                                                                   \
    }
#define W4P_GROUP(G_)                                                                     \
    {                                                                                     \
      W4P_MFMA(G_, 0)                                                                     \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr ((G_) < 8) {                                                           \
        if constexpr (dx) dma_x(G_, sx, kx, nxx ? xv_n : xv_c);                           \
      } else if constexpr (dw) {                                                          \
        dma_w((G_) & 7, swl, kw, nxw ? ws_n : ws_c);                                      \
      }                                                                                   \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      W4P_MFMA(G_, 1)                                                                     \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr ((G_) < 8) W4P_FRAG(2 * (G_));                                         \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      W4P_MFMA(G_, 2)                                                                     \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr ((G_) < 8) W4P_FRAG(2 * (G_) + 1);                                     \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      W4P_MFMA(G_, 3)                                                                     \
      __builtin_amdgcn_sched_barrier(0);                                                  \
    }
    W4P_GROUP(0) W4P_GROUP(1) W4P_GROUP(2) W4P_GROUP(3) W4P_GROUP(4) W4P_GROUP(5)
    W4P_GROUP(6) W4P_GROUP(7) W4P_GROUP(8) W4P_GROUP(9) W4P_GROUP(10) W4P_GROUP(11)
    W4P_GROUP(12) W4P_GROUP(13) W4P_GROUP(14) W4P_GROUP(15)
#undef W4P_GROUP
#undef W4P_MFMA
#undef W4P_FRAG
  };
  // K-tile boundary: VM8 leaves the 8 youngest pieces (the W DMA two K-tiles ahead) in
  // flight; after an epilogue (its stores are younger) everything is waited for
  auto mid = [&](auto VM) {
    if constexpr (decltype(VM)::value == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (decltype(VM)::value == 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
    else if constexpr (decltype(VM)::value == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wait_frags(f1);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;
  using V8 = std::integral_constant<int, 8>;
  // W(2) + this wave's epilogue stores per tile (plain 32, SwiGLU 16; all 16 bytes)
  using V40 = std::integral_constant<int, EPI == kW4Swiglu ? 24 : 40>;
  const int nk = K / 64;                          // >= 4, even

  // this workgroup's units: round-robin whole tiles g, g + G, ... < dp_end, then (SK) the
  // chunk run [c0, c1) over tiles dp_end.. (a unit: tile id, K-tiles [kb, ke))
  const int g = blockIdx.x;
  const int dp_end = SK ? nwg - sk_tiles : nwg;
  const int ndp = g < dp_end ? (dp_end - 1 - g) / G + 1 : 0;
  const int cpt = nk >> 2;                        // 4-K-tile chunks per tile
  const int csk = SK ? sk_tiles * cpt : 0;
  const int c0 = (int)((int64_t)g * csk / G), c1 = (int)((int64_t)(g + 1) * csk / G);
  auto unit = [&](int u, int& uid, int& kb, int& ke) {
    if (u < ndp) {
      uid = g + u * G;
      kb = 0;
      ke = nk;
      return true;
    }
    if constexpr (!SK) {
      return false;
    } else {
      const int tv = c0 / cpt + (u - ndp);
      const int cs = u == ndp ? c0 : tv * cpt;
      if (cs >= c1) return false;
      const int ce = min(c1, (tv + 1) * cpt);
      uid = dp_end + tv;
      kb = (cs - tv * cpt) * 4;
      ke = (ce - tv * cpt) * 4;
      return true;
    }
  };
  int u = 0, id, kb, ke, nid = 0, nkb = 0, nke = 0;
  if (!unit(0, id, kb, ke)) return;
  bool more = unit(1, nid, nkb, nke);
  addrs(id, kb, xv_c, ws_c);
  if (more) addrs(nid, nkb, xv_n, ws_n);
  else addrs(id, kb, xv_n, ws_n);
  // ---- first tile's prologue: W0 X0 X1 W1 W2 (slots W 0-2, X 0-1)
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_w(q, 0, 0, ws_c);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_x(q, 0, 0, xv_c);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_x(q, 1, 64, xv_c);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_w(q, 1, 64, ws_c);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_w(q, 2, 128, ws_c);
  // X1 / W1 landed too (W2 in flight): K-tile 0's boundary below waits vmcnt(40 / 24),
  // which is what a continued tile needs and a no-op here
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  {
    w4_lds_c* const pw = wbase(0) + wo + lo0;
    w4_lds_c* const px = xbase(0) + xo + lo0;
    W4_READ(f0[0], pw, 0);     W4_READ(f0[1], pw, 2048);  W4_READ(f0[2], pw, 4096);
    W4_READ(f0[3], pw, 6144);  W4_READ(f0[4], pw, 8192);  W4_READ(f0[5], pw, 10240);
    W4_READ(f0[6], pw, 12288); W4_READ(f0[7], pw, 14336);
    W4_READ(f0[8], px, 0);     W4_READ(f0[9], px, 2048);  W4_READ(f0[10], px, 4096);
    W4_READ(f0[11], px, 6144); W4_READ(f0[12], px, 8192); W4_READ(f0[13], px, 10240);
    W4_READ(f0[14], px, 12288); W4_READ(f0[15], px, 14336);
  }
  int wofs = 0;                                   // W slot of this tile's K-tile 0
  while (true) {
    const int nku = __builtin_amdgcn_readfirstlane(ke - kb);   // K-tiles of this unit
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K-tile 0: K-tile 1 must have landed; younger than its pieces are W(2) and the
    // previous tile's epilogue stores (32, SwiGLU 16) (a fixed count: rows past M are clipped by the
    // output buffer's range, not skipped), so they stay in flight
    int t = 0;
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, wofs % 3, 0, F_{}, F_{}, 0, 0, F_{}, F_{}, 0, 0);
    mid(V40{});
    half(f1, f0, T_{}, H0{}, (wofs + 1) % 3, 1, T_{}, F_{}, 0, 2 * 64, T_{}, F_{}, wofs % 3,
         3 * 64);
    for (t = 1; t + 3 < nku; ++t) {
      wait_frags(f0);
      half(f0, f1, T_{}, H1{}, (wofs + t) % 3, t & 1, F_{}, F_{}, 0, 0, F_{}, F_{}, 0, 0);
      mid(V8{});
      half(f1, f0, T_{}, H0{}, (wofs + t + 1) % 3, (t + 1) & 1, T_{}, F_{}, t & 1, (t + 2) * 64,
           T_{}, F_{}, (wofs + t) % 3, (t + 3) * 64);
    }
    // t = nk-3: X(nk-1) of this tile, W(0) of the next
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, (wofs + t) % 3, 1, F_{}, F_{}, 0, 0, F_{}, F_{}, 0, 0);
    mid(V8{});
    half(f1, f0, T_{}, H0{}, (wofs + t + 1) % 3, 0, T_{}, F_{}, 1, (nku - 1) * 64, T_{}, T_{},
         (wofs + t) % 3, 0);
    ++t;
    // t = nk-2: X(0), W(1) of the next tile
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, (wofs + t) % 3, 0, F_{}, F_{}, 0, 0, F_{}, F_{}, 0, 0);
    mid(V8{});
    half(f1, f0, T_{}, H0{}, (wofs + t + 1) % 3, 1, T_{}, T_{}, 0, 0, T_{}, T_{}, (wofs + t) % 3,
         64);
    ++t;
    // t = nk-1: the last half issues the next tile's X(1), W(2); its K-tile 0 landed at
    // this boundary, and its first fragments are read after the epilogue (reading them
    // here would keep 64 more registers live through the stores)
    wait_frags(f0);
    half(f0, f1, T_{}, H1{}, (wofs + t) % 3, 1, F_{}, F_{}, 0, 0, F_{}, F_{}, 0, 0);
    mid(V8{});
    half(f1, f0, F_{}, H0{}, 0, 0, T_{}, T_{}, 1, 64, T_{}, T_{}, (wofs + t) % 3, 128);

    // ---- stream-K partial units (see above): a partner publishes its fp32 accumulators
    // and moves on; an owner first waits for its partners' flags, then adds their slabs
    // row block by row block inside the epilogue (the accumulators are only ever read
    // there, in the epilogue's order: any other read or write of them spills)
    const bool pub = SK && kb != 0;
    const bool own = SK && kb == 0 && ke != nk;
    const int tend = SK ? (id - dp_end + 1) * cpt : 0;      // chunk past this tile
    const __amdgpu_buffer_rsrc_t sr =
        __builtin_amdgcn_make_buffer_rsrc((void*)sk_ws, (short)0, 0x7fffffff, 0x00020000);
    if constexpr (SK) {
      if (own) {
        if (tid == 0) {
          for (int pw = g + 1; pw < G && (int)((int64_t)pw * csk / G) < tend; ++pw) {
            if ((int64_t)(pw + 1) * csk / G == (int64_t)pw * csk / G) continue;   // empty run
            // bounded wait (1 s): on a timeout the owner counts an error (the runner then
            // fails the step) and leaves the flag alone -- clearing a flag it never saw
            // set would let the late partner's 1 satisfy the next launch early
            bool seen = false;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (!(seen = __hip_atomic_load(sk_flag + pw, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) != 0)) {
              if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) break;
              __builtin_amdgcn_s_sleep(2);
            }
            if (seen)
              __hip_atomic_store(sk_flag + pw, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
              report_error(sk_err, kErrStreamK);
          }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every slab load is sc1
      }
    }
    // ---- epilogue of tile id (the next tile's pieces are in flight).  A fixed number of
    // stores per wave (32, SwiGLU 16): buffer stores whose rows past M fall outside the
    // output range and are dropped; two lanes' 8-byte runs are paired into one 16-byte
    // store each (the partner is lane ^ 16: ds_swizzle xor 0x10).
    {
      int tm, tn;
      tile_of(id, tm, tn);
      const int row0 = tm * kW4M;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // a never-taken, opaque branch per row block keeps the compiler from hoisting
        // every block's accumulator reads to the top (that spilled); the store count
        // stays fixed, which the next tile's vmcnt(40) relies on
        if (__builtin_amdgcn_readfirstlane(nku + j) < 0) continue;
        float t[8][4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) t[i][e] = acc[i][j][e];
        if constexpr (SK) {
          // slab offset: lane part in one VGPR, (i, j) part as soffset
          if (pub) {
            const int base = (g * 64 * 256 + tid) * 16;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              u32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = __float_as_uint(t[i][e]);
              __builtin_amdgcn_raw_buffer_store_b128(v, sr, base, (i * 8 + j) * 4096, 16);
            }
            continue;
          }
          if (own) {
            for (int pw = g + 1; pw < G && (int)((int64_t)pw * csk / G) < tend; ++pw) {
              if ((int64_t)(pw + 1) * csk / G == (int64_t)pw * csk / G) continue;
              const int base = (pw * 64 * 256 + tid) * 16;
              u32x4 v[8];
#pragma unroll
              for (int i = 0; i < 8; ++i)
                v[i] = __builtin_amdgcn_raw_buffer_load_b128(sr, base, (i * 8 + j) * 4096, 16);
#pragma unroll
              for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) t[i][e] += __uint_as_float(v[i][e]);
            }
          }
        }
        const int trow = 128 * wm + 16 * j + rr;
        const int rowb = (row0 + trow) * (int)ldo * 2;        // byte offset of the row
        const bool odd = kq & 1;
        if constexpr (EPI == kW4Swiglu) {
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            uint32_t h[2][2];                     // [subtile 2 pr + e][dword]
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              float o[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const float gf = bf2f(f2bf(t[2 * pr + e][u]));
                const float sg = gf / (1.f + __expf(-gf));
                o[u] = bf2f(f2bf(sg)) * bf2f(f2bf(t[4 + 2 * pr + e][u]));
              }
              h[e][0] = pack_bf16x2(o[0], o[1]);
              h[e][1] = pack_bf16x2(o[2], o[3]);
            }
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(odd ? h[0][0] : h[1][0]), 0x401F);
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(odd ? h[0][1] : h[1][1]), 0x401F);
            u32x4 v;
            v[0] = odd ? r0 : h[0][0];
            v[1] = odd ? r1 : h[0][1];
            v[2] = odd ? h[1][0] : r0;
            v[3] = odd ? h[1][1] : r1;
            const int col = tn * 128 + 64 * wn + 16 * (2 * pr + (odd ? 1 : 0)) + 4 * (kq & 2);
            __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, rowb + col * 2, 0, 0);
          }
        } else {
#pragma unroll
          for (int pr = 0; pr < 4; ++pr) {
            const uint32_t a0 = pack_bf16x2(t[2 * pr][0], t[2 * pr][1]);
            const uint32_t a1 = pack_bf16x2(t[2 * pr][2], t[2 * pr][3]);
            const uint32_t b0 = pack_bf16x2(t[2 * pr + 1][0], t[2 * pr + 1][1]);
            const uint32_t b1 = pack_bf16x2(t[2 * pr + 1][2], t[2 * pr + 1][3]);
            // even kq keeps subtile 2 pr (its 4 columns + the partner's next 4), odd kq
            // subtile 2 pr + 1 (the partner's 4 columns + its own)
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(odd ? a0 : b0), 0x401F);
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(odd ? a1 : b1), 0x401F);
            u32x4 v;
            v[0] = odd ? r0 : a0;
            v[1] = odd ? r1 : a1;
            v[2] = odd ? b0 : r0;
            v[3] = odd ? b1 : r1;
            const int col = tn * kW4N + 128 * wn + 16 * (2 * pr + (odd ? 1 : 0)) + 4 * (kq & 2);
            __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, rowb + col * 2, 0, 0);
          }
        }
      }
    }
    if constexpr (SK) {
      if (pub) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // every wave's slab stores landed
        __syncthreads();
        if (tid == 0) __hip_atomic_store(sk_flag + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (!more) break;
    ++u;
    id = nid;
    kb = nkb;
    ke = nke;
    more = unit(u + 1, nid, nkb, nke);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      xv_c[q] = xv_n[q];
      ws_c[q] = ws_n[q];
    }
    if (more) addrs(nid, nkb, xv_n, ws_n);
    else addrs(id, kb, xv_n, ws_n);
    wofs = (wofs + nku) % 3;
    {
      w4_lds_c* const pw = wbase(wofs) + wo + lo0;
      w4_lds_c* const px = xbase(0) + xo + lo0;
      W4_READ(f0[0], pw, 0);     W4_READ(f0[1], pw, 2048);  W4_READ(f0[2], pw, 4096);
      W4_READ(f0[3], pw, 6144);  W4_READ(f0[4], pw, 8192);  W4_READ(f0[5], pw, 10240);
      W4_READ(f0[6], pw, 12288); W4_READ(f0[7], pw, 14336);
      W4_READ(f0[8], px, 0);     W4_READ(f0[9], px, 2048);  W4_READ(f0[10], px, 4096);
      W4_READ(f0[11], px, 6144); W4_READ(f0[12], px, 8192); W4_READ(f0[13], px, 10240);
      W4_READ(f0[14], px, 12288); W4_READ(f0[15], px, 14336);
    }
  }
  // the last tile's "next" pieces (its own K-tiles 0-2 again) land before the workgroup
  // ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
#undef W4_READ

// Grouped (MoE) form of the W3 kernel (cfg 5768's structure: DMA spread over the MFMA
// groups, early fragment reads, the weight image in three LDS slots); the contract of
// gemm_dense.hip launch_gemm_grouped.  K % 128 == 0.
void launch_gemm_w4_grouped(const bf16_t* x, const bf16_t* w, bf16_t* out,
                            const int32_t* expert_offsets, int max_blocks, int n_out, int K,
                            int E, int64_t w_rows, bool swiglu, hipStream_t s, float* outf,
                            int slab_rows, int split_cus) {
  if (max_blocks <= 0) return;
  const int tiles_n = swiglu ? n_out / 128 : n_out / kW4N;
  const int chunks = (max_blocks + E) / 2 + 1;    // live 256-row tiles <= this
  const int grid = chunks * tiles_n;
  const int64_t estride = w_rows * K;
  constexpr int lds3 = 5 * kW4Img * 2;            // 160 KB
  if (outf != nullptr && !swiglu)                 // outf: float [2][slab_rows][n_out]
    gemm_w4_kernel<kW4Store, 0, true, true, 16, true, true, 2><<<2 * grid, 256, lds3, s>>>(
        x, K, w, K, out, n_out, slab_rows, K, n_out, 0, tiles_n, 4, expert_offsets, E,
        estride, outf, split_cus);
  else if (swiglu)
    gemm_w4_kernel<kW4Swiglu, 0, true, true, 16, true, true><<<grid, 256, lds3, s>>>(
        x, K, w, K, out, n_out, max_blocks * 128, K, n_out, 0, tiles_n, 4, expert_offsets, E,
        estride);
  else
    gemm_w4_kernel<kW4Store, 0, true, true, 16, true, true><<<grid, 256, lds3, s>>>(
        x, K, w, K, out, n_out, max_blocks * 128, K, n_out, 0, tiles_n, 4, expert_offsets, E,
        estride);
}

// Stream-K slabs (256 KB per workgroup: 64 accumulators x 256 lanes x 16 B) and zeroed
// flags for g workgroups, allocated on first use outside stream capture (64 MB at 256
// CUs); false = run the plain persistent kernel instead.  One set per (device, stream):
// two stream-K launches in flight on different streams (the runner's capture stream, an
// overlap experiment) never share slabs or flags.  At most kSkStreams streams
// per device get a set; launches on further streams take the plain kernel.
static bool gemm_w4p_sk_ws(int g, hipStream_t stream, float** ws, int** flags) {
  constexpr int kMaxDev = 16, kSkStreams = 4;
  static std::mutex mu;
  static hipStream_t s_stream[kMaxDev][kSkStreams] = {};
  static float* s_ws[kMaxDev][kSkStreams] = {};
  static int* s_flags[kMaxDev][kSkStreams] = {};
  static int s_cap[kMaxDev][kSkStreams] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return false;
  std::lock_guard<std::mutex> lock(mu);
  int slot = -1;
  for (int i = 0; i < kSkStreams && slot < 0; ++i)
    if (s_ws[dev][i] != nullptr && s_stream[dev][i] == stream) slot = i;
  if (slot < 0) {
    for (int i = 0; i < kSkStreams && slot < 0; ++i)
      if (s_ws[dev][i] == nullptr) slot = i;
    if (slot < 0) return false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone)
      return false;
    float* p = nullptr;
    int* f = nullptr;
    if (hipMalloc(&p, (size_t)g * 64 * 256 * 16) != hipSuccess) return false;
    if (hipMalloc(&f, g * sizeof(int)) != hipSuccess || hipMemset(f, 0, g * sizeof(int)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return false;
    }
    s_stream[dev][slot] = stream;
    s_ws[dev][slot] = p;
    s_flags[dev][slot] = f;
    s_cap[dev][slot] = g;
  }
  if (g > s_cap[dev][slot]) return false;
  *ws = s_ws[dev][slot];
  *flags = s_flags[dev][slot];
  return true;
}

// out = x w^T ([M, N]) or, swiglu, act = silu(x Wg^T) * (x Wu^T) ([M, F], w = [2F, K], up
// rows at up_off = F).  n_out = N or F.
void launch_gemm_w4(const bf16_t* x, int64_t ldx, const bf16_t* w, int64_t ldw, bf16_t* out,
                    int64_t ldo, int M, int n_out, int K, int up_off, bool swiglu, int abl,
                    hipStream_t s) {
  if (M <= 0) return;
  const int tiles_m = (M + kW4M - 1) / kW4M;
  const int tiles_n = swiglu ? n_out / 128 : n_out / kW4N;
  const int grid = tiles_m * tiles_n;
  // abl bits 4-5: row tiles per L2 group (16, 8, 4, 32): the 32 blocks an XCD runs at
  // once are group x (32 / group) tiles
  const int gmr = ((abl >> 4) & 3) == 0 ? 16 : ((abl >> 4) & 3) == 1 ? 8 : ((abl >> 4) & 3) == 2 ? 4 : 32;
  if ((abl & 7) && !swiglu) {
#define W4_ABL(A)                                                                       \
  gemm_w4_kernel<kW4Store, A><<<grid, 256, kW4Lds, s>>>(x, ldx, w, ldw, out, ldo, M, K, \
                                                        up_off, tiles_m, tiles_n, gmr)
    switch (abl & 7) {
      case 1: W4_ABL(1); break;
      case 2: W4_ABL(2); break;
      case 3: W4_ABL(3); break;
      case 4: W4_ABL(4); break;
      case 5: W4_ABL(5); break;
      case 6: W4_ABL(6); break;
      default: W4_ABL(7); break;
    }
#undef W4_ABL
    return;
  }
  const bool spread = abl & 8, early = abl & 64, mf32 = abl & 128;
  if (spread && early && !mf32 && (abl & 256) && (abl & 512) && K % 256 == 0 &&
      (int64_t)M * ldx * 2 < (int64_t)1 << 31 &&   // X / output offsets are 32-bit buffer
      (int64_t)M * ldo * 2 < (int64_t)1 << 31) {   // offsets
    // persistent: one workgroup per CU (160 KB of LDS each), at most one per tile
    static const int ncu = [] {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return n >= 8 ? n / 8 * 8 : 8;
    }();
    const int g = grid < ncu ? grid : ncu;
    constexpr int lds3 = 5 * kW4Img * 2;
    // abl bit 10 (cfg bit 14): stream-K over the last rounds, one workgroup per CU.  The
    // stream-K region: the partly filled last round (or the whole grid, when it is below
    // one round) when it is at least half full, else that round plus the full one before
    // it, so a split tile has one or two partners; none on whole rounds.  Each workgroup
    // needs >= 2 chunks of 4 K-tiles.
    if (abl & 1024) {
      const int r = grid % ncu, rounds = grid / ncu;
      const int sk = r == 0 ? 0 : (2 * r >= ncu ? r : (rounds >= 1 ? r + ncu : 0));
      float* ws = nullptr;
      int* flags = nullptr;
      if (sk > 0 && (int64_t)sk * (K / 256) >= 2 * ncu && gemm_w4p_sk_ws(ncu, s, &ws, &flags)) {
        uint32_t* err = kernel_error_words(s);
        if (swiglu)
          gemm_w4p_kernel<kW4Swiglu, true><<<ncu, 256, lds3, s>>>(
              x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr, sk, ws, flags, err);
        else
          gemm_w4p_kernel<kW4Store, true><<<ncu, 256, lds3, s>>>(
              x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr, sk, ws, flags, err);
        return;
      }
    }
    if (swiglu)
      gemm_w4p_kernel<kW4Swiglu><<<g, 256, lds3, s>>>(x, ldx, w, ldw, out, ldo, M, K, up_off,
                                                      tiles_m, tiles_n, gmr);
    else
      gemm_w4p_kernel<kW4Store><<<g, 256, lds3, s>>>(x, ldx, w, ldw, out, ldo, M, K, up_off,
                                                     tiles_m, tiles_n, gmr);
    return;
  }
  if (spread && early && !mf32 && (abl & 256)) {   // W image in three LDS slots
    constexpr int lds3 = 5 * kW4Img * 2;           // 160 KB
    if (swiglu)
      gemm_w4_kernel<kW4Swiglu, 0, true, true, 16, true><<<grid, 256, lds3, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr);
    else
      gemm_w4_kernel<kW4Store, 0, true, true, 16, true><<<grid, 256, lds3, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr);
    return;
  }
  if (spread && early && mf32) {
    if (swiglu)
      gemm_w4_kernel<kW4Swiglu, 0, true, true, 32><<<grid, 256, kW4Lds, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr);
    else
      gemm_w4_kernel<kW4Store, 0, true, true, 32><<<grid, 256, kW4Lds, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr);
    return;
  }
  if (spread && early) {
    if (swiglu)
      gemm_w4_kernel<kW4Swiglu, 0, true, true><<<grid, 256, kW4Lds, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr);
    else
      gemm_w4_kernel<kW4Store, 0, true, true><<<grid, 256, kW4Lds, s>>>(
          x, ldx, w, ldw, out, ldo, M, K, up_off, tiles_m, tiles_n, gmr);
    return;
  }
  if (swiglu) {
    if (spread)
      gemm_w4_kernel<kW4Swiglu, 0, true><<<grid, 256, kW4Lds, s>>>(x, ldx, w, ldw, out, ldo, M, K,
                                                                   up_off, tiles_m, tiles_n, gmr);
    else
      gemm_w4_kernel<kW4Swiglu><<<grid, 256, kW4Lds, s>>>(x, ldx, w, ldw, out, ldo, M, K, up_off,
                                                          tiles_m, tiles_n, gmr);
  } else {
    if (spread)
      gemm_w4_kernel<kW4Store, 0, true><<<grid, 256, kW4Lds, s>>>(x, ldx, w, ldw, out, ldo, M, K,
                                                                  up_off, tiles_m, tiles_n, gmr);
    else
      gemm_w4_kernel<kW4Store><<<grid, 256, kW4Lds, s>>>(x, ldx, w, ldw, out, ldo, M, K, up_off,
                                                         tiles_m, tiles_n, gmr);
  }
}

}  // namespace rfq
