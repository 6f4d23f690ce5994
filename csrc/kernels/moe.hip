// Mixture-of-experts kernels for Mixtral-8x7B (BASELINE config 5; SURVEY.md
// §2.4 K15-K18): router top-k, expert alignment (sort + pad), row gather,
// MFMA grouped GEMM, weighted combine.
//
// Flow per MoE layer (T tokens, top-k, E experts):
//   router_logits[T,E] --moe_topk--> (w[T,k], id[T,k])
//   --moe_align--> sorted_ids[P] (pair index t*k+j or -1), inv_pos[T*k],
//                  expert_of_block[P/128], num_blocks
//   --moe_gather--> xs[P, d]            (rows grouped by expert, padded to 128)
//   --grouped_gemm(w13)--> [P, 2F] --silu_mul--> [P, F] --grouped_gemm(w2)--> y[P, d]
//   --moe_combine--> out[T, d] = sum_j w[t,j] * y[inv_pos[t*k+j]]
// Every buffer is sized by the host from upper bounds and the GEMM reads the
// live block count from device memory, so the whole chain is graph-capturable.
#include <cstdlib>

#include "common.h"

namespace rfq {

// ---------------------------------------------------------------- router top-k
__global__ void moe_topk_kernel(const bf16_t* __restrict__ logits, int64_t stride, int T, int E,
                                int k, float* __restrict__ w_out, int32_t* __restrict__ id_out,
                                bool renorm) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  float l[64];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    l[e] = bf2f(logits[(int64_t)t * stride + e]);
    mx = fmaxf(mx, l[e]);
  }
  float den = 0.f;
  for (int e = 0; e < E; ++e) den += __expf(l[e] - mx);
  uint64_t taken = 0;
  float sel_sum = 0.f;
  float wv[8];
  int iv[8];
  for (int j = 0; j < k; ++j) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e)
      if (!((taken >> e) & 1ull) && (best < 0 || l[e] > bv)) { bv = l[e]; best = e; }
    taken |= 1ull << best;
    wv[j] = __expf(bv - mx) / den;
    iv[j] = best;
    sel_sum += wv[j];
  }
  for (int j = 0; j < k; ++j) {
    w_out[(int64_t)t * k + j] = renorm ? wv[j] / sel_sum : wv[j];
    id_out[(int64_t)t * k + j] = iv[j];
  }
}

// ------------------------------------------- fused router GEMV + top-k (small T)
// Latency path (T <= 64 tokens): one workgroup per token computes the E router
// logits (x . router_w^T, fp32 accumulate, rounded to bf16 like the hipBLASLt GEMM the
// throughput path uses) and the softmax top-k in one launch, instead of a
// 16x16-tile library GEMM plus moe_topk_kernel.
constexpr int kRouteMaxE = 16;

// EP: compile-time expert count (8 for Mixtral; 16 covers the rest, rows >= E are
// read as row 0 and ignored) so every router/x load of a thread is issued before the
// first FMA waits: one memory round trip instead of one per expert row.
template <int EP>
__global__ __launch_bounds__(256) void moe_route_kernel(
    const bf16_t* __restrict__ x, int64_t x_stride, const bf16_t* __restrict__ router, int d,
    int E, int k, float* __restrict__ w_out, int32_t* __restrict__ id_out, bool renorm) {
  __shared__ float part[EP][4];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = d >> 3;
  const s16x8* xr = reinterpret_cast<const s16x8*>(x + (int64_t)t * x_stride);
  float acc[EP];
#pragma unroll
  for (int e = 0; e < EP; ++e) acc[e] = 0.f;
  for (int c0 = threadIdx.x; c0 < nch; c0 += 2 * blockDim.x) {
    const int c1 = c0 + blockDim.x;
    const bool has1 = c1 < nch;
    s16x8 xv[2], wv[2][EP];
    xv[0] = xr[c0];
    xv[1] = xr[has1 ? c1 : c0];
#pragma unroll
    for (int e = 0; e < EP; ++e) {
      const s16x8* rr = reinterpret_cast<const s16x8*>(router + (int64_t)(e < E ? e : 0) * d);
      wv[0][e] = rr[c0];
      wv[1][e] = rr[has1 ? c1 : c0];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !has1) break;
      float xf[8];
      unpack8(xv[h], xf);
#pragma unroll
      for (int e = 0; e < EP; ++e) {
        float wf[8];
        unpack8(wv[h][e], wf);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[e] += xf[i] * wf[i];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EP; ++e) {
    const float v = wave_sum(acc[e]);
    if (lane == 0) part[e][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float l[EP];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    const float v = part[e][0] + part[e][1] + part[e][2] + part[e][3];
    l[e] = bf2f(f2bf(v));                      // the bf16 logits of the GEMM path
    mx = fmaxf(mx, l[e]);
  }
  float den = 0.f;
  for (int e = 0; e < E; ++e) den += __expf(l[e] - mx);
  uint32_t taken = 0;
  float sel_sum = 0.f, wsel[8];
  int isel[8];
  for (int j = 0; j < k; ++j) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e)
      if (!((taken >> e) & 1u) && (best < 0 || l[e] > bv)) { bv = l[e]; best = e; }
    taken |= 1u << best;
    wsel[j] = __expf(bv - mx) / den;
    isel[j] = best;
    sel_sum += wsel[j];
  }
  for (int j = 0; j < k; ++j) {
    w_out[(int64_t)t * k + j] = renorm ? wsel[j] / sel_sum : wsel[j];
    id_out[(int64_t)t * k + j] = isel[j];
  }
}

// ------------------------------------------------------------ align (one block)
// Counting sort of the T*k (token, slot) pairs by expert; each expert segment is
// padded to a multiple of block_m with -1 entries.
__global__ __launch_bounds__(1024) void moe_align_kernel(
    const int32_t* __restrict__ ids, int n, int E, int block_m, int32_t* __restrict__ sorted_ids,
    int32_t* __restrict__ inv_pos, int32_t* __restrict__ expert_of_block,
    int32_t* __restrict__ expert_offsets, int32_t* __restrict__ num_blocks, int cap,
    int block_cap) {
  __shared__ int cnt[64];
  __shared__ int off[65];
  __shared__ int cursor[64];
  for (int e = threadIdx.x; e < 64; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      off[e] = acc;
      cursor[e] = acc;
      acc += (cnt[e] + block_m - 1) / block_m * block_m;
    }
    off[E] = acc;
    *num_blocks = acc / block_m;
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= E; e += blockDim.x) expert_offsets[e] = off[e];
  const int total = off[E];
  for (int i = threadIdx.x; i < cap; i += blockDim.x) sorted_ids[i] = -1;
  for (int bi = threadIdx.x; bi < block_cap; bi += blockDim.x) {
    int e_of = -1;
    const int r = bi * block_m;
    if (r < total)
      for (int e = 0; e < E; ++e)
        if (r >= off[e] && r < off[e + 1]) e_of = e;
    expert_of_block[bi] = e_of;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int p = atomicAdd(&cursor[ids[i]], 1);
    sorted_ids[p] = i;
    inv_pos[i] = p;
  }
}

// ------------------------------------------------------------------- gather
__global__ __launch_bounds__(256) void moe_gather_kernel(const bf16_t* __restrict__ x,
                                                         int64_t x_stride,
                                                         const int32_t* __restrict__ sorted_ids,
                                                         int P, int d, int topk,
                                                         bf16_t* __restrict__ out) {
  const int cpr = d >> 3;
  const int64_t total = (int64_t)P * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr);
    const int sid = sorted_ids[r];
    s16x8 v = (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
    if (sid >= 0) v = reinterpret_cast<const s16x8*>(x + (int64_t)(sid / topk) * x_stride)[c];
    reinterpret_cast<s16x8*>(out + r * d)[c] = v;
  }
}

// --------------------------------------------------------------- grouped GEMM
// out[r, n] = sum_k x[r, k] * w[e(r), n, k]   (x: [P, K], w: [E, N, K] row-major)
// Tile 128x128, K-step 64, 4 waves each owning a 64x64 quadrant as 2x2
// mfma_f32_32x32x16_bf16 accumulators.  Both operands are K-contiguous, so the
// LDS images are [128 rows][64 k] with 128-B rows; chunk ch of row r lives at
// ch ^ ((r >> 1) & 7), which makes the 16-lane ds_read_b128 groups hit 16
// distinct 16-B slots (T2).  Register-staged double buffering: the next K-tile's
// global loads are issued before the current tile's MFMAs (T14).
constexpr int kBM = 128, kBN = 128, kBK = 64;

__device__ __forceinline__ int swz64(int row, int ch) { return ch ^ ((row >> 1) & 7); }

__global__ __launch_bounds__(256) void moe_grouped_gemm_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
    const int32_t* __restrict__ expert_of_block, const int32_t* __restrict__ num_blocks, int N,
    int K, int E) {
  __shared__ __attribute__((aligned(16))) bf16_t a_lds[kBM * kBK];
  __shared__ __attribute__((aligned(16))) bf16_t b_lds[kBN * kBK];
  const int ntn = N / kBN;
  const int rb = blockIdx.x / ntn, cn = blockIdx.x % ntn;
  if (rb >= *num_blocks) return;
  const int e = expert_of_block[rb];
  if (e < 0 || e >= E) return;      // padding block, or a remote expert's segment (EP)
  const bf16_t* xa = x + (int64_t)rb * kBM * K;
  const bf16_t* wb = w + ((int64_t)e * N + (int64_t)cn * kBN) * K;

  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h2 = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;  // quadrant

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  // staging: 128 rows x 8 chunks = 1024 chunks per operand, 4 per thread
  s16x8 ra[4], rbv[4];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7;
      ra[i] = reinterpret_cast<const s16x8*>(xa + (int64_t)row * K + k0)[ch];
      rbv[i] = reinterpret_cast<const s16x8*>(wb + (int64_t)row * K + k0)[ch];
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7;
      reinterpret_cast<s16x8*>(a_lds + row * kBK)[swz64(row, ch)] = ra[i];
      reinterpret_cast<s16x8*>(b_lds + row * kBK)[swz64(row, ch)] = rbv[i];
    }
  };

  load_tile(0);
  for (int k0 = 0; k0 < K; k0 += kBK) {
    store_tile();
    __syncthreads();
    if (k0 + kBK < K) load_tile(k0 + kBK);  // in flight under the MFMAs
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ++ks) {
      s16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + r;
        af[i] = reinterpret_cast<const s16x8*>(a_lds + row * kBK)[swz64(row, 2 * ks + h2)];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wn * 64 + j * 32 + r;
        bfr[j] = reinterpret_cast<const s16x8*>(b_lds + row * kBK)[swz64(row, 2 * ks + h2)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(af[i]), as_bf16x8(bfr[j]),
                                                              acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // C layout: col = lane & 31, row = (q&3) + 8(q>>2) + 4*h2
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = rb * kBM + wm * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h2;
        const int col = cn * kBN + wn * 64 + j * 32 + r;
        out[(int64_t)row * N + col] = f2bf(acc[i][j][q]);
      }
}

// Same tile and MFMA schedule, staged by LDS-DMA: every operand chunk goes
// global -> LDS with global_load_lds_dwordx4 (no VGPR round trip, no ds_write
// pass), two LDS stages so tile k+1 streams in while tile k is multiplied, and
// raw s_barrier + counted vmcnt so the in-flight stage survives the barrier
// (a __syncthreads() would drain it).  The LDS image is written lane-linearly,
// so the XOR swizzle is applied to the *source* address: the lane that fills
// slot (row, c') fetches global chunk c' ^ ((row >> 1) & 7) — the involution the
// ds_read side already uses.  All LDS lives in one __shared__ array.
// (glds16: common.h)

// BN = 128: 4 waves as 2x2 quadrants of 64x64 (4 MFMAs per 4 ds_read_b128).
// BN = 256: 4 waves as 2x2 of 64x128 (8 MFMAs per 6 reads) — LDS read traffic per
// MFMA drops by a third, which is what limits the 128-wide tile.
template <int BN>
__global__ __launch_bounds__(256) void moe_grouped_gemm_glds_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
    const int32_t* __restrict__ expert_of_block, const int32_t* __restrict__ num_blocks, int N,
    int K, int E) {
  constexpr int NJ = BN / 64;                       // 32-col MFMA tiles per wave
  constexpr int BI = BN / 32;                       // B glds instructions per thread per stage
  constexpr int STAGE = (kBM + BN) * kBK;           // elements per stage
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int ntn = N / BN;
  const int rb = blockIdx.x / ntn, cn = blockIdx.x % ntn;
  if (rb >= *num_blocks) return;
  const int e = expert_of_block[rb];
  if (e < 0 || e >= E) return;      // padding block, or a remote expert's segment (EP)
  const bf16_t* xa = x + (int64_t)rb * kBM * K;
  const bf16_t* wb = w + ((int64_t)e * N + (int64_t)cn * BN) * K;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h2 = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;

  // lane's source offset / wave-uniform LDS destination per glds instruction
  int src_off[BI];
  int dst_base[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int idx0 = wid * 64 + 256 * i;
    const int idx = idx0 + lane, row = idx >> 3, chp = idx & 7;
    src_off[i] = row * K + (chp ^ ((row >> 1) & 7)) * 8;
    dst_base[i] = idx0 * 8;
  }
  auto issue = [&](int stage, int k0) {
    bf16_t* sa = smem + stage * STAGE;
    bf16_t* sb = sa + kBM * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xa + src_off[i] + k0, sa + dst_base[i]);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      glds16(wb + src_off[i] + k0, sb + dst_base[i]);
  };

  f32x16 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk = K / kBK;
  issue(0, 0);
  if (nk > 1) issue(1, kBK);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) {
      if constexpr (BN == 256) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const bf16_t* a_lds = smem + st * STAGE;
    const bf16_t* b_lds = a_lds + kBM * kBK;
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ++ks) {
      s16x8 af[2], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + r;
        af[i] = reinterpret_cast<const s16x8*>(a_lds + row * kBK)[swz64(row, 2 * ks + h2)];
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * (BN / 2) + j * 32 + r;
        bfr[j] = reinterpret_cast<const s16x8*>(b_lds + row * kBK)[swz64(row, 2 * ks + h2)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(af[i]), as_bf16x8(bfr[j]),
                                                              acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                 // stage st fully consumed by every wave
    if (kt + 2 < nk) issue(st, (kt + 2) * kBK);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = rb * kBM + wm * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h2;
        const int col = cn * BN + wn * (BN / 2) + j * 32 + r;
        out[(int64_t)row * N + col] = f2bf(acc[i][j][q]);
      }
}


// ------------------------------------------------------------------ combine
__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16_t* __restrict__ y,
                                                          const int32_t* __restrict__ inv_pos,
                                                          const float* __restrict__ wts, int T,
                                                          int k, int d, bf16_t* __restrict__ out,
                                                          int64_t out_stride) {
  const int cpr = d >> 3;
  const int64_t total = (int64_t)T * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / cpr;
    const int c = (int)(i - t * cpr);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = wts[t * k + j];
      if (wj == 0.f) continue;        // pair routed to another rank's expert (EP)
      const int p = inv_pos[t * k + j];
      float v[8];
      unpack8(reinterpret_cast<const s16x8*>(y + (int64_t)p * d)[c], v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * v[q];
    }
    reinterpret_cast<s16x8*>(out + t * out_stride)[c] = pack8(acc);
  }
}

// Split-K variant: y = sum over `splits` fp32 slabs (moe_skinny split-K w2 partials).
__global__ __launch_bounds__(256) void moe_combine_splitk_kernel(
    const float* __restrict__ yf, int splits, int64_t slab, const int32_t* __restrict__ inv_pos,
    const float* __restrict__ wts, int T, int k, int d, bf16_t* __restrict__ out,
    int64_t out_stride) {
  const int cpr = d >> 3;
  const int64_t total = (int64_t)T * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / cpr;
    const int c = (int)(i - t * cpr);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = wts[t * k + j];
      if (wj == 0.f) continue;        // pair routed to another rank's expert (EP)
      const int p = inv_pos[t * k + j];
      for (int sl = 0; sl < splits; ++sl) {
        const float4* src = reinterpret_cast<const float4*>(yf + sl * slab + (int64_t)p * d) + 2 * c;
        const float4 a = src[0], b = src[1];
        acc[0] += wj * a.x; acc[1] += wj * a.y; acc[2] += wj * a.z; acc[3] += wj * a.w;
        acc[4] += wj * b.x; acc[5] += wj * b.y; acc[6] += wj * b.z; acc[7] += wj * b.w;
      }
    }
    reinterpret_cast<s16x8*>(out + t * out_stride)[c] = pack8(acc);
  }
}

// Combine after the throughput-path w2 (gemm_w4.hip GROUPED KS = 2): the same split rule
// on the same offsets tells which the GEMM wrote -- two fp32 K-slice slabs (yf, slab
// stride in floats) or the bf16 rows y.
__global__ __launch_bounds__(256) void moe_combine_w2_kernel(
    const bf16_t* __restrict__ y, const float* __restrict__ yf, int64_t slab,
    const int32_t* __restrict__ offs, int E, int tiles_n, int cus,
    const int32_t* __restrict__ inv_pos, const float* __restrict__ wts, int T, int k, int d,
    bf16_t* __restrict__ out, int64_t out_stride) {
  const bool split = moe_w2_ksplit(moe_live_chunks(offs, E) * tiles_n, cus) == 2;
  const int cpr = d >> 3;
  const int64_t total = (int64_t)T * cpr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / cpr;
    const int c = (int)(i - t * cpr);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = wts[t * k + j];
      if (wj == 0.f) continue;        // pair routed to another rank's expert (EP)
      const int p = inv_pos[t * k + j];
      if (split) {
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          const float4* src = reinterpret_cast<const float4*>(yf + sl * slab + (int64_t)p * d) + 2 * c;
          const float4 a = src[0], b = src[1];
          acc[0] += wj * a.x; acc[1] += wj * a.y; acc[2] += wj * a.z; acc[3] += wj * a.w;
          acc[4] += wj * b.x; acc[5] += wj * b.y; acc[6] += wj * b.z; acc[7] += wj * b.w;
        }
      } else {
        float v[8];
        unpack8(reinterpret_cast<const s16x8*>(y + (int64_t)p * d)[c], v);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += wj * v[q];
      }
    }
    reinterpret_cast<s16x8*>(out + t * out_stride)[c] = pack8(acc);
  }
}

static inline int moe_stream_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

void launch_moe_topk(const bf16_t* logits, int64_t stride, int T, int E, int k, float* w,
                     int32_t* ids, bool renorm, hipStream_t s) {
  if (T == 0) return;
  moe_topk_kernel<<<(T + 127) / 128, 128, 0, s>>>(logits, stride, T, E, k, w, ids, renorm);
}

void launch_moe_route(const bf16_t* x, int64_t x_stride, const bf16_t* router, int T, int d,
                      int E, int k, float* w, int32_t* ids, bool renorm, hipStream_t s) {
  if (T == 0) return;
  if (E <= 8)
    moe_route_kernel<8><<<T, 256, 0, s>>>(x, x_stride, router, d, E, k, w, ids, renorm);
  else
    moe_route_kernel<kRouteMaxE><<<T, 256, 0, s>>>(x, x_stride, router, d, E, k, w, ids, renorm);
}

void launch_moe_align(const int32_t* ids, int n, int E, int block_m, int32_t* sorted_ids,
                      int32_t* inv_pos, int32_t* expert_of_block, int32_t* expert_offsets,
                      int32_t* num_blocks, int cap, int block_cap, hipStream_t s) {
  moe_align_kernel<<<1, 1024, 0, s>>>(ids, n, E, block_m, sorted_ids, inv_pos, expert_of_block,
                                      expert_offsets, num_blocks, cap, block_cap);
}

void launch_moe_gather(const bf16_t* x, int64_t x_stride, const int32_t* sorted_ids, int P,
                         int d, int topk, bf16_t* out, hipStream_t s) {
  if (P == 0) return;
  moe_gather_kernel<<<moe_stream_grid((int64_t)P * (d >> 3)), 256, 0, s>>>(x, x_stride, sorted_ids,
                                                                          P, d, topk, out);
}

// ------------------------------------------------------ grouped GEMM, 8 waves
// out[r, n] = sum_k x[r, k] * w[e(r), n, k] on a 128 (rows) x 256 (weight rows) tile,
// K-step 64, 512 threads = 8 waves as 2 (64 rows) x 4 (64 weight rows).
//  * operands swapped (C^T = W X^T): the weight tile is the MFMA A operand, so a
//    lane ends up holding 4 consecutive output columns of one row (8-byte stores)
//    and, with SWI, the gate and up values of the same (row, column) -- the wave's
//    64 weight rows are 32 gate rows + the 32 matching up rows (up_off apart in w),
//    so the SwiGLU epilogue writes act directly (no h13 round trip, no silu_mul);
//  * LDS-DMA (global_load_lds_dwordx4) into a 3-stage ring (3 x 48 KB): stage k+2
//    is issued while stage k is multiplied and waited with a counted vmcnt, one raw
//    barrier per K-step (the in-flight stage survives it);
//  * images [rows][64 k] with chunk ch of row r at ch ^ ((r >> 1) & 7) (T2), the
//    swizzle applied on the DMA source address (lane-linear destination).
// Block order (weight-tile reuse): the ~2 GB of Mixtral w13 is far larger than L2
// and the MALL, so every (expert, weight tile) must be consumed by all of that
// expert's row blocks while it is resident.  The live blocks (< num_blocks x ntn)
// are renumbered expert-major, then weight tile, then row block, and that order is
// laid out contiguously per XCD (bijective T1 remap over the live count, so
// padding capacity does not unbalance the XCDs): the few row blocks of one expert
// that share a weight tile run back to back on one XCD and hit its L2.
constexpr int kM8 = 128, kN8 = 256, kK8 = 64;
constexpr int kStage8 = (kM8 + kN8) * kK8;        // bf16 elements per stage
constexpr int kRing8 = 3;

template <bool SWI>
__global__ __launch_bounds__(512) void moe_gemm8_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
    const int32_t* __restrict__ expert_of_block, const int32_t* __restrict__ num_blocks,
    const int32_t* __restrict__ expert_offsets, int n_out, int K, int E, int64_t w_rows,
    int up_off) {
  extern __shared__ __attribute__((aligned(16))) char smem8[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem8);
  const int ntn = SWI ? n_out / 128 : n_out / kN8;
  const int nlive = *num_blocks * ntn;
  const int bid = blockIdx.x;
  if (bid >= nlive) return;
  const int q8 = nlive >> 3, r8 = nlive & 7, xcd = bid & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int e = expert_of_block[wg / ntn];
  if (e < 0 || e >= E) return;      // padding block, or a remote expert's segment (EP)
  const int s0 = expert_offsets[e] / kM8, nbe = expert_offsets[e + 1] / kM8 - s0;
  const int local = wg - s0 * ntn;
  const int cn = local / nbe, rb = s0 + local % nbe;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h2 = lane >> 5;
  const int wm = wid & 1, wn = wid >> 1;
  const bf16_t* xa = x + (int64_t)rb * kM8 * K;
  const bf16_t* we = w + (int64_t)e * w_rows * K;

  // DMA: per stage 16 (A) + 32 (B) wave-instructions of 1 KiB (8 rows of 128 B);
  // wave w issues A pieces 2w, 2w+1 and B pieces 4w..4w+3
  const int prow = lane >> 3, pch = lane & 7;
  const bf16_t* asrc[2];
  const bf16_t* bsrc[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (2 * wid + i) + prow;
    asrc[i] = xa + (int64_t)row * K + 8 * (pch ^ ((row >> 1) & 7));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 8 * (4 * wid + i) + prow;     // tile row
    int64_t wr;
    if constexpr (SWI) {
      // tile rows [64v, 64v + 32) = gate rows cn*128 + 32v + c, [64v + 32, 64v + 64) = up
      const int v = j >> 6, h = (j >> 5) & 1, c = j & 31;
      wr = (h ? up_off : 0) + cn * 128 + 32 * v + c;
    } else {
      wr = (int64_t)cn * kN8 + j;
    }
    bsrc[i] = we + wr * K + 8 * (pch ^ ((j >> 1) & 7));
  }
  auto issue = [&](int kt) {
    bf16_t* st = lds + (kt % kRing8) * kStage8;
    const int k0 = kt * kK8;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(asrc[i] + k0, (lds_void_t*)(st + (2 * wid + i) * 512), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(bsrc[i] + k0,
                                       (lds_void_t*)(st + kM8 * kK8 + (4 * wid + i) * 512), 16, 0, 0);
  };

  f32x16 acc[2][2];                 // [weight subtile i][row subtile j]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk = K / kK8;
  issue(0);
  if (nk > 1) issue(1);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) issue(kt + 2);            // into the stage kt-1 vacated
    const bf16_t* a_lds = lds + (kt % kRing8) * kStage8;   // x rows
    const bf16_t* b_lds = a_lds + kM8 * kK8;               // weight rows
    s16x8 wf[4][2], xf[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wn * 64 + i * 32 + r;
        wf[ks][i] = reinterpret_cast<const s16x8*>(b_lds + row * kK8)[swz64(row, 2 * ks + h2)];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wm * 64 + j * 32 + r;
        xf[ks][j] = reinterpret_cast<const s16x8*>(a_lds + row * kK8)[swz64(row, 2 * ks + h2)];
      }
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wf[ks][i]),
                                                              as_bf16x8(xf[ks][j]), acc[i][j],
                                                              0, 0, 0);
    // fragments two k-slices ahead of their MFMAs (the compiler otherwise issues each
    // slice's reads right before its MFMAs and waits out the LDS latency 4x per step)
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      if (ks < 2) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
    }
    // stage kt+1 landed (kt+2 may stay in flight); every wave done with stage kt
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // C^T lane layout: weight row (q&3) + 8(q>>2) + 4h2 of subtile i, x row r of subtile j
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t row = (int64_t)rb * kM8 + wm * 64 + j * 32 + r;
    if constexpr (SWI) {
      bf16_t* orow = out + row * n_out + cn * 128 + wn * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float gf = bf2f(f2bf(acc[0][j][4 * g + u]));   // = the h13 GEMM's bf16
          const float sg = gf / (1.f + __expf(-gf));
          o[u] = bf2f(f2bf(sg)) * bf2f(f2bf(acc[1][j][4 * g + u]));
        }
        uint2 v;
        v.x = pack_bf16x2(o[0], o[1]);
        v.y = pack_bf16x2(o[2], o[3]);
        *reinterpret_cast<uint2*>(orow + 8 * g + 4 * h2) = v;
      }
    } else {
      bf16_t* orow = out + row * n_out + cn * kN8 + wn * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint2 v;
          v.x = pack_bf16x2(acc[i][j][4 * g + 0], acc[i][j][4 * g + 1]);
          v.y = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          *reinterpret_cast<uint2*>(orow + 32 * i + 8 * g + 4 * h2) = v;
        }
    }
  }
}

// out = x W_e^T per 128-row expert block (SWI: out = silu(x Wg^T) * (x Wu^T), n_out = F,
// w = [Wg; Wu] with up rows at up_off).  Shapes: n_out % 256 == 0 (128 with SWI),
// K % 64 == 0.
// ---------------------------------------------------- grouped GEMM, 256 x 256 tile
// Same contract as moe_gemm8 on a 256-row x 256-weight-row tile: a third fewer
// staged bytes per FLOP (the 128 x 256 tile is bound by the per-CU vector-memory
// path, profiles/r2_moe_grouped_gemm.md).  A tile covers two consecutive 128-row
// blocks of ONE expert; when an expert has an odd block count its last tile holds
// one block, and the waves of the empty half skip their DMA pieces and MFMAs (the
// SIMD then runs one wave instead of two, so the half tile costs about half).
// 8 waves = 2 (128 rows) x 4 (64 weight rows), 8 accumulators of 32 x 32 per wave,
// K-step 64, two 64-KB LDS stages by LDS-DMA, one barrier per K-step.
constexpr int kM16 = 256, kN16 = 256, kK16 = 64;
constexpr int kStage16 = (kM16 + kN16) * kK16;     // bf16 elements per stage

template <bool SWI>
__global__ __launch_bounds__(512) void moe_gemm16_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
    const int32_t* __restrict__ num_blocks, const int32_t* __restrict__ expert_offsets,
    int n_out, int K, int E, int64_t w_rows, int up_off) {
  extern __shared__ __attribute__((aligned(16))) char smem16[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem16);
  const int ntn = SWI ? n_out / 128 : n_out / kN16;
  // live tiles: sum over experts of ceil(blocks / 2) per weight tile
  int nchunks = 0;
  for (int e = 0; e < E; ++e) {
    const int nb = expert_offsets[e + 1] / kM8 - expert_offsets[e] / kM8;
    nchunks += (nb + 1) >> 1;
  }
  const int nlive = nchunks * ntn;
  const int bid = blockIdx.x;
  if (bid >= nlive || *num_blocks == 0) return;
  const int q8 = nlive >> 3, r8 = nlive & 7, xcd = bid & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // expert-major, then weight tile, then 256-row chunk (T1 remap above keeps the
  // chunks that share a weight tile back to back on one XCD)
  int e = 0, p0 = 0, s0 = 0, nbe = 0, che = 0;
  for (; e < E; ++e) {
    s0 = expert_offsets[e] / kM8;
    nbe = expert_offsets[e + 1] / kM8 - s0;
    che = (nbe + 1) >> 1;
    if (wg < (p0 + che) * ntn) break;
    p0 += che;
  }
  if (e >= E) return;
  const int local = wg - p0 * ntn;
  const int cn = local / che, chunk = local % che;
  const int rb = s0 + 2 * chunk;                   // first 128-row block of the tile
  const bool two = 2 * chunk + 1 < nbe;            // second block present
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h2 = lane >> 5;
  const int wm = wid >> 2, wn = wid & 3;           // waves 4-7 own rows 128-255
  const bool active = two || wm == 0;              // wave-uniform
  const bf16_t* xa = x + (int64_t)rb * kM8 * K;
  const bf16_t* we = w + (int64_t)e * w_rows * K;

  // DMA: 32 A pieces (8 rows each) + 32 B pieces per stage; wave w issues A pieces
  // 4w..4w+3 (rows 32w.. -> waves 4-7 fill the second block) and B pieces 4w..4w+3
  const int prow = lane >> 3, pch = lane & 7;
  const bf16_t* asrc[4];
  const bf16_t* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wid + i) + prow;
    asrc[i] = xa + (int64_t)row * K + 8 * (pch ^ ((row >> 1) & 7));
    const int j = row;                             // weight tile row
    int64_t wr;
    if constexpr (SWI) {
      const int v = j >> 6, h = (j >> 5) & 1, c = j & 31;
      wr = (h ? up_off : 0) + cn * 128 + 32 * v + c;
    } else {
      wr = (int64_t)cn * kN16 + j;
    }
    bsrc[i] = we + wr * K + 8 * (pch ^ ((j >> 1) & 7));
  }
  auto issue = [&](int kt) {
    bf16_t* st = lds + (kt & 1) * kStage16;
    const int k0 = kt * kK16;
    if (active) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds(asrc[i] + k0, (lds_void_t*)(st + (4 * wid + i) * 512), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(bsrc[i] + k0,
                                       (lds_void_t*)(st + kM16 * kK16 + (4 * wid + i) * 512), 16, 0, 0);
  };

  f32x16 acc[2][4];                 // [weight subtile i][row subtile j]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk = K / kK16;
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) issue(kt + 1);                // into the stage kt-1 vacated
    if (active) {
      const bf16_t* a_lds = lds + (kt & 1) * kStage16;    // x rows
      const bf16_t* b_lds = a_lds + kM16 * kK16;           // weight rows
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s16x8 wf[2], xf[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wn * 64 + i * 32 + r;
          wf[i] = reinterpret_cast<const s16x8*>(b_lds + row * kK16)[swz64(row, 2 * ks + h2)];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wm * 128 + j * 32 + r;
          xf[j] = reinterpret_cast<const s16x8*>(a_lds + row * kK16)[swz64(row, 2 * ks + h2)];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(wf[i]), as_bf16x8(xf[j]),
                                                                acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // stage kt+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every wave done with stage kt
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (!active) return;

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t row = (int64_t)rb * kM8 + wm * 128 + j * 32 + r;
    if constexpr (SWI) {
      bf16_t* orow = out + row * n_out + cn * 128 + wn * 32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float gf = bf2f(f2bf(acc[0][j][4 * g + u]));   // = the h13 GEMM's bf16
          const float sg = gf / (1.f + __expf(-gf));
          o[u] = bf2f(f2bf(sg)) * bf2f(f2bf(acc[1][j][4 * g + u]));
        }
        uint2 v;
        v.x = pack_bf16x2(o[0], o[1]);
        v.y = pack_bf16x2(o[2], o[3]);
        *reinterpret_cast<uint2*>(orow + 8 * g + 4 * h2) = v;
      }
    } else {
      bf16_t* orow = out + row * n_out + cn * kN16 + wn * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint2 v;
          v.x = pack_bf16x2(acc[i][j][4 * g + 0], acc[i][j][4 * g + 1]);
          v.y = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          *reinterpret_cast<uint2*>(orow + 32 * i + 8 * g + 4 * h2) = v;
        }
    }
  }
}

void launch_moe_gemm8(const bf16_t* x, const bf16_t* w, bf16_t* out,
                      const int32_t* expert_of_block, const int32_t* num_blocks,
                      const int32_t* expert_offsets, int max_blocks, int n_out, int K, int E,
                      int64_t w_rows, int up_off, bool swiglu, int tile, hipStream_t s) {
  if (max_blocks == 0) return;
  if (tile == 256) {
    // live 256-row tiles <= (blocks + experts) / 2 per weight tile
    const int chunks = (max_blocks + E) / 2 + 1;
    const size_t lds16 = 2 * kStage16 * sizeof(bf16_t);
    if (swiglu)
      moe_gemm16_kernel<true><<<chunks * (n_out / 128), 512, lds16, s>>>(
          x, w, out, num_blocks, expert_offsets, n_out, K, E, w_rows, up_off);
    else
      moe_gemm16_kernel<false><<<chunks * (n_out / kN16), 512, lds16, s>>>(
          x, w, out, num_blocks, expert_offsets, n_out, K, E, w_rows, up_off);
    return;
  }
  const size_t lds = kRing8 * kStage8 * sizeof(bf16_t);
  if (swiglu)
    moe_gemm8_kernel<true><<<max_blocks * (n_out / 128), 512, lds, s>>>(
        x, w, out, expert_of_block, num_blocks, expert_offsets, n_out, K, E, w_rows, up_off);
  else
    moe_gemm8_kernel<false><<<max_blocks * (n_out / kN8), 512, lds, s>>>(
        x, w, out, expert_of_block, num_blocks, expert_offsets, n_out, K, E, w_rows, up_off);
}

void launch_moe_grouped_gemm(const bf16_t* x, const bf16_t* w, bf16_t* out,
                             const int32_t* expert_of_block, const int32_t* num_blocks,
                             int max_blocks, int N, int K, int E, hipStream_t s) {
  if (max_blocks == 0) return;
  static const int impl = [] {
    const char* v = getenv("RFQ_MOE_GEMM");
    return v ? atoi(v) : 1;
  }();
  if (impl == 2 && N % 256 == 0)
    moe_grouped_gemm_glds_kernel<256><<<max_blocks * (N / 256), 256, 0, s>>>(
        x, w, out, expert_of_block, num_blocks, N, K, E);
  else if (impl >= 1)
    moe_grouped_gemm_glds_kernel<128><<<max_blocks * (N / kBN), 256, 0, s>>>(
        x, w, out, expert_of_block, num_blocks, N, K, E);
  else
    moe_grouped_gemm_kernel<<<max_blocks * (N / kBN), 256, 0, s>>>(x, w, out, expert_of_block,
                                                                    num_blocks, N, K, E);
}

void launch_moe_combine_splitk(const float* yf, int splits, int64_t slab, const int32_t* inv_pos,
                               const float* w, int T, int k, int d, bf16_t* out,
                               int64_t out_stride, hipStream_t s) {
  if (T == 0) return;
  moe_combine_splitk_kernel<<<moe_stream_grid((int64_t)T * (d >> 3)), 256, 0, s>>>(
      yf, splits, slab, inv_pos, w, T, k, d, out, out_stride);
}

void launch_moe_combine_w2(const bf16_t* y, const float* yf, int64_t slab, const int32_t* offs,
                           int E, int tiles_n, int cus, const int32_t* inv_pos, const float* w,
                           int T, int k, int d, bf16_t* out, int64_t out_stride, hipStream_t s) {
  if (T == 0) return;
  moe_combine_w2_kernel<<<moe_stream_grid((int64_t)T * (d >> 3)), 256, 0, s>>>(
      y, yf, slab, offs, E, tiles_n, cus, inv_pos, w, T, k, d, out, out_stride);
}

void launch_moe_combine(const bf16_t* y, const int32_t* inv_pos, const float* w, int T, int k,
                        int d, bf16_t* out, int64_t out_stride, hipStream_t s) {
  if (T == 0) return;
  moe_combine_kernel<<<moe_stream_grid((int64_t)T * (d >> 3)), 256, 0, s>>>(y, inv_pos, w, T, k, d,
                                                                          out, out_stride);
}

}  // namespace rfq
