// Split-K weight-streaming GEMV core (M <= 16) and its epilogues, used by
// gemm_skinny.hip (gemv_splitk / skinny kernels).
#pragma once
#include "common.h"

namespace rfq {

template <bool NTL>
__device__ __forceinline__ s16x8 ldw(const bf16_t* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(p));
  else return *reinterpret_cast<const s16x8*>(p);
}

typedef __attribute__((address_space(1))) unsigned long long gu64;   // global, for sc1 access

// Optional epilogue of the o / down projections on the latency path (TP = 1):
// residual <- bf16(Y + residual); out <- rmsnorm(residual) * w, i.e. the next
// fused_add_rms_norm, run by the workgroup that finishes last.  Every workgroup
// publishes its Y tile write-through (8-byte sc1 stores, vmcnt(0) in every wave,
// barrier, then a relaxed agent-scope ticket on *counter: no release fence); the one
// drawing gridDim.x - 1 reads Y back with sc1 loads (no acquire), normalises the M
// rows and resets the counter for the next launch on the stream
// (cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2, §6 Guideline 16 R1).
// No workgroup waits on another, so there is no spin and no co-residency assumption.
struct NormEpi {
  bf16_t* residual;
  int64_t res_stride;
  const bf16_t* w;
  bf16_t* out;
  int64_t out_stride;
  float eps;
  unsigned* counter;
  float* partials;    // split-K (KS > 1): fp32 partial slabs [KS][M][N], slab stride pslab
  int64_t pslab;
};

constexpr int kNormMaxChunks = 4;       // hidden <= 8 * threads * 4 (8192 at 256 threads)

template <int NTH, int KS = 1>
__device__ __forceinline__ void last_block_add_norm(const bf16_t* Y, int64_t ldy, int N, int M,
                                                    const NormEpi& ep, float* scratch) {
  const int nchunk = N >> 3;
  const s16x8* wr = reinterpret_cast<const s16x8*>(ep.w);
  for (int m = 0; m < M; ++m) {
    const s16x8* yr = reinterpret_cast<const s16x8*>(Y + (int64_t)m * ldy);
    s16x8* rr = reinterpret_cast<s16x8*>(ep.residual + (int64_t)m * ep.res_stride);
    s16x8* orow = reinterpret_cast<s16x8*>(ep.out + (int64_t)m * ep.out_stride);
    float v[kNormMaxChunks][8];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < kNormMaxChunks; ++k) {
      const int c = threadIdx.x + k * NTH;
      if (c < nchunk) {
        float a[8], b[8];
        if constexpr (KS == 1) {
          const gu64* yq = (const gu64*)(yr + c);
          const unsigned long long y0 = __hip_atomic_load(yq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned long long y1 = __hip_atomic_load(yq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            a[i] = bf2f((bf16_t)(y0 >> (16 * i)));
            a[4 + i] = bf2f((bf16_t)(y1 >> (16 * i)));
          }
        } else {
          // sum the K slices' fp32 partials (sc1 loads), round like the GEMM output
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = 0.f;
#pragma unroll
          for (int sl = 0; sl < KS; ++sl) {
            const gu64* pq = (const gu64*)(ep.partials + sl * ep.pslab + (int64_t)m * N + c * 8);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const unsigned long long u =
                  __hip_atomic_load(pq + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              a[2 * q] += __uint_as_float((uint32_t)u);
              a[2 * q + 1] += __uint_as_float((uint32_t)(u >> 32));
            }
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = bf2f(f2bf(a[i]));
        }
        unpack8(rr[c], b);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] += b[i];
        const s16x8 packed = pack8(a);
        rr[c] = packed;
        unpack8(packed, v[k]);           // normalise the rounded residual (= fused_add_rms_norm)
#pragma unroll
        for (int i = 0; i < 8; ++i) ss += v[k][i] * v[k][i];
      }
    }
    ss = block_sum(ss, scratch);
    const float r = rsqrtf(ss / (float)N + ep.eps);
#pragma unroll
    for (int k = 0; k < kNormMaxChunks; ++k) {
      const int c = threadIdx.x + k * NTH;
      if (c < nchunk) {
        float wf[8], o[8];
        unpack8(wr[c], wf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = v[k][i] * r * wf[i];
        orow[c] = pack8(o);
      }
    }
  }
}

// Optional epilogue of the fused QKV projection on the latency path: NeoX RoPE on
// q and k and the paged KV-cache append (rope_kv.hip) applied to the fp32
// accumulators.  The workgroup's two 16-feature tiles are the rotate-half partners
// [h*128 + 16j, +16) and [h*128 + 64 + 16j, +16) of one head, so every lane holds both
// halves of its 4 rotary pairs in the same accumulator slots: no shuffles.  q goes
// back to Y (attention reads it there), k/v go straight to the cache.
struct RopeEpi {
  const int32_t* positions;
  const float* cos_sin;          // [max_pos, 128] fp32: cos at [d], sin at [64 + d]
  const int32_t* slots;          // KV slot per token, -1 = padding (no cache write)
  bf16_t* k_cache;               // [blocks, Hkv, BS, 128]
  bf16_t* v_cache;
  int Hq, Hkv, BS;
};

// ---------------------------------------------------------------------------
// Split-K weight-streaming GEMV (M <= 16) with an in-launch reduction.
//
// The o / down projections have only N/16 = 256 output tiles: one workgroup per CU
// whose waves each stream a long K range as a few dependent load rounds, so the
// kernel is bound by (rounds x HBM latency), not by bandwidth.  Here the grid is
// tiles x KS: KS workgroups per output tile each stream K/KS (more, shorter
// streams in flight on every CU), publish their fp32 partial tile write-through,
// and the last of a tile's KS arrivals (per-tile ticket) sums the slices in slice
// order and runs the epilogue.  Every hand-off is the "every load sc1" form of
// cdna_hip_programming.md §6 Guideline 16: sc1 8-byte stores drained by vmcnt(0) +
// barrier, relaxed agent tickets, sc1 loads of all handed-off bytes; counters are
// left at zero.
//
// Epilogues (EPI):
//   kGvPlain  Y[M, N] bf16.
//   kGvNorm   Y, then finished tiles take a second ticket and the grid's last one
//             runs the residual-add RMSNorm (last_block_add_norm).
//   kGvSwi    the tile is a (gate, up) pair of 16-row blocks [n0, +16) and
//             [up_off + n0, +16) of the stacked gate|up weight; Y[M, F] = SwiGLU,
//             rounded exactly like the skinny SWI epilogue / act.hip silu_mul.
//             Small shards (TP = 8: F = 3,584 -> 224 tiles < 256 CUs) get KS x more
//             workgroups than the one-tile-per-workgroup skinny kernel.
//   kGvRope   the tile is a rotate-half pair [h*128 + 16j, +16), [h*128 + 64 + 16j,
//             +16) of one head (RopeEpi): NeoX RoPE on q / k, q to Y, k / v appended
//             to the paged cache.  The TP = 8 QKV shard (N = 1,280) has only 40 such
//             pairs: split K is what lets it use more than 40 CUs.
enum { kGvPlain = 0, kGvNorm = 1, kGvSwi = 2, kGvRope = 3 };

//
// TL (cfg bit 4): W is stored in the decode-tiled layout (ops.tile_weight): for
// every 16-row tile T and 128-wide k block B, the four 16x32 MFMA A-fragments in
// lane order, i.e. element ((T * K/128 + B) * 4 + j) * 512 + lane * 8 + e holds
// W[16 T + (lane & 15)][128 B + 32 j + 8 (lane >> 4) + e].  Every wave load is then
// 1 KB contiguous (8 whole 128-B lines) instead of 16 half lines of 16 rows, and a
// tile's k-blocks follow each other: one sequential 4 KB stream per k-step.
// NTL (cfg bit 5): weight loads non-temporal (nt): each weight byte is read once per
// step by one CU, so it need not displace the activations / partials in L2.
// One work unit (16-row tile bt = unit / KS, K slice unit % KS) of the split-K GEMV;
// every early return below is workgroup-uniform.
template <int NW, int U, int EPI, bool TL, bool NTL>
__device__ __forceinline__ void gemv_splitk_unit(
    int unit, int ntile, const bf16_t* __restrict__ X, int64_t ldx,
    const bf16_t* __restrict__ W, int K, bf16_t* __restrict__ Y, int64_t ldy, int M, int KS,
    float* __restrict__ part, int Nn, unsigned* __restrict__ tile_cnt, const NormEpi& ep,
    const RopeEpi& re, int up_off) {
  constexpr int NT = (EPI == kGvSwi || EPI == kGvRope) ? 2 : 1;
  __shared__ f32x4 red[NW][NT][64];
  __shared__ float nscratch[17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int bt = unit / KS, slice = unit - bt * KS;
  // GEMM rows of the tile's NT 16-row blocks
  int row0[NT];
  if constexpr (EPI == kGvRope) {
    row0[0] = (bt >> 2) * 128 + (bt & 3) * 16;
    row0[NT - 1] = row0[0] + 64;
  } else if constexpr (EPI == kGvSwi) {
    row0[0] = bt * 16;
    row0[NT - 1] = up_off + bt * 16;
  } else {
    row0[0] = bt * 16;
  }
  const int nks_all = K >> 7;
  const int sl0 = slice * nks_all / KS, nks = (slice + 1) * nks_all / KS - sl0;
  const int ks0 = sl0 + wave * nks / NW, ks1 = sl0 + (wave + 1) * nks / NW;
  const bf16_t* wp[NT];
  // element step between k-steps (128 k) and between the four 32-k MFMA slices
  constexpr int KSTEP = TL ? 2048 : 128, JSTEP = TL ? 512 : 32;
#pragma unroll
  for (int a = 0; a < NT; ++a)
    wp[a] = TL ? W + (int64_t)(row0[a] >> 4) * (K >> 7) * 2048 + lane * 8
               : W + (int64_t)(row0[a] + r) * K + g * 8;
  const bool xv = r < M;

  const bf16_t* xp = X + (int64_t)(xv ? r : 0) * ldx + g * 8;
  const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  f32x4 acc[NT];
#pragma unroll
  for (int a = 0; a < NT; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  int ks = ks0;
  for (; ks + U <= ks1; ks += U) {
    s16x8 w[U][NT][4], x[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          w[u][a][j] = ldw<NTL>(wp[a] + (int64_t)(ks + u) * KSTEP + j * JSTEP);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        x[u][j] = xv ? *reinterpret_cast<const s16x8*>(xp + (ks + u) * 128 + j * 32) : zero;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < NT; ++a)
          acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[u][a][j]), as_bf16x8(x[u][j]),
                                                           acc[a], 0, 0, 0);
  }
  if (ks < ks1) {                       // tail: all loads before the first MFMA
    const int rem = ks1 - ks;
    s16x8 w[U][NT][4], x[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < rem) {
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            w[u][a][j] = ldw<NTL>(wp[a] + (int64_t)(ks + u) * KSTEP + j * JSTEP);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[u][j] = xv ? *reinterpret_cast<const s16x8*>(xp + (ks + u) * 128 + j * 32) : zero;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < rem) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int a = 0; a < NT; ++a)
            acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(w[u][a][j]),
                                                             as_bf16x8(x[u][j]), acc[a], 0, 0, 0);
      }
  }
#pragma unroll
  for (int a = 0; a < NT; ++a) red[wave][a][lane] = acc[a];
  __syncthreads();
  // D layout: lane holds GEMM rows row0[a] + g*4 + i for token r.
  if (wave == 0 && xv) {
#pragma unroll
    for (int a = 0; a < NT; ++a) {
      f32x4 s = red[0][a][lane];
#pragma unroll
      for (int w2 = 1; w2 < NW; ++w2) s += red[w2][a][lane];
      gu64* slab = (gu64*)(part + ((int64_t)slice * M + r) * Nn + row0[a] + g * 4);
      __hip_atomic_store(slab, (unsigned long long)__float_as_uint(s[0]) |
                                   ((unsigned long long)__float_as_uint(s[1]) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(slab + 1, (unsigned long long)__float_as_uint(s[2]) |
                                       ((unsigned long long)__float_as_uint(s[3]) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(tile_cnt + bt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    nscratch[16] = (prev == (unsigned)KS - 1) ? 1.f : 0.f;
  }
  __syncthreads();
  if (nscratch[16] == 0.f) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every handed-off load is sc1
  if (threadIdx.x == 0)
    __hip_atomic_store(tile_cnt + bt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wave == 0 && xv) {
    float s[NT][4];
#pragma unroll
    for (int a = 0; a < NT; ++a) {
      s[a][0] = s[a][1] = s[a][2] = s[a][3] = 0.f;
      for (int sl = 0; sl < KS; ++sl) {
        const gu64* q = (const gu64*)(part + ((int64_t)sl * M + r) * Nn + row0[a] + g * 4);
        const unsigned long long u0 = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long u1 =
            __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s[a][0] += __uint_as_float((uint32_t)u0);
        s[a][1] += __uint_as_float((uint32_t)(u0 >> 32));
        s[a][2] += __uint_as_float((uint32_t)u1);
        s[a][3] += __uint_as_float((uint32_t)(u1 >> 32));
      }
    }
    if constexpr (EPI == kGvSwi) {
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gf = bf2f(f2bf(s[0][i]));              // = the gate_up GEMM's bf16 output
        const float sg = gf / (1.f + __expf(-gf));
        o[i] = bf2f(f2bf(sg)) * bf2f(f2bf(s[NT - 1][i]));
      }
      uint2 v;
      v.x = pack_bf16x2(o[0], o[1]);
      v.y = pack_bf16x2(o[2], o[3]);
      *reinterpret_cast<uint2*>(Y + (int64_t)r * ldy + bt * 16 + g * 4) = v;
    } else if constexpr (EPI == kGvRope) {
      const int h = bt >> 2;                               // head in [q | k | v]
      const int d0 = (bt & 3) * 16 + g * 4;                // rotary index of s[0][0]
      float o1[4], o2[4];
      if (h < re.Hq + re.Hkv) {
        const float* cs = re.cos_sin + (int64_t)re.positions[r] * 128;
        const float4 c = *reinterpret_cast<const float4*>(cs + d0);
        const float4 sn = *reinterpret_cast<const float4*>(cs + 64 + d0);
        const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o1[i] = s[0][i] * cc[i] - s[NT - 1][i] * ss[i];
          o2[i] = s[NT - 1][i] * cc[i] + s[0][i] * ss[i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o1[i] = s[0][i];
          o2[i] = s[NT - 1][i];
        }
      }
      uint2 v1, v2;
      v1.x = pack_bf16x2(o1[0], o1[1]);
      v1.y = pack_bf16x2(o1[2], o1[3]);
      v2.x = pack_bf16x2(o2[0], o2[1]);
      v2.y = pack_bf16x2(o2[2], o2[3]);
      bf16_t* dst = nullptr;
      if (h < re.Hq) {
        dst = Y + (int64_t)r * ldy + h * 128;
      } else {
        const int slot = re.slots[r];
        if (slot >= 0) {                                   // -1 = padding row: no KV write
          const bool is_k = h < re.Hq + re.Hkv;
          const int kvh = is_k ? h - re.Hq : h - re.Hq - re.Hkv;
          dst = (is_k ? re.k_cache : re.v_cache) +
                (((int64_t)(slot / re.BS) * re.Hkv + kvh) * re.BS + slot % re.BS) * 128;
        }
      }
      if (dst != nullptr) {
        *reinterpret_cast<uint2*>(dst + d0) = v1;
        *reinterpret_cast<uint2*>(dst + 64 + d0) = v2;
      }
    } else {
      uint2 v;
      v.x = pack_bf16x2(s[0][0], s[0][1]);
      v.y = pack_bf16x2(s[0][2], s[0][3]);
      bf16_t* yp = Y + (int64_t)r * ldy + row0[0] + g * 4;
      if constexpr (EPI == kGvNorm)
        __hip_atomic_store((gu64*)yp, (unsigned long long)v.x | ((unsigned long long)v.y << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        *reinterpret_cast<uint2*>(yp) = v;
    }
  }
  if constexpr (EPI == kGvNorm) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev =
          __hip_atomic_fetch_add(ep.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nscratch[16] = (prev == (unsigned)ntile - 1) ? 1.f : 0.f;
    }
    __syncthreads();
    if (nscratch[16] == 0.f) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (threadIdx.x == 0)
      __hip_atomic_store(ep.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_block_add_norm<NW * 64, 1>(Y, ldy, ntile * 16, M, ep, nscratch);
  }
}

}  // namespace rfq
