// Skinny-M GEMM for the latency path: Y[M, N] = X[M, K] . W[N, K]^T, M <= 64.
//
// At small batch (a single /parse-text/ request decodes 1 sampled token plus a
// few jump-forward tokens per step) every projection is a weight stream: the
// step is bound by reading the 16 GB of Llama-3-8B weights from HBM3E, and the
// library GEMMs tile for large M and leave most of that bandwidth idle.  This
// kernel is shaped for the stream instead of the FLOPs:
//
//   * W is the MFMA A operand (16 output features x 32 k per
//     mfma_f32_16x16x32_bf16), X^T the B operand (k x 16 tokens).  Because the
//     k-reduction is order independent, lane-group g = lane>>4 owns a contiguous
//     32-element (64 B) slice of each W row per 128-k step and feeds it to four
//     MFMAs (j = 0..3): every lane issues 4 x 16 B loads per row per step — full
//     64 B segments, no LDS staging, no shuffles.
//   * A workgroup owns NT*16 output features; its NW waves split K, and the
//     partial 16x16 tiles are reduced through LDS and written as bf16 once
//     (no second pass, no atomics).  U k-steps are in flight per wave so every
//     CU keeps enough bytes outstanding to cover HBM latency.
//   * X (a few KB to ~1 MB) is read straight from L2; NT > 1 reuses each X
//     fragment for several W tiles to keep the L2 traffic well below the W stream.
//
// Requires K % 128 == 0, N % (16*NT) == 0, 16-byte aligned rows.
#include "gemv_core.h"

namespace rfq {


// CMAP: k-permutation.  false: lane-group g owns 32 contiguous k (4 x 16 B, one per
// MFMA j); true: MFMA j reads k [j*32, j*32+32) and group g the 8-element slice g
// of it, so the 4 groups of one row read 64 contiguous bytes per load instruction.
// GX: X is a [M, 2K] gate|up activation and the B operand is silu(gate) * up,
// computed while loading (rounded like silu_mul: bf16(silu(g)) * u -> bf16), so the
// down projection consumes the SwiGLU input without the separate act.hip pass.
template <bool GX>
__device__ __forceinline__ s16x8 ldx8(const bf16_t* p, int K) {
  if constexpr (!GX) {
    return *reinterpret_cast<const s16x8*>(p);
  } else {
    const s16x8 g = *reinterpret_cast<const s16x8*>(p);
    const s16x8 u = *reinterpret_cast<const s16x8*>(p + K);
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float gf = bf2f_s(g[i]);
      const float sg = bf2f(f2bf(gf / (1.f + __expf(-gf))));
      o[i] = sg * bf2f_s(u[i]);
    }
    return pack8(o);
  }
}



// KS > 1 (NORM only): the KS workgroups of an output tile each stream one K slice and
// publish fp32 partials; the last workgroup sums them before the add + RMSNorm.  For
// N = 4096 projections (o, down: 256 tiles) this doubles the workgroups in flight.
// SWI (MT = 1, NT = 2): tile 0 = gate rows [n0, n0+16), tile 1 = up rows
// [up_off + n0, ...) of the stacked gate|up weight; the epilogue writes
// silu(gate) * up rounded exactly like act.hip's silu_mul (gate and up rounded to bf16
// first), so the gate|up GEMM, the SwiGLU pass and its [M, 2F] intermediate become one
// kernel whose output is the down projection's [M, F] input.
template <int MT, int NT, int NW, int U, bool CMAP, bool NTL, bool GX = false, bool NORM = false,
          bool ROPE = false, int KS = 1, bool SWI = false>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(
    const bf16_t* __restrict__ X, int64_t ldx, const bf16_t* __restrict__ W, int K, int64_t wstr,
    bf16_t* __restrict__ Y, int64_t ldy, int M, NormEpi ep, RopeEpi re = RopeEpi{},
    int up_off = 0) {
  static_assert(!ROPE || (MT == 1 && NT == 2 && !NORM && !GX), "RoPE epilogue: MT=1, NT=2");
  static_assert(!SWI || (MT == 1 && NT == 2 && !NORM && !GX && !ROPE), "SwiGLU: MT=1, NT=2");
  static_assert(KS == 1 || (NORM && MT == 1), "split-K only with the norm epilogue");
  __shared__ f32x4 red[NW][NT * MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  // ROPE: block b owns head b/4, rotary pair block b%4 (features n0 and n0 + 64)
  const int bt = KS > 1 ? blockIdx.x / KS : blockIdx.x, slice = KS > 1 ? blockIdx.x % KS : 0;
  const int n0 = ROPE ? (bt >> 2) * 128 + (bt & 3) * 16 : (SWI ? bt * 16 : bt * (16 * NT));
  const int astride = ROPE ? 64 : (SWI ? up_off : 16);
  const int nks_all = K >> 7;
  const int sl0 = slice * nks_all / KS, nks = (slice + 1) * nks_all / KS - sl0;
  const int ks0 = sl0 + wave * nks / NW, ks1 = sl0 + (wave + 1) * nks / NW;

  const bf16_t* wp[NT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
    wp[a] = W + (int64_t)(n0 + a * astride + r) * wstr + g * (CMAP ? 8 : 32);
  constexpr int JS = CMAP ? 32 : 8;                 // element stride between MFMA chunks
  const bf16_t* xp[MT];
  bool xv[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + r;
    xv[t] = m < M;
    xp[t] = X + (int64_t)(xv[t] ? m : 0) * ldx + g * (CMAP ? 8 : 32);
  }
  f32x4 acc[NT][MT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};

  int ks = ks0;
  for (; ks + U <= ks1; ks += U) {
    s16x8 w[U][NT][4], x[U][MT][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          w[u][a][j] = ldw<NTL>(wp[a] + (int64_t)(ks + u) * 128 + j * JS);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[u][t][j] = xv[t] ? ldx8<GX>(xp[t] + (ks + u) * 128 + j * JS, K) : zero;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
          for (int t = 0; t < MT; ++t)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                as_bf16x8(w[u][a][j]), as_bf16x8(x[u][t][j]), acc[a][t], 0, 0, 0);
  }
  // tail (< U k-steps): every load is issued before the first MFMA, so a short K
  // range (e.g. the TP=8 o projection, K = 1024: 2 steps per wave) costs one HBM
  // round trip instead of one per step
  if (ks < ks1) {
    const int rem = ks1 - ks;
    s16x8 w[U][NT][4], x[U][MT][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < rem) {
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            w[u][a][j] = ldw<NTL>(wp[a] + (int64_t)(ks + u) * 128 + j * JS);
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            x[u][t][j] = xv[t] ? ldx8<GX>(xp[t] + (ks + u) * 128 + j * JS, K) : zero;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < rem) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int a = 0; a < NT; ++a)
#pragma unroll
            for (int t = 0; t < MT; ++t)
              acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  as_bf16x8(w[u][a][j]), as_bf16x8(x[u][t][j]), acc[a][t], 0, 0, 0);
      }
  }

  if (NW > 1) {
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) red[wave][a * MT + t][lane] = acc[a][t];
    __syncthreads();
  }
  if constexpr (SWI) {
    if (wave != 0) return;
    f32x4 s0 = NW == 1 ? acc[0][0] : red[0][0][lane];
    f32x4 s1 = NW == 1 ? acc[1][0] : red[0][1][lane];
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) {
      s0 += red[w2][0][lane];
      s1 += red[w2][1][lane];
    }
    if (r >= M) return;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float gf = bf2f(f2bf(s0[i]));                // = the gate_up GEMM's bf16 output
      const float sg = gf / (1.f + __expf(-gf));
      o[i] = bf2f(f2bf(sg)) * bf2f(f2bf(s1[i]));
    }
    uint2 v;
    v.x = pack_bf16x2(o[0], o[1]);
    v.y = pack_bf16x2(o[2], o[3]);
    *reinterpret_cast<uint2*>(Y + (int64_t)r * ldy + n0 + g * 4) = v;
    return;
  }
  if constexpr (ROPE) {
    if (wave != 0) return;
    f32x4 x1 = NW == 1 ? acc[0][0] : red[0][0][lane];
    f32x4 x2 = NW == 1 ? acc[1][0] : red[0][1][lane];
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) {
      x1 += red[w2][0][lane];
      x2 += red[w2][1][lane];
    }
    const int m = r;                                   // token (MT = 1)
    if (m >= M) return;
    const int h = blockIdx.x >> 2;                     // head in [q | k | v]
    const int d0 = (blockIdx.x & 3) * 16 + g * 4;      // rotary index of x1[0]
    float o1[4], o2[4];
    if (h < re.Hq + re.Hkv) {
      const float* cs = re.cos_sin + (int64_t)re.positions[m] * 128;
      const float4 c = *reinterpret_cast<const float4*>(cs + d0);
      const float4 sn = *reinterpret_cast<const float4*>(cs + 64 + d0);
      const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o1[i] = x1[i] * cc[i] - x2[i] * ss[i];
        o2[i] = x2[i] * cc[i] + x1[i] * ss[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o1[i] = x1[i];
        o2[i] = x2[i];
      }
    }
    uint2 v1, v2;
    v1.x = pack_bf16x2(o1[0], o1[1]);
    v1.y = pack_bf16x2(o1[2], o1[3]);
    v2.x = pack_bf16x2(o2[0], o2[1]);
    v2.y = pack_bf16x2(o2[2], o2[3]);
    bf16_t* dst;
    if (h < re.Hq) {
      dst = Y + (int64_t)m * ldy + h * 128;
    } else {
      const int slot = re.slots[m];
      if (slot < 0) return;                            // padding row: no KV write
      const bool is_k = h < re.Hq + re.Hkv;
      const int kvh = is_k ? h - re.Hq : h - re.Hq - re.Hkv;
      dst = (is_k ? re.k_cache : re.v_cache) +
            (((int64_t)(slot / re.BS) * re.Hkv + kvh) * re.BS + slot % re.BS) * 128;
    }
    *reinterpret_cast<uint2*>(dst + d0) = v1;
    *reinterpret_cast<uint2*>(dst + 64 + d0) = v2;
    return;
  }
  // D layout (16x16): lane holds rows (g*4 + i) = output features, col r = token.
  for (int tile = wave; tile < NT * MT; tile += NW) {
    const int a = tile / MT, t = tile % MT;
    f32x4 s = red[0][tile][lane];
    if (NW == 1) s = acc[a][t];
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) s += red[w2][tile][lane];
    const int m = t * 16 + r;
    if (KS > 1 && m < M) {   // fp32 partial of this K slice, write-through (sc1)
      const int Nn = (gridDim.x / KS) * 16 * NT;
      gu64* pq = (gu64*)(ep.partials + slice * ep.pslab + (int64_t)m * Nn + n0 + a * 16 + g * 4);
      __hip_atomic_store(pq, (unsigned long long)__float_as_uint(s[0]) |
                                 ((unsigned long long)__float_as_uint(s[1]) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pq + 1, (unsigned long long)__float_as_uint(s[2]) |
                                     ((unsigned long long)__float_as_uint(s[3]) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (m < M) {
      uint2 v;
      v.x = pack_bf16x2(s[0], s[1]);
      v.y = pack_bf16x2(s[2], s[3]);
      bf16_t* yp = Y + (int64_t)m * ldy + n0 + a * 16 + g * 4;
      if constexpr (NORM)   // write-through (sc1) so the last workgroup reads it without a release
        __hip_atomic_store((gu64*)yp,
                           (unsigned long long)v.x | ((unsigned long long)v.y << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        *reinterpret_cast<uint2*>(yp) = v;
    }
  }

  if constexpr (NORM) {
    // publish this tile and take a ticket; the last workgroup runs the add + RMSNorm
    __shared__ float nscratch[17];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev =
          __hip_atomic_fetch_add(ep.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nscratch[16] = (prev == gridDim.x - 1) ? 1.f : 0.f;
    }
    __syncthreads();
    if (nscratch[16] == 0.f) return;
    // every load of the handed-off Y is an sc1 load (last_block_add_norm), so a
    // wavefront-scope fence (compiler ordering only) replaces the agent acquire
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (threadIdx.x == 0)
      __hip_atomic_store(ep.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_block_add_norm<NW * 64, KS>(Y, ldy, (gridDim.x / KS) * 16 * NT, M, ep, nscratch);
  }
}

template <int MT, int NT, int NW, int U>
static void launch_cfg(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K, int64_t wstr,
                       bf16_t* Y, int64_t ldy, int M, int variant, bool norm, const NormEpi& ep,
                       hipStream_t s) {
  dim3 grid(N / (16 * NT));
  if constexpr (MT == 1) {  // fused add + RMSNorm epilogue (M <= 16): contiguous-k, plain loads
    if (norm) {
      const dim3 g2(grid.x * 2);
      if (variant >= 4 && ep.partials)
        hipLaunchKernelGGL((skinny_gemm_kernel<1, NT, NW, U, true, false, true, true, false, 2>),
                           g2, dim3(NW * 64), 0, s, X, ldx, W, K, wstr, Y, ldy, M, ep);
      else if (variant >= 4)
        hipLaunchKernelGGL((skinny_gemm_kernel<1, NT, NW, U, true, false, true, true>), grid,
                           dim3(NW * 64), 0, s, X, ldx, W, K, wstr, Y, ldy, M, ep);
      else if (ep.partials)
        hipLaunchKernelGGL((skinny_gemm_kernel<1, NT, NW, U, true, false, false, true, false, 2>),
                           g2, dim3(NW * 64), 0, s, X, ldx, W, K, wstr, Y, ldy, M, ep);
      else
        hipLaunchKernelGGL((skinny_gemm_kernel<1, NT, NW, U, true, false, false, true>), grid,
                           dim3(NW * 64), 0, s, X, ldx, W, K, wstr, Y, ldy, M, ep);
      return;
    }
  }
  if (variant >= 4) {   // gated X (silu(gate) * up), contiguous-k, plain loads
    hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, NW, U, true, false, true>), grid, dim3(NW * 64),
                       0, s, X, ldx, W, K, wstr, Y, ldy, M, ep);
    return;
  }
#define SK_LAUNCH(cm, nt)                                                                   \
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, NW, U, cm, nt>), grid, dim3(NW * 64), 0, s, \
                     X, ldx, W, K, wstr, Y, ldy, M, ep)
  switch (variant) {
    case 0: SK_LAUNCH(false, true); break;
    case 1: SK_LAUNCH(true, true); break;
    case 2: SK_LAUNCH(false, false); break;
    default: SK_LAUNCH(true, false); break;
  }
#undef SK_LAUNCH
}

// cfg bits: [1:0] tile (0: NT=1 NW=4, 1: NT=2 NW=4, 2: NT=1 NW=8, 3: NT=2 NW=8),
// [3:2] variant (bit2 contiguous k-map, bit3 plain loads instead of non-temporal),
// bit 4: gated X (x is [M, 2K] gate|up; B operand = silu(gate) * up).
static void skinny_dispatch(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                            int64_t wstr, bf16_t* Y, int64_t ldy, int M, int cfg, bool norm,
                            const NormEpi& ep, hipStream_t s) {
  const int MT = (M + 15) / 16;
  const int v = (cfg & 16) ? 4 : ((cfg >> 2) & 3);
#define SK_CASE(mt, u1, u2)                                                                    \
  case mt:                                                                                     \
    switch (cfg & 3) {                                                                         \
      case 0: launch_cfg<mt, 1, 4, u1>(X, ldx, W, N, K, wstr, Y, ldy, M, v, norm, ep, s); break;     \
      case 1: launch_cfg<mt, 2, 4, u2>(X, ldx, W, N, K, wstr, Y, ldy, M, v, norm, ep, s); break;     \
      case 2: launch_cfg<mt, 1, 8, u1>(X, ldx, W, N, K, wstr, Y, ldy, M, v, norm, ep, s); break;     \
      default: launch_cfg<mt, 2, 8, u2>(X, ldx, W, N, K, wstr, Y, ldy, M, v, norm, ep, s); break;    \
    }                                                                                          \
    break;
  switch (MT) {
    SK_CASE(1, 4, 2)
    SK_CASE(2, 3, 2)
    SK_CASE(3, 2, 1)
    default: SK_CASE(4, 2, 1)
  }
#undef SK_CASE
}

void launch_skinny_gemm(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K, int64_t wstr,
                        bf16_t* Y, int64_t ldy, int M, int cfg, hipStream_t s) {
  skinny_dispatch(X, ldx, W, N, K, wstr, Y, ldy, M, cfg, false, NormEpi{}, s);
}

// Fused QKV projection + RoPE + KV append (M <= 16, N = (Hq + 2 Hkv) * 128; cfg bit 0
// must select NT = 2; bit 1 picks 4 or 8 waves).  Only the q columns of Y are written.
void launch_skinny_gemm_rope(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                             bf16_t* Y, int64_t ldy, int M, int cfg, const int32_t* positions,
                             const float* cos_sin, const int32_t* slots, bf16_t* k_cache,
                             bf16_t* v_cache, int Hq, int Hkv, int BS, hipStream_t s) {
  const RopeEpi re{positions, cos_sin, slots, k_cache, v_cache, Hq, Hkv, BS};
  const int64_t wstr = K;
  const dim3 grid(N / 32);
  if (cfg & 2)
    hipLaunchKernelGGL((skinny_gemm_kernel<1, 2, 8, 2, true, false, false, false, true>), grid,
                       dim3(512), 0, s, X, ldx, W, K, wstr, Y, ldy, M, NormEpi{}, re);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<1, 2, 4, 2, true, false, false, false, true>), grid,
                       dim3(256), 0, s, X, ldx, W, K, wstr, Y, ldy, M, NormEpi{}, re);
}

// Y = X W^T, then residual <- Y + residual, out <- rmsnorm(residual) * norm_w (M <= 16,
// N <= 8192; counter: one zero-initialised uint32 per stream, left at zero).
// cfg bit 6 (64): split K in two slices per tile (partials: fp32 [2][M][N] workspace).
void launch_skinny_gemm_norm(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                             bf16_t* Y, int64_t ldy, int M, int cfg, bf16_t* residual,
                             int64_t res_stride, const bf16_t* norm_w, bf16_t* out,
                             int64_t out_stride, float eps, unsigned* counter, float* partials,
                             hipStream_t s) {
  const NormEpi ep{residual,          res_stride, norm_w, out, out_stride, eps, counter,
                   (cfg & 64) ? partials : nullptr, (int64_t)M * N};
  cfg &= 63;
  skinny_dispatch(X, ldx, W, N, K, (int64_t)K, Y, ldy, M, cfg, true, ep, s);
}

// out[M, F] = silu(x Wg^T) * (x Wu^T) for w = [Wg; Wu] ([2F, K]); M <= 16.
// cfg bit 1 picks 4 or 8 waves.
void launch_skinny_gemm_swiglu(const bf16_t* X, int64_t ldx, const bf16_t* W, int F, int K,
                               bf16_t* Y, int64_t ldy, int M, int cfg, hipStream_t s) {
  const dim3 grid(F / 16);
  if (cfg & 2)
    hipLaunchKernelGGL((skinny_gemm_kernel<1, 2, 8, 2, true, false, false, false, false, 1, true>),
                       grid, dim3(512), 0, s, X, ldx, W, K, (int64_t)K, Y, ldy, M, NormEpi{},
                       RopeEpi{}, F);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<1, 2, 4, 2, true, false, false, false, false, 1, true>),
                       grid, dim3(256), 0, s, X, ldx, W, K, (int64_t)K, Y, ldy, M, NormEpi{},
                       RopeEpi{}, F);
}


// PERSIST (cfg bit 6, tiled layout only): a grid of about four 4-wave (two 8-wave)
// workgroups per CU walks the work units in strides of the grid, so a CU's waves stay
// resident and one unit's reduction / hand-off overlaps the other workgroups' streams
// instead of a workgroup being torn down and launched per unit.
template <int NW, int U, int EPI, bool TL = false, bool NTL = false, bool PERSIST = false>
__global__ __launch_bounds__(NW * 64) void gemv_splitk_kernel(
    const bf16_t* __restrict__ X, int64_t ldx, const bf16_t* __restrict__ W, int K,
    bf16_t* __restrict__ Y, int64_t ldy, int M, int KS, float* __restrict__ part, int Nn,
    unsigned* __restrict__ tile_cnt, NormEpi ep, RopeEpi re, int up_off, int units) {
  if constexpr (!PERSIST) {
    gemv_splitk_unit<NW, U, EPI, TL, NTL>(blockIdx.x, units / KS, X, ldx, W, K, Y, ldy, M, KS,
                                          part, Nn, tile_cnt, ep, re, up_off);
  } else {
    for (int unit = blockIdx.x; unit < units; unit += gridDim.x) {
      gemv_splitk_unit<NW, U, EPI, TL, NTL>(unit, units / KS, X, ldx, W, K, Y, ldy, M, KS,
                                            part, Nn, tile_cnt, ep, re, up_off);
      __syncthreads();                 // red / nscratch are reused by the next unit
    }
  }
}

// cfg bits: [1:0] KS = 2 << bits (2, 4, 8, 16); bit 2: 8 waves (else 4); bit 3: U = 2 (else 4;
// U = 8 needs 256+ VGPRs: the X fragments take as many registers as the W ones);
// bit 4: W in the decode-tiled layout (TL above); bit 5: non-temporal weight loads (NTL);
// bit 6: persistent grid (PERSIST, with bit 4 only).
// part: fp32 [KS][M][Nn] (Nn = GEMM rows); tile_cnt: one zeroed uint32 per output tile
// (left at zero).  ntile: N/16 (plain, norm), F/16 (swiglu), N/32 (rope).
template <int EPI>
static void launch_gemv_splitk_epi(const bf16_t* X, int64_t ldx, const bf16_t* W, int ntile, int Nn,
                                   int K, bf16_t* Y, int64_t ldy, int M, int cfg, float* part,
                                   unsigned* tile_cnt, const NormEpi& ep, const RopeEpi& re,
                                   int up_off, hipStream_t s) {
  const int KS = 2 << (cfg & 3);
  const int units = ntile * KS;
  const bool persist = (cfg & 64) && (cfg & 16);          // tiled layout only
  const int per_cu = (cfg & 4) ? 2 : 4;                   // 8-wave : 4-wave workgroups
  const dim3 grid(persist ? min(units, 256 * per_cu) : units);
#define GV_LAUNCH1(nw, u, tl, nt, pe)                                                           \
  hipLaunchKernelGGL((gemv_splitk_kernel<nw, u, EPI, tl, nt, pe>), grid, dim3(nw * 64), 0, s, X, \
                     ldx, W, K, Y, ldy, M, KS, part, Nn, tile_cnt, ep, re, up_off, units)
#define GV_LAUNCH(nw, u)                                                                        \
  switch (((cfg >> 4) & 3) | (persist ? 4 : 0)) {                                               \
    case 0: GV_LAUNCH1(nw, u, false, false, false); break;                                      \
    case 1: GV_LAUNCH1(nw, u, true, false, false); break;                                       \
    case 2: GV_LAUNCH1(nw, u, false, true, false); break;                                       \
    case 3: GV_LAUNCH1(nw, u, true, true, false); break;                                        \
    case 5: GV_LAUNCH1(nw, u, true, false, true); break;                                        \
    default: GV_LAUNCH1(nw, u, true, true, true); break;                                        \
  }
  switch ((cfg >> 2) & 3) {
    case 0: GV_LAUNCH(4, 4); break;
    case 1: GV_LAUNCH(8, 4); break;
    case 2: GV_LAUNCH(4, 2); break;
    default: GV_LAUNCH(8, 2); break;
  }
#undef GV_LAUNCH
#undef GV_LAUNCH1
}

void launch_gemv_splitk_norm(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                             bf16_t* Y, int64_t ldy, int M, int cfg, float* part,
                             unsigned* tile_cnt, bf16_t* residual, int64_t res_stride,
                             const bf16_t* norm_w, bf16_t* out, int64_t out_stride, float eps,
                             unsigned* counter, hipStream_t s) {
  const NormEpi ep{residual, res_stride, norm_w, out, out_stride, eps, counter, nullptr, 0};
  launch_gemv_splitk_epi<kGvNorm>(X, ldx, W, N / 16, N, K, Y, ldy, M, cfg, part, tile_cnt, ep,
                                  RopeEpi{}, 0, s);
}

void launch_gemv_splitk_plain(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                              bf16_t* Y, int64_t ldy, int M, int cfg, float* part,
                              unsigned* tile_cnt, hipStream_t s) {
  launch_gemv_splitk_epi<kGvPlain>(X, ldx, W, N / 16, N, K, Y, ldy, M, cfg, part, tile_cnt,
                                   NormEpi{}, RopeEpi{}, 0, s);
}

// Y[M, F] = silu(x Wg^T) * (x Wu^T), w = [Wg; Wu] [2F, K]
void launch_gemv_splitk_swiglu(const bf16_t* X, int64_t ldx, const bf16_t* W, int F, int K,
                               bf16_t* Y, int64_t ldy, int M, int cfg, float* part,
                               unsigned* tile_cnt, hipStream_t s) {
  launch_gemv_splitk_epi<kGvSwi>(X, ldx, W, F / 16, 2 * F, K, Y, ldy, M, cfg, part, tile_cnt,
                                 NormEpi{}, RopeEpi{}, F, s);
}

// qkv = x w^T with RoPE + KV append (N = (Hq + 2 Hkv) * 128); only q columns of Y written
void launch_gemv_splitk_rope(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                             bf16_t* Y, int64_t ldy, int M, int cfg, float* part,
                             unsigned* tile_cnt, const int32_t* positions, const float* cos_sin,
                             const int32_t* slots, bf16_t* k_cache, bf16_t* v_cache, int Hq,
                             int Hkv, int BS, hipStream_t s) {
  const RopeEpi re{positions, cos_sin, slots, k_cache, v_cache, Hq, Hkv, BS};
  launch_gemv_splitk_epi<kGvRope>(X, ldx, W, N / 32, N, K, Y, ldy, M, cfg, part, tile_cnt,
                                  NormEpi{}, re, 0, s);
}

// ---------------------------------------------------------------------------
// MoE latency path: the same weight-streaming structure applied per expert.
//
// Rows are the (token, slot) pairs grouped by expert by moe_align (segments
// [expert_offsets[e], expert_offsets[e+1]) padded to 16).  One workgroup owns a
// 16-column output tile of one expert; experts with no rows return before
// touching their weights, so a decode step streams only the routed experts
// (2 of 8 for one token) instead of 128-row-padded tiles of every block.
//   GATHER: X rows are looked up through sorted_ids (pair -> token), so the
//           routed activations are never materialised.
//   GATED:  the tile computes the gate rows [n0, n0+16) and the matching up rows
//           [up_off + n0, ...) of w13 together and writes silu(gate) * up — the
//           w13 GEMM, SwiGLU and its [rows, 2F] intermediate in one pass.
//   SPLIT > 1 (w2 only): the SPLIT workgroups of a tile each stream one K slice and
//           write fp32 partials to Yf[slice][row][n] (slab stride `slab` floats);
//           moe_combine_splitk sums the slices while it combines the top-k pairs.
//           w2 has only 256 output tiles per expert against K = 14336, so without
//           it one decode token's 2 experts keep too few bytes in flight per CU.
template <int MT, bool GATED, bool GATHER, int NW, int U, int SPLIT = 1>
__global__ __launch_bounds__(NW * 64) void moe_skinny_kernel(
    const bf16_t* __restrict__ X, int64_t ldx, const int32_t* __restrict__ sorted_ids, int topk,
    const int32_t* __restrict__ expert_offsets, const bf16_t* __restrict__ W,
    int64_t w_expert_stride, int K, int up_off, bf16_t* __restrict__ Y, int64_t ldy,
    int tiles_per_expert, float* __restrict__ Yf = nullptr, int64_t slab = 0) {
  constexpr int NT = GATED ? 2 : 1;
  static_assert(SPLIT == 1 || !GATED, "split-K is for the plain (w2) projection");
  __shared__ f32x4 red[NW][NT * MT][64];
  const int per_e = tiles_per_expert * SPLIT;
  const int e = blockIdx.x / per_e, rem = blockIdx.x % per_e;
  const int tile = rem / SPLIT, slice = rem % SPLIT;
  const int r0 = expert_offsets[e], r1 = expert_offsets[e + 1];
  if (r0 >= r1) return;                              // expert not routed this step
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = tile * 16;
  const int nks_all = K >> 7;
  const int sl0 = slice * nks_all / SPLIT, nks = (slice + 1) * nks_all / SPLIT - sl0;
  const int ks0 = sl0 + wave * nks / NW, ks1 = sl0 + (wave + 1) * nks / NW;
  const bf16_t* we = W + (int64_t)e * w_expert_stride;
  const bf16_t* wp[NT];
  wp[0] = we + (int64_t)(n0 + r) * K + g * 8;
  if (GATED) wp[NT - 1] = we + (int64_t)(up_off + n0 + r) * K + g * 8;
  const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};

  for (int mb = r0; mb < r1; mb += 16 * MT) {
    const bf16_t* xp[MT];
    bool xv[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int row = mb + t * 16 + r;
      bool v = row < r1;
      int src = row;
      if (GATHER) {
        const int sid = v ? sorted_ids[row] : -1;
        v = sid >= 0;
        src = v ? sid / topk : 0;
      }
      xv[t] = v;
      xp[t] = X + (int64_t)(v ? src : 0) * ldx + g * 8;
    }
    f32x4 acc[NT][MT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    int ks = ks0;
    for (; ks + U <= ks1; ks += U) {
      s16x8 w[U][NT][4], x[U][MT][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
          for (int j = 0; j < 4; ++j) w[u][a][j] = ldw<false>(wp[a] + (int64_t)(ks + u) * 128 + j * 32);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            x[u][t][j] = xv[t] ? *reinterpret_cast<const s16x8*>(xp[t] + (ks + u) * 128 + j * 32)
                               : zero;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int a = 0; a < NT; ++a)
#pragma unroll
            for (int t = 0; t < MT; ++t)
              acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  as_bf16x8(w[u][a][j]), as_bf16x8(x[u][t][j]), acc[a][t], 0, 0, 0);
    }
    for (; ks < ks1; ++ks) {
      s16x8 w[NT][4], x[MT][4];
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j) w[a][j] = ldw<false>(wp[a] + (int64_t)ks * 128 + j * 32);
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[t][j] = xv[t] ? *reinterpret_cast<const s16x8*>(xp[t] + ks * 128 + j * 32) : zero;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
          for (int t = 0; t < MT; ++t)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                as_bf16x8(w[a][j]), as_bf16x8(x[t][j]), acc[a][t], 0, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int t = 0; t < MT; ++t) red[wave][a * MT + t][lane] = acc[a][t];
    __syncthreads();
    for (int t = wave; t < MT; t += NW) {
      f32x4 s = red[0][t][lane];
#pragma unroll
      for (int w2 = 1; w2 < NW; ++w2) s += red[w2][t][lane];
      if (GATED) {
        f32x4 u = red[0][MT + t][lane];
#pragma unroll
        for (int w2 = 1; w2 < NW; ++w2) u += red[w2][MT + t][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] = s[i] / (1.f + __expf(-s[i])) * u[i];
      }
      const int row = mb + t * 16 + r;
      if (row < r1) {
        if constexpr (SPLIT > 1) {
          *reinterpret_cast<f32x4*>(Yf + slice * slab + (int64_t)row * ldy + n0 + g * 4) = s;
        } else {
          uint2 v;
          v.x = pack_bf16x2(s[0], s[1]);
          v.y = pack_bf16x2(s[2], s[3]);
          *reinterpret_cast<uint2*>(Y + (int64_t)row * ldy + n0 + g * 4) = v;
        }
      }
    }
    __syncthreads();                                   // red is reused by the next chunk
  }
}

template <int MT, bool GATED, bool GATHER>
static void moe_skinny_cfg(const bf16_t* X, int64_t ldx, const int32_t* sorted_ids, int topk,
                           const int32_t* expert_offsets, const bf16_t* W, int64_t wstride,
                           int K, int up_off, bf16_t* Y, int64_t ldy, int E, int n_out,
                           int max_rows, hipStream_t s) {
  constexpr int U = MT == 1 ? 4 : (MT == 2 ? 3 : 2);
  const int tiles = n_out / 16;
  // Long-K, few-tile projections (w2: 4096 outputs x K = 14336) launch only 256
  // workgroups per routed expert.  With at most 2 (token, expert) pairs (one decode
  // token: 2 experts) 8 waves split K so each CU keeps twice the bytes in flight
  // (tools/bench_moe_skinny.py, w2 at 2 experts: 83.2 -> 67.1 us); with more experts
  // there are enough workgroups and 4 waves are faster (5 experts: 144 vs 157 us).
  static const int nw_env = [] {
    const char* v = getenv("RFQ_MOE_SKINNY_NW");
    return v ? atoi(v) : 0;
  }();
  const bool wide = nw_env ? nw_env == 8 : (!GATED && K >= 8192 && max_rows <= 2);
  if (wide)
    hipLaunchKernelGGL((moe_skinny_kernel<MT, GATED, GATHER, 8, U>), dim3(E * tiles), dim3(512),
                       0, s, X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K, up_off, Y,
                       ldy, tiles);
  else
    hipLaunchKernelGGL((moe_skinny_kernel<MT, GATED, GATHER, 4, U>), dim3(E * tiles), dim3(256),
                       0, s, X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K, up_off, Y,
                       ldy, tiles);
}

// Split-K w2 (plain X, no gather): Yf [SPLIT][rows][n_out] fp32 partial slabs.
void launch_moe_skinny_splitk(const bf16_t* X, int64_t ldx, const int32_t* sorted_ids, int topk,
                              const int32_t* expert_offsets, const bf16_t* W, int K, float* Yf,
                              int64_t slab, int E, int n_out, int max_rows, int splits,
                              hipStream_t s) {
  const int tiles = n_out / 16;
  const int64_t wstride = (int64_t)n_out * K;
#define SPK_CASE(mt, u)                                                                        \
  if (splits == 4)                                                                             \
    hipLaunchKernelGGL((moe_skinny_kernel<mt, false, false, 4, u, 4>), dim3(E * tiles * 4),     \
                       dim3(256), 0, s, X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K,\
                       0, nullptr, (int64_t)n_out, tiles, Yf, slab);                           \
  else                                                                                         \
    hipLaunchKernelGGL((moe_skinny_kernel<mt, false, false, 4, u, 2>), dim3(E * tiles * 2),     \
                       dim3(256), 0, s, X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K,\
                       0, nullptr, (int64_t)n_out, tiles, Yf, slab);
  const int MT = max_rows <= 16 ? 1 : (max_rows <= 32 ? 2 : (max_rows <= 48 ? 3 : 4));
  if (MT == 1) { SPK_CASE(1, 4) }
  else if (MT == 2) { SPK_CASE(2, 3) }
  else if (MT == 3) { SPK_CASE(3, 2) }
  else { SPK_CASE(4, 2) }
#undef SPK_CASE
}

// gated: W [E, 2*n_out, K] (gate | up), Y [rows, n_out] = silu(X W_g^T) * (X W_u^T)
// else:  W [E, n_out, K], Y [rows, n_out]
void launch_moe_skinny(const bf16_t* X, int64_t ldx, const int32_t* sorted_ids, int topk,
                       const int32_t* expert_offsets, const bf16_t* W, int K, bf16_t* Y,
                       int64_t ldy, int E, int n_out, int max_rows, bool gated, bool gather,
                       hipStream_t s) {
  const int MT = max_rows <= 16 ? 1 : (max_rows <= 32 ? 2 : (max_rows <= 48 ? 3 : 4));
  const int64_t wstride = (int64_t)(gated ? 2 * n_out : n_out) * K;
#define MS_CASE(mt)                                                                            \
  case mt:                                                                                     \
    if (gated && gather)                                                                       \
      moe_skinny_cfg<mt, true, true>(X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K,  \
                                     n_out, Y, ldy, E, n_out, max_rows, s);                              \
    else if (gated)                                                                            \
      moe_skinny_cfg<mt, true, false>(X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K, \
                                      n_out, Y, ldy, E, n_out, max_rows, s);                             \
    else if (gather)                                                                           \
      moe_skinny_cfg<mt, false, true>(X, ldx, sorted_ids, topk, expert_offsets, W, wstride, K, \
                                      0, Y, ldy, E, n_out, max_rows, s);                                 \
    else                                                                                       \
      moe_skinny_cfg<mt, false, false>(X, ldx, sorted_ids, topk, expert_offsets, W, wstride,   \
                                       K, 0, Y, ldy, E, n_out, max_rows, s);                             \
    break;
  switch (MT) {
    MS_CASE(1)
    MS_CASE(2)
    MS_CASE(3)
    default: MS_CASE(4)
  }
#undef MS_CASE
}

}  // namespace rfq
