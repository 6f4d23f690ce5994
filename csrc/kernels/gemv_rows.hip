// Row-streaming GEMV for the batch-1 latency path: Y[M, N] = X[M, K] . W[N, K]^T,
// M <= 4 tokens, K % 512 == 0.
//
// Why a third GEMV form.  The split-K GEMV (gemv_core.h) and the skinny GEMM
// (gemm_skinny.hip) both tile W by 16-row MFMA blocks.  On the 70B TP = 8 rank shard
// the QKV weight has only 80 such blocks (1,280 rows), so the split-K kernel has to cut
// K across workgroups and pay a cross-workgroup hand-off per tile (write-through fp32
// partials, drained stores, a ticket, sc1 read-back by the last arriver): a chain of
// 3-4 dependent memory round trips after the weight stream that set the launch's time
// (9.8 us for 21 MB, profiles/r4/tp8_rank_kernel_window.md).
//
// Here the unit of work is a WAVE owning whole rows over the full K:
//   * lane l of the wave reads bytes [16 l, 16 l + 16) of every 1 KB chunk of its row:
//     one 1 KB fully-coalesced load per wave-instruction, straight from the row-major
//     weight (no tiled copy needed), non-temporal (each weight byte is read once per
//     step by one CU: MI355X_MICROARCH.md 'nt-weights');
//   * the dot product runs on v_dot2c_f32_bf16 (two bf16 products per instruction, fp32
//     accumulation): at M <= 4 the VALU work is a few percent of the stream's cycles,
//     and the 15/16 of an MFMA wasted on padding tokens is not needed;
//   * the wave sums its 64 lanes with four DPP steps and two swizzles -- no LDS round
//     trip, no cross-workgroup traffic, no tickets, no workspace.
// Grids are rows / RW waves: 1,280-8,192 waves on the TP = 8 shard, 4,096-28,672 on 8B,
// i.e. 5-112 waves per CU, every CU streams.
//
// Epilogues:
//   kRwPlain  Y[m, row] bf16.
//   kRwSwi    waves 2j / 2j+1 of a workgroup own gate row q and up row F + q of the
//             stacked gate|up weight; the pair meets in LDS and Y[m, q] = SwiGLU rounded
//             like act.hip silu_mul (gate and up rounded to bf16 first).
//   kRwRope   waves 2j / 2j+1 own the rotate-half partners h*128 + d and h*128 + 64 + d
//             of one head: NeoX RoPE on the fp32 sums (as gemv_core.h kGvRope), q to Y,
//             k / v appended to the paged cache (slot -1 = padding: no write).
//
// Folded-norm forms (FL, the TP = 1 latency path, models/llama.py _forward_fold):
//   kRwNormX  (SwiGLU / RoPE) X is the UN-normalised residual stream and W carries the
//             RMSNorm weight folded into its columns (W' = W diag(g), DecoderLM
//             fold_norms): rmsnorm(x) g . W^T = rsqrt(mean(x^2) + eps) (x . W'^T).  Every
//             wave reads the whole X row anyway, so it also accumulates sum(x^2) with the
//             same dot2 (x . x) and scales its sums once: no norm launch, no cross-
//             workgroup reduction.
//   kRwResAdd (plain) Y is the residual stream: Y <- bf16(bf16(x . W^T) + Y), the
//             residual add of the o / down projections (what fused_add_rms_norm did
//             before the norm itself moved into the next projection).
#include "common.h"
#include "gemv_core.h"
#include "rows_core.h"

namespace rfq {

enum { kRwPlain = 0, kRwSwi = 1, kRwRope = 2 };
enum { kRwNormX = 1, kRwResAdd = 2 };
constexpr int kRwWaves = 4;          // waves per workgroup
constexpr int kRwMaxM = 4;

// 16-byte buffer load (SRSRC form, cdna_hip_programming.md T8): the per-chunk offsets
// are wave-uniform and go in soffset, so no per-lane 64-bit address arithmetic
template <int AUX>
__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX));
}

// MM: token capacity (runtime M <= MM); RW: rows per wave (plain only; paired epilogues
// use one row per wave); CU: 1 KB chunks per row in flight per loop iteration.
// PW (paired epilogues): ONE wave owns both rows of a pair (gate q and up q, or the two
// rotate-half partners), RW = 2 with the second row rstride rows after the first: X is
// loaded once for both rows (at M = 3-4 the X re-reads, not the weights, bound the
// one-row-per-wave form) and the pair meets in registers, no LDS.
template <int MM, int RW, int CU, int EPI, bool NTL, int FL = 0, bool PW = false>
__global__ __launch_bounds__(kRwWaves * 64) void gemv_rows_kernel(
    const bf16_t* __restrict__ X, int64_t ldx, const bf16_t* __restrict__ W, int N, int K,
    bf16_t* __restrict__ Y, int64_t ldy, int M, int up_off, RopeEpi re, float eps) {
  static_assert(EPI == kRwPlain || RW == (PW ? 2 : 1), "paired epilogues: one row per wave, "
                "or both rows of the pair (PW)");
  static_assert(!PW || EPI != kRwPlain, "PW: paired epilogues only");
  static_assert(!(FL & kRwNormX) || EPI != kRwPlain, "normalised X: SwiGLU / RoPE forms");
  static_assert(!(FL & kRwResAdd) || EPI == kRwPlain, "residual add: plain form");
  constexpr bool NX = FL & kRwNormX;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gw = blockIdx.x * kRwWaves + wave;
  // rows of this wave
  int row0, rstride = 1;
  bool valid;
  if constexpr (EPI == kRwPlain) {
    row0 = gw * RW;
    valid = row0 < N;
  } else if constexpr (PW) {
    const int q = gw;                              // one pair per wave
    row0 = EPI == kRwSwi ? q : (q >> 6) * 128 + (q & 63);
    rstride = EPI == kRwSwi ? up_off : 64;
    valid = q < N;
  } else if constexpr (EPI == kRwSwi) {
    const int q = gw >> 1;                        // N = F here
    row0 = (wave & 1) ? up_off + q : q;
    valid = q < N;
  } else {
    const int q = gw >> 1;                        // pair index; N = rows / 2 pairs
    row0 = (q >> 6) * 128 + (q & 63) + ((wave & 1) ? 64 : 0);
    valid = q < N;
  }
  float acc[RW][MM], ssq[MM];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int m = 0; m < MM; ++m) acc[r][m] = 0.f;
#pragma unroll
  for (int m = 0; m < MM; ++m) ssq[m] = 0.f;
  if (valid) {
    const int nch = K >> 9;
    // W: the wave's RW rows (wave-uniform base, RW * K * 2 bytes; the plain form's last
    // wave may own fewer than RW rows when RW does not divide N: its records stop at row
    // N, so loads of rows past the weight return zeros instead of reading past it); X: the
    // M token rows, records end at row M so the loads of rows m >= M return zeros
    const int rows_here = EPI == kRwPlain ? min(RW, N - row0) : RW;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(W + (int64_t)__builtin_amdgcn_readfirstlane(row0) * K), (short)0,
        ((rows_here - 1) * rstride + 1) * K * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)(M * ldx * 2), 0x00020000);
    const int voff = lane * 16;
    constexpr int WAUX = NTL ? 2 : 0;
    // CU chunks per iteration, all of an iteration's loads in flight at once; the last
    // iteration's chunks past the row are loaded at an out-of-range offset (zeros, no
    // bytes moved), so a K that is not a multiple of CU chunks costs one more round trip
    // instead of one per remaining chunk (the serial tail loop it replaces made 8B down,
    // 28 chunks, pay up to 12 dependent round trips).  Adding the zero products leaves
    // every sum bit-identical.
    constexpr int kOob = 0x7ffffff0;
    for (int c = 0; c < nch; c += CU) {
      u32x4 w[RW][CU], x[MM][CU];
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int u = 0; u < CU; ++u)
          w[r][u] = bload<WAUX>(wr, voff,
                                c + u < nch ? (r * rstride * K + (c + u) * 512) * 2 : kOob);
#pragma unroll
      for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int u = 0; u < CU; ++u)
          x[m][u] = bload<0>(xr, voff, c + u < nch ? (int)(m * ldx + (c + u) * 512) * 2 : kOob);
#pragma unroll
      for (int u = 0; u < CU; ++u)
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int m = 0; m < MM; ++m) acc[r][m] = dot8(w[r][u], x[m][u], acc[r][m]);
      if constexpr (NX) {
#pragma unroll
        for (int u = 0; u < CU; ++u)
#pragma unroll
          for (int m = 0; m < MM; ++m) ssq[m] = dot8(x[m][u], x[m][u], ssq[m]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int m = 0; m < MM; ++m) acc[r][m] = wave_sum_dpp(acc[r][m]);
  if constexpr (NX) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      const float rs = rsqrtf(wave_sum_dpp(ssq[m]) / (float)K + eps);
#pragma unroll
      for (int r = 0; r < RW; ++r) acc[r][m] *= rs;
    }
  }

  if constexpr (EPI == kRwPlain) {
    if (!valid) return;
    // lane r * MM + m stores row0 + r of token m
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int m = 0; m < MM; ++m)
        if (lane == r * MM + m && m < M && row0 + r < N) {
          bf16_t* yp = Y + (int64_t)m * ldy + row0 + r;
          if constexpr (FL & kRwResAdd)
            *yp = f2bf(bf2f(f2bf(acc[r][m])) + bf2f(*yp));   // residual <- bf16(y + residual)
          else
            *yp = f2bf(acc[r][m]);
        }
  } else {
    float a = 0.f, b = 0.f;
    int q;
    if constexpr (PW) {
      if (!valid || lane >= M) return;
#pragma unroll
      for (int m = 0; m < MM; ++m)
        if (lane == m) {
          a = acc[0][m];
          b = acc[RW - 1][m];
        }
      q = gw;
    } else {
      __shared__ float pair_s[kRwWaves / 2][MM];
      if ((wave & 1) && lane == 0) {
#pragma unroll
        for (int m = 0; m < MM; ++m) pair_s[wave >> 1][m] = acc[0][m];
      }
      __syncthreads();
      if ((wave & 1) || !valid || lane >= M) return;
      // lane m < M of the even wave finishes token m
#pragma unroll
      for (int m = 0; m < MM; ++m)
        if (lane == m) {
          a = acc[0][m];
          b = pair_s[wave >> 1][m];
        }
      q = gw >> 1;
    }
    const int m = lane;
    if constexpr (EPI == kRwSwi) {
      const float gf = bf2f(f2bf(a));                 // = the gate_up GEMM's bf16 output
      const float sg = gf / (1.f + __expf(-gf));
      Y[(int64_t)m * ldy + q] = f2bf(bf2f(f2bf(sg)) * bf2f(f2bf(b)));
    } else {
      const int h = q >> 6, d = q & 63;
      float o1 = a, o2 = b;
      if (h < re.Hq + re.Hkv) {
        const float* cs = re.cos_sin + (int64_t)re.positions[m] * 128;
        const float cc = cs[d], ss = cs[64 + d];
        o1 = a * cc - b * ss;
        o2 = b * cc + a * ss;
      }
      bf16_t* dst = nullptr;
      if (h < re.Hq) {
        dst = Y + (int64_t)m * ldy + h * 128;
      } else {
        const int slot = re.slots[m];
        if (slot >= 0) {
          const bool is_k = h < re.Hq + re.Hkv;
          const int kvh = is_k ? h - re.Hq : h - re.Hq - re.Hkv;
          dst = (is_k ? re.k_cache : re.v_cache) +
                (((int64_t)(slot / re.BS) * re.Hkv + kvh) * re.BS + slot % re.BS) * 128;
        }
      }
      if (dst != nullptr) {
        dst[d] = f2bf(o1);
        dst[64 + d] = f2bf(o2);
      }
    }
  }
}

// cfg bits: [1:0] RW = 1 << b (plain only), [3:2] CU = 2 << b (2, 4, 8, 16), bit 6: PW
// (paired epilogues: both rows of a pair in one wave).
// Host-checked: K % 512 == 0, 1 <= M <= 4, (RW + MM) * CU <= 40 loads in flight per lane.
template <int EPI, int MM, int FL>
static void launch_rows_fl(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                           bf16_t* Y, int64_t ldy, int M, int cfg, int up_off, const RopeEpi& re,
                           int waves, float eps, hipStream_t s) {
  if constexpr (EPI != kRwPlain) {
    if (cfg & 64) {                       // PW: one wave per pair -> half the waves
      const dim3 grid((waves / 2 + kRwWaves - 1) / kRwWaves), block(kRwWaves * 64);
      switch (2 << ((cfg >> 2) & 3)) {
#define RW_PW(cu)                                                                              \
  hipLaunchKernelGGL((gemv_rows_kernel<MM, 2, cu, EPI, true, FL, true>), grid, block, 0, s, X, \
                     ldx, W, N, K, Y, ldy, M, up_off, re, eps)
        case 4: RW_PW(4); break;
        case 16: RW_PW(16); break;
        default: RW_PW(8); break;
#undef RW_PW
      }
      return;
    }
  }
  const dim3 grid((waves + kRwWaves - 1) / kRwWaves), block(kRwWaves * 64);
#define RW_L(rw, cu) \
  hipLaunchKernelGGL((gemv_rows_kernel<MM, rw, cu, EPI, true, FL>), grid, block, 0, s, X, ldx, W, \
                     N, K, Y, ldy, M, up_off, re, eps)
  const int rw = 1 << (cfg & 3), cu = 2 << ((cfg >> 2) & 3);
  if constexpr (EPI == kRwPlain) {
    switch (rw * 100 + cu) {
      case 104: RW_L(1, 4); break;
      case 108: RW_L(1, 8); break;
      case 116: RW_L(1, 16); break;
      case 204: RW_L(2, 4); break;
      case 208: RW_L(2, 8); break;
      case 402: RW_L(4, 2); break;
      case 404: RW_L(4, 4); break;
      default: RW_L(8, 2); break;
    }
  } else {
    switch (cu) {
      case 4: RW_L(1, 4); break;
      case 16: RW_L(1, 16); break;
      default: RW_L(1, 8); break;
    }
  }
#undef RW_L
}

// cfg bit 4: kRwNormX (SwiGLU / RoPE), bit 5: kRwResAdd (plain)
template <int EPI, int MM>
static void launch_rows_mm(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                           bf16_t* Y, int64_t ldy, int M, int cfg, int up_off, const RopeEpi& re,
                           int waves, float eps, hipStream_t s) {
  if constexpr (EPI == kRwPlain) {
    if (cfg & 32)
      launch_rows_fl<EPI, MM, kRwResAdd>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
    else
      launch_rows_fl<EPI, MM, 0>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
  } else {
    if (cfg & 16)
      launch_rows_fl<EPI, MM, kRwNormX>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
    else
      launch_rows_fl<EPI, MM, 0>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
  }
}

template <int EPI>
static void launch_rows(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K, bf16_t* Y,
                        int64_t ldy, int M, int cfg, int up_off, const RopeEpi& re, int waves,
                        float eps, hipStream_t s) {
  if (M <= 1)
    launch_rows_mm<EPI, 1>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
  else if (M <= 2)
    launch_rows_mm<EPI, 2>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
  else
    launch_rows_mm<EPI, 4>(X, ldx, W, N, K, Y, ldy, M, cfg, up_off, re, waves, eps, s);
}

void launch_gemv_rows(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K, bf16_t* Y,
                      int64_t ldy, int M, int cfg, hipStream_t s) {
  const int rw = 1 << (cfg & 3);
  launch_rows<kRwPlain>(X, ldx, W, N, K, Y, ldy, M, cfg, 0, RopeEpi{}, (N + rw - 1) / rw, 0.f, s);
}

// Y[M, F] = silu(x Wg^T) * (x Wu^T), w = [Wg; Wu] [2F, K]
void launch_gemv_rows_swiglu(const bf16_t* X, int64_t ldx, const bf16_t* W, int F, int K,
                             bf16_t* Y, int64_t ldy, int M, int cfg, float eps, hipStream_t s) {
  launch_rows<kRwSwi>(X, ldx, W, F, K, Y, ldy, M, cfg, F, RopeEpi{}, 2 * F, eps, s);
}

// qkv = x w^T with RoPE + KV append (N = (Hq + 2 Hkv) * 128); only q columns of Y written
void launch_gemv_rows_rope(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K,
                           bf16_t* Y, int64_t ldy, int M, int cfg, const int32_t* positions,
                           const float* cos_sin, const int32_t* slots, bf16_t* k_cache,
                           bf16_t* v_cache, int Hq, int Hkv, int BS, float eps, hipStream_t s) {
  const RopeEpi re{positions, cos_sin, slots, k_cache, v_cache, Hq, Hkv, BS};
  launch_rows<kRwRope>(X, ldx, W, N / 2, K, Y, ldy, M, cfg, 0, re, N, eps, s);
}

}  // namespace rfq
