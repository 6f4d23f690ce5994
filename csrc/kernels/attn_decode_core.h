// Decode attention core (paged, GQA, split-K) of attn_decode.hip.
// The design notes are at the top of attn_decode.hip.
#pragma once
#include "common.h"

namespace rfq {

constexpr int kD = 128;
constexpr int kPage = 32;  // tokens per KV block; one key tile == one page
constexpr int kMinPrefixPages = 4;

typedef __attribute__((address_space(1))) unsigned long long gu64;   // global, sc1 access
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ unsigned long long pack_f2(float lo, float hi) {
  return (unsigned long long)__float_as_uint(lo) | ((unsigned long long)__float_as_uint(hi) << 32);
}

struct PrefixArgs {
  const int32_t* meta;     // [0] shared prefix length in tokens (P * kPage), [1] row count
  const int32_t* pflag;    // per sequence: 1 = keys [0, P*32) come from the prefix pass
  const int32_t* rowlist;  // q rows of the participating sequences (meta[1] of them)
  float* pre_o;            // [rows][Hq][128] unnormalised prefix output
  float* pre_ml;           // [rows][Hq][2] running max (log2 domain), softmax sum
};

// (64, 2): two waves per SIMD — NT=2 fits in 244 VGPRs without AGPR spill-over.
// NTK: K / V pages past the first kNtFromPage of a sequence are loaded non-temporal.
// Those pages belong to one sequence and are read once per step per layer; the leading
// pages hold the prompt prefix every request shares (prefix cache), which the other
// sequences' waves re-read from L2 / MALL and keep the default policy.
constexpr int kNtFromPage = 16;

template <bool NTL>
__device__ __forceinline__ s16x8 ld16(const bf16_t* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(p));
  else return *reinterpret_cast<const s16x8*>(p);
}

template <int NT, int MODE = 0, bool NTK = false>
__device__ __forceinline__ void attn_decode_body(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    int bt_stride, const int32_t* __restrict__ seq_q_start, const int32_t* __restrict__ seq_q_len,
    const int32_t* __restrict__ seq_kv_len, const int32_t* __restrict__ work_seq,
    const int32_t* __restrict__ work_ct, bf16_t* __restrict__ out, int64_t out_stride,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hq, int Hkv, float scale_log2,
    int num_splits, const PrefixArgs& px, int32_t* __restrict__ tickets, int split, int kvh,
    int w, bf16_t* __restrict__ v_lds) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;   // 16-lane group
  const int c = lane & 15;   // MFMA column
  const int G = Hq / Hkv;
  bool act[NT], cvalid[NT];
  int h[NT], qrow[NT], lim[NT];
  int seq, ql, kvl, base = 0;
  if constexpr (MODE == 2) {
    // columns are (row, head) pairs of the participating rows, 16 * NT per work item
    const int P = px.meta[0], nrow = px.meta[1];
    if (P == 0 || w * 16 * NT >= nrow * G) return;
    seq = 0; ql = 1; kvl = P;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = (w * NT + t) * 16 + c;
      act[t] = (w * NT + t) * 16 < nrow * G;           // wave-uniform
      cvalid[t] = col < nrow * G;
      qrow[t] = px.rowlist[cvalid[t] ? col / G : 0];
      h[t] = kvh * G + (cvalid[t] ? col % G : 0);
      lim[t] = P;                                      // the whole prefix is visible
    }
  } else {
    seq = work_seq[w];
    if (seq < 0) return;       // padding work item (graph-captured buckets)
    ql = seq_q_len[seq];
    kvl = seq_kv_len[seq];
    if constexpr (MODE == 1) base = px.pflag[seq] ? px.meta[0] : 0;
    // NT column tiles per work item share every K fragment and V tile they load
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tile = work_ct[w] * NT + t;
      act[t] = tile * 16 < ql * G;                       // wave-uniform
      const int col = tile * 16 + c;
      cvalid[t] = col < ql * G;
      const int qi = cvalid[t] ? col / G : 0;
      h[t] = kvh * G + (cvalid[t] ? col % G : 0);
      qrow[t] = seq_q_start[seq] + qi;
      lim[t] = kvl - ql + qi + 1;                        // keys [0, lim) visible
    }
  }

  // MODE 0: split s takes the pages s, s + S, s + 2S, ... (interleaved): its first block-
  // table entry does not depend on kv_len, so that scalar load goes out together with the
  // kv_len / q_len loads and the first K / V page waits on one round trip fewer.  The
  // cascade modes keep contiguous key ranges (their prefix boundary is a page count).
  constexpr bool ILV = MODE == 0;
  const int32_t* bt = block_tables + (int64_t)seq * bt_stride;
  int pg_next = 0;
  if constexpr (ILV) pg_next = bt[__builtin_amdgcn_readfirstlane(min(split, bt_stride - 1))];
  int tps = (kvl - base + num_splits - 1) / num_splits;
  tps = (tps + kPage - 1) / kPage * kPage;
  const int npg_all = (kvl + kPage - 1) / kPage;
  const int start = ILV ? split * kPage : base + split * tps;
  const int end = ILV ? kvl : min(kvl, start + tps);

  float m_run[NT], l_run[NT];
  f32x4 o[NT][8];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    m_run[t] = -INFINITY;
    l_run[t] = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) o[t][m] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  if (start < end && ql > 0) {
    // Q^T fragments: B[k = dh][col]; lane holds Q[qrow, h][32ks + 8g .. +7]
    s16x8 qf[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16_t* qp = q + (int64_t)qrow[t] * q_stride + (int64_t)h[t] * kD;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        qf[t][ks] = reinterpret_cast<const s16x8*>(qp + 32 * ks + 8 * g)[0];
        if (!cvalid[t]) qf[t][ks] = (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
    // pages of this split: contiguous [pg0, pg_last], or interleaved pg0 + j * S
    const int pstep = ILV ? num_splits : 1;
    const int pg0 = start / kPage;
    const int np = ILV ? (npg_all - split + num_splits - 1) / num_splits
                       : (end - 1) / kPage - pg0 + 1;
    const int pg_last = pg0 + (np - 1) * pstep;
    // block-table entries by wave-uniform (scalar, lgkmcnt-counted) loads, one page
    // ahead: a vector load here would make every page's K / V issue wait on vmcnt(0),
    // i.e. drain the page loads already in flight
    if constexpr (!ILV) pg_next = bt[__builtin_amdgcn_readfirstlane(pg0)];
    // issue page j's K fragments (A operand: row = key, k = dh) and V rows (g + 4i,
    // chunk c) into registers; must be called with j = 0, 1, 2, ...
    auto fetch = [&](int j, s16x8 (&kf)[2][4], s16x8 (&vr)[8]) {
      const int64_t page = pg_next;
      pg_next = bt[__builtin_amdgcn_readfirstlane(min(pg0 + (j + 1) * pstep, pg_last))];
      const bf16_t* kb = k_cache + ((page * Hkv + kvh) * kPage) * kD;
      const bf16_t* vb = v_cache + ((page * Hkv + kvh) * kPage) * kD;
      if (NTK && pg0 + j >= kNtFromPage) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            kf[mt][ks] = ld16<true>(kb + (16 * mt + c) * kD + 32 * ks + 8 * g);
#pragma unroll
        for (int i = 0; i < 8; ++i) vr[i] = ld16<true>(vb + (g + 4 * i) * kD + 8 * c);
      } else {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            kf[mt][ks] = ld16<false>(kb + (16 * mt + c) * kD + 32 * ks + 8 * g);
#pragma unroll
        for (int i = 0; i < 8; ++i) vr[i] = ld16<false>(vb + (g + 4 * i) * kD + 8 * c);
      }
    };
    auto process = [&](int j, const s16x8 (&kf)[2][4], const s16x8 (&vr)[8]) {
      const int kt = start + j * pstep * kPage;
      const int nvalid = end - kt;  // keys of this tile inside the split (>= 1; > 32 = all)
      // ---- V tile -> LDS (swizzled), rows past the split/context zeroed ----
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = g + 4 * i, ch = c;
        const s16x8 v = row >= nvalid ? (s16x8){0, 0, 0, 0, 0, 0, 0, 0} : vr[i];
        const int pch = ch ^ ((row & 7) << 1);
        reinterpret_cast<s16x8*>(v_lds + row * kD)[pch] = v;
      }

      s16x8 pb[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (!act[t]) continue;
        // ---- S^T = K Q^T ----
        f32x4 s[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          s[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(kf[mt][ks]),
                                                            as_bf16x8(qf[t][ks]), s[mt], 0, 0, 0);
        }
        // lane holds S^T[key = 16mt + 4g + i][column c]
        float mx = -INFINITY;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = 16 * mt + 4 * g + i;
            float v = s[mt][i] * scale_log2;
            if (key >= nvalid || kt + key >= lim[t]) v = -INFINITY;
            s[mt][i] = v;
            mx = fmaxf(mx, v);
          }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run[t], mx);
        const float m_use = (m_new == -INFINITY) ? 0.f : m_new;  // fully-masked column so far
        const float alpha = fast_exp2(m_run[t] - m_use);
        float psum = 0.f;
        float p[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          p[jj] = fast_exp2(s[jj >> 2][jj & 3] - m_use);
          psum += p[jj];
        }
        l_run[t] = l_run[t] * alpha + psum;
        m_run[t] = m_new;
#pragma unroll
        for (int m = 0; m < 8; ++m) o[t][m] *= alpha;
        // P^T as B operand: element j <-> key pi(g,j) = (j<4 ? 4g+j : 16+4g+j-4)
        pb[t] = pack8(p);
      }

      __syncthreads();  // V tile visible

      // ---- O^T += V^T P^T (one transposed V read feeds every tile) ----
      const int q4 = c >> 2, p4 = c & 3;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int r0 = 4 * g + q4, r1 = 16 + 4 * g + q4;
        const int ch = 2 * m + (p4 >> 1), sub = (p4 & 1) * 4;
        const s16x4 a0 = ds_read_tr16(v_lds + r0 * kD + ((ch ^ ((r0 & 7) << 1)) * 8) + sub);
        const s16x4 a1 = ds_read_tr16(v_lds + r1 * kD + ((ch ^ ((r1 & 7) << 1)) * 8) + sub);
        const s16x8 a = (s16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (act[t])
            o[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(pb[t]),
                                                              o[t][m], 0, 0, 0);
      }
      __syncthreads();  // before the next tile overwrites v_lds
    };

    s16x8 kA[2][4], vA[8];
    if constexpr (NT == 1) {
      // NT 1 has the registers for a second page in flight: page j+1's K / V loads
      // are issued before page j is processed (two register sets, unrolled by two), so
      // a split walking several pages pays one memory round trip, not one per page
      // The counted wait (a real S_WAITCNT, which the compiler's wait pass accounts
      // for) retires page j -- in flight during page j-1 -- BEFORE page j+1 is issued.
      // Without it the wait pass, merging its scoreboard over the loop back edge, treats
      // page j's loads as the newest and waits on page j+1's too (vmcnt 15..0).
      constexpr int kVmcnt0 = 0x0F70;          // vmcnt(0), expcnt / lgkmcnt untouched
      s16x8 kB[2][4], vB[8];
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
    } else {
      for (int j = 0; j < np; ++j) {
        fetch(j, kA, vA);
        process(j, kA, vA);
      }
    }
  }

#pragma unroll
  for (int t = 0; t < NT; ++t) {
    // total softmax denominator for column c (lanes c, c+16, c+32, c+48)
    float l_tot = l_run[t];
    l_tot += __shfl_xor(l_tot, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (!cvalid[t]) continue;
    if constexpr (MODE == 2) {
      const int64_t pidx = (int64_t)qrow[t] * Hq + h[t];
      float* po = px.pre_o + pidx * kD;
#pragma unroll
      for (int m = 0; m < 8; ++m) *reinterpret_cast<f32x4*>(po + 16 * m + 4 * g) = o[t][m];
      if (g == 0) {
        px.pre_ml[pidx * 2 + 0] = m_run[t];
        px.pre_ml[pidx * 2 + 1] = l_tot;
      }
      continue;
    }
    if (MODE == 1 && num_splits == 1 && base > 0) {
      // merge the shared-prefix partial of this (row, head) column
      const int64_t pidx = (int64_t)qrow[t] * Hq + h[t];
      const float pm = px.pre_ml[pidx * 2 + 0], pl = px.pre_ml[pidx * 2 + 1];
      const float* po = px.pre_o + pidx * kD;
      const float mt = fmaxf(m_run[t], pm);
      const float mu = mt == -INFINITY ? 0.f : mt;
      const float a1 = fast_exp2(m_run[t] - mu), a2 = fast_exp2(pm - mu);
      l_tot = l_tot * a1 + pl * a2;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const f32x4 pv = *reinterpret_cast<const f32x4*>(po + 16 * m + 4 * g);
        o[t][m] = o[t][m] * a1 + pv * a2;
      }
    }
    if (num_splits == 1) {
      const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
      bf16_t* orow = out + (int64_t)qrow[t] * out_stride + (int64_t)h[t] * kD;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        uint2 wv;
        wv.x = pack_bf16x2(o[t][m][0] * inv, o[t][m][1] * inv);
        wv.y = pack_bf16x2(o[t][m][2] * inv, o[t][m][3] * inv);
        *reinterpret_cast<uint2*>(orow + 16 * m + 4 * g) = wv;
      }
    } else {
      // partials write-through (8-byte agent-scope atomic stores = sc1): the in-kernel
      // merge below reads them without a release / acquire pair
      const int64_t pidx = ((int64_t)qrow[t] * Hq + h[t]) * num_splits + split;
      float* po = part_o + pidx * kD;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        gu64* d = (gu64*)(po + 16 * m + 4 * g);
        __hip_atomic_store(d, pack_f2(o[t][m][0], o[t][m][1]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d + 1, pack_f2(o[t][m][2], o[t][m][3]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      if (g == 0)
        __hip_atomic_store((gu64*)(part_ml + pidx * 2), pack_f2(m_run[t], l_tot),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (MODE != 0 || num_splits == 1 || tickets == nullptr) return;

  // Single pass (cdna_hip_programming.md §6 Guideline 16, R1 counter form): the
  // partials above are sc1 stores, drained by this wave's vmcnt(0) before its relaxed
  // agent-scope ticket add; the last of the num_splits waves of this (work item, kv
  // head) reads every partial with sc1 loads (no L1 copy can be stale, so no acquire
  // fence), merges them and writes the bf16 output -- no second reduce launch -- then
  // zeroes the ticket for the next launch on the stream.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  gu32* tk = (gu32*)(tickets + (int64_t)w * Hkv + kvh);
  unsigned prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __builtin_amdgcn_readfirstlane(prev);   // uniform: the merge branch stays scalar
  if (prev != (unsigned)num_splits - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every handed-off load is sc1
  if (lane == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // The merge uses the whole wave per group of 4 columns: lane l serves column
  // 4 r + (l >> 4) and split j = l & 15 of the (max, sum) pairs, and dims
  // [8 j, 8 j + 8) of every split's partial row.  Every split's partial loads of the
  // group are issued at once (32 x 16 B per lane), so a group costs ONE dependent round
  // trip, not one per split pair (the r2 form: 8 chained rounds for 16 splits).
  const int mj = lane & 15, mq = lane >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (!act[t]) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cc = 4 * r + mq;                          // column this lane merges
      const int v_cc = __shfl((int)cvalid[t], cc, 64);
      const int q_cc = __shfl(qrow[t], cc, 64), h_cc = __shfl(h[t], cc, 64);
      if (!__builtin_amdgcn_ballot_w64(v_cc != 0)) continue;       // wave-uniform: group empty
      const int64_t pbase = ((int64_t)q_cc * Hq + h_cc) * num_splits;
      const bool live = v_cc != 0;
      // (max, sum) of split mj, and every split's dims [8 mj, 8 mj + 8)
      unsigned long long mlx = 0xff800000ull;             // (-inf, 0)
      if (live && mj < num_splits)
        mlx = __hip_atomic_load((const gu64*)(part_ml + (pbase + mj) * 2), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
      f32x4 pv[16][2];
#pragma unroll
      for (int sp = 0; sp < 16; ++sp) {
        if (live && sp < num_splits) {
          const gu64* d = (const gu64*)(part_o + (pbase + sp) * kD + 8 * mj);
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const unsigned long long x0 =
                __hip_atomic_load(d + 2 * u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long x1 =
                __hip_atomic_load(d + 2 * u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pv[sp][u] = (f32x4){__uint_as_float((unsigned)x0), __uint_as_float((unsigned)(x0 >> 32)),
                                __uint_as_float((unsigned)x1), __uint_as_float((unsigned)(x1 >> 32))};
          }
        } else {
          pv[sp][0] = pv[sp][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
      const float m_j = __uint_as_float((unsigned)mlx), l_j = __uint_as_float((unsigned)(mlx >> 32));
      float gm = m_j;                                     // max over the 16 lanes of the column
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) gm = fmaxf(gm, __shfl_xor(gm, o2, 64));
      const float w_j = (gm == -INFINITY || m_j == -INFINITY) ? 0.f : fast_exp2(m_j - gm);
      float den = w_j * l_j;
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) den += __shfl_xor(den, o2, 64);
      f32x4 num[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int sp = 0; sp < 16; ++sp) {
        const float wsp = __shfl(w_j, (lane & 48) | sp, 64);   // split sp's weight
#pragma unroll
        for (int u = 0; u < 2; ++u) num[u] += wsp * pv[sp][u];
      }
      if (!live) continue;
      const float inv = den > 0.f ? 1.f / den : 0.f;
      uint4 ov;
      ov.x = pack_bf16x2(num[0][0] * inv, num[0][1] * inv);
      ov.y = pack_bf16x2(num[0][2] * inv, num[0][3] * inv);
      ov.z = pack_bf16x2(num[1][0] * inv, num[1][1] * inv);
      ov.w = pack_bf16x2(num[1][2] * inv, num[1][3] * inv);
      *reinterpret_cast<uint4*>(out + (int64_t)q_cc * out_stride + (int64_t)h_cc * kD + 8 * mj) = ov;
    }
  }
}

}  // namespace rfq
