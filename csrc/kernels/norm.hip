// RMSNorm and fused residual-add + RMSNorm (Llama / Mixtral pre-norm blocks).
//
// Implied compute of the remote llama3-70b call (rfq_agent.py:62,163 in the
// reference); SURVEY.md §2.4 K2.  Memory-bound: one workgroup per row, each lane
// owns NCH 16-byte chunks held in registers between the reduction and the store,
// so the row is read once and written once (twice for the fused form: residual
// and normed output).
#include "common.h"

namespace rfq {

template <int NCH>
__global__ __launch_bounds__(256) void rms_norm_kernel(
    const bf16_t* __restrict__ x, int64_t x_stride, const bf16_t* __restrict__ w,
    bf16_t* __restrict__ out, int64_t out_stride, int d, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nchunk = d >> 3;
  const s16x8* xr = reinterpret_cast<const s16x8*>(x + row * x_stride);
  const s16x8* wr = reinterpret_cast<const s16x8*>(w);
  float v[NCH][8];
  s16x8 wv[NCH];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      wv[k] = wr[c];                  // weight fetched with x: one memory round trip
      unpack8(xr[c], v[k]);
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[k][i] * v[k][i];
    }
  }
  ss = block_sum(ss, scratch);
  const float r = rsqrtf(ss / (float)d + eps);
  s16x8* orow = reinterpret_cast<s16x8*>(out + row * out_stride);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      float wf[8], o[8];
      unpack8(wv[k], wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[k][i] * r * wf[i];
      orow[c] = pack8(o);
    }
  }
}

// residual <- bf16(x + residual);  out <- rmsnorm(residual) * w.   out may alias x.
template <int NCH>
__global__ __launch_bounds__(256) void fused_add_rms_norm_kernel(
    const bf16_t* x, int64_t x_stride, bf16_t* __restrict__ residual, int64_t res_stride,
    const bf16_t* __restrict__ w, bf16_t* out, int64_t out_stride, int d, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nchunk = d >> 3;
  const s16x8* xr = reinterpret_cast<const s16x8*>(x + row * x_stride);
  s16x8* rr = reinterpret_cast<s16x8*>(residual + row * res_stride);
  const s16x8* wr = reinterpret_cast<const s16x8*>(w);
  float v[NCH][8];
  s16x8 wv[NCH];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      wv[k] = wr[c];                  // weight fetched with x: one memory round trip
      float a[8], b[8];
      unpack8(xr[c], a);
      unpack8(rr[c], b);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += b[i];
      s16x8 packed = pack8(a);
      rr[c] = packed;
      unpack8(packed, v[k]);  // normalise the rounded residual (matches the unfused oracle)
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[k][i] * v[k][i];
    }
  }
  ss = block_sum(ss, scratch);
  const float r = rsqrtf(ss / (float)d + eps);
  s16x8* orow = reinterpret_cast<s16x8*>(out + row * out_stride);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      float wf[8], o[8];
      unpack8(wv[k], wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[k][i] * r * wf[i];
      orow[c] = pack8(o);
    }
  }
}

#define NCH_DISPATCH(d, ...)                         \
  do {                                               \
    const int nch_ = ((d) / 8 + 255) / 256;          \
    if (nch_ <= 1) { constexpr int NCH = 1; __VA_ARGS__; }      \
    else if (nch_ <= 2) { constexpr int NCH = 2; __VA_ARGS__; } \
    else if (nch_ <= 4) { constexpr int NCH = 4; __VA_ARGS__; } \
    else { constexpr int NCH = 8; __VA_ARGS__; }               \
  } while (0)

void launch_rms_norm(const bf16_t* x, int64_t x_stride, const bf16_t* w, bf16_t* out,
                     int64_t out_stride, int rows, int d, float eps, hipStream_t s) {
  if (rows == 0) return;
  NCH_DISPATCH(d, rms_norm_kernel<NCH><<<rows, 256, 0, s>>>(x, x_stride, w, out, out_stride, d, eps));
}

void launch_fused_add_rms_norm(const bf16_t* x, int64_t x_stride, bf16_t* residual,
                               int64_t res_stride, const bf16_t* w, bf16_t* out,
                               int64_t out_stride, int rows, int d, float eps, hipStream_t s) {
  if (rows == 0) return;
  NCH_DISPATCH(d, fused_add_rms_norm_kernel<NCH><<<rows, 256, 0, s>>>(
                      x, x_stride, residual, res_stride, w, out, out_stride, d, eps));
}

}  // namespace rfq
