// Debug check for SURVEY.md §5.2: count non-finite (Inf / NaN) values in a bf16 matrix
// (the step's logits) into a device counter, without a host sync, so the check can sit
// inside a captured decode graph.  The runner reads the counter together with the
// sampled tokens (RFQ_CHECK_FINITE=1) and fails the step if it is non-zero.
#include "common.h"

namespace rfq {

__global__ __launch_bounds__(256) void count_nonfinite_kernel(const bf16_t* __restrict__ x,
                                                              int64_t stride, int rows, int cols,
                                                              int32_t* __restrict__ counter) {
  const int cpr = cols >> 3;
  int bad = 0;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    const s16x8* row = reinterpret_cast<const s16x8*>(x + (int64_t)r * stride);
    for (int c = threadIdx.x; c < cpr; c += blockDim.x) {
      const s16x8 v = row[c];
#pragma unroll
      for (int k = 0; k < 8; ++k) bad += ((unsigned short)v[k] & 0x7F80u) == 0x7F80u;  // exp all 1s
    }
    for (int c = cpr * 8 + threadIdx.x; c < cols; c += blockDim.x)   // tail columns
      bad += ((unsigned short)x[(int64_t)r * stride + c] & 0x7F80u) == 0x7F80u;
  }
  // one atomic per wave with a non-zero count
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(counter, bad);
}

void launch_count_nonfinite(const bf16_t* x, int64_t stride, int rows, int cols,
                            int32_t* counter, hipStream_t s) {
  if (rows == 0 || cols == 0) return;
  count_nonfinite_kernel<<<rows < 1024 ? rows : 1024, 256, 0, s>>>(x, stride, rows, cols, counter);
}

}  // namespace rfq
