// One-shot (decode-size) and two-shot (prefill-size) all-reduce over xGMI peer
// memory for tensor-parallel steps (SURVEY.md §2.2 custom_allreduce, §2.5 C1/C2, §5.8).
//
// A decode step of Llama-3-70B at TP=8 issues 160 all-reduces of a few KB to
// ~1 MB.  At that size the cost is latency, not bandwidth: every rank simply
// reads the other ranks' copies over its 7 xGMI links at once and sums them —
// one kernel, no ring, no second pass.
//
// Memory: each rank owns one uncached (hipDeviceMallocUncached) region,
// exported with hipIpcGetMemHandle and opened by every peer:
//
//   [ Signal (flags + per-block counters) | data staging area ]
//
// Per call, workgroup b of every rank owns element slice b:
//   1. copy its slice of the input into the rank's own staging area;
//   2. release-store its block counter c into start[b][rank] of every peer;
//   3. acquire-spin on its own start[b][p] == c for all p (slice b of every
//      peer is now visible);
//   4. sum slice b across all ranks' staging areas (fp32), write the output;
//   5. release end[b][rank] = c to every peer and spin on end[b][p] == c, so no
//      rank starts the next call (overwriting slice b) while a peer still reads.
// The counter is per block and lives in device memory, so the kernel is
// graph-capturable (replays keep counting).  Every spin is bounded: on timeout
// the kernel records an error in its signal area and falls through instead of
// hanging the GPU; the host checks it (car_check) and falls back to RCCL.
#include <hip/hip_runtime.h>

#include "../kernels/common.h"
#include "car_core.h"

namespace rfq {

__global__ __launch_bounds__(kCarThreads) void car_oneshot_kernel(
    CarPeers peers, int rank, int world, const bf16_t* __restrict__ in,
    bf16_t* __restrict__ out, int64_t n8) {
  CarSignal* self = reinterpret_cast<CarSignal*>(peers.base[rank]);
  const int b = blockIdx.x, nb = gridDim.x;
  const int tid = threadIdx.x;
  const int64_t per = (n8 + nb - 1) / nb;          // 16-byte chunks per block
  const int64_t c0 = b * per, c1 = min(n8, c0 + per);
  __shared__ uint32_t cnt_s;
  __shared__ int fail_s;
  if (tid == 0) {
    cnt_s = self->counter[b] + 1;
    fail_s = 0;
  }
  // 1. stage own slice
  s16x8* own = reinterpret_cast<s16x8*>(peers.base[rank] + kCarDataOffset);
  const s16x8* src = reinterpret_cast<const s16x8*>(in);
  for (int64_t i = c0 + tid; i < c1; i += kCarThreads) own[i] = src[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // system scope: staged slice visible
  __syncthreads();
  const uint32_t c = cnt_s;
  // 2-3. publish, then wait for every peer's slice b
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->start[b][rank], c);
    if (!car_wait(self, &self->start[b][tid], c, kCarStart, b, tid)) fail_s = 1;
  }
  __syncthreads();
  // 4. reduce slice b
  for (int64_t i = c0 + tid; i < c1; i += kCarThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      const s16x8 v = reinterpret_cast<const s16x8*>(peers.base[p] + kCarDataOffset)[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f_s(v[j]);
    }
    reinterpret_cast<s16x8*>(out)[i] = pack8(acc);
  }
  __syncthreads();
  // 5. everyone is done reading slice b before anyone reuses it
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->end[b][rank], c);
    if (!car_wait(self, &self->end[b][tid], c, kCarEnd, b, tid)) fail_s = 1;
  }
  __syncthreads();
  if (tid == 0) {
    self->counter[b] = c;
    if (fail_s) atomicAdd(&self->error, 1u);
  }
}

// Two-shot all-reduce for prefill-size messages: a one-shot
// call makes every rank read world x n bytes over xGMI, which stops paying once the
// message is bandwidth-bound.  Here the message is cut into `world` slices and
// every rank moves only ~2n bytes, striped over all of its links at once:
//   1. stage sub-range b of every slice into the own region; flags start[b];
//   2. reduce-scatter: rank r sums sub-range b of slice r over every peer's staged
//      copy and writes the sum back into slice r of its own staging (safe: in this
//      step peer q reads only slice q of this rank's staging); flags mid[b];
//   3. all-gather: out[slice p, sub-range b] = peer p's reduced sub-range b;
//      flags end[b] so no rank overwrites its staging while a peer still reads.
// Block b of every rank owns the same sub-range of every slice, so the per-block
// flag protocol of the one-shot kernel carries over unchanged.
__global__ __launch_bounds__(kCarThreads) void car_twoshot_kernel(
    CarPeers peers, int rank, int world, const bf16_t* __restrict__ in,
    bf16_t* __restrict__ out, int64_t n8) {
  CarSignal* self = reinterpret_cast<CarSignal*>(peers.base[rank]);
  const int b = blockIdx.x, nb = gridDim.x;
  const int tid = threadIdx.x;
  const int64_t slice = (n8 + world - 1) / world;   // 16-byte chunks per slice
  const int64_t per = (slice + nb - 1) / nb;        // ... per block within a slice
  const int64_t o0 = b * per, o1 = min(slice, o0 + per);
  __shared__ uint32_t cnt_s;
  __shared__ int fail_s;
  if (tid == 0) {
    cnt_s = self->counter[b] + 1;
    fail_s = 0;
  }
  s16x8* own = reinterpret_cast<s16x8*>(peers.base[rank] + kCarDataOffset);
  const s16x8* src = reinterpret_cast<const s16x8*>(in);
  // 1. stage sub-range b of every slice
  for (int sl = 0; sl < world; ++sl) {
    const int64_t base = sl * slice;
    for (int64_t i = o0 + tid; i < o1; i += kCarThreads)
      if (base + i < n8) own[base + i] = src[base + i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  const uint32_t c = cnt_s;
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->start[b][rank], c);
    if (!car_wait(self, &self->start[b][tid], c, kCarStart, b, tid)) fail_s = 1;
  }
  __syncthreads();
  // 2. reduce-scatter: own slice, summed over every rank's staged copy
  {
    const int64_t base = rank * slice;
    for (int64_t i = o0 + tid; i < o1; i += kCarThreads) {
      if (base + i >= n8) break;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < world; ++p) {
        const s16x8 v = reinterpret_cast<const s16x8*>(peers.base[p] + kCarDataOffset)[base + i];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f_s(v[j]);
      }
      own[base + i] = pack8(acc);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->mid[b][rank], c);
    if (!car_wait(self, &self->mid[b][tid], c, kCarMid, b, tid)) fail_s = 1;
  }
  __syncthreads();
  // 3. all-gather the reduced slices
  s16x8* dst = reinterpret_cast<s16x8*>(out);
  for (int p = 0; p < world; ++p) {
    const s16x8* rem = reinterpret_cast<const s16x8*>(peers.base[p] + kCarDataOffset);
    const int64_t base = p * slice;
    for (int64_t i = o0 + tid; i < o1; i += kCarThreads)
      if (base + i < n8) dst[base + i] = rem[base + i];
  }
  __syncthreads();
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->end[b][rank], c);
    if (!car_wait(self, &self->end[b][tid], c, kCarEnd, b, tid)) fail_s = 1;
  }
  __syncthreads();
  if (tid == 0) {
    self->counter[b] = c;
    if (fail_s) atomicAdd(&self->error, 1u);
  }
}

// One-shot all-reduce fused with the residual-add RMSNorm that follows every
// row-parallel projection of a TP decoder layer (o and down):
//   residual <- bf16(bf16(sum_p x_p) + residual);  out <- rmsnorm(residual) * w.
// At decode sizes the all-reduce and the norm are both pure launch latency, so one
// kernel instead of two saves one dispatch per all-reduce (160 per Llama-3-70B
// step at TP=8).  Workgroup b owns row b (whole rows, so the norm's reduction
// stays inside the workgroup); the flag protocol is the one-shot kernel's, on the
// same per-block counters.  Thread layout, rounding points and the block_sum
// order are those of fused_add_rms_norm_kernel (norm.hip), so the result is
// bit-identical to car_oneshot_kernel followed by fused_add_rms_norm_kernel.
template <int NCH>
__global__ __launch_bounds__(256) void car_oneshot_add_norm_kernel(
    CarPeers peers, int rank, int world, const bf16_t* in, bf16_t* __restrict__ residual,
    int64_t res_stride, const bf16_t* __restrict__ w, bf16_t* out, int64_t out_stride, int d,
    float eps) {
  CarSignal* self = reinterpret_cast<CarSignal*>(peers.base[rank]);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int nchunk = d >> 3;
  __shared__ uint32_t cnt_s;
  __shared__ int fail_s;
  __shared__ float scratch[16];
  if (tid == 0) {
    cnt_s = self->counter[b] + 1;
    fail_s = 0;
  }
  // 1. stage own row (the data area holds rows back to back, as the input)
  const int64_t row0 = (int64_t)b * nchunk;
  s16x8* own = reinterpret_cast<s16x8*>(peers.base[rank] + kCarDataOffset) + row0;
  const s16x8* src = reinterpret_cast<const s16x8*>(in) + row0;
  s16x8* rr = reinterpret_cast<s16x8*>(residual + b * res_stride);
  const s16x8* wr = reinterpret_cast<const s16x8*>(w);
  s16x8 rv[NCH], wv[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = tid + k * 256;
    if (c < nchunk) {
      own[c] = src[c];
      rv[k] = rr[c];                  // residual and weight ride along with the staging
      wv[k] = wr[c];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // system scope: staged row visible
  __syncthreads();
  const uint32_t c = cnt_s;
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->start[b][rank], c);
    if (!car_wait(self, &self->start[b][tid], c, kCarStart, b, tid)) fail_s = 1;
  }
  __syncthreads();
  // 2. sum row b over the ranks (rank order, fp32, rounded to bf16 = the all-reduce
  //    output), add the residual, round, keep the rounded residual for the norm
  float v[NCH][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + k * 256;
    if (ch < nchunk) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < world; ++p) {
        const s16x8 pv =
            (reinterpret_cast<const s16x8*>(peers.base[p] + kCarDataOffset) + row0)[ch];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f_s(pv[j]);
      }
      float a[8], r[8];
      unpack8(pack8(acc), a);
      unpack8(rv[k], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += r[j];
      const s16x8 packed = pack8(a);
      rr[ch] = packed;
      unpack8(packed, v[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
    }
  }
  __syncthreads();
  // 3. every peer is done reading row b of this rank before anyone restages it
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->end[b][rank], c);
    if (!car_wait(self, &self->end[b][tid], c, kCarEnd, b, tid)) fail_s = 1;
  }
  ss = block_sum(ss, scratch);        // its barriers also order the end handshake
  const float rs = rsqrtf(ss / (float)d + eps);
  s16x8* orow = reinterpret_cast<s16x8*>(out + b * out_stride);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + k * 256;
    if (ch < nchunk) {
      float wf[8], o[8];
      unpack8(wv[k], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * rs * wf[j];
      orow[ch] = pack8(o);
    }
  }
  if (tid == 0) {
    self->counter[b] = c;
    if (fail_s) atomicAdd(&self->error, 1u);
  }
}


// Push one-shot all-reduce + residual-add RMSNorm for decode rows (the latency path's
// 160 all-reduces per Llama-3-70B step at TP=8).  One xGMI hop instead of the staged
// form's three (flag out, remote read, end flag):
//   1. every rank WRITES its row b into slot [parity][rank][b] of every peer's staging
//      (remote stores over its links, all peers at once), drains them (system-scope
//      release), then stores the call counter c into flag push[parity][b][rank] of
//      every peer;
//   2. it waits on its OWN flags push[parity][b][*] == c (local polls);
//   3. it sums the world rows that landed in its own staging (local reads), adds the
//      residual and normalises, exactly like car_oneshot_add_norm.
// No end barrier: parity = c & 1 alternates the staging and flag sets, and a rank can
// only reach call c + 2 of row b after every peer published call c + 1 of row b, i.e.
// after every peer's kernel of call c -- the last reader of the parity-c slots -- has
// completed on its stream.  Same rounding points and block_sum order as the staged
// kernel, so the result is bit-identical to it (and to all_reduce + fused_add_rms_norm).
template <int NCH>
__global__ __launch_bounds__(256) void car_push_add_norm_kernel(
    CarPeers peers, int rank, int world, const bf16_t* in, bf16_t* __restrict__ residual,
    int64_t res_stride, const bf16_t* __restrict__ w, bf16_t* out, int64_t out_stride, int d,
    int rows, float eps) {
  CarSignal* self = reinterpret_cast<CarSignal*>(peers.base[rank]);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int nchunk = d >> 3;
  __shared__ uint32_t cnt_s;
  __shared__ int fail_s;
  __shared__ float scratch[16];
  if (tid == 0) {
    cnt_s = self->counter[b] + 1;
    fail_s = 0;
  }
  __syncthreads();
  const uint32_t c = cnt_s;
  const int par = (int)(c & 1u);
  const s16x8* src = reinterpret_cast<const s16x8*>(in) + (int64_t)b * nchunk;
  s16x8 xv[NCH], rv[NCH], wv[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + k * 256;
    if (ch < nchunk) xv[k] = src[ch];
  }
  car_push_preload<NCH>(b, residual, res_stride, w, d, rv, wv);
  // 1. push the row into every rank's slot [par][rank][b] (own region included)
  for (int p = 0; p < world; ++p) {
    s16x8* dst = car_push_slot(peers.base[p], par, rank, b);
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int ch = tid + k * 256;
      if (ch < nchunk) dst[ch] = xv[k];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // system scope: pushed rows landed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < world) {
    CarSignal* peer = reinterpret_cast<CarSignal*>(peers.base[tid]);
    car_store(&peer->push[par][b][rank], c);
    // 2. wait for row b of peer `tid` in the own staging
    if (!car_wait(self, &self->push[par][b][tid], c, kCarPush, b, tid)) fail_s = 1;
  }
  __syncthreads();
  // 3. sum row b over the ranks, add the residual, normalise
  car_push_sum_norm_row<NCH>(peers.base[rank], par, world, b, residual, res_stride, rv, wv, out,
                             out_stride, d, eps, scratch);
  if (tid == 0) {
    self->counter[b] = c;
    if (fail_s) atomicAdd(&self->error, 1u);
  }
}

// ------------------------------------------------------------------ host side
int64_t car_signal_bytes() { return kCarDataOffset; }

int car_norm_max_rows() { return kCarMaxBlocks; }

void launch_car_oneshot_add_norm(char* const* bases, int rank, int world, const bf16_t* in,
                                 bf16_t* residual, int64_t res_stride, const bf16_t* w,
                                 bf16_t* out, int64_t out_stride, int rows, int d, float eps,
                                 hipStream_t s) {
  CarPeers peers{};
  for (int p = 0; p < world; ++p) peers.base[p] = bases[p];
  const int nch = (d / 8 + 255) / 256;
#define CAR_NORM_LAUNCH(N)                                                              \
  car_oneshot_add_norm_kernel<N><<<rows, 256, 0, s>>>(peers, rank, world, in, residual, \
                                                      res_stride, w, out, out_stride, d, eps)
  if (nch <= 1) CAR_NORM_LAUNCH(1);
  else if (nch <= 2) CAR_NORM_LAUNCH(2);
  else if (nch <= 4) CAR_NORM_LAUNCH(4);
  else CAR_NORM_LAUNCH(8);
#undef CAR_NORM_LAUNCH
}

// the push form's fixed slot layout [2][kCarMaxRanks][kCarPushRows][kCarPushD] bf16 (4 MiB)
// fits the staging capacity and the call's rows / width fit a slot
bool car_push_fits(int world, int rows, int d, int64_t capacity) {
  return world <= kCarMaxRanks && rows >= 1 && rows <= kCarPushRows && d <= kCarPushD &&
         2ll * kCarMaxRanks * kCarPushRows * kCarPushD * 2 <= capacity;
}

void launch_car_push_add_norm(char* const* bases, int rank, int world, const bf16_t* in,
                              bf16_t* residual, int64_t res_stride, const bf16_t* w,
                              bf16_t* out, int64_t out_stride, int rows, int d, float eps,
                              hipStream_t s) {
  CarPeers peers{};
  for (int p = 0; p < world; ++p) peers.base[p] = bases[p];
  const int nch = (d / 8 + 255) / 256;
#define CAR_PUSH_LAUNCH(N)                                                                   \
  car_push_add_norm_kernel<N><<<rows, 256, 0, s>>>(peers, rank, world, in, residual,          \
                                                   res_stride, w, out, out_stride, d, rows, eps)
  if (nch <= 1) CAR_PUSH_LAUNCH(1);
  else if (nch <= 2) CAR_PUSH_LAUNCH(2);
  else if (nch <= 4) CAR_PUSH_LAUNCH(4);
  else CAR_PUSH_LAUNCH(8);
#undef CAR_PUSH_LAUNCH
}

hipError_t car_alloc(int64_t data_bytes, void** ptr) {
  const int64_t bytes = kCarDataOffset + data_bytes;
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  return hipMemset(*ptr, 0, kCarDataOffset);
}

void launch_car_oneshot(char* const* bases, int rank, int world, const bf16_t* in, bf16_t* out,
                        int64_t numel, hipStream_t s) {
  CarPeers peers{};
  for (int p = 0; p < world; ++p) peers.base[p] = bases[p];
  const int64_t n8 = numel / 8;
  int nb = (int)((n8 + kCarThreads * 2 - 1) / (kCarThreads * 2));
  nb = nb < 1 ? 1 : (nb > kCarMaxBlocks ? kCarMaxBlocks : nb);
  car_oneshot_kernel<<<nb, kCarThreads, 0, s>>>(peers, rank, world, in, out, n8);
}

void launch_car_twoshot(char* const* bases, int rank, int world, const bf16_t* in, bf16_t* out,
                        int64_t numel, hipStream_t s) {
  CarPeers peers{};
  for (int p = 0; p < world; ++p) peers.base[p] = bases[p];
  const int64_t n8 = numel / 8;
  const int64_t slice = (n8 + world - 1) / world;
  int nb = (int)((slice + kCarThreads * 2 - 1) / (kCarThreads * 2));
  nb = nb < 1 ? 1 : (nb > kCarMaxBlocks ? kCarMaxBlocks : nb);
  car_twoshot_kernel<<<nb, kCarThreads, 0, s>>>(peers, rank, world, in, out, n8);
}

uint32_t car_read_error(const void* base) {
  uint32_t err = 0;
  hipMemcpy(&err, reinterpret_cast<const char*>(base) + offsetof(CarSignal, error), 4,
            hipMemcpyDeviceToHost);
  return err;
}

uint32_t car_read_info(const void* base) {
  uint32_t info = 0;
  hipMemcpy(&info, reinterpret_cast<const char*>(base) + offsetof(CarSignal, info), 4,
            hipMemcpyDeviceToHost);
  return info;
}

}  // namespace rfq
