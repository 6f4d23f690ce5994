// Single-workgroup streaming bandwidth: how fast can ONE CU (or a handful) pull a
// few hundred KB from HBM when the rest of the chip is idle?  Input to the batch-1
// decode attention design (docs/ROUND6_STATUS.md item 2): the split-KV form spreads
// 0.5-4 MB of KV over 16-128 workgroups and pays a global merge; a per-kv-head
// workgroup could merge in LDS if one CU streams its share fast enough.
//
// Each of G workgroups (1024 threads = 16 waves) reads B contiguous bytes with 16-byte
// loads, 4 in flight per thread per iteration, and writes one float (vector store) so
// the loads are not dead.  Every launch reads a fresh window of a 2 GiB buffer (8x the
// 256 MB Infinity Cache) so the data comes from HBM, as the KV of a new layer does.
// Build: hipcc --offload-arch=gfx950 -O3 tools/cu_bw.hip -o tools/cu_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) void stream_kernel(const f4* __restrict__ src,
                                                      long long per_wg_vec, float* out) {
  const f4* p = src + (long long)blockIdx.x * per_wg_vec;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int t = threadIdx.x;
  // 4 independent loads per thread per iteration (64 KB per workgroup iteration)
  for (long long i = t; i < per_wg_vec; i += 4 * 1024) {
    f4 a = p[i];
    f4 b = i + 1024 < per_wg_vec ? p[i + 1024] : f4{0.f, 0.f, 0.f, 0.f};
    f4 c = i + 2048 < per_wg_vec ? p[i + 2048] : f4{0.f, 0.f, 0.f, 0.f};
    f4 d = i + 3072 < per_wg_vec ? p[i + 3072] : f4{0.f, 0.f, 0.f, 0.f};
    acc += a + b + c + d;
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 123.456f) out[blockIdx.x * 1024 + t] = s;   // practically never: keeps loads live
}

__global__ void empty_kernel(float* out) {
  if (threadIdx.x == 4096) out[0] = 1.f;   // never (blockDim 1024)
}

int main() {
  const size_t buf_bytes = 2ull << 30;
  f4* buf;
  float* out;
  CHECK(hipMalloc(&buf, buf_bytes));
  CHECK(hipMalloc(&out, 256 * 1024 * sizeof(float)));
  CHECK(hipMemset(buf, 0, buf_bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 64;

  // launch floor: back-to-back empty kernels of one workgroup
  float ms = 0.f;
  for (int rep = 0; rep < 2; ++rep) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) empty_kernel<<<1, 1024>>>(out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
  }
  const double floor_us = ms * 1e3 / iters;
  std::printf("{\"empty_us\": %.2f}\n", floor_us);

  const int groups[] = {1, 2, 8, 16, 64, 256};
  const long long sizes_kb[] = {64, 256, 512, 1024, 2048};
  for (int g : groups) {
    for (long long kb : sizes_kb) {
      const long long bytes = kb * 1024;
      const long long per_wg_vec = bytes / 16;
      const long long launch_bytes = bytes * g;
      if (launch_bytes > (long long)(buf_bytes / 4)) continue;
      const long long windows = (long long)buf_bytes / launch_bytes;
      for (int rep = 0; rep < 2; ++rep) {
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) {
          const f4* src = buf + (long long)(i % windows) * (launch_bytes / 16);
          stream_kernel<<<g, 1024>>>(src, per_wg_vec, out);
        }
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
      }
      CHECK(hipGetLastError());
      const double us = ms * 1e3 / iters;
      const double body = us - floor_us > 0.05 ? us - floor_us : 0.05;
      std::printf(
          "{\"wgs\": %d, \"kb_per_wg\": %lld, \"us\": %.2f, \"us_above_empty\": %.2f, "
          "\"GBps_per_wg\": %.1f, \"GBps_total\": %.1f}\n",
          g, kb, us, body, bytes / body / 1e3, launch_bytes / body / 1e3);
      std::fflush(stdout);
    }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
