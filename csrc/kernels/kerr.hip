// Device error words of the in-launch hand-offs (stream-K slabs in gemm_w4.hip, the
// persistent decode layer's stage counters in decode_persist.hip).  Every cross-workgroup
// wait in those kernels is bounded in wall time; a wait that gives up adds 1 to its slot
// here instead of hanging the GPU, and the runner fails the step when a slot moved
// (engine/runner.py, like the custom all-reduce's error counter).
//
// The words live in mapped, coherent (fine-grained) pinned host memory: the kernels
// update them with system-scope atomics and the host reads them with a plain load after
// the step's token readback -- no extra device synchronisation per step.
#include <mutex>
#include <cstring>

#include "common.h"

namespace rfq {

static std::mutex g_kerr_mu;
static uint32_t* g_kerr_host = nullptr;
static uint32_t* g_kerr_dev = nullptr;

// nullptr while the stream is being captured and nothing was allocated yet (a kernel then
// reports nothing; the engine allocates the words at start-up, before any capture)
uint32_t* kernel_error_words(hipStream_t s) {
  if (g_kerr_dev != nullptr) return g_kerr_dev;
  std::lock_guard<std::mutex> lock(g_kerr_mu);
  if (g_kerr_dev != nullptr) return g_kerr_dev;
  if (s != nullptr) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone)
      return nullptr;
  }
  void* h = nullptr;
  if (hipHostMalloc(&h, kKernelErrorWords * 4, hipHostMallocMapped | hipHostMallocCoherent) !=
      hipSuccess)
    return nullptr;
  std::memset(h, 0, kKernelErrorWords * 4);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return nullptr;
  }
  g_kerr_host = static_cast<uint32_t*>(h);
  g_kerr_dev = static_cast<uint32_t*>(d);
  return g_kerr_dev;
}

uint32_t kernel_error_read(int slot) {
  if (g_kerr_host == nullptr || slot < 0 || slot >= kKernelErrorWords) return 0;
  return __atomic_load_n(g_kerr_host + slot, __ATOMIC_SEQ_CST);
}

}  // namespace rfq
