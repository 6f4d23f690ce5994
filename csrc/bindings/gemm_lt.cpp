// hipBLASLt with an explicit, start-up-measured algorithm per (M bucket, N, K).
//
// torch.matmul asks hipBLASLt's heuristic for ONE algorithm per call.  On gfx950 the
// heuristic's first choice is uneven across token counts (profiles/r1_gemm_m_sweep.md:
// the down projection at 0.91 PFLOP/s at M = 6656 vs 1.63 at M = 4096), so the engine
// times the heuristic's top candidates on the model's own weights at start-up
// (ops/autotune.py: tune_lt) and calls the winner directly through this file.
//
//   Y[M, N] = X[M, K] . W[N, K]^T  (bf16 in/out, fp32 accumulate), row-major, i.e. the
//   column-major problem D^T[N, M] = op(W)^T . X^T with transA = T, transB = N.
//
// Algorithms are kept in a process-wide table; Python refers to them by index.  A call
// whose algorithm rejects the actual shape returns a non-zero status and the caller
// falls back to torch.matmul (an algorithm tuned at the bucket's upper M is usually,
// not always, valid for the smaller M inside the bucket).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <mutex>
#include <vector>

namespace {

using at::Tensor;

struct LtState {
  hipblasLtHandle_t handle = nullptr;
  void* workspace = nullptr;
  size_t ws_bytes = 0;
  std::vector<hipblasLtMatmulAlgo_t> algos;
  std::mutex mu;
};

LtState& lt() {
  static LtState s;
  return s;
}

constexpr size_t kWorkspace = 64ull << 20;   // 64 MiB, allocated once per process

bool ensure_init() {
  LtState& s = lt();
  if (s.handle) return true;
  if (hipblasLtCreate(&s.handle) != HIPBLAS_STATUS_SUCCESS) return false;
  if (hipMalloc(&s.workspace, kWorkspace) != hipSuccess) return false;
  s.ws_bytes = kWorkspace;
  return true;
}

// RAII descriptors for one problem shape
struct Problem {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  bool ok = false;
  Problem(int64_t M, int64_t N, int64_t K, int64_t ldx, int64_t ldw, int64_t ldd) {
    if (hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
      return;
    const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    // A = W viewed column-major [K, N] (ld ldw), B = X^T column-major [K, M] (ld ldx),
    // D = Y^T column-major [N, M] (ld ldd)
    ok = hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, K, N, ldw) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, K, M, ldx) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutCreate(&d, HIP_R_16BF, N, M, ldd) == HIPBLAS_STATUS_SUCCESS;
  }
  ~Problem() {
    if (a) hipblasLtMatrixLayoutDestroy(a);
    if (b) hipblasLtMatrixLayoutDestroy(b);
    if (d) hipblasLtMatrixLayoutDestroy(d);
    if (op) hipblasLtMatmulDescDestroy(op);
  }
};

// Top `count` heuristic algorithms for Y[M, N] = X[M, K] W[N, K]^T (contiguous rows);
// returns their indices in the process-wide table (empty if hipBLASLt offers none).
std::vector<int64_t> lt_heuristic(int64_t M, int64_t N, int64_t K, int64_t count) {
  std::vector<int64_t> ids;
  if (!ensure_init() || count <= 0) return ids;
  LtState& s = lt();
  Problem p(M, N, K, K, K, N);
  if (!p.ok) return ids;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return ids;
  const uint64_t wsb = s.ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                        sizeof(wsb));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(count);
  int got = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(
      s.handle, p.op, p.a, p.b, p.d, p.d, pref, (int)count, res.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS) return ids;
  std::lock_guard<std::mutex> g(s.mu);
  for (int i = 0; i < got; ++i) {
    if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > s.ws_bytes) continue;
    ids.push_back((int64_t)s.algos.size());
    s.algos.push_back(res[i].algo);
  }
  return ids;
}

// out = x . w^T with table algorithm `algo`; returns the hipBLASLt status (0 = done).
int64_t lt_matmul(const Tensor& x, const Tensor& w, const Tensor& out, int64_t algo) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  out.scalar_type() == at::kBFloat16, "lt_matmul: bf16 GPU tensors");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 &&
                  w.stride(1) == 1 && out.stride(1) == 1, "lt_matmul: row-major 2-D tensors");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N, "lt_matmul: shapes");
  if (!ensure_init()) return -1;
  LtState& s = lt();
  const hipblasLtMatmulAlgo_t* a = nullptr;
  {
    std::lock_guard<std::mutex> g(s.mu);
    if (algo < 0 || algo >= (int64_t)s.algos.size()) return -2;
    a = &s.algos[algo];
  }
  Problem p(M, N, K, x.stride(0), w.stride(0), out.stride(0));
  if (!p.ok) return -3;
  const float alpha = 1.f, beta = 0.f;
  const hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const hipblasStatus_t r = hipblasLtMatmul(s.handle, p.op, &alpha, w.data_ptr(), p.a,
                                            x.data_ptr(), p.b, &beta, out.data_ptr(), p.d,
                                            out.data_ptr(), p.d, a, s.workspace, s.ws_bytes, st);
  return (int64_t)r;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(rfq_amd, m) {
  m.def("lt_heuristic(int M, int N, int K, int count) -> int[]", &lt_heuristic);
  m.def("lt_matmul(Tensor x, Tensor w, Tensor(a!) out, int algo) -> int");
}

TORCH_LIBRARY_IMPL(rfq_amd, CUDA, m) { m.impl("lt_matmul", &lt_matmul); }
