// torch op registrations for the gfx950 kernels (namespace torch.ops.rfq_amd).
//
// Every op launches on the caller's current HIP stream, allocates nothing and
// never synchronises, so whole decode steps can be captured into a hipGraph
// (torch.cuda.CUDAGraph on ROCm) — cdna_hip_programming.md Guideline 9.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstring>
#include <vector>
#include <algorithm>

namespace rfq {
typedef uint16_t bf16_t;
void launch_rms_norm(const bf16_t*, int64_t, const bf16_t*, bf16_t*, int64_t, int, int, float, hipStream_t);
void launch_fused_add_rms_norm(const bf16_t*, int64_t, bf16_t*, int64_t, const bf16_t*, bf16_t*,
                               int64_t, int, int, float, hipStream_t);
void launch_skinny_gemm(const bf16_t*, int64_t, const bf16_t*, int, int, int64_t, bf16_t*, int64_t,
                        int, int, hipStream_t);
void launch_skinny_gemm_norm(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t, int,
                             int, bf16_t*, int64_t, const bf16_t*, bf16_t*, int64_t, float,
                             unsigned*, float*, hipStream_t);
void launch_skinny_gemm_rope(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t, int,
                             int, const int32_t*, const float*, const int32_t*, bf16_t*, bf16_t*,
                             int, int, int, hipStream_t);
void launch_silu_mul(const bf16_t*, int64_t, bf16_t*, int64_t, int, int, hipStream_t);
void launch_count_nonfinite(const bf16_t*, int64_t, int, int, int32_t*, hipStream_t);
void launch_skinny_gemm_swiglu(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t,
                               int, int, hipStream_t);
void launch_gemv_splitk_plain(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t,
                              int, int, float*, unsigned*, hipStream_t);
void launch_gemv_splitk_norm(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t,
                             int, int, float*, unsigned*, bf16_t*, int64_t, const bf16_t*,
                             bf16_t*, int64_t, float, unsigned*, hipStream_t);
void launch_gemv_splitk_swiglu(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t,
                               int, int, float*, unsigned*, hipStream_t);
void launch_gemv_splitk_rope(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t, int,
                             int, float*, unsigned*, const int32_t*, const float*, const int32_t*,
                             bf16_t*, bf16_t*, int, int, int, hipStream_t);
void launch_gemv_rows(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t, int, int,
                      hipStream_t);
void launch_gemv_rows_swiglu(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t,
                             int, int, float, hipStream_t);
void launch_gemv_rows_rope(const bf16_t*, int64_t, const bf16_t*, int, int, bf16_t*, int64_t, int,
                           int, const int32_t*, const float*, const int32_t*, bf16_t*, bf16_t*, int,
                           int, int, float, hipStream_t);
void launch_attn_decode_reduce(const float*, const float*, bf16_t*, int64_t, int, int, int,
                               hipStream_t);
void launch_embed(const int32_t*, const bf16_t*, bf16_t*, int, int, int, int, hipStream_t);
void launch_rope_kv(bf16_t*, int64_t, const int32_t*, const float*, const int32_t*, bf16_t*,
                    bf16_t*, int, int, int, int, hipStream_t);
void launch_attn_decode(const bf16_t*, int64_t, const bf16_t*, const bf16_t*, const int32_t*, int,
                        const int32_t*, const int32_t*, const int32_t*, const int32_t*,
                        const int32_t*, int, int, bf16_t*, int64_t, float*, float*, int, int,
                        float, int, int, int32_t*, hipStream_t, bool);
void launch_attn_decode_shared(const bf16_t*, int64_t, const bf16_t*, const bf16_t*,
                               const int32_t*, int, const int32_t*, const int32_t*,
                               const int32_t*, int, const int32_t*, const int32_t*, int, int,
                               bf16_t*, int64_t, int32_t*, float*, float*, int, int, float, int,
                               bool, hipStream_t);
void launch_attn_prefill(const bf16_t*, int64_t, const bf16_t*, const bf16_t*, const int32_t*, int,
                         const int32_t*, const int32_t*, const int32_t*, const int32_t*,
                         const int32_t*, int, bf16_t*, int64_t, int, int, float, int, int,
                         float*, int32_t*, int, hipStream_t);
int prefill_split_ws_floats();
void set_attn_prefill_timing(uint64_t*);
int prefill_split_tickets();
void launch_sample_partial(const bf16_t*, int64_t, int, int, int, const uint32_t*, int,
                           const int32_t*, const float*, const uint64_t*, float*, int32_t*, int,
                           hipStream_t);
void launch_sample_final(const float*, const int32_t*, int, int, int, int32_t*, hipStream_t);
void launch_moe_topk(const bf16_t*, int64_t, int, int, int, float*, int32_t*, bool, hipStream_t);
void launch_moe_route(const bf16_t*, int64_t, const bf16_t*, int, int, int, int, float*, int32_t*,
                      bool, hipStream_t);
void launch_moe_align(const int32_t*, int, int, int, int32_t*, int32_t*, int32_t*, int32_t*,
                      int32_t*, int, int, hipStream_t);
void launch_moe_gather(const bf16_t*, int64_t, const int32_t*, int, int, int, bf16_t*, hipStream_t);
void launch_moe_gemm8(const bf16_t*, const bf16_t*, bf16_t*, const int32_t*, const int32_t*,
                      const int32_t*, int, int, int, int, int64_t, int, bool, int, hipStream_t);
void launch_moe_grouped_gemm(const bf16_t*, const bf16_t*, bf16_t*, const int32_t*, const int32_t*,
                             int, int, int, int, hipStream_t);
void launch_moe_combine(const bf16_t*, const int32_t*, const float*, int, int, int, bf16_t*,
                        int64_t, hipStream_t);
void launch_gemm_dense(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, int, int,
                       int, int, bool, int, hipStream_t);
void launch_gemm_grouped(const bf16_t*, const bf16_t*, bf16_t*, const int32_t*, int, int, int,
                         int, int64_t, bool, hipStream_t);
void launch_gemm_w4_grouped(const bf16_t*, const bf16_t*, bf16_t*, const int32_t*, int, int, int,
                            int, int64_t, bool, hipStream_t, float*, int, int);
void launch_moe_combine_w2(const bf16_t*, const float*, int64_t, const int32_t*, int, int, int,
                           const int32_t*, const float*, int, int, int, bf16_t*, int64_t,
                           hipStream_t);
int64_t car_signal_bytes();
uint32_t* kernel_error_words(hipStream_t);
int decode_persist_counter_words(int);
int decode_persist_lds_bytes(int, int, int);
int decode_persist_grid();
int decode_engine_layout(int, int, int, int, int, int, int*, int*, int*, int*);
void launch_decode_persist_op(const int64_t*, int, int, int, int, int, int, int, int, bf16_t*,
                              bf16_t*, int, bf16_t*, bf16_t*, const int32_t*, const float*,
                              const int32_t*, int, const int32_t*, int, const int32_t*,
                              const int32_t*, const int32_t*, const int32_t*, const int32_t*, int,
                              int, float*, float*, int32_t*, float, uint32_t*, float, int,
                              hipStream_t);
uint32_t kernel_error_read(int);
hipError_t car_alloc(int64_t, void**);
void launch_car_oneshot(char* const*, int, int, const bf16_t*, bf16_t*, int64_t, hipStream_t);
void launch_car_twoshot(char* const*, int, int, const bf16_t*, bf16_t*, int64_t, hipStream_t);
uint32_t car_read_error(const void*);
uint32_t car_read_info(const void*);
int car_norm_max_rows();
bool car_push_fits(int, int, int, int64_t);
void launch_car_push_add_norm(char* const*, int, int, const bf16_t*, bf16_t*, int64_t,
                              const bf16_t*, bf16_t*, int64_t, int, int, float, hipStream_t);
void launch_car_oneshot_add_norm(char* const*, int, int, const bf16_t*, bf16_t*, int64_t,
                                 const bf16_t*, bf16_t*, int64_t, int, int, float, hipStream_t);
void launch_moe_skinny(const bf16_t*, int64_t, const int32_t*, int, const int32_t*, const bf16_t*,
                       int, bf16_t*, int64_t, int, int, int, bool, bool, hipStream_t);
void launch_moe_skinny_splitk(const bf16_t*, int64_t, const int32_t*, int, const int32_t*,
                              const bf16_t*, int, float*, int64_t, int, int, int, int, hipStream_t);
void launch_moe_combine_splitk(const float*, int, int64_t, const int32_t*, const float*, int, int,
                               int, bf16_t*, int64_t, hipStream_t);
}  // namespace rfq

namespace {

using at::Tensor;

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_ROWMAJOR(t) TORCH_CHECK((t).dim() == 2 && (t).stride(1) == 1, #t " must be 2-D row-major")

inline const rfq::bf16_t* bp(const Tensor& t) {
  return reinterpret_cast<const rfq::bf16_t*>(t.data_ptr());
}
inline rfq::bf16_t* bpm(const Tensor& t) { return reinterpret_cast<rfq::bf16_t*>(t.data_ptr()); }

void rms_norm(const Tensor& x, const Tensor& w, double eps, const Tensor& out) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && d <= 16384 && w.numel() == d, "rms_norm: bad hidden size");
  rfq::launch_rms_norm(bp(x), x.stride(0), bp(w), bpm(out), out.stride(0), x.size(0), d,
                       (float)eps, cur_stream());
}

void fused_add_rms_norm(const Tensor& x, const Tensor& residual, const Tensor& w, double eps,
                        const Tensor& out) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(residual); CHECK_ROWMAJOR(out);
  const int d = x.size(1);
  TORCH_CHECK(d % 8 == 0 && d <= 16384 && w.numel() == d && residual.size(1) == d,
              "fused_add_rms_norm: bad hidden size");
  TORCH_CHECK(residual.size(0) == x.size(0) && out.size(0) == x.size(0), "row mismatch");
  rfq::launch_fused_add_rms_norm(bp(x), x.stride(0), bpm(residual), residual.stride(0), bp(w),
                                 bpm(out), out.stride(0), x.size(0), d, (float)eps, cur_stream());
}

// out[M, N] = x[M, K] . w[N, K]^T for M <= 64 (weight-streaming latency path)
void skinny_gemm(const Tensor& x, const Tensor& w, const Tensor& out, int64_t cfg) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0,
              "skinny_gemm: w must be row-major [N, K] with 16-byte aligned rows");
  const bool gated = cfg & 16;          // x = [M, 2K] gate|up, B operand silu(gate)*up
  const int M = x.size(0), K = gated ? x.size(1) / 2 : x.size(1), N = w.size(0);
  const int nt = (cfg & 1) ? 2 : 1;  // bits 2-3 select the load variant
  TORCH_CHECK(!gated || x.size(1) == 2 * K, "skinny_gemm: gated x must be [M, 2K]");
  TORCH_CHECK(M >= 1 && M <= 64, "skinny_gemm: M must be in [1, 64]");
  TORCH_CHECK(w.size(1) == K && K % 128 == 0 && N % (16 * nt) == 0,
              "skinny_gemm: K % 128 and N % tile required");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "skinny_gemm: out shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 4 == 0, "skinny_gemm: alignment");
  TORCH_CHECK(w.stride(0) >= K, "skinny_gemm: w row stride < K");
  rfq::launch_skinny_gemm(bp(x), x.stride(0), bp(w), N, K, w.stride(0), bpm(out), out.stride(0), M,
                          (int)cfg, cur_stream());
}

// y = x . w^T (skinny, M <= 16), then residual <- y + residual and
// out <- rmsnorm(residual) * norm_w in the grid's last workgroup (= skinny_gemm followed
// by fused_add_rms_norm(y, residual, norm_w, eps, out)).  counter: int32 [>= 1], zero,
// owned by the stream (the kernel leaves it at zero).
void skinny_gemm_norm(const Tensor& x, const Tensor& w, const Tensor& y, const Tensor& residual,
                      const Tensor& norm_w, double eps, const Tensor& out, const Tensor& counter,
                      const Tensor& partials, int64_t cfg) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_BF16(residual);
  CHECK_BF16(norm_w); CHECK_BF16(out); CHECK_I32(counter);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(y); CHECK_ROWMAJOR(residual); CHECK_ROWMAJOR(out);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "skinny_gemm_norm: w must be contiguous [N, K]");
  const bool gated = cfg & 16;
  const int M = x.size(0), K = gated ? x.size(1) / 2 : x.size(1), N = w.size(0);
  const int nt = (cfg & 1) ? 2 : 1;
  const int threads = (cfg & 2) ? 512 : 256;
  TORCH_CHECK(!gated || x.size(1) == 2 * K, "skinny_gemm_norm: gated x must be [M, 2K]");
  TORCH_CHECK(M >= 1 && M <= 16, "skinny_gemm_norm: M must be in [1, 16]");
  TORCH_CHECK(w.size(1) == K && K % 128 == 0 && N % (16 * nt) == 0 && N % 8 == 0 &&
                  N / 8 <= 4 * threads,
              "skinny_gemm_norm: K % 128, N % tile and N <= 32 * threads required");
  TORCH_CHECK(y.size(0) == M && y.size(1) == N && residual.size(0) == M &&
                  residual.size(1) == N && out.size(0) == M && out.size(1) == N &&
                  norm_w.numel() == N,
              "skinny_gemm_norm: shapes");
  TORCH_CHECK(x.stride(0) % 8 == 0 && y.stride(0) % 8 == 0 && residual.stride(0) % 8 == 0 &&
                  out.stride(0) % 8 == 0,
              "skinny_gemm_norm: alignment");
  TORCH_CHECK(counter.is_cuda() && counter.numel() >= 1, "skinny_gemm_norm: counter");
  TORCH_CHECK(!(cfg & 64) || (partials.is_cuda() && partials.scalar_type() == at::kFloat &&
                              partials.numel() >= 2 * (int64_t)M * N),
              "skinny_gemm_norm: split-K needs an fp32 partials workspace of 2*M*N");
  rfq::launch_skinny_gemm_norm(bp(x), x.stride(0), bp(w), N, K, bpm(y), y.stride(0), M, (int)cfg,
                               bpm(residual), residual.stride(0), bp(norm_w), bpm(out),
                               out.stride(0), (float)eps,
                               reinterpret_cast<unsigned*>(counter.data_ptr()),
                               (cfg & 64) ? partials.data_ptr<float>() : nullptr, cur_stream());
}

// out[M, F] = silu(x . Wg^T) * (x . Wu^T), w = [Wg; Wu] [2F, K] (M <= 16): the gate|up
// projection with the SwiGLU in its epilogue (= skinny_gemm then silu_mul).
void skinny_gemm_swiglu(const Tensor& x, const Tensor& w, const Tensor& out, int64_t cfg) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "skinny_gemm_swiglu: w must be contiguous [2F, K]");
  const int M = x.size(0), K = x.size(1), F = w.size(0) / 2;
  TORCH_CHECK(M >= 1 && M <= 16, "skinny_gemm_swiglu: M must be in [1, 16]");
  TORCH_CHECK(w.size(0) == 2 * F && w.size(1) == K && K % 128 == 0 && F % 16 == 0,
              "skinny_gemm_swiglu: w [2F, K] with K % 128 == 0, F % 16 == 0");
  TORCH_CHECK(out.size(0) == M && out.size(1) == F, "skinny_gemm_swiglu: out [M, F]");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 4 == 0, "skinny_gemm_swiglu: alignment");
  rfq::launch_skinny_gemm_swiglu(bp(x), x.stride(0), bp(w), F, K, bpm(out), out.stride(0), M,
                                 (int)cfg, cur_stream());
}

// y_cols: the output's column count (N, or F = N/2 for the SwiGLU epilogue);
// tiles: output tiles = ticket counters the launch uses
static void check_splitk(const char* what, const Tensor& x, const Tensor& w, const Tensor& y,
                         const Tensor& part, const Tensor& tile_cnt, int64_t cfg,
                         int64_t y_cols = -1, int64_t tiles = -1) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_I32(tile_cnt);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(y);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), what, ": w must be contiguous [N, K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0), KS = 2 << (cfg & 3);
  if (y_cols < 0) y_cols = N;
  if (tiles < 0) tiles = N / 16;
  TORCH_CHECK(M >= 1 && M <= 16, what, ": M must be in [1, 16]");
  TORCH_CHECK(w.size(1) == K && K % 128 == 0 && N % 16 == 0 && (K / 128) >= KS, what,
              ": K % 128 == 0, N % 16 == 0 and K / 128 >= KS required");
  TORCH_CHECK(y.size(0) == M && y.size(1) == y_cols, what, ": y shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && y.stride(0) % 4 == 0, what, ": alignment");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.numel() >= KS * M * N,
              what, ": fp32 partials workspace of KS*M*N floats");
  TORCH_CHECK(tile_cnt.is_cuda() && tile_cnt.numel() >= tiles, what, ": one counter per tile");
}

// out[M, F] = silu(x Wg^T) * (x Wu^T) for w = [Wg; Wu] [2F, K], split K (M <= 16)
void gemv_splitk_swiglu(const Tensor& x, const Tensor& w, const Tensor& out, const Tensor& part,
                        const Tensor& tile_cnt, int64_t cfg) {
  const int64_t F = w.size(0) / 2;
  TORCH_CHECK(F % 16 == 0 && w.size(0) == 2 * F, "gemv_splitk_swiglu: w [2F, K], F % 16 == 0");
  check_splitk("gemv_splitk_swiglu", x, w, out, part, tile_cnt, cfg, F, F / 16);
  rfq::launch_gemv_splitk_swiglu(bp(x), x.stride(0), bp(w), (int)F, x.size(1), bpm(out),
                                 out.stride(0), x.size(0), (int)cfg, part.data_ptr<float>(),
                                 reinterpret_cast<unsigned*>(tile_cnt.data_ptr()), cur_stream());
}

// qkv = x w^T with NeoX RoPE on q / k and the paged KV append, split K (M <= 16);
// only qkv's q columns are written (= gemv_splitk + rope_kv)
void gemv_splitk_rope(const Tensor& x, const Tensor& w, const Tensor& qkv, const Tensor& positions,
                      const Tensor& cos_sin, const Tensor& slot_mapping, const Tensor& k_cache,
                      const Tensor& v_cache, int64_t Hq, int64_t Hkv, const Tensor& part,
                      const Tensor& tile_cnt, int64_t cfg) {
  const int64_t N = w.size(0);
  check_splitk("gemv_splitk_rope", x, w, qkv, part, tile_cnt, cfg, N, N / 32);
  CHECK_BF16(k_cache); CHECK_BF16(v_cache); CHECK_I32(positions); CHECK_I32(slot_mapping);
  TORCH_CHECK(N == (Hq + 2 * Hkv) * 128, "gemv_splitk_rope: w must be [(Hq + 2 Hkv) * 128, K]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
                  cos_sin.size(1) == 128,
              "gemv_splitk_rope: cos_sin must be fp32 [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == 128 &&
                  k_cache.is_contiguous() && v_cache.is_contiguous() &&
                  v_cache.sizes() == k_cache.sizes(),
              "gemv_splitk_rope: cache must be [blocks, Hkv, BS, 128]");
  TORCH_CHECK(positions.numel() >= x.size(0) && slot_mapping.numel() >= x.size(0),
              "gemv_splitk_rope: metadata");
  rfq::launch_gemv_splitk_rope(bp(x), x.stride(0), bp(w), (int)N, x.size(1), bpm(qkv),
                               qkv.stride(0), x.size(0), (int)cfg, part.data_ptr<float>(),
                               reinterpret_cast<unsigned*>(tile_cnt.data_ptr()),
                               positions.data_ptr<int32_t>(), cos_sin.data_ptr<float>(),
                               slot_mapping.data_ptr<int32_t>(), bpm(k_cache), bpm(v_cache),
                               (int)Hq, (int)Hkv, k_cache.size(2), cur_stream());
}

// Row-streaming GEMV (gemv_rows.hip) for M <= 4: one wave per weight row (or RW rows),
// full K, no workspace.  cfg bits [1:0] RW = 1 << b (plain only), [3:2] CU = 2 << b.
static void check_rows(const char* what, const Tensor& x, const Tensor& w, const Tensor& y,
                       int64_t cfg, int64_t y_cols) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(y);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), what, ": w must be contiguous [N, K]");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 4, what, ": M must be in [1, 4]");
  TORCH_CHECK(w.size(1) == K && K % 512 == 0, what, ": K % 512 == 0 required");
  TORCH_CHECK(w.numel() < ((int64_t)1 << 40), what, ": weight too large");
  TORCH_CHECK(y.size(0) == M && y.size(1) == y_cols, what, ": y shape");
  TORCH_CHECK(x.stride(0) % 8 == 0, what, ": x rows must be 16-byte aligned");
  TORCH_CHECK(cfg >= 0 && cfg < 128, what, ": cfg");
}

// cfg bit 5: y is the residual stream, y <- bf16(x . w^T) + y (residual add)
void gemv_rows(const Tensor& x, const Tensor& w, const Tensor& y, int64_t cfg) {
  check_rows("gemv_rows", x, w, y, cfg, w.size(0));
  TORCH_CHECK(!(cfg & 80), "gemv_rows: cfg bits 4 / 6 (normalised x, pair per wave) are for "
              "the SwiGLU / RoPE forms");
  rfq::launch_gemv_rows(bp(x), x.stride(0), bp(w), w.size(0), x.size(1), bpm(y), y.stride(0),
                        x.size(0), (int)cfg, cur_stream());
}

// cfg bit 4: x is the un-normalised residual, w carries the RMSNorm weight folded in
// (rows scaled by rsqrt(mean(x^2) + eps) in the kernel)
void gemv_rows_swiglu(const Tensor& x, const Tensor& w, const Tensor& out, int64_t cfg,
                      double eps) {
  const int64_t F = w.size(0) / 2;
  TORCH_CHECK(w.size(0) == 2 * F, "gemv_rows_swiglu: w [2F, K]");
  check_rows("gemv_rows_swiglu", x, w, out, cfg, F);
  TORCH_CHECK(!(cfg & 32), "gemv_rows_swiglu: cfg bit 5 (residual add) is for the plain form");
  rfq::launch_gemv_rows_swiglu(bp(x), x.stride(0), bp(w), (int)F, x.size(1), bpm(out),
                               out.stride(0), x.size(0), (int)cfg, (float)eps, cur_stream());
}

void gemv_rows_rope(const Tensor& x, const Tensor& w, const Tensor& qkv, const Tensor& positions,
                    const Tensor& cos_sin, const Tensor& slot_mapping, const Tensor& k_cache,
                    const Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t cfg, double eps) {
  const int64_t N = w.size(0);
  check_rows("gemv_rows_rope", x, w, qkv, cfg, N);
  TORCH_CHECK(!(cfg & 32), "gemv_rows_rope: cfg bit 5 (residual add) is for the plain form");
  CHECK_BF16(k_cache); CHECK_BF16(v_cache); CHECK_I32(positions); CHECK_I32(slot_mapping);
  TORCH_CHECK(N == (Hq + 2 * Hkv) * 128, "gemv_rows_rope: w must be [(Hq + 2 Hkv) * 128, K]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
                  cos_sin.size(1) == 128,
              "gemv_rows_rope: cos_sin must be fp32 [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == 128 &&
                  k_cache.is_contiguous() && v_cache.is_contiguous() &&
                  v_cache.sizes() == k_cache.sizes(),
              "gemv_rows_rope: cache must be [blocks, Hkv, BS, 128]");
  TORCH_CHECK(positions.numel() >= x.size(0) && slot_mapping.numel() >= x.size(0),
              "gemv_rows_rope: metadata");
  rfq::launch_gemv_rows_rope(bp(x), x.stride(0), bp(w), (int)N, x.size(1), bpm(qkv),
                             qkv.stride(0), x.size(0), (int)cfg, positions.data_ptr<int32_t>(),
                             cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int32_t>(),
                             bpm(k_cache), bpm(v_cache), (int)Hq, (int)Hkv, k_cache.size(2),
                             (float)eps, cur_stream());
}

// Merge split-K decode-attention partials into bf16 rows (attn_decode_reduce).
void attn_decode_merge(const Tensor& part_o, const Tensor& part_ml, const Tensor& out, int64_t Hq,
                       int64_t num_splits) {
  CHECK_DEV(out); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  const int rows = out.size(0);
  TORCH_CHECK(num_splits >= 1 && num_splits <= 32, "attn_decode_merge: num_splits in [1, 32]");
  TORCH_CHECK(part_o.scalar_type() == at::kFloat && part_ml.scalar_type() == at::kFloat &&
                  part_o.numel() >= (int64_t)rows * Hq * num_splits * 128 &&
                  part_ml.numel() >= (int64_t)rows * Hq * num_splits * 2,
              "attn_decode_merge: fp32 partial buffers too small");
  TORCH_CHECK(out.size(1) >= Hq * 128, "attn_decode_merge: out [rows, >= Hq * 128]");
  rfq::launch_attn_decode_reduce(part_o.data_ptr<float>(), part_ml.data_ptr<float>(), bpm(out),
                                 out.stride(0), rows, (int)Hq, (int)num_splits, cur_stream());
}

// Diagnostics: while `buf` is set (int64, >= 8 words per workgroup), every attn_prefill
// launch stamps each workgroup's phases (s_memrealtime, 100 MHz) into it; an empty
// tensor clears it.
void attn_prefill_timing(const Tensor& buf) {
  CHECK_DEV(buf);
  TORCH_CHECK(buf.scalar_type() == at::kLong && buf.is_contiguous(),
              "attn_prefill_timing: int64 buffer");
  rfq::set_attn_prefill_timing(
      buf.numel() > 0 ? reinterpret_cast<uint64_t*>(buf.data_ptr()) : nullptr);
}

// y = x . w^T, split-K over (N/16) x KS workgroups with the in-launch per-tile
// reduction (M <= 16).  tile_cnt: int32 [>= N/16], zero, left at zero.
void gemv_splitk(const Tensor& x, const Tensor& w, const Tensor& y, const Tensor& part,
                 const Tensor& tile_cnt, int64_t cfg) {
  check_splitk("gemv_splitk", x, w, y, part, tile_cnt, cfg);
  rfq::launch_gemv_splitk_plain(bp(x), x.stride(0), bp(w), w.size(0), x.size(1), bpm(y),
                                y.stride(0), x.size(0), (int)cfg, part.data_ptr<float>(),
                                reinterpret_cast<unsigned*>(tile_cnt.data_ptr()), cur_stream());
}

// gemv_splitk followed, in the same launch, by residual <- y + residual and
// out <- rmsnorm(residual) * norm_w (= fused_add_rms_norm).
void gemv_splitk_norm(const Tensor& x, const Tensor& w, const Tensor& y, const Tensor& residual,
                      const Tensor& norm_w, double eps, const Tensor& out, const Tensor& counter,
                      const Tensor& part, const Tensor& tile_cnt, int64_t cfg) {
  check_splitk("gemv_splitk_norm", x, w, y, part, tile_cnt, cfg);
  CHECK_BF16(residual); CHECK_BF16(norm_w); CHECK_BF16(out); CHECK_I32(counter);
  CHECK_ROWMAJOR(residual); CHECK_ROWMAJOR(out);
  const int64_t M = x.size(0), N = w.size(0);
  const int threads = (cfg & 4) ? 512 : 256;
  TORCH_CHECK(N % 8 == 0 && N / 8 <= 4 * threads, "gemv_splitk_norm: N <= 32 * threads");
  TORCH_CHECK(residual.size(0) == M && residual.size(1) == N && out.size(0) == M &&
                  out.size(1) == N && norm_w.numel() == N,
              "gemv_splitk_norm: shapes");
  TORCH_CHECK(y.stride(0) % 8 == 0 && residual.stride(0) % 8 == 0 && out.stride(0) % 8 == 0,
              "gemv_splitk_norm: alignment");
  TORCH_CHECK(counter.is_cuda() && counter.numel() >= 1, "gemv_splitk_norm: counter");
  rfq::launch_gemv_splitk_norm(bp(x), x.stride(0), bp(w), N, x.size(1), bpm(y), y.stride(0), M,
                               (int)cfg, part.data_ptr<float>(),
                               reinterpret_cast<unsigned*>(tile_cnt.data_ptr()), bpm(residual),
                               residual.stride(0), bp(norm_w), bpm(out), out.stride(0),
                               (float)eps, reinterpret_cast<unsigned*>(counter.data_ptr()),
                               cur_stream());
}

// qkv = x . w^T (skinny, M <= 16) with NeoX RoPE on q/k and the paged KV append in the
// epilogue (= skinny_gemm followed by rope_kv); only qkv's q columns are written.
void skinny_gemm_rope(const Tensor& x, const Tensor& w, const Tensor& qkv, const Tensor& positions,
                      const Tensor& cos_sin, const Tensor& slot_mapping, const Tensor& k_cache,
                      const Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t cfg) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(qkv); CHECK_BF16(k_cache);
  CHECK_BF16(v_cache); CHECK_I32(positions); CHECK_I32(slot_mapping);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(qkv);
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "skinny_gemm_rope: w must be contiguous [N, K]");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 16, "skinny_gemm_rope: M must be in [1, 16]");
  TORCH_CHECK((cfg & 1) && !(cfg & 16), "skinny_gemm_rope: cfg must select NT = 2, plain x");
  TORCH_CHECK(w.size(1) == K && K % 128 == 0 && N == (Hq + 2 * Hkv) * 128,
              "skinny_gemm_rope: w must be [(Hq + 2 Hkv) * 128, K], K % 128 == 0");
  TORCH_CHECK(qkv.size(0) == M && qkv.size(1) == N && qkv.stride(0) % 4 == 0 &&
                  x.stride(0) % 8 == 0,
              "skinny_gemm_rope: qkv shape / alignment");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
                  cos_sin.size(1) == 128,
              "skinny_gemm_rope: cos_sin must be fp32 [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == 128 &&
                  k_cache.is_contiguous() && v_cache.is_contiguous() &&
                  v_cache.sizes() == k_cache.sizes(),
              "skinny_gemm_rope: cache must be [blocks, Hkv, BS, 128]");
  TORCH_CHECK(positions.numel() >= M && slot_mapping.numel() >= M, "skinny_gemm_rope: metadata");
  rfq::launch_skinny_gemm_rope(bp(x), x.stride(0), bp(w), N, K, bpm(qkv), qkv.stride(0), M,
                               (int)cfg, positions.data_ptr<int32_t>(), cos_sin.data_ptr<float>(),
                               slot_mapping.data_ptr<int32_t>(), bpm(k_cache), bpm(v_cache),
                               (int)Hq, (int)Hkv, k_cache.size(2), cur_stream());
}

// counter[0] += number of Inf / NaN entries of the bf16 matrix x (rows x cols, row stride)
void count_nonfinite(const Tensor& x, const Tensor& counter) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x); CHECK_I32(counter);
  TORCH_CHECK(x.dim() == 2 && x.stride(0) % 8 == 0, "count_nonfinite: 2-D, 16-byte aligned rows");
  rfq::launch_count_nonfinite(bp(x), x.stride(0), x.size(0), x.size(1),
                              counter.data_ptr<int32_t>(), cur_stream());
}

void silu_mul(const Tensor& gate_up, const Tensor& out) {
  CHECK_DEV(gate_up); CHECK_BF16(gate_up); CHECK_BF16(out);
  CHECK_ROWMAJOR(gate_up); CHECK_ROWMAJOR(out);
  const int F = out.size(1);
  TORCH_CHECK(gate_up.size(1) == 2 * F && F % 8 == 0 && out.size(0) == gate_up.size(0),
              "silu_mul: shape mismatch");
  rfq::launch_silu_mul(bp(gate_up), gate_up.stride(0), bpm(out), out.stride(0), out.size(0), F,
                       cur_stream());
}

void embed(const Tensor& ids, const Tensor& table, const Tensor& out, int64_t vocab_start) {
  CHECK_DEV(ids); CHECK_I32(ids); CHECK_BF16(table); CHECK_BF16(out);
  TORCH_CHECK(table.is_contiguous() && out.is_contiguous(), "embed: contiguous tensors required");
  const int d = table.size(1);
  TORCH_CHECK(out.size(1) == d && out.size(0) == ids.numel() && d % 8 == 0, "embed: shape");
  rfq::launch_embed(ids.data_ptr<int32_t>(), bp(table), bpm(out), ids.numel(), d,
                    (int)vocab_start, (int)(vocab_start + table.size(0)), cur_stream());
}

void rope_kv(const Tensor& qkv, const Tensor& positions, const Tensor& cos_sin,
             const Tensor& slot_mapping, const Tensor& k_cache, const Tensor& v_cache,
             int64_t Hq, int64_t Hkv) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_ROWMAJOR(qkv);
  CHECK_I32(positions); CHECK_I32(slot_mapping); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.size(1) == 128,
              "rope_kv: cos_sin must be fp32 [max_pos, 128]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == 128 &&
                  k_cache.is_contiguous() && v_cache.is_contiguous(),
              "rope_kv: cache must be [blocks, Hkv, BS, 128]");
  const int T = qkv.size(0);
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * 128 && positions.numel() >= T &&
                  slot_mapping.numel() >= T,
              "rope_kv: shape mismatch");
  rfq::launch_rope_kv(bpm(qkv), qkv.stride(0), positions.data_ptr<int32_t>(),
                      cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int32_t>(), bpm(k_cache),
                      bpm(v_cache), T, Hq, Hkv, k_cache.size(2), cur_stream());
}

// Paged decode / short-extend attention.  Rows of q/out [rows, *] belong to
// sequences described by (seq_q_start, seq_q_len, seq_kv_len, block_tables);
// work items (work_seq, work_ct) = (sequence, 16-column tile of q_len*G columns),
// work_seq = -1 marks padding.
void attn_decode(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache,
                 const Tensor& block_tables, const Tensor& seq_q_start, const Tensor& seq_q_len,
                 const Tensor& seq_kv_len, const Tensor& work_seq, const Tensor& work_ct,
                 const Tensor& out, const Tensor& part_o, const Tensor& part_ml, int64_t Hq,
                 int64_t Hkv, double scale, int64_t num_splits, int64_t tiles_per_item,
                 const std::optional<Tensor>& tickets, bool reduce) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_ROWMAJOR(q); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(tiles_per_item == 1 || tiles_per_item == 2, "attn_decode: tiles_per_item in {1, 2}");
  CHECK_I32(block_tables); CHECK_ROWMAJOR(block_tables);
  CHECK_I32(seq_q_start); CHECK_I32(seq_q_len); CHECK_I32(seq_kv_len);
  CHECK_I32(work_seq); CHECK_I32(work_ct);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 32 && k_cache.size(3) == 128 &&
                  k_cache.size(1) == Hkv,
              "attn_decode: cache must be [blocks, Hkv, 32, 128]");
  TORCH_CHECK(Hq % Hkv == 0 && Hq / Hkv <= 16, "attn_decode: GQA group must be <= 16");
  const int rows = out.size(0);
  TORCH_CHECK(q.size(0) >= rows, "attn_decode: q has fewer rows than out");
  TORCH_CHECK(work_seq.numel() == work_ct.numel(), "work list mismatch");
  TORCH_CHECK(block_tables.size(0) >= seq_q_len.numel() && seq_kv_len.numel() >= seq_q_len.numel()
                  && seq_q_start.numel() >= seq_q_len.numel(),
              "attn_decode: per-sequence arrays mismatch");
  TORCH_CHECK(num_splits >= 1 && num_splits <= 32, "attn_decode: num_splits in [1, 32]");
  if (num_splits > 1) {
    TORCH_CHECK(part_o.scalar_type() == at::kFloat && part_ml.scalar_type() == at::kFloat,
                "partials must be fp32");
    TORCH_CHECK(part_o.numel() >= (int64_t)rows * Hq * num_splits * 128 &&
                    part_ml.numel() >= (int64_t)rows * Hq * num_splits * 2,
                "attn_decode: partial buffers too small");
  }
  TORCH_CHECK(reduce || !tickets.has_value(),
              "attn_decode: reduce=False leaves the partials to the consumer (no tickets)");
  int32_t* tk = nullptr;
  if (tickets.has_value() && num_splits > 1) {
    // zero-initialised once by the caller; the merging wave resets its entry
    CHECK_DEV(*tickets); CHECK_I32(*tickets);
    TORCH_CHECK(tickets->numel() >= work_seq.numel() * Hkv, "attn_decode: ticket buffer too small");
    TORCH_CHECK(num_splits <= 16, "attn_decode: the in-kernel merge takes at most 16 splits");
    tk = tickets->data_ptr<int32_t>();
  }
  rfq::launch_attn_decode(bp(q), q.stride(0), bp(k_cache), bp(v_cache),
                          block_tables.data_ptr<int32_t>(), block_tables.stride(0),
                          seq_q_start.data_ptr<int32_t>(), seq_q_len.data_ptr<int32_t>(),
                          seq_kv_len.data_ptr<int32_t>(), work_seq.data_ptr<int32_t>(),
                          work_ct.data_ptr<int32_t>(), work_seq.numel(), rows, bpm(out),
                          out.stride(0), num_splits > 1 ? part_o.data_ptr<float>() : nullptr,
                          num_splits > 1 ? part_ml.data_ptr<float>() : nullptr, Hq, Hkv,
                          (float)scale, num_splits, tiles_per_item, tk, cur_stream(), reduce);
}

// Shared-prefix (cascade) decode attention, num_splits == 1; see attn_decode.hip.
// ws_i32 >= 2 + nseq + rows int32; pre_o >= rows*Hq*128, pre_ml >= rows*Hq*2 fp32.
void attn_decode_shared(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache,
                        const Tensor& block_tables, const Tensor& seq_q_start,
                        const Tensor& seq_q_len, const Tensor& seq_kv_len, const Tensor& work_seq,
                        const Tensor& work_ct, const Tensor& out, const Tensor& ws_i32,
                        const Tensor& pre_o, const Tensor& pre_ml, int64_t Hq, int64_t Hkv,
                        double scale, int64_t tiles_per_item, bool run_meta) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_ROWMAJOR(q); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(tiles_per_item == 1 || tiles_per_item == 2, "attn_decode_shared: tiles_per_item");
  CHECK_I32(block_tables); CHECK_ROWMAJOR(block_tables);
  CHECK_I32(seq_q_start); CHECK_I32(seq_q_len); CHECK_I32(seq_kv_len);
  CHECK_I32(work_seq); CHECK_I32(work_ct); CHECK_I32(ws_i32);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 32 && k_cache.size(3) == 128 &&
                  k_cache.size(1) == Hkv,
              "attn_decode_shared: cache must be [blocks, Hkv, 32, 128]");
  TORCH_CHECK(Hq % Hkv == 0 && Hq / Hkv <= 16, "attn_decode_shared: GQA group must be <= 16");
  const int rows = out.size(0);
  const int nseq = seq_q_len.numel();
  TORCH_CHECK(q.size(0) >= rows, "attn_decode_shared: q has fewer rows than out");
  TORCH_CHECK(work_seq.numel() == work_ct.numel(), "work list mismatch");
  TORCH_CHECK(block_tables.size(0) >= nseq && seq_kv_len.numel() >= nseq &&
                  seq_q_start.numel() >= nseq,
              "attn_decode_shared: per-sequence arrays mismatch");
  TORCH_CHECK(ws_i32.numel() >= 2 + nseq + rows, "attn_decode_shared: int32 workspace too small");
  TORCH_CHECK(pre_o.scalar_type() == at::kFloat && pre_ml.scalar_type() == at::kFloat &&
                  pre_o.numel() >= (int64_t)rows * Hq * 128 &&
                  pre_ml.numel() >= (int64_t)rows * Hq * 2,
              "attn_decode_shared: prefix partial buffers too small / not fp32");
  rfq::launch_attn_decode_shared(
      bp(q), q.stride(0), bp(k_cache), bp(v_cache), block_tables.data_ptr<int32_t>(),
      block_tables.stride(0), seq_q_start.data_ptr<int32_t>(), seq_q_len.data_ptr<int32_t>(),
      seq_kv_len.data_ptr<int32_t>(), nseq, work_seq.data_ptr<int32_t>(),
      work_ct.data_ptr<int32_t>(), work_seq.numel(), rows, bpm(out), out.stride(0),
      ws_i32.data_ptr<int32_t>(), pre_o.data_ptr<float>(), pre_ml.data_ptr<float>(), Hq, Hkv,
      (float)scale, tiles_per_item, run_meta, cur_stream());
}

void attn_prefill(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache,
                  const Tensor& block_tables, const Tensor& seq_q_start, const Tensor& seq_q_len,
                  const Tensor& seq_kv_len, const Tensor& work_seq, const Tensor& work_qblk,
                  const Tensor& out, int64_t Hq, int64_t Hkv, double scale, int64_t qblk,
                  int64_t hsplit_below, const std::optional<Tensor>& ws,
                  const std::optional<Tensor>& tickets, int64_t small_mode) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_ROWMAJOR(q); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  CHECK_I32(block_tables); CHECK_ROWMAJOR(block_tables);
  CHECK_I32(seq_q_start); CHECK_I32(seq_q_len); CHECK_I32(seq_kv_len);
  CHECK_I32(work_seq); CHECK_I32(work_qblk);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 32 && k_cache.size(3) == 128 &&
                  k_cache.size(1) == Hkv,
              "attn_prefill: cache must be [blocks, Hkv, 32, 128]");
  TORCH_CHECK(Hq % Hkv == 0 && (Hq / Hkv) % 4 == 0, "attn_prefill: GQA group must be a multiple of 4");
  TORCH_CHECK(work_seq.numel() == work_qblk.numel(), "work list mismatch");
  const int64_t nw = qblk * (Hq / Hkv) / 32;
  TORCH_CHECK((qblk == 32 || qblk == 64) && (nw == 4 || nw == 8),
              "attn_prefill: qblk * (Hq / Hkv) must be 128 or 256 (4 or 8 waves)");
  TORCH_CHECK(small_mode >= 0 && small_mode <= 3, "attn_prefill: small_mode must be 0-3");
  float* split_ws = nullptr;
  int32_t* split_tk = nullptr;
  if (ws.has_value() && tickets.has_value()) {
    CHECK_DEV(*ws); CHECK_DEV(*tickets); CHECK_I32(*tickets);
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= rfq::prefill_split_ws_floats() &&
                    tickets->numel() >= rfq::prefill_split_tickets(),
                "attn_prefill: split-KV workspace too small (ops.prefill_split_ws)");
    split_ws = ws->data_ptr<float>();
    split_tk = tickets->data_ptr<int32_t>();
  }
  rfq::launch_attn_prefill(bp(q), q.stride(0), bp(k_cache), bp(v_cache),
                           block_tables.data_ptr<int32_t>(), block_tables.stride(0),
                           seq_q_start.data_ptr<int32_t>(), seq_q_len.data_ptr<int32_t>(),
                           seq_kv_len.data_ptr<int32_t>(), work_seq.data_ptr<int32_t>(),
                           work_qblk.data_ptr<int32_t>(), work_seq.numel(), bpm(out),
                           out.stride(0), Hq, Hkv, (float)scale, (int)qblk, (int)hsplit_below,
                           split_ws, split_tk, (int)small_mode, cur_stream());
}

// sizes of the split-KV prefill workspace: (fp32 floats, int32 zeroed tickets)
std::vector<int64_t> prefill_split_ws_sizes() {
  return {rfq::prefill_split_ws_floats(), rfq::prefill_split_tickets()};
}

void sample_partial(const Tensor& logits, int64_t v0, const Tensor& mask_table,
                    const Tensor& mask_idx, const Tensor& temps, const Tensor& seeds,
                    const Tensor& part_val, const Tensor& part_idx) {
  CHECK_DEV(logits); CHECK_BF16(logits); CHECK_ROWMAJOR(logits);
  TORCH_CHECK(mask_table.scalar_type() == at::kInt && mask_table.dim() == 2 &&
                  mask_table.is_contiguous(),
              "mask_table must be int32 [n_masks, words]");
  CHECK_I32(mask_idx);
  TORCH_CHECK(temps.scalar_type() == at::kFloat, "temps must be fp32");
  TORCH_CHECK(seeds.scalar_type() == at::kLong, "seeds must be int64");
  TORCH_CHECK(part_val.dim() == 2 && part_idx.dim() == 2, "partials must be [B, splits]");
  const int B = part_val.size(0), nsplit = part_val.size(1);
  const int Vl = logits.size(1);
  TORCH_CHECK(Vl % 8 == 0 && v0 % 8 == 0, "vocab shard must be 8-aligned");
  TORCH_CHECK(logits.size(0) >= B && mask_idx.numel() >= B && temps.numel() >= B &&
                  seeds.numel() >= B,
              "sample_partial: batch mismatch");
  TORCH_CHECK((v0 + Vl + 31) / 32 <= mask_table.size(1), "mask table too narrow");
  rfq::launch_sample_partial(bp(logits), logits.stride(0), B, Vl, v0,
                             reinterpret_cast<const uint32_t*>(mask_table.data_ptr<int32_t>()),
                             mask_table.size(1), mask_idx.data_ptr<int32_t>(),
                             temps.data_ptr<float>(),
                             reinterpret_cast<const uint64_t*>(seeds.data_ptr<int64_t>()),
                             part_val.data_ptr<float>(), part_idx.data_ptr<int32_t>(), nsplit,
                             cur_stream());
}

// part_val/part_idx: [groups, B, n] (groups = TP ranks after all-gather, or 1)
void sample_final(const Tensor& part_val, const Tensor& part_idx, const Tensor& out) {
  CHECK_DEV(part_val); CHECK_I32(part_idx); CHECK_I32(out);
  TORCH_CHECK(part_val.dim() == 3 && part_val.is_contiguous() && part_idx.is_contiguous(),
              "partials must be contiguous [groups, B, n]");
  const int groups = part_val.size(0), B = part_val.size(1), n = part_val.size(2);
  TORCH_CHECK(out.numel() >= B, "out too small");
  rfq::launch_sample_final(part_val.data_ptr<float>(), part_idx.data_ptr<int32_t>(), B, n, groups,
                           out.data_ptr<int32_t>(), cur_stream());
}

void moe_topk(const Tensor& router_logits, int64_t topk, bool renorm, const Tensor& weights,
              const Tensor& ids) {
  CHECK_DEV(router_logits); CHECK_BF16(router_logits); CHECK_ROWMAJOR(router_logits);
  TORCH_CHECK(weights.scalar_type() == at::kFloat && ids.scalar_type() == at::kInt, "topk outputs");
  const int T = router_logits.size(0), E = router_logits.size(1);
  TORCH_CHECK(E <= 64 && topk <= 8, "moe_topk: E <= 64, k <= 8");
  rfq::launch_moe_topk(bp(router_logits), router_logits.stride(0), T, E, topk,
                       weights.data_ptr<float>(), ids.data_ptr<int32_t>(), renorm, cur_stream());
}

// router logits (x . router^T) + softmax top-k in one launch, one workgroup per token
void moe_route(const Tensor& x, const Tensor& router, int64_t topk, bool renorm,
               const Tensor& weights, const Tensor& ids) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(router); CHECK_ROWMAJOR(x);
  CHECK_I32(ids);
  TORCH_CHECK(router.dim() == 2 && router.is_contiguous() && router.size(1) == x.size(1),
              "moe_route: router must be contiguous [E, d]");
  const int T = x.size(0), d = x.size(1), E = router.size(0);
  TORCH_CHECK(E <= 16 && topk >= 1 && topk <= 8 && topk <= E && d % 8 == 0 &&
                  x.stride(0) % 8 == 0,
              "moe_route: E <= 16, topk <= 8, d % 8 == 0");
  TORCH_CHECK(weights.scalar_type() == at::kFloat && weights.numel() >= (int64_t)T * topk &&
                  ids.numel() >= (int64_t)T * topk,
              "moe_route: outputs");
  rfq::launch_moe_route(bp(x), x.stride(0), bp(router), T, d, E, (int)topk,
                        weights.data_ptr<float>(), ids.data_ptr<int32_t>(), renorm, cur_stream());
}

// Sort (token, k) pairs by expert, pad each expert's segment to a multiple of
// `block_m`.  Outputs: sorted_ids [max_padded] (token*k+slot, or -1 padding),
// expert_of_block [max_blocks], expert_offsets [E+1], num_blocks [1].
// Per-expert weight-streaming GEMM for small token counts (gemm_skinny.hip).
void moe_skinny(const Tensor& x, const Tensor& sorted_ids, int64_t topk,
                const Tensor& expert_offsets, const Tensor& w, const Tensor& out, bool gated,
                bool gather, int64_t max_rows) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(out); CHECK_I32(sorted_ids); CHECK_I32(expert_offsets);
  TORCH_CHECK(w.dim() == 3 && w.is_contiguous(), "moe_skinny: w must be [E, N, K] contiguous");
  const int E = w.size(0), K = w.size(2);
  const int n_out = out.size(1);
  TORCH_CHECK(x.size(1) == K && K % 128 == 0, "moe_skinny: K mismatch or K % 128 != 0");
  TORCH_CHECK(w.size(1) == (gated ? 2 : 1) * n_out && n_out % 16 == 0, "moe_skinny: N mismatch");
  TORCH_CHECK(expert_offsets.numel() >= E + 1, "moe_skinny: expert_offsets too small");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 4 == 0, "moe_skinny: alignment");
  TORCH_CHECK(out.size(0) >= sorted_ids.numel() || !gather, "moe_skinny: out rows < sorted rows");
  rfq::launch_moe_skinny(bp(x), x.stride(0), sorted_ids.data_ptr<int32_t>(), (int)topk,
                         expert_offsets.data_ptr<int32_t>(), bp(w), K, bpm(out), out.stride(0), E,
                         n_out, (int)max_rows, gated, gather, cur_stream());
}

// w2 of the MoE latency path with split-K: yf [splits, rows, n_out] fp32 partials
void moe_skinny_splitk(const Tensor& x, const Tensor& sorted_ids, int64_t topk,
                       const Tensor& expert_offsets, const Tensor& w, const Tensor& yf,
                       int64_t max_rows, int64_t splits) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x); CHECK_BF16(w); CHECK_I32(sorted_ids);
  CHECK_I32(expert_offsets);
  TORCH_CHECK(w.dim() == 3 && w.is_contiguous(), "moe_skinny_splitk: w must be [E, N, K]");
  TORCH_CHECK(yf.scalar_type() == at::kFloat && yf.dim() == 3 && yf.is_contiguous(),
              "moe_skinny_splitk: yf must be fp32 [splits, rows, N] contiguous");
  TORCH_CHECK(splits == 2 || splits == 4, "moe_skinny_splitk: splits in {2, 4}");
  const int E = w.size(0), K = w.size(2), n_out = w.size(1);
  TORCH_CHECK(x.size(1) == K && K % 128 == 0 && n_out % 16 == 0, "moe_skinny_splitk: shapes");
  TORCH_CHECK(yf.size(0) >= splits && yf.size(2) == n_out && yf.size(1) >= sorted_ids.numel() &&
                  x.size(0) >= sorted_ids.numel() && x.stride(0) % 8 == 0,
              "moe_skinny_splitk: rows / alignment");
  TORCH_CHECK(expert_offsets.numel() >= E + 1, "moe_skinny_splitk: expert_offsets too small");
  rfq::launch_moe_skinny_splitk(bp(x), x.stride(0), sorted_ids.data_ptr<int32_t>(), (int)topk,
                                expert_offsets.data_ptr<int32_t>(), bp(w), K,
                                yf.data_ptr<float>(), yf.stride(0), E, n_out, (int)max_rows,
                                (int)splits, cur_stream());
}

void moe_combine_splitk(const Tensor& yf, int64_t splits, const Tensor& inv_pos,
                        const Tensor& weights, int64_t topk, const Tensor& out) {
  CHECK_DEV(yf); CHECK_I32(inv_pos); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(yf.scalar_type() == at::kFloat && yf.dim() == 3 && yf.is_contiguous() &&
                  yf.size(0) >= splits && yf.size(2) == out.size(1) && out.size(1) % 8 == 0,
              "moe_combine_splitk: yf must be fp32 [splits, rows, d]");
  TORCH_CHECK(weights.scalar_type() == at::kFloat, "weights fp32");
  const int T = out.size(0), d = out.size(1);
  rfq::launch_moe_combine_splitk(yf.data_ptr<float>(), (int)splits, yf.stride(0),
                                 inv_pos.data_ptr<int32_t>(), weights.data_ptr<float>(), T,
                                 (int)topk, d, bpm(out), out.stride(0), cur_stream());
}

// ---- custom all-reduce (csrc/comm/custom_ar.hip)
int64_t car_alloc_op(int64_t data_bytes) {
  void* p = nullptr;
  TORCH_CHECK(rfq::car_alloc(data_bytes, &p) == hipSuccess, "car_alloc: hipExtMallocWithFlags failed");
  return reinterpret_cast<int64_t>(p);
}

void car_free_op(int64_t ptr) { (void)hipFree(reinterpret_cast<void*>(ptr)); }

Tensor car_ipc_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  TORCH_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)) == hipSuccess,
              "hipIpcGetMemHandle failed");
  Tensor t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

int64_t car_ipc_open(const Tensor& handle) {
  TORCH_CHECK(handle.numel() == (int64_t)sizeof(hipIpcMemHandle_t) && !handle.is_cuda(),
              "car_ipc_open: expects the 64-byte CPU handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data_ptr(), sizeof(h));
  void* p = nullptr;
  TORCH_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess,
              "hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

void car_ipc_close(int64_t ptr) { (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)); }

int64_t car_data_offset() { return rfq::car_signal_bytes(); }

// Persistent decode layers (decode_persist.hip): [counter words, LDS bytes, grid] for a
// launch of nst stages at M tokens, hidden d and widest stage input Kx.
std::vector<int64_t> decode_persist_info(int64_t M, int64_t d, int64_t Kx, int64_t nst) {
  return {(int64_t)rfq::decode_persist_counter_words((int)nst),
          (int64_t)rfq::decode_persist_lds_bytes((int)M, (int)d, (int)Kx),
          (int64_t)rfq::decode_persist_grid()};
}

// Engine form's LDS bytes and ring slots for (M, d, Hq, Hkv, F) on this device: [bytes, slots]
// (bytes 0: does not fit)
std::vector<int64_t> decode_engine_info(int64_t M, int64_t d, int64_t Hq, int64_t Hkv, int64_t F) {
  int r = 0, p, a, o;
  const int b = rfq::decode_engine_layout((int)M, (int)d, (int)Hq, (int)Hkv, (int)F,
                                          rfq::decode_persist_grid(), &r, &p, &a, &o);
  return {(int64_t)b, (int64_t)r};
}

void decode_persist(const Tensor& residual, const Tensor& layers, const Tensor& qbuf,
                    const Tensor& attn, const Tensor& act, const Tensor& positions,
                    const Tensor& cos_sin, const Tensor& slots, const Tensor& block_tables,
                    const Tensor& q_start, const Tensor& q_len, const Tensor& kv_len,
                    const Tensor& work_seq, const Tensor& work_ct, const Tensor& part_o,
                    const Tensor& part_ml, const Tensor& tickets, const Tensor& counters,
                    int64_t l0, int64_t l1, int64_t stages, int64_t Hq, int64_t Hkv, int64_t F,
                    int64_t BS, int64_t splits, double scale, double eps, int64_t flags) {
  CHECK_DEV(residual); CHECK_BF16(residual); CHECK_BF16(qbuf); CHECK_BF16(attn); CHECK_BF16(act);
  CHECK_I32(positions); CHECK_I32(slots); CHECK_I32(block_tables); CHECK_I32(q_start);
  CHECK_I32(q_len); CHECK_I32(kv_len); CHECK_I32(work_seq); CHECK_I32(work_ct);
  CHECK_I32(tickets); CHECK_I32(counters);
  TORCH_CHECK(residual.is_contiguous() && residual.dim() == 2, "decode_persist: residual [M, d]");
  const int64_t M = residual.size(0), d = residual.size(1);
  TORCH_CHECK(M >= 1 && M <= 4, "decode_persist: 1 <= M <= 4 tokens");
  TORCH_CHECK(d % 512 == 0 && (Hq * 128) % 512 == 0 && F % 512 == 0,
              "decode_persist: d, Hq * 128 and F must be multiples of 512");
  TORCH_CHECK(Hkv >= 1 && Hq % Hkv == 0 && Hq / Hkv <= 16, "decode_persist: GQA group <= 16");
  TORCH_CHECK(layers.scalar_type() == at::kLong && layers.is_cuda() && layers.dim() == 2 &&
              layers.size(1) == 8 && layers.is_contiguous(), "decode_persist: layers [L, 8] int64");
  TORCH_CHECK(0 <= l0 && l0 < l1 && l1 <= layers.size(0), "decode_persist: layer range");
  TORCH_CHECK(stages > 0 && stages < 32, "decode_persist: stage mask in [1, 31]");
  TORCH_CHECK(qbuf.dim() == 2 && qbuf.stride(1) == 1 && qbuf.size(0) >= M &&
              qbuf.size(1) >= Hq * 128, "decode_persist: qbuf [M, >= Hq * 128]");
  TORCH_CHECK(attn.is_contiguous() && attn.size(0) >= M && attn.size(1) == Hq * 128,
              "decode_persist: attn [M, Hq * 128]");
  TORCH_CHECK(act.is_contiguous() && act.size(0) >= M && act.size(1) == F, "decode_persist: act [M, F]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == 128,
              "decode_persist: cos_sin fp32 [max_pos, 128]");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M, "decode_persist: positions / slots");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.stride(1) == 1, "decode_persist: block tables");
  const int64_t W = work_seq.numel();
  TORCH_CHECK(work_ct.numel() == W && W >= 1, "decode_persist: work list");
  TORCH_CHECK(splits >= 1 && splits <= 16, "decode_persist: 1 <= splits <= 16");
  if (splits > 1) {
    TORCH_CHECK(part_o.numel() >= M * Hq * splits * 128 && part_ml.numel() >= M * Hq * splits * 2,
                "decode_persist: split partial buffers too small");
    TORCH_CHECK(tickets.numel() >= W * Hkv, "decode_persist: ticket buffer too small");
  }
  int nper = 0;
  for (int i = 0; i < 5; ++i) nper += (stages >> i) & 1;
  const int64_t nst = (l1 - l0) * nper;
  TORCH_CHECK(counters.numel() >= rfq::decode_persist_counter_words((int)nst),
              "decode_persist: counter buffer too small");
  const int64_t Kx = std::max<int64_t>(Hq * 128, F);
  TORCH_CHECK(!(flags & 256) || ((flags & 16) && splits > 1 && part_ml.numel() >= 1024),
              "decode_persist: the timeline stamps (flags bit 8) need the engine form and a "
              "split partial buffer of >= 1024 floats (they are written there)");
  if (flags & 16) {
    // engine form: M <= 2, a row spans at most 3 ring slots, >= 5 slots fit next to the rows
    int r, p, a, o;
    TORCH_CHECK(M <= 2, "decode_persist engine: M <= 2 tokens");
    TORCH_CHECK(std::max<int64_t>(d, Kx) / 512 <= 33, "decode_persist engine: K / 512 <= 33");
    TORCH_CHECK(rfq::decode_engine_layout((int)M, (int)d, (int)Hq, (int)Hkv, (int)F,
                                          rfq::decode_persist_grid(), &r, &p, &a, &o) > 0,
                "decode_persist engine: the rows leave fewer than 5 ring slots in LDS");
  }
  TORCH_CHECK(rfq::decode_persist_lds_bytes((int)M, (int)d, (int)Kx) <= 160 * 1024,
              "decode_persist: the step's rows do not fit in LDS (M * (d + max(Hq*128, F)))");
  rfq::launch_decode_persist_op(
      reinterpret_cast<const int64_t*>(layers.data_ptr()), (int)l0, (int)l1, (int)stages, (int)M,
      (int)d, (int)Hq, (int)Hkv, (int)F, bpm(residual), bpm(qbuf), (int)qbuf.stride(0), bpm(attn),
      bpm(act), positions.data_ptr<int32_t>(), cos_sin.data_ptr<float>(), slots.data_ptr<int32_t>(),
      (int)BS, block_tables.data_ptr<int32_t>(), (int)block_tables.stride(0),
      q_start.data_ptr<int32_t>(), q_len.data_ptr<int32_t>(), kv_len.data_ptr<int32_t>(),
      work_seq.data_ptr<int32_t>(), work_ct.data_ptr<int32_t>(), (int)W, (int)splits,
      splits > 1 ? part_o.data_ptr<float>() : nullptr,
      splits > 1 ? part_ml.data_ptr<float>() : nullptr, tickets.data_ptr<int32_t>(), (float)scale,
      reinterpret_cast<uint32_t*>(counters.data_ptr<int32_t>()), (float)eps, (int)flags,
      cur_stream());
}

// Error words of the bounded in-launch waits (csrc/kernels/kerr.hip): allocated by the
// first call (the engine calls it at start-up, before any graph capture); returns the
// slots' counts (all 0 when no GPU / nothing allocated).
std::vector<int64_t> kernel_errors() {
  (void)rfq::kernel_error_words(nullptr);
  std::vector<int64_t> out;
  for (int i = 0; i < 3; ++i) out.push_back((int64_t)rfq::kernel_error_read(i));
  return out;
}

int64_t car_error_info(int64_t ptr) {
  return (int64_t)rfq::car_read_info(reinterpret_cast<const void*>(ptr));
}

int64_t car_error(int64_t ptr) {
  return (int64_t)rfq::car_read_error(reinterpret_cast<const void*>(ptr));
}

// algo: 0 = auto (two-shot above 512 KiB on > 2 ranks), 1 = one-shot, 2 = two-shot
void car_allreduce(const Tensor& inp, const Tensor& out, c10::IntArrayRef bases, int64_t rank,
                   int64_t capacity_bytes, int64_t algo) {
  CHECK_DEV(inp); CHECK_BF16(inp); CHECK_BF16(out);
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.numel() == out.numel(),
              "car_allreduce: contiguous tensors of equal size required");
  TORCH_CHECK(inp.numel() % 8 == 0, "car_allreduce: numel % 8 != 0");
  TORCH_CHECK(inp.numel() * 2 <= capacity_bytes, "car_allreduce: message exceeds the buffer");
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "car_allreduce: world");
  char* b[8];
  for (int i = 0; i < world; ++i) b[i] = reinterpret_cast<char*>(bases[i]);
  const bool two = algo == 2 || (algo == 0 && world > 2 && inp.numel() * 2 > (512 << 10));
  if (two)
    rfq::launch_car_twoshot(b, (int)rank, world, bp(inp), bpm(out), inp.numel(), cur_stream());
  else
    rfq::launch_car_oneshot(b, (int)rank, world, bp(inp), bpm(out), inp.numel(), cur_stream());
}

// residual <- bf16(allreduce(inp) + residual); out <- rmsnorm(residual) * w, one launch
// (custom_ar.hip).  inp: contiguous [rows, d] bf16.  algo: 0 = push form when the
// double-buffered per-rank slots fit (rows <= 16), else staged; 1 = staged one-shot
// (car_oneshot_add_norm_kernel); 2 = push (car_push_add_norm_kernel).
void car_allreduce_add_norm(const Tensor& inp, const Tensor& residual, const Tensor& w,
                            double eps, const Tensor& out, c10::IntArrayRef bases, int64_t rank,
                            int64_t capacity_bytes, int64_t algo) {
  CHECK_DEV(inp); CHECK_BF16(inp); CHECK_BF16(residual); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(inp.dim() == 2 && inp.is_contiguous(), "car_allreduce_add_norm: inp [rows, d]");
  const int64_t rows = inp.size(0), d = inp.size(1);
  TORCH_CHECK(residual.dim() == 2 && out.dim() == 2 && residual.size(0) == rows &&
                  out.size(0) == rows && residual.size(1) == d && out.size(1) == d &&
                  residual.stride(1) == 1 && out.stride(1) == 1 && w.numel() == d &&
                  w.is_contiguous(),
              "car_allreduce_add_norm: residual/out [rows, d] with unit column stride, w [d]");
  TORCH_CHECK(d % 8 == 0 && d <= 16384 && residual.stride(0) % 8 == 0 && out.stride(0) % 8 == 0,
              "car_allreduce_add_norm: d % 8 == 0, d <= 16384, 16-byte aligned rows");
  TORCH_CHECK(rows >= 1 && rows <= rfq::car_norm_max_rows(), "car_allreduce_add_norm: rows");
  for (const Tensor* t : {&inp, &residual, &w, &out})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "car_allreduce_add_norm: 16-byte aligned tensors required");
  TORCH_CHECK(rows * d * 2 <= capacity_bytes, "car_allreduce_add_norm: message exceeds the buffer");
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "car_allreduce_add_norm: world");
  char* b[8];
  for (int i = 0; i < world; ++i) b[i] = reinterpret_cast<char*>(bases[i]);
  const bool push_ok = rfq::car_push_fits(world, (int)rows, (int)d, capacity_bytes);
  TORCH_CHECK(algo != 2 || push_ok, "car_allreduce_add_norm: push slots exceed the buffer");
  if (algo == 2 || (algo == 0 && push_ok && rows <= 16))
    rfq::launch_car_push_add_norm(b, (int)rank, world, bp(inp), bpm(residual), residual.stride(0),
                                  bp(w), bpm(out), out.stride(0), (int)rows, (int)d, (float)eps,
                                  cur_stream());
  else
    rfq::launch_car_oneshot_add_norm(b, (int)rank, world, bp(inp), bpm(residual),
                                     residual.stride(0), bp(w), bpm(out), out.stride(0), (int)rows,
                                     (int)d, (float)eps, cur_stream());
}

void moe_align(const Tensor& topk_ids, int64_t E, int64_t block_m, const Tensor& sorted_ids,
               const Tensor& inv_pos, const Tensor& expert_of_block,
               const Tensor& expert_offsets, const Tensor& num_blocks) {
  CHECK_DEV(topk_ids); CHECK_I32(topk_ids); CHECK_I32(sorted_ids); CHECK_I32(expert_of_block);
  CHECK_I32(expert_offsets); CHECK_I32(num_blocks); CHECK_I32(inv_pos);
  TORCH_CHECK(E <= 64 && expert_offsets.numel() >= E + 1, "moe_align: E <= 64");
  TORCH_CHECK(inv_pos.numel() >= topk_ids.numel(), "moe_align: inv_pos too small");
  const int64_t need = topk_ids.numel() + E * (block_m - 1);
  TORCH_CHECK(sorted_ids.numel() >= need && expert_of_block.numel() * block_m >= need,
              "moe_align: output buffers too small");
  rfq::launch_moe_align(topk_ids.data_ptr<int32_t>(), topk_ids.numel(), E, block_m,
                        sorted_ids.data_ptr<int32_t>(), inv_pos.data_ptr<int32_t>(),
                        expert_of_block.data_ptr<int32_t>(), expert_offsets.data_ptr<int32_t>(),
                        num_blocks.data_ptr<int32_t>(), sorted_ids.numel(),
                        expert_of_block.numel(), cur_stream());
}

void moe_gather(const Tensor& x, const Tensor& sorted_ids, int64_t topk, const Tensor& out) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x); CHECK_I32(sorted_ids); CHECK_BF16(out);
  TORCH_CHECK(out.is_contiguous() && out.size(0) >= sorted_ids.numel() && out.size(1) == x.size(1),
              "moe_gather: out shape");
  rfq::launch_moe_gather(bp(x), x.stride(0), sorted_ids.data_ptr<int32_t>(), sorted_ids.numel(),
                         x.size(1), topk, bpm(out), cur_stream());
}

// out[rows, N] = x[rows, K] @ w[e]^T for row blocks of 128 owned by expert e.
void moe_grouped_gemm(const Tensor& x, const Tensor& w, const Tensor& out,
                      const Tensor& expert_of_block, const Tensor& num_blocks) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(w.dim() == 3, "w must be [E, N, K]");
  const int E = w.size(0), N = w.size(1), K = w.size(2);
  TORCH_CHECK(x.size(1) == K && out.size(1) == N && out.size(0) == x.size(0), "moe gemm shape");
  TORCH_CHECK(K % 64 == 0 && N % 128 == 0, "moe gemm: K % 64, N % 128");
  TORCH_CHECK(x.size(0) % 128 == 0, "moe gemm: rows must be padded to 128");
  rfq::launch_moe_grouped_gemm(bp(x), bp(w), bpm(out), expert_of_block.data_ptr<int32_t>(),
                               num_blocks.data_ptr<int32_t>(), x.size(0) / 128, N, K, E,
                               cur_stream());
}

// 8-wave 128x256 grouped GEMM (moe.hip moe_gemm8_kernel).  swiglu: w = [E, 2F, K]
// (gate | up), out = [rows, F] = silu(x Wg^T) * (x Wu^T); else out = [rows, N] = x W^T.
void moe_gemm8(const Tensor& x, const Tensor& w, const Tensor& out,
               const Tensor& expert_of_block, const Tensor& num_blocks,
               const Tensor& expert_offsets, bool swiglu, int64_t tile) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(w.dim() == 3, "w must be [E, N, K]");
  const int E = w.size(0), N = w.size(1), K = w.size(2);
  const int n_out = swiglu ? N / 2 : N;
  TORCH_CHECK(x.size(1) == K && out.size(1) == n_out && out.size(0) == x.size(0),
              "moe gemm8 shape");
  TORCH_CHECK(K % 64 == 0 && (swiglu ? (N % 2 == 0 && n_out % 128 == 0) : N % 256 == 0),
              "moe gemm8: K % 64, N % 256 (F % 128 with swiglu)");
  TORCH_CHECK(x.size(0) % 128 == 0, "moe gemm8: rows must be padded to 128");
  TORCH_CHECK(expert_of_block.numel() >= x.size(0) / 128, "expert_of_block too short");
  TORCH_CHECK(expert_offsets.numel() >= E + 1, "expert_offsets too short");
  TORCH_CHECK(tile == 128 || tile == 256, "moe gemm8: tile rows 128 or 256");
  rfq::launch_moe_gemm8(bp(x), bp(w), bpm(out), expert_of_block.data_ptr<int32_t>(),
                        num_blocks.data_ptr<int32_t>(), expert_offsets.data_ptr<int32_t>(),
                        x.size(0) / 128, n_out, K, E, N, n_out, swiglu, (int)tile, cur_stream());
}

// Dense large-M GEMM (gemm_dense.hip): out[M, N] = x[M, K] . w[N, K]^T, or with swiglu
// (w = [Wg; Wu] [2F, K]) out[M, F] = silu(x Wg^T) * (x Wu^T).
void gemm_dense(const Tensor& x, const Tensor& w, const Tensor& out, bool swiglu, int64_t cfg) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1, "gemm_dense: w must be row-major [N, K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  const int64_t n_out = swiglu ? N / 2 : N;
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && K >= 64, "gemm_dense: w [N, K], K % 64 == 0");
  TORCH_CHECK(!(cfg & 4) || (K % 128 == 0 && w.size(0) % 16 == 0 && w.is_contiguous()),
              "gemm_dense: the decode-tiled weight layout (cfg bit 2) needs K % 128 == 0");
  TORCH_CHECK(!(cfg & 8) || (K % 128 == 0 && !(cfg & 4)),
              "gemm_dense: the one-wave-per-SIMD kernel (cfg bit 3) needs K % 128 == 0 and a "
              "row-major weight");
  TORCH_CHECK(swiglu ? (N % 256 == 0) : (N % 256 == 0),
              "gemm_dense: N % 256 == 0 (2F with F % 128 == 0 for swiglu)");
  TORCH_CHECK(out.size(0) == M && out.size(1) == n_out, "gemm_dense: out shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && out.stride(0) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0,
              "gemm_dense: 16-byte aligned operand rows");
  TORCH_CHECK(x.stride(0) * 256 < (int64_t)INT32_MAX && N * w.stride(0) < (int64_t)INT32_MAX,
              "gemm_dense: operand offsets exceed int32");
  // gemm_w4 / gemm_w4p (cfg bit 3) address W, X and out through buffer resources with
  // 32-bit BYTE offsets: a weight over 2 GiB (e.g. a 152064 x 8192 LM head) would wrap
  TORCH_CHECK(!(cfg & 8) || (N * w.stride(0) * 2 < (int64_t)INT32_MAX &&
                             M * x.stride(0) * 2 < (int64_t)INT32_MAX &&
                             M * out.stride(0) * 2 < (int64_t)INT32_MAX),
              "gemm_dense: cfg bit 3 (gemm_w4) needs every operand under 2 GiB");
  rfq::launch_gemm_dense(bp(x), x.stride(0), bp(w), w.stride(0), bpm(out), out.stride(0), (int)M,
                         (int)n_out, (int)K, (int)n_out, swiglu, (int)cfg, cur_stream());
}

// Grouped MoE GEMM on the dense kernel's structure (gemm_dense.hip GROUPED): x = the
// expert-sorted rows padded to 128 per expert, w [E, N, K], expert_offsets [E+1] (device).
// cfg bit 3: the one-wave-per-SIMD gemm_w4 structure (gemm_w4.hip GROUPED, K % 128),
// else gemm_dense's 8-wave ping-pong
void moe_gemm_dense(const Tensor& x, const Tensor& w, const Tensor& out,
                    const Tensor& expert_offsets, bool swiglu, int64_t cfg) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_I32(expert_offsets);
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(w.dim() == 3, "w must be [E, N, K]");
  const int E = w.size(0), N = w.size(1), K = w.size(2);
  const int n_out = swiglu ? N / 2 : N;
  TORCH_CHECK(x.size(1) == K && out.size(1) == n_out && out.size(0) == x.size(0),
              "moe_gemm_dense shape");
  TORCH_CHECK(K % 64 == 0 && (swiglu ? n_out % 128 == 0 : N % 256 == 0),
              "moe_gemm_dense: K % 64, N % 256 (F % 128 with swiglu)");
  TORCH_CHECK(x.size(0) % 128 == 0, "moe_gemm_dense: rows must be padded to 128");
  TORCH_CHECK(expert_offsets.numel() >= E + 1, "expert_offsets too short");
  TORCH_CHECK((int64_t)x.size(0) * K < (int64_t)INT32_MAX && (int64_t)N * K < (int64_t)INT32_MAX,
              "moe_gemm_dense: offsets exceed int32");
  TORCH_CHECK(!(cfg & 8) || K % 128 == 0, "moe_gemm_dense: the gemm_w4 form needs K % 128");
  if (cfg & 8)
    rfq::launch_gemm_w4_grouped(bp(x), bp(w), bpm(out), expert_offsets.data_ptr<int32_t>(),
                                x.size(0) / 128, n_out, K, E, N, swiglu, cur_stream(), nullptr, 0, 0);
  else
    rfq::launch_gemm_grouped(bp(x), bp(w), bpm(out), expert_offsets.data_ptr<int32_t>(),
                             x.size(0) / 128, n_out, K, E, N, swiglu, cur_stream());
}

// Throughput-path w2 + top-k combine (gemm_w4.hip GROUPED KS = 2, moe.hip
// moe_combine_w2_kernel): both kernels decide on the device, from the expert offsets and
// `cus`, whether the GEMM runs two K slices into yf (fp32 [2, >= rows, N]) or one into y
// (bf16 [rows, N]); the combine reads whichever was written.  cus <= 0: never split.
void moe_w2_combine(const Tensor& x, const Tensor& w, const Tensor& y, const Tensor& yf,
                    const Tensor& expert_offsets, const Tensor& inv_pos, const Tensor& weights,
                    int64_t topk, const Tensor& out, int64_t cus) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); CHECK_I32(expert_offsets);
  CHECK_I32(inv_pos); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && y.is_contiguous() && yf.is_contiguous(),
              "contiguous");
  TORCH_CHECK(w.dim() == 3, "w must be [E, N, K]");
  const int E = w.size(0), N = w.size(1), K = w.size(2);
  TORCH_CHECK(x.size(1) == K && x.size(0) % 128 == 0, "moe_w2_combine: x [rows % 128, K]");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == N, "moe_w2_combine: y [rows, N]");
  TORCH_CHECK(yf.scalar_type() == at::kFloat && yf.dim() == 3 && yf.size(0) == 2 &&
                  yf.size(1) >= x.size(0) && yf.size(2) == N,
              "moe_w2_combine: yf must be fp32 [2, >= rows, N]");
  TORCH_CHECK(N % 256 == 0 && K % 256 == 0 && K >= 512,
              "moe_w2_combine: N % 256, K % 256 (each K slice % 128), K >= 512");
  TORCH_CHECK(out.size(1) == N && weights.scalar_type() == at::kFloat &&
                  weights.size(0) == out.size(0) && weights.size(1) == topk &&
                  inv_pos.numel() >= out.size(0) * topk,
              "moe_w2_combine: out [T, N], weights fp32 [T, topk], inv_pos [T * topk]");
  TORCH_CHECK(expert_offsets.numel() >= E + 1, "expert_offsets too short");
  TORCH_CHECK((int64_t)x.size(0) * K < (int64_t)INT32_MAX && (int64_t)N * K < (int64_t)INT32_MAX,
              "moe_w2_combine: offsets exceed int32");
  const int tiles_n = N / 256;
  rfq::launch_gemm_w4_grouped(bp(x), bp(w), bpm(y), expert_offsets.data_ptr<int32_t>(),
                              x.size(0) / 128, N, K, E, N, false, cur_stream(),
                              yf.data_ptr<float>(), (int)yf.size(1), (int)cus);
  rfq::launch_moe_combine_w2(bp(y), yf.data_ptr<float>(), yf.stride(0),
                             expert_offsets.data_ptr<int32_t>(), E, tiles_n, (int)cus,
                             inv_pos.data_ptr<int32_t>(), weights.data_ptr<float>(),
                             out.size(0), (int)topk, N, bpm(out), out.stride(0), cur_stream());
}

// out[t] = sum_k weights[t,k] * y[pos of (t,k)]
void moe_combine(const Tensor& y, const Tensor& inv_pos, const Tensor& weights, int64_t topk,
                 const Tensor& out) {
  CHECK_DEV(y); CHECK_BF16(y); CHECK_I32(inv_pos); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(weights.scalar_type() == at::kFloat, "weights fp32");
  const int T = out.size(0), d = out.size(1);
  rfq::launch_moe_combine(bp(y), inv_pos.data_ptr<int32_t>(), weights.data_ptr<float>(), T,
                          topk, d, bpm(out), out.stride(0), cur_stream());
}

}  // namespace

TORCH_LIBRARY(rfq_amd, m) {
  m.def("rms_norm(Tensor x, Tensor w, float eps, Tensor(a!) out) -> ()");
  m.def("fused_add_rms_norm(Tensor x, Tensor(a!) residual, Tensor w, float eps, Tensor(b!) out) -> ()");
  m.def("silu_mul(Tensor gate_up, Tensor(a!) out) -> ()");
  m.def("skinny_gemm(Tensor x, Tensor w, Tensor(a!) out, int cfg) -> ()");
  m.def("skinny_gemm_norm(Tensor x, Tensor w, Tensor(a!) y, Tensor(b!) residual, Tensor norm_w, "
        "float eps, Tensor(c!) out, Tensor(d!) counter, Tensor(e!) partials, int cfg) -> ()");
  m.def("skinny_gemm_swiglu(Tensor x, Tensor w, Tensor(a!) out, int cfg) -> ()");
  m.def("gemv_rows(Tensor x, Tensor w, Tensor(a!) y, int cfg) -> ()");
  m.def("gemv_rows_swiglu(Tensor x, Tensor w, Tensor(a!) out, int cfg, float eps=0.0) -> ()");
  m.def("gemv_rows_rope(Tensor x, Tensor w, Tensor(a!) qkv, Tensor positions, Tensor cos_sin, "
        "Tensor slot_mapping, Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, "
        "int cfg, float eps=0.0) -> ()");
  m.def("gemv_splitk(Tensor x, Tensor w, Tensor(a!) y, Tensor(b!) part, Tensor(c!) tile_cnt, "
        "int cfg) -> ()");
  m.def("gemv_splitk_norm(Tensor x, Tensor w, Tensor(a!) y, Tensor(b!) residual, Tensor norm_w, "
        "float eps, Tensor(c!) out, Tensor(d!) counter, Tensor(e!) part, Tensor(f!) tile_cnt, "
        "int cfg) -> ()");
  m.def("gemv_splitk_swiglu(Tensor x, Tensor w, Tensor(a!) out, Tensor(b!) part, "
        "Tensor(c!) tile_cnt, int cfg) -> ()");
  m.def("gemv_splitk_rope(Tensor x, Tensor w, Tensor(a!) qkv, Tensor positions, Tensor cos_sin, "
        "Tensor slot_mapping, Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, "
        "Tensor(d!) part, Tensor(e!) tile_cnt, int cfg) -> ()");
  m.def("attn_decode_merge(Tensor part_o, Tensor part_ml, Tensor(a!) out, int Hq, "
        "int num_splits) -> ()");
  m.def("skinny_gemm_rope(Tensor x, Tensor w, Tensor(a!) qkv, Tensor positions, Tensor cos_sin, "
        "Tensor slot_mapping, Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, int cfg) -> ()");
  m.def("car_allreduce(Tensor inp, Tensor(a!) out, int[] bases, int rank, int capacity_bytes, "
        "int algo=0) -> ()");
  m.def("car_allreduce_add_norm(Tensor inp, Tensor(a!) residual, Tensor w, float eps, "
        "Tensor(b!) out, int[] bases, int rank, int capacity_bytes, int algo=0) -> ()");
  // host-side setup of the custom all-reduce regions (no tensor dispatch)
  m.def("car_alloc(int data_bytes) -> int", &car_alloc_op);
  m.def("car_free(int ptr) -> ()", &car_free_op);
  m.def("car_ipc_handle(int ptr) -> Tensor", &car_ipc_handle);
  m.def("car_ipc_open(Tensor handle) -> int", &car_ipc_open);
  m.def("car_ipc_close(int ptr) -> ()", &car_ipc_close);
  m.def("car_data_offset() -> int", &car_data_offset);
  m.def("kernel_errors() -> int[]", &kernel_errors);
  m.def("decode_persist_info(int M, int d, int Kx, int nst) -> int[]", &decode_persist_info);
  m.def("decode_engine_info(int M, int d, int Hq, int Hkv, int F) -> int[]", &decode_engine_info);
  m.def("decode_persist(Tensor(a!) residual, Tensor layers, Tensor(b!) qbuf, Tensor(c!) attn, "
        "Tensor(d!) act, Tensor positions, Tensor cos_sin, Tensor slots, Tensor block_tables, "
        "Tensor q_start, Tensor q_len, Tensor kv_len, Tensor work_seq, Tensor work_ct, "
        "Tensor(e!) part_o, Tensor(f!) part_ml, Tensor(g!) tickets, Tensor(h!) counters, int l0, "
        "int l1, int stages, int Hq, int Hkv, int F, int BS, int splits, float scale, float eps, "
        "int flags) -> ()");
  m.def("car_error(int ptr) -> int", &car_error);
  m.def("car_error_info(int ptr) -> int", &car_error_info);
  m.def("moe_skinny(Tensor x, Tensor sorted_ids, int topk, Tensor expert_offsets, Tensor w, "
        "Tensor(a!) out, bool gated, bool gather, int max_rows) -> ()");
  m.def("embed(Tensor ids, Tensor table, Tensor(a!) out, int vocab_start) -> ()");
  m.def("rope_kv(Tensor(a!) qkv, Tensor positions, Tensor cos_sin, Tensor slot_mapping, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv) -> ()");
  m.def("attn_decode(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor seq_q_start, Tensor seq_q_len, Tensor seq_kv_len, Tensor work_seq, Tensor work_ct, "
        "Tensor(a!) out, Tensor(b!) part_o, Tensor(c!) part_ml, int Hq, int Hkv, float scale, "
        "int num_splits, int tiles_per_item=1, Tensor(d!)? tickets=None, "
        "bool reduce=True) -> ()");
  m.def("attn_decode_shared(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor seq_q_start, Tensor seq_q_len, Tensor seq_kv_len, Tensor work_seq, "
        "Tensor work_ct, Tensor(a!) out, Tensor(b!) ws_i32, Tensor(c!) pre_o, Tensor(d!) pre_ml, "
        "int Hq, int Hkv, float scale, int tiles_per_item, bool run_meta) -> ()");
  m.def("attn_prefill_timing(Tensor(a!) buf) -> ()");
  m.def("attn_prefill(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor seq_q_start, Tensor seq_q_len, Tensor seq_kv_len, Tensor work_seq, "
        "Tensor work_qblk, Tensor(a!) out, int Hq, int Hkv, float scale, int qblk=32, "
        "int hsplit_below=0, Tensor(b!)? ws=None, Tensor(c!)? tickets=None, "
        "int small_mode=0) -> ()");
  m.def("prefill_split_ws_sizes() -> int[]", &prefill_split_ws_sizes);
  m.def("sample_partial(Tensor logits, int v0, Tensor mask_table, Tensor mask_idx, Tensor temps, "
        "Tensor seeds, Tensor(a!) part_val, Tensor(b!) part_idx) -> ()");
  m.def("sample_final(Tensor part_val, Tensor part_idx, Tensor(a!) out) -> ()");
  m.def("moe_topk(Tensor router_logits, int topk, bool renorm, Tensor(a!) weights, Tensor(b!) ids) -> ()");
  m.def("moe_route(Tensor x, Tensor router, int topk, bool renorm, Tensor(a!) weights, "
        "Tensor(b!) ids) -> ()");
  m.def("moe_align(Tensor topk_ids, int E, int block_m, Tensor(a!) sorted_ids, Tensor(b!) inv_pos, "
        "Tensor(c!) expert_of_block, Tensor(d!) expert_offsets, Tensor(e!) num_blocks) -> ()");
  m.def("moe_gather(Tensor x, Tensor sorted_ids, int topk, Tensor(a!) out) -> ()");
  m.def("count_nonfinite(Tensor x, Tensor(a!) counter) -> ()");
  m.def("moe_gemm8(Tensor x, Tensor w, Tensor(a!) out, Tensor expert_of_block, "
        "Tensor num_blocks, Tensor expert_offsets, bool swiglu, int tile=256) -> ()");
  m.def("moe_grouped_gemm(Tensor x, Tensor w, Tensor(a!) out, Tensor expert_of_block, "
        "Tensor num_blocks) -> ()");
  m.def("moe_combine(Tensor y, Tensor inv_pos, Tensor weights, int topk, Tensor(a!) out) -> ()");
  m.def("gemm_dense(Tensor x, Tensor w, Tensor(a!) out, bool swiglu=False, int cfg=0) -> ()");
  m.def("moe_gemm_dense(Tensor x, Tensor w, Tensor(a!) out, Tensor expert_offsets, "
        "bool swiglu, int cfg=0) -> ()");
  m.def("moe_w2_combine(Tensor x, Tensor w, Tensor(a!) y, Tensor(b!) yf, Tensor expert_offsets, "
        "Tensor inv_pos, Tensor weights, int topk, Tensor(c!) out, int cus) -> ()");
  m.def("moe_skinny_splitk(Tensor x, Tensor sorted_ids, int topk, Tensor expert_offsets, Tensor w, "
        "Tensor(a!) yf, int max_rows, int splits) -> ()");
  m.def("moe_combine_splitk(Tensor yf, int splits, Tensor inv_pos, Tensor weights, int topk, "
        "Tensor(a!) out) -> ()");
}

TORCH_LIBRARY_IMPL(rfq_amd, CUDA, m) {
  m.impl("rms_norm", &rms_norm);
  m.impl("fused_add_rms_norm", &fused_add_rms_norm);
  m.impl("silu_mul", &silu_mul);
  m.impl("skinny_gemm", &skinny_gemm);
  m.impl("skinny_gemm_norm", &skinny_gemm_norm);
  m.impl("skinny_gemm_rope", &skinny_gemm_rope);
  m.impl("skinny_gemm_swiglu", &skinny_gemm_swiglu);
  m.impl("gemv_rows", &gemv_rows);
  m.impl("decode_persist", &decode_persist);
  m.impl("gemv_rows_swiglu", &gemv_rows_swiglu);
  m.impl("gemv_rows_rope", &gemv_rows_rope);
  m.impl("gemv_splitk", &gemv_splitk);
  m.impl("gemv_splitk_norm", &gemv_splitk_norm);
  m.impl("gemv_splitk_swiglu", &gemv_splitk_swiglu);
  m.impl("gemv_splitk_rope", &gemv_splitk_rope);
  m.impl("attn_decode_merge", &attn_decode_merge);
  m.impl("car_allreduce", &car_allreduce);
  m.impl("car_allreduce_add_norm", &car_allreduce_add_norm);
  m.impl("moe_skinny", &moe_skinny);
  m.impl("embed", &embed);
  m.impl("rope_kv", &rope_kv);
  m.impl("attn_decode", &attn_decode);
  m.impl("attn_decode_shared", &attn_decode_shared);
  m.impl("attn_prefill", &attn_prefill);
  m.impl("attn_prefill_timing", &attn_prefill_timing);
  m.impl("sample_partial", &sample_partial);
  m.impl("sample_final", &sample_final);
  m.impl("moe_topk", &moe_topk);
  m.impl("moe_route", &moe_route);
  m.impl("moe_align", &moe_align);
  m.impl("moe_gather", &moe_gather);
  m.impl("moe_grouped_gemm", &moe_grouped_gemm);
  m.impl("moe_gemm8", &moe_gemm8);
  m.impl("count_nonfinite", &count_nonfinite);
  m.impl("moe_combine", &moe_combine);
  m.impl("gemm_dense", &gemm_dense);
  m.impl("moe_gemm_dense", &moe_gemm_dense);
  m.impl("moe_w2_combine", &moe_w2_combine);
  m.impl("moe_skinny_splitk", &moe_skinny_splitk);
  m.impl("moe_combine_splitk", &moe_combine_splitk);
}
