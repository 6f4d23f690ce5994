// The TP row-parallel o / down projection with its all-reduce and residual-add RMSNorm
// in one launch (gemv_core.h kGvPush): the split-K GEMV pushes its bf16 outputs straight
// into every rank's custom all-reduce staging (push form, car_core.h) and the grid's last
// workgroup runs the all-reduce sum + norm.  VERDICT r3 item 4 / SURVEY.md §2.4 K8 ("AR
// epilogue (custom AR)" on the o projection).
#include "../kernels/gemv_core.h"

namespace rfq {

template <int NW, int U, bool TL, bool NTL>
__global__ __launch_bounds__(NW * 64) void gemv_push_norm_kernel(
    const bf16_t* __restrict__ X, int64_t ldx, const bf16_t* __restrict__ W, int K, int M, int KS,
    float* __restrict__ part, int Nn, unsigned* __restrict__ tile_cnt, NormEpi ep, PushEpi pe,
    int units) {
  gemv_splitk_unit<NW, U, kGvPush, TL, NTL, false, false>(
      blockIdx.x, units / KS, X, ldx, W, K, nullptr, 0, M, KS, part, Nn, tile_cnt, ep, RopeEpi{},
      0, nullptr, AttnMerge{}, pe);
}

bool gemv_push_fits(int world, int M, int N, int K, int cfg) {
  const int KS = 2 << (cfg & 3);
  return world >= 1 && world <= kCarMaxRanks && M >= 1 && M <= kGvPushMaxM && N % 16 == 0 &&
         N <= kCarPushD && K % 128 == 0 && K / 128 >= KS && !(cfg & 64);
}

// y = x . w^T ([M, N], not stored) all-reduced over the TP group, then residual <- bf16(y +
// residual), out <- rmsnorm(residual) * norm_w.  cfg: split-K GEMV cfg (gemm_skinny.hip
// launch_gemv_splitk_epi bits 0-5); bases: every rank's custom all-reduce region.
void launch_gemv_push_norm(const bf16_t* X, int64_t ldx, const bf16_t* W, int N, int K, int M,
                           int cfg, float* part, unsigned* tile_cnt, bf16_t* residual,
                           int64_t res_stride, const bf16_t* norm_w, bf16_t* out,
                           int64_t out_stride, float eps, unsigned* counter, char* const* bases,
                           int rank, int world, hipStream_t s) {
  const int KS = 2 << (cfg & 3);
  const int units = (N / 16) * KS;
  const NormEpi ep{residual, res_stride, norm_w, out, out_stride, eps, counter, nullptr, 0};
  PushEpi pe{};
  for (int p = 0; p < world; ++p) pe.base[p] = bases[p];
  pe.rank = rank;
  pe.world = world;
#define GP_LAUNCH1(nw, u, tl, nt)                                                          \
  hipLaunchKernelGGL((gemv_push_norm_kernel<nw, u, tl, nt>), dim3(units), dim3(nw * 64), 0, s, \
                     X, ldx, W, K, M, KS, part, N, tile_cnt, ep, pe, units)
#define GP_LAUNCH(nw, u)                                                                   \
  switch ((cfg >> 4) & 3) {                                                                \
    case 0: GP_LAUNCH1(nw, u, false, false); break;                                        \
    case 1: GP_LAUNCH1(nw, u, true, false); break;                                         \
    case 2: GP_LAUNCH1(nw, u, false, true); break;                                         \
    default: GP_LAUNCH1(nw, u, true, true); break;                                         \
  }
  switch ((cfg >> 2) & 3) {
    case 0: GP_LAUNCH(4, 4); break;
    case 1: GP_LAUNCH(8, 4); break;
    case 2: GP_LAUNCH(4, 2); break;
    default: GP_LAUNCH(8, 2); break;
  }
#undef GP_LAUNCH
#undef GP_LAUNCH1
}

}  // namespace rfq
