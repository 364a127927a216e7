// The split-bf16 (x3) fp32 GEMM kernels (pw_gemm_f32_tile<..., X3 = true>,
// kernels/gemm_f32.h), in a translation unit of their own: built with the MFMA
// results in VGPRs (see gemm_f32.h).
#include <stdexcept>

#include "kernels/gemm_f32.h"

namespace nnsx {
namespace kernels {

namespace {
template <int BM, int BN>
void launch_tile(bool w3, dim3 grid, hipStream_t s, const float* x, const float* wt, X3W w3p, const float* bias,
                 const float* res, float* y, int M, int N, int K, int Kpad, int Npad, int act, int kchunk, YLayout yl) {
  if (w3)
    hipLaunchKernelGGL((pw_gemm_f32_kernel<BM, BN, true, true>), grid, dim3(256), 0, s, x, wt, w3p, bias, res, y, M, N, K,
                       Kpad, Npad, act, kchunk, yl);
  else
    hipLaunchKernelGGL((pw_gemm_f32_kernel<BM, BN, true>), grid, dim3(256), 0, s, x, wt, X3W{}, bias, res, y, M, N, K,
                       Kpad, Npad, act, kchunk, yl);
}
}  // namespace

void pw_gemm_x3_launch(int BM, int BN, bool w3, dim3 grid, hipStream_t s, const float* x, const float* wt, X3W w3p,
                       const float* bias, const float* res, float* y, int M, int N, int K, int Kpad, int Npad,
                       int act, int kchunk, YLayout yl) {
  switch (BM * 1000 + BN) {
    case 64064: launch_tile<64, 64>(w3, grid, s, x, wt, w3p, bias, res, y, M, N, K, Kpad, Npad, act, kchunk, yl); break;
    case 128064: launch_tile<128, 64>(w3, grid, s, x, wt, w3p, bias, res, y, M, N, K, Kpad, Npad, act, kchunk, yl); break;
    case 64128: launch_tile<64, 128>(w3, grid, s, x, wt, w3p, bias, res, y, M, N, K, Kpad, Npad, act, kchunk, yl); break;
    case 128128: launch_tile<128, 128>(w3, grid, s, x, wt, w3p, bias, res, y, M, N, K, Kpad, Npad, act, kchunk, yl); break;
    case 128192: launch_tile<128, 192>(w3, grid, s, x, wt, w3p, bias, res, y, M, N, K, Kpad, Npad, act, kchunk, yl); break;
    default: throw std::invalid_argument("pw_gemm_x3: no such tile");
  }
}

void pw_gemm_group_x3_launch(bool w3, unsigned blocks, hipStream_t s, const GemmGroupArgs& g) {
  if (w3)
    hipLaunchKernelGGL((pw_gemm_group_f32_kernel<64, 64, true, true>), dim3(blocks), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((pw_gemm_group_f32_kernel<64, 64, true>), dim3(blocks), dim3(256), 0, s, g);
}

}  // namespace kernels
}  // namespace nnsx
