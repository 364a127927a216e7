// Decoder kernels for gfx950: argmax reductions (image_labeling K15,
// batched per-frame labels).  Wave64 shuffle reduction -> LDS per wave ->
// block result; ties resolve to the lowest index ("first max wins",
// gst/nnstreamer tensordec-imagelabel.c:148-161).
#include <hip/hip_runtime.h>

#include <cfloat>

#include "kernels/dtype.h"
#include "kernels/kernels.h"

namespace nnsx {
namespace kernels {

namespace {

constexpr int kArgBlock = 1024;

__device__ __forceinline__ void better(double& bv, int64_t& bi, double v, int64_t i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

template <typename T>
__global__ void __launch_bounds__(kArgBlock) argmax_rows_kernel(const T* __restrict__ in, uint64_t n,
                                                                int32_t* __restrict__ out) {
  const T* row = in + static_cast<uint64_t>(blockIdx.x) * n;
  double bv = -DBL_MAX;
  int64_t bi = INT64_MAX;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) better(bv, bi, Num<T>::as_double(row[i]), static_cast<int64_t>(i));
  for (int off = 32; off > 0; off >>= 1) {
    double ov = __shfl_down(bv, off, 64);
    int64_t oi = __shfl_down(bi, off, 64);
    better(bv, bi, ov, oi);
  }
  __shared__ double sv[kArgBlock / 64];
  __shared__ int64_t si[kArgBlock / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[wave] = bv;
    si[wave] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = sv[0];
    int64_t ix = si[0];
    for (int w = 1; w < static_cast<int>(blockDim.x >> 6); ++w) better(v, ix, sv[w], si[w]);
    out[blockIdx.x] = static_cast<int32_t>(ix == INT64_MAX ? 0 : ix);
  }
}

}  // namespace

void argmax_rows(const void* in, DType t, uint64_t n, uint32_t batch, int32_t* out_index, hipStream_t s) {
  if (batch == 0) return;
  unsigned threads = n >= 1024 ? 1024 : (n >= 256 ? 256 : 64);
#define NNSX_T(T) \
  hipLaunchKernelGGL(argmax_rows_kernel<T>, dim3(batch), dim3(threads), 0, s, static_cast<const T*>(in), n, out_index)
  NNSX_DTYPE_CASES(t, NNSX_T)
#undef NNSX_T
}

void argmax(const void* in, DType t, uint64_t n, int32_t* out_index, hipStream_t s) {
  argmax_rows(in, t, n, 1, out_index, s);
}

}  // namespace kernels
}  // namespace nnsx
