// Sparse tensor codec on the GPU (tensor_sparse_enc / tensor_sparse_dec,
// reference: gst/nnstreamer/elements/gsttensor_sparseutil.c:20-255).
//
// Payload (after the 128-B meta header): nnz values of the element type, then
// nnz uint32 flat indices, ascending.  "Non-zero" is bitwise (the reference's
// memcmp against zero: -0.0f counts as non-zero).
//
// Encode is an order-preserving stream compaction in two passes over the
// tensor: (1) one workgroup per 4096-element tile counts its non-zeros, a
// single-workgroup scan turns the counts into tile offsets and the total;
// (2) after the host has sized the output from the total, every tile
// recomputes its flags, ranks them with a wave ballot + workgroup scan, and
// writes values and indices at their global positions (block 0 also writes
// the header).  Decode zero-fills and scatters, flagging out-of-range
// indices.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kernels/dtype.h"
#include "kernels/kernels.h"
#include "runtime/hip_util.h"

namespace nnsx {
namespace kernels {

namespace {

constexpr int SP_THREADS = 256;
constexpr int SP_ITEMS = 16;  // consecutive elements per thread
constexpr int SP_TILE = SP_THREADS * SP_ITEMS;

template <typename T>
__device__ __forceinline__ bool nz(T v) {
  return v != T(0);
}

// exclusive scan of one value per thread over the workgroup (256 = 4 waves)
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[SP_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint32_t base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < SP_THREADS / 64; ++w) {
    if (w < wave) base += wsum[w];
    all += wsum[w];
  }
  if (total) *total = all;
  __syncthreads();  // wsum reusable
  return base + inc - v;
}

template <typename T>
__global__ void __launch_bounds__(SP_THREADS) sparse_count_kernel(const T* __restrict__ x, uint64_t n,
                                                                  uint32_t* __restrict__ counts) {
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * SP_TILE;
  uint32_t c = 0;
  // strided within the tile: coalesced reads
#pragma unroll
  for (int i = 0; i < SP_ITEMS; ++i) {
    const uint64_t k = base + static_cast<uint64_t>(i) * SP_THREADS + threadIdx.x;
    if (k < n && nz(x[k])) ++c;
  }
  uint32_t total;
  block_exclusive_scan(c, &total);
  if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

// in-place exclusive scan of the tile counts (one workgroup), total -> *nnz
__global__ void __launch_bounds__(SP_THREADS) sparse_scan_kernel(uint32_t* __restrict__ counts, uint32_t ntiles,
                                                                 uint32_t* __restrict__ nnz) {
  uint32_t carry = 0;
  for (uint32_t b = 0; b < ntiles; b += SP_THREADS) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? counts[i] : 0;
    uint32_t total;
    const uint32_t ex = block_exclusive_scan(v, &total);
    if (i < ntiles) counts[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) *nnz = carry;
}

struct SparseHeader {
  uint32_t w[32];  // the 128-B meta header
};

template <typename T>
__global__ void __launch_bounds__(SP_THREADS) sparse_compact_kernel(const T* __restrict__ x, uint64_t n,
                                                                    const uint32_t* __restrict__ offsets,
                                                                    uint8_t* __restrict__ out, uint32_t nnz,
                                                                    SparseHeader hdr) {
  T* vals = reinterpret_cast<T*>(out + 128);
  // the index block starts right after nnz values: 4-byte aligned only for 4/8-byte types
  uint8_t* idx = out + 128 + static_cast<uint64_t>(nnz) * sizeof(T);
  if (blockIdx.x == 0 && threadIdx.x < 32) reinterpret_cast<uint32_t*>(out)[threadIdx.x] = hdr.w[threadIdx.x];
  // thread t owns SP_ITEMS consecutive elements: the ranks then follow the order
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * SP_TILE + static_cast<uint64_t>(threadIdx.x) * SP_ITEMS;
  T v[SP_ITEMS];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < SP_ITEMS; ++i) {
    const uint64_t k = base + i;
    v[i] = k < n ? x[k] : T(0);
    c += nz(v[i]) ? 1u : 0u;
  }
  uint32_t pos = offsets[blockIdx.x] + block_exclusive_scan(c, nullptr);
#pragma unroll
  for (int i = 0; i < SP_ITEMS; ++i) {
    if (nz(v[i])) {
      vals[pos] = v[i];
      const uint32_t flat = static_cast<uint32_t>(base + i);
      if constexpr (sizeof(T) >= 4)
        reinterpret_cast<uint32_t*>(idx)[pos] = flat;
      else
        __builtin_memcpy(idx + 4ull * pos, &flat, 4);
      ++pos;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(SP_THREADS) sparse_scatter_kernel(const uint8_t* __restrict__ payload, uint32_t nnz,
                                                                    T* __restrict__ out, uint64_t n,
                                                                    int* __restrict__ bad) {
  const T* vals = reinterpret_cast<const T*>(payload);
  const uint8_t* idx = payload + static_cast<uint64_t>(nnz) * sizeof(T);
  for (uint32_t k = blockIdx.x * SP_THREADS + threadIdx.x; k < nnz; k += gridDim.x * SP_THREADS) {
    // unaligned-safe index read (the value block may leave it at any byte)
    uint32_t i;
    __builtin_memcpy(&i, idx + 4ull * k, 4);
    if (i < n) {
      out[i] = vals[k];
    } else {
      *bad = 1;
    }
  }
}

template <typename T>
void encode_t(const void* x, uint64_t n, uint32_t* counts, uint32_t ntiles, uint32_t* nnz, hipStream_t s) {
  hipLaunchKernelGGL(sparse_count_kernel<T>, dim3(ntiles), dim3(SP_THREADS), 0, s, static_cast<const T*>(x), n, counts);
  hipLaunchKernelGGL(sparse_scan_kernel, dim3(1), dim3(SP_THREADS), 0, s, counts, ntiles, nnz);
}

template <typename T>
void compact_t(const void* x, uint64_t n, const uint32_t* offsets, uint32_t ntiles, void* out, uint32_t nnz,
               const SparseHeader& h, hipStream_t s) {
  hipLaunchKernelGGL(sparse_compact_kernel<T>, dim3(ntiles), dim3(SP_THREADS), 0, s, static_cast<const T*>(x), n,
                     offsets, static_cast<uint8_t*>(out), nnz, h);
}

template <typename T>
void scatter_t(const void* payload, uint32_t nnz, void* out, uint64_t n, int* bad, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>((nnz + SP_THREADS - 1) / SP_THREADS, 4096)));
  hipLaunchKernelGGL(sparse_scatter_kernel<T>, dim3(grid), dim3(SP_THREADS), 0, s,
                     static_cast<const uint8_t*>(payload), nnz, static_cast<T*>(out), n, bad);
}

// ---------------------------------------------------- tensor_if average ----
// K22: the mean of a device tensor for tensor_if compared-value=
// TENSOR_AVERAGE_VALUE (gsttensor_if.c:901-928), without a D2H of the
// tensor.  Each workgroup sums a contiguous slab in fp64 (fixed per-thread
// order, then a fixed tree), the partials are added in index order by one
// workgroup, and only the 8-byte mean crosses to the host.  (The reference's
// sequential running mean avg += (x - avg) / (i + 1) and this fp64 sum / n
// agree to O(n * 2^-53) before the cast to the tensor type.)
constexpr int MEAN_BLOCKS_MAX = 1024;

template <typename T>
__global__ void __launch_bounds__(SP_THREADS) mean_partial_kernel(const T* __restrict__ x, uint64_t n, uint64_t slab,
                                                                  double* __restrict__ part) {
  __shared__ double red[SP_THREADS];
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * slab;
  const uint64_t b1 = b0 + slab < n ? b0 + slab : n;
  double acc = 0.0;
  for (uint64_t k = b0 + threadIdx.x; k < b1; k += SP_THREADS) acc += Num<T>::as_double(x[k]);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = SP_THREADS / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(SP_THREADS) mean_final_kernel(const double* __restrict__ part, int nparts,
                                                                uint64_t n, double* __restrict__ mean) {
  __shared__ double red[SP_THREADS];
  double acc = 0.0;
  for (int k = threadIdx.x; k < nparts; k += SP_THREADS) acc += part[k];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = SP_THREADS / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *mean = n ? red[0] / static_cast<double>(n) : 0.0;
}

template <typename T>
void mean_t(const void* x, uint64_t n, double* ws, double* mean, hipStream_t s) {
  const uint64_t want = (n + 8 * SP_THREADS - 1) / (8 * SP_THREADS);  // >= 8 elements per thread
  const int blocks = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(want, MEAN_BLOCKS_MAX)));
  const uint64_t slab = (n + blocks - 1) / blocks;
  hipLaunchKernelGGL(mean_partial_kernel<T>, dim3(blocks), dim3(SP_THREADS), 0, s, static_cast<const T*>(x), n, slab,
                     ws);
  hipLaunchKernelGGL(mean_final_kernel, dim3(1), dim3(SP_THREADS), 0, s, ws, blocks, n, mean);
}

}  // namespace

size_t mean_workspace_bytes() { return (MEAN_BLOCKS_MAX + 1) * sizeof(double); }

bool tensor_mean(const void* x, DType t, uint64_t n, double* d_ws, hipStream_t s) {
  double* mean = d_ws + MEAN_BLOCKS_MAX;
#define NNSX_MEAN(T) mean_t<T>(x, n, d_ws, mean, s)
  switch (t) {
    case DType::INT32: NNSX_MEAN(int32_t); return true;
    case DType::UINT32: NNSX_MEAN(uint32_t); return true;
    case DType::INT16: NNSX_MEAN(int16_t); return true;
    case DType::UINT16: NNSX_MEAN(uint16_t); return true;
    case DType::INT8: NNSX_MEAN(int8_t); return true;
    case DType::UINT8: NNSX_MEAN(uint8_t); return true;
    case DType::FLOAT64: NNSX_MEAN(double); return true;
    case DType::FLOAT32: NNSX_MEAN(float); return true;
    case DType::INT64: NNSX_MEAN(int64_t); return true;
    case DType::UINT64: NNSX_MEAN(uint64_t); return true;
    case DType::FLOAT16: NNSX_MEAN(f16s); return true;
    case DType::BFLOAT16: NNSX_MEAN(bf16s); return true;
    default: return false;
  }
#undef NNSX_MEAN
}

uint32_t sparse_tiles(uint64_t n) { return static_cast<uint32_t>((n + SP_TILE - 1) / SP_TILE); }

bool sparse_count(const void* x, int elem_size, uint64_t n, uint32_t* d_counts, uint32_t* d_nnz, hipStream_t s) {
  const uint32_t nt = sparse_tiles(n);
  if (nt == 0) return hipMemsetAsync(d_nnz, 0, 4, s) == hipSuccess;
  switch (elem_size) {
    case 1: encode_t<uint8_t>(x, n, d_counts, nt, d_nnz, s); return true;
    case 2: encode_t<uint16_t>(x, n, d_counts, nt, d_nnz, s); return true;
    case 4: encode_t<uint32_t>(x, n, d_counts, nt, d_nnz, s); return true;
    case 8: encode_t<uint64_t>(x, n, d_counts, nt, d_nnz, s); return true;
    default: return false;
  }
}

bool sparse_compact(const void* x, int elem_size, uint64_t n, const uint32_t* d_offsets, void* out, uint32_t nnz,
                    const void* header128, hipStream_t s) {
  SparseHeader h;
  __builtin_memcpy(h.w, header128, 128);
  const uint32_t nt = sparse_tiles(n);
  if (nt == 0) return hipMemcpyAsync(out, header128, 128, hipMemcpyHostToDevice, s) == hipSuccess;
  switch (elem_size) {
    case 1: compact_t<uint8_t>(x, n, d_offsets, nt, out, nnz, h, s); return true;
    case 2: compact_t<uint16_t>(x, n, d_offsets, nt, out, nnz, h, s); return true;
    case 4: compact_t<uint32_t>(x, n, d_offsets, nt, out, nnz, h, s); return true;
    case 8: compact_t<uint64_t>(x, n, d_offsets, nt, out, nnz, h, s); return true;
    default: return false;
  }
}

bool sparse_scatter(const void* payload, int elem_size, uint32_t nnz, void* out, uint64_t n, int* d_bad,
                    hipStream_t s) {
  if (nnz == 0) return true;
  switch (elem_size) {
    case 1: scatter_t<uint8_t>(payload, nnz, out, n, d_bad, s); return true;
    case 2: scatter_t<uint16_t>(payload, nnz, out, n, d_bad, s); return true;
    case 4: scatter_t<uint32_t>(payload, nnz, out, n, d_bad, s); return true;
    case 8: scatter_t<uint64_t>(payload, nnz, out, n, d_bad, s); return true;
    default: return false;
  }
}

}  // namespace kernels
}  // namespace nnsx
