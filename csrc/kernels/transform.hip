// tensor_transform kernels for gfx950.
//
// * arith: fused typecast + add/mul/div chain (+ per-channel operands, clamp)
//   in one pass over HBM -- the reference needs one ORC pass per operator
//   (gst/nnstreamer/elements/gsttensor_transform.c:1241-1412).  Semantics
//   follow the reference's C path: every operator runs in the output type
//   with the operand cast to it first (integer ops wrap, integer div
//   truncates), half types round after each op.
// * permute: transpose / dimchg as one gather pass with coalesced writes.
// * stand: fp64 two-pass mean / population std (tensor_data.c:315-493), a
//   deterministic two-level reduction (no atomics, coalesced reads).
//
// Memory-bound: 8 elements per lane, 256-thread blocks, grid capped at
// 8 blocks per CU x 256 CUs with a grid-stride loop (cdna_hip_programming.md G11).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <type_traits>

#include "kernels/dtype.h"
#include "kernels/kernels.h"

namespace nnsx {
namespace kernels {

namespace {

constexpr int kBlock = 256;
constexpr int kVec = 8;

inline unsigned grid_for(uint64_t work_items) {
  uint64_t g = (work_items + kBlock - 1) / kBlock;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(g, 2048)));
}

template <typename T>
__device__ __forceinline__ T apply_op(T v, const ArithOp& op) {
  if constexpr (is_intlike<T>::value) {
    using W = typename std::conditional<is_unsigned_int<T>::value, uint64_t, int64_t>::type;
    if (op.kind == OP_CLAMP) {
      double d = static_cast<double>(v);
      d = d < op.fval ? op.fval : (d > op.fval2 ? op.fval2 : d);
      return static_cast<T>(d);
    }
    W a = static_cast<W>(v);
    W b = static_cast<W>(static_cast<T>(op.ival));
    switch (op.kind) {
      case OP_ADD: return static_cast<T>(a + b);
      case OP_MUL: return static_cast<T>(a * b);
      default: return b == 0 ? static_cast<T>(0) : static_cast<T>(a / b);
    }
  } else if constexpr (std::is_same<T, f16s>::value || std::is_same<T, bf16s>::value) {
    float a = to_f32(v);
    float b = static_cast<float>(op.fval);
    float r;
    switch (op.kind) {
      case OP_ADD: r = a + to_f32(Num<T>::from(b)); break;
      case OP_MUL: r = a * to_f32(Num<T>::from(b)); break;
      case OP_DIV: r = a / to_f32(Num<T>::from(b)); break;
      default: r = a < op.fval ? static_cast<float>(op.fval) : (a > op.fval2 ? static_cast<float>(op.fval2) : a); break;
    }
    return Num<T>::from(r);
  } else {
    T b = static_cast<T>(op.fval);
    switch (op.kind) {
      case OP_ADD: return v + b;
      case OP_MUL: return v * b;
      case OP_DIV: return v / b;
      default: {
        double d = static_cast<double>(v);
        d = d < op.fval ? op.fval : (d > op.fval2 ? op.fval2 : d);
        return static_cast<T>(d);
      }
    }
  }
}

template <typename InT, typename OutT>
__device__ __forceinline__ OutT eval(InT x, const ArithParams& p, uint64_t idx) {
  OutT v = Num<OutT>::from(x);
  if (p.ch_count) {
    int ch = static_cast<int>((idx / p.ch_size) % p.ch_count);
    for (int k = 0; k < p.nops; ++k)
      if (p.ops[k].ch < 0 || p.ops[k].ch == ch) v = apply_op<OutT>(v, p.ops[k]);
  } else {
    for (int k = 0; k < p.nops; ++k) v = apply_op<OutT>(v, p.ops[k]);
  }
  return v;
}

template <typename T, int N>
struct alignas(sizeof(T) * N) VecT {
  T v[N];
};

// Vector path: n is a multiple of kVec and both pointers are aligned.
template <typename InT, typename OutT>
__global__ void __launch_bounds__(kBlock) arith_vec_kernel(const InT* __restrict__ in, OutT* __restrict__ out,
                                                           uint64_t nvec, ArithParams p) {
  const auto* vin = reinterpret_cast<const VecT<InT, kVec>*>(in);
  auto* vout = reinterpret_cast<VecT<OutT, kVec>*>(out);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < nvec;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    VecT<InT, kVec> a = vin[i];
    VecT<OutT, kVec> b;
#pragma unroll
    for (int k = 0; k < kVec; ++k) b.v[k] = eval<InT, OutT>(a.v[k], p, i * kVec + k);
    vout[i] = b;
  }
}

template <typename InT, typename OutT>
__global__ void __launch_bounds__(kBlock) arith_scalar_kernel(const InT* __restrict__ in, OutT* __restrict__ out,
                                                              uint64_t begin, uint64_t n, ArithParams p) {
  for (uint64_t i = begin + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = eval<InT, OutT>(in[i], p, i);
}

template <typename InT, typename OutT>
void launch_arith(const void* in, void* out, uint64_t n, const ArithParams& p, hipStream_t s) {
  const InT* a = static_cast<const InT*>(in);
  OutT* b = static_cast<OutT*>(out);
  bool aligned = (reinterpret_cast<uintptr_t>(in) % (sizeof(InT) * kVec) == 0) &&
                 (reinterpret_cast<uintptr_t>(out) % (sizeof(OutT) * kVec) == 0);
  uint64_t done = 0;
  if (aligned && n >= kVec) {
    uint64_t nvec = n / kVec;
    hipLaunchKernelGGL((arith_vec_kernel<InT, OutT>), dim3(grid_for(nvec)), dim3(kBlock), 0, s, a, b, nvec, p);
    done = nvec * kVec;
  }
  if (done < n)
    hipLaunchKernelGGL((arith_scalar_kernel<InT, OutT>), dim3(grid_for(n - done)), dim3(kBlock), 0, s, a, b, done,
                       n, p);
}

template <typename InT>
void dispatch_out(DType out_t, const void* in, void* out, uint64_t n, const ArithParams& p, hipStream_t s) {
#define NNSX_OUT(T) launch_arith<InT, T>(in, out, n, p, s)
  NNSX_DTYPE_CASES(out_t, NNSX_OUT)
#undef NNSX_OUT
}

// ------------------------------------------------------------------ permute ----
struct PermParams {
  int rank;
  uint64_t out_dim[8];
  uint64_t in_stride_for_out[8];  // input stride (elements) of the axis that becomes out axis k
  uint64_t total;
};

template <typename E>
__global__ void __launch_bounds__(kBlock) permute_kernel(const E* __restrict__ in, E* __restrict__ out, PermParams p) {
  for (uint64_t o = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; o < p.total;
       o += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint64_t rem = o, src = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= p.rank) break;
      uint64_t c = rem % p.out_dim[k];
      rem /= p.out_dim[k];
      src += c * p.in_stride_for_out[k];
    }
    out[o] = in[src];
  }
}

// General permute, after merging axes that stay adjacent: the input's
// innermost axis (0) and the output's innermost axis (input axis `a`) span a
// 32 x 32 LDS tile, every other axis is a batch index decomposed ONCE per
// workgroup (no per-element div/mod); reads run along input axis 0 and writes
// along input axis a, both coalesced.  a == 0 (innermost axis kept): each
// workgroup copies whole contiguous rows.
struct TiledPerm {
  int nb;                      // batch axes
  uint32_t bdim[6];            // their extents (innermost first)
  uint64_t bin[6], bout[6];    // their input / output strides (elements)
  uint32_t d0, da;             // extents of input axis 0 and axis a
  uint64_t in_sa, out_s0;      // input stride of axis a, output stride of axis 0
  uint64_t nbatch;
};

template <typename E>
__global__ void __launch_bounds__(256) permute_tiled_kernel(const E* __restrict__ in, E* __restrict__ out,
                                                            TiledPerm p) {
  __shared__ E tile[32][33];
  const uint32_t t0 = (blockIdx.x % ((p.d0 + 31) / 32)) * 32, ta = (blockIdx.x / ((p.d0 + 31) / 32)) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (uint64_t bt = blockIdx.y; bt < p.nbatch; bt += gridDim.y) {
    uint64_t rem = bt, bi = 0, bo = 0;
    for (int k = 0; k < p.nb; ++k) {
      const uint64_t c = rem % p.bdim[k];
      rem /= p.bdim[k];
      bi += c * p.bin[k];
      bo += c * p.bout[k];
    }
    // read: rows along axis a, columns along axis 0 (contiguous in the input)
    for (int k = ty; k < 32; k += 8) {
      const uint32_t xa = ta + k, x0 = t0 + tx;
      if (xa < p.da && x0 < p.d0) tile[k][tx] = in[bi + xa * p.in_sa + x0];
    }
    __syncthreads();
    // write: rows along axis 0, columns along axis a (contiguous in the output)
    for (int k = ty; k < 32; k += 8) {
      const uint32_t x0 = t0 + k, xa = ta + tx;
      if (xa < p.da && x0 < p.d0) out[bo + x0 * p.out_s0 + xa] = tile[tx][k];
    }
    __syncthreads();
  }
}

// a == 0: rows of d0 contiguous elements; one workgroup walks rows, the row's
// source offset decomposed once per row
template <typename E>
__global__ void __launch_bounds__(256) permute_rows_kernel(const E* __restrict__ in, E* __restrict__ out,
                                                           TiledPerm p) {
  for (uint64_t row = blockIdx.x; row < p.nbatch; row += gridDim.x) {
    uint64_t rem = row, bi = 0, bo = 0;
    for (int k = 0; k < p.nb; ++k) {
      const uint64_t c = rem % p.bdim[k];
      rem /= p.bdim[k];
      bi += c * p.bin[k];
      bo += c * p.bout[k];
    }
    for (uint32_t x = threadIdx.x; x < p.d0; x += 256) out[bo + x] = in[bi + x];
  }
}

// HWC->CHW style transpose of the two innermost "super axes" through an LDS
// tile (32 x 33 pad: conflict-free column reads).  in: [B][R][C] -> out: [B][C][R]
template <typename E>
__global__ void __launch_bounds__(kBlock) transpose2d_kernel(const E* __restrict__ in, E* __restrict__ out,
                                                             uint64_t R, uint64_t C) {
  __shared__ E tile[32][33];
  const uint64_t b = blockIdx.z;
  const uint64_t r0 = static_cast<uint64_t>(blockIdx.y) * 32, c0 = static_cast<uint64_t>(blockIdx.x) * 32;
  const E* src = in + b * R * C;
  E* dst = out + b * R * C;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8 threads
  for (int k = ty; k < 32; k += 8) {
    uint64_t r = r0 + k, c = c0 + tx;
    if (r < R && c < C) tile[k][tx] = src[r * C + c];
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    uint64_t c = c0 + k, r = r0 + tx;
    if (r < R && c < C) dst[c * R + r] = tile[tx][k];
  }
}

// -------------------------------------------------------------------- stand ----
// Deterministic two-level reduction over the [rows][C] tensor (channel
// innermost; C = 1 for the global statistics), no atomics: level 1 -- block b
// owns rows [b * rpb, (b + 1) * rpb) and writes one fp64 partial per channel,
// its threads reading the rows' contiguous bytes in order (coalesced; for C <=
// kBlock a multiple of C threads is active, so thread t always meets channel
// t % C); level 2 -- one thread per channel adds the block partials in block
// order.  Same result on every run, whatever the dispatch order.
constexpr uint32_t kStandMaxBlocks = 256;

template <typename InT>
__global__ void __launch_bounds__(kBlock) stand_partial_kernel(const InT* __restrict__ in, uint64_t rows, uint32_t C,
                                                               uint64_t rpb, const double* __restrict__ mean,
                                                               double* __restrict__ part, int pass) {
  __shared__ double red[kBlock];
  const uint64_t r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  double* out = part + static_cast<uint64_t>(blockIdx.x) * C;
  if (C <= kBlock) {
    const uint32_t lanes = (kBlock / C) * C, t = threadIdx.x, ch = t % C;
    const double m = pass ? mean[ch] : 0.0;
    double local = 0.0;
    if (t < lanes && r0 < r1)
      for (uint64_t i = r0 * C + t, end = r1 * C; i < end; i += lanes) {
        const double x = Num<InT>::as_double(in[i]);
        local += pass ? (x - m) * (x - m) : x;
      }
    red[t] = local;
    __syncthreads();
    if (t < C) {
      double acc = 0.0;
      for (uint32_t j = t; j < lanes; j += C) acc += red[j];
      out[t] = acc;
    }
  } else {
    for (uint32_t ch = threadIdx.x; ch < C; ch += kBlock) {  // consecutive threads, consecutive channels
      const double m = pass ? mean[ch] : 0.0;
      double acc = 0.0;
      for (uint64_t r = r0; r < r1; ++r) {
        const double x = Num<InT>::as_double(in[r * C + ch]);
        acc += pass ? (x - m) * (x - m) : x;
      }
      out[ch] = acc;
    }
  }
}

__global__ void stand_combine_kernel(const double* __restrict__ part, uint32_t nblocks, uint32_t C, uint64_t count,
                                     double* __restrict__ res, int pass) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double acc = 0.0;
  for (uint32_t b = 0; b < nblocks; ++b) acc += part[static_cast<uint64_t>(b) * C + c];
  const double v = acc / static_cast<double>(count);
  res[c] = pass == 0 ? v : (v != 0.0 ? sqrt(v) : 1e-10);
}

template <typename InT, typename OutT>
__global__ void __launch_bounds__(kBlock) stand_apply_kernel(const InT* __restrict__ in, OutT* __restrict__ out,
                                                             uint64_t n, uint32_t C, bool per_channel, int mode,
                                                             const double* __restrict__ mean,
                                                             const double* __restrict__ stdv) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint32_t ch = per_channel ? static_cast<uint32_t>(i % C) : 0;
    double x = Num<InT>::as_double(in[i]);
    double r = mode == 0 ? fabs((x - mean[ch]) / stdv[ch]) : x - mean[ch];
    out[i] = Num<OutT>::from(r);
  }
}

template <typename InT>
void launch_stand(const void* in, DType out_t, void* out, uint64_t n, uint32_t C, int mode, bool per_channel,
                  void* ws, hipStream_t s) {
  const uint32_t nch = per_channel ? C : 1;
  double* mean = static_cast<double*>(ws);
  double* stdv = mean + nch;
  double* part = stdv + nch;
  const uint64_t rows = n / nch;
  const uint64_t rpb = std::max<uint64_t>(1, (rows + kStandMaxBlocks - 1) / kStandMaxBlocks);
  const uint32_t nblocks = static_cast<uint32_t>((rows + rpb - 1) / rpb);
  const InT* a = static_cast<const InT*>(in);
  const dim3 fin((nch + 63) / 64);
  hipLaunchKernelGGL((stand_partial_kernel<InT>), dim3(nblocks), dim3(kBlock), 0, s, a, rows, nch, rpb, mean, part, 0);
  hipLaunchKernelGGL(stand_combine_kernel, fin, dim3(64), 0, s, part, nblocks, nch, rows, mean, 0);
  if (mode == 0) {
    hipLaunchKernelGGL((stand_partial_kernel<InT>), dim3(nblocks), dim3(kBlock), 0, s, a, rows, nch, rpb, mean, part,
                       1);
    hipLaunchKernelGGL(stand_combine_kernel, fin, dim3(64), 0, s, part, nblocks, nch, rows, stdv, 1);
  }
#define NNSX_OUT(T)                                                                                          \
  hipLaunchKernelGGL((stand_apply_kernel<InT, T>), dim3(grid_for(n)), dim3(kBlock), 0, s, a,               \
                     static_cast<T*>(out), n, C, per_channel, mode, mean, stdv)
  NNSX_DTYPE_CASES(out_t, NNSX_OUT)
#undef NNSX_OUT
}

}  // namespace

void arith(const void* in, DType in_t, void* out, DType out_t, uint64_t n, const ArithParams& p, hipStream_t s) {
  if (n == 0) return;
#define NNSX_IN(T) dispatch_out<T>(out_t, in, out, n, p, s)
  NNSX_DTYPE_CASES(in_t, NNSX_IN)
#undef NNSX_IN
}

// the general case through permute_tiled / permute_rows; false when the
// shape does not fit their limits (the per-element kernel takes it)
static bool launch_tiled_permute(const void* in, void* out, size_t es, const uint32_t in_dim[8], const int perm[8],
                                 hipStream_t s) {
  // merge input axes i, i+1 that the output keeps adjacent and in order; drop unit axes
  uint64_t dim[8], istr[8];
  int map[8], r = 0;  // merged axis of each input axis (-1: unit)
  uint64_t acc = 1;
  for (int k = 0; k < 8; ++k) {
    const uint64_t st = acc;
    acc *= in_dim[k];
    if (in_dim[k] == 1) {
      map[k] = -1;
      continue;
    }
    dim[r] = in_dim[k];
    istr[r] = st;
    map[k] = r++;
  }
  if (r == 0 || acc == 0) return false;
  // the output order of merged axes
  int oq[8], no = 0;
  for (int k = 0; k < 8; ++k)
    if (map[perm[k]] >= 0) oq[no++] = map[perm[k]];
  // fuse runs (j, j+1) adjacent in both orders
  uint64_t fdim[8], fistr[8];
  int fid[8], nf = 0, fo[8], nfo = 0;
  for (int k = 0; k < no; ++k) {
    if (k > 0 && oq[k] == oq[k - 1] + 1) {
      fdim[nf - 1] *= dim[oq[k]];
      continue;
    }
    fid[oq[k]] = nf;
    fdim[nf] = dim[oq[k]];
    fistr[nf] = istr[oq[k]];
    fo[nfo++] = nf++;
  }
  (void)fid;
  // fused axes in input order: sort by input stride
  int byin[8];
  for (int k = 0; k < nf; ++k) byin[k] = k;
  std::sort(byin, byin + nf, [&](int x, int y) { return fistr[x] < fistr[y]; });
  // output strides of each fused axis
  uint64_t fostr[8], oacc = 1;
  for (int k = 0; k < nfo; ++k) {
    fostr[fo[k]] = oacc;
    oacc *= fdim[fo[k]];
  }
  if (nf > 8 || nf - 2 > 6) return false;
  const int ax0 = byin[0], axa = fo[0];  // input-innermost, output-innermost
  TiledPerm p{};
  p.d0 = static_cast<uint32_t>(fdim[ax0]);
  if (fdim[ax0] >= (1ull << 32)) return false;
  if (axa == ax0) {
    // innermost kept: rows
    p.nbatch = acc / fdim[ax0];
    for (int k = 0; k < nf; ++k) {
      const int ax = byin[k];
      if (ax == ax0) continue;
      p.bdim[p.nb] = static_cast<uint32_t>(fdim[ax]);
      p.bin[p.nb] = fistr[ax];
      p.bout[p.nb++] = fostr[ax];
    }
    if (p.nb > 6) return false;
    const unsigned g = static_cast<unsigned>(std::min<uint64_t>(p.nbatch, 65535));
    switch (es) {
      case 1: hipLaunchKernelGGL(permute_rows_kernel<uint8_t>, dim3(g), dim3(256), 0, s, (const uint8_t*)in, (uint8_t*)out, p); return true;
      case 2: hipLaunchKernelGGL(permute_rows_kernel<uint16_t>, dim3(g), dim3(256), 0, s, (const uint16_t*)in, (uint16_t*)out, p); return true;
      case 4: hipLaunchKernelGGL(permute_rows_kernel<uint32_t>, dim3(g), dim3(256), 0, s, (const uint32_t*)in, (uint32_t*)out, p); return true;
      case 8: hipLaunchKernelGGL(permute_rows_kernel<uint64_t>, dim3(g), dim3(256), 0, s, (const uint64_t*)in, (uint64_t*)out, p); return true;
      default: return false;
    }
  }
  if (fdim[axa] >= (1ull << 32)) return false;
  p.da = static_cast<uint32_t>(fdim[axa]);
  p.in_sa = fistr[axa];
  p.out_s0 = fostr[ax0];
  p.nbatch = acc / (fdim[ax0] * fdim[axa]);
  for (int k = 0; k < nf; ++k) {
    const int ax = byin[k];
    if (ax == ax0 || ax == axa) continue;
    p.bdim[p.nb] = static_cast<uint32_t>(fdim[ax]);
    p.bin[p.nb] = fistr[ax];
    p.bout[p.nb++] = fostr[ax];
  }
  if (p.nb > 6) return false;
  const uint64_t tiles = ((p.d0 + 31ull) / 32) * ((p.da + 31ull) / 32);
  if (tiles > 0x7fffffffull) return false;
  dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(std::min<uint64_t>(p.nbatch, 65535)));
  switch (es) {
    case 1: hipLaunchKernelGGL(permute_tiled_kernel<uint8_t>, grid, dim3(256), 0, s, (const uint8_t*)in, (uint8_t*)out, p); return true;
    case 2: hipLaunchKernelGGL(permute_tiled_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)in, (uint16_t*)out, p); return true;
    case 4: hipLaunchKernelGGL(permute_tiled_kernel<uint32_t>, grid, dim3(256), 0, s, (const uint32_t*)in, (uint32_t*)out, p); return true;
    case 8: hipLaunchKernelGGL(permute_tiled_kernel<uint64_t>, grid, dim3(256), 0, s, (const uint64_t*)in, (uint64_t*)out, p); return true;
    default: return false;
  }
}

void permute(const void* in, void* out, size_t elem_size, const uint32_t in_dim[8], const int perm[8],
             hipStream_t s) {
  uint64_t in_stride[8];
  uint64_t acc = 1;
  for (int k = 0; k < 8; ++k) {
    in_stride[k] = acc;
    acc *= in_dim[k];
  }
  PermParams p{};
  p.rank = 8;
  p.total = acc;
  for (int k = 0; k < 8; ++k) {
    p.out_dim[k] = in_dim[perm[k]];
    p.in_stride_for_out[k] = in_stride[perm[k]];
  }
  // trim trailing unit axes for a cheaper index computation
  while (p.rank > 1 && p.out_dim[p.rank - 1] == 1) --p.rank;
  if (acc == 0) return;

  // Special case: a pure 2-D transpose of super-axes [A][B] -> [B][A] with a
  // batch above (e.g. HWC -> CHW: A = W*H, B = C).  Detect: out = (in axes
  // j..r-1, then 0..j-1) for some split j, rest identity.
  int r = 8;
  while (r > 1 && in_dim[r - 1] == 1 && perm[r - 1] == r - 1) --r;
  for (int j = 1; j < r; ++j) {
    bool ok = true;
    for (int k = 0; k < r; ++k) {
      int expect = k < r - j ? k + j : k - (r - j);
      if (perm[k] != expect) {
        ok = false;
        break;
      }
    }
    // batch = outermost axis kept in place is handled by the generic path
    if (ok) {
      uint64_t B = 1, A = 1;
      for (int k = 0; k < j; ++k) B *= in_dim[k];  // innermost block of the input
      for (int k = j; k < r; ++k) A *= in_dim[k];
      // in viewed as [A rows][B cols] -> out [B rows][A cols]
      dim3 grid(static_cast<unsigned>((B + 31) / 32), static_cast<unsigned>((A + 31) / 32), 1);
      if (grid.y <= 65535 && A >= 32 && B >= 32) {
        switch (elem_size) {
          case 1: hipLaunchKernelGGL(transpose2d_kernel<uint8_t>, grid, dim3(256), 0, s, (const uint8_t*)in, (uint8_t*)out, A, B); return;
          case 2: hipLaunchKernelGGL(transpose2d_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)in, (uint16_t*)out, A, B); return;
          case 4: hipLaunchKernelGGL(transpose2d_kernel<uint32_t>, grid, dim3(256), 0, s, (const uint32_t*)in, (uint32_t*)out, A, B); return;
          case 8: hipLaunchKernelGGL(transpose2d_kernel<uint64_t>, grid, dim3(256), 0, s, (const uint64_t*)in, (uint64_t*)out, A, B); return;
          default: break;
        }
      }
      break;
    }
  }
  // transpose with the outermost axis kept (HWC->CHW with N frames): batch over the last kept axis
  {
    int rr = r;
    if (rr >= 2 && perm[rr - 1] == rr - 1) {
      int r2 = rr - 1;
      for (int j = 1; j < r2; ++j) {
        bool ok = true;
        for (int k = 0; k < r2; ++k) {
          int expect = k < r2 - j ? k + j : k - (r2 - j);
          if (perm[k] != expect) {
            ok = false;
            break;
          }
        }
        if (ok) {
          uint64_t Bc = 1, A = 1;
          for (int k = 0; k < j; ++k) Bc *= in_dim[k];
          for (int k = j; k < r2; ++k) A *= in_dim[k];
          uint64_t batch = in_dim[rr - 1];
          dim3 grid(static_cast<unsigned>((Bc + 31) / 32), static_cast<unsigned>((A + 31) / 32),
                    static_cast<unsigned>(batch));
          if (grid.y <= 65535 && batch <= 65535 && A >= 32 && Bc >= 32) {
            switch (elem_size) {
              case 1: hipLaunchKernelGGL(transpose2d_kernel<uint8_t>, grid, dim3(256), 0, s, (const uint8_t*)in, (uint8_t*)out, A, Bc); return;
              case 2: hipLaunchKernelGGL(transpose2d_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)in, (uint16_t*)out, A, Bc); return;
              case 4: hipLaunchKernelGGL(transpose2d_kernel<uint32_t>, grid, dim3(256), 0, s, (const uint32_t*)in, (uint32_t*)out, A, Bc); return;
              case 8: hipLaunchKernelGGL(transpose2d_kernel<uint64_t>, grid, dim3(256), 0, s, (const uint64_t*)in, (uint64_t*)out, A, Bc); return;
              default: break;
            }
          }
          break;
        }
      }
    }
  }
  if (launch_tiled_permute(in, out, elem_size, in_dim, perm, s)) return;
  unsigned g = grid_for(acc);
  switch (elem_size) {
    case 1: hipLaunchKernelGGL(permute_kernel<uint8_t>, dim3(g), dim3(kBlock), 0, s, (const uint8_t*)in, (uint8_t*)out, p); break;
    case 2: hipLaunchKernelGGL(permute_kernel<uint16_t>, dim3(g), dim3(kBlock), 0, s, (const uint16_t*)in, (uint16_t*)out, p); break;
    case 4: hipLaunchKernelGGL(permute_kernel<uint32_t>, dim3(g), dim3(kBlock), 0, s, (const uint32_t*)in, (uint32_t*)out, p); break;
    case 8: hipLaunchKernelGGL(permute_kernel<uint64_t>, dim3(g), dim3(kBlock), 0, s, (const uint64_t*)in, (uint64_t*)out, p); break;
    default: break;
  }
}

size_t stand_workspace_bytes(uint32_t channels) {
  return sizeof(double) * (2 + kStandMaxBlocks) * (channels ? channels : 1);
}

void stand(const void* in, DType in_t, void* out, DType out_t, uint64_t n, uint32_t channels, int mode,
           bool per_channel, void* ws, hipStream_t s) {
  if (n == 0) return;
#define NNSX_IN(T) launch_stand<T>(in, out_t, out, n, channels, mode, per_channel, ws, s)
  NNSX_DTYPE_CASES(in_t, NNSX_IN)
#undef NNSX_IN
}

// ----------------------------------------------------------------- gather ----
namespace {

constexpr uint32_t kGatherLds = 32768;

// padded frame: stage whole source rows (16-B loads, padding included) through
// LDS, then write the packed rows out with consecutive lanes on consecutive bytes
__device__ void gather_padded(const char* __restrict__ src, char* __restrict__ d, uint64_t bytes, uint32_t row,
                              uint32_t stride, int part, int parts, uint4* lds4) {
  char* lds = reinterpret_cast<char*>(lds4);
  const uint32_t rows = static_cast<uint32_t>(bytes / row);
  const uint32_t R = (kGatherLds / stride) & ~3u;  // rows per stage; R * stride % 16 == 0
  const bool vec = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  for (uint32_t r0 = static_cast<uint32_t>(part) * R; r0 < rows; r0 += static_cast<uint32_t>(parts) * R) {
    const uint32_t nr = min(R, rows - r0);
    const char* s = src + static_cast<uint64_t>(r0) * stride;
    const uint32_t span = (nr - 1) * stride + row;  // the last row's padding may not exist
    if (vec) {
      const uint32_t nv = span / 16;
      const uint4* s4 = reinterpret_cast<const uint4*>(s);
      for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) lds4[i] = s4[i];
      for (uint32_t i = nv * 16 + threadIdx.x; i < span; i += blockDim.x) lds[i] = s[i];
    } else {
      for (uint32_t i = threadIdx.x; i < span; i += blockDim.x) lds[i] = s[i];
    }
    __syncthreads();
    char* o = d + static_cast<uint64_t>(r0) * row;
    const uint32_t n = nr * row;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t y = i / row, x = i - y * row;
      o[i] = lds[y * stride + x];
    }
    __syncthreads();
  }
}

template <bool kPad>
__global__ void __launch_bounds__(256) gather_kernel(GatherArgs g, char* __restrict__ dst) {
  const GatherSeg sg = g.seg[blockIdx.y];
  char* d = dst + sg.dst_off;
  const char* src = static_cast<const char*>(sg.src);
  const uint64_t bytes = sg.bytes & ~kGatherPadded;
  if constexpr (kPad) {
    __shared__ uint4 lds[kGatherLds / 16];
    if (sg.bytes & kGatherPadded) {
      gather_padded(src, d, bytes, g.row, g.stride, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x), lds);
      return;
    }
  }
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d) | bytes) & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(d);
    const uint64_t n = bytes / 16;
    // 4 independent 16-B loads in flight per lane (host reads cross the bus)
    for (uint64_t i = t0; i < n; i += 4 * stride) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * stride < n) v[u] = s4[i + u * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * stride < n) d4[i + u * stride] = v[u];
    }
  } else {
    for (uint64_t i = t0; i < bytes; i += stride) d[i] = src[i];
  }
}

// padded frames already in HBM (one DMA of the padded bytes per frame): pack
// their rows.  Each lane writes 16 consecutive output bytes with one 16-byte
// store (the output is one packed [frames][rows][row] block) and gathers them
// byte by byte from the staged rows, which sit in L2 right after the DMA.
// (28 us for DeepLab b8's 8 x 513 x 1539-byte rows; a form with 32-bit index
// math and five aligned dword loads + v_alignbyte per chunk ran the same 28 us
// and left the DeepLab step unchanged: not the bound.)
__global__ void __launch_bounds__(256) unpad_rows_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         uint64_t total, uint32_t row, uint32_t stride, uint32_t rows,
                                                         uint64_t src_frame) {
  const uint64_t fsz = static_cast<uint64_t>(row) * rows;
  for (uint64_t q = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; q * 16 < total;
       q += static_cast<uint64_t>(gridDim.x) * 256) {
    uint64_t o = q * 16;
    uint64_t f = o / fsz;
    uint64_t rem = o - f * fsz;
    uint32_t y = static_cast<uint32_t>(rem / row);
    uint32_t x = static_cast<uint32_t>(rem - static_cast<uint64_t>(y) * row);
    union {
      uint8_t b[16];
      uint4 v;
    } u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      u.b[i] = o + i < total ? src[f * src_frame + static_cast<uint64_t>(y) * stride + x] : 0;
      if (++x == row) {
        x = 0;
        if (++y == rows) {
          y = 0;
          ++f;
        }
      }
    }
    if (o + 16 <= total) {
      *reinterpret_cast<uint4*>(dst + o) = u.v;
    } else {
      for (uint64_t i = o; i < total; ++i) dst[i] = u.b[i - o];
    }
  }
}

}  // namespace

void unpad_rows(const void* src, void* dst, uint32_t frames, uint32_t row, uint32_t stride, uint32_t rows,
                uint64_t src_frame_bytes, hipStream_t s) {
  if (!frames || !rows || !row) return;
  if (row > stride || src_frame_bytes < static_cast<uint64_t>(stride) * (rows - 1) + row)
    throw std::invalid_argument("unpad_rows: row <= stride and a staged frame holds every row");
  const uint64_t total = static_cast<uint64_t>(frames) * row * rows;
  const uint64_t nq = (total + 15) / 16;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>((nq + 255) / 256, 8192)));
  hipLaunchKernelGGL(unpad_rows_kernel, dim3(grid), dim3(256), 0, s, static_cast<const uint8_t*>(src),
                     static_cast<uint8_t*>(dst), total, row, stride, rows, src_frame_bytes);
}

void gather_copy(const GatherArgs& g, void* dst, hipStream_t s) {
  if (g.n <= 0) return;
  // Host-link bound: 1-2 workgroups per frame already saturate the bus
  // (~57 GB/s for 128 x 270 KB frames, scripts/micro/h2d_gather.hip), and a
  // small grid leaves the CUs to the model kernels this copy overlaps with.
  const unsigned bx = static_cast<unsigned>(std::max(1, std::min(4, 256 / g.n)));
  bool pad = false;
  for (int i = 0; i < g.n; ++i) pad |= (g.seg[i].bytes & kGatherPadded) != 0;
  if (pad) {
    if (g.row == 0 || g.row > g.stride || g.stride > kGatherMaxStride || (g.stride & 3))
      throw std::invalid_argument("gather_copy: padded rows need 0 < row <= stride <= 8192, stride % 4 == 0");
    hipLaunchKernelGGL(gather_kernel<true>, dim3(bx, static_cast<unsigned>(g.n)), dim3(256), 0, s, g,
                       static_cast<char*>(dst));
  } else {
    hipLaunchKernelGGL(gather_kernel<false>, dim3(bx, static_cast<unsigned>(g.n)), dim3(256), 0, s, g,
                       static_cast<char*>(dst));
  }
}

}  // namespace kernels
}  // namespace nnsx
