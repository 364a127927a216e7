// Host-side launch API of the hand-written CDNA4 (gfx950) kernels.
// Every launcher is asynchronous on the given stream, allocation-free and
// graph-capturable (no hipMalloc / sync inside).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

#include "core/types.h"

namespace nnsx {
namespace kernels {

// --------------------------------------------------------------- transform ----
enum ArithKind : int { OP_ADD = 0, OP_MUL = 1, OP_DIV = 2, OP_CLAMP = 3 };

struct ArithOp {
  int kind;          // ArithKind
  double fval;       // operand as double (floats)
  int64_t ival;      // operand as int64 (integer compute types)
  double fval2;      // clamp max
  int ch;            // -1 = all channels
};

constexpr int kMaxArithOps = 16;

struct ArithParams {
  int nops = 0;
  ArithOp ops[kMaxArithOps];
  // per-channel: channel = (i / ch_size) % ch_count ; ch_count = 0 disables
  uint64_t ch_size = 1;
  uint32_t ch_count = 0;
};

// out[i] = ops(cast<out_t>(in[i]))   (tensor_transform typecast / arithmetic / clamp)
void arith(const void* in, DType in_t, void* out, DType out_t, uint64_t n, const ArithParams& p,
           hipStream_t s);

// Generic permutation of up to 8 axes: out.dim[k] = in.dim[perm[k]]
// (tensor_transform transpose / dimchg).  dims are innermost-first.
void permute(const void* in, void* out, size_t elem_size, const uint32_t in_dim[8], const int perm[8],
             hipStream_t s);

// Standardisation (tensor_transform stand): two-pass, fp64 statistics.
// mode 0 = default |x-mean|/std, 1 = dc-average x-mean; per_channel reduces over d0.
// `ws` must hold at least stand_workspace_bytes(ch) bytes.
size_t stand_workspace_bytes(uint32_t channels);
void stand(const void* in, DType in_t, void* out, DType out_t, uint64_t n, uint32_t channels, int mode,
           bool per_channel, void* ws, hipStream_t s);

// -------------------------------------------------------------------- copy ----
// One-launch gather of many host-pinned / device segments into one device block
// (tensor_converter frames-per-tensor batching): replaces a hipMemcpyAsync per
// frame.  Pinned host memory is read in place over the bus (zero copy).
// A segment flagged kGatherPadded is a video frame whose rows sit `stride`
// bytes apart in the source (GStreamer 4-byte row alignment); `row` bytes of
// each are copied, so the destination is packed ([H][W*C], K7 remove-padding).
constexpr uint64_t kGatherPadded = 1ull << 63;
constexpr uint32_t kGatherMaxStride = 8192;  // 4 padded rows fit the 32 KB LDS stage
struct GatherSeg {
  const void* src;
  uint64_t dst_off;
  uint64_t bytes;  // destination bytes | kGatherPadded
};
constexpr int kGatherMax = 128;  // segments per launch (kernel-argument budget)
struct GatherArgs {
  int n = 0;
  uint32_t row = 0, stride = 0;  // geometry of the padded segments
  GatherSeg seg[kGatherMax];
};
void gather_copy(const GatherArgs& g, void* dst, hipStream_t s);
// Padded video frames staged in HBM as they were in host memory (one DMA of
// `src_frame_bytes` per frame on the copy engine): pack `row` bytes of each of
// the `rows` rows (`stride` apart) of every frame into dst [frames][rows][row].
// Replaces the bus-reading gather for padded frames (K7 remove-padding).
void unpad_rows(const void* src, void* dst, uint32_t frames, uint32_t row, uint32_t stride, uint32_t rows,
                uint64_t src_frame_bytes, hipStream_t s);

// ------------------------------------------------------------------ decode ----
// Global argmax over n elements (first max wins).  out_index: int32 on device.
void argmax(const void* in, DType t, uint64_t n, int32_t* out_index, hipStream_t s);
// Batched argmax: rows of `n` elements, `batch` rows -> out_index[batch]
void argmax_rows(const void* in, DType t, uint64_t n, uint32_t batch, int32_t* out_index, hipStream_t s);

// sparse tensor codec (sparse.hip; gsttensor_sparseutil.c): elem_size 1/2/4/8.
// Encode = sparse_count (tile counts -> exclusive offsets in d_counts, total
// -> *d_nnz; d_counts holds sparse_tiles(n) entries) then, once the host knows
// nnz, sparse_compact (header + nnz values + nnz uint32 indices into out).
uint32_t sparse_tiles(uint64_t n);
bool sparse_count(const void* x, int elem_size, uint64_t n, uint32_t* d_counts, uint32_t* d_nnz, hipStream_t s);
bool sparse_compact(const void* x, int elem_size, uint64_t n, const uint32_t* d_offsets, void* out, uint32_t nnz,
                    const void* header128, hipStream_t s);
// decode: out (n elements, zero-filled by the caller) <- payload (values then
// indices); *d_bad = 1 on an index >= n
bool sparse_scatter(const void* payload, int elem_size, uint32_t nnz, void* out, uint64_t n, int* d_bad,
                    hipStream_t s);

// tensor_if TENSOR_AVERAGE on a device tensor (sparse.hip, K22): the fp64
// mean lands at d_ws[mean_workspace_bytes() / 8 - 1]; d_ws holds
// mean_workspace_bytes()
size_t mean_workspace_bytes();
bool tensor_mean(const void* x, DType t, uint64_t n, double* d_ws, hipStream_t s);

// debug: hold stream s busy for `us` microseconds (bounded to 0.2 s; kernels/debug.hip)
void spin_us(hipStream_t s, int us);

}  // namespace kernels
}  // namespace nnsx
