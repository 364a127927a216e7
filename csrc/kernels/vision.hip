// Segmentation and pose post-processing kernels for gfx950.
//
// segment_argmax_color: the per-pixel label probabilities ([L] innermost,
// e.g. DeepLabV3 21 x 513 x 513) are staged through LDS with fully coalesced
// global loads (a 256-pixel tile is one contiguous 256*L float run), then each
// lane scans its own L values from LDS -- L is odd for the common label counts,
// so the stride-L LDS reads are bank-conflict free -- and writes the RGBA
// colour directly (argmax, threshold and colour map fused, one HBM pass).
// pose_heatmap_argmax: one workgroup per (keypoint, frame) reduces the heatmap
// grid with the reference's first-maximum-in-row-major order.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "kernels/vision.h"

namespace nnsx {
namespace kernels {

namespace {

constexpr int kSegTile = 256;
constexpr int kSegMaxLdsLabels = 64;

__device__ inline uint32_t label_color(uint32_t label, uint32_t rgb_mod) {
  // color_map[i] = rgb_modifier * i with alpha byte 0xff; background (0) stays transparent
  return label == 0 ? 0u : ((rgb_mod * label) & 0x00ffffffu) | 0xff000000u;
}

__global__ void __launch_bounds__(kSegTile) seg_argmax_lds_kernel(const float* __restrict__ prob, int labels,
                                                                  uint64_t total, uint32_t rgb_mod, float thr,
                                                                  uint32_t* __restrict__ out) {
  __shared__ float tile[kSegTile * kSegMaxLdsLabels];
  const uint64_t p0 = static_cast<uint64_t>(blockIdx.x) * kSegTile;
  const int npx = static_cast<int>(min<uint64_t>(kSegTile, total - p0));
  const float* src = prob + p0 * labels;
  const int nvals = npx * labels;
  for (int i = threadIdx.x; i < nvals; i += kSegTile) tile[i] = src[i];
  __syncthreads();
  if (static_cast<int>(threadIdx.x) >= npx) return;
  const float* v = tile + threadIdx.x * labels;
  float best = v[0];
  int bi = 0;
  for (int l = 1; l < labels; ++l) {
    const float x = v[l];
    if (x > best) {
      best = x;
      bi = l;
    }
  }
  out[p0 + threadIdx.x] = best > thr ? label_color(static_cast<uint32_t>(bi), rgb_mod) : 0u;
}

__global__ void __launch_bounds__(256) seg_argmax_direct_kernel(const float* __restrict__ prob, int labels,
                                                                uint64_t total, uint32_t rgb_mod, float thr,
                                                                uint32_t* __restrict__ out) {
  const uint64_t p = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (p >= total) return;
  const float* v = prob + p * labels;
  float best = v[0];
  int bi = 0;
  for (int l = 1; l < labels; ++l)
    if (v[l] > best) {
      best = v[l];
      bi = l;
    }
  out[p] = best > thr ? label_color(static_cast<uint32_t>(bi), rgb_mod) : 0u;
}

__global__ void __launch_bounds__(256) seg_index_kernel(const float* __restrict__ idx, uint64_t total,
                                                        int max_labels, uint32_t rgb_mod,
                                                        uint32_t* __restrict__ out) {
  const uint64_t p = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (p >= total) return;
  const float f = idx[p];
  // out-of-range labels are not drawn (reference: label_idx > max_labels -> skip)
  if (!(f >= 0.f) || f >= static_cast<float>(max_labels) + 1.f) {
    out[p] = 0u;
    return;
  }
  out[p] = label_color(static_cast<uint32_t>(f), rgb_mod);
}

__global__ void __launch_bounds__(256) depth_max_kernel(const float* __restrict__ in, uint64_t npix,
                                                        uint32_t* __restrict__ max_bits) {
  const int b = blockIdx.y;
  const float* f = in + static_cast<uint64_t>(b) * npix;
  float m = 0.f;  // the reference starts from 0 (negative depths never win)
  for (uint64_t p = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; p < npix;
       p += static_cast<uint64_t>(gridDim.x) * 256)
    m = fmaxf(m, f[p]);
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(&max_bits[b], __float_as_uint(m));  // m >= 0: bit order == value order
}

__global__ void __launch_bounds__(256) depth_color_kernel(const float* __restrict__ in, uint64_t npix,
                                                          const uint32_t* __restrict__ max_bits,
                                                          uint32_t* __restrict__ out) {
  const int b = blockIdx.y;
  const uint64_t p = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (p >= npix) return;
  const float mx = __uint_as_float(max_bits[b]);
  const uint64_t o = static_cast<uint64_t>(b) * npix + p;
  if (mx == 0.f) {
    out[o] = 0u;
    return;
  }
  const float g = in[o] / mx * 255.f;
  const uint32_t gray = g >= 0.f ? static_cast<uint32_t>(g) : 0xffffffffu;
  out[o] = gray > 255u ? 0u : (gray | (gray << 8) | (gray << 16) | 0xff000000u);
}

__global__ void __launch_bounds__(256) pose_argmax_kernel(const float* __restrict__ heat, int k, int gw, int gh,
                                                          int sigmoid, float* __restrict__ out) {
  const int kp = blockIdx.x, b = blockIdx.y;
  const float* h = heat + static_cast<uint64_t>(b) * gw * gh * k;
  float best = FLT_MIN;
  int bi = 0x7fffffff;
  const int n = gw * gh;
  for (int p = threadIdx.x; p < n; p += 256) {
    // element (x = p % gw, y = p / gw): index x*K + y*gw*K + kp
    float v = h[static_cast<uint64_t>(p) * k + kp];
    if (sigmoid) v = 1.f / (1.f + expf(-v));
    if (v > best) {
      best = v;
      bi = p;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(best, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = best;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i)
      if (sv[i] > best || (sv[i] == best && si[i] < bi)) {
        best = sv[i];
        bi = si[i];
      }
    if (bi == 0x7fffffff) bi = 0;  // nothing above FLT_MIN: reference keeps (0, 0)
    float* o = out + (static_cast<uint64_t>(b) * k + kp) * 3;
    o[0] = static_cast<float>(bi % gw);
    o[1] = static_cast<float>(bi / gw);
    o[2] = best;
  }
}

}  // namespace

void segment_argmax_color(const float* prob, int labels, uint64_t pixels, uint32_t rgb_modifier, float threshold,
                          uint32_t* out, hipStream_t s) {
  if (pixels == 0) return;
  const unsigned blocks = static_cast<unsigned>((pixels + kSegTile - 1) / kSegTile);
  if (labels <= kSegMaxLdsLabels)
    hipLaunchKernelGGL(seg_argmax_lds_kernel, dim3(blocks), dim3(kSegTile), 0, s, prob, labels, pixels, rgb_modifier,
                       threshold, out);
  else
    hipLaunchKernelGGL(seg_argmax_direct_kernel, dim3(blocks), dim3(256), 0, s, prob, labels, pixels, rgb_modifier,
                       threshold, out);
}

void segment_index_color(const float* index_map, uint64_t pixels, int max_labels, uint32_t rgb_modifier,
                         uint32_t* out, hipStream_t s) {
  if (pixels == 0) return;
  hipLaunchKernelGGL(seg_index_kernel, dim3(static_cast<unsigned>((pixels + 255) / 256)), dim3(256), 0, s, index_map,
                     pixels, max_labels, rgb_modifier, out);
}

void segment_depth_gray(const float* in, uint64_t pixels, int batch, uint32_t* ws, uint32_t* out, hipStream_t s) {
  if (pixels == 0 || batch == 0) return;
  hipMemsetAsync(ws, 0, sizeof(uint32_t) * batch, s);
  const unsigned bx = static_cast<unsigned>(std::min<uint64_t>((pixels + 255) / 256, 1024));
  hipLaunchKernelGGL(depth_max_kernel, dim3(bx, batch), dim3(256), 0, s, in, pixels, ws);
  hipLaunchKernelGGL(depth_color_kernel, dim3(static_cast<unsigned>((pixels + 255) / 256), batch), dim3(256), 0, s,
                     in, pixels, ws, out);
}

void pose_heatmap_argmax(const float* heat, int keypoints, int grid_w, int grid_h, int batch, bool sigmoid,
                         float* out, hipStream_t s) {
  if (keypoints == 0 || batch == 0) return;
  hipLaunchKernelGGL(pose_argmax_kernel, dim3(keypoints, batch), dim3(256), 0, s, heat, keypoints, grid_w, grid_h,
                     sigmoid ? 1 : 0, out);
}

}  // namespace kernels
}  // namespace nnsx
