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

#include "decoders/font.h"
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


// Pose skeleton rasteriser: one workgroup per frame.  Keypoint positions are
// refined from the argmax (heatmap-offset mode adds the offset tensor) exactly
// like the host path; connections are drawn one per lane (Bresenham, same pixel
// value -> order free); labels are drawn keypoint by keypoint behind barriers
// because their cells (which also write background zeros) may overlap.
__device__ inline void pose_setpixel(uint32_t* f, int W, int H, int x, int y) {
  if (x < 0 || x >= W || y < 0 || y >= H) return;
  f[y * W + x] = 0xFFFFFFFFu;
  if (x + 1 < W) f[y * W + x + 1] = 0xFFFFFFFFu;
  if (y + 1 < H) f[(y + 1) * W + x] = 0xFFFFFFFFu;
}

__constant__ int kDotX[40] = {-4, 0, 4, 0,  -3, -3, -3, -2, -2, -2, -2, -2, -1, -1, -1, -1, -1, -1, -1, 0,
                              0,  0, 0, 0,  0,  1,  1,  1,  1,  1,  1,  1,  2,  2,  2,  2,  2,  3,  3,  3};
__constant__ int kDotY[40] = {0,  -4, 0,  4,  -1, 0,  1,  -2, -1, 0,  1,  2,  -3, -2, -1, 0,  1,  2,  3,  -3,
                              -2, -1, 1,  2,  3,  -3, -2, -1, 0,  1,  2,  3,  -2, -1, 0,  1,  2,  -1, 0,  1};
__constant__ uint8_t kFontPose[95][13] = NNSX_FONT8X13_DATA;

// keypoint k of frame b: raster position and validity, exactly as the host
// path refines it (tensordec-pose.c:760-800)
__device__ inline void pose_point(const PoseDrawArgs& a, int b, int k, int* px, int* py, bool* valid) {
  const int K = a.keypoints;
  const float* o = a.kp + (static_cast<uint64_t>(b) * K + k) * 3;
  const int mx = static_cast<int>(o[0]), my = static_cast<int>(o[1]);
  int x, y;
  if (a.offsets) {
    const uint64_t oi = static_cast<uint64_t>(b) * a.gw * a.gh * 2 * K + (static_cast<uint64_t>(my) * a.gw + mx) * K * 2 + k;
    const float offy = a.offsets[oi], offx = a.offsets[oi + K];
    const float fx = (static_cast<float>(mx) / (a.gw - 1)) * a.i_w + offx;
    const float fy = (static_cast<float>(my) / (a.gh - 1)) * a.i_h + offy;
    x = static_cast<int>(fx * a.W / a.i_w);
    y = static_cast<int>(fy * a.H / a.i_h);
  } else {
    x = static_cast<int>((static_cast<unsigned>(mx) * a.W) / a.i_w);
    y = static_cast<int>((static_cast<unsigned>(my) * a.H) / a.i_h);
  }
  *px = static_cast<int>(min(static_cast<unsigned>(a.W), static_cast<unsigned>(max(0, x))));
  *py = static_cast<int>(min(static_cast<unsigned>(a.H), static_cast<unsigned>(max(0, y))));
  *valid = o[2] >= 0.5f;
}

// Skeleton, one wave per connection (grid: frames x edge groups of 4): the
// end dots by 40 lanes each, the Bresenham line by one lane.  Every pixel gets
// the same value, so the edges of a frame need no order among themselves.
__global__ void __launch_bounds__(256) pose_lines_kernel(PoseDrawArgs a) {
  const int b = blockIdx.x;
  const int e = blockIdx.y * 4 + static_cast<int>(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= a.n_edges) return;
  uint32_t* f = a.frames + static_cast<uint64_t>(b) * a.W * a.H;
  const int i = a.edges[2 * e], k = a.edges[2 * e + 1];
  int xi, yi, xk, yk;
  bool vi, vk;
  pose_point(a, b, i, &xi, &yi, &vi);
  pose_point(a, b, k, &xk, &yk, &vk);
  if (!vi || !vk) return;
  int xs = xi, ys = yi, xe = xk, ye = yk;
  if (xs > xe) {
    int t = xs; xs = xe; xe = t;
    t = ys; ys = ye; ye = t;
  }
  if (lane < 40) {
    int yy = ys + kDotY[lane], xx = xs + kDotX[lane];
    if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) f[yy * a.W + xx] = 0xFFFFFFFFu;
    yy = ye + kDotY[lane];
    xx = xe + kDotX[lane];
    if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) f[yy * a.W + xx] = 0xFFFFFFFFu;
  }
  // The host's Bresenham walk (err = (dx > dy ? dx : -dy) / 2; e2 > -dx steps
  // x, e2 < dy steps y) in closed form, so the wave's lanes draw its pixels in
  // parallel: with dx > dy x steps every iteration and after t steps y has
  // stepped ceil((dy t - e0) / dx) times (e0 = dx / 2; the error stays in
  // [0, dx) + dy t - dx ny(t) >= 0, so the x test always passes); dx <= dy is
  // the mirror (y every step, x ceil((dx t - dy / 2) / dy) times).  The walk
  // ends after max(dx, dy) steps: that many + 1 pixels, all the same value.
  const int dx = abs(xe - xs), sx = xs < xe ? 1 : -1;
  const int dy = abs(ye - ys), sy = ys < ye ? 1 : -1;
  auto ceil_div = [](int n, int d) { return n >= 0 ? (n + d - 1) / d : -((-n) / d); };
  const bool xmajor = dx > dy;
  const int steps = xmajor ? dx : dy;
  for (int t = lane; t <= steps; t += 64) {
    int x, y;
    if (xmajor) {
      x = xs + sx * t;
      y = ys + sy * ceil_div(dy * t - dx / 2, dx);
    } else if (dy > 0) {
      y = ys + sy * t;
      x = xs + sx * ceil_div(dx * t - dy / 2, dy);
    } else {  // (a single point)
      x = xs;
      y = ys;
    }
    pose_setpixel(f, a.W, a.H, x, y);
  }
}

// Labels, one workgroup per (frame, keypoint), after the skeleton (stream
// order).  The host draws them in keypoint order, a later label's cells
// (background zeros included) overwriting an earlier one's: here a pixel of
// label k is written only if no later valid label covers it, so every label of
// every frame draws at once and the result is the ordered one.
__global__ void __launch_bounds__(256) pose_labels_kernel(PoseDrawArgs a) {
  __shared__ int px[64], py[64], fit[64];
  __shared__ int valid[64];
  const int b = blockIdx.x, k = blockIdx.y;
  const int K = a.keypoints;
  for (int j = threadIdx.x; j < K; j += blockDim.x) {
    bool v;
    pose_point(a, b, j, &px[j], &py[j], &v);
    valid[j] = v;
    const char* lab = a.labels + a.label_offs[j];
    int len = 0;
    while (lab[len]) ++len;
    int n = 0;
    while (n < len && px[j] + 9 * n + 8 <= a.W) ++n;
    fit[j] = n;
  }
  __syncthreads();
  if (!valid[k]) return;
  uint32_t* f = a.frames + static_cast<uint64_t>(b) * a.W * a.H;
  const char* lab = a.labels + a.label_offs[k];
  const int ly = max(0, py[k] - 14);
  for (int p = threadIdx.x; p < fit[k] * 13 * 8; p += blockDim.x) {
    const int ch = p / 104, rem = p % 104, row = rem / 8, col = rem % 8;
    const int yy = ly + row, xx = px[k] + 9 * ch + col;
    if (yy >= a.H || xx >= a.W) continue;
    bool later = false;
    for (int j = k + 1; j < K && !later; ++j) {
      if (!valid[j]) continue;
      const int jy = max(0, py[j] - 14), dxj = xx - px[j];
      later = yy >= jy && yy < jy + 13 && dxj >= 0 && dxj < 9 * fit[j] && dxj % 9 < 8;
    }
    if (!later)
      f[yy * a.W + xx] = font::cell_on(kFontPose, static_cast<unsigned char>(lab[ch]), row, col) ? 0xFFFFFFFFu : 0u;
  }
}

// ------------------------------------------------ bilinear (align_corners) ----
// Source taps of output index dst for an in -> out resize with align_corners
// (the rule of PyTorch's upsample_bilinear2d: src = dst * (in-1)/(out-1) in
// fp32, i1 = i0 + 1 clamped at the last row/column).
struct BilinearTap {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ BilinearTap bilinear_tap(int dst, int in, int out) {
  const float scale = out > 1 ? static_cast<float>(in - 1) / static_cast<float>(out - 1) : 0.f;
  const float src = scale * static_cast<float>(dst);
  const int i0 = min(static_cast<int>(src), in - 1);
  const float l1 = src - static_cast<float>(i0);
  return BilinearTap{i0, i0 + (i0 < in - 1 ? 1 : 0), 1.f - l1, l1};
}
__device__ __forceinline__ float bilinear_mix(const BilinearTap& ty, const BilinearTap& tx, float v00, float v01,
                                              float v10, float v11) {
  return ty.l0 * (tx.l0 * v00 + tx.l1 * v01) + ty.l1 * (tx.l0 * v10 + tx.l1 * v11);
}

// upsample + argmax + colour in one pass: one workgroup per (output row, frame)
// stages the two source rows of label scores ([w][L] each, e.g. 33 x 21 floats
// for DeepLab at output stride 16) in LDS; each lane then interpolates its
// output pixel's L scores and keeps the first maximum.  The full-resolution
// score map (H x W x L floats) is never written.  (23 us for DeepLab b8's 8 x
// 513 x 513 x 21.  Measured slower and dropped: 8-row workgroups with the
// vertical mix staged once in LDS, 33 us; a lane per run of 16 columns with its
// four label vectors in registers, 52 us (64-B-strided stores); a lane per column
// and run of 8-16 rows, horizontal mix hoisted per run, max + equality argmax,
// 32-37 us.)
template <bool LDS>
__global__ void __launch_bounds__(256) seg_upsample_argmax_kernel(const float* __restrict__ logits, int h, int w,
                                                                  int L, int H, int W, uint32_t rgb_mod, float thr,
                                                                  uint32_t* __restrict__ out) {
  extern __shared__ float rows[];  // [2][w * L]
  const int Y = blockIdx.x, b = blockIdx.y;
  const BilinearTap ty = bilinear_tap(Y, h, H);
  const int n = w * L;
  const float* src = logits + static_cast<int64_t>(b) * h * n;
  const float* r0 = src + static_cast<int64_t>(ty.i0) * n;
  const float* r1 = src + static_cast<int64_t>(ty.i1) * n;
  if constexpr (LDS) {
    for (int i = threadIdx.x; i < n; i += 256) {
      rows[i] = r0[i];
      rows[n + i] = r1[i];
    }
    __syncthreads();
    r0 = rows;
    r1 = rows + n;
  }
  uint32_t* o = out + (static_cast<int64_t>(b) * H + Y) * W;
  for (int X = threadIdx.x; X < W; X += 256) {
    const BilinearTap tx = bilinear_tap(X, w, W);
    const float* a0 = r0 + tx.i0 * L;
    const float* a1 = r0 + tx.i1 * L;
    const float* c0 = r1 + tx.i0 * L;
    const float* c1 = r1 + tx.i1 * L;
    float best = bilinear_mix(ty, tx, a0[0], a1[0], c0[0], c1[0]);
    int bi = 0;
    for (int l = 1; l < L; ++l) {
      const float v = bilinear_mix(ty, tx, a0[l], a1[l], c0[l], c1[l]);
      if (v > best) {
        best = v;
        bi = l;
      }
    }
    o[X] = best > thr ? label_color(static_cast<uint32_t>(bi), rgb_mod) : 0u;
  }
}

// plain NHWC bilinear resize (align_corners): grid (row chunks of W*C, H, B)
__global__ void __launch_bounds__(256) upsample_bilinear_nhwc_kernel(const float* __restrict__ x, int h, int w,
                                                                     int C, int H, int W, float* __restrict__ y) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= W * C) return;
  const int Y = blockIdx.y, b = blockIdx.z;
  const int X = j / C, c = j - X * C;
  const BilinearTap ty = bilinear_tap(Y, h, H), tx = bilinear_tap(X, w, W);
  const float* src = x + static_cast<int64_t>(b) * h * w * C + c;
  const float* r0 = src + static_cast<int64_t>(ty.i0) * w * C;
  const float* r1 = src + static_cast<int64_t>(ty.i1) * w * C;
  y[(static_cast<int64_t>(b) * H + Y) * W * C + j] =
      bilinear_mix(ty, tx, r0[tx.i0 * C], r0[tx.i1 * C], r1[tx.i0 * C], r1[tx.i1 * C]);
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

void pose_draw(const PoseDrawArgs& a, int batch, hipStream_t s) {
  if (batch == 0) return;
  if (a.keypoints > 64) throw std::invalid_argument("pose_draw: at most 64 keypoints");
  if (a.n_edges > 0)
    hipLaunchKernelGGL(pose_lines_kernel, dim3(static_cast<unsigned>(batch), static_cast<unsigned>((a.n_edges + 3) / 4)),
                       dim3(256), 0, s, a);
  hipLaunchKernelGGL(pose_labels_kernel, dim3(static_cast<unsigned>(batch), static_cast<unsigned>(a.keypoints)),
                     dim3(256), 0, s, a);
}

void segment_upsample_argmax_color(const float* logits, int labels, int h, int w, int batch, int H, int W,
                                   uint32_t rgb_modifier, float threshold, uint32_t* out, hipStream_t s) {
  if (batch == 0 || H == 0 || W == 0) return;
  const size_t lds = 2 * static_cast<size_t>(w) * labels * sizeof(float);
  if (lds <= 64 * 1024)
    hipLaunchKernelGGL(seg_upsample_argmax_kernel<true>, dim3(H, batch), dim3(256), lds, s, logits, h, w, labels, H, W,
                       rgb_modifier, threshold, out);
  else
    hipLaunchKernelGGL(seg_upsample_argmax_kernel<false>, dim3(H, batch), dim3(256), 0, s, logits, h, w, labels, H, W,
                       rgb_modifier, threshold, out);
}

void upsample_bilinear_nhwc(const float* x, int batch, int h, int w, int C, int H, int W, float* y, hipStream_t s) {
  if (batch == 0 || H == 0 || W == 0 || C == 0) return;
  hipLaunchKernelGGL(upsample_bilinear_nhwc_kernel, dim3((W * C + 255) / 256, H, batch), dim3(256), 0, s, x, h, w, C,
                     H, W, y);
}

}  // namespace kernels
}  // namespace nnsx
