// Detection post-processing kernels for gfx950 (see detect.h).
//
// Candidate extraction runs one 64-lane wavefront per anchor: the class row is
// read coalesced and __ballot picks the first passing class (SSD) or a wave
// max-reduction picks the best class (YOLO).  Each frame's candidates are then
// sorted by a workgroup bitonic sort in LDS (global-memory fallback for very
// large candidate sets), the pairwise IoU bit matrix is computed row-parallel,
// and one wavefront performs the greedy suppression scan with the "removed"
// bitset held one 64-bit word per lane -- the exact greedy NMS of the
// reference (tensordec-boundingbox.c:1215-1262) in O(n) wave steps.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "decoders/font.h"
#include "kernels/detect.h"

namespace nnsx {
namespace kernels {

namespace {

__constant__ uint8_t kFontDev[95][13] = NNSX_FONT8X13_DATA;

constexpr int kLdsKeys = 8192;  // 64 KiB of keys per workgroup

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

// exp as the host decoder computes it (glibc expf, correctly rounded in
// practice): the fp64 exp rounded once to fp32, so device and host boxes
// truncate to the same integers
__device__ inline float exp_ref(float x) { return static_cast<float>(exp(static_cast<double>(x))); }

// sort keys that keep the input order (modes drawn without NMS)
__device__ inline uint64_t order_key(int anchor) { return static_cast<uint32_t>(anchor); }

__device__ inline uint64_t make_key(float score, int anchor) {
  // ascending key order == score descending, anchor ascending (stable sort order)
  return (static_cast<uint64_t>(~__float_as_uint(score)) << 32) | static_cast<uint32_t>(anchor);
}

__global__ void __launch_bounds__(256) ssd_cand_kernel(const float* __restrict__ boxes,
                                                       const float* __restrict__ scores,
                                                       const float* __restrict__ priors, int c, SsdParams p,
                                                       DetScratch s) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int n = s.n;
  if (a >= n) return;
  const float* det = scores + (static_cast<size_t>(b) * n + a) * c;
  int found = -1;
  for (int base = 1; base < c; base += 64) {
    const int cl = base + lane;
    const bool hit = cl < c && det[cl] >= p.sigmoid_threshold;
    const unsigned long long m = __ballot(hit);
    if (m) {
      found = base + __ffsll(m) - 1;
      break;
    }
  }
  if (found < 0 || lane != 0) return;
  const float* bx = boxes + (static_cast<size_t>(b) * n + a) * 4;
  const float score = 1.f / (1.f + exp_ref(-det[found]));
  const float py = priors[a], px = priors[n + a], ph = priors[2 * n + a], pw = priors[3 * n + a];
  const float ycenter = bx[0] / p.y_scale * ph + py;
  const float xcenter = bx[1] / p.x_scale * pw + px;
  const float h = exp_ref(bx[2] / p.h_scale) * ph;
  const float w = exp_ref(bx[3] / p.w_scale) * pw;
  const float ymin = ycenter - h / 2.f;
  const float xmin = xcenter - w / 2.f;
  const int x = static_cast<int>(xmin * p.i_width);
  const int y = static_cast<int>(ymin * p.i_height);
  const int bw = static_cast<int>(w * p.i_width);
  const int bh = static_cast<int>(h * p.i_height);
  const size_t o = static_cast<size_t>(b) * n + a;
  s.box[o] = make_int4(max(0, x), max(0, y), bw, bh);
  s.cls[o] = found;
  s.prob[o] = score;
  const int slot = atomicAdd(&s.count[b], 1);
  s.keys[static_cast<size_t>(b) * s.key_cap + slot] = make_key(score, a);
}

__global__ void __launch_bounds__(256) yolo_cand_kernel(const float* __restrict__ in, int classes, float thr,
                                                        int scaled, int iw, int ih, DetScratch s) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int n = s.n;
  if (a >= n) return;
  const int row_len = classes + 5;
  const float* r = in + (static_cast<size_t>(b) * n + a) * row_len;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = lane; c < classes; c += 64) {
    const float v = r[5 + c];
    if (v > best) {
      best = v;
      bi = c;
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
  if (lane != 0) return;
  const float score = best * r[4];
  if (!(score > thr)) return;
  float cx = r[0], cy = r[1], w = r[2], h = r[3];
  if (!scaled) {
    cx *= static_cast<float>(iw);
    cy *= static_cast<float>(ih);
    w *= static_cast<float>(iw);
    h *= static_cast<float>(ih);
  }
  const size_t o = static_cast<size_t>(b) * n + a;
  s.box[o] = make_int4(static_cast<int>(fmaxf(0.f, cx - w / 2.f)), static_cast<int>(fmaxf(0.f, cy - h / 2.f)),
                       static_cast<int>(fminf(static_cast<float>(iw), w)),
                       static_cast<int>(fminf(static_cast<float>(ih), h)));
  s.cls[o] = bi;
  s.prob[o] = score;
  const int slot = atomicAdd(&s.count[b], 1);
  s.keys[static_cast<size_t>(b) * s.key_cap + slot] = make_key(score, a);
}

// mobilenet-ssd-postprocess / tf-ssd (K10, tensordec-boundingbox.c:1309-1341):
// the model already ran NMS; every detection d < num with score >= threshold
// is drawn, in input order.  Float32 arithmetic as the host path.
__global__ void __launch_bounds__(256) pp_cand_kernel(const float* __restrict__ loc, const float* __restrict__ cls,
                                                      const float* __restrict__ score, const float* __restrict__ num,
                                                      int bpi, float thr, int iw, int ih, DetScratch s) {
#pragma clang fp contract(off)
  const int d = blockIdx.x * 256 + threadIdx.x;
  const int n = min(static_cast<int>(num[0]), s.n);
  if (d >= n) return;
  const float sc = score[d];
  if (sc < thr) return;
  auto c01 = [](float v) { return fminf(fmaxf(v, 0.f), 1.f); };
  const float* b = loc + static_cast<size_t>(d) * bpi;
  const float y1 = c01(b[0]), x1 = c01(b[1]), y2 = c01(b[2]), x2 = c01(b[3]);
  s.box[d] = make_int4(static_cast<int>(x1 * static_cast<float>(iw)), static_cast<int>(y1 * static_cast<float>(ih)),
                       static_cast<int>((x2 - x1) * static_cast<float>(iw)),
                       static_cast<int>((y2 - y1) * static_cast<float>(ih)));
  s.cls[d] = static_cast<int>(cls[d]);
  s.prob[d] = sc;
  const int slot = atomicAdd(&s.count[0], 1);
  s.keys[slot] = order_key(d);
}

// ov-person-detection / ov-face-detection: [200][7] rows (image_id, label,
// conf, x_min, y_min, x_max, y_max); the list ends at the first negative
// image_id; rows with conf >= 0.8 are drawn in order (fp64 box math as the
// host path).  One workgroup: the end marker is a workgroup min-reduction.
__global__ void __launch_bounds__(256) ov_cand_kernel(const float* __restrict__ in, int rows, float conf, int iw,
                                                      int ih, DetScratch s) {
  __shared__ int first_end;
  const int d = threadIdx.x;
  if (d == 0) first_end = rows;
  __syncthreads();
  const float* r = in + static_cast<size_t>(d) * 7;
  if (d < rows && static_cast<int>(static_cast<double>(r[0])) < 0) atomicMin(&first_end, d);
  __syncthreads();
  if (d >= first_end || d >= rows) return;
  if (static_cast<double>(r[2]) < static_cast<double>(conf)) return;
  const double x0 = r[3], y0 = r[4], x1 = r[5], y1 = r[6];
  s.box[d] = make_int4(static_cast<int>(x0 * iw), static_cast<int>(y0 * ih), static_cast<int>((x1 - x0) * iw),
                       static_cast<int>((y1 - y0) * ih));
  s.cls[d] = -1;
  s.prob[d] = 1.f;
  const int slot = atomicAdd(&s.count[0], 1);
  s.keys[slot] = order_key(d);
}

// mp-palm-detection (K12, tensordec-boundingbox.c:1407-1451): sigmoid of the
// clamped logit, anchor-relative box; NMS at IoU 0.05 follows.
__global__ void __launch_bounds__(256) palm_cand_kernel(const float* __restrict__ boxes,
                                                        const float* __restrict__ scores,
                                                        const float* __restrict__ anchors, int bpi, float thr, int iw,
                                                        int ih, DetScratch s) {
#pragma clang fp contract(off)
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= s.n) return;
  float sc = fminf(fmaxf(scores[d], -100.f), 100.f);
  sc = 1.0f / (1.0f + exp_ref(-sc));
  if (sc < thr) return;
  const float* a = anchors + static_cast<size_t>(d) * 4;  // xc, yc, w, h
  const float* b = boxes + static_cast<size_t>(d) * bpi;
  const float fw = static_cast<float>(iw), fh = static_cast<float>(ih);
  const float yc = b[0] / fh * a[3] + a[1];
  const float xc = b[1] / fw * a[2] + a[0];
  const float h = b[2] / fh * a[3];
  const float w = b[3] / fw * a[2];
  const float ymin = yc - h / 2.f, xmin = xc - w / 2.f;
  s.box[d] = make_int4(max(0, static_cast<int>(xmin * fw)), max(0, static_cast<int>(ymin * fh)),
                       static_cast<int>(w * fw), static_cast<int>(h * fh));
  s.cls[d] = 0;
  s.prob[d] = sc;
  const int slot = atomicAdd(&s.count[0], 1);
  s.keys[slot] = make_key(sc, d);
}

// modes without NMS: keep every sorted candidate
__global__ void keep_all_kernel(DetScratch s) {
  const int b = blockIdx.x;
  const int n = s.count[b];
  for (int i = threadIdx.x; i < n; i += blockDim.x) s.kept[static_cast<size_t>(b) * s.k + i] = i;
  if (threadIdx.x == 0) s.nkept[b] = n;
}

__device__ void bitonic_sort(uint64_t* a, int m) {
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __threadfence_block();
      __syncthreads();
    }
  }
}

__global__ void __launch_bounds__(1024) sort_kernel(DetScratch s) {
  extern __shared__ uint64_t lds_keys[];
  const int b = blockIdx.x;
  const int count = min(s.count[b], s.n);
  uint64_t* g = s.keys + static_cast<size_t>(b) * s.key_cap;
  int m = 1;
  while (m < count) m <<= 1;
  uint64_t* a;
  if (m <= kLdsKeys) {
    for (int i = threadIdx.x; i < m; i += blockDim.x) lds_keys[i] = i < count ? g[i] : ~0ull;
    a = lds_keys;
  } else {
    for (int i = count + threadIdx.x; i < m; i += blockDim.x) g[i] = ~0ull;
    a = g;
  }
  __threadfence_block();
  __syncthreads();
  if (count > 1) bitonic_sort(a, m);
  const int keep = min(count, s.k);
  for (int i = threadIdx.x; i < keep; i += blockDim.x) {
    const int anchor = static_cast<int>(a[i] & 0xffffffffu);
    const size_t src = static_cast<size_t>(b) * s.n + anchor;
    const size_t dst = static_cast<size_t>(b) * s.k + i;
    s.sbox[dst] = s.box[src];
    s.scls[dst] = s.cls[src];
    s.sprob[dst] = s.prob[src];
  }
  __syncthreads();
  if (threadIdx.x == 0) s.count[b] = keep;
}

__device__ inline float iou_ref(int4 a, int4 b) {
#pragma clang fp contract(off)
  const int x1 = max(a.x, b.x), y1 = max(a.y, b.y);
  const int x2 = min(a.x + a.z, b.x + b.z), y2 = min(a.y + a.w, b.y + b.w);
  const int w = max(0, x2 - x1 + 1), h = max(0, y2 - y1 + 1);
  const float inter = static_cast<float>(w * h);
  const float area_a = static_cast<float>(a.z * a.w);
  const float area_b = static_cast<float>(b.z * b.w);
  const float o = inter / (area_a + area_b - inter);
  return o >= 0 ? o : 0;
}

__global__ void __launch_bounds__(256) nms_mask_kernel(DetScratch s, float thr) {
  const int b = blockIdx.y;
  const int n = s.count[b];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int words = s.k / 64;
  const int4* sb = s.sbox + static_cast<size_t>(b) * s.k;
  const int4 bi = sb[i];
  uint64_t* row = s.mask + (static_cast<size_t>(b) * s.k + i) * words;
  const int nw = (n + 63) / 64;
  for (int w = i / 64; w < nw; ++w) {
    uint64_t bits = 0;
    const int j0 = w * 64;
    const int j1 = min(n, j0 + 64);
    for (int j = max(j0, i + 1); j < j1; ++j)
      if (iou_ref(bi, sb[j]) > thr) bits |= 1ull << (j - j0);
    row[w] = bits;
  }
}

__global__ void __launch_bounds__(64) nms_reduce_kernel(DetScratch s) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = s.count[b];
  const int words = s.k / 64;
  const uint64_t* mask = s.mask + static_cast<size_t>(b) * s.k * words;
  int* kept = s.kept + static_cast<size_t>(b) * s.k;
  uint64_t removed = 0;
  int nk = 0;
  const int nw = (n + 63) / 64;
  for (int i = 0; i < n; ++i) {
    const int w = i >> 6;
    const uint64_t rw = __shfl(removed, w, 64);
    if (!((rw >> (i & 63)) & 1ull)) {
      if (lane >= w && lane < nw) removed |= mask[static_cast<size_t>(i) * words + lane];
      if (lane == 0) kept[nk] = i;
      ++nk;
    }
  }
  if (lane == 0) s.nkept[b] = nk;
}

__global__ void __launch_bounds__(256) draw_kernel(DetScratch s, uint32_t* frames, int W, int H, int iw, int ih,
                                                   const char* labels, const int* offs, int n_labels,
                                                   int use_labels, int label_style) {
  const int b = blockIdx.x;
  uint32_t* f = frames + static_cast<size_t>(b) * W * H;
  const int nk = s.nkept[b];
  const int* kept = s.kept + static_cast<size_t>(b) * s.k;
  for (int t = 0; t < nk; ++t) {
    const int idx = kept[t];
    const size_t o = static_cast<size_t>(b) * s.k + idx;
    const int cls = s.scls[o];
    if (use_labels && (cls < 0 || cls >= n_labels)) continue;
    const int4 a = s.sbox[o];
    // box corners on the output surface (reference draw(): integer scaling)
    const int64_t x1 = (static_cast<int64_t>(W) * a.x) / iw;
    const int64_t x2 = min(static_cast<int64_t>(W - 1), (static_cast<int64_t>(W) * (a.x + a.z)) / iw);
    const int64_t y1 = (static_cast<int64_t>(H) * a.y) / ih;
    const int64_t y2 = min(static_cast<int64_t>(H - 1), (static_cast<int64_t>(H) * (a.y + a.w)) / ih);
    // horizontal edges
    for (int64_t x = x1 + threadIdx.x; x <= x2; x += blockDim.x) {
      if (x < 0 || x >= W) continue;
      if (y1 >= 0 && y1 < H) f[y1 * W + x] = font::kPixel;
      if (y2 >= 0 && y2 < H) f[y2 * W + x] = font::kPixel;
    }
    // vertical edges
    for (int64_t y = y1 + 1 + threadIdx.x; y < y2; y += blockDim.x) {
      if (y < 0 || y >= H) continue;
      if (x1 >= 0 && x1 < W) f[y * W + x1] = font::kPixel;
      if (x2 >= 0 && x2 < W) f[y * W + x2] = font::kPixel;
    }
    __syncthreads();
    if (use_labels && label_style != 0) {
      const char* lab = labels + offs[cls];
      int len = 0;
      while (lab[len]) ++len;
      // characters that fit: (x1 + 9*j + 8) <= W
      int fit = 0;
      while (fit < len && x1 + font::kAdvance * fit + 8 <= W) ++fit;
      const int64_t ly = y1 - font::kAboveBox > 0 ? y1 - font::kAboveBox : 0;
      const int pixels = fit * font::kCellH * font::kCellW;
      for (int p = threadIdx.x; p < pixels; p += blockDim.x) {
        const int ch = p / (font::kCellH * font::kCellW);
        const int rem = p % (font::kCellH * font::kCellW);
        const int row = rem / font::kCellW, col = rem % font::kCellW;
        const int64_t yy = ly + row, xx = x1 + font::kAdvance * ch + col;
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
        f[yy * W + xx] =
            (label_style == 2 || font::cell_on(kFontDev, static_cast<unsigned char>(lab[ch]), row, col)) ? font::kPixel
                                                                                                      : 0u;
      }
    }
    __syncthreads();
  }
}

}  // namespace

size_t det_scratch_bytes(int n, int k, int batch) {
  const int key_cap = next_pow2(n);
  size_t t = 0;
  t += align256(sizeof(int) * batch);
  t += align256(sizeof(uint64_t) * static_cast<size_t>(batch) * key_cap);
  t += align256(sizeof(int4) * static_cast<size_t>(batch) * n);
  t += align256(sizeof(int) * static_cast<size_t>(batch) * n);
  t += align256(sizeof(float) * static_cast<size_t>(batch) * n);
  t += align256(sizeof(int4) * static_cast<size_t>(batch) * k);
  t += align256(sizeof(int) * static_cast<size_t>(batch) * k);
  t += align256(sizeof(float) * static_cast<size_t>(batch) * k);
  t += align256(sizeof(uint64_t) * static_cast<size_t>(batch) * k * (k / 64));
  t += align256(sizeof(int) * static_cast<size_t>(batch) * k);
  t += align256(sizeof(int) * batch);
  return t;
}

DetScratch det_scratch_carve(void* base, int n, int k, int batch) {
  DetScratch s;
  s.n = n;
  s.k = k;
  s.key_cap = next_pow2(n);
  char* p = static_cast<char*>(base);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += align256(bytes);
    return r;
  };
  s.count = reinterpret_cast<int*>(take(sizeof(int) * batch));
  s.keys = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * static_cast<size_t>(batch) * s.key_cap));
  s.box = reinterpret_cast<int4*>(take(sizeof(int4) * static_cast<size_t>(batch) * n));
  s.cls = reinterpret_cast<int*>(take(sizeof(int) * static_cast<size_t>(batch) * n));
  s.prob = reinterpret_cast<float*>(take(sizeof(float) * static_cast<size_t>(batch) * n));
  s.sbox = reinterpret_cast<int4*>(take(sizeof(int4) * static_cast<size_t>(batch) * k));
  s.scls = reinterpret_cast<int*>(take(sizeof(int) * static_cast<size_t>(batch) * k));
  s.sprob = reinterpret_cast<float*>(take(sizeof(float) * static_cast<size_t>(batch) * k));
  s.mask = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * static_cast<size_t>(batch) * k * (k / 64)));
  s.kept = reinterpret_cast<int*>(take(sizeof(int) * static_cast<size_t>(batch) * k));
  s.nkept = reinterpret_cast<int*>(take(sizeof(int) * batch));
  return s;
}

void ssd_candidates(const float* boxes, const float* scores, const float* priors, int c, int batch,
                    const SsdParams& p, const DetScratch& s, hipStream_t stream) {
  hipMemsetAsync(s.count, 0, sizeof(int) * batch, stream);
  dim3 grid((s.n + 3) / 4, batch);
  hipLaunchKernelGGL(ssd_cand_kernel, grid, dim3(256), 0, stream, boxes, scores, priors, c, p, s);
}

void yolov5_candidates(const float* in, int classes, int batch, float conf_threshold, int scaled_output,
                       int i_width, int i_height, const DetScratch& s, hipStream_t stream) {
  hipMemsetAsync(s.count, 0, sizeof(int) * batch, stream);
  dim3 grid((s.n + 3) / 4, batch);
  hipLaunchKernelGGL(yolo_cand_kernel, grid, dim3(256), 0, stream, in, classes, conf_threshold, scaled_output,
                     i_width, i_height, s);
}

void pp_candidates(const float* loc, const float* cls, const float* score, const float* num, int bpi, float thr,
                   int i_width, int i_height, const DetScratch& s, hipStream_t stream) {
  hipMemsetAsync(s.count, 0, sizeof(int), stream);
  hipLaunchKernelGGL(pp_cand_kernel, dim3((s.n + 255) / 256), dim3(256), 0, stream, loc, cls, score, num, bpi, thr,
                     i_width, i_height, s);
}

void ov_candidates(const float* in, float conf, int i_width, int i_height, const DetScratch& s, hipStream_t stream) {
  hipMemsetAsync(s.count, 0, sizeof(int), stream);
  hipLaunchKernelGGL(ov_cand_kernel, dim3(1), dim3(256), 0, stream, in, std::min(s.n, 256), conf, i_width, i_height,
                     s);
}

void palm_candidates(const float* boxes, const float* scores, const float* anchors, int bpi, float thr, int i_width,
                     int i_height, const DetScratch& s, hipStream_t stream) {
  hipMemsetAsync(s.count, 0, sizeof(int), stream);
  hipLaunchKernelGGL(palm_cand_kernel, dim3((s.n + 255) / 256), dim3(256), 0, stream, boxes, scores, anchors, bpi,
                     thr, i_width, i_height, s);
}

void sort_keep_all(const DetScratch& s, int batch, hipStream_t stream) {
  const int lds_keys = std::min(s.key_cap, kLdsKeys);
  hipLaunchKernelGGL(sort_kernel, dim3(batch), dim3(1024), sizeof(uint64_t) * lds_keys, stream, s);
  hipLaunchKernelGGL(keep_all_kernel, dim3(batch), dim3(256), 0, stream, s);
}

void sort_nms(const DetScratch& s, int batch, float iou_threshold, hipStream_t stream) {
  const int lds_keys = std::min(s.key_cap, kLdsKeys);
  hipLaunchKernelGGL(sort_kernel, dim3(batch), dim3(1024), sizeof(uint64_t) * lds_keys, stream, s);
  hipLaunchKernelGGL(nms_mask_kernel, dim3((s.k + 255) / 256, batch), dim3(256), 0, stream, s, iou_threshold);
  hipLaunchKernelGGL(nms_reduce_kernel, dim3(batch), dim3(64), 0, stream, s);
}

void draw_boxes(const DetScratch& s, int batch, uint32_t* frames, int width, int height, int i_width,
                int i_height, const char* labels, const int* label_offsets, int n_labels, bool use_labels,
                int label_style, hipStream_t stream) {
  hipLaunchKernelGGL(draw_kernel, dim3(batch), dim3(256), 0, stream, s, frames, width, height, i_width, i_height,
                     labels, label_offsets, n_labels, use_labels ? 1 : 0, label_style);
}

}  // namespace kernels
}  // namespace nnsx
