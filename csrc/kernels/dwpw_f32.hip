// Depthwise-separable conv pairs as one fp32 MFMA GEMM (dwpw_f32): y =
// act(pw(relu6(dw3x3_s(x) + bd)) + bias), the depthwise conv computed inside
// the GEMM's A-operand staging -- its output never exists in HBM.  One
// grouped launch may carry several independent problems (up to 16).
//
// Users:
//   * MobileNetV1 (PoseNet, BASELINE config 5): each of the 13 dw (stride 1|2)
//     + pw pairs is one launch instead of two, and the heatmap / offset 1x1
//     heads (no depthwise) one grouped launch writing their exact columns;
//   * SSDLite prediction heads (config 3), below.
//
// SSDLite prediction heads in one launch: every box / class head of every
// feature map -- depthwise 3x3 + BN + ReLU6, then the 1x1 predictor conv +
// bias -- as ONE grouped GEMM.
//
// The reference runs these heads inside the TFLite / PyTorch model it is handed
// (SSD box encodings + class logits feeding tensordec-boundingbox.c:1158-1221);
// a plain implementation is 2 kernels per head (24 launches for SSDLite's 6
// feature maps x {box, class}), each depthwise output making a round trip
// through HBM and the small maps (5x5 .. 1x1) running 4-20 us of pure launch and
// tail.  Here:
//   * one workgroup = one 64 x 64 output tile of one head (the tile list of all
//     heads is concatenated: blockIdx -> (head, m tile, n tile));
//   * per 32-channel k stage the workgroup computes the depthwise output of its
//     64 pixels x 32 channels straight from the NHWC feature map (9 taps per
//     element, the image's zero padding by masking; a tile may span images) into
//     the B-operand LDS image, and stages the 64 x 32 predictor weights beside it;
//   * MFMA v_mfma_f32_16x16x4_f32 (exact fp32 products), 2 x 2 waves of 32 x 32;
//   * the epilogue adds the bias and writes the head's rows of the concatenated
//     [B][anchors][C] output (box encodings / class logits), as the decoder reads them.
// Operand layout and LDS swizzle as pw_gemm_f32 (mbv2_f32.hip); tiles BM x BN
// = 64 x 64 or 64 x 128 (4 waves of 32 x BN/2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>

#include "kernels/mbv2.h"

namespace nnsx {
namespace kernels {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int HKT = 32;       // k per stage
constexpr int HKQ = HKT / 4;  // k-quads per stage

__device__ __forceinline__ f32x4_t hmfma_k16(f32x4_t a, f32x4_t b, f32x4_t c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
}

__device__ __forceinline__ float relu6f(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

template <int BN>
__global__ void __launch_bounds__(256) dwpw_f32_kernel(SepHeadsArgs args) {
  constexpr int BM = 64, RN = BN / 32, VW = BN * HKQ / 256;
  __shared__ __attribute__((aligned(16))) float xs[2][HKQ][BM][4];
  __shared__ __attribute__((aligned(16))) float ws[2][HKQ][BN][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 15, g = lane >> 4;
  const f32x4_t zero = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- which problem / tile (problems in order; the big ones first keeps the tail short)
  int h = 0, t = static_cast<int>(blockIdx.x);
  while (h + 1 < args.n && t >= args.h[h].tiles) {
    t -= args.h[h].tiles;
    ++h;
  }
  const SepHead& P = args.h[h];
  const int ntn = (P.N + BN - 1) / BN;
  const int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;
  const int Ho = P.Ho, Wo = P.Wo, HWo = Ho * Wo;
  const int M = P.B * HWo;
  const int nk = (P.K + HKT - 1) / HKT;
  const bool dw = P.wd != nullptr;

  // this thread's two staged A elements per stage: (row, k-quad) v = tid + i*256
  int pb[2], py[2], px[2];
  bool pok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + i * 256, row = v >> 3;
    const int p = m0 + row;
    pok[i] = p < M;
    const int pp = pok[i] ? p : 0;
    pb[i] = pp / HWo;
    const int r = pp - pb[i] * HWo;
    py[i] = r / Wo;
    px[i] = r - py[i] * Wo;
  }

  f32x4_t dv[2], wv[VW];
  // A: depthwise 3x3 (stride S, padding 1) + bias + ReLU6 of this thread's
  // elements at k stage k0 (or the plain input without a depthwise); B: the
  // stage's pointwise weights.  Registers; stored to LDS by lstore.
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + i * 256, kq = v & 7;
      const int k = k0 + kq * 4;
      f32x4_t acc = zero;
      if (pok[i] && k < P.K) {
        const float* xb = P.x + static_cast<int64_t>(pb[i]) * P.H * P.W * P.K + k;
        if (!dw) {
          acc = *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(py[i] * P.W + px[i]) * P.K);
        } else {
          acc = *reinterpret_cast<const f32x4_t*>(P.bd + k);
          const int D = P.dil;
          const int iy = py[i] * P.stride - D, ix = px[i] * P.stride - D;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            const int yy = iy + ky * D;
            if (yy < 0 || yy >= P.H) continue;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const int xx = ix + kx * D;
              if (xx < 0 || xx >= P.W) continue;
              const f32x4_t xv = *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(yy * P.W + xx) * P.K);
              const f32x4_t w4 = *reinterpret_cast<const f32x4_t*>(P.wd + (ky * 3 + kx) * P.K + k);
              acc = __builtin_elementwise_fma(xv, w4, acc);
            }
          }
          acc = f32x4_t{relu6f(acc[0]), relu6f(acc[1]), relu6f(acc[2]), relu6f(acc[3])};
        }
      }
      dv[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const int v = tid + i * 256, kq = v & 7, n = n0 + (v >> 3);
      const int k = k0 + kq * 4;
      wv[i] = (n < P.Npad && k < P.Kpad) ? *reinterpret_cast<const f32x4_t*>(P.wt + static_cast<int64_t>(n) * P.Kpad + k)
                                         : zero;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + i * 256, kq = v & 7, row = v >> 3;
      *reinterpret_cast<f32x4_t*>(&xs[buf][kq][row ^ kq][0]) = dv[i];
    }
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const int v = tid + i * 256, kq = v & 7, row = v >> 3;
      *reinterpret_cast<f32x4_t*>(&ws[buf][kq][row ^ kq][0]) = wv[i];
    }
  };

  f32x4_t acc[2][RN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = zero;

  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) gload((ks + 1) * HKT);  // next stage's depthwise + weights during this stage's MFMAs
#pragma unroll
    for (int s = 0; s < HKT / 16; ++s) {
      const int kq = 4 * s + g;
      f32x4_t a[RN], b[2];
#pragma unroll
      for (int j = 0; j < RN; ++j)
        a[j] = *reinterpret_cast<const f32x4_t*>(&ws[buf][kq][(wn * (BN / 2) + j * 16 + li) ^ kq][0]);
#pragma unroll
      for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const f32x4_t*>(&xs[buf][kq][(wm * 32 + i * 16 + li) ^ kq][0]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = hmfma_k16(a[j], b[i], acc[i][j]);
    }
    if (ks + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: + bias (+ act) -> out[b * bstride + q * ldo + n] (NHWC: ldo =
  // N; the SSD heads: the rows of the concatenated [B][anchors][C] output)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 32 + i * 16 + li;
    if (m >= M) continue;
    const int b = m / HWo, q = m - b * HWo;
    float* orow = P.out + static_cast<int64_t>(b) * P.bstride + static_cast<int64_t>(q) * P.ldo;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + g * 4;
      if (n >= P.N) continue;
      f32x4_t v = acc[i][j] + *reinterpret_cast<const f32x4_t*>(P.bias + n);
      if (P.res) {  // (an inverted residual's skip: NHWC, the output's layout, N % 4 == 0)
        const float* rrow = P.res + static_cast<int64_t>(b) * P.bstride + static_cast<int64_t>(q) * P.ldo;
        v += *reinterpret_cast<const f32x4_t*>(rrow + n);
      }
      if (P.act == 1) v = f32x4_t{relu6f(v[0]), relu6f(v[1]), relu6f(v[2]), relu6f(v[3])};
      if (n + 4 <= P.N && (P.ldo & 3) == 0) {
        *reinterpret_cast<f32x4_t*>(orow + n) = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < P.N) orow[n + r] = v[r];
      }
    }
  }
}

}  // namespace

// one launch over every problem of `a`; BN = 128 when every problem is at
// least 128 wide (fewer depthwise recomputations per pixel), else 64
void dwpw_f32(SepHeadsArgs a, hipStream_t s) {
  if (a.n <= 0 || a.n > kSepHeadsMax) throw std::invalid_argument("dwpw_f32: 1..16 problems");
  // 128-wide tiles recompute the depthwise half as often; worth it where the
  // N padding stays small
  bool wide = true;
  for (int i = 0; i < a.n; ++i) wide = wide && (a.h[i].N >= 512 || a.h[i].N % 128 == 0);
  const int BN = wide ? 128 : 64;
  int64_t tiles = 0;
  for (int i = 0; i < a.n; ++i) {
    SepHead& h = a.h[i];
    if (h.stride != 1 && h.stride != 2) throw std::invalid_argument("dwpw_f32: stride 1 or 2");
    if (h.dil < 1) throw std::invalid_argument("dwpw_f32: dilation >= 1");
    if (h.res && (h.N % 4 || (h.ldo > 0 && h.ldo != h.N))) throw std::invalid_argument("dwpw_f32: residual needs NHWC, N % 4");
    if (h.Ho <= 0) h.Ho = (h.H - 1) / h.stride + 1;
    if (h.Wo <= 0) h.Wo = (h.W - 1) / h.stride + 1;
    if (!h.wd && (h.stride != 1 || h.Ho != h.H || h.Wo != h.W))
      throw std::invalid_argument("dwpw_f32: a problem without a depthwise keeps the map");
    if (h.ldo <= 0) h.ldo = h.N;
    if (h.K % 4 || h.Kpad < h.K || h.Kpad % 4 || h.Npad < (h.N + 3) / 4 * 4)
      throw std::invalid_argument("dwpw_f32: K % 4, Kpad >= K, Npad >= N rounded to 4");
    const int64_t M = static_cast<int64_t>(h.B) * h.Ho * h.Wo;
    h.tiles = static_cast<int>(((M + 63) / 64) * ((h.N + BN - 1) / BN));
    tiles += h.tiles;
  }
  if (tiles <= 0) return;
  if (wide)
    hipLaunchKernelGGL(dwpw_f32_kernel<128>, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(dwpw_f32_kernel<64>, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, s, a);
}

void sep_heads_f32(SepHeadsArgs a, hipStream_t s) { dwpw_f32(a, s); }

}  // namespace kernels
}  // namespace nnsx
