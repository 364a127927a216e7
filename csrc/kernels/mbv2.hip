// MobileNetV2 inference kernels for gfx950 (bf16 NHWC activations, BN folded).
//
// The model in the reference runs through tensor_filter framework=pytorch
// (MIOpen).  On MI355X that path spends ~30% of its time in a naive fp64
// depthwise convolution; these kernels replace every layer:
//
//  * pw_gemm   1x1 convolution / FC as an MFMA GEMM (v_mfma_f32_16x16x32_bf16)
//              with bias + ReLU6 + residual fused in the epilogue.  Computed
//              transposed (D^T = W^T X^T) so each lane owns 4 consecutive
//              output channels -> 8-byte NHWC stores.  Tile per wave: 32 pixels
//              x 64 channels; 4 waves per block stacked along pixels.
//  * dw3x3     depthwise 3x3 (stride 1/2, pad 1) + bias + ReLU6: one lane per
//              pixel x 8 channels, 16-byte loads/stores (bandwidth bound).
//  * stem      3x3/2 conv 3->32 on the f32 NHWC frame + bias + ReLU6 -> bf16.
//  * avgpool   global average pool [B,HW,C] -> [B,C].
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/mbv2.h"

namespace nnsx {
namespace kernels {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_mfma __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round-nearest-even (inputs are finite)
  return static_cast<uint16_t>(u >> 16);
}
// two floats -> packed bf16 pair (lo = a), round-to-nearest-even: one v_cvt_pk_bf16_f32 on gfx950
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, b2v));
}

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return fminf(fmaxf(v, 0.f), 6.f);  // ReLU6
  if (act == 2) return fmaxf(v, 0.f);                // ReLU
  return v;
}

// ------------------------------------------------------------------ pw_gemm ----
constexpr int PW_RM = 2;   // 16-pixel tiles per wave
constexpr int PW_RN = 4;   // 16-channel tiles per wave
constexpr int PW_WAVES = 4;
constexpr int PW_BM = PW_WAVES * PW_RM * 16;  // 128 pixels per block
constexpr int PW_BN = PW_RN * 16;             // 64 channels per block

template <bool OUT_F32>
__global__ void __launch_bounds__(256) pw_gemm_kernel(const uint16_t* __restrict__ x,   // [M][K]
                                                      const uint16_t* __restrict__ wt,  // [Npad][Kpad]
                                                      const float* __restrict__ bias,   // [N]
                                                      const uint16_t* __restrict__ res, // [M][N] or null
                                                      void* __restrict__ y,             // [M][N]
                                                      int M, int N, int K, int Kpad, int act) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int m_base = blockIdx.x * PW_BM + wave * (PW_RM * 16);
  const int n_base = blockIdx.y * PW_BN;
  const int li = lane & 15;       // row within a 16-tile
  const int kq = (lane >> 4) * 8;  // k offset of this lane's 8-element chunk

  f32x4_t acc[PW_RM][PW_RN];
#pragma unroll
  for (int i = 0; i < PW_RM; ++i)
#pragma unroll
    for (int j = 0; j < PW_RN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // row pointers (clamped rows read row 0 and are masked at the store)
  const uint16_t* xrow[PW_RM];
#pragma unroll
  for (int i = 0; i < PW_RM; ++i) {
    int m = m_base + i * 16 + li;
    xrow[i] = x + static_cast<int64_t>(m < M ? m : 0) * K;
  }
  const uint16_t* wrow[PW_RN];
#pragma unroll
  for (int j = 0; j < PW_RN; ++j) wrow[j] = wt + static_cast<int64_t>(n_base + j * 16 + li) * Kpad;

  for (int k0 = 0; k0 < Kpad; k0 += 32) {
    const int k = k0 + kq;
    bf16x8_t bfrag[PW_RM];
#pragma unroll
    for (int i = 0; i < PW_RM; ++i) {
      if (k < K)
        bfrag[i] = *reinterpret_cast<const bf16x8_t*>(xrow[i] + k);
      else
        bfrag[i] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
    bf16x8_t afrag[PW_RN];
#pragma unroll
    for (int j = 0; j < PW_RN; ++j) afrag[j] = *reinterpret_cast<const bf16x8_t*>(wrow[j] + k);
#pragma unroll
    for (int i = 0; i < PW_RM; ++i)
#pragma unroll
      for (int j = 0; j < PW_RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, afrag[j]),
                                                            __builtin_bit_cast(bf16x8_mfma, bfrag[i]), acc[i][j],
                                                            0, 0, 0);
  }

  // epilogue: lane owns channels n..n+3 of pixel m
#pragma unroll
  for (int i = 0; i < PW_RM; ++i) {
    const int m = m_base + i * 16 + li;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < PW_RN; ++j) {
      const int n = n_base + j * 16 + (lane >> 4) * 4;
      if (n >= N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[n + r];
      if (res) {
        uint2 rr = *reinterpret_cast<const uint2*>(res + static_cast<int64_t>(m) * N + n);
        v[0] += bf2f(rr.x & 0xffff);
        v[1] += bf2f(rr.x >> 16);
        v[2] += bf2f(rr.y & 0xffff);
        v[3] += bf2f(rr.y >> 16);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
      if (OUT_F32) {
        float4 o{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<float4*>(static_cast<float*>(y) + static_cast<int64_t>(m) * N + n) = o;
      } else {
        uint2 o;
        o.x = pk_bf16(v[0], v[1]);
        o.y = pk_bf16(v[2], v[3]);
        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(y) + static_cast<int64_t>(m) * N + n) = o;
      }
    }
  }
}

// -------------------------------------------------------------------- dw3x3 ----
__global__ void __launch_bounds__(256) dw3x3_kernel(const uint16_t* __restrict__ x,  // [B][H][W][C]
                                                    const uint16_t* __restrict__ w,  // [9][C]
                                                    const float* __restrict__ bias,  // [C]
                                                    uint16_t* __restrict__ y,        // [B][Ho][Wo][C]
                                                    int B, int H, int W, int C, int Ho, int Wo, int stride,
                                                    int dil, int act) {
  const int cg = C >> 3;
  const int64_t total = static_cast<int64_t>(B) * Ho * Wo * cg;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(t % cg);
    int64_t p = t / cg;
    const int ox = static_cast<int>(p % Wo);
    p /= Wo;
    const int oy = static_cast<int>(p % Ho);
    const int b = static_cast<int>(p / Ho);
    const int c = c8 * 8;
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = bias[c + q];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * stride - dil + ky * dil;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * stride - dil + kx * dil;
        if (ix < 0 || ix >= W) continue;
        const uint4 xv = *reinterpret_cast<const uint4*>(x + ((static_cast<int64_t>(b) * H + iy) * W + ix) * C + c);
        const uint4 wv = *reinterpret_cast<const uint4*>(w + (ky * 3 + kx) * C + c);
        const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w};
        const uint32_t ws[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[2 * q] += bf2f(xs[q] & 0xffff) * bf2f(ws[q] & 0xffff);
          acc[2 * q + 1] += bf2f(xs[q] >> 16) * bf2f(ws[q] >> 16);
        }
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = pk_bf16(act_fn(acc[2 * q], act), act_fn(acc[2 * q + 1], act));
    *reinterpret_cast<uint4*>(y + ((static_cast<int64_t>(b) * Ho + oy) * Wo + ox) * C + c) = uint4{o[0], o[1], o[2], o[3]};
  }
}

// --------------------------------------------------------------------- stem ----
// x: f32 [B][H][W][3]; w: f32 [3][3][3][32] (ky,kx,ci,co); y: bf16 [B][Ho][Wo][32]
// T = float: the normalised frame; T = uint8_t: the raw RGB frame, normalised on
// the fly through a 256-entry LUT lut[u] = (u + add) / div (bit-identical to the
// tensor_transform arithmetic it replaces, padding stays 0 in the normalised domain)
template <typename T>
__global__ void __launch_bounds__(256) stem_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ bias, uint16_t* __restrict__ y, int B,
                                                   int H, int W, int Ho, int Wo, int act, float add, float div) {
  __shared__ float sw[27 * 32];
  __shared__ float sb[32];
  __shared__ float lut[256];
  for (int i = threadIdx.x; i < 27 * 32; i += blockDim.x) sw[i] = w[i];
  if (threadIdx.x < 32) sb[threadIdx.x] = bias[threadIdx.x];
  if (sizeof(T) == 1) lut[threadIdx.x] = (static_cast<float>(threadIdx.x) + add) / div;
  __syncthreads();
  const int64_t total = static_cast<int64_t>(B) * Ho * Wo * 4;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int og = static_cast<int>(t & 3);  // 8-channel output group
    int64_t p = t >> 2;
    const int ox = static_cast<int>(p % Wo);
    p /= Wo;
    const int oy = static_cast<int>(p % Ho);
    const int b = static_cast<int>(p / Ho);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = sb[og * 8 + q];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * 2 - 1 + ky;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * 2 - 1 + kx;
        if (ix < 0 || ix >= W) continue;
        const T* px = x + ((static_cast<int64_t>(b) * H + iy) * W + ix) * 3;
        float in0, in1, in2;
        if (sizeof(T) == 1) {
          in0 = lut[static_cast<int>(px[0])];
          in1 = lut[static_cast<int>(px[1])];
          in2 = lut[static_cast<int>(px[2])];
        } else {
          in0 = static_cast<float>(px[0]);
          in1 = static_cast<float>(px[1]);
          in2 = static_cast<float>(px[2]);
        }
        const float* wk = sw + ((ky * 3 + kx) * 3) * 32 + og * 8;
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += in0 * wk[q] + in1 * wk[32 + q] + in2 * wk[64 + q];
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = pk_bf16(act_fn(acc[2 * q], act), act_fn(acc[2 * q + 1], act));
    *reinterpret_cast<uint4*>(y + ((static_cast<int64_t>(b) * Ho + oy) * Wo + ox) * 32 + og * 8) = uint4{o[0], o[1], o[2], o[3]};
  }
}

// ------------------------------------------------------------------ avgpool ----
__global__ void __launch_bounds__(256) avgpool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B,
                                                      int HW, int C) {
  const int cg = C >> 3;
  const int64_t total = static_cast<int64_t>(B) * cg;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(t % cg) * 8;
    const int b = static_cast<int>(t / cg);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < HW; ++p) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + (static_cast<int64_t>(b) * HW + p) * C + c);
      const uint32_t vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += bf2f(vs[q] & 0xffff);
        acc[2 * q + 1] += bf2f(vs[q] >> 16);
      }
    }
    const float inv = 1.f / HW;
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = pk_bf16(acc[2 * q] * inv, acc[2 * q + 1] * inv);
    *reinterpret_cast<uint4*>(y + static_cast<int64_t>(b) * C + c) = uint4{o[0], o[1], o[2], o[3]};
  }
}

inline unsigned grid_cap(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return static_cast<unsigned>(g);
}

}  // namespace

void pw_gemm(const void* x, const void* wt, const float* bias, const void* res, void* y, int M, int N, int K, int Kpad,
             int act, bool out_f32, hipStream_t s) {
  dim3 grid((M + PW_BM - 1) / PW_BM, (N + PW_BN - 1) / PW_BN);
  if (out_f32)
    hipLaunchKernelGGL(pw_gemm_kernel<true>, grid, dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<const uint16_t*>(wt), bias, static_cast<const uint16_t*>(res), y, M, N, K, Kpad, act);
  else
    hipLaunchKernelGGL(pw_gemm_kernel<false>, grid, dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<const uint16_t*>(wt), bias, static_cast<const uint16_t*>(res), y, M, N, K, Kpad, act);
}

void dw3x3(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int C, int stride, int dil,
           int act, hipStream_t s) {
  // padding == dilation keeps "same" geometry: Ho = (H - 1) / stride + 1
  int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  int64_t work = static_cast<int64_t>(B) * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(dw3x3_kernel, dim3(grid_cap(work)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<const uint16_t*>(w), bias, static_cast<uint16_t*>(y), B, H, W, C, Ho, Wo, stride, dil, act);
}

void stem3x3(const float* x, const float* w, const float* bias, void* y, int B, int H, int W, int act, hipStream_t s) {
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  int64_t work = static_cast<int64_t>(B) * Ho * Wo * 4;
  hipLaunchKernelGGL(stem_kernel<float>, dim3(grid_cap(work)), dim3(256), 0, s, x, w, bias, static_cast<uint16_t*>(y),
                     B, H, W, Ho, Wo, act, 0.f, 1.f);
}

void stem3x3_u8(const uint8_t* x, const float* w, const float* bias, void* y, int B, int H, int W, int act, float add,
                float div, hipStream_t s) {
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  int64_t work = static_cast<int64_t>(B) * Ho * Wo * 4;
  hipLaunchKernelGGL(stem_kernel<uint8_t>, dim3(grid_cap(work)), dim3(256), 0, s, x, w, bias,
                     static_cast<uint16_t*>(y), B, H, W, Ho, Wo, act, add, div);
}

void avgpool(const void* x, void* y, int B, int HW, int C, hipStream_t s) {
  int64_t work = static_cast<int64_t>(B) * (C / 8);
  hipLaunchKernelGGL(avgpool_kernel, dim3(grid_cap(work)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<uint16_t*>(y), B, HW, C);
}

}  // namespace kernels
}  // namespace nnsx
