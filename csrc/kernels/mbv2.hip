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

#include <cstdlib>

#include <algorithm>
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
                                                      int M, int N, int K, int Kpad, int act,
                                                      int kchunk) {  // k-steps of this grid.z slice
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

  const int kbeg = blockIdx.z * kchunk * 32;
  const int kend = min(Kpad, kbeg + kchunk * 32);
  // unrolled so the loads of 4 k-steps are in flight together (the kernel has
  // no LDS stage: with ~3 waves per SIMD a load -> MFMA chain per k-step left
  // the small 7x7 / classifier GEMMs latency bound)
#pragma unroll 4
  for (int k0 = kbeg; k0 < kend; k0 += 32) {
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
      if (OUT_F32 && gridDim.z > 1) {  // split-K partial sum (fp32, no residual / activation)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          atomicAdd(static_cast<float*>(y) + static_cast<int64_t>(m) * N + n + r,
                    acc[i][j][r] + (blockIdx.z == 0 ? bias[n + r] : 0.f));
        continue;
      }
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

// LDS-staged pointwise GEMM for the large-M layers (7x7 / 14x14 stages, the
// head): the BM x 32 pixel tile and BN x 32 weight tile of each k-step are
// loaded once per workgroup (coalesced 16-B vectors, prefetched into
// registers one k-step ahead, double-buffered LDS, one barrier per k-step) and
// shared by the 2 x 2 waves; each wave computes a (BM/2) x (BN/2) sub-tile.
// The register-direct kernel above re-reads x once per 64-channel block and
// the weights once per wave: ~120 MB of L2 traffic for the 6272 x 320 x 1280
// head GEMM.  LDS rows are 48 bf16 (96 B): fragment reads conflict-free.
constexpr int GP = 48;

template <int BM, int BN, bool OUT_F32>
__global__ void __launch_bounds__(256) pw_gemm_lds_kernel(const uint16_t* __restrict__ x,   // [M][K]
                                                          const uint16_t* __restrict__ wt,  // [Npad][Kpad]
                                                          const float* __restrict__ bias,   // [N]
                                                          const uint16_t* __restrict__ res, // [M][N] or null
                                                          void* __restrict__ y,             // [M][N]
                                                          int M, int N, int K, int Kpad, int Npad, int act) {
  constexpr int RM = BM / 32, RN = BN / 32;  // 16-row tiles per wave
  constexpr int VX = BM / 64, VW = BN / 64;  // 16-B vectors per thread per tile
  __shared__ __attribute__((aligned(16))) uint16_t xs[2][BM * GP];
  __shared__ __attribute__((aligned(16))) uint16_t ws[2][BN * GP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 15, kq = (lane >> 4) * 8;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const bf16x8_t zero = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};

  bf16x8_t px[VX], pw[VW];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int v = tid + i * 256, row = v >> 2, k = k0 + (v & 3) * 8;
      const int m = m0 + row;
      px[i] = (m < M && k < K) ? *reinterpret_cast<const bf16x8_t*>(x + static_cast<int64_t>(m) * K + k) : zero;
    }
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const int v = tid + i * 256, row = v >> 2, k = k0 + (v & 3) * 8;
      const int n = n0 + row;
      pw[i] = n < Npad ? *reinterpret_cast<const bf16x8_t*>(wt + static_cast<int64_t>(n) * Kpad + k) : zero;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int v = tid + i * 256;
      *reinterpret_cast<bf16x8_t*>(&xs[buf][(v >> 2) * GP + (v & 3) * 8]) = px[i];
    }
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const int v = tid + i * 256;
      *reinterpret_cast<bf16x8_t*>(&ws[buf][(v >> 2) * GP + (v & 3) * 8]) = pw[i];
    }
  };

  f32x4_t acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = Kpad / 32;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) gload((ks + 1) * 32);  // in flight during this k-step's MFMAs
    bf16x8_t a[RN], b[RM];
#pragma unroll
    for (int j = 0; j < RN; ++j)
      a[j] = *reinterpret_cast<const bf16x8_t*>(&ws[buf][(wn * (BN / 2) + j * 16 + li) * GP + kq]);
#pragma unroll
    for (int i = 0; i < RM; ++i)
      b[i] = *reinterpret_cast<const bf16x8_t*>(&xs[buf][(wm * (BM / 2) + i * 16 + li) * GP + kq]);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a[j]),
                                                            __builtin_bit_cast(bf16x8_mfma, b[i]), acc[i][j], 0, 0, 0);
    if (ks + 1 < nk) lstore(buf ^ 1);  // buf ^ 1 was last read before the previous barrier
    __syncthreads();
  }

  // epilogue: lane owns channels n..n+3 of pixel m (as pw_gemm_kernel)
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int m = m0 + wm * (BM / 2) + i * 16 + li;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + (lane >> 4) * 4;
      if (n >= N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[n + r];
      if (res) {
        const uint2 rr = *reinterpret_cast<const uint2*>(res + static_cast<int64_t>(m) * N + n);
        v[0] += bf2f(rr.x & 0xffff);
        v[1] += bf2f(rr.x >> 16);
        v[2] += bf2f(rr.y & 0xffff);
        v[3] += bf2f(rr.y >> 16);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
      if (OUT_F32) {
        *reinterpret_cast<float4*>(static_cast<float*>(y) + static_cast<int64_t>(m) * N + n) =
            float4{v[0], v[1], v[2], v[3]};
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
// I = int for every tensor below 2^31 lanes of work: 64-bit div/mod is a
// ~40-instruction VALU sequence per op on CDNA (no integer divider), and the
// index split below needs three of them per output.
template <typename I>
__global__ void __launch_bounds__(256) dw3x3_kernel(const uint16_t* __restrict__ x,  // [B][H][W][C]
                                                    const uint16_t* __restrict__ w,  // [9][C]
                                                    const float* __restrict__ bias,  // [C]
                                                    uint16_t* __restrict__ y,        // [B][Ho][Wo][C]
                                                    int B, int H, int W, int C, int Ho, int Wo, int stride,
                                                    int dil, int act) {
  const I cg = C >> 3;
  const I total = static_cast<I>(B) * Ho * Wo * cg;
  for (I t = blockIdx.x * static_cast<I>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<I>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(t % cg);
    I p = t / cg;
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
// the fly through a 256-entry LUT (the tensor_transform arithmetic folded into
// a table by the filter; padding stays 0 in the normalised domain)
// MFMA stem: the 3x3/2 conv 3 -> 32 as D[co][px] = W[co][k] . P[px][k]^T with
// k = (ky, kx, ci) = 27 padded to 32 -- two v_mfma_f32_16x16x32_bf16 per 16
// output pixels.  A workgroup owns STEM_R output rows of one image: the
// 2 * STEM_R + 1 input rows are normalised once into LDS (bf16, a zero column
// on the left = the conv padding), each lane gathers its 8 patch values from
// LDS (per-lane offsets fixed for the whole tile walk), and the epilogue writes
// bias + act as bf16 NHWC.  The VALU direct-conv version did 27 byte loads and
// 216 FMAs per 8 outputs and ran at ~1 TB/s of output; this one is bound by
// the bf16 output stream.
constexpr int STEM_R = 2;

template <typename T>
__global__ void __launch_bounds__(256) stem_mfma_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                        int H, int W, int Ho, int Wo, int act, const float* __restrict__ lut_g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xin[];  // [2R+1][(W + 2) * 3] bf16
  __shared__ float lut[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, kq = (lane >> 4) * 8;
  const int row_groups = (Ho + STEM_R - 1) / STEM_R;
  const int b = blockIdx.x / row_groups;
  const int oy0 = (blockIdx.x % row_groups) * STEM_R;
  const int pitch = (W + 2) * 3;  // columns ix = -1 .. W (both pads)
  if (sizeof(T) == 1) lut[tid] = lut_g[tid];
  // A fragments (weights, rows = output channels) + this lane's bias values
  bf16x8_t a[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kq + j;
      a[t][j] = static_cast<short>(k < 27 ? f2bf(w[k * 32 + t * 16 + li]) : 0);
    }
  float bv[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[t][r] = bias[t * 16 + (lane >> 4) * 4 + r];
  // this lane's 8 patch offsets relative to the pixel's top-left tap
  int off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kq + j;
    off[j] = k < 27 ? (k / 9) * pitch + ((k % 9) / 3) * 3 + (k % 3) : -1;
  }
  __syncthreads();  // lut
  const int iy0 = oy0 * 2 - 1;
  const int n_in = (2 * STEM_R + 1) * pitch;
  const T* xb = x + static_cast<int64_t>(b) * H * W * 3;
  if (sizeof(T) == 1 && (W * 3) % 4 == 0) {
    // raw uint8 rows: 4 bytes per load (a row starts 4-aligned), LUT-normalised into LDS
    const int wpr = W * 3 / 4;  // words per row
    for (int i = tid; i < (2 * STEM_R + 1) * wpr; i += 256) {
      const int r = i / wpr, wd = i % wpr;
      const int iy = iy0 + r;
      uint32_t v4 = 0;
      const bool in = iy >= 0 && iy < H;
      if (in) v4 = reinterpret_cast<const uint32_t*>(xb + static_cast<int64_t>(iy) * W * 3)[wd];
      uint16_t* dst = xin + r * pitch + 3 + wd * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = in ? f2bf(lut[(v4 >> (8 * j)) & 255]) : 0;
    }
    for (int i = tid; i < (2 * STEM_R + 1) * 6; i += 256) {  // left / right padding columns
      const int r = i / 6, j = i % 6;
      xin[r * pitch + (j < 3 ? j : pitch - 6 + j)] = 0;
    }
  } else {
    for (int i = tid; i < n_in; i += 256) {
      const int r = i / pitch, c = i % pitch;  // c = (ix + 1) * 3 + ci
      const int iy = iy0 + r, ix = c / 3 - 1;
      float v = 0.f;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
        const T raw = xb[(static_cast<int64_t>(iy) * W + ix) * 3 + c % 3];
        v = sizeof(T) == 1 ? lut[static_cast<int>(raw)] : static_cast<float>(raw);
      }
      xin[i] = f2bf(v);
    }
  }
  __syncthreads();
  const int tiles_x = (Wo + 15) / 16;
  for (int t = wave; t < STEM_R * tiles_x; t += 4) {
    const int oyl = t / tiles_x, ox = (t % tiles_x) * 16 + li;
    const int oy = oy0 + oyl;
    // top-left tap of pixel ox: input row 2*oyl (local), column 2*ox - 1 (+1 pad) -> 2*ox
    const int base = 2 * oyl * pitch + 2 * ox * 3;
    const bool valid = ox < Wo && oy < Ho;
    bf16x8_t bf;
#pragma unroll
    for (int j = 0; j < 8; ++j) bf[j] = static_cast<short>(valid && off[j] >= 0 ? xin[base + off[j]] : 0);
    const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const f32x4_t d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a[0]),
                                                               __builtin_bit_cast(bf16x8_mfma, bf), z, 0, 0, 0);
    const f32x4_t d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a[1]),
                                                               __builtin_bit_cast(bf16x8_mfma, bf), z, 0, 0, 0);
    if (!valid) continue;
    uint16_t* yp = y + ((static_cast<int64_t>(b) * Ho + oy) * Wo + ox) * 32 + (lane >> 4) * 4;
    uint2 o0, o1;
    o0.x = pk_bf16(act_fn(d0[0] + bv[0][0], act), act_fn(d0[1] + bv[0][1], act));
    o0.y = pk_bf16(act_fn(d0[2] + bv[0][2], act), act_fn(d0[3] + bv[0][3], act));
    o1.x = pk_bf16(act_fn(d1[0] + bv[1][0], act), act_fn(d1[1] + bv[1][1], act));
    o1.y = pk_bf16(act_fn(d1[2] + bv[1][2], act), act_fn(d1[3] + bv[1][3], act));
    *reinterpret_cast<uint2*>(yp) = o0;
    *reinterpret_cast<uint2*>(yp + 16) = o1;
  }
}

// ------------------------------------------------------------------ avgpool ----
// One workgroup = one image x 64 channel groups (of 8); the 4 waves split the
// pixels and meet in LDS.  (A thread per image x channel group gave only
// B * C / 8 / 256 = 80 workgroups at batch 128: 18 us for 16 MB.)
__global__ void __launch_bounds__(256) avgpool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B,
                                                      int HW, int C) {
  __shared__ float part[4][64][9];  // +1: conflict-free column reads
  const int cg = C >> 3;
  const int groups = (cg + 63) / 64;
  const int b = blockIdx.x / groups;
  const int g = (blockIdx.x % groups) * 64 + (threadIdx.x & 63);
  const int wave = threadIdx.x >> 6;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g < cg) {
    for (int p = wave; p < HW; p += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + (static_cast<int64_t>(b) * HW + p) * C + g * 8);
      const uint32_t vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += bf2f(vs[q] & 0xffff);
        acc[2 * q + 1] += bf2f(vs[q] >> 16);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) part[wave][threadIdx.x & 63][q] = acc[q];
  __syncthreads();
  if (wave != 0 || g >= cg) return;
  const float inv = 1.f / HW;
  float s[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[q] = (part[0][threadIdx.x][q] + part[1][threadIdx.x][q] + part[2][threadIdx.x][q] +
                                      part[3][threadIdx.x][q]) * inv;
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = pk_bf16(s[2 * q], s[2 * q + 1]);
  *reinterpret_cast<uint4*>(y + static_cast<int64_t>(b) * C + g * 8) = uint4{o[0], o[1], o[2], o[3]};
}

inline unsigned grid_cap(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return static_cast<unsigned>(g);
}

}  // namespace

void pw_gemm(const void* x, const void* wt, const float* bias, const void* res, void* y, int M, int N, int K, int Kpad,
             int act, bool out_f32, hipStream_t s, int Npad) {
  if (Npad <= 0) Npad = (N + 63) / 64 * 64;
  // large M (the 7x7 / 14x14 stages and the head at batch >= 32): LDS-staged tiles,
  // 128 x 128 when that still gives every CU a workgroup, else 64 x 64
  if (M >= 2048 && K % 8 == 0 && N % 4 == 0) {
    const auto* xp = static_cast<const uint16_t*>(x);
    const auto* wp = static_cast<const uint16_t*>(wt);
    const auto* rp = static_cast<const uint16_t*>(res);
    const int big = ((M + 127) / 128) * ((N + 127) / 128);
    if (big >= 256) {
      const dim3 g((M + 127) / 128, (N + 127) / 128);
      if (out_f32)
        hipLaunchKernelGGL((pw_gemm_lds_kernel<128, 128, true>), g, dim3(256), 0, s, xp, wp, bias, rp, y, M, N, K, Kpad,
                           Npad, act);
      else
        hipLaunchKernelGGL((pw_gemm_lds_kernel<128, 128, false>), g, dim3(256), 0, s, xp, wp, bias, rp, y, M, N, K,
                           Kpad, Npad, act);
    } else {
      const dim3 g((M + 63) / 64, (N + 63) / 64);
      if (out_f32)
        hipLaunchKernelGGL((pw_gemm_lds_kernel<64, 64, true>), g, dim3(256), 0, s, xp, wp, bias, rp, y, M, N, K, Kpad,
                           Npad, act);
      else
        hipLaunchKernelGGL((pw_gemm_lds_kernel<64, 64, false>), g, dim3(256), 0, s, xp, wp, bias, rp, y, M, N, K, Kpad,
                           Npad, act);
    }
    return;
  }
  dim3 grid((M + PW_BM - 1) / PW_BM, (N + PW_BN - 1) / PW_BN);
  const int ksteps = Kpad / 32;
  int chunk = ksteps;
  // A small output grid (the classifier: M = batch, 16 workgroups) leaves most
  // CUs idle while each workgroup walks all of K serially: split K over grid.z
  // and reduce with fp32 atomics (fp32 output without residual / activation)
  const int tiles = static_cast<int>(grid.x * grid.y);
  if (out_f32 && !res && act == 0 && tiles < 256 && ksteps >= 16) {
    // >= 8 k-steps per slice: more slices only add fp32 atomics on the same outputs
    // (20 slices x 2 k-steps ran 2x slower than no split for the 128 x 1000 x 1280 classifier)
    const int splits = std::min(ksteps / 8, (256 + tiles - 1) / tiles);
    chunk = (ksteps + splits - 1) / splits;
    grid.z = static_cast<unsigned>((ksteps + chunk - 1) / chunk);
    (void)hipMemsetAsync(y, 0, static_cast<size_t>(M) * N * sizeof(float), s);
  }
  if (out_f32)
    hipLaunchKernelGGL(pw_gemm_kernel<true>, grid, dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<const uint16_t*>(wt), bias, static_cast<const uint16_t*>(res), y, M, N, K, Kpad, act,
                       chunk);
  else
    hipLaunchKernelGGL(pw_gemm_kernel<false>, grid, dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<const uint16_t*>(wt), bias, static_cast<const uint16_t*>(res), y, M, N, K, Kpad, act,
                       chunk);
}

void dw3x3(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int C, int stride, int dil,
           int act, hipStream_t s) {
  // padding == dilation keeps "same" geometry: Ho = (H - 1) / stride + 1
  int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  int64_t work = static_cast<int64_t>(B) * Ho * Wo * (C / 8);
  auto k = work + static_cast<int64_t>(grid_cap(work)) * 256 < (int64_t(1) << 31) ? dw3x3_kernel<uint32_t> : dw3x3_kernel<int64_t>;
  hipLaunchKernelGGL(k, dim3(grid_cap(work)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<const uint16_t*>(w), bias, static_cast<uint16_t*>(y), B, H, W, C, Ho, Wo, stride, dil, act);
}

template <typename T>
void stem_launch(const T* x, const float* w, const float* bias, void* y, int B, int H, int W, int act,
                 const float* lut, hipStream_t s) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const size_t lds = sizeof(uint16_t) * (2 * STEM_R + 1) * (W + 2) * 3;
  const unsigned grid = static_cast<unsigned>(B * ((Ho + STEM_R - 1) / STEM_R));
  if (lds > 64 * 1024) {  // rows wider than ~3.6k pixels: opt into the full 160 KiB
    static const bool ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_mfma_kernel<T>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!ok || lds > 160 * 1024) return;
  }
  hipLaunchKernelGGL(stem_mfma_kernel<T>, dim3(grid), dim3(256), lds, s, x, w, bias, static_cast<uint16_t*>(y), H, W,
                     Ho, Wo, act, lut);
}

void stem3x3(const float* x, const float* w, const float* bias, void* y, int B, int H, int W, int act, hipStream_t s) {
  stem_launch<float>(x, w, bias, y, B, H, W, act, nullptr, s);
}

void stem3x3_u8(const uint8_t* x, const float* w, const float* bias, void* y, int B, int H, int W, int act,
                const float* lut, hipStream_t s) {
  stem_launch<uint8_t>(x, w, bias, y, B, H, W, act, lut, s);
}

void avgpool(const void* x, void* y, int B, int HW, int C, hipStream_t s) {
  const int groups = (C / 8 + 63) / 64;
  hipLaunchKernelGGL(avgpool_kernel, dim3(static_cast<unsigned>(B * groups)), dim3(256), 0, s,
                     static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), B, HW, C);
}

}  // namespace kernels
}  // namespace nnsx
