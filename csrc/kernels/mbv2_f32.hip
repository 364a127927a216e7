// fp32 MobileNet-family kernels for gfx950: the reference-precision engine.
//
// The reference runs MobileNetV2 through tensor_filter framework=pytorch on
// float32 tensors (ext/nnstreamer/tensor_filter/tensor_filter_pytorch.cc
// :517-536).  These kernels keep that precision end to end -- fp32
// activations in HBM and LDS, fp32 weights, fp32 accumulation -- and put
// every GEMM-shaped op on the matrix cores with v_mfma_f32_16x16x4_f32
// (exact fp32 products, 64 FLOP/clk/SIMD on gfx950: the fp32 MFMA rate
// equals the fp32 VALU rate, so the depthwise convs stay on the VALU).
//
// Operand convention (all MFMA kernels here): D[n][m] = A[n][k] . B[m][k]^T
// with A = weights (rows = output channels), B = activations (rows =
// pixels).  One lane (li = lane & 15, g = lane >> 4) loads a float4 of 4
// consecutive k of each operand: MFMA j of the four consumes component j,
// so lane-group g covers k = 16s + 4g + j -- a permutation of the 16 k of
// step s applied to both operands, which a dot product does not see.
// The 16x16 result puts 4 consecutive output channels (4g..4g+3) of one
// pixel (li) in each lane: one float4 NHWC store.
//
// LDS images are "k4-major": [k/4][row][4] floats.  A fragment read (16
// lanes of one g read 16 consecutive rows at one k-quad) is then 256
// contiguous bytes: conflict-free ds_read_b128 for every lane group.
//
//  * pw_gemm_f32   1x1 conv / FC: LDS-staged 128x128 or 64x64 tiles,
//                  32-k stages, double buffered; bias + act + residual
//                  epilogue; split-K with fp32 atomics for small grids.
//  * dw3x3_f32     depthwise 3x3 (stride 1/2, dilation d) + bias + act.
//  * stem_f32      3x3/2 conv 3 -> 32 (uint8 frame normalised in-kernel, or
//                  f32 frame) as 7 MFMA k-steps of 4 (27 taps + 1 zero).
//  * avgpool_f32   global average pool.
//  * ir_block_f32  the fused inverted residual (expand -> dw -> project),
//                  hidden activation in LDS; see the comment at the kernel.
//  * irw_f32       the wave-split fused inverted residual (each wave walks its
//                  own hidden subtiles; no barriers in the channel loop).
//  * stem_ir1w_f32 stem + first block, one wave per 8x8 tile (the model's
//                  default; stem_ir1_f32 is the 8-wave 16x16 variant).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels/gemm_f32.h"
#include "kernels/irw_common.h"
#include "kernels/mbv2.h"
#include "kernels/x3.h"

namespace nnsx {
namespace kernels {

namespace {


// split-K epilogue: y = act(sum_z ws[z] + bias), slabs added in z order
// (deterministic, unlike fp32 atomics whose arrival order varies)
__global__ void __launch_bounds__(256) gemm_splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                                 const float* __restrict__ bias, int act,
                                                                 float* __restrict__ y) {
  const int64_t plane = static_cast<int64_t>(M) * N, nq = plane / 4;
  for (int64_t q = blockIdx.x * 256 + threadIdx.x; q < nq; q += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4_t v = reinterpret_cast<const f32x4_t*>(ws)[q];
    for (int z = 1; z < splits; ++z) v += reinterpret_cast<const f32x4_t*>(ws + z * plane)[q];
    v += *reinterpret_cast<const f32x4_t*>(bias + (q * 4) % N);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
    reinterpret_cast<f32x4_t*>(y)[q] = v;
  }
}

// ------------------------------------------------------------ pw_small_f32 ----
// Small-M 1x1 conv / FC (M <= 16 rows, or M <= 64 with K <= 512: the
// small-batch classifier and 1x1-map GEMMs; the head through POOL) in ONE
// launch, no split-K workspace and no reduce
// launch: a workgroup = 16 output channels x up to 64 rows, its 4 waves =
// RT row tiles x KS k-slices (RT * KS = 4: M <= 16 -> one row tile and 4
// k-slices, <= 32 -> 2 x 2, else 4 x 1).  Each wave runs 4 independent
// MFMA chains (k16 steps s mod 4, added at the end) so the 40-cycle MFMA
// dependency is hidden; k-slices are added through LDS in slice order
// (deterministic).  A / B fragments come straight from global memory (the
// operands are L2-resident at these sizes).
// POOL: rows = the HW pixels of image blockIdx.y (waves walk its 16-pixel
// tiles), output = act(.) averaged over the pixels -> y [B][N] (head conv +
// global average pool in one pass; the pooled sum is over pixel tiles in
// order, pixels within a tile by a fixed butterfly).
template <bool POOL>
__global__ void __launch_bounds__(256) pw_small_f32_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ res, float* __restrict__ y,
                                                           int M, int N, int K, int Kpad, int Npad, int act, int HW) {
  __shared__ f32x4_t red[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  int RT = 4, KS = 1;
  if (!POOL && M <= 16) RT = 1, KS = 4;
  else if (!POOL && M <= 32) RT = 2, KS = 2;
  const int rt = wave % RT, ks = wave / RT;
  const int nsteps = (K + 15) / 16;
  const int s0 = ks * nsteps / KS, s1 = (ks + 1) * nsteps / KS;
  const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int wrow = n0 + li;
  const float* wp = wt + static_cast<int64_t>(wrow < Npad ? wrow : 0) * Kpad;
  // rows of this wave: POOL -> pixel tiles rt, rt + 4, ... of image blockIdx.y;
  // else the single tile blockIdx.y * 64 + rt * 16
  const int ntiles = POOL ? (HW + 15) / 16 : 1;
  f32x4_t pooled = z;
  for (int t = POOL ? rt : 0; t < ntiles; t += (POOL ? 4 : 1)) {
    const int m = POOL ? t * 16 + li : static_cast<int>(blockIdx.y) * 64 + rt * 16 + li;
    const bool mok = POOL ? m < HW : m < M;
    const float* xp = x + (POOL ? static_cast<int64_t>(blockIdx.y) * HW : 0) * K + static_cast<int64_t>(mok ? m : 0) * K;
    // operands in chunks of U k16-steps, the next chunk's loads in flight
    // during this chunk's MFMAs (one exposed memory latency per kernel, not
    // one per step); out-of-range steps load nothing and add zeros
    constexpr int U = 8;
    f32x4_t c[4] = {z, z, z, z};
    f32x4_t av[2][U], bv[2][U];
    auto load = [&](int st0, int buf) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = 16 * (st0 + u) + 4 * g;
        const bool kok = st0 + u < s1 && k < K;
        av[buf][u] = (kok && wrow < Npad) ? *reinterpret_cast<const f32x4_t*>(wp + k) : z;
        bv[buf][u] = (kok && mok) ? *reinterpret_cast<const f32x4_t*>(xp + k) : z;
      }
    };
    auto mma = [&](int buf) {
#pragma unroll
      for (int u = 0; u < U; ++u) c[u & 3] = mfma_k16(av[buf][u], bv[buf][u], c[u & 3]);
    };
    if (s0 < s1) load(s0, 0);
    for (int st = s0; st < s1; st += 2 * U) {
      if (st + U < s1) load(st + U, 1);
      mma(0);
      if (st + U >= s1) break;
      if (st + 2 * U < s1) load(st + 2 * U, 0);
      mma(1);
    }
    f32x4_t acc = (c[0] + c[1]) + (c[2] + c[3]);
    if (KS > 1) {  // k-slices through LDS, added in slice order by slice 0
      red[wave][lane] = acc;
      __syncthreads();
      if (ks == 0)
        for (int q = 1; q < KS; ++q) acc += red[q * RT + rt][lane];
    }
    if (ks != 0) continue;
    const int co = n0 + 4 * g;
    const f32x4_t b4 = co < N ? *reinterpret_cast<const f32x4_t*>(bias + co) : z;
    f32x4_t v = acc + b4;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
    if constexpr (POOL) {
      if (!mok) v = z;
#pragma unroll
      for (int d = 1; d < 16; d <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += __shfl_xor(v[r], d, 64);
      pooled += v;
    } else {
      if (mok && co < N) {
        if (res) v += *reinterpret_cast<const f32x4_t*>(res + static_cast<int64_t>(m) * N + co);
        *reinterpret_cast<f32x4_t*>(y + static_cast<int64_t>(m) * N + co) = v;
      }
    }
  }
  if constexpr (POOL) {
    __syncthreads();
    red[wave][lane] = pooled;  // every lane of a 16-lane group holds its group's sum
    __syncthreads();
    if (wave == 0 && li == 0) {
      f32x4_t sum = red[0][lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) sum += red[w][lane];
      const int co = n0 + 4 * g;
      if (co < N) *reinterpret_cast<f32x4_t*>(y + static_cast<int64_t>(blockIdx.y) * N + co) = sum * (1.f / HW);
    }
  }
}

// --------------------------------------------------------------- dw3x3_f32 ----
// one lane = one output pixel x 4 channels (float4 loads/stores)
__global__ void __launch_bounds__(256) dw3x3_f32_kernel(const float* __restrict__ x,     // [B][H][W][C]
                                                        const float* __restrict__ w,     // [9][C]
                                                        const float* __restrict__ bias,  // [C]
                                                        float* __restrict__ y,           // [B][Ho][Wo][C]
                                                        int B, int H, int W, int C, int Ho, int Wo, int stride,
                                                        int dil, int act) {
  // act bit 1: the input is a pre-activation map (a linear GEMM's output whose
  // ReLU6 was deferred to this consumer): clamp every tap to [0, 6]
  const bool ic = (act & 2) != 0;
  act &= 1;
  const uint32_t cg = static_cast<uint32_t>(C) >> 2;
  const uint32_t total = static_cast<uint32_t>(B) * Ho * Wo * cg;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % cg) * 4;
    uint32_t p = t / cg;
    const int ox = static_cast<int>(p % Wo);
    p /= Wo;
    const int oy = static_cast<int>(p % Ho);
    const int b = static_cast<int>(p / Ho);
    f32x4_t acc = *reinterpret_cast<const f32x4_t*>(bias + c);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * stride - dil + ky * dil;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * stride - dil + kx * dil;
        if (ix < 0 || ix >= W) continue;
        f32x4_t xv = *reinterpret_cast<const f32x4_t*>(x + ((static_cast<int64_t>(b) * H + iy) * W + ix) * C + c);
        if (ic) xv = relu6x4(xv);
        const f32x4_t wv = *reinterpret_cast<const f32x4_t*>(w + (ky * 3 + kx) * C + c);
        acc = __builtin_elementwise_fma(xv, wv, acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = act_fn(acc[r], act);
    *reinterpret_cast<f32x4_t*>(y + ((static_cast<int64_t>(b) * Ho + oy) * Wo + ox) * C + c) = acc;
  }
}

// column form (dilation 1): one lane = R vertically adjacent output pixels x
// CW horizontally adjacent ones x 4 channels, so each loaded input row feeds up
// to 3 of them ((R-1)S+3 row loads instead of 3R) and each loaded column up to 3
// ((CW-1)S+3 column loads instead of 3CW)
template <int R, int S, int CW = 1>
__device__ __forceinline__ void dw3x3_f32_col(const float* __restrict__ x, const float* __restrict__ w,
                                              const float* __restrict__ bias, float* __restrict__ y, int B, int H,
                                              int W, int C, int Ho, int Wo, int act, uint32_t t0, uint32_t step) {
  constexpr int NR = (R - 1) * S + 3, NX = (CW - 1) * S + 3;
  const bool ic = (act & 2) != 0;  // (deferred input ReLU6, dw3x3_f32_kernel)
  act &= 1;
  const uint32_t cg = static_cast<uint32_t>(C) >> 2;
  const uint32_t rg = static_cast<uint32_t>((Ho + R - 1) / R);
  const uint32_t wg = static_cast<uint32_t>((Wo + CW - 1) / CW);
  const uint32_t total = static_cast<uint32_t>(B) * rg * wg * cg;
  for (uint32_t t = t0; t < total; t += step) {
    const int c = static_cast<int>(t % cg) * 4;
    uint32_t p = t / cg;
    const int ox0 = static_cast<int>(p % wg) * CW;
    p /= wg;
    const int oy0 = static_cast<int>(p % rg) * R;
    const int b = static_cast<int>(p / rg);
    f32x4_t wv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wv[k] = *reinterpret_cast<const f32x4_t*>(w + k * C + c);
    const f32x4_t bv = *reinterpret_cast<const f32x4_t*>(bias + c);
    f32x4_t acc[R][CW];
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int q = 0; q < CW; ++q) acc[j][q] = bv;
    const float* xb = x + static_cast<int64_t>(b) * H * W * C + c;
#pragma unroll
    for (int ir = 0; ir < NR; ++ir) {
      const int iy = oy0 * S - 1 + ir;
      if (iy < 0 || iy >= H) continue;
      f32x4_t xv[NX];
#pragma unroll
      for (int kx = 0; kx < NX; ++kx) {
        const int ix = ox0 * S - 1 + kx;
        xv[kx] = (ix >= 0 && ix < W) ? *reinterpret_cast<const f32x4_t*>(xb + (static_cast<int64_t>(iy) * W + ix) * C)
                                     : f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (ic) xv[kx] = relu6x4(xv[kx]);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int ky = ir - j * S;
        if (ky < 0 || ky > 2) continue;
#pragma unroll
        for (int q = 0; q < CW; ++q)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
            acc[j][q] = __builtin_elementwise_fma(xv[q * S + kx], wv[ky * 3 + kx], acc[j][q]);
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int oy = oy0 + j;
      if (oy >= Ho) break;
#pragma unroll
      for (int q = 0; q < CW; ++q) {
        const int ox = ox0 + q;
        if (CW > 1 && ox >= Wo) break;
        f32x4_t v = acc[j][q];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
        *reinterpret_cast<f32x4_t*>(y + ((static_cast<int64_t>(b) * Ho + oy) * Wo + ox) * C + c) = v;
      }
    }
  }
}

template <int R, int S, int CW = 1>
__global__ void __launch_bounds__(256) dw3x3_f32_col_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float* __restrict__ y,
                                                            int B, int H, int W, int C, int Ho, int Wo, int act) {
  dw3x3_f32_col<R, S, CW>(x, w, bias, y, B, H, W, C, Ho, Wo, act, blockIdx.x * blockDim.x + threadIdx.x,
                             gridDim.x * blockDim.x);
}

// Dilated stride-1 depthwise (DeepLab's output-stride-16 blocks), parity form:
// output (oy, ox) reads only inputs of its own residue (oy mod D, ox mod D), so
// the map is D x D independent plain 3x3 convolutions on its residue grids.  A
// lane owns R x CW outputs D apart inside one residue grid: (R + 2) x (CW + 2)
// loads for R x CW outputs -- 36 per 16 at 4 x 4 against 64 for the contiguous
// 4 x 4 block over the dilated window (dw3x3_f32_col<4, 1, 4, 2>).  Row blocks
// are numbered residue by residue (residue r has ceil((H - r) / D) rows).
template <int R, int CW, int D>
__global__ void __launch_bounds__(256) dw3x3_f32_dil_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float* __restrict__ y,
                                                            int B, int H, int W, int C, int act) {
  const bool ic = (act & 2) != 0;  // (deferred input ReLU6, dw3x3_f32_kernel)
  act &= 1;
  auto blocks = [](int n, int r, int per) { return ((n - r + D - 1) / D + per - 1) / per; };
  int rbt = 0, cbt = 0;
#pragma unroll
  for (int r = 0; r < D; ++r) {
    rbt += blocks(H, r, R);
    cbt += blocks(W, r, CW);
  }
  const uint32_t cg = static_cast<uint32_t>(C) >> 2;
  const uint32_t total = static_cast<uint32_t>(B) * rbt * cbt * cg;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % cg) * 4;
    uint32_t p = t / cg;
    int kx = static_cast<int>(p % cbt);
    p /= cbt;
    int ky = static_cast<int>(p % rbt);
    const int b = static_cast<int>(p / rbt);
    int py = 0, px = 0;
#pragma unroll
    for (int r = 0; r < D - 1; ++r) {
      const int nr = blocks(H, py, R), nc = blocks(W, px, CW);
      if (ky >= nr) {
        ky -= nr;
        ++py;
      }
      if (kx >= nc) {
        kx -= nc;
        ++px;
      }
    }
    const int oy0 = py + ky * R * D, ox0 = px + kx * CW * D;
    f32x4_t wv[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wv[k] = *reinterpret_cast<const f32x4_t*>(w + k * C + c);
    const f32x4_t bv = *reinterpret_cast<const f32x4_t*>(bias + c);
    f32x4_t acc[R][CW];
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int q = 0; q < CW; ++q) acc[j][q] = bv;
    const float* xb = x + static_cast<int64_t>(b) * H * W * C + c;
#pragma unroll
    for (int ir = 0; ir < R + 2; ++ir) {
      const int iy = oy0 + (ir - 1) * D;
      if (iy < 0 || iy >= H) continue;
      f32x4_t xv[CW + 2];
#pragma unroll
      for (int k = 0; k < CW + 2; ++k) {
        const int ix = ox0 + (k - 1) * D;
        xv[k] = (ix >= 0 && ix < W) ? *reinterpret_cast<const f32x4_t*>(xb + (static_cast<int64_t>(iy) * W + ix) * C)
                                    : f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (ic) xv[k] = relu6x4(xv[k]);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int tap = ir - j;
        if (tap < 0 || tap > 2) continue;
#pragma unroll
        for (int q = 0; q < CW; ++q)
#pragma unroll
          for (int k = 0; k < 3; ++k) acc[j][q] = __builtin_elementwise_fma(xv[q + k], wv[tap * 3 + k], acc[j][q]);
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int oy = oy0 + j * D;
      if (oy >= H) break;
#pragma unroll
      for (int q = 0; q < CW; ++q) {
        const int ox = ox0 + q * D;
        if (ox >= W) break;
        f32x4_t v = acc[j][q];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
        *reinterpret_cast<f32x4_t*>(y + ((static_cast<int64_t>(b) * H + oy) * W + ox) * C + c) = v;
      }
    }
  }
}

// several stride-1 depthwise problems in one launch (the SSD heads); problem i
// owns blocks [start[i], start[i + 1]) and walks its work with that stride
struct DwGroupArgs {
  int n = 0;
  int start[kGroupMax + 1] = {};
  DwProb p[kGroupMax];
};

__global__ void __launch_bounds__(256) dw3x3_group_f32_kernel(DwGroupArgs g) {
  const int bid = blockIdx.x;
  int i = 0;
  while (i + 1 < g.n && bid >= g.start[i + 1]) ++i;
  const DwProb& p = g.p[i];
  dw3x3_f32_col<4, 1, 4>(p.x, p.w, p.bias, p.y, p.B, p.H, p.W, p.C, p.H, p.W, p.act,
                      static_cast<uint32_t>(bid - g.start[i]) * 256u + threadIdx.x,
                      static_cast<uint32_t>(g.start[i + 1] - g.start[i]) * 256u);
}

// ---------------------------------------------------------------- stem_f32 ----
// 3x3/2 conv 3 -> 32 as D[co][px] = W[co][k] . P[px][k]^T, k = (ky, kx, ci)
// = 27 taps + 1 zero = 7 MFMA steps of 4 (step t: lane group g holds
// k = 4t + g).  A workgroup owns STEM_R output rows of one image: the
// 2 * STEM_R + 1 input rows are normalised once into LDS as fp32 (a zero
// column each side = the conv padding); each lane gathers its 7 patch values
// per 16-pixel tile from LDS.  T = uint8_t: raw RGB mapped through the
// 256-entry input table (the pipeline's tensor_transform arithmetic).
constexpr int STEM_R = 2;

template <typename T>
__global__ void __launch_bounds__(256) stem_f32_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ y, int H,
                                                       int W, int Ho, int Wo, int act, const float* __restrict__ lut) {
  extern __shared__ __attribute__((aligned(16))) float xin[];  // [2R+1][(W + 2) * 3]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int row_groups = (Ho + STEM_R - 1) / STEM_R;
  const int b = blockIdx.x / row_groups;
  const int oy0 = (blockIdx.x % row_groups) * STEM_R;
  const int pitch = (W + 2) * 3;
  float a[2][7];
  int off[7];
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    const int k = 4 * t + g;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) a[ct][t] = k < 27 ? w[k * 32 + ct * 16 + li] : 0.f;
    off[t] = k < 27 ? (k / 9) * pitch + ((k % 9) / 3) * 3 + (k % 3) : 0;
  }
  const f32x4_t bv0 = *reinterpret_cast<const f32x4_t*>(bias + g * 4);
  const f32x4_t bv1 = *reinterpret_cast<const f32x4_t*>(bias + 16 + g * 4);
  const int iy0 = oy0 * 2 - 1;
  const T* xb = x + static_cast<int64_t>(b) * H * W * 3;
  // staging in chunks of 8 elements per thread, branch-free: the 8 loads (out-of-
  // image elements read the image's first one and select zero) go out back to
  // back, then the 8 table lookups -- a load under a branch waited for its own
  // round trip each iteration (PoseNet 257x257 at batch 64: 71 us)
  const int nst = (2 * STEM_R + 1) * pitch;
  for (int i0 = tid; i0 < nst; i0 += 256 * 8) {
    T raw[8];
    bool ok[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256;
      const int r = i / pitch, c = i - r * pitch;  // c = (ix + 1) * 3 + ci
      const int iy = iy0 + r, ix = c / 3 - 1;
      ok[u] = i < nst && iy >= 0 && iy < H && ix >= 0 && ix < W;
      raw[u] = xb[ok[u] ? (static_cast<int64_t>(iy) * W + ix) * 3 + (c - (c / 3) * 3) : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256;
      const float v = sizeof(T) == 1 ? lut[static_cast<int>(raw[u])] : static_cast<float>(raw[u]);
      if (i < nst) xin[i] = ok[u] ? v : 0.f;
    }
  }
  __syncthreads();
  const int tiles_x = (Wo + 15) / 16;
  for (int t = wave; t < STEM_R * tiles_x; t += 4) {
    const int oyl = t / tiles_x, ox = (t % tiles_x) * 16 + li;
    const int oy = oy0 + oyl;
    const bool valid = ox < Wo && oy < Ho;
    const int base = 2 * oyl * pitch + 2 * (valid ? ox : 0) * 3;
    f32x4_t d0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, d1 = d0;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const float bval = (4 * s + g < 27) ? xin[base + off[s]] : 0.f;
      d0 = mfma4(a[0][s], bval, d0);
      d1 = mfma4(a[1][s], bval, d1);
    }
    if (!valid) continue;
    float* yp = y + ((static_cast<int64_t>(b) * Ho + oy) * Wo + ox) * 32 + g * 4;
    f32x4_t o0 = d0 + bv0, o1 = d1 + bv1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o0[r] = act_fn(o0[r], act);
      o1[r] = act_fn(o1[r], act);
    }
    *reinterpret_cast<f32x4_t*>(yp) = o0;
    *reinterpret_cast<f32x4_t*>(yp + 16) = o1;
  }
}

// ------------------------------------------------------------- avgpool_f32 ----
// one workgroup = one image x 64 channel quads; the 4 waves split the pixels
// global average pool [B][HW][C] -> [B][C]: a workgroup = 16 channel quads x
// 16 pixel stripes; each lane keeps 4 independent partial sums (4 loads in
// flight), then the stripes are added in a fixed order through LDS
// (deterministic).  DeepLab's 33x33x320 maps at batch 8: 40 workgroups instead
// of 16 with one dependent load chain of 272 pixels per lane (67 us).
// Q channel quads x (256 / Q) pixel stripes per workgroup; the stripes' sums are
// added in a fixed order (bitwise repeatable).  Q = 4 where 16-quad groups would
// leave most CUs idle: DeepLab b8's 8 x 1089 x 320 map, 40 workgroups of 16
// quads, read at 1.4 TB/s.
template <int Q>
__global__ void __launch_bounds__(256) avgpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int HW,
                                                          int C) {
  constexpr int S = 256 / Q;
  __shared__ f32x4_t part[S][Q];
  const int cq = C >> 2;
  const int groups = (cq + Q - 1) / Q;
  const int b = blockIdx.x / groups;
  const int q = (blockIdx.x % groups) * Q + (threadIdx.x % Q);
  const int stripe = threadIdx.x / Q;
  const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t a0 = z, a1 = z, a2 = z, a3 = z;
  if (q < cq) {
    const float* xb = x + static_cast<int64_t>(b) * HW * C + q * 4;
    int p = stripe;
    for (; p + 3 * S < HW; p += 4 * S) {
      a0 += *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(p) * C);
      a1 += *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(p + S) * C);
      a2 += *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(p + 2 * S) * C);
      a3 += *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(p + 3 * S) * C);
    }
    for (; p < HW; p += S) a0 += *reinterpret_cast<const f32x4_t*>(xb + static_cast<int64_t>(p) * C);
  }
  part[stripe][threadIdx.x % Q] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (stripe != 0 || q >= cq) return;
  f32x4_t s = part[0][threadIdx.x];
#pragma unroll
  for (int k = 1; k < S; ++k) s += part[k][threadIdx.x];
  *reinterpret_cast<f32x4_t*>(y + static_cast<int64_t>(b) * C + q * 4) = s * (1.f / HW);
}

// ------------------------------------------------------------ ir_block_f32 ----
// Fused inverted residual, fp32:  y = project(dw3x3(expand(x))) (+ x).
//
// One workgroup = one TY x TX output tile of one image (4 waves).  Per tile:
//   * the in-image part of the input halo tile ((TY-1)S+3 x (TX-1)S+3, clipped
//     to the image) is staged in LDS, compactly (pixel c of the clipped
//     rectangle), k4-major;
//   * the hidden channels are walked in chunks of HC:
//       expand  MFMA over the compact pixels only (no work for the conv's
//               zero padding), bias + ReLU6, written into the chunk's hidden
//               image laid out as the full halo grid (out-of-image cells are
//               zeroed once per tile: they are the depthwise zero padding);
//       dw 3x3  VALU, lane = one output pixel x 4 channels, bias + ReLU6,
//               into a per-wave image of the wave's own output pixels;
//       project MFMA accumulated in registers across chunks;
//   * epilogue: bias (+ residual from the staged input tile) -> fp32 NHWC.
// The hidden image is double-buffered, so one barrier per chunk orders
// expand(c + 1) after every wave's dw(c).
// has_expand = 0 (t = 1): the chunk's hidden image is a copy of the input.
template <int S, int TY, int TX, int HC, int NOT, int KIN>
struct IrF32Geom {
  static constexpr int TIY = (TY - 1) * S + 3, TIX = (TX - 1) * S + 3;
  static constexpr int PIN = TIY * TIX;           // halo grid cells
  static constexpr int NC16 = (PIN + 15) / 16 * 16;  // compact pixels, padded
  static constexpr int NPT = (TY * TX + 15) / 16;   // output pixel tiles
  static constexpr int PTW = (NPT + 3) / 4;         // per wave
  static constexpr int KQ = KIN / 4;
  static constexpr int HQ = HC / 4;
  static constexpr size_t xs_floats = static_cast<size_t>(KQ) * NC16 * 4;
  static constexpr size_t hid_floats = static_cast<size_t>(2) * HQ * PIN * 4;
  static constexpr size_t dwo_floats = static_cast<size_t>(HQ) * NPT * 16 * 4;
  static size_t lds_bytes(int hid) { return 4 * (xs_floats + hid_floats + dwo_floats + static_cast<size_t>(10) * hid); }
};

template <int S, int TY, int TX, int HC, int NOT, int KIN>
__global__ void __launch_bounds__(256) ir_block_f32_kernel(IrBlockF32Args a) {
  using G = IrF32Geom<S, TY, TX, HC, NOT, KIN>;
  constexpr int TIY = G::TIY, TIX = G::TIX, PIN = G::PIN, NC16 = G::NC16;
  constexpr int NPT = G::NPT, PTW = G::PTW, KQ = G::KQ, HQ = G::HQ;
  constexpr int NS16 = KIN / 16;         // full 16-k expand steps
  constexpr bool KT8 = (KIN % 16) != 0;  // plus an 8-k tail
  static_assert(KIN % 8 == 0 && HC % 16 == 0, "ir_block_f32: KIN % 8, HC % 16");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xs = smem;                        // [KQ][NC16][4]   compact input tile
  float* hidb = xs + G::xs_floats;         // [2][HQ][PIN][4] hidden chunk, halo grid
  float* dwo = hidb + G::hid_floats;       // [HQ][NPT*16][4] dw output (project B operand)
  float* wds = dwo + G::dwo_floats;        // [9][hid] depthwise weights
  float* bds = wds + 9 * a.hid;            // [hid]    depthwise bias

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int tiles_img = a.tiles_x * a.tiles_y;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int b = tile / tiles_img;
  const int tyx = tile - b * tiles_img;
  const int oy0 = (tyx / a.tiles_x) * TY, ox0 = (tyx % a.tiles_x) * TX;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const int ry0 = max(iy0, 0), ry1 = min(iy0 + TIY, a.H);
  const int rx0 = max(ix0, 0), rx1 = min(ix0 + TIX, a.W);
  const int RW = rx1 - rx0, NC = (ry1 - ry0) * RW;
  const float* xb = a.x + static_cast<int64_t>(b) * a.H * a.W * a.cin;

  // ---- stage the compact input tile (k4-major) + the depthwise weights
  for (int v = tid; v < NC16 * KQ; v += 256) {
    const int c = v / KQ, kq = v - c * KQ;
    f32x4_t val = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (c < NC && kq * 4 < a.cin) {
      const int yy = ry0 + c / RW, xx = rx0 + c % RW;
      val = *reinterpret_cast<const f32x4_t*>(xb + (static_cast<int64_t>(yy) * a.W + xx) * a.cin + kq * 4);
    }
    *reinterpret_cast<f32x4_t*>(xs + (kq * NC16 + c) * 4) = val;
  }
  for (int v = tid; v < 9 * a.hid / 4; v += 256)
    reinterpret_cast<f32x4_t*>(wds)[v] = reinterpret_cast<const f32x4_t*>(a.wd)[v];
  for (int v = tid; v < a.hid; v += 256) bds[v] = a.bd[v];
  // out-of-image halo cells are the depthwise zero padding: zero them in both
  // hidden buffers (expand only ever writes in-image cells)
  if (ry0 > iy0 || ry1 < iy0 + TIY || rx0 > ix0 || rx1 < ix0 + TIX) {
    for (int v = tid; v < 2 * HQ * PIN; v += 256) {
      const int p = v % PIN;
      const int yy = iy0 + p / TIX, xx = ix0 + p % TIX;
      if (yy < ry0 || yy >= ry1 || xx < rx0 || xx >= rx1)
        reinterpret_cast<f32x4_t*>(hidb)[v] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  }

  // expand pixel tiles of this wave: halo-grid cell of each lane's compact pixel
  constexpr int NBT_MAX = NC16 / 16;
  constexpr int BTW = (NBT_MAX + 3) / 4;
  const int nbt = (NC + 15) / 16;
  int hcell[BTW];
#pragma unroll
  for (int j = 0; j < BTW; ++j) {
    const int c = (wave + 4 * j) * 16 + li;
    hcell[j] = c < NC ? (ry0 + c / RW - iy0) * TIX + (rx0 + c % RW - ix0) : -1;
  }
  // depthwise / project pixels of this wave: output pixel q -> its top-left halo cell
  int dcell[PTW];
#pragma unroll
  for (int j = 0; j < PTW; ++j) {
    const int q = (wave + 4 * j) * 16 + li;
    const int qq = q < TY * TX ? q : 0;
    dcell[j] = (qq / TX) * S * TIX + (qq % TX) * S;
  }

  f32x4_t acc[PTW][NOT];
#pragma unroll
  for (int j = 0; j < PTW; ++j)
#pragma unroll
    for (int o = 0; o < NOT; ++o) acc[j][o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // xs, wds, zeroed halo

  int buf = 0;
  for (int c0 = 0; c0 < a.hid; c0 += HC, buf ^= 1) {
    float* hid = hidb + buf * (HQ * PIN * 4);
    // project weights of this chunk (A operand), in flight during expand + dw
    f32x4_t pa[NOT][HC / 16];
#pragma unroll
    for (int o = 0; o < NOT; ++o)
#pragma unroll
      for (int s = 0; s < HC / 16; ++s)
        pa[o][s] = *reinterpret_cast<const f32x4_t*>(a.wp + static_cast<int64_t>(o * 16 + li) * a.hid + c0 + 16 * s +
                                                     4 * g);

    // ---- expand (MFMA over the compact in-image pixels) -> hidden halo grid
    if (a.has_expand) {
#pragma unroll
      for (int t = 0; t < HC / 16; ++t) {
        const float* wrow = a.we + static_cast<int64_t>(c0 + t * 16 + li) * KIN;
        f32x4_t ea[NS16 > 0 ? NS16 : 1];
        f32x2_t et = f32x2_t{0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NS16; ++s) ea[s] = *reinterpret_cast<const f32x4_t*>(wrow + 16 * s + 4 * g);
        if constexpr (KT8) et = *reinterpret_cast<const f32x2_t*>(wrow + 16 * NS16 + 2 * g);
        const f32x4_t eb = *reinterpret_cast<const f32x4_t*>(a.be + c0 + t * 16 + 4 * g);
#pragma unroll
        for (int j = 0; j < BTW; ++j) {
          const int bt = wave + 4 * j;
          if (bt >= nbt) break;
          const int c = bt * 16 + li;
          f32x4_t e = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < NS16; ++s)
            e = mfma_k16(ea[s], *reinterpret_cast<const f32x4_t*>(xs + ((4 * s + g) * NC16 + c) * 4), e);
          if constexpr (KT8)
            e = mfma_k8(et, *reinterpret_cast<const f32x2_t*>(xs + ((4 * NS16 + g / 2) * NC16 + c) * 4 + 2 * (g & 1)),
                        e);
          if (hcell[j] >= 0) *reinterpret_cast<f32x4_t*>(hid + ((t * 4 + g) * PIN + hcell[j]) * 4) = relu6x4(e + eb);
        }
      }
    } else {
      // t = 1: the hidden chunk is the input tile's channels c0 .. c0+HC
      for (int v = tid; v < nbt * 16 * HQ; v += 256) {
        const int c = v % (nbt * 16), hq = v / (nbt * 16);
        if (c >= NC) continue;
        const int cell = (ry0 + c / RW - iy0) * TIX + (rx0 + c % RW - ix0);
        *reinterpret_cast<f32x4_t*>(hid + (hq * PIN + cell) * 4) =
            *reinterpret_cast<const f32x4_t*>(xs + ((c0 / 4 + hq) * NC16 + c) * 4);
      }
    }
    __syncthreads();  // hidden chunk complete (and, double buffered, dw(c-1) done everywhere)

    // ---- depthwise 3x3 + bias + ReLU6: lane = output pixel (li) x channel quads g, g+4, ...
#pragma unroll
    for (int hq = g; hq < HQ; hq += 4) {
      const int ch = c0 + hq * 4;
      f32x4_t wv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wv[t] = *reinterpret_cast<const f32x4_t*>(wds + t * a.hid + ch);
      const f32x4_t bb = *reinterpret_cast<const f32x4_t*>(bds + ch);
      const float* hrow = hid + hq * PIN * 4;
#pragma unroll
      for (int j = 0; j < PTW; ++j) {
        const int pt = wave + 4 * j;
        if (pt >= NPT) break;
        f32x4_t d = bb;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
            d = __builtin_elementwise_fma(
                *reinterpret_cast<const f32x4_t*>(hrow + (dcell[j] + ky * TIX + kx) * 4), wv[ky * 3 + kx], d);
        *reinterpret_cast<f32x4_t*>(dwo + (hq * NPT * 16 + pt * 16 + li) * 4) = relu6x4(d);
      }
    }
    // dwo pixel tiles of this wave are written and read by this wave only
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- project: acc[pt][o] += Wp[o][chunk] . dw[pt][chunk]^T
#pragma unroll
    for (int j = 0; j < PTW; ++j) {
      const int pt = wave + 4 * j;
      if (pt >= NPT) break;
#pragma unroll
      for (int s = 0; s < HC / 16; ++s) {
        const f32x4_t bf = *reinterpret_cast<const f32x4_t*>(dwo + ((4 * s + g) * NPT * 16 + pt * 16 + li) * 4);
#pragma unroll
        for (int o = 0; o < NOT; ++o) acc[j][o] = mfma_k16(pa[o][s], bf, acc[j][o]);
      }
    }
  }

  // ---- epilogue: bias (+ residual from the staged input tile) -> fp32 NHWC
#pragma unroll
  for (int j = 0; j < PTW; ++j) {
    const int pt = wave + 4 * j;
    if (pt >= NPT) break;
    const int q = pt * 16 + li;
    if (q >= TY * TX) continue;
    const int gy = oy0 + q / TX, gx = ox0 + q % TX;
    if (gy >= a.Ho || gx >= a.Wo) continue;
    float* yp = a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * a.cout;
    const int rc = (gy - ry0) * RW + (gx - rx0);  // compact index of the same pixel (stride 1)
#pragma unroll
    for (int o = 0; o < NOT; ++o) {
      const int co = o * 16 + g * 4;
      if (co >= a.cout) continue;
      f32x4_t v = acc[j][o] + *reinterpret_cast<const f32x4_t*>(a.bp + co);
      if (a.residual) v += *reinterpret_cast<const f32x4_t*>(xs + ((co / 4) * NC16 + rc) * 4);
      *reinterpret_cast<f32x4_t*>(yp + co) = v;
    }
  }
}

// ------------------------------------------------------------- irw_f32 ----
// Wave-split fused inverted residual (fp32): the same expand -> dw -> project
// as ir_block_f32, partitioned for the fp32 MFMA/VALU balance of the low-res
// stages (28x28, 14x14, 7x7 maps).
//
// One workgroup = one TY x TX output tile (x one of `hsplit` hidden-channel
// parts).  The compact in-image input tile is staged in LDS once; then each of
// the 4 waves walks its OWN 16-channel hidden subtiles (hs = wave, wave+4, ..)
// end to end with no workgroup barrier:
//   expand  MFMA over all compact pixels of the tile (NBT independent
//           accumulators), + bias, ReLU6 -> the wave's private hidden image
//           (halo grid, out-of-image cells zeroed once);
//   dw 3x3  VALU, lane = output pixel x channel quad, + bias, ReLU6 -> the
//           wave's private project operand;
//   project MFMA, acc[pixel tile][cout tile] += Wp[:, subtile] . dw^T,
//           accumulated over the wave's subtiles (a k-split of the project).
// Expand weights of the next subtile are in flight during dw + project.  At the
// end the 4 waves' partial sums are added through LDS in a fixed order (w0 +
// w1 + w2 + w3, deterministic), plus bias / residual, and stored; with
// hsplit > 1 each part stores its slab of a workspace and irw_reduce adds the
// slabs in part order (deterministic).  The MFMA pipe of a SIMD then alternates between waves of
// different workgroups that are never held at a common barrier, so one wave's
// depthwise VALU work hides under another's matrix work.
// (second launch bound = minimum waves per SIMD: 2 keeps every configuration
// but the 7x7 / 160-channel one within 256 VGPRs, two workgroups per CU)
//
// FULL = true (large maps, where most tiles are interior): the expand runs over
// the whole halo grid (pixel index = halo cell, compile-time geometry, no
// index tables) and writes zeros for out-of-image cells; FULL = false (small
// maps, where every tile touches the border): only the in-image pixels are
// expanded (compact index, halos zeroed once per tile).
// (A persistent variant -- a resident grid walking the tiles with the next
// tile's input prefetched into registers -- needed 190 VGPRs on the 112 -> 56
// block, 2 waves per SIMD instead of 3, and ran 757 vs 545 us at batch 512:
// profiles/r3_irw_persistent_ab_b512.txt.)
// DIL: depthwise dilation (padding DIL; DeepLab's output-stride-16 blocks)
// XE: the expand on split-bf16 MFMAs (x3, kernels/x3.h) -- the input tile split
// into three bf16 planes while it is staged (as irw_x3 does), the expand
// weights pre-split (we3), 6 v_mfma_f32_16x16x32_bf16 per 32 input channels
// against 8 x 4 v_mfma_f32_16x16x4_f32; the depthwise and the project stay
// native fp32.  (irw_x3 also moves the project to x3, which costs a register
// split of every depthwise output and 32x32 accumulators.)
template <int S, int TY, int TX, int KIN, int NOT, int NW, bool FULL, int DIL = 1, bool XE = false>
struct IrwXEGeom {
  using Base = IrwGeom<S, TY, TX, KIN, NOT, NW, FULL, DIL>;
  static constexpr int KP = (KIN + 31) / 32 * 32, K8 = KP / 8, NK32 = KP / 32;
  static constexpr size_t xs_b = XE ? static_cast<size_t>(3) * K8 * Base::XSP * 16 : 16 * Base::xs_q;
  static size_t lds_bytes(int) { return std::max(xs_b + 16 * Base::hid_q, 16 * Base::red_q); }
};

template <int S, int TY, int TX, int KIN, int NOT, int NW, bool FULL, int DIL = 1, bool XE = false>
__global__ void __launch_bounds__(64 * NW, (IrwGeom<S, TY, TX, KIN, NOT, NW, FULL>::MINB)) irw_f32_kernel(IrBlockF32Args a) {
  using G = IrwGeom<S, TY, TX, KIN, NOT, NW, FULL, DIL>;
  using GX = IrwXEGeom<S, TY, TX, KIN, NOT, NW, FULL, DIL, XE>;
  constexpr int NT = 64 * NW;
  constexpr int TIY = G::TIY, TIX = G::TIX, PIN = G::PIN, NC16 = G::NC16, NBT = G::NBT, XSP = G::XSP;
  constexpr int PINP = G::PINP;
  static_assert(FULL || PINP > PIN, "irw_f32: the compact expand needs a scratch hidden cell");
  constexpr int KQ = G::KQ, NPT = G::NPT, NPX = G::NPX;
  constexpr int NS16 = KIN / 16;
  constexpr bool KT8 = (KIN % 16) != 0;
  constexpr int KP = GX::KP, K8 = GX::K8, NK32 = GX::NK32;
  static_assert(KIN % 8 == 0, "irw_f32: KIN % 8");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  f32x4_t* xs = reinterpret_cast<f32x4_t*>(smem);     // [KQ][XSP] (fp32 expand)
  bf16x8_t* xs3 = reinterpret_cast<bf16x8_t*>(smem);  // [3][K8][XSP] (XE), cell swizzled by k8
  f32x4_t* hidw = reinterpret_cast<f32x4_t*>(reinterpret_cast<char*>(smem) + GX::xs_b);  // [NW][4][PINP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int nparts = a.hsplit;
  const int tiles_img = a.tiles_x * a.tiles_y;

  // ---- stage the input tile (coalesced reads: consecutive threads, consecutive
  // quads).  Two phases with branch-free loads: every load of the tile is
  // issued back to back (out-of-tile lanes read the image's first quad and
  // select zero), then the LDS stores.  A load under a branch became
  // load / s_waitcnt vmcnt(0) / store per iteration, one exposed memory
  // latency per 256 quads of the tile.
  constexpr int KQS = XE ? KP / 4 : KQ;  // quads staged per cell (XE: zeros up to the 32-channel pad)
  constexpr int NSV = NC16 * KQS, NSIT = (NSV + NT - 1) / NT;
  f32x4_t sv[NSIT];
  bool sok[NSIT];
  // c / RW for the small compact indices (c < 1024): (c + 0.5) * (1 / RW) in
  // fp32 is at least 0.5 / RW away from an integer, so truncation is exact
  auto load_tile = [&](int t) {
    const int tb = t / tiles_img, tt = t - tb * tiles_img;
    const int ty0 = (tt / a.tiles_x) * TY * S - DIL, tx0 = (tt % a.tiles_x) * TX * S - DIL;
    const int qy0 = max(ty0, 0), qy1 = min(ty0 + TIY, a.H);
    const int qx0 = max(tx0, 0), qx1 = min(tx0 + TIX, a.W);
    const int qw = qx1 - qx0, qn = FULL ? PIN : (qy1 - qy0) * qw;
    const float qr = 1.f / static_cast<float>(qw);
    const float* qb = a.x + static_cast<int64_t>(tb) * a.H * a.W * a.cin;
    // a tile whose halo grid lies inside the image (wave-uniform; its compact
    // index is the grid index): no per-cell bounds tests
    if (ty0 >= 0 && tx0 >= 0 && ty0 + TIY <= a.H && tx0 + TIX <= a.W) {
#pragma unroll
      for (int it = 0; it < NSIT; ++it) {
        const int v = tid + it * NT;
        const int c = v / KQS, kq = v - c * KQS;
        sok[it] = (NSV % NT == 0 || v < NSV) && c < PIN && kq * 4 < a.cin;
        const int64_t off =
            sok[it] ? (static_cast<int64_t>(ty0 + c / TIX) * a.W + (tx0 + c % TIX)) * a.cin + kq * 4 : 0;
        sv[it] = *reinterpret_cast<const f32x4_t*>(qb + off);
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < NSIT; ++it) {
      const int v = tid + it * NT;
      const int c = v / KQS, kq = v - c * KQS;
      int yy, xx;
      if constexpr (FULL) {
        yy = ty0 + c / TIX;
        xx = tx0 + c % TIX;
      } else {
        const int cy = static_cast<int>((static_cast<float>(c) + 0.5f) * qr);
        yy = qy0 + cy;
        xx = qx0 + c - cy * qw;
      }
      sok[it] = (NSV % NT == 0 || v < NSV) && c < qn && kq * 4 < a.cin && yy >= 0 && yy < a.H && xx >= 0 &&
                xx < a.W;
      const int64_t off = sok[it] ? (static_cast<int64_t>(yy) * a.W + xx) * a.cin + kq * 4 : 0;
      sv[it] = *reinterpret_cast<const f32x4_t*>(qb + off);
    }
  };

  const int wg = xcd_remap(blockIdx.x, gridDim.x);  // the parts of a tile stay adjacent (same XCD / L2)
  const int part = wg % nparts, tile = wg / nparts;
  const int b = tile / tiles_img;
  const int tyx = tile - b * tiles_img;
  const int oy0 = (tyx / a.tiles_x) * TY, ox0 = (tyx % a.tiles_x) * TX;
  const int iy0 = oy0 * S - DIL, ix0 = ox0 * S - DIL;
  const int ry0 = max(iy0, 0), ry1 = min(iy0 + TIY, a.H);
  const int rx0 = max(ix0, 0), rx1 = min(ix0 + TIX, a.W);
  const int RW = rx1 - rx0, NC = FULL ? PIN : (ry1 - ry0) * RW;
  const bool tile_in = iy0 >= 0 && ix0 >= 0 && iy0 + TIY <= a.H && ix0 + TIX <= a.W;  // whole halo grid in the image
  const float rrw = 1.f / static_cast<float>(RW);
  load_tile(tile);
#pragma unroll
  for (int it = 0; it < NSIT; ++it) {
    const int v = tid + it * NT;
    if (NSV % NT != 0 && v >= NSV) break;
    const int c = v / KQS, kq = v - c * KQS;
    const f32x4_t q = sok[it] ? sv[it] : f32x4_t{0.f, 0.f, 0.f, 0.f};
    if constexpr (XE) {
      // three bf16 planes [part][k8][cell], 8 channels (16 B) per cell, cells
      // XOR-swizzled by k8 within their 16-cell group (irw_x3's layout)
      typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
      const int k8 = kq >> 1;
      bf16x2_t h0, m0, l0, h1, m1, l1;
      split2(f32x2_t{q[0], q[1]}, h0, m0, l0);
      split2(f32x2_t{q[2], q[3]}, h1, m1, l1);
      char* p = reinterpret_cast<char*>(xs3) + (static_cast<size_t>(k8) * XSP + (c ^ (k8 & 15))) * 16 + (kq & 1) * 8;
      constexpr size_t PS = static_cast<size_t>(K8) * XSP * 16;  // part stride (bytes)
      *reinterpret_cast<bf16x4_t*>(p) = __builtin_shufflevector(h0, h1, 0, 1, 2, 3);
      *reinterpret_cast<bf16x4_t*>(p + PS) = __builtin_shufflevector(m0, m1, 0, 1, 2, 3);
      *reinterpret_cast<bf16x4_t*>(p + 2 * PS) = __builtin_shufflevector(l0, l1, 0, 1, 2, 3);
    } else {
      xs[kq * XSP + (c ^ (kq & 3))] = q;
    }
  }
  // out-of-image halo cells of every wave's hidden image = the depthwise zero padding
  // (FULL: the expand itself writes them as zeros)
  if (!FULL && (ry0 > iy0 || ry1 < iy0 + TIY || rx0 > ix0 || rx1 < ix0 + TIX)) {
    for (int v = tid; v < 4 * NW * PIN; v += NT) {
      const int pl = v / PIN, p = v - pl * PIN;
      const int yy = iy0 + p / TIX, xx = ix0 + p % TIX;
      if (yy < ry0 || yy >= ry1 || xx < rx0 || xx >= rx1) hidw[pl * PINP + p] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  }
  // expand pixel j*16+li -> its hidden cell (compact), or in-image flag (FULL)
  int hcell[NBT];
#pragma unroll
  for (int j = 0; j < NBT; ++j) {
    const int c = j * 16 + li;
    if constexpr (FULL) {
      const int yy = iy0 + c / TIX, xx = ix0 + c % TIX;
      hcell[j] = (c < PIN && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) ? 1 : 0;
    } else {
      const int cy = static_cast<int>((static_cast<float>(c) + 0.5f) * rrw);
      hcell[j] = c < NC ? (ry0 + cy - iy0) * TIX + (rx0 + c - cy * RW - ix0) : PIN;  // PIN: scratch cell
    }
  }
  int dcell[NPT];
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) {
    const int q = pt * 16 + li;
    const int qq = q < TY * TX ? q : 0;
    dcell[pt] = (qq / TX) * S * TIX + (qq % TX) * S;
  }
  const int nbt = (NC + 15) / 16;  // pixel tiles holding in-image pixels (wave-uniform)

  // NOT = 0: no project -- the depthwise output itself is the result
  // ([B][Ho][Wo][hid] in a.y; blocks whose project is a plain GEMM)
  constexpr int NOA = NOT > 0 ? NOT : 1;
  f32x4_t acc[NPT][NOA];
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
    for (int o = 0; o < NOA; ++o) acc[pt][o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // xs + zeroed halos

  const int nsub = a.hid >> 4;
  const int sub0 = part * nsub / nparts, sub1 = (part + 1) * nsub / nparts;
  f32x4_t* myhid = hidw + (wave * 4 + g) * PINP;
  f32x4_t ea[XE ? 1 : (NS16 > 0 ? NS16 : 1)];
  X3Frag ea3[XE ? NK32 : 1];
  f32x2_t et = f32x2_t{0.f, 0.f};
  f32x4_t be4 = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // PREB: the expand bias is fetched one subtile ahead with the expand
  // weights.  vmcnt waits count in issue order, so a bias load issued after the
  // subtile's depthwise / project weights makes the first expand epilogue wait
  // for all of them (vmcnt(0)); fetched ahead, the expand waits only for loads
  // issued a subtile earlier and the dw / project weights land during the
  // expand.  Measured at batch 512: 112->56 594 -> 569 us, 56x56 465 -> 456; on
  // the other blocks the 4-12 extra VGPRs cost more (56->28 and 28->14 lose a
  // wave per SIMD; 14x14/96 278 -> 306 us, 7x7 223 -> 240), so only the two
  // large-map 3-wave configurations use it.
  constexpr bool PREB = FULL && NW == 3 && TY * TX >= 32;
  auto load_ea = [&](int hs) {
    if constexpr (XE) {
      // we3 [3][hid][KP] bf16: lane (li, g) holds k 8g .. 8g + 7 of each 32-k step of row hs * 16 + li
      const int64_t wes = static_cast<int64_t>(a.hid) * KP;
#pragma unroll
      for (int c = 0; c < NK32; ++c)
        ea3[c] = load_x3(a.we3, wes, static_cast<int64_t>(hs * 16 + li) * KP + 32 * c + 8 * g);
    } else {
      const float* wrow = a.we + static_cast<int64_t>(hs * 16 + li) * KIN;
#pragma unroll
      for (int s = 0; s < NS16; ++s) ea[s] = *reinterpret_cast<const f32x4_t*>(wrow + 16 * s + 4 * g);
      if constexpr (KT8) et = *reinterpret_cast<const f32x2_t*>(wrow + 16 * NS16 + 2 * g);
    }
    if constexpr (PREB) be4 = *reinterpret_cast<const f32x4_t*>(a.be + hs * 16 + 4 * g);
  };
  int hs = sub0 + wave;
  if (a.has_expand && hs < sub1) load_ea(hs);
  for (; hs < sub1; hs += NW) {
    const int ch = hs * 16 + 4 * g;  // this lane's channel quad (dw, biases)
    f32x4_t pa[NOA];
#pragma unroll
    for (int o = 0; o < NOT; ++o)
      pa[o] = *reinterpret_cast<const f32x4_t*>(a.wp + static_cast<int64_t>(o * 16 + li) * a.hid + ch);
    f32x4_t wd4[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wd4[t] = *reinterpret_cast<const f32x4_t*>(a.wd + t * a.hid + ch);
    const f32x4_t bd4 = *reinterpret_cast<const f32x4_t*>(a.bd + ch);

    // ---- expand -> private hidden image
    if (a.has_expand) {
      if constexpr (!PREB) be4 = *reinterpret_cast<const f32x4_t*>(a.be + ch);
      // pixel tiles in pairs (two independent MFMA chains); a pair past the
      // in-image pixels is skipped wave-uniformly, a half-valid one computes zeros
      // PREX (whole halo grid, one 16-k step): the next pair's B operands are
      // read before this pair's MFMAs and hidden stores -- xs and the hidden
      // images share the LDS array, so reads placed after the stores cannot be
      // hoisted above them and each pair waited for its own LDS round trip
      constexpr bool PREX = FULL && NS16 == 1 && !XE;
      f32x4_t bx0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, bx1 = bx0;
      if constexpr (PREX) {
        bx0 = xs[g * XSP + (li ^ g)];
        bx1 = xs[g * XSP + (NBT > 1 ? 16 : 0) + (li ^ g)];
      }
#pragma unroll
      for (int j = 0; j < NBT; j += 2) {
        if (FULL || j < nbt) {
          const int j1 = j + 1 < NBT ? j + 1 : j;
          f32x4_t e0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, e1 = e0;
          if constexpr (XE) {
#pragma unroll
            for (int c = 0; c < NK32; ++c) {
              const int k8 = 4 * c + g;
              const bf16x8_t* pl = xs3 + k8 * XSP;
              const int c0 = (j * 16 + li) ^ (k8 & 15), c1 = (j1 * 16 + li) ^ (k8 & 15);
              X3Frag b0, b1;
              b0.h = pl[c0];
              b0.m = pl[K8 * XSP + c0];
              b0.l = pl[2 * K8 * XSP + c0];
              b1.h = pl[c1];
              b1.m = pl[K8 * XSP + c1];
              b1.l = pl[2 * K8 * XSP + c1];
              e0 += mfma_x3(ea3[c], b0);
              e1 += mfma_x3(ea3[c], b1);
            }
          } else if constexpr (PREX) {
            f32x4_t n0 = bx0, n1 = bx1;
            if (j + 2 < NBT) {
              const int k1 = j + 3 < NBT ? j + 3 : j + 2;
              n0 = xs[g * XSP + (j + 2) * 16 + (li ^ g)];
              n1 = xs[g * XSP + k1 * 16 + (li ^ g)];
            }
            e0 = mfma_k16(ea[0], bx0, e0);
            e1 = mfma_k16(ea[0], bx1, e1);
            bx0 = n0;
            bx1 = n1;
          } else {
#pragma unroll
            for (int s = 0; s < NS16; ++s) {
              e0 = mfma_k16(ea[s], xs[(4 * s + g) * XSP + j * 16 + (li ^ g)], e0);
              e1 = mfma_k16(ea[s], xs[(4 * s + g) * XSP + j1 * 16 + (li ^ g)], e1);
            }
          }
          if constexpr (KT8 && !XE) {
            // tail plane kq = 4 NS16 + g/2: swizzle (kq & 3) = g >> 1
            const f32x2_t* t0 =
                reinterpret_cast<const f32x2_t*>(&xs[(4 * NS16 + g / 2) * XSP + j * 16 + (li ^ (g >> 1))]);
            const f32x2_t* t1 =
                reinterpret_cast<const f32x2_t*>(&xs[(4 * NS16 + g / 2) * XSP + j1 * 16 + (li ^ (g >> 1))]);
            e0 = mfma_k8(et, t0[g & 1], e0);
            e1 = mfma_k8(et, t1[g & 1], e1);
          }
          if constexpr (FULL) {
            if (tile_in) {  // (wave-uniform: no per-cell select; cells past PIN are never read)
              myhid[j * 16 + li] = relu6x4(e0 + be4);
              if (j + 1 < NBT) myhid[j1 * 16 + li] = relu6x4(e1 + be4);
            } else {
              const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
              myhid[j * 16 + li] = hcell[j] ? relu6x4(e0 + be4) : z;
              if (j + 1 < NBT) myhid[j1 * 16 + li] = hcell[j1] ? relu6x4(e1 + be4) : z;
            }
          } else {
            // branch-free: padding pixels store to the unused cell PIN (a per-lane
            // `if` compiled to exec-mask branches that kept the next pair's LDS
            // reads from overlapping this epilogue)
            myhid[hcell[j]] = relu6x4(e0 + be4);
            if (j + 1 < NBT) myhid[hcell[j1]] = relu6x4(e1 + be4);
          }
        }
      }
      if (hs + NW < sub1) load_ea(hs + NW);  // next subtile's weights: in flight during dw + project
    } else {
      // t = 1: the hidden channels are the input channels
#pragma unroll
      for (int j = 0; j < NBT; ++j) {
        if constexpr (FULL)
          myhid[j * 16 + li] = xs[(hs * 4 + g) * XSP + j * 16 + (li ^ g)];  // (staged zeros outside the image)
        else if (hcell[j] >= 0)
          myhid[hcell[j]] = xs[(hs * 4 + g) * XSP + j * 16 + (li ^ g)];
      }
    }
    wave_sync();

    // ---- depthwise 3x3 + bias + ReLU6, straight into the project MFMA: the
    // lane computing output pixel pt*16+li, channel quad g is exactly the lane
    // that holds that k-quad of column li in the B operand (mfma_k16 layout)
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) {
      f32x4_t d = bd4;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
          d = __builtin_elementwise_fma(myhid[dcell[pt] + (ky * TIX + kx) * DIL], wd4[ky * 3 + kx], d);
      const f32x4_t bf = relu6x4(d);
      if constexpr (NOT == 0) {
        const int q = pt * 16 + li;
        const int gy = oy0 + q / TX, gx = ox0 + q % TX;
        if (q < TY * TX && gy < a.Ho && gx < a.Wo)
          *reinterpret_cast<f32x4_t*>(a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * a.hid + ch) = bf;
        continue;
      }
      // ---- project: k-split partial over this subtile's 16 channels
#pragma unroll
      for (int o = 0; o < NOT; ++o) acc[pt][o] = mfma_k16(pa[o], bf, acc[pt][o]);
    }
    wave_sync();  // this wave's hidden image is read out before the next subtile's expand
  }
  if constexpr (NOT == 0) return;

  // ---- cross-wave reduction (fixed order) + bias + residual -> NHWC
  __syncthreads();  // every wave is done with xs / hidden / dwo: the LDS becomes the reduction buffer
  f32x4_t* red = reinterpret_cast<f32x4_t*>(smem);
#pragma unroll
  for (int o = 0; o < NOT; ++o) {
    f32x4_t* rb = red + (o & 1) * (4 * NW * NPX);
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) rb[(wave * 4 + g) * NPX + pt * 16 + li] = acc[pt][o];
    __syncthreads();
    const int co = o * 16 + 4 * g;
    for (int pt = wave; pt < NPT; pt += NW) {
      const int q = pt * 16 + li;
      f32x4_t v = rb[g * NPX + q];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += rb[(4 * w + g) * NPX + q];
      if (q >= TY * TX || co >= a.cout) continue;
      const int gy = oy0 + q / TX, gx = ox0 + q % TX;
      if (gy >= a.Ho || gx >= a.Wo) continue;
      const int64_t pix = (static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx;
      if (a.ws) {  // hidden parts: this part's slab of the workspace (irw_reduce adds them in order)
        const int64_t plane = static_cast<int64_t>(a.B) * a.Ho * a.Wo * a.cout;
        if (a.tickets) {  // in-launch combine: written through (sc1) to where every XCD reads it
          const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
              a.ws, 0, static_cast<int>(nparts * plane * sizeof(float)), 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), slab,
                                                 static_cast<int>((part * plane + pix * a.cout + co) * 4), 0, 16);
        } else {
          *reinterpret_cast<f32x4_t*>(a.ws + part * plane + pix * a.cout + co) = v;
        }
        continue;
      }
      if (part == 0) {
        v += *reinterpret_cast<const f32x4_t*>(a.bp + co);
        if (a.residual) v += *reinterpret_cast<const f32x4_t*>(a.x + pix * a.cin + co);
      }
      float* yp = a.y + pix * a.cout + co;
      if (nparts > 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(yp + r, v[r]);
      } else {
        *reinterpret_cast<f32x4_t*>(yp) = v;
      }
    }
  }
  if (!a.ws || !a.tickets) return;

  irw_inlaunch_combine<TY, TX, NT>(a, smem, tile, part, nparts, b, oy0, ox0, tid);
}

// ------------------------------------------------------- stem_ir1w_f32 ----
// The stem (3x3/2 conv 3 -> 32 on the raw uint8 frame, mapped in-kernel
// through the 256-entry input table, + bias, ReLU6) fused with MobileNetV2's
// first block (t = 1: dw 3x3 on those 32 channels + ReLU6, project 32 -> 16):
// the 32-channel stem output -- the largest activation of the network -- never
// leaves LDS.  One WAVE per tile: a
// workgroup is a single wave that owns a TY x TX output tile end to end --
// both 16-channel halves of the stem over the (TY+2) x (TX+2) halo grid, the
// depthwise 3x3 over all 32 channels and the whole K = 32 project -- so there
// is no workgroup barrier and no cross-wave reduction anywhere.  8 x 8 tiles
// keep a wave's LDS (input patch + 32-channel hidden image + normalisation
// table) under 20 KB, so 8 waves are resident per CU and one wave's MFMA
// work overlaps the others' staging / depthwise VALU work.  The price is the
// halo: 100 stem cells per 64 outputs (1.56x) against 324 per 256 (1.27x).
// (second launch bound: 2 waves per SIMD = 256 VGPRs; 8 such waves per CU.
// Moving the depthwise weights to LDS for 3 waves per SIMD (168 VGPRs) spilled
// 44 VGPRs and ran 642 vs 501 us at batch 512: profiles/r3_stem_variants_b512.txt.)
// Persistent: a resident set of waves walks the tiles; the next tile's input
// bytes are in flight while the current one computes.  (The patch rows at a
// 78-dword LDS pitch -- bank-conflict-free B reads, 125 against 195 LDS cycles
// per tile's stem reads -- measured neutral: MobileNetV2 b512 -0.1 %, DeepLab b8
// within noise; SQ_LDS_BANK_CONFLICT 43 % is not this kernel's bound.)
template <int TY, int TX, bool PAIR>
__global__ void __launch_bounds__(64, 2) stem_ir1w_f32_kernel(StemIr1F32Args a) {
  constexpr int HY = TY + 2, HX = TX + 2, PIN = HY * HX;
  constexpr int NBT = (PIN + 15) / 16;
  constexpr int IY = 2 * HY + 1, IX = 2 * HX + 1, PITCH = IX * 3;
  constexpr int NIN = IY * PITCH;
  constexpr int XIN = (NIN + 3) / 4 * 4;
  constexpr int NPT = (TY * TX + 15) / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xin = smem;                                             // [IY][PITCH] normalised input
  float* lut = smem + XIN;                                       // [256] input table
  f32x4_t* hid = reinterpret_cast<f32x4_t*>(smem + XIN + 256);  // [8 quads][PIN] (32 channels)

  const int lane = threadIdx.x;
  const int li = lane & 15, g = lane >> 4;
  const int tiles_img = a.tiles_x * a.tiles_y;
  const int ntiles = tiles_img * a.B;

#pragma unroll
  for (int i = 0; i < 4; ++i) lut[lane * 4 + i] = a.lut[lane * 4 + i];
  float sa[2][7];  // stem weights: half h, k = 4t + g (27 taps + 1 zero); A row li = channel 16h + li
  int off[7];
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    const int k = 4 * t + g;
    sa[0][t] = k < 27 ? a.ws[k * 32 + li] : 0.f;
    sa[1][t] = k < 27 ? a.ws[k * 32 + 16 + li] : 0.f;
    off[t] = k < 27 ? (k / 9) * PITCH + ((k % 9) / 3) * 3 + (k % 3) : 0;
  }
  f32x4_t bs4[2], bd4[2], pa[2], wd4[2][9];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ch = 16 * h + 4 * g;  // this lane's channel quad in half h
    bs4[h] = *reinterpret_cast<const f32x4_t*>(a.bs + ch);
    bd4[h] = *reinterpret_cast<const f32x4_t*>(a.bd + ch);
    pa[h] = *reinterpret_cast<const f32x4_t*>(a.wp + li * 32 + ch);  // project A: row li, k = 16h + 4g + j
#pragma unroll
    for (int t = 0; t < 9; ++t) wd4[h][t] = *reinterpret_cast<const f32x4_t*>(a.wd + t * 32 + ch);
  }
  const f32x4_t bp4 = *reinterpret_cast<const f32x4_t*>(a.bp + 4 * g);
  const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // the patch is fetched row by row, lane = byte column (PITCH <= 64): the
  // per-lane address terms are then the same for every row (few live registers)
  static_assert(PITCH <= 64, "stem_ir1w: one patch row per wave load");
  const int pcol = lane < PITCH ? lane : 0;
  const int pdx = pcol / 3, pch = pcol - 3 * pdx;
  const int rowb = a.W * 3;  // bytes per image row
  int raw[IY];
  // branch-free: every row's byte is loaded from a valid address (row 0 of the
  // image for out-of-image taps) and replaced by -1 afterwards, so the IY loads
  // issue back to back; the address is the wave-uniform image base plus a 32-bit
  // per-lane offset (no 64-bit address math per load)
  auto fetch = [&](int tile) {
    const int b = tile / tiles_img;
    const int tyx = tile - b * tiles_img;
    const int iy0 = 2 * ((tyx / a.tiles_x) * TY - 1) - 1, ix = 2 * ((tyx % a.tiles_x) * TX - 1) - 1 + pdx;
    const bool colok = lane < PITCH && ix >= 0 && ix < a.W;
    const uint8_t* img = a.x + static_cast<int64_t>(b) * a.H * rowb;
    const uint32_t col = colok ? static_cast<uint32_t>(ix * 3 + pch) : 0u;
    uint8_t v[IY];
    bool ok[IY];
#pragma unroll
    for (int r = 0; r < IY; ++r) {
      const int iy = iy0 + r;
      ok[r] = colok && iy >= 0 && iy < a.H;
      v[r] = img[(ok[r] ? static_cast<uint32_t>(iy * rowb) : 0u) + col];
    }
#pragma unroll
    for (int r = 0; r < IY; ++r) raw[r] = ok[r] ? static_cast<int>(v[r]) : -1;
  };

  int tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tiles_img;
    const int tyx = tile - b * tiles_img;
    const int oy0 = (tyx / a.tiles_x) * TY, ox0 = (tyx % a.tiles_x) * TX;
    const int hy0 = oy0 - 1, hx0 = ox0 - 1;  // hidden halo origin (stem-output coords)
    // every halo cell inside the stem output (most tiles of a 112x112 map)
    const bool interior = hy0 >= 0 && hx0 >= 0 && hy0 + HY <= a.Ho && hx0 + HX <= a.Wo;
    __syncthreads();  // (one wave: orders the previous tile's LDS reads before these writes; lut on entry)
    if (lane < PITCH) {
      // all table reads first, then the stores: lut and xin share the LDS
      // array, so read / store pairs in one loop were ordered one after the
      // other (an LDS round trip per patch row)
      float nv[IY];
#pragma unroll
      for (int r = 0; r < IY; ++r) nv[r] = lut[raw[r] >= 0 ? raw[r] : 0];
#pragma unroll
      for (int r = 0; r < IY; ++r) xin[r * PITCH + lane] = raw[r] >= 0 ? nv[r] : 0.f;
    }
    if (tile + static_cast<int>(gridDim.x) < ntiles) fetch(tile + gridDim.x);
    __syncthreads();

    // ---- stem MFMA, both channel halves per pixel tile (two independent chains
    // sharing each B operand read)
    // (the next pixel tile's 7 B operands are read before this tile's MFMAs and
    // hidden stores: xin and hid share the LDS array, so reads placed after the
    // stores could not be hoisted above them)
    auto patch_base = [&](int c) { return c < PIN ? 2 * (c / HX) * PITCH + 6 * (c % HX) : 0; };
    float xv[7];
    {
      const int base = patch_base(li);
#pragma unroll
      for (int t = 0; t < 7; ++t) xv[t] = xin[base + off[t]];
    }
#pragma unroll 1
    for (int j = 0; j < NBT; ++j) {
      const int c = j * 16 + li;
      const int hy = c / HX, hx = c - hy * HX;
      float xn[7];
      const int nbase = patch_base(c + 16);
#pragma unroll
      for (int t = 0; t < 7; ++t) xn[t] = j + 1 < NBT ? xin[nbase + off[t]] : 0.f;
      f32x4_t e0 = z, e1 = z;
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        e0 = mfma4(sa[0][t], xv[t], e0);
        e1 = mfma4(sa[1][t], xv[t], e1);
      }
#pragma unroll
      for (int t = 0; t < 7; ++t) xv[t] = xn[t];
      if (c < PIN) {
        if (interior) {  // (wave-uniform: no per-cell bounds test and selects)
          hid[g * PIN + c] = relu6x4(e0 + bs4[0]);
          hid[(4 + g) * PIN + c] = relu6x4(e1 + bs4[1]);
        } else {
          const bool in = hy0 + hy >= 0 && hy0 + hy < a.Ho && hx0 + hx >= 0 && hx0 + hx < a.Wo;
          hid[g * PIN + c] = in ? relu6x4(e0 + bs4[0]) : z;
          hid[(4 + g) * PIN + c] = in ? relu6x4(e1 + bs4[1]) : z;
        }
      }
    }
    __syncthreads();

    // ---- depthwise 3x3 + bias + ReLU6 (32 channels), straight into the K = 32
    // project MFMA (lane (li, g) holds pixel li's channel quad g of each half:
    // exactly its B-operand k-quad), + bias -> [B][Ho][Wo][16]
    if constexpr (PAIR) {
      // pixel tiles 2pp and 2pp + 1 hold vertically adjacent outputs in each
      // lane (row 2pp + 4 (li / 8) and the row below, column li % 8), so the
      // two 3x3 windows share 2 of their 4 input rows: 12 LDS reads, not 18
      static_assert(TX == 8 && TY == 8, "stem_ir1w: pair mapping assumes 8 x 8 tiles");
#pragma unroll 1
      for (int pp = 0; pp < 2; ++pp) {
        const int oy = 2 * pp + 4 * (li >> 3), ox = li & 7;
        f32x4_t acc0 = z, acc1 = z;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4_t* hp = hid + (4 * h + g) * PIN + oy * HX + ox;
          f32x4_t d0 = bd4[h], d1 = bd4[h];
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const f32x4_t v = hp[r * HX + kx];
              if (r < 3) d0 = __builtin_elementwise_fma(v, wd4[h][r * 3 + kx], d0);
              if (r > 0) d1 = __builtin_elementwise_fma(v, wd4[h][(r - 1) * 3 + kx], d1);
            }
          acc0 = mfma_k16(pa[h], relu6x4(d0), acc0);
          acc1 = mfma_k16(pa[h], relu6x4(d1), acc1);
        }
        const int gy = oy0 + oy, gx = ox0 + ox;
        float* yp = a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * 16 + 4 * g;
        if (gx < a.Wo) {
          if (gy < a.Ho) *reinterpret_cast<f32x4_t*>(yp) = acc0 + bp4;
          if (gy + 1 < a.Ho) *reinterpret_cast<f32x4_t*>(yp + static_cast<int64_t>(a.Wo) * 16) = acc1 + bp4;
        }
      }
    } else {
#pragma unroll 1
      for (int pt = 0; pt < NPT; ++pt) {
        const int q = pt * 16 + li;
        const int qq = q < TY * TX ? q : 0;
        const int cell = (qq / TX) * HX + (qq % TX);
        f32x4_t acc = z;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4_t* hp = hid + (4 * h + g) * PIN + cell;
          f32x4_t d = bd4[h];
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) d = __builtin_elementwise_fma(hp[ky * HX + kx], wd4[h][ky * 3 + kx], d);
          acc = mfma_k16(pa[h], relu6x4(d), acc);
        }
        const int gy = oy0 + qq / TX, gx = ox0 + qq % TX;
        if (q < TY * TX && gy < a.Ho && gx < a.Wo)
          *reinterpret_cast<f32x4_t*>(a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * 16 + 4 * g) =
              acc + bp4;
      }
    }
  }
}

// the hidden-split partials of irw_f32 (> 2 parts), added in part order
// (deterministic), + bias (+ residual)
__global__ void __launch_bounds__(256) irw_reduce_kernel(const float* __restrict__ ws, int parts, int64_t plane,
                                                         const float* __restrict__ bias, const float* __restrict__ x,
                                                         int cin, int cout, int residual, float* __restrict__ y) {
  const int64_t nq = plane / 4;
  for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < nq; q += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t e = q * 4;
    f32x4_t v = *reinterpret_cast<const f32x4_t*>(ws + e);
    for (int p = 1; p < parts; ++p) v += *reinterpret_cast<const f32x4_t*>(ws + p * plane + e);
    const int64_t pix = e / cout;
    const int co = static_cast<int>(e - pix * cout);
    v += *reinterpret_cast<const f32x4_t*>(bias + co);
    if (residual) v += *reinterpret_cast<const f32x4_t*>(x + pix * cin + co);
    *reinterpret_cast<f32x4_t*>(y + e) = v;
  }
}

// configurations (one instantiation each): MobileNetV2's fused blocks
struct IrF32Cfg {
  int S, TY, TX, HC, NOT, KIN;
  void (*kernel)(IrBlockF32Args);
  size_t (*lds)(int);
};

#define NNSX_IRF32(S, TY, TX, HC, NOT, KIN)                                                      \
  IrF32Cfg {                                                                                     \
    S, TY, TX, HC, NOT, KIN, &ir_block_f32_kernel<S, TY, TX, HC, NOT, KIN>,                      \
        &IrF32Geom<S, TY, TX, HC, NOT, KIN>::lds_bytes                                           \
  }

const IrF32Cfg kIrF32Cfgs[] = {
    // 112x112, t = 1 (32 -> 32 -> 16)
    NNSX_IRF32(1, 14, 14, 16, 1, 32),
    // 112 -> 56 (16 -> 96 -> 24)
    NNSX_IRF32(2, 8, 8, 16, 2, 16),
    // 56x56 (24 -> 144 -> 24)
    NNSX_IRF32(1, 14, 14, 16, 2, 24),
    // 56 -> 28 (24 -> 144 -> 32)
    NNSX_IRF32(2, 7, 7, 16, 2, 24),
    // 28x28 (32 -> 192 -> 32)
    NNSX_IRF32(1, 14, 14, 16, 2, 32),
    // 28 -> 14 (32 -> 192 -> 64)
    NNSX_IRF32(2, 7, 7, 16, 4, 32),
    // 14x14 (64 -> 384 -> 64 | 96, 96 -> 576 -> 96)
    NNSX_IRF32(1, 7, 7, 16, 4, 64),
    NNSX_IRF32(1, 7, 7, 16, 6, 64),
    NNSX_IRF32(1, 7, 7, 16, 6, 96),
};
#undef NNSX_IRF32

// tile shape per (stride, feature-map size): larger tiles cut the expand halo
// recompute (14x14 tile: 1.31x the useful pixels, 8x8: 1.75x) within the LDS
// budget of 2 workgroups per CU.  Any instantiated tile of the right stride
// is correct for any map size (partial tiles are masked); the preference only
// avoids partial tiles.
int tile_pref(int S, int H, int W, int TY, int TX) {
  const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
  const bool fits = Ho % TY == 0 && Wo % TX == 0;
  if (S == 1 && TY == 14 && TX == 14) return fits && Ho >= 28 ? 0 : 3;
  if (S == 2 && TY == 8 && TX == 8) return fits && Ho >= 56 ? 0 : 3;
  return fits ? 1 : 2;
}

#define NNSX_IRW(S, TY, TX, KIN, NOT, NW, F)                                                    \
  IrwCfg {                                                                                      \
    S, TY, TX, KIN, NOT, NW, F, &irw_f32_kernel<S, TY, TX, KIN, NOT, NW, F>,                    \
        &IrwGeom<S, TY, TX, KIN, NOT, NW, F>::lds_bytes, 1                                      \
  }
#define NNSX_IRWB(S, TY, TX, KIN, NOT, NW, F, MB)                                               \
  IrwCfg {                                                                                      \
    S, TY, TX, KIN, NOT, NW, F, &irw_f32_kernel<S, TY, TX, KIN, NOT, NW, F>,                    \
        &IrwGeom<S, TY, TX, KIN, NOT, NW, F>::lds_bytes, 1, MB                                  \
  }
// (NW = waves per workgroup: a divisor of the hidden subtile count where possible,
// so every wave walks the same number of 16-channel subtiles)
const IrwCfg kIrwCfgs[] = {
    NNSX_IRW(2, 4, 8, 16, 2, 3, true),     // 112 -> 56  16 -> 96 -> 24   (6 subtiles)
    NNSX_IRW(1, 8, 8, 24, 2, 3, true),     // 56x56      24 -> 144 -> 24  (9)
    NNSX_IRW(2, 4, 4, 24, 2, 3, true),     // 56 -> 28   24 -> 144 -> 32  (9)
    NNSX_IRW(2, 7, 4, 24, 2, 3, true),     // 56 -> 28   24 -> 144 -> 32  (9)
    NNSX_IRW(1, 7, 7, 32, 2, 4, false),    // 28x28      32 -> 192 -> 32  (12)
    NNSX_IRW(2, 2, 7, 32, 4, 4, false),    // 28 -> 14   32 -> 192 -> 64  (12)
    // 14x14 64 -> 384 -> 64 at batch >= 16: 7 x 14 tiles (expand 144 / 98 cells, project
    // 112 / 98 against 96 / 49, 64 / 49 at 7 x 7), 127.9 vs 140.5 us per block at batch 512
    // (profiles/r4_fp32_layers_b512_t714.txt); small batches keep the 7 x 7 tiles' parallelism
    NNSX_IRWB(1, 7, 14, 64, 4, 4, false, 16),
    NNSX_IRW(1, 7, 7, 64, 4, 4, false),    // 14x14      64 -> 384 -> 64  (24)
    NNSX_IRW(1, 7, 7, 64, 6, 4, false),    // 14x14      64 -> 384 -> 96  (24)
    NNSX_IRW(1, 7, 7, 96, 6, 4, false),    // 14x14      96 -> 576 -> 96  (36)
    NNSX_IRW(1, 7, 7, 160, 10, 4, false),  // 7x7       160 -> 960 -> 160 (60, two parts)
    NNSX_IRW(2, 7, 7, 96, 10, 4, false),   // 14 -> 7    96 -> 576 -> 160 (36, two parts; 154 KB LDS)
    // expand + depthwise only (NOT = 0: the depthwise output goes to HBM and
    // the project is a plain GEMM): 7x7 160 -> 960 whose project (-> 320)
    // needs more accumulators than a wave holds
    NNSX_IRW(1, 7, 7, 160, 0, 4, false),
    // candidates with less halo / padding work (A/B with NNSX_IRW_SKIP=<indices of
    // the defaults above>; find_irw takes the first configuration that fits)
    NNSX_IRW(1, 7, 14, 32, 2, 4, false),   // 28x28: expand 136/98 cells, project 112/98 (7x7: 88/49, 64/49)
    NNSX_IRW(1, 8, 16, 24, 2, 3, true),    // 56x56: expand 192/128 (8x8: 112/64)
    NNSX_IRW(2, 4, 8, 24, 2, 3, true),     // 56 -> 28: expand 160/128 input px (4x4: 96/64)
    NNSX_IRW(2, 8, 8, 16, 2, 3, true),     // 112 -> 56: expand 304/256 (4x8: 160/128)
    // SSD-300's 10x10 stage (exact 5 x 5 tiles: 2 x 2 tiles of 7 x 7 computed 196 cells
    // per 100 outputs) -- found only for maps a multiple of 5 that no 7 x 7 tile fits
    NNSX_IRW(1, 5, 5, 160, 10, 4, false),  // 10x10     160 -> 960 -> 160
    NNSX_IRW(2, 5, 5, 96, 10, 4, false),   // 19 -> 10   96 -> 576 -> 160
    NNSX_IRW(1, 5, 5, 160, 0, 4, false),   // 10x10     160 -> 960 (expand + depthwise)
    NNSX_IRW(1, 7, 14, 64, 6, 4, false),   // 14x14 64 -> 384 -> 96
    NNSX_IRW(1, 7, 14, 96, 6, 4, false),   // 14x14 96 -> 576 -> 96: expand 144/98 cells (7x7: 96/49), project 112/98
    // SSD's 19x19 blocks (least padding: 20 x 20 outputs per 19 x 19): 5 x 10 tiles -- the
    // 7 x 7 tile's LDS and registers, 525 expand cells per image against 625 on 5 x 5 --
    // and the 5 x 5 tiles
    NNSX_IRW(1, 5, 10, 96, 6, 4, false),   // 96 -> 576 -> 96
    NNSX_IRW(1, 5, 10, 64, 4, 4, false),   // 64 -> 384 -> 64
    NNSX_IRW(1, 5, 10, 64, 6, 4, false),   // 64 -> 384 -> 96
    NNSX_IRW(1, 5, 5, 96, 6, 4, false),
    NNSX_IRW(1, 5, 5, 64, 4, 4, false),
    NNSX_IRW(1, 5, 5, 64, 6, 4, false),
    // 32 -> 192 -> 32 on SSD's 38x38 and DeepLab's 65x65 maps (1600 / 4550 outputs against
    // 1764 / 4900 on 7 x 7) and 24 -> 144 -> 24 on SSD's 75x75 (exact) and DeepLab's 129x129:
    // SSD b64 1.786 -> 1.758 ms, DeepLab b8 0.947 -> 0.944 ms.  (Measured and dropped: 11 x 5
    // tiles on DeepLab's 33x33 blocks -- 1155 outputs per 1089, no gain -- and exact 5 x 13
    // tiles on 65x65, +1 % there: its x3 twin's 32-pixel project tiles hold 96 per 65;
    // profiles/r5_odd_map_tiles.txt)
    NNSX_IRW(1, 5, 10, 32, 2, 4, false),
    NNSX_IRW(1, 5, 15, 24, 2, 3, true),
    // (dilation 2 -- DeepLab's output-stride-16 blocks on 33x33 maps -- as
    // NNSX_IRWD(1, 7, 7, 160, 10, 4, false, 2) etc. ran 156 vs 120 us for the
    // unfused expand GEMM + dilated depthwise + project GEMM at batch 8 (the
    // 11x11 halo window needs 112 KB of LDS: one workgroup per CU), and at
    // batch 1 / 2 0.499 / 0.654 vs 0.488 / 0.565 ms per step, so the dilated
    // blocks stay unfused: profiles/r3_config_trace_deeplab_b8.txt,
    // profiles/r5_deeplab_b1.txt)
    // (one wave per 16-channel subtile -- 6 waves on 112 -> 56, 9 on 56 -> 28 --
    // ran 2x slower: the hidden images of all waves then limit the CU to one
    // workgroup; profiles/r3_irw_waves_ab_b512.txt)
};
#undef NNSX_IRW
#undef NNSX_IRWB

// NNSX_X3_IRW (A/B): 1 = every fused block on its irw_x3 twin, 2 = every
// block with an expand-x3 twin (irw_f32 XE) on it; unset = the measured defaults
static int x3_irw_mode() {
  static const int m = [] {
    const char* e = std::getenv("NNSX_X3_IRW");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  return m;
}
bool x3_irw_enabled() { return x3_irw_mode() == 1; }

// the expand-x3 twins (irw_f32_kernel<..., XE = true>) of the native configurations
#define NNSX_IRWE(S, TY, TX, KIN, NOT, NW, F)                                                   \
  IrwCfg {                                                                                      \
    S, TY, TX, KIN, NOT, NW, F, &irw_f32_kernel<S, TY, TX, KIN, NOT, NW, F, 1, true>,           \
        &IrwXEGeom<S, TY, TX, KIN, NOT, NW, F, 1, true>::lds_bytes, 1                           \
  }
const IrwCfg kIrwXECfgs[] = {
    NNSX_IRWE(2, 4, 8, 16, 2, 3, true),   NNSX_IRWE(1, 8, 8, 24, 2, 3, true),   NNSX_IRWE(2, 4, 4, 24, 2, 3, true),
    NNSX_IRWE(2, 2, 7, 32, 4, 4, false),  NNSX_IRWE(1, 7, 14, 64, 4, 4, false), NNSX_IRWE(1, 7, 7, 64, 4, 4, false),
    NNSX_IRWE(1, 7, 7, 64, 6, 4, false),  NNSX_IRWE(1, 7, 7, 96, 6, 4, false),  NNSX_IRWE(2, 7, 7, 96, 10, 4, false),
};
#undef NNSX_IRWE

// the expand-x3 twin of a native configuration (same tile, waves and parts)
static const IrwCfg* xe_twin(const IrwCfg* c, const IrBlockF32Args& a) {
  if (!c || f32_math() != F32Math::kX3 || !a.we3 || !a.has_expand) return nullptr;
  // by default where measured faster (scripts/x3_blocks_ab.py with NNSX_X3_IRW=2,
  // batch 512, profiles/r5_xe_blocks_ab.txt): 56 -> 28 265 -> 244 us, 28 -> 14
  // 129 -> 121 us; 56x56 and the 14x14 blocks lost 6-27 % (the split planes'
  // LDS and the extra registers; the 14x14 configurations spill)
  const bool dflt = c->S == 2 && ((c->KIN == 24 && c->TY == 4 && c->TX == 4) || (c->KIN == 32 && c->NOT == 4));
  if (x3_irw_mode() != 2 && !dflt) return nullptr;
  for (const IrwCfg& x : kIrwXECfgs)
    if (x.S == c->S && x.TY == c->TY && x.TX == c->TX && x.KIN == c->KIN && x.NOT == c->NOT && x.NW == c->NW &&
        x.full == c->full && x.dil == c->dil && x.lds(a.hid) <= 160 * 1024)
      return &x;
  return nullptr;
}

// the x3 twin of a configuration, when the method is x3 and both weight
// parts are given (the expand-only form needs no project weights)
const IrwCfg* x3_twin(const IrwCfg* c, const IrBlockF32Args& a) {
  if (!c || f32_math() != F32Math::kX3 || !a.we3 || (c->NOT > 0 && !a.wp3)) return nullptr;
  // by default only where the x3 kernel measured faster than the native one
  // (scripts/x3_blocks_ab.py, batch 512, profiles/r5_x3_blocks_ab_v2.txt): the
  // 960-hidden 7 x 7 blocks 155 vs 211 us, their expand + depthwise (the 960 ->
  // 320 chain) ~107 vs ~125 us, the 28 x 28 32 -> 192 -> 32 blocks 185 vs 192 us.
  // The LDS traffic of the split operands -- 3 x 16 B per 32-channel B fragment
  // against 2 x 16 B of fp32 -- bounds the other blocks.  (56 x 56 24 -> 144 ->
  // 24, 430 vs 447 us, stays native: at batch 1 its max error vs fp64 is 1.16x
  // the native kernel's -- the accuracy gate of test_gpu_x3.py.  The 5 x 10
  // 32-channel tiles stay native too: DeepLab b8's 65x65 blocks 22.4 vs 23.2-23.7
  // us, profiles/r5_deeplab_twins.txt, r5_parts3_n510.txt.)
  // NNSX_X3_IRW=1: every configuration with a twin that passes the accuracy gate
  // (A/B) -- not the 56x56 24 -> 144 -> 24 one (max error 1.16x native's at batch 1)
  const bool dflt = c->S == 1 && ((c->KIN == 160 && (c->NOT == 10 || c->NOT == 0)) || (c->KIN == 32 && c->NOT == 2 && c->TX != 10));
  const bool gate_fails = c->S == 1 && c->KIN == 24 && c->NOT == 2;
  if (x3_irw_mode() == 2 || (!x3_irw_enabled() && !dflt) || gate_fails) return xe_twin(c, a);
  // the same tile, else (7 x 14 tiles: their 4 32-pixel project tiles hold more
  // accumulators than two waves per SIMD allow) the 7 x 7 tile of the shape
  for (int pass = 0; pass < 2; ++pass)
    for (const IrwCfg& x : x3_irw_cfgs())
      if (x.S == c->S && (pass == 0 ? (x.TY == c->TY && x.TX == c->TX) : (x.TY == 7 && x.TX == 7 && c->TX == 14)) &&
          x.KIN == c->KIN && x.NOT == c->NOT && x.NW == c->NW && x.full == c->full && x.dil == c->dil &&
          x.lds(a.hid) <= 160 * 1024)
        return &x;
  return nullptr;
}

// indices of kIrwCfgs that find_irw skips (A/B experiments): NNSX_IRW_SKIP=1,4
bool irw_skipped(size_t i) {
  static const std::vector<size_t> skip = [] {
    std::vector<size_t> v;
    if (const char* e = std::getenv("NNSX_IRW_SKIP"))
      for (const char* p = e; *p;) {
        char* end = nullptr;
        const unsigned long x = std::strtoul(p, &end, 10);
        if (end == p) break;
        v.push_back(x);
        p = *end ? end + 1 : end;
      }
    return v;
  }();
  return std::find(skip.begin(), skip.end(), i) != skip.end();
}

const IrwCfg* find_irw(int S, int H, int W, int cin, int hid, int cout, bool has_expand, int dil = 1, int B = 0) {
  if (!has_expand || hid % 16) return nullptr;
  const int kin = (cin + 7) / 8 * 8;
  const int nout = (cout + 15) / 16;
  const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
  // an exact tiling first; else (odd maps: DeepLab's 129 / 65 / 33, SSD's 75 /
  // 38 / 19) the configuration of the shape with masked partial tiles that
  // computes the fewest padded outputs, the first in order on a tie (SSD's 19x19
  // blocks: 400 outputs per 361 on 5 x 5 tiles against 441 on 7 x 7, 1.917 ->
  // 1.886 ms per batch-64 step, profiles/r5_ssd_tiles.txt; on 5 x 10 tiles
  // (also 400, fewer halo cells) 1.864 -> 1.758 ms, profiles/r5_dw_dil.txt)
  const IrwCfg* best = nullptr;
  int64_t best_area = 0;
  for (int exact = 1; exact >= 0 && !best; --exact)
    for (size_t i = 0; i < sizeof(kIrwCfgs) / sizeof(kIrwCfgs[0]); ++i) {
      const IrwCfg& c = kIrwCfgs[i];
      if (c.S == S && c.dil == dil && c.KIN == kin && c.NOT == nout && (!exact || (Ho % c.TY == 0 && Wo % c.TX == 0)) &&
          c.lds(hid) <= 160 * 1024 && !irw_skipped(i) && (c.min_batch == 0 || (exact && B >= c.min_batch)) &&
          (c.max_batch == 0 || (B > 0 && B <= c.max_batch))) {
        if (exact) return &c;
        const int64_t area = static_cast<int64_t>((Ho + c.TY - 1) / c.TY * c.TY) * ((Wo + c.TX - 1) / c.TX * c.TX);
        if (!best || area < best_area) {
          best = &c;
          best_area = area;
        }
      }
    }
  return best;
}

const IrwCfg* find_irw_dw(int S, int H, int W, int cin, int hid, int dil = 1, int B = 0) {
  if (hid % 16) return nullptr;
  const int kin = (cin + 7) / 8 * 8;
  const int Ho = (H - 1) / S + 1, Wo = (W - 1) / S + 1;
  for (int exact = 1; exact >= 0; --exact)
    for (size_t i = 0; i < sizeof(kIrwCfgs) / sizeof(kIrwCfgs[0]); ++i) {
      const IrwCfg& c = kIrwCfgs[i];
      if (c.NOT == 0 && c.S == S && c.dil == dil && c.KIN == kin && (!exact || (Ho % c.TY == 0 && Wo % c.TX == 0)) &&
          c.lds(hid) <= 160 * 1024 && !irw_skipped(i) && (c.max_batch == 0 || (B > 0 && B <= c.max_batch)))
        return &c;
    }
  return nullptr;
}

const IrF32Cfg* find_cfg(int S, int H, int W, int cin, int hid, int cout, bool has_expand) {
  const int kin = (cin + 7) / 8 * 8;
  const int nout = (cout + 15) / 16;
  if (!has_expand && hid != cin) return nullptr;
  const IrF32Cfg* best = nullptr;
  int best_pref = 1 << 30;
  for (const auto& c : kIrF32Cfgs) {
    if (c.S != S || c.KIN != kin || c.NOT != nout || hid % c.HC) continue;
    if (c.lds(hid) > 160 * 1024) continue;
    const int pref = tile_pref(S, H, W, c.TY, c.TX);
    if (pref < best_pref) {
      best = &c;
      best_pref = pref;
    }
  }
  return best;
}

}  // namespace

// ---- fp32 product method ----------------------------------------------------
// kX3: the fp32 GEMM-shaped products on split-bf16 MFMAs (split_x3: error vs
// fp64 below the native fp32 MFMA's); kNative: v_mfma_f32_16x16x4_f32.  The
// process default comes from NNSX_F32_MATH (x3 | fp32); graph capture bakes the
// method in at capture time.
static F32Math g_f32_math = [] {
  const char* e = std::getenv("NNSX_F32_MATH");
  if (e && (std::string(e) == "fp32" || std::string(e) == "native")) return F32Math::kNative;
  return F32Math::kX3;
}();
F32Math f32_math() { return g_f32_math; }
void set_f32_math(F32Math m) { g_f32_math = m; }
const char* f32_math_name(F32Math m) { return m == F32Math::kX3 ? "x3" : "fp32"; }

// K-split slices for a small output grid (the classifier: M = batch, 32
// tiles of 64 x 64) -- otherwise most CUs idle while each workgroup walks all
// of K.  Returns the k-stages per slice (kstages: no split).
static int gemm_kchunk(int tiles, int kstages, int N, bool plain) {
  // (K < 384: the reduce launch costs about what the split saves -- DeepLab's
  // batch-1 ASPP 1x1 conv, K = 320, runs unsplit: one launch fewer)
  if (!plain || tiles >= 128 || kstages < 12 || N % 4) return kstages;
  const int splits = std::min(kstages / 4, (512 + tiles - 1) / tiles);
  return (kstages + splits - 1) / splits;
}

template <int BM, int BN>
static int gemm_splits(int M, int N, int Kpad, bool plain) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int kstages = (Kpad + GKT - 1) / GKT;
  const int chunk = gemm_kchunk(tiles, kstages, N, plain);
  return (kstages + chunk - 1) / chunk;
}

template <int BM, int BN>
static void pw_gemm_f32_launch(const float* x, const float* wt, const float* bias, const float* res, float* y, int M,
                               int N, int K, int Kpad, int Npad, int act, float* ws, hipStream_t s,
                               const YLayout& yl = YLayout{}, X3W w3 = X3W{}) {
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN);
  const int kstages = (Kpad + GKT - 1) / GKT;
  int chunk = (ws && !yl.rpb && !yl.brpb && !yl.pool) ? gemm_kchunk(static_cast<int>(grid.x * grid.y), kstages, N, !res) : kstages;
  grid.z = static_cast<unsigned>((kstages + chunk - 1) / chunk);
  const bool x3 = f32_math() == F32Math::kX3;
  // pre-split weights must cover every row and k-stage a tile reads
  const bool w3ok = x3 && w3.p && w3.stages >= kstages && w3.rows >= static_cast<int>(grid.y) * BN;
  const bool split = grid.z > 1;
  float* out = split ? ws : y;
  const YLayout ylo = split ? YLayout{} : yl;
  const int kc = split ? chunk : kstages;
  if (x3)
    pw_gemm_x3_launch(BM, BN, w3ok, grid, s, x, wt, w3ok ? w3 : X3W{}, bias, res, out, M, N, K, Kpad, Npad, act, kc,
                      ylo);
  else
    hipLaunchKernelGGL((pw_gemm_f32_kernel<BM, BN>), grid, dim3(256), 0, s, x, wt, X3W{}, bias, res, out, M, N, K, Kpad,
                       Npad, act, kc, ylo);
  if (!split) return;
  const int64_t nq = static_cast<int64_t>(M) * N / 4;
  const unsigned rg = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((nq + 255) / 256, 2048)));
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(rg), dim3(256), 0, s, ws, static_cast<int>(grid.z), M, N, bias,
                     act, y);
}

// Tile choice: the candidate with the least modelled time, where a workgroup
// costs its MFMA work (BM x BN x Kpad, padding included) plus a fixed
// prologue/epilogue share, and the grid runs in rounds of 512 co-resident
// workgroups (256 CUs x 2; every tile here fits two per CU in LDS).
static int pick_gemm_tile(int M, int N, int Kpad) {
  // x3: 64 x 64 tiles, but 128 x 64 for deep products (K >= 768) on large grids.
  // Measured (profiles/r5_x3_tiles_w3.txt, pre-split weights): 64 x 64 is the
  // best or within 0.5 % on every benched shape but the 7x7 chain's 960 -> 320
  // (122 vs 113.5 us at 128 x 64); DeepLab's 8712 x 320 x 256 19.0 vs 22.9 us,
  // MobileNetV2's 100352 x 96 x 576 118.8 vs 125.3, PoseNet's 69696 x 256 x 256
  // 74.7 vs 79.5.
  // (the batch-512 classifier, 512 x 1280 x 1000, keeps 128 x 64 as below)
  // Deep products take 128 x 64 only on a grid of >= 3 workgroups per CU (or a
  // split-K grid): under that the 64 x 64 grid's two resident workgroups per CU
  // win -- DeepLab b8's 8712 x 960 -> 160 / 320 projects 40.7 -> 34.5 / 55.3 ->
  // 47.3 us, SSD b64's 6400 x 1280 -> 256 47.2 -> 40.4, PoseNet b64's 5184 x
  // 1024 -> 1024 even (profiles/r5_gemm_fill.txt)
  if (f32_math() == F32Math::kX3 && M >= 64) {
    // wide products on large grids: 64 x 128 tiles (each staged, split activation
    // tile feeds twice the columns) -- MobileNetV2 b512's 25088 x 320 -> 1280 head
    // 164.5 -> 149.7 us, PoseNet b64's 18496 x 512 -> 512 75.1 -> 72.0 and 5184 x
    // 1024 -> 1024 86.3 -> 81.9 (profiles/r5_gemm_fill.txt)
    if (N >= 512 && Kpad >= 256 && (M >= 16384 || Kpad >= 1024) &&
        static_cast<int64_t>((M + 63) / 64) * ((N + 127) / 128) >= 256)
      return 64128;
    const bool big = static_cast<int64_t>((M + 63) / 64) * ((N + 63) / 64) >= 128;
    const int64_t t128 = static_cast<int64_t>((M + 127) / 128) * ((N + 63) / 64);
    const bool deep = (M >= 8192 && Kpad >= 768) || (M >= 512 && Kpad >= 1024);
    return big && deep && (t128 >= 768 || t128 < 128) ? 128064 : 64064;
  }
  // Large grids (>= 128 tiles of 64 x 64; M >= 8192, or M >= 512 with a deep
  // K): 128 x 64 tiles, which re-read the weights half as often per output.
  // The round model below ties them with 64 x 64 there; measured at batch 512
  // (M = 25088 / 512): 7x7 expand + project chain 300 -> 289 us, head 210 ->
  // 203 us, classifier 37 -> 24 us.  At batch 128 (M = 6272) the same switch
  // was neutral to slightly slower (chain 89 -> 92 us), so it stays off there.
  if (M >= 512 && (M >= 8192 || Kpad >= 1024) &&
      static_cast<int64_t>((M + 63) / 64) * ((N + 63) / 64) >= 128)
    return 128064;
  static const int cand[][2] = {{64, 64}, {128, 64}, {64, 128}, {128, 128}};
  int best = 0;
  double best_t = 1e30;
  for (int i = 0; i < 4; ++i) {
    const int bm = cand[i][0], bn = cand[i][1];
    const double tiles = static_cast<double>((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const double rounds = std::ceil(tiles / 512.0);
    // per-workgroup time ~ MFMA cycles (4 SIMDs) + ~25 % of a 32-k stage per k-stage of fill/drain
    const double per_wg = static_cast<double>(bm) * bn * (Kpad + 96) / 4.0;
    // a partially filled last round still costs a whole workgroup time per slot, but a
    // CU with one resident workgroup runs it at about 1.3x the two-workgroup rate
    const double t = rounds * per_wg * (tiles < 256 ? 0.75 : 1.0);
    if (t < best_t * 0.97) {
      best_t = t;
      best = i;
    }
  }
  return cand[best][0] * 1000 + cand[best][1];
}

// (tile > 0: an instantiated tile asked for by the caller -- pw_conv_f32_tile, A/B tools)
static int resolve_tile(int M, int N, int Kpad, int tile) { return tile > 0 ? tile : pick_gemm_tile(M, N, Kpad); }

// small-M GEMMs (batch-1 projects / head / classifier) run pw_small_f32: one
// launch instead of a split-K GEMM + reduce
static bool use_small_m(int M, int K, int tile, const YLayout& yl) {
  // (a workgroup streams its rows' whole K range through one CU: at M = 49,
  // K = 960 -- the batch-1 7x7 project -- that took 16.7 us against 12 us for
  // the split-K GEMM + reduce, so the many-row deep-K shapes keep split-K;
  // a two-workgroup K split with order-free atomics needed a memset node
  // that cost more than it saved: profiles/r3b_b1_forward_trace.txt)
  return tile == 0 && M <= 64 && (M <= 16 || K <= 512) && !yl.rpb && !yl.brpb && !yl.pool;
}

size_t pw_gemm_f32_workspace_bytes(int M, int N, int Kpad, bool has_res, int tile) {
  if (use_small_m(M, static_cast<int>(Kpad), tile, YLayout{})) return 0;
  int splits = 1;
  switch (resolve_tile(M, N, Kpad, tile)) {
    case 64064: splits = gemm_splits<64, 64>(M, N, Kpad, !has_res); break;
    case 128064: splits = gemm_splits<128, 64>(M, N, Kpad, !has_res); break;
    case 64128: splits = gemm_splits<64, 128>(M, N, Kpad, !has_res); break;
    case 128192: splits = gemm_splits<128, 192>(M, N, Kpad, !has_res); break;
    default: splits = gemm_splits<128, 128>(M, N, Kpad, !has_res); break;
  }
  return splits > 1 ? static_cast<size_t>(splits) * M * N * sizeof(float) : 0;
}

void pw_gemm_f32(const float* x, const float* wt, const float* bias, const float* res, float* y, int M, int N, int K,
                 int Kpad, int Npad, int act, hipStream_t s, int tile, float* ws, const YLayout& yl, X3W w3) {
  if (use_small_m(M, Kpad, tile, yl)) {
    const dim3 grid(static_cast<unsigned>((N + 15) / 16), static_cast<unsigned>((M + 63) / 64));
    hipLaunchKernelGGL(pw_small_f32_kernel<false>, grid, dim3(256), 0, s, x, wt, bias, res, y, M, N, K, Kpad, Npad, act, 0);
    return;
  }
  switch (resolve_tile(M, N, Kpad, tile)) {
    case 64064: pw_gemm_f32_launch<64, 64>(x, wt, bias, res, y, M, N, K, Kpad, Npad, act, ws, s, yl, w3); break;
    case 128064: pw_gemm_f32_launch<128, 64>(x, wt, bias, res, y, M, N, K, Kpad, Npad, act, ws, s, yl, w3); break;
    case 64128: pw_gemm_f32_launch<64, 128>(x, wt, bias, res, y, M, N, K, Kpad, Npad, act, ws, s, yl, w3); break;
    case 128192: pw_gemm_f32_launch<128, 192>(x, wt, bias, res, y, M, N, K, Kpad, Npad, act, ws, s, yl, w3); break;
    default: pw_gemm_f32_launch<128, 128>(x, wt, bias, res, y, M, N, K, Kpad, Npad, act, ws, s, yl, w3); break;
  }
}

void pw_gemm_f32_group(const GemmProb* p, int n, hipStream_t s) {
  if (n <= 0 || n > kGroupMax) throw std::invalid_argument("pw_gemm_f32_group: 1..16 problems");
  GemmGroupArgs g;
  g.n = n;
  int64_t blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (p[i].yl.pool || p[i].yl.brpb || p[i].K % 4 || p[i].N % 4 || p[i].Kpad < p[i].K || p[i].Npad < p[i].N)
      throw std::invalid_argument("pw_gemm_f32_group: unsupported problem");
    g.p[i] = p[i];
    g.start[i] = static_cast<int>(blocks);
    blocks += static_cast<int64_t>((p[i].M + 63) / 64) * ((p[i].N + 63) / 64);
  }
  if (blocks <= 0 || blocks > (1 << 30)) throw std::invalid_argument("pw_gemm_f32_group: grid");
  g.start[n] = static_cast<int>(blocks);
  bool w3ok = true;
  for (int i = 0; i < n; ++i)
    w3ok = w3ok && p[i].w3.p && p[i].w3.stages >= (p[i].Kpad + GKT - 1) / GKT && p[i].w3.rows >= (p[i].N + 63) / 64 * 64;
  if (f32_math() == F32Math::kX3)
    pw_gemm_group_x3_launch(w3ok, static_cast<unsigned>(blocks), s, g);
  else
    hipLaunchKernelGGL((pw_gemm_group_f32_kernel<64, 64>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, g);
}

void dw3x3_f32_group(const DwProb* p, int n, hipStream_t s) {
  if (n <= 0 || n > kGroupMax) throw std::invalid_argument("dw3x3_f32_group: 1..16 problems");
  DwGroupArgs g;
  g.n = n;
  int64_t blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (p[i].C % 4) throw std::invalid_argument("dw3x3_f32_group: C % 4");
    g.p[i] = p[i];
    g.start[i] = static_cast<int>(blocks);
    const int64_t work = static_cast<int64_t>(p[i].B) * ((p[i].H + 3) / 4) * ((p[i].W + 3) / 4) * (p[i].C / 4);
    blocks += std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 16384));
  }
  g.start[n] = static_cast<int>(blocks);
  hipLaunchKernelGGL(dw3x3_group_f32_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, g);
}

void dw3x3_f32(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int C, int stride,
               int dil, int act, hipStream_t s) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  // Lane shapes (rows x columns of outputs per lane), measured with
  // scripts/dw_roofline.py (profiles/r4_dw_lane_shapes.txt): stride 1 4 x 4 --
  // 7x7x960 at batch 512 56.3 -> 39.4 us, 14x14x576 130.6 -> 96.2 us, PoseNet's
  // 17x17x512 21.2 -> 18.7 us; stride 2 2 x 2 -- 129 -> 65 x 64 66.3 -> 60.9 us.
  // Dilation 2: residue-grid lanes (dw3x3_f32_dil), DeepLab b8's 33x33x960 24.3 ->
  // 16.9 us, batch 1 6.0 -> 5.3 us (profiles/r5_dw_dil.txt).
  // The multi-pixel lanes only where they still give every CU a workgroup
  // (>= 256 x 256 lanes): at batch 1 their few long lanes leave most CUs idle --
  // PoseNet batch-1 p50 0.36 -> 0.38 ms, DeepLab 0.525 -> 0.543 ms.
  constexpr int rows = 4;
  const int R2 = stride == 1 ? 4 : 2, C2 = stride == 1 ? 4 : 2;
  const int64_t lanes = static_cast<int64_t>(B) * ((Ho + R2 - 1) / R2) * ((Wo + C2 - 1) / C2) * (C / 4);
  const bool big = lanes >= 65536;
  if (stride == 1 && dil == 2) {  // residue-grid lanes: 4 x 4 on large grids, else 2 x 2
    const int r = big ? 4 : 2;
    const int64_t work = static_cast<int64_t>(B) * ((H + 1) / 2 / r + 2) * ((W + 1) / 2 / r + 2) * (C / 4) * 4;
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 65535))));
    if (big)
      hipLaunchKernelGGL((dw3x3_f32_dil_kernel<4, 4, 2>), grid, dim3(256), 0, s, x, w, bias, y, B, H, W, C, act);
    else
      hipLaunchKernelGGL((dw3x3_f32_dil_kernel<2, 2, 2>), grid, dim3(256), 0, s, x, w, bias, y, B, H, W, C, act);
    return;
  }
  if (big && dil == 1) {
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((lanes + 255) / 256, 65535))));
    if (stride == 1)
      hipLaunchKernelGGL((dw3x3_f32_col_kernel<4, 1, 4>), grid, dim3(256), 0, s, x, w, bias, y, B, H, W, C, Ho, Wo, act);
    else
      hipLaunchKernelGGL((dw3x3_f32_col_kernel<2, 2, 2>), grid, dim3(256), 0, s, x, w, bias, y, B, H, W, C, Ho, Wo, act);
    return;
  }
  if (dil == 1) {  // (small grids: 4 rows per lane)
    const int64_t work = static_cast<int64_t>(B) * ((Ho + rows - 1) / rows) * Wo * (C / 4);
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 65535)));
    if (stride == 1)
      hipLaunchKernelGGL((dw3x3_f32_col_kernel<rows, 1>), dim3(grid), dim3(256), 0, s, x, w, bias, y, B, H, W, C, Ho, Wo,
                         act);
    else
      hipLaunchKernelGGL((dw3x3_f32_col_kernel<rows, 2>), dim3(grid), dim3(256), 0, s, x, w, bias, y, B, H, W, C, Ho, Wo,
                         act);
    return;
  }
  const int64_t work = static_cast<int64_t>(B) * Ho * Wo * (C / 4);
  const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 16384)));
  hipLaunchKernelGGL(dw3x3_f32_kernel, dim3(grid), dim3(256), 0, s, x, w, bias, y, B, H, W, C, Ho, Wo, stride, dil,
                     act);
}

template <typename T>
static void stem_f32_launch(const T* x, const float* w, const float* bias, float* y, int B, int H, int W, int act,
                            const float* lut, hipStream_t s) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const size_t lds = sizeof(float) * (2 * STEM_R + 1) * (W + 2) * 3;
  if (lds > 64 * 1024) {
    static const bool ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_f32_kernel<T>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!ok || lds > 160 * 1024) return;
  }
  const unsigned grid = static_cast<unsigned>(B * ((Ho + STEM_R - 1) / STEM_R));
  hipLaunchKernelGGL(stem_f32_kernel<T>, dim3(grid), dim3(256), lds, s, x, w, bias, y, H, W, Ho, Wo, act, lut);
}

void stem3x3_f32(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int act,
                 hipStream_t s) {
  stem_f32_launch<float>(x, w, bias, y, B, H, W, act, nullptr, s);
}

void stem3x3_u8_f32(const uint8_t* x, const float* w, const float* bias, float* y, int B, int H, int W, int act,
                    const float* lut, hipStream_t s) {
  stem_f32_launch<uint8_t>(x, w, bias, y, B, H, W, act, lut, s);
}

namespace {
__global__ void __launch_bounds__(256) x3_split_weights_kernel(const float* __restrict__ w, int rows, int cols,
                                                               uint16_t* __restrict__ out, int stages, int rows3) {
  // pairs (r, c), (r, c + 1) of consecutive k, c even; rows past `rows` are zeros
  const int64_t npair = static_cast<int64_t>(stages) * rows3 * 16;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; q < npair;
       q += static_cast<int64_t>(gridDim.x) * 256) {
    const int kp = static_cast<int>(q % 16);
    const int64_t rs = q / 16;
    const int r = static_cast<int>(rs % rows3), ks = static_cast<int>(rs / rows3);
    const int c = ks * 32 + 2 * kp;
    f32x2_t v;
    v[0] = r < rows && c < cols ? w[static_cast<int64_t>(r) * cols + c] : 0.f;
    v[1] = r < rows && c + 1 < cols ? w[static_cast<int64_t>(r) * cols + c + 1] : 0.f;
    bf16x2_t h, m, l;
    split2(v, h, m, l);
    uint16_t* o = out + (static_cast<int64_t>(ks) * rows3 + r) * 96 + 2 * kp;
    *reinterpret_cast<bf16x2_t*>(o) = h;
    *reinterpret_cast<bf16x2_t*>(o + 32) = m;
    *reinterpret_cast<bf16x2_t*>(o + 64) = l;
  }
}
}  // namespace

int x3_split_rows(int rows) { return (rows + 383) / 384 * 384; }

void x3_split_weights(const float* w, int rows, int cols, uint16_t* out, hipStream_t s) {
  if (rows <= 0 || cols <= 0) throw std::invalid_argument("x3_split_weights: empty weights");
  const int stages = (cols + GKT - 1) / GKT, rows3 = x3_split_rows(rows);
  const int64_t npair = static_cast<int64_t>(stages) * rows3 * 16;
  const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((npair + 255) / 256, 4096)));
  hipLaunchKernelGGL(x3_split_weights_kernel, dim3(grid), dim3(256), 0, s, w, rows, cols, out, stages, rows3);
}

void pw_pool_f32(const float* x, const float* wt, const float* bias, float* y, int B, int HW, int N, int K, int Kpad,
                 int Npad, int act, hipStream_t s, X3W w3) {
  // larger batches: the tiled GEMM with the pooling epilogue (no [B][HW][N]
  // head output in HBM and no avgpool launch)
  if (B > 8 && HW <= 64) {
    (void)hipMemsetAsync(y, 0, static_cast<size_t>(B) * N * sizeof(float), s);
    YLayout yl;
    yl.pool = HW;
    const int M = B * HW;
    if (M >= 8192)
      pw_gemm_f32_launch<128, 64>(x, wt, bias, nullptr, y, M, N, K, Kpad, Npad, act, nullptr, s, yl, w3);
    else
      pw_gemm_f32_launch<64, 64>(x, wt, bias, nullptr, y, M, N, K, Kpad, Npad, act, nullptr, s, yl, w3);
    return;
  }
  const dim3 grid(static_cast<unsigned>((N + 15) / 16), static_cast<unsigned>(B));
  hipLaunchKernelGGL(pw_small_f32_kernel<true>, grid, dim3(256), 0, s, x, wt, bias, nullptr, y, B * HW, N, K, Kpad, Npad,
                     act, HW);
}

void avgpool_f32(const float* x, float* y, int B, int HW, int C, hipStream_t s) {
  const int groups = (C / 4 + 15) / 16;
  if (B * groups >= 512 || HW < 256) {
    hipLaunchKernelGGL(avgpool_f32_kernel<16>, dim3(static_cast<unsigned>(B * groups)), dim3(256), 0, s, x, y, HW, C);
    return;
  }
  const int g4 = (C / 4 + 3) / 4;
  hipLaunchKernelGGL(avgpool_f32_kernel<4>, dim3(static_cast<unsigned>(B * g4)), dim3(256), 0, s, x, y, HW, C);
}

bool ir_block_f32_supported(int stride, int H, int W, int cin, int hid, int cout, bool has_expand, int dil, int B) {
  if (stride != 1 && stride != 2) return false;
  if (cin % 8 || cout % 4 || hid % 16) return false;
  if (f32_math() == F32Math::kX3 && B > 0) {
    // the image-per-workgroup x3 kernels (kernels/irp_x3.hip) cover some blocks
    // no fp32 kernel does (7 x 7 160 -> 960 -> 320); the callers pass the split weights
    IrBlockF32Args q;
    q.stride = stride;
    q.H = H;
    q.W = W;
    q.cin = cin;
    q.hid = hid;
    q.cout = cout;
    q.B = B;
    q.dil = dil;
    q.has_expand = has_expand;
    q.residual = stride == 1 && cin == cout;
    static const uint16_t dummy[8] = {};
    q.we3 = q.wp3 = dummy;
    if (irp_x3_supported(q)) return true;
  }
  if (dil != 1) return find_irw(stride, H, W, cin, hid, cout, has_expand, dil, B) != nullptr;
  return find_irw(stride, H, W, cin, hid, cout, has_expand) != nullptr ||
         find_cfg(stride, H, W, cin, hid, cout, has_expand) != nullptr;
}

// Hidden-channel parts per tile.  Fewer tiles than CUs: split the hidden
// channels over workgroups (every wave keeps >= 1 subtile).  The parts write
// workspace slabs that irw_reduce adds in part order.  (Adding two parts into a
// zeroed output with fp32 atomics was also
// deterministic but measured 86 vs 71 us on the 7x7 960-hidden block at batch
// 128: the L2 atomic unit, 4 B per request, is the bottleneck.)
static int irw_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// two hidden parts write workspace slabs like more parts (adding them into a
// zeroed output with fp32 atomics measured slower, above)
static bool irw_atomic2() { return false; }

// NNSX_F32_IRW_INLAUNCH: 0 = irw_reduce launch, 1 = last-arriver combine,
// 2 = spread combine (default: every part waits for its tile's other parts,
// then adds a 1/parts share; 64-bit monotone counters: two int32 ticket
// entries per tile).  Batch 1 at a 500 fps live camera: filter device time
// 317-319 vs 329-335 us, p50 356-363 vs 368-383 us with the reduce launches
// (profiles/r3_b1_launch_count_ab.txt); back-to-back replays are unchanged.
static int irw_inlaunch_mode() {
  static const int m = irw_env("NNSX_F32_IRW_INLAUNCH", 2);
  return m;
}

static thread_local bool t_device_shared = false;
SharedDeviceScope::SharedDeviceScope(bool on) : prev_(t_device_shared) { t_device_shared = prev_ || on; }
SharedDeviceScope::~SharedDeviceScope() { t_device_shared = prev_; }
bool device_shared() { return t_device_shared; }
bool set_device_shared(bool on) {
  const bool prev = t_device_shared;
  t_device_shared = on;
  return prev;
}

// the model's ticket buffer (ir_block_f32_tickets ints, zeroed once): the
// spread form's 64-bit counters in [0, kSpreadTickets), the last-arriver
// form's self-resetting ints after them (kLastTickets).  Hidden parts > 1 only
// below 256 tiles (irw_parts), so both regions hold every splitting launch.
constexpr int kSpreadTickets = 512, kLastTickets = 256;

// workgroups of configuration c the spread combine may keep waiting at once:
// one per CU under what the occupancy query reports (it can over-report)
static int irw_spread_slots(const IrwCfg* c, int hid) {
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(c->kernel), 64 * c->NW,
                                                   c->lds(hid)) != hipSuccess)
    return 0;
  return ncu * std::max(1, per_cu - 1);
}

static int irw_parts(const IrwCfg* c, int tiles, int hid) {
  const int nsub = hid / 16;
  if (c->NOT == 0)  // depthwise output: parts need no reduction, so fill the chip
    return std::max(1, std::min((1024 + tiles - 1) / tiles, nsub / c->NW));
  if (tiles >= 256 || nsub < 8) return 1;
  // (three parts where two leave the waves unevenly loaded -- DeepLab b8's 33x33
  // 96 -> 576 -> 96, 18 subtiles = 5 / 5 / 4 / 4 per wave -- measured slower:
  // DeepLab b8 +1.6 %, MobileNetV2 b128 -5.5 %, profiles/r5_parts3_n510.txt)
  if (tiles >= 128) return 2;
  const int want = (512 + tiles - 1) / tiles;
  int parts = std::max(2, std::min(want, nsub / c->NW));
  // more than 4 parts combine in the launch only in the spread form, which
  // needs the whole grid resident: trim the parts to what fits when that
  // keeps >= 3/4 of them (batch 8, 14x14 96 -> 576 -> 96: 8 parts of 32
  // tiles instead of 9 and an irw_reduce launch)
  if (parts > 4 && irw_inlaunch_mode() == 2) {
    const int fit = irw_spread_slots(c, hid) / tiles;
    if (fit < parts && 4 * fit >= 3 * parts) parts = fit;
  }
  return parts;
}

static void irw_geometry(const IrwCfg* c, IrBlockF32Args* a) {
  a->Ho = (a->H - 1) / a->stride + 1;
  a->Wo = (a->W - 1) / a->stride + 1;
  a->tiles_y = (a->Ho + c->TY - 1) / c->TY;
  a->tiles_x = (a->Wo + c->TX - 1) / c->TX;
  a->hsplit = irw_parts(c, a->tiles_x * a->tiles_y * a->B, a->hid);
}

static bool launch_irw(const IrwCfg* c, IrBlockF32Args a, hipStream_t s) {
  irw_geometry(c, &a);
  const int tiles = a.tiles_x * a.tiles_y * a.B;
  const int64_t plane = static_cast<int64_t>(a.B) * a.Ho * a.Wo * a.cout;
  const bool slabs = a.hsplit > 2 || (a.hsplit == 2 && !irw_atomic2());
  if (slabs && !a.ws) return false;  // the caller sizes the workspace (ir_block_f32_workspace_bytes)
  if (!slabs) a.ws = nullptr;
  const size_t lds = c->lds(a.hid);
  if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(c->kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
    return false;
  if (a.hsplit == 2 && !slabs) (void)hipMemsetAsync(a.y, 0, static_cast<size_t>(plane) * sizeof(float), s);
  // (a shared device -- replay lanes, other model instances -- may run this
  // block's launches concurrently, and the tickets are the model's one buffer:
  // the parts are then added by a separate reduce launch)
  if (!a.ws || tiles > kLastTickets || device_shared()) a.tickets = nullptr;
  a.spread = 0;
  if (a.tickets) {
    // the spread combine waits inside the launch for the other parts of a
    // tile: only when every workgroup of the grid is resident at once (one
    // block per CU under what the occupancy query reports, which can over-report)
    int dev = 0, ncu = 0, per_cu = 0;
    if (irw_inlaunch_mode() == 2 && 2 * tiles <= kSpreadTickets && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(c->kernel), 64 * c->NW, lds) ==
            hipSuccess &&
        static_cast<int64_t>(tiles) * a.hsplit <= static_cast<int64_t>(ncu) * std::max(1, per_cu - 1))
      a.spread = 1;
    else if (irw_inlaunch_mode() == 1 || a.hsplit <= 4)
      // last-arriver form (self-resetting int tickets, their own region of the
      // buffer: the spread form's counters there only grow): a grid larger than
      // the chip -- DeepLab's 33x33 blocks at batch 8, 200 tiles x 2 parts --
      // has few slabs per tile, so the last part adds them alone cheaply
      a.tickets += kSpreadTickets;
    else
      a.tickets = nullptr;  // (separate reduce launch: many slabs, spread over its grid)
  }
  hipLaunchKernelGGL(c->kernel, dim3(static_cast<unsigned>(tiles * a.hsplit)), dim3(64 * c->NW), lds, s, a);
  if (a.ws && !a.tickets) {
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((plane / 4 + 255) / 256, 4096)));
    hipLaunchKernelGGL(irw_reduce_kernel, dim3(grid), dim3(256), 0, s, a.ws, a.hsplit, plane, a.bp, a.x, a.cin,
                       a.cout, a.residual, a.y);
  }
  return true;
}

// used for small batches only: at batch 128 the 7x7 160 -> 960 expand GEMM +
// depthwise kernel (46 us) beat this kernel (54 us); at batch 1 it saves a
// launch and 4 us
bool ir_expand_dw_f32_supported(int stride, int H, int W, int cin, int hid, int B, int dil) {
  const IrwCfg* c = cin % 8 == 0 ? find_irw_dw(stride, H, W, cin, hid, dil, B) : nullptr;
  if (!c) return false;
  if (dil != 1) return true;  // (the alternative is an unfused dilated depthwise pass over the hidden map)
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  return B <= 0 || B * (Ho / c->TY) * (Wo / c->TX) <= 32;
}

bool ir_expand_dw_f32(const IrBlockF32Args& args, hipStream_t s) {
  IrBlockF32Args a = args;
  const IrwCfg* c = find_irw_dw(a.stride, a.H, a.W, a.cin, a.hid, a.dil, a.B);
  if (!c || !a.has_expand) return false;
  if (const IrwCfg* x = x3_twin(c, a)) c = x;
  irw_geometry(c, &a);
  a.ws = nullptr;
  const size_t lds = c->lds(a.hid);
  if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(c->kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
    return false;
  const int tiles = a.tiles_x * a.tiles_y * a.B;
  hipLaunchKernelGGL(c->kernel, dim3(static_cast<unsigned>(tiles * a.hsplit)), dim3(64 * c->NW), lds, s, a);
  return true;
}

size_t ir_block_f32_workspace_bytes(const IrBlockF32Args& args) {
  if (f32_math() == F32Math::kX3 && irp_x3_supported(args)) return 0;  // (one image per workgroup: no parts)
  const IrwCfg* c = find_irw(args.stride, args.H, args.W, args.cin, args.hid, args.cout, args.has_expand != 0, args.dil,
                             args.B);
  if (!c) return 0;
  size_t best = 0;
  // (the x3 twin's parts can differ where they depend on residency: size for both)
  for (const IrwCfg* k : {c, x3_twin(c, args)}) {
    if (!k) continue;
    IrBlockF32Args a = args;
    irw_geometry(k, &a);
    if (a.hsplit < 2 || (a.hsplit == 2 && irw_atomic2())) continue;
    best = std::max(best, static_cast<size_t>(a.hsplit) * a.B * a.Ho * a.Wo * a.cout * sizeof(float));
  }
  return best;
}

// the in-launch combine of the hidden parts: the spread form by default when
// the grid is resident, else the last-arriver form for <= 4 parts
// (irw_inlaunch_mode, launch_irw); the last-arriver form everywhere
// (NNSX_F32_IRW_INLAUNCH=1) measured at batch 1
// (profiles/r3_b1_inlaunch_combine_trace.txt):
// with release/acquire fences and per-block ticket fills, 456 vs 306 us per
// forward; with write-through slabs, no fences and self-resetting tickets,
// still 386 us -- the last part of a tile adds all slabs alone (15 slabs x 31 KB
// on the 7x7 960-hidden block: 50 vs 16 + 5.5 us for the kernel + irw_reduce,
// whose grid spreads the same adds over many workgroups).
size_t ir_block_f32_tickets(const IrBlockF32Args& args) {
  const int mode = irw_inlaunch_mode();
  if (!mode || !ir_block_f32_workspace_bytes(args)) return 0;
  IrBlockF32Args a = args;
  const IrwCfg* c = find_irw(a.stride, a.H, a.W, a.cin, a.hid, a.cout, a.has_expand != 0, a.dil, a.B);
  if (!c || c->NOT == 0) return 0;
  irw_geometry(c, &a);
  return a.tiles_x * a.tiles_y * a.B <= kLastTickets ? kSpreadTickets + kLastTickets : 0;
}

// one wave per 8 x 8 tile (stem_ir1w_f32_kernel)
constexpr int kStemW = 8;
static size_t stem_ir1w_lds_bytes() {
  constexpr int HY = kStemW + 2, HX = kStemW + 2, PIN = HY * HX;
  constexpr int NIN = (2 * HY + 1) * (2 * HX + 1) * 3;
  return static_cast<size_t>((NIN + 3) / 4 * 4 + 256) * 4 + 16 * 8 * PIN;
}

// (variants measured and removed: the 8-wave 16 x 16 tile kernel -- 510-525 us
// against 492-514 at batch 512, profiles/r2_pmc_stem_ir1.txt -- and the
// line-buffer band kernel -- 552.6 vs 471.0 us, barrier-bound,
// profiles/r4_fp32_layers_b512_final.txt)
bool stem_ir1_f32(const StemIr1F32Args& args, hipStream_t s) {
  StemIr1F32Args a = args;
  a.Ho = (a.H - 1) / 2 + 1;
  a.Wo = (a.W - 1) / 2 + 1;
  a.tiles_y = (a.Ho + kStemW - 1) / kStemW;
  a.tiles_x = (a.Wo + kStemW - 1) / kStemW;
  const size_t lds = stem_ir1w_lds_bytes();
  const void* fn = reinterpret_cast<const void*>(&stem_ir1w_f32_kernel<kStemW, kStemW, true>);
  // persistent grid: exactly the waves that fit resident at once
  static const int resident = [fn, lds] {
    int dev = 0, ncu = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    return ncu * per_cu;
  }();
  const int tiles = a.tiles_x * a.tiles_y * a.B;
  const unsigned grid = static_cast<unsigned>(std::min(tiles, resident));
  hipLaunchKernelGGL((stem_ir1w_f32_kernel<kStemW, kStemW, true>), dim3(grid), dim3(64), lds, s, a);
  return true;
}

const char* ir_block_f32_method(int stride, int H, int W, int cin, int hid, int cout, int B, int dil) {
  {
    IrBlockF32Args q;
    q.stride = stride;
    q.H = H;
    q.W = W;
    q.cin = cin;
    q.hid = hid;
    q.cout = cout;
    q.B = B;
    q.dil = dil;
    static const uint16_t dummy[8] = {};
    q.we3 = q.wp3 = dummy;
    if (f32_math() == F32Math::kX3 && irp_x3_supported(q)) return "x3";
  }
  const IrwCfg* c = find_irw(stride, H, W, cin, hid, cout, true, dil, B);
  if (!c) return ir_block_f32_supported(stride, H, W, cin, hid, cout, true, dil) ? "fp32" : "";
  IrBlockF32Args a;
  a.hid = hid;
  static const uint16_t dummy[8] = {};
  a.we3 = a.wp3 = dummy;
  return x3_twin(c, a) ? "x3" : "fp32";
}

bool ir_block_f32(const IrBlockF32Args& args, hipStream_t s) {
  IrBlockF32Args a = args;
  // 14 x 14 blocks on the x3 method: one image per workgroup (kernels/irp_x3.hip)
  if (f32_math() == F32Math::kX3 && irp_x3(a, s)) return true;
  if (const IrwCfg* w = find_irw(a.stride, a.H, a.W, a.cin, a.hid, a.cout, a.has_expand != 0, a.dil, a.B)) {
    if (const IrwCfg* x = x3_twin(w, a)) return launch_irw(x, a, s);
    return launch_irw(w, a, s);
  }
  if (a.dil != 1) return false;
  const IrF32Cfg* c = find_cfg(a.stride, a.H, a.W, a.cin, a.hid, a.cout, a.has_expand != 0);
  if (!c) return false;
  a.Ho = (a.H - 1) / a.stride + 1;
  a.Wo = (a.W - 1) / a.stride + 1;
  a.tiles_y = (a.Ho + c->TY - 1) / c->TY;
  a.tiles_x = (a.Wo + c->TX - 1) / c->TX;
  const size_t lds = c->lds(a.hid);
  if (lds > 64 * 1024) {
    // opt in to the full 160 KiB once per instantiation
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(c->kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return false;
  }
  const unsigned grid = static_cast<unsigned>(a.tiles_x * a.tiles_y * a.B);
  hipLaunchKernelGGL(c->kernel, dim3(grid), dim3(256), lds, s, a);
  return true;
}

}  // namespace kernels
}  // namespace nnsx
