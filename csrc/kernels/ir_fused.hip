// Fused MobileNetV2 inverted-residual block for gfx950:
//   y = project(dw3x3(expand(x))) (+ x)
// in ONE kernel, the 6x-wide hidden activation never leaves the CU.
//
// The unfused chain (pw_gemm -> dw3x3 -> pw_gemm) moves the hidden tensor
// through HBM four times (expand write, dw read, dw write, project read); at
// batch 256 that is ~85% of MobileNetV2's 26 MB/frame of activation traffic
// and both kernels sit at ~2 TB/s.  Here each workgroup owns an 8x8 output
// tile of one image:
//
//   1. the input halo tile ((8-1)*s+3)^2 x Cin is staged once in LDS (zero
//      padded: out-of-image pixels are zero, K padded to 32);
//   2. the hidden channels are walked in chunks of 32:
//        expand  : MFMA 16x16x32 bf16, D[hid][px] = We[hid][k] . X[px][k]^T,
//                  bias + ReLU6, halo pixels outside the image forced to 0
//                  (= the dw conv's zero padding), bf16 into LDS;
//        dw 3x3  : one lane = 1 output pixel x 8 channels from LDS,
//                  bias + ReLU6, bf16 into LDS;
//        project : MFMA accumulate D[out][px] += Wp[out][hid] . dw[px][hid]^T
//                  into registers (wave w owns output pixels 16w..16w+15);
//   3. epilogue: bias + residual (read from the LDS input tile) -> bf16 NHWC.
//
// HBM traffic per block drops to input + output (+ weights through L2).
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
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
__device__ __forceinline__ float relu6(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

constexpr int TO = 8;       // output tile edge
constexpr int HC = 32;      // hidden channels per chunk (= one MFMA K step)
constexpr int HROW = HC + 8;  // LDS row pitch (elements) of the hidden / dw tiles

__host__ __device__ constexpr int tile_in(int s) { return (TO - 1) * s + 3; }
__host__ __device__ constexpr int tile_in_px16(int s) { return (tile_in(s) * tile_in(s) + 15) / 16 * 16; }

template <int S, int NOT>
__global__ void __launch_bounds__(256) ir_block_kernel(IrBlockArgs a) {
  constexpr int TI = tile_in(S);
  constexpr int PIN = TI * TI;
  constexpr int PIN16 = tile_in_px16(S);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int xrow = a.cin32 + 8;  // LDS pitch of the input tile
  uint16_t* xs = smem;                        // [PIN16][xrow]
  uint16_t* hid = xs + PIN16 * xrow;          // [PIN16][HROW]
  uint16_t* dwo = hid + PIN16 * HROW;         // [64][HROW]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 15;
  const int kq = (lane >> 4) * 8;

  // block -> (image, tile)
  const int tiles = a.tiles_x * a.tiles_y;
  const int b = blockIdx.x / tiles;
  const int t = blockIdx.x % tiles;
  const int ty = t / a.tiles_x, tx = t % a.tiles_x;
  const int oy0 = ty * TO, ox0 = tx * TO;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- 1. stage the input halo tile (16-byte vectors; zero outside the image / K pad)
  const uint16_t* xb = a.x + static_cast<int64_t>(b) * a.H * a.W * a.cin;
  const int vec_per_px = a.cin32 / 8;
  for (int v = tid; v < PIN16 * vec_per_px; v += 256) {
    const int p = v / vec_per_px;
    const int k = (v % vec_per_px) * 8;
    bf16x8_t val = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    if (p < PIN && k < a.cin) {
      const int iy = iy0 + p / TI, ix = ix0 + p % TI;
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        val = *reinterpret_cast<const bf16x8_t*>(xb + (static_cast<int64_t>(iy) * a.W + ix) * a.cin + k);
    }
    *reinterpret_cast<bf16x8_t*>(xs + p * xrow + k) = val;
  }
  __syncthreads();

  f32x4_t acc[NOT];
#pragma unroll
  for (int i = 0; i < NOT; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ksteps = a.cin32 / 32;
  for (int c0 = 0; c0 < a.hid; c0 += HC) {
    // ---- 2a. expand (or copy, for t=1 blocks) into hid[px][0..32)
    if (a.has_expand) {
      constexpr int NB = PIN16 / 16;
      for (int pair = wave; pair < 2 * NB; pair += 4) {
        const int at = pair & 1, bt = pair >> 1;
        f32x4_t e = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const uint16_t* wrow = a.we + static_cast<int64_t>(c0 + at * 16 + li) * a.cin32 + kq;
        const uint16_t* xrowp = xs + (bt * 16 + li) * xrow + kq;
        for (int ks = 0; ks < ksteps; ++ks) {
          const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(wrow + ks * 32);
          const bf16x8_t bf = *reinterpret_cast<const bf16x8_t*>(xrowp + ks * 32);
          e = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, af),
                                                      __builtin_bit_cast(bf16x8_mfma, bf), e, 0, 0, 0);
        }
        // lane: hidden rows (lane>>4)*4+r of tile `at`, pixel bt*16+li
        const int p = bt * 16 + li;
        const int iy = iy0 + p / TI, ix = ix0 + p % TI;
        const bool inside = p < PIN && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const int hc = at * 16 + (lane >> 4) * 4;
        uint16_t o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = inside ? f2bf(relu6(e[r] + a.be[c0 + hc + r])) : 0;
        uint2 packed;
        packed.x = static_cast<uint32_t>(o[0]) | (static_cast<uint32_t>(o[1]) << 16);
        packed.y = static_cast<uint32_t>(o[2]) | (static_cast<uint32_t>(o[3]) << 16);
        *reinterpret_cast<uint2*>(hid + p * HROW + hc) = packed;
      }
    } else {
      for (int v = tid; v < PIN16 * (HC / 8); v += 256) {
        const int p = v / (HC / 8), k = (v % (HC / 8)) * 8;
        *reinterpret_cast<bf16x8_t*>(hid + p * HROW + k) = *reinterpret_cast<const bf16x8_t*>(xs + p * xrow + c0 + k);
      }
    }
    __syncthreads();

    // ---- 2b. depthwise 3x3 + bias + ReLU6: lane = 1 output pixel x 8 channels
    {
      const int q = tid >> 2;
      const int g = (tid & 3) * 8;
      const int oy = q / TO, ox = q % TO;
      float d[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) d[r] = a.bd[c0 + g + r];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int p = (oy * S + ky) * TI + (ox * S + kx);
          const bf16x8_t hv = *reinterpret_cast<const bf16x8_t*>(hid + p * HROW + g);
          const bf16x8_t wv = *reinterpret_cast<const bf16x8_t*>(a.wd + (ky * 3 + kx) * a.hid + c0 + g);
#pragma unroll
          for (int r = 0; r < 8; ++r)
            d[r] += bf2f(static_cast<uint16_t>(hv[r])) * bf2f(static_cast<uint16_t>(wv[r]));
        }
      bf16x8_t o;
#pragma unroll
      for (int r = 0; r < 8; ++r) o[r] = static_cast<short>(f2bf(relu6(d[r])));
      *reinterpret_cast<bf16x8_t*>(dwo + q * HROW + g) = o;
    }
    __syncthreads();

    // ---- 2c. project: wave owns output pixels 16*wave .. +15
    {
      const bf16x8_t bf = *reinterpret_cast<const bf16x8_t*>(dwo + (wave * 16 + li) * HROW + kq);
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot) {
        const bf16x8_t af =
            *reinterpret_cast<const bf16x8_t*>(a.wp + static_cast<int64_t>(ot * 16 + li) * a.hid + c0 + kq);
        acc[ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, af),
                                                          __builtin_bit_cast(bf16x8_mfma, bf), acc[ot], 0, 0, 0);
      }
    }
  }

  // ---- 3. epilogue: bias (+ residual from the LDS input tile) -> bf16
  const int q = wave * 16 + li;
  const int oy = q / TO, ox = q % TO;
  const int gy = oy0 + oy, gx = ox0 + ox;
  if (gy >= a.Ho || gx >= a.Wo) return;
  uint16_t* yb = a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * a.cout;
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int co = ot * 16 + (lane >> 4) * 4;
    if (co >= a.cout) continue;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = acc[ot][r] + a.bp[co + r];
    if (a.residual) {  // stride 1, cin == cout: centre pixel of the halo tile
      const uint16_t* rp = xs + ((oy + 1) * TI + (ox + 1)) * xrow + co;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += bf2f(rp[r]);
    }
    uint2 o;
    o.x = static_cast<uint32_t>(f2bf(v[0])) | (static_cast<uint32_t>(f2bf(v[1])) << 16);
    o.y = static_cast<uint32_t>(f2bf(v[2])) | (static_cast<uint32_t>(f2bf(v[3])) << 16);
    *reinterpret_cast<uint2*>(yb + co) = o;
  }
}

template <int S>
bool launch_s(const IrBlockArgs& a, int n_ot, size_t lds, dim3 grid, hipStream_t s) {
#define NNSX_IR_CASE(N)                                                                         \
  case N:                                                                                       \
    hipLaunchKernelGGL((ir_block_kernel<S, N>), grid, dim3(256), lds, s, a);                    \
    return true;
  switch (n_ot) {
    NNSX_IR_CASE(1)
    NNSX_IR_CASE(2)
    NNSX_IR_CASE(4)
    NNSX_IR_CASE(6)
    NNSX_IR_CASE(8)
    NNSX_IR_CASE(10)
    NNSX_IR_CASE(12)
    NNSX_IR_CASE(16)
    NNSX_IR_CASE(20)
    default:
      return false;
  }
#undef NNSX_IR_CASE
}

}  // namespace

size_t ir_block_lds_bytes(int stride, int cin32) {
  const int pin16 = tile_in_px16(stride);
  return sizeof(uint16_t) * (static_cast<size_t>(pin16) * (cin32 + 8) + static_cast<size_t>(pin16) * HROW + 64 * HROW);
}

bool ir_block_supported(int stride, int cin, int hid, int cout) {
  if (stride != 1 && stride != 2) return false;
  if (cin % 8 || cout % 8 || hid % HC) return false;
  const int n_ot = (cout + 15) / 16;
  if (n_ot > 20 || (n_ot != 1 && n_ot != 2 && n_ot % 2)) return false;
  return ir_block_lds_bytes(stride, (cin + 31) / 32 * 32) <= 64 * 1024;
}

bool ir_block(const IrBlockArgs& args, hipStream_t s) {
  IrBlockArgs a = args;
  a.cin32 = (a.cin + 31) / 32 * 32;
  a.Ho = (a.H - 1) / a.stride + 1;
  a.Wo = (a.W - 1) / a.stride + 1;
  a.tiles_y = (a.Ho + TO - 1) / TO;
  a.tiles_x = (a.Wo + TO - 1) / TO;
  if (!ir_block_supported(a.stride, a.cin, a.hid, a.cout)) return false;
  const int n_ot = (a.cout + 15) / 16;
  const size_t lds = ir_block_lds_bytes(a.stride, a.cin32);
  dim3 grid(static_cast<unsigned>(a.tiles_x * a.tiles_y * a.B));
  return a.stride == 1 ? launch_s<1>(a, n_ot, lds, grid, s) : launch_s<2>(a, n_ot, lds, grid, s);
}

}  // namespace kernels
}  // namespace nnsx
