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

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "kernels/mbv2.h"

namespace nnsx {
namespace kernels {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_mfma __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
// two floats -> packed bf16 pair (lo = a), round-to-nearest-even: one v_cvt_pk_bf16_f32 on gfx950
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 b2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, b2v));
}
__device__ __forceinline__ float relu6(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

constexpr size_t kLdsLimit = 160 * 1024;  // gfx950 LDS per CU (one workgroup may own it all)
constexpr int TO = 8;       // output tile edge
constexpr int HC = 32;      // hidden channels per chunk (= one MFMA K step)
// LDS row pitches (elements).  Hidden tile: the depthwise lanes of one 32-lane
// half read 8 pixels (stride S) x 4 channel quads with ds_read_b64, so a pixel's
// pitch in dwords must tile the 64 banks: 24 dwords for S=1, 20 for S=2.
// The hidden tile is fp32 (F = true: no bf16 pack/unpack on the VALU between
// expand and dw; pitch 36 floats: expand stores conflict-free, dw reads 2-way)
// when that costs no workgroup per CU, else bf16 (pitch: see above).
__host__ __device__ constexpr int hrow(int s, bool f) { return f ? HC + 4 : (s == 1 ? HC + 16 : HC + 8); }
__host__ __device__ constexpr int hbytes(bool f) { return f ? 4 : 2; }
constexpr int DROW = HC + 8;  // dw output tile (project B operand)

__host__ __device__ constexpr int tile_in(int s) { return (TO - 1) * s + 3; }
__host__ __device__ constexpr int tile_in_px16(int s) { return (tile_in(s) * tile_in(s) + 15) / 16 * 16; }

template <int S, bool F32H, int NOT, int KS_MAX>
__global__ void __launch_bounds__(256) ir_block_kernel(IrBlockArgs a) {
  constexpr int TI = tile_in(S);
  constexpr int PIN = TI * TI;
  constexpr int PIN16 = tile_in_px16(S);
  constexpr int NB = PIN16 / 16;                       // 16-pixel B tiles of the halo tile
  constexpr int NV = (PIN16 * 4 * KS_MAX + 255) / 256;  // 16-B input vectors per thread per tile
  constexpr int HROW = hrow(S, F32H);
  using HT = typename std::conditional<F32H, float, uint16_t>::type;  // hidden tile element
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // a.cin32 == 32 * KS_MAX (the launcher picks the instantiation): every
  // input-tile index below divides by compile-time constants
  constexpr int CIN32 = 32 * KS_MAX;
  constexpr int xrow = CIN32 + 8;  // LDS pitch of the input tile
  uint16_t* xs = smem;                                                // [PIN16][xrow]
  HT* hidbuf = reinterpret_cast<HT*>(xs + PIN16 * xrow);             // 2 x [PIN16][HROW] (double buffered)
  // (bf16 without expand: no hidden tile at all, the depthwise stage reads xs)
  uint16_t* dwo = reinterpret_cast<uint16_t*>(hidbuf + (a.has_expand || F32H ? 2 * PIN16 * HROW : 0));  // [64][DROW]
  HT* wds = reinterpret_cast<HT*>(dwo + 64 * DROW);                  // [9][hid] depthwise weights (staged once)
  float* bds = reinterpret_cast<float*>(wds + 9 * a.hid);            // [hid] depthwise bias

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 15;
  const int kq = (lane >> 4) * 8;
  constexpr int vec_per_px = CIN32 / 8;
  const int tiles_img = a.tiles_x * a.tiles_y;
  const int total_tiles = tiles_img * a.B;
  // persistent walk: this workgroup owns tiles [t_begin, t_end) (consecutive along x)
  const int t_begin = blockIdx.x * a.tiles_per_wg;
  const int t_end = min(total_tiles, t_begin + a.tiles_per_wg);

  // expand operands of one chunk (registers): A fragments of both 16-row tiles + biases
  bf16x8_t ea[2][KS_MAX];
  float eb[2][4];
  auto load_expand = [&](int c0) {
#pragma unroll
    for (int at = 0; at < 2; ++at) {
      const uint16_t* wrow = a.we + static_cast<int64_t>(c0 + at * 16 + li) * CIN32 + kq;
#pragma unroll
      for (int ks = 0; ks < KS_MAX; ++ks) ea[at][ks] = *reinterpret_cast<const bf16x8_t*>(wrow + ks * 32);
#pragma unroll
      for (int r = 0; r < 4; ++r) eb[at][r] = a.be[c0 + at * 16 + (lane >> 4) * 4 + r];
    }
  };

  // next tile's input vectors are fetched into registers while the current tile computes
  bf16x8_t pf[NV];
  // tile coordinates advance incrementally (one SALU division per workgroup,
  // not four per tile: at 112x112 a workgroup walks ~65 tiles)
  struct TileXY {
    int b, ty, tx;
  };
  auto next_xy = [&](TileXY c) {
    if (++c.tx == a.tiles_x) {
      c.tx = 0;
      if (++c.ty == a.tiles_y) {
        c.ty = 0;
        ++c.b;
      }
    }
    return c;
  };
  auto fetch_tile = [&](TileXY c) {
    const int b = c.b;
    const int iy0 = c.ty * TO * S - 1, ix0 = c.tx * TO * S - 1;
    const uint16_t* xb = a.x + static_cast<int64_t>(b) * a.H * a.W * a.cin;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * 256;
      const int p = v / vec_per_px;
      const int k = (v % vec_per_px) * 8;
      bf16x8_t val = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      if (p < PIN && k < a.cin) {
        const int iy = iy0 + p / TI, ix = ix0 + p % TI;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          val = *reinterpret_cast<const bf16x8_t*>(xb + (static_cast<int64_t>(iy) * a.W + ix) * a.cin + k);
      }
      pf[i] = val;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * 256;
      const int p = v / vec_per_px;
      if (p < PIN16) *reinterpret_cast<bf16x8_t*>(xs + p * xrow + (v % vec_per_px) * 8) = pf[i];
    }
  };

  if (t_begin >= t_end) return;
  TileXY cur;
  cur.b = t_begin / tiles_img;
  cur.ty = (t_begin - cur.b * tiles_img) / a.tiles_x;
  cur.tx = t_begin - cur.b * tiles_img - cur.ty * a.tiles_x;
  if (a.has_expand) load_expand(0);
  fetch_tile(cur);
  for (int v = tid; v < 9 * a.hid / 8; v += 256) {
    const bf16x8_t w8 = *reinterpret_cast<const bf16x8_t*>(a.wd + v * 8);
    if constexpr (F32H) {
#pragma unroll
      for (int r = 0; r < 8; ++r) wds[v * 8 + r] = bf2f(static_cast<uint16_t>(w8[r]));
    } else {
      *reinterpret_cast<bf16x8_t*>(wds + v * 8) = w8;
    }
  }
  for (int v = tid; v < a.hid; v += 256) bds[v] = a.bd[v];

  // depthwise lane mapping: wave w owns output rows 2w, 2w+1 (= the project
  // B-tile pixels 16w..16w+15); lane = column dx x channel quad dq, both rows
  const int dx = lane & 7;
  const int dq = (lane >> 3) * 4;

  for (int tile = t_begin; tile < t_end; ++tile, cur = next_xy(cur)) {
    store_tile();
    __syncthreads();
    if (tile + 1 < t_end) fetch_tile(next_xy(cur));  // in flight during this tile's compute

    const int b = cur.b;
    const int oy0 = cur.ty * TO, ox0 = cur.tx * TO;
    const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

    f32x4_t acc[NOT];
#pragma unroll
    for (int i = 0; i < NOT; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    int buf = 0;
    for (int c0 = 0; c0 < a.hid; c0 += HC, buf ^= 1) {
      HT* hid = hidbuf + buf * PIN16 * HROW;
      // issue this chunk's project weight loads early (consumed after the barrier)
      bf16x8_t pa[NOT];
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
        pa[ot] = *reinterpret_cast<const bf16x8_t*>(a.wp + static_cast<int64_t>(ot * 16 + li) * a.hid + c0 + kq);

      // ---- expand: wave w computes B tiles w, w+4, ... for both 16-channel A tiles
      if (a.has_expand) {
#pragma unroll
        for (int it = 0; it < (NB + 3) / 4; ++it) {
          const int bt = wave + 4 * it;
          if (bt >= NB) break;
          f32x4_t e0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, e1 = e0;
          const uint16_t* xrowp = xs + (bt * 16 + li) * xrow + kq;
#pragma unroll
          for (int ks = 0; ks < KS_MAX; ++ks) {
            const bf16x8_mfma bfr =
                __builtin_bit_cast(bf16x8_mfma, *reinterpret_cast<const bf16x8_t*>(xrowp + ks * 32));
            e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, ea[0][ks]), bfr, e0, 0, 0, 0);
            e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, ea[1][ks]), bfr, e1, 0, 0, 0);
          }
          const int p = bt * 16 + li;
          const int iy = iy0 + p / TI, ix = ix0 + p % TI;
          const bool inside = p < PIN && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
          const int hc = (lane >> 4) * 4;
          if constexpr (F32H) {
            f32x4_t v0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, v1 = v0;
            if (inside) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                v0[r] = relu6(e0[r] + eb[0][r]);
                v1[r] = relu6(e1[r] + eb[1][r]);
              }
            }
            *reinterpret_cast<f32x4_t*>(hid + p * HROW + hc) = v0;
            *reinterpret_cast<f32x4_t*>(hid + p * HROW + 16 + hc) = v1;
          } else {
            uint2 p0 = make_uint2(0u, 0u), p1 = make_uint2(0u, 0u);
            if (inside) {
              p0.x = pk_bf16(relu6(e0[0] + eb[0][0]), relu6(e0[1] + eb[0][1]));
              p0.y = pk_bf16(relu6(e0[2] + eb[0][2]), relu6(e0[3] + eb[0][3]));
              p1.x = pk_bf16(relu6(e1[0] + eb[1][0]), relu6(e1[1] + eb[1][1]));
              p1.y = pk_bf16(relu6(e1[2] + eb[1][2]), relu6(e1[3] + eb[1][3]));
            }
            *reinterpret_cast<uint2*>(hid + p * HROW + hc) = p0;
            *reinterpret_cast<uint2*>(hid + p * HROW + 16 + hc) = p1;
          }
        }
        // prefetch the next chunk's (or the next tile's first chunk's) expand operands
        load_expand(c0 + HC < a.hid ? c0 + HC : 0);
      } else if constexpr (F32H) {
        // no expand (t = 1): the hidden tile is the input tile, widened to fp32
        for (int v = tid; v < PIN16 * (HC / 8); v += 256) {
          const int p = v / (HC / 8), k = (v % (HC / 8)) * 8;
          const bf16x8_t x8 = *reinterpret_cast<const bf16x8_t*>(xs + p * xrow + c0 + k);
          f32x4_t lo, hi;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] = bf2f(static_cast<uint16_t>(x8[r]));
            hi[r] = bf2f(static_cast<uint16_t>(x8[r + 4]));
          }
          *reinterpret_cast<f32x4_t*>(hid + p * HROW + k) = lo;
          *reinterpret_cast<f32x4_t*>(hid + p * HROW + k + 4) = hi;
        }
      }  // bf16, no expand: the depthwise stage reads the input tile in place
      // one block barrier per chunk: hid is double buffered, dw/project are wave-local
      __syncthreads();

      // ---- depthwise 3x3 + bias + ReLU6: lane = 2 vertically adjacent output
      // pixels x 4 channels.  The S+3 input rows are read once for both pixels
      // (ds_read_b64) and the taps' bf16 weights once per chunk; packed fp32
      // math, 2 channels per v_pk_fma_f32 (bf16 -> f32: shift low / mask high)
      {
        const int ch = c0 + dq;
        const f32x4_t bb = *reinterpret_cast<const f32x4_t*>(bds + ch);
        f32x2_t d0[2] = {f32x2_t{bb[0], bb[1]}, f32x2_t{bb[2], bb[3]}};
        f32x2_t d1[2] = {d0[0], d0[1]};
        f32x2_t w[9][2];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          if constexpr (F32H) {
            const f32x4_t wv = *reinterpret_cast<const f32x4_t*>(wds + t * a.hid + ch);
            w[t][0] = f32x2_t{wv[0], wv[1]};
            w[t][1] = f32x2_t{wv[2], wv[3]};
          } else {
            const uint2 wv = *reinterpret_cast<const uint2*>(wds + t * a.hid + ch);
            w[t][0] = f32x2_t{__uint_as_float(wv.x << 16), __uint_as_float(wv.x & 0xffff0000u)};
            w[t][1] = f32x2_t{__uint_as_float(wv.y << 16), __uint_as_float(wv.y & 0xffff0000u)};
          }
        }
        const int r0 = wave * 2 * S;
#pragma unroll
        for (int rr = 0; rr < S + 3; ++rr)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int p = (r0 + rr) * TI + dx * S + kx;
            f32x2_t h0, h1;
            if constexpr (F32H) {
              const f32x4_t hv = *reinterpret_cast<const f32x4_t*>(hid + p * HROW + dq);
              h0 = f32x2_t{hv[0], hv[1]};
              h1 = f32x2_t{hv[2], hv[3]};
            } else {
              const uint2 hv = a.has_expand ? *reinterpret_cast<const uint2*>(hid + p * HROW + dq)
                                            : *reinterpret_cast<const uint2*>(xs + p * xrow + c0 + dq);
              h0 = f32x2_t{__uint_as_float(hv.x << 16), __uint_as_float(hv.x & 0xffff0000u)};
              h1 = f32x2_t{__uint_as_float(hv.y << 16), __uint_as_float(hv.y & 0xffff0000u)};
            }
            if (rr <= 2) {
              d0[0] = __builtin_elementwise_fma(h0, w[rr * 3 + kx][0], d0[0]);
              d0[1] = __builtin_elementwise_fma(h1, w[rr * 3 + kx][1], d0[1]);
            }
            if (rr >= S && rr - S <= 2) {
              d1[0] = __builtin_elementwise_fma(h0, w[(rr - S) * 3 + kx][0], d1[0]);
              d1[1] = __builtin_elementwise_fma(h1, w[(rr - S) * 3 + kx][1], d1[1]);
            }
          }
        auto pk = [](f32x2_t v) {
          return pk_bf16(relu6(v[0]), relu6(v[1]));
        };
        *reinterpret_cast<uint2*>(dwo + (wave * 16 + dx) * DROW + dq) = make_uint2(pk(d0[0]), pk(d0[1]));
        *reinterpret_cast<uint2*>(dwo + (wave * 16 + 8 + dx) * DROW + dq) = make_uint2(pk(d1[0]), pk(d1[1]));
      }
      // dwo rows of this wave were written by this wave only: a wave-level fence suffices
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

      // ---- project: D[out][px] += Wp[out][hid] . dw[px][hid]^T
      {
        const bf16x8_mfma bfr =
            __builtin_bit_cast(bf16x8_mfma, *reinterpret_cast<const bf16x8_t*>(dwo + (wave * 16 + li) * DROW + kq));
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
          acc[ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, pa[ot]), bfr, acc[ot], 0,
                                                            0, 0);
      }
    }

    // ---- epilogue: bias (+ residual from the LDS input tile) -> bf16
    {
      const int qo = wave * 16 + li;
      const int oy = qo / TO, ox = qo % TO;
      const int gy = oy0 + oy, gx = ox0 + ox;
      if (gy < a.Ho && gx < a.Wo) {
        uint16_t* yb = a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * a.cout;
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) {
          const int co = ot * 16 + (lane >> 4) * 4;
          if (co >= a.cout) continue;
          float v[4];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) v[rr] = acc[ot][rr] + a.bp[co + rr];
          if (a.residual) {  // stride 1, cin == cout: centre pixel of the halo tile
            const uint16_t* rp = xs + ((oy + 1) * TI + (ox + 1)) * xrow + co;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) v[rr] += bf2f(rp[rr]);
          }
          uint2 o;
          o.x = pk_bf16(v[0], v[1]);
          o.y = pk_bf16(v[2], v[3]);
          *reinterpret_cast<uint2*>(yb + co) = o;
        }
      }
    }
    __syncthreads();  // xs / hid are rewritten by the next tile
  }
}

template <int S, bool F, int NOT, int KS>
bool launch_one(const IrBlockArgs& a, size_t lds, dim3 grid, hipStream_t s) {
  // dynamic LDS above 64 KiB must be opted into once per instantiation (a workgroup may use all 160 KiB)
  static const bool attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&ir_block_kernel<S, F, NOT, KS>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  static_cast<int>(kLdsLimit)) == hipSuccess;
  if (!attr_ok && lds > 64 * 1024) return false;
  hipLaunchKernelGGL((ir_block_kernel<S, F, NOT, KS>), grid, dim3(256), lds, s, a);
  return true;
}

template <int S, bool F, int NOT>
bool launch_ks(const IrBlockArgs& a, size_t lds, dim3 grid, hipStream_t s) {
  switch (a.cin32 / 32) {
    case 1: return launch_one<S, F, NOT, 1>(a, lds, grid, s);
    case 2: return launch_one<S, F, NOT, 2>(a, lds, grid, s);
    case 3: return launch_one<S, F, NOT, 3>(a, lds, grid, s);
    case 5: return launch_one<S, F, NOT, 5>(a, lds, grid, s);
    default: return false;
  }
}

template <int S, bool F>
bool launch_s(const IrBlockArgs& a, int n_ot, size_t lds, dim3 grid, hipStream_t s) {
  switch (n_ot) {
    case 1: return launch_ks<S, F, 1>(a, lds, grid, s);
    case 2: return launch_ks<S, F, 2>(a, lds, grid, s);
    case 4: return launch_ks<S, F, 4>(a, lds, grid, s);
    case 6: return launch_ks<S, F, 6>(a, lds, grid, s);
    case 10: return launch_ks<S, F, 10>(a, lds, grid, s);
    case 20: return launch_ks<S, F, 20>(a, lds, grid, s);
    default: return false;
  }
}

}  // namespace

namespace {
size_t lds_total(int stride, bool f, int cin32, int hid, bool has_expand = true) {
  const int pin16 = tile_in_px16(stride);
  return sizeof(uint16_t) * (static_cast<size_t>(pin16) * (cin32 + 8) + 64 * DROW) +
         (has_expand || f ? static_cast<size_t>(hbytes(f)) * 2 * static_cast<size_t>(pin16) * hrow(stride, f) : 0) +
         (9 * static_cast<size_t>(hbytes(f)) + sizeof(float)) * static_cast<size_t>(hid);  // dw weights + bias
}
// fp32 hidden tile when it costs no workgroup per CU, or on the large early
// feature maps (>= 56x56, many tiles per workgroup) as long as two workgroups
// still fit.  Measured at batch 256 (scripts/bench_ir.py): fp32 wins at
// 112/56 px even at 3-vs-4 workgroups per CU, loses at 28 px (3 vs 4) and
// whenever it drops to 1 workgroup, ties at 14 px.
bool use_f32_hidden(int stride, int cin32, int hid, int hw, bool has_expand) {
  if (!has_expand) return false;  // bf16: the depthwise stage reads the input tile in place
  const size_t f = lds_total(stride, true, cin32, hid), b = lds_total(stride, false, cin32, hid);
  if (f > kLdsLimit) return false;
  return kLdsLimit / f >= kLdsLimit / b || (hw >= 56 * 56 && kLdsLimit / f >= 2);
}
}  // namespace

size_t ir_block_lds_total(int stride, int cin32, int hid) {
  return lds_total(stride, false, cin32, hid);  // the bf16 tile: what ir_block_supported() checks
}

bool ir_block_supported(int stride, int cin, int hid, int cout) {
  if (stride != 1 && stride != 2) return false;
  if (cin % 8 || cout % 8 || hid % HC || cin > 160) return false;
  const int n_ot = (cout + 15) / 16;
  if (n_ot != 1 && n_ot != 2 && n_ot != 4 && n_ot != 6 && n_ot != 10 && n_ot != 20) return false;
  const int ks = (cin + 31) / 32;
  if (ks != 1 && ks != 2 && ks != 3 && ks != 5) return false;
  return ir_block_lds_total(stride, (cin + 31) / 32 * 32, hid) <= kLdsLimit;
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
  const bool f = use_f32_hidden(a.stride, a.cin32, a.hid, a.H * a.W, a.has_expand != 0);
  const size_t lds = lds_total(a.stride, f, a.cin32, a.hid, a.has_expand != 0);
  // persistent grid: enough workgroups for every CU to hold several (LDS-limited), each
  // walking a run of consecutive tiles so the next tile's input loads overlap compute
  // one resident round: every workgroup slot of the chip walks an equal run of tiles
  const int total_tiles = a.tiles_x * a.tiles_y * a.B;
  const int per_cu = std::max<int>(1, std::min<int>(8, static_cast<int>(kLdsLimit / lds)));
  const int max_wgs = 256 * per_cu;
  a.tiles_per_wg = std::max(1, (total_tiles + max_wgs - 1) / max_wgs);
  dim3 grid(static_cast<unsigned>((total_tiles + a.tiles_per_wg - 1) / a.tiles_per_wg));
  if (a.stride == 1) return f ? launch_s<1, true>(a, n_ot, lds, grid, s) : launch_s<1, false>(a, n_ot, lds, grid, s);
  return f ? launch_s<2, true>(a, n_ot, lds, grid, s) : launch_s<2, false>(a, n_ot, lds, grid, s);
}

}  // namespace kernels
}  // namespace nnsx
