// fp32 GEMM tile kernels (pw_gemm_f32), shared by two translation units:
// kernels/mbv2_f32.hip instantiates the native-fp32 forms and kernels/gemm_x3.hip
// the split-bf16 (x3) ones.  gemm_x3.hip is compiled with the MFMA results in
// VGPRs (-mllvm -amdgpu-mfma-vgpr-form, nnstreamer_amd/_build.py): the x3
// tile adds each 32-k partial to its fp32 accumulator on the VALU, and in AGPRs
// every partial first went through v_accvgpr_read (32 per k-stage of a 128 x 64
// tile) -- the x3 GEMMs ran 2-7 % faster without them
// (profiles/r5_vgpr_form_ab.txt); the native-fp32 fused blocks, whose large
// accumulators live in AGPRs, lost up to 8 % under the same flag, so it is
// set for this unit only.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kernels/mbv2.h"
#include "kernels/x3.h"

namespace nnsx {
namespace kernels {

// Several independent GEMMs in one launch (pw_gemm_group_f32_kernel)
struct GemmGroupArgs {
  int n = 0;
  int start[kGroupMax + 1] = {};
  GemmProb p[kGroupMax];
};

// the x3 launches (kernels/gemm_x3.hip): tile BM x BN, grid / k-stages per
// z-slice as pw_gemm_f32_launch computed them; w3: the weights are pre-split
void pw_gemm_x3_launch(int BM, int BN, bool w3, dim3 grid, hipStream_t s, const float* x, const float* wt, X3W w3p,
                       const float* bias, const float* res, float* y, int M, int N, int K, int Kpad, int Npad,
                       int act, int kchunk, YLayout yl);
void pw_gemm_group_x3_launch(bool w3, unsigned blocks, hipStream_t s, const GemmGroupArgs& g);

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// one 16-k step: lane (li, g) holds k = 16s + 4g + j in component j of a and b
__device__ __forceinline__ f32x4_t mfma_k16(f32x4_t a, f32x4_t b, f32x4_t c) {
  c = mfma4(a[0], b[0], c);
  c = mfma4(a[1], b[1], c);
  c = mfma4(a[2], b[2], c);
  return mfma4(a[3], b[3], c);
}
// an 8-k tail step: lane (li, g) holds k = 2g + j in component j
__device__ __forceinline__ f32x4_t mfma_k8(f32x2_t a, f32x2_t b, f32x4_t c) {
  c = mfma4(a[0], b[0], c);
  return mfma4(a[1], b[1], c);
}

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return fminf(fmaxf(v, 0.f), 6.f);  // ReLU6
  if (act == 2) return fmaxf(v, 0.f);                // ReLU
  return v;
}
__device__ __forceinline__ float relu6(float v) { return fminf(fmaxf(v, 0.f), 6.f); }
__device__ __forceinline__ f32x4_t relu6x4(f32x4_t v) {
  return f32x4_t{relu6(v[0]), relu6(v[1]), relu6(v[2]), relu6(v[3])};
}

// XCD-aware workgroup order: the dispatcher places consecutive workgroup ids
// round-robin over the 8 XCDs (each with its own L2).  Renumber so that each
// XCD walks a contiguous range of tiles: neighbouring tiles share halo rows
// and the same image, and stay in one L2.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  if (n % 8) return bid;
  return (bid % 8) * (n / 8) + bid / 8;
}

// ------------------------------------------------------------- pw_gemm_f32 ----
constexpr int GKT = 32;       // k per LDS stage
constexpr int GKQ = GKT / 4;  // k-quads per stage

// one BM x BN output tile over k-stages [kbeg, kbeg + nk * GKT); zs / slab: this
// block's split-K slice and whether the grid is split (then y is the slab workspace)
// X3: the products on split-bf16 MFMAs (see split_x3), the LDS images and the
// epilogue unchanged
// W3 (X3 only): the weights come pre-split (wt3 [stages][rows3][3][32] bf16,
// X3W) and are staged as they are -- only the activation operand is split per tile
template <int BM, int BN, bool X3 = false, bool W3 = false>
__device__ __forceinline__ void pw_gemm_f32_tile(const float* __restrict__ x,     // [M][K]
                                                 const float* __restrict__ wt,    // [Npad][Kpad]
                                                 const uint16_t* __restrict__ wt3, int rows3,
                                                 const float* __restrict__ bias,  // [N]
                                                 const float* __restrict__ res,   // [M][N] or null
                                                 float* __restrict__ y,           // [M][N]
                                                 int M, int N, int K, int Kpad, int Npad, int act, int kbeg, int nk,
                                                 int zs, bool slab, const YLayout& yl, int m0, int n0) {
  constexpr int RM = BM / 32, RN = BN / 32;  // 16-row fragments per wave (2 x 2 waves)
  constexpr int VX = BM * GKQ / 256, VW = BN * GKQ / 256;
  // k4-major images, row index XOR-swizzled with the k-quad (kq < 8): the
  // staging writes (8 lanes = 8 k-quads of one row) then spread over the
  // banks, and fragment reads stay conflict-free (16 rows of one 16-aligned
  // block, permuted)
  // X3: both operands are split once, while they are staged, into three bf16
  // planes [part][k8][row] of 8 consecutive k (16 B) -- the fragment of a
  // 32-k step is then 3 ds_read_b128 per operand and no VALU; rows
  // XOR-swizzled by k8 (staging writes spread, fragment reads stay 256
  // contiguous bytes per 16 lanes)
  __shared__ __attribute__((aligned(16))) float xs[X3 ? 1 : 2][GKQ][X3 ? 4 : BM][4];
  __shared__ __attribute__((aligned(16))) float ws[X3 ? 1 : 2][GKQ][X3 ? 4 : BN][4];
  // X3 part planes [buf][part][k8][row] in 16-B cells, each part padded by 4
  // cells (64 B), and rows swizzled by x3_swz: conflict-free for the staging
  // writes (ds_write_b64 of the activation split: 16 lanes = 2 rows x 8 k-quads;
  // ds_write_b128 of pre-split weights: 8 lanes over 2-3 parts of a row) and
  // for the fragment reads (ds_read_b128 lane groups mixing two k8 planes).
  // (Swizzling by k8 alone left 2-way conflicts: SQ_LDS_BANK_CONFLICT 33 % of
  // the LDS cycles, profiles/r5_pmc_gemm_x3.txt.)
  constexpr int XP3 = 4 * BM + 4, WP3 = 4 * BN + 4;
  __shared__ __attribute__((aligned(16))) bf16x8_t xs3[X3 ? 2 * 3 * XP3 : 1];
  __shared__ __attribute__((aligned(16))) bf16x8_t ws3[X3 ? 2 * 3 * WP3 : 1];
  auto x3_swz = [](int row, int k8) { return row ^ k8 ^ ((row & 1) * 12); };
  auto xi = [&](int buf, int part, int k8, int row) { return (buf * 3 + part) * XP3 + k8 * BM + x3_swz(row, k8); };
  auto wi = [&](int buf, int part, int k8, int row) { return (buf * 3 + part) * WP3 + k8 * BN + x3_swz(row, k8); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 15, g = lane >> 4;
  const f32x4_t zero = f32x4_t{0.f, 0.f, 0.f, 0.f};

  static_assert(!W3 || X3, "pw_gemm_f32: pre-split weights are an x3 form");
  constexpr int VW3 = W3 ? BN * 12 / 256 : 1;  // bf16x8 (8 k of one part of one row) per thread
  static_assert(!W3 || (BN * 12) % 256 == 0, "pw_gemm_f32: W3 staging");
  f32x4_t px[VX], pw[W3 ? 1 : VW];
  bf16x8_t pw3[VW3];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int v = tid + i * 256, kq = v & 7, row = v >> 3;
      const int m = m0 + row, k = k0 + kq * 4;
      px[i] = (m < M && k < K) ? *reinterpret_cast<const f32x4_t*>(x + static_cast<int64_t>(m) * K + k) : zero;
    }
    if constexpr (W3) {
      // pre-split weights: the tile's rows of stage k0 / 32 are one contiguous
      // block of 192-B rows (16 B = 8 k of one part per lane, consecutive lanes
      // consecutive chunks).  rows3 covers every row of the grid's tiles (the
      // host checks), so the loads carry no bounds select: a select on a
      // prefetched value made the compiler wait for it before the MFMAs.
      const uint16_t* stg = wt3 + (static_cast<int64_t>(k0 / GKT) * rows3 + n0) * 96;
#pragma unroll
      for (int i = 0; i < VW3; ++i) pw3[i] = *reinterpret_cast<const bf16x8_t*>(stg + (tid + i * 256) * 8);
    } else {
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        const int v = tid + i * 256, kq = v & 7, row = v >> 3;
        const int n = n0 + row, k = k0 + kq * 4;
        pw[i] = (n < Npad && k < Kpad) ? *reinterpret_cast<const f32x4_t*>(wt + static_cast<int64_t>(n) * Kpad + k)
                                       : zero;
      }
    }
  };
  // (X3) a staged quad -> its three bf16 parts, 8 B into each part plane
  auto st3 = [&](bf16x8_t* base, size_t part_stride, f32x4_t q) {
    bf16x2_t h0, m0, l0, h1, m1, l1;
    split2(f32x2_t{q[0], q[1]}, h0, m0, l0);
    split2(f32x2_t{q[2], q[3]}, h1, m1, l1);
    typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
    char* p = reinterpret_cast<char*>(base);
    *reinterpret_cast<bf16x4_t*>(p) = __builtin_shufflevector(h0, h1, 0, 1, 2, 3);
    *reinterpret_cast<bf16x4_t*>(p + part_stride) = __builtin_shufflevector(m0, m1, 0, 1, 2, 3);
    *reinterpret_cast<bf16x4_t*>(p + 2 * part_stride) = __builtin_shufflevector(l0, l1, 0, 1, 2, 3);
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int v = tid + i * 256, kq = v & 7, row = v >> 3;
      if constexpr (X3) {
        const int k8 = kq >> 1;
        st3(reinterpret_cast<bf16x8_t*>(reinterpret_cast<char*>(&xs3[xi(buf, 0, k8, row)]) + (kq & 1) * 8),
            XP3 * sizeof(bf16x8_t), px[i]);
      } else {
        *reinterpret_cast<f32x4_t*>(&xs[buf][kq][row ^ kq][0]) = px[i];
      }
    }
    if constexpr (W3) {
#pragma unroll
      for (int i = 0; i < VW3; ++i) {
        const int v = tid + i * 256, row = v / 12, c = v - row * 12, part = c >> 2, k8 = c & 3;
        ws3[wi(buf, part, k8, row)] = pw3[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        const int v = tid + i * 256, kq = v & 7, row = v >> 3;
        if constexpr (X3) {
          const int k8 = kq >> 1;
          st3(reinterpret_cast<bf16x8_t*>(reinterpret_cast<char*>(&ws3[wi(buf, 0, k8, row)]) + (kq & 1) * 8),
              WP3 * sizeof(bf16x8_t), pw[i]);
        } else {
          *reinterpret_cast<f32x4_t*>(&ws[buf][kq][row ^ kq][0]) = pw[i];
        }
      }
    }
  };

  f32x4_t acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = zero;

  if (nk > 0) {
    gload(kbeg);
    lstore(0);
    __syncthreads();
  }
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) gload(kbeg + (ks + 1) * GKT);  // in flight during this stage's MFMAs
    if constexpr (X3) {
      static_assert(GKT == 32, "x3: one 32-k step per stage");
      // lane (li, g): k 8g .. 8g + 7 of its row = plane k8 = g
      X3Frag a[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int r = wn * (BN / 2) + j * 16 + li;
        a[j].h = ws3[wi(buf, 0, g, r)];
        a[j].m = ws3[wi(buf, 1, g, r)];
        a[j].l = ws3[wi(buf, 2, g, r)];
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int r = wm * (BM / 2) + i * 16 + li;
        X3Frag b;
        b.h = xs3[xi(buf, 0, g, r)];
        b.m = xs3[xi(buf, 1, g, r)];
        b.l = xs3[xi(buf, 2, g, r)];
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] += mfma_x3(a[j], b);
      }
    }
#pragma unroll
    for (int s = 0; s < (X3 ? 0 : GKT / 16); ++s) {
      const int kq = 4 * s + g;
      f32x4_t a[RN], b[RM];
#pragma unroll
      for (int j = 0; j < RN; ++j)
        a[j] = *reinterpret_cast<const f32x4_t*>(&ws[buf][kq][(wn * (BN / 2) + j * 16 + li) ^ kq][0]);
#pragma unroll
      for (int i = 0; i < RM; ++i)
        b[i] = *reinterpret_cast<const f32x4_t*>(&xs[buf][kq][(wm * (BM / 2) + i * 16 + li) ^ kq][0]);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = mfma_k16(a[j], b[i], acc[i][j]);
    }
    if (ks + 1 < nk) lstore(buf ^ 1);  // buf ^ 1 was last read before the previous barrier
    __syncthreads();
  }

  // epilogue: lane owns channels n..n+3 of pixel m.  Bias (and residual)
  // values are all loaded up front, branch-free: loaded at each store behind
  // the bounds checks they were fetched and waited for one at a time.
  if constexpr (BN == 64) {
    if (yl.pool && !slab) {
      // head conv + act + global average pool: the activated tile goes through
      // the (now free) staging LDS, quads XOR-swizzled by row; each thread sums
      // one (image, channel) column of the tile in row order and adds sum / pool
      float* t = X3 ? reinterpret_cast<float*>(&xs3[0]) : &xs[0][0][0][0];  // [BM][64]
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int ml = wm * (BM / 2) + i * 16 + li, m = m0 + ml;
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const int nl = wn * (BN / 2) + j * 16 + g * 4, n = n0 + nl;
          f32x4_t v = acc[i][j] + *reinterpret_cast<const f32x4_t*>(bias + (n < N ? n : 0));
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
          *reinterpret_cast<f32x4_t*>(t + ml * 64 + (((nl >> 2) ^ (ml & 15)) << 2)) = m < M ? v : zero;
        }
      }
      __syncthreads();
      const int hw = yl.pool, mend = min(m0 + BM, M), b0 = m0 / hw, nb = (mend - 1) / hw - b0 + 1;
      const float inv = 1.f / static_cast<float>(hw);
      for (int v = tid; v < nb * 64; v += 256) {
        const int bi = b0 + v / 64, nl = v % 64, n = n0 + nl;
        const int r0 = max(bi * hw, m0) - m0, r1 = min((bi + 1) * hw, mend) - m0;
        float sum = 0.f;
        for (int r = r0; r < r1; ++r) sum += t[r * 64 + (((nl >> 2) ^ (r & 15)) << 2) + (nl & 3)];
        if (n < N) atomicAdd(y + static_cast<int64_t>(bi) * N + n, sum * inv);
      }
      return;
    }
  }
  f32x4_t bv[RN], rv[RM][RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + g * 4;
    bv[j] = slab ? zero : *reinterpret_cast<const f32x4_t*>(bias + (n < N ? n : 0));
  }
  if (res && !slab) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = m0 + wm * (BM / 2) + i * 16 + li;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn * (BN / 2) + j * 16 + g * 4;
        const int64_t off = (m < M && n < N) ? static_cast<int64_t>(m) * N + n : 0;
        rv[i][j] = *reinterpret_cast<const f32x4_t*>(res + off);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int m = m0 + wm * (BM / 2) + i * 16 + li;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + g * 4;
      if (n >= N) continue;
      float* yp = y + static_cast<int64_t>(m) * N + n;
      if (slab) {  // split-K: this slice's slab of the workspace (gemm_splitk_reduce adds them)
        *reinterpret_cast<f32x4_t*>(y + static_cast<int64_t>(zs) * M * N + static_cast<int64_t>(m) * N + n) = acc[i][j];
        continue;
      }
      f32x4_t v = acc[i][j] + (yl.brpb ? *reinterpret_cast<const f32x4_t*>(bias + static_cast<int64_t>(m / yl.brpb) * N + n)
                                        : bv[j]);
      if (res) v += rv[i][j];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
      if (yl.rpb) {  // a slice of a concatenated output: row m of batch m / rpb, first ncols columns
        if (n >= yl.ncols) continue;
        float* yd = y + static_cast<int64_t>(m / yl.rpb) * yl.bstride + static_cast<int64_t>(m % yl.rpb) * yl.ncols + n;
        if (n + 4 <= yl.ncols && (yl.ncols & 3) == 0) {
          *reinterpret_cast<f32x4_t*>(yd) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < yl.ncols) yd[r] = v[r];
        }
        continue;
      }
      *reinterpret_cast<f32x4_t*>(yp) = v;
    }
  }
}

template <int BM, int BN, bool X3 = false, bool W3 = false>
__global__ void __launch_bounds__(256) pw_gemm_f32_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                          X3W w3, const float* __restrict__ bias,
                                                          const float* __restrict__ res,
                                                          float* __restrict__ y, int M, int N, int K, int Kpad, int Npad,
                                                          int act,
                                                          int kchunk,  // k-stages of this grid.z slice
                                                          YLayout yl) {
  const int nbx = gridDim.x, nby = gridDim.y;
  const int flat = xcd_remap(blockIdx.y * nbx + blockIdx.x, nbx * nby);
  const int kbeg = blockIdx.z * kchunk * GKT;
  const int kend = min(Kpad, kbeg + kchunk * GKT);
  pw_gemm_f32_tile<BM, BN, X3, W3>(x, wt, w3.p, w3.rows, bias, res, y, M, N, K, Kpad, Npad, act, kbeg,
                                   (kend - kbeg + GKT - 1) / GKT,
                               static_cast<int>(blockIdx.z), gridDim.z > 1, yl, (flat % nbx) * BM, (flat / nbx) * BN);
}

// Several independent GEMMs in one launch (the SSD prediction heads): block b
// takes a tile of the problem whose block range holds it.  No XCD remap: the
// dispatcher deals blocks round robin over the XCDs, so each XCD gets the same
// mix of deep (long) and shallow tiles instead of one problem's eighth.

template <int BM, int BN, bool X3 = false, bool W3 = false>
__global__ void __launch_bounds__(256) pw_gemm_group_f32_kernel(GemmGroupArgs g) {
  const int flat = blockIdx.x;
  int i = 0;
  while (i + 1 < g.n && flat >= g.start[i + 1]) ++i;
  const GemmProb& p = g.p[i];
  const int local = flat - g.start[i], gx = (p.M + BM - 1) / BM;
  pw_gemm_f32_tile<BM, BN, X3, W3>(p.x, p.wt, p.w3.p, p.w3.rows, p.bias, nullptr, p.y, p.M, p.N, p.K, p.Kpad,
                                   p.Npad, p.act, 0,
                           (p.Kpad + GKT - 1) / GKT, 0, false, p.yl, (local % gx) * BM, (local / gx) * BN);
}


}  // namespace
}  // namespace kernels
}  // namespace nnsx
