// irp_x3: the 14 x 14 fused inverted residual (MobileNetV2's 64 -> 384 -> 64/96
// and 96 -> 576 -> 96 blocks), one IMAGE per workgroup, on split-bf16 MFMAs
// (kernels/x3.h), in a VGPR-form unit of its own (kernels/irw_common.h).
//
// Why a second kernel family next to irw_x3 (wave-split by hidden channel):
// there every wave holds the partial project sums of ALL the tile's outputs
// (acc[pixels][cout]) and re-reads the input tile's split planes from LDS for
// every 16-channel subtile -- 256+ VGPRs and MFMA pipe busy 0.17 on the 14 x 14
// blocks (profiles/r5_pmc_irw_x3_14x14.txt), and a 7 x 7 tile recomputes the
// expand on a 9 x 9 halo (96 of 49 cells).  Here the workgroup owns the whole
// 14 x 14 image, so the expand runs on the 196 pixels only (the hidden image's
// border is the depthwise padding: zeros), and the PIXELS are split over the
// waves instead of the hidden channels:
//   * 7 waves; wave w owns image rows 2w and 2w + 1 (28 pixels) as two 16-pixel
//     MFMA tiles: tile t holds the pixels of column parity t, so lane li of tile
//     0 and lane li of tile 1 are horizontal neighbours (the depthwise reads a
//     3 x 4 window for both: 12 cells instead of 18);
//   * the wave's input pixels are split into their bf16 parts ONCE and stay in
//     registers as the expand's B fragments for every hidden step (no LDS
//     image of the input, no re-split);
//   * per 32-channel hidden step every wave: expand (A = the step's pre-split
//     weights from LDS) -> bias + ReLU6 -> its cells of the shared hidden
//     image in LDS; barrier; depthwise 3 x 3 + bias + ReLU6 of its pixels (lane:
//     2 pixels x 8 channels, the project's B fragment layout), split, project
//     into its own accumulators (32 pixels x cout: 32 / 48 VGPRs);
//   * weights staged through registers into LDS one phase ahead (expand weights
//     during the depthwise + project phase, project / depthwise weights during
//     the expand phase), two barriers per step, single LDS buffers;
//   * epilogue: + bias (+ residual) straight from the accumulators to NHWC.
// Reference: the inverted residual is what MobileNetV2's TorchScript runs in
// tensor_filter_pytorch.cc:517-557 at float32; the x3 products' error against
// fp64 is gated by tests/test_gpu_x3.py.
#include "kernels/irw_common.h"

#include <atomic>
#include <cstdlib>

namespace nnsx {
namespace kernels {

namespace {

constexpr int kIrpH = 14;           // map size handled (S = 1)
// hidden grid row pitch (cells): 14 + 2 border + 1 pad.  The depthwise reads
// (ds_read_b128, lane = pixel pair li of rows r0 / r0 + 1, quad 2 g + qq) put
// lanes li and li + 7 -- same columns, adjacent rows -- on the same bank slot
// at a 16-cell pitch (2-way in every lane group); at 17 the next row moves one
// 16-B slot over and all 16 lanes of a group land on distinct slots.
constexpr int kIrpRow = 17;
constexpr int kIrpCells = 16 * kIrpRow + 16;  // + one scratch row for the padding lanes (a multiple of 16 slots)

// Physical 16-B chunk of chunk `ch` of weight row `row` in a stage of NCH
// chunks per row (rows unpadded).  An MFMA A-fragment read has lane (li, g)
// read row 16 t + li, chunk 4 c + g; ds_read_b128 serves a wave in four 16-lane
// groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, + 32) on 64 banks = 16 slots,
// so a plain or odd-padded pitch leaves two lanes per slot (2-way).  The XOR
// below gives every group 16 distinct slots for NCH = 4, 8, 12 (checked for
// every row / k-step by scripts/lds_banks.py) and keeps the chunk inside its
// row (a bijection of 0..NCH-1).
template <int NCH>
__device__ __forceinline__ int wsw(int row, int ch) {
  static_assert(NCH == 4 || NCH == 8 || NCH == 12, "wsw: chunks per row");
  if constexpr (NCH == 8)
    return ch ^ (2 * ((row >> 1) & 3));
  else
    return ch ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3);  // {0, 2, 3, 1}[(row >> 2) & 3]
}

// TPW = 16-pixel MFMA tiles per wave: 2 -> 7 waves, a wave owns a row pair and
// its lanes hold horizontal pixel pairs (the depthwise reads one 3 x 4 window
// for both); 1 -> 14 waves, a wave owns one column parity of a row pair (half
// the input fragments and accumulators per wave: the 96-channel blocks fit
// four waves per SIMD without spilling)
template <int CIN, int COUT, int TPW, bool XL = false>
struct IrpGeom {
  static constexpr int NW = 14 / TPW, NT = 64 * NW;
  static constexpr int NK32 = CIN / 32;        // expand k-steps
  static constexpr int NO16 = COUT / 16;       // project output tiles
  static constexpr int WEP = CIN / 8;          // expand weight row pitch (16-B chunks, swizzled: wsw)
  static constexpr int WPP = 32 / 8;           // project weight row pitch (chunks, swizzled)
  static constexpr size_t hid_b = static_cast<size_t>(8) * kIrpCells * 16;      // [quad][cell] f32x4
  static constexpr size_t we_b = static_cast<size_t>(3) * 32 * WEP * 16;        // [part][hid row][chunk]
  static constexpr size_t wp_b = static_cast<size_t>(3) * COUT * WPP * 16;      // [part][cout row][chunk]
  static constexpr size_t wd_b = static_cast<size_t>(10) * 32 * 4;              // [tap | bias][ch] f32
  static constexpr size_t be_b = static_cast<size_t>(32) * 4;
  // XL: the input image in LDS, fp32, pixel rows padded to CIN + 4 floats (a
  // 16-lane fragment read then hits 16 distinct bank quads), read and split per
  // step instead of held split in registers (the 96-channel blocks' registers)
  static constexpr int XP = CIN + 4;
  static constexpr size_t x_b = XL ? static_cast<size_t>(kIrpH * kIrpH) * XP * 4 : 0;
  static constexpr size_t lds = hid_b + we_b + wp_b + wd_b + be_b + x_b;
  // 16-B chunks staged per step
  static constexpr int WE_CH = 3 * 32 * (CIN / 8) + 8;   // + expand bias (32 f32)
  static constexpr int WP_CH = 3 * COUT * 4 + 80;         // + depthwise taps and bias (10 x 32 f32)
  static constexpr int WE_IT = (WE_CH + NT - 1) / NT;
  static constexpr int WP_IT = (WP_CH + NT - 1) / NT;
  static constexpr int MINW = TPW == 2 ? 2 : 4;  // waves per SIMD the registers are sized for
};

template <int CIN, int COUT, int TPW, bool XL>
__global__ void __launch_bounds__((IrpGeom<CIN, COUT, TPW, XL>::NT), (IrpGeom<CIN, COUT, TPW, XL>::MINW))
    irp_x3_kernel(IrBlockF32Args a) {
  using G = IrpGeom<CIN, COUT, TPW, XL>;
  constexpr int NK32 = G::NK32, NO16 = G::NO16, WEP = G::WEP, WPP = G::WPP, NT = G::NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  f32x4_t* hb = reinterpret_cast<f32x4_t*>(smem);                                   // [8][kIrpCells]
  char* wel = reinterpret_cast<char*>(smem) + G::hid_b;                              // expand weights
  char* wpl = wel + G::we_b;                                                         // project weights
  float* wdl = reinterpret_cast<float*>(wpl + G::wp_b);                              // [10][32]
  float* bel = wdl + 320;                                                            // [32]
  float* xl = bel + 32;                                                              // XL: [196][XP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const int hid = a.hid, nsteps = hid / 32;
  const int r0 = 2 * (TPW == 2 ? wave : wave >> 1);
  const int par = TPW == 2 ? 0 : (wave & 1);  // column parity of tile 0
  // this lane's pixel slot: row y, columns x0 + par + t (t < TPW)
  const bool real = li < 14;
  const int y = r0 + (li >= 7 ? 1 : 0);
  const int x0 = 2 * (li >= 7 ? li - 7 : li);
  const int ys = real ? y : r0, x0s = real ? x0 : 0;  // (padding lanes read a valid window)

  // ---- zero the hidden image (its border is the depthwise padding) ----
  for (int v = tid; v < 8 * kIrpCells; v += NT) hb[v] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- weight staging (16-B chunks through registers) ----
  const int64_t wes = static_cast<int64_t>(hid) * CIN;     // we3 part stride (elements)
  const int64_t wps = static_cast<int64_t>(COUT) * hid;    // wp3 part stride (cout multiple of 32)
  u32x4_t we_st[G::WE_IT], wp_st[G::WP_IT];
  auto we_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.we3 + p * wes + static_cast<int64_t>(32 * s + h) * CIN + kc * 8);
      } else {
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.be + 32 * s + 4 * (v - (G::WE_CH - 8)));
      }
    }
  };
  auto we_store = [&]() {
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        *reinterpret_cast<u32x4_t*>(wel + ((p * 32 + h) * WEP + wsw<WEP>(h, kc)) * 16) = we_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(bel + 4 * (v - (G::WE_CH - 8))) = we_st[it];
      }
    }
  };
  auto wp_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>(a.wp3 + p * wps + static_cast<int64_t>(co) * hid + 32 * s + kc * 8);
      } else {
        const int q = v - (G::WP_CH - 80), t = q >> 3, c4 = q & 7;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>((t < 9 ? a.wd + t * hid : a.bd) + 32 * s + 4 * c4);
      }
    }
  };
  auto wp_store = [&]() {
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        *reinterpret_cast<u32x4_t*>(wpl + ((p * COUT + co) * WPP + wsw<WPP>(co, kc)) * 16) = wp_st[it];
      } else {
        const int q = v - (G::WP_CH - 80);
        *reinterpret_cast<u32x4_t*>(wdl + 4 * q) = wp_st[it];
      }
    }
  };
  we_load(0);
  wp_load(0);

  // ---- the wave's input pixels, split once: B fragments of every expand ----
  X3Frag xin[XL ? 1 : TPW][XL ? 1 : NK32];
  const float* xb = a.x + static_cast<int64_t>(b) * kIrpH * kIrpH * CIN;
  if constexpr (XL) {
    // the image into LDS (16-B chunks; rows padded to XP floats)
    for (int v = tid; v < kIrpH * kIrpH * (CIN / 4); v += NT) {
      const int px = v / (CIN / 4), q = v - px * (CIN / 4);
      *reinterpret_cast<f32x4_t*>(xl + px * G::XP + 4 * q) = *reinterpret_cast<const f32x4_t*>(xb + px * CIN + 4 * q);
    }
  } else {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int64_t off = (static_cast<int64_t>(ys) * kIrpH + x0s + par + t) * CIN + 8 * g;
#pragma unroll
      for (int c = 0; c < NK32; ++c) {
        f32x4_t lo = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c);
        f32x4_t hi = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c + 4);
        if (!real) lo = hi = f32x4_t{0.f, 0.f, 0.f, 0.f};
        xin[t][c] = split_x3(lo, hi);
      }
    }
  }
  // XL: this lane's fragment rows in the LDS image (tile t), zeros for the padding lanes
  auto xfrag = [&](int t, int c) -> X3Frag {
    if constexpr (XL) {
      const float* r = xl + (ys * kIrpH + x0s + par + t) * G::XP + 32 * c + 8 * g;
      f32x4_t lo = *reinterpret_cast<const f32x4_t*>(r);
      f32x4_t hi = *reinterpret_cast<const f32x4_t*>(r + 4);
      if (!real) lo = hi = f32x4_t{0.f, 0.f, 0.f, 0.f};
      return split_x3(lo, hi);
    } else {
      return xin[t][c];
    }
  };
  we_store();
  wp_store();
  __syncthreads();  // zeroed hidden image, step-0 weights

  f32x4_t acc[TPW][NO16];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int o = 0; o < NO16; ++o) acc[t][o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // expand output cell of this lane for tile t (column x0 + par + t); padding lanes -> scratch row
  int ecell[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) ecell[t] = real ? (y + 1) * kIrpRow + x0 + par + t + 1 : 16 * kIrpRow + li;
  // depthwise window origin: cell (ys - 1, x0s + par - 1) of the bordered grid
  const int wcell = ys * kIrpRow + x0s + par;

  // Two barriers per step, single weight buffers: the project / depthwise
  // weights of step s are loaded at the start of its expand phase and stored at
  // its end (their last readers, D(s - 1), finished before the previous B2; B1
  // publishes them to D(s)); the expand weights of step s + 1 are loaded after
  // B1 and stored at the end of D(s) (their readers, E(s), finished before B1;
  // B2 publishes them to E(s + 1)).
  for (int s = 0; s < nsteps; ++s) {
    if (s > 0) wp_load(s);
    // ================= expand (A: weights of hidden rows 16 ht + li) =================
    f32x4_t e[2][TPW];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
      for (int t = 0; t < TPW; ++t) e[ht][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NK32; ++c) {
      X3Frag xf[TPW];
#pragma unroll
      for (int t = 0; t < TPW; ++t) xf[t] = xfrag(t, c);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        X3Frag wa;
        const char* wr = wel + ((ht * 16 + li) * WEP + wsw<WEP>(li, 4 * c + g)) * 16;
        wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
        wa.m = *reinterpret_cast<const bf16x8_t*>(wr + 32 * WEP * 16);
        wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * 32 * WEP * 16);
#pragma unroll
        for (int t = 0; t < TPW; ++t) e[ht][t] += mfma_x3(wa, xf[t]);
      }
      // (the 14-wave forms: one k-step's operands live at a time, else the
      // scheduler hoists every step's LDS reads and spills past 128 VGPRs)
      if constexpr (TPW == 1) __builtin_amdgcn_sched_barrier(0);
    }
    // bias + ReLU6 -> the shared hidden image (lane: pixel slot li, channels 16 ht + 4 g .. + 3)
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
      const f32x4_t be4 = *reinterpret_cast<const f32x4_t*>(bel + ht * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < TPW; ++t) hb[(ht * 4 + g) * kIrpCells + ecell[t]] = relu6x4(e[ht][t] + be4);
    }
    if (s > 0) wp_store();
    __syncthreads();  // B1: hidden image and this step's project weights complete; wel free
    if (s + 1 < nsteps) we_load(s + 1);

    // ================= depthwise 3 x 3 (+ bias, ReLU6): TPW pixels x 8 channels =================
    f32x4_t d[2][TPW];  // [quad 2g + qq][pixel t]
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int q = 2 * g + qq;
      const f32x4_t bd4 = *reinterpret_cast<const f32x4_t*>(wdl + 9 * 32 + 4 * q);
      f32x4_t o[TPW];
#pragma unroll
      for (int t = 0; t < TPW; ++t) o[t] = bd4;
      const f32x4_t* hp = hb + q * kIrpCells + wcell;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        f32x4_t cc[TPW + 2];
#pragma unroll
        for (int j = 0; j < TPW + 2; ++j) cc[j] = hp[dy * kIrpRow + j];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const f32x4_t w = *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy + dx) * 32 + 4 * q);
#pragma unroll
          for (int t = 0; t < TPW; ++t) o[t] = __builtin_elementwise_fma(cc[t + dx], w, o[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) d[qq][t] = relu6x4(o[t]);
    }
    X3Frag bf[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) bf[t] = split_x3(d[0][t], d[1][t]);
    // ================= project (A: weights of output rows 16 o + li, k = this step's 32) =================
#pragma unroll
    for (int o = 0; o < NO16; ++o) {
      X3Frag wa;
      const char* wr = wpl + ((o * 16 + li) * WPP + wsw<WPP>(li, g)) * 16;
      wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
      wa.m = *reinterpret_cast<const bf16x8_t*>(wr + COUT * WPP * 16);
      wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * COUT * WPP * 16);
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t][o] += mfma_x3(wa, bf[t]);
    }
    if (s + 1 < nsteps) we_store();
    __syncthreads();  // B2: the next expand weights complete; hb, wpl and wdl free
  }

  // ---- epilogue: + bias (+ residual) -> NHWC ----
  if (!real) return;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int64_t pix = (static_cast<int64_t>(b) * kIrpH + y) * kIrpH + x0 + par + t;
#pragma unroll
    for (int o = 0; o < NO16; ++o) {
      const int co = o * 16 + 4 * g;
      f32x4_t v = acc[t][o] + *reinterpret_cast<const f32x4_t*>(a.bp + co);
      if (a.residual) {
        if constexpr (XL)
          v += *reinterpret_cast<const f32x4_t*>(xl + ((y * kIrpH) + x0 + par + t) * G::XP + co);
        else
          v += *reinterpret_cast<const f32x4_t*>(a.x + pix * CIN + co);
      }
      *reinterpret_cast<f32x4_t*>(a.y + pix * COUT + co) = v;
    }
  }
}

// ---------------------------------------------------------------------------
// irpp: the same block, software-pipelined over the hidden steps.  A 7-wave
// workgroup at 200+ VGPRs (or a 14-wave one at 128) is ONE workgroup per CU,
// so the LDS the second workgroup would have used is free: the hidden image
// and both weight stages are double-buffered, and step s runs the expand of
// step s + 1 (into hidden buffer (s + 1) & 1) next to the depthwise + project
// of step s (from buffer s & 1) -- ONE barrier per step instead of two, and
// half the waves (a.irp_order: the odd ones by default) take the two phases in the other
// order, so a SIMD's waves overlap one's MFMA expand with another's VALU / LDS
// depthwise instead of the whole CU alternating between them.
template <int CIN, int COUT, int TPW>
struct IrppGeom {
  static constexpr int NW = 14 / TPW, NT = 64 * NW;
  static constexpr int NK32 = CIN / 32, NO16 = COUT / 16;
  static constexpr int WEP = CIN / 8, WPP = 32 / 8;  // swizzled rows (wsw)
  static constexpr size_t hid1 = static_cast<size_t>(8) * kIrpCells * 16;
  static constexpr size_t we_w = static_cast<size_t>(3) * 32 * WEP * 16;     // expand weights of a stage
  static constexpr size_t we1 = we_w + 32 * 4;                               // + expand bias
  static constexpr size_t wp_w = static_cast<size_t>(3) * COUT * WPP * 16;   // project weights of a stage
  static constexpr size_t wp1 = wp_w + 10 * 32 * 4;                          // + depthwise taps and bias
  static constexpr size_t lds = 2 * (hid1 + we1 + wp1);
  static_assert(lds <= 160 * 1024, "irpp: LDS");
  static constexpr int WE_CH = 3 * 32 * (CIN / 8) + 8;
  static constexpr int WP_CH = 3 * COUT * 4 + 80;
  static constexpr int WE_IT = (WE_CH + NT - 1) / NT;
  static constexpr int WP_IT = (WP_CH + NT - 1) / NT;
  static constexpr int MINW = TPW == 2 ? 2 : 4;
};

template <int CIN, int COUT, int TPW>
__global__ void __launch_bounds__((IrppGeom<CIN, COUT, TPW>::NT), (IrppGeom<CIN, COUT, TPW>::MINW))
    irpp_x3_kernel(IrBlockF32Args a) {
  using G = IrppGeom<CIN, COUT, TPW>;
  constexpr int NK32 = G::NK32, NO16 = G::NO16, WEP = G::WEP, WPP = G::WPP, NT = G::NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* const base = reinterpret_cast<char*>(smem);
  // [hidden 0][hidden 1][expand stage 0][expand stage 1][project stage 0][project stage 1]
  auto hbuf = [&](int i) { return reinterpret_cast<f32x4_t*>(base + i * G::hid1); };
  auto webuf = [&](int i) { return base + 2 * G::hid1 + i * G::we1; };
  auto wpbuf = [&](int i) { return base + 2 * G::hid1 + 2 * G::we1 + i * G::wp1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const int hid = a.hid, nsteps = hid / 32;
  const int r0 = 2 * (TPW == 2 ? wave : wave >> 1);
  const int par = TPW == 2 ? 0 : (wave & 1);
  const bool real = li < 14;
  const int y = r0 + (li >= 7 ? 1 : 0);
  const int x0 = 2 * (li >= 7 ? li - 7 : li);
  const int ys = real ? y : r0, x0s = real ? x0 : 0;
  // phase order of this wave: 0 = expand first, 1 = depthwise + project first
  const int late_e = a.irp_order == 0 ? 0 : (a.irp_order == 2 ? (wave & 1) : ((wave >> 2) & 1));

  for (int v = tid; v < 2 * 8 * kIrpCells; v += NT) hbuf(0)[v] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int64_t wes = static_cast<int64_t>(hid) * CIN;
  const int64_t wps = static_cast<int64_t>(COUT) * hid;
  u32x4_t we_st[G::WE_IT], wp_st[G::WP_IT];
  auto we_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.we3 + p * wes + static_cast<int64_t>(32 * s + h) * CIN + kc * 8);
      } else {
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.be + 32 * s + 4 * (v - (G::WE_CH - 8)));
      }
    }
  };
  auto we_store = [&](int i) {
    char* wel = webuf(i);
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        *reinterpret_cast<u32x4_t*>(wel + ((p * 32 + h) * WEP + wsw<WEP>(h, kc)) * 16) = we_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(wel + G::we_w + 16 * (v - (G::WE_CH - 8))) = we_st[it];
      }
    }
  };
  auto wp_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>(a.wp3 + p * wps + static_cast<int64_t>(co) * hid + 32 * s + kc * 8);
      } else {
        const int q = v - (G::WP_CH - 80), t = q >> 3, c4 = q & 7;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>((t < 9 ? a.wd + t * hid : a.bd) + 32 * s + 4 * c4);
      }
    }
  };
  auto wp_store = [&](int i) {
    char* wpl = wpbuf(i);
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        *reinterpret_cast<u32x4_t*>(wpl + ((p * COUT + co) * WPP + wsw<WPP>(co, kc)) * 16) = wp_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(wpl + G::wp_w + 16 * (v - (G::WP_CH - 80))) = wp_st[it];
      }
    }
  };

  X3Frag xin[TPW][NK32];
  const float* xb = a.x + static_cast<int64_t>(b) * kIrpH * kIrpH * CIN;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int64_t off = (static_cast<int64_t>(ys) * kIrpH + x0s + par + t) * CIN + 8 * g;
#pragma unroll
    for (int c = 0; c < NK32; ++c) {
      f32x4_t lo = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c);
      f32x4_t hi = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c + 4);
      if (!real) lo = hi = f32x4_t{0.f, 0.f, 0.f, 0.f};
      xin[t][c] = split_x3(lo, hi);
    }
  }
  int ecell[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) ecell[t] = real ? (y + 1) * kIrpRow + x0 + par + t + 1 : 16 * kIrpRow + li;
  const int wcell = ys * kIrpRow + x0s + par;

  // expand of hidden step s: weights of stage s & 1 -> hidden buffer s & 1
  auto expand = [&](int s) {
    const char* wel = webuf(s & 1);
    f32x4_t* hb = hbuf(s & 1);
    f32x4_t e[2][TPW];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
      for (int t = 0; t < TPW; ++t) e[ht][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NK32; ++c) {
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        X3Frag wa;
        const char* wr = wel + ((ht * 16 + li) * WEP + wsw<WEP>(li, 4 * c + g)) * 16;
        wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
        wa.m = *reinterpret_cast<const bf16x8_t*>(wr + 32 * WEP * 16);
        wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * 32 * WEP * 16);
#pragma unroll
        for (int t = 0; t < TPW; ++t) e[ht][t] += mfma_x3(wa, xin[t][c]);
      }
      if constexpr (TPW == 1) __builtin_amdgcn_sched_barrier(0);
    }
    const float* bel = reinterpret_cast<const float*>(wel + G::we_w);
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
      const f32x4_t be4 = *reinterpret_cast<const f32x4_t*>(bel + ht * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < TPW; ++t) hb[(ht * 4 + g) * kIrpCells + ecell[t]] = relu6x4(e[ht][t] + be4);
    }
  };

  f32x4_t acc[TPW][NO16];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int o = 0; o < NO16; ++o) acc[t][o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // depthwise + project of hidden step s: hidden buffer s & 1, weights of stage s & 1
  auto dwproj = [&](int s) {
    const f32x4_t* hb = hbuf(s & 1);
    const char* wpl = wpbuf(s & 1);
    const float* wdl = reinterpret_cast<const float*>(wpl + G::wp_w);
    f32x4_t d[2][TPW];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int q = 2 * g + qq;
      const f32x4_t bd4 = *reinterpret_cast<const f32x4_t*>(wdl + 9 * 32 + 4 * q);
      f32x4_t o[TPW];
#pragma unroll
      for (int t = 0; t < TPW; ++t) o[t] = bd4;
      const f32x4_t* hp = hb + q * kIrpCells + wcell;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        f32x4_t cc[TPW + 2];
#pragma unroll
        for (int j = 0; j < TPW + 2; ++j) cc[j] = hp[dy * kIrpRow + j];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const f32x4_t w = *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy + dx) * 32 + 4 * q);
#pragma unroll
          for (int t = 0; t < TPW; ++t) o[t] = __builtin_elementwise_fma(cc[t + dx], w, o[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) d[qq][t] = relu6x4(o[t]);
    }
    X3Frag bf[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) bf[t] = split_x3(d[0][t], d[1][t]);
#pragma unroll
    for (int o = 0; o < NO16; ++o) {
      X3Frag wa;
      const char* wr = wpl + ((o * 16 + li) * WPP + wsw<WPP>(li, g)) * 16;
      wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
      wa.m = *reinterpret_cast<const bf16x8_t*>(wr + COUT * WPP * 16);
      wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * COUT * WPP * 16);
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t][o] += mfma_x3(wa, bf[t]);
    }
  };

  // prologue: stage 0 (expand + project) and stage 1 (expand), the expand of step 0
  we_load(0);
  wp_load(0);
  we_store(0);
  wp_store(0);
  if (nsteps > 1) {
    we_load(1);
    we_store(1);
  }
  __syncthreads();
  expand(0);
  __syncthreads();

  // Step s: E(s + 1) -> hidden (s + 1) & 1 and D/P(s) <- hidden s & 1, in this
  // wave's order; the stages loaded now (project s + 1, expand s + 2) go to
  // buffers whose readers (D/P(s - 1), E(s)) finished before the last barrier,
  // as did the readers of hidden (s + 1) & 1 (D/P(s - 1)).  One barrier.
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps, more2 = s + 2 < nsteps;
    if (more) wp_load(s + 1);
    if (more2) we_load(s + 2);
#pragma nounroll
    for (int ph = 0; ph < 2; ++ph) {
      if (ph == late_e) {
        if (more) expand(s + 1);
      } else {
        dwproj(s);
      }
      // (stored between the phases: the staging registers live across one phase)
      if (ph == 0) {
        if (more) wp_store((s + 1) & 1);
        if (more2) we_store(s & 1);
      }
    }
    __syncthreads();
  }

  if (!real) return;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int64_t pix = (static_cast<int64_t>(b) * kIrpH + y) * kIrpH + x0 + par + t;
#pragma unroll
    for (int o = 0; o < NO16; ++o) {
      const int co = o * 16 + 4 * g;
      f32x4_t v = acc[t][o] + *reinterpret_cast<const f32x4_t*>(a.bp + co);
      if (a.residual) v += *reinterpret_cast<const f32x4_t*>(a.x + pix * CIN + co);
      *reinterpret_cast<f32x4_t*>(a.y + pix * COUT + co) = v;
    }
  }
}

// ---------------------------------------------------------------------------
// irps: the stride-2 14 x 14 -> 7 x 7 block (96 -> 576 -> 160), one image per
// workgroup, pipelined like irpp.  8 waves:
//   * expand: the 196 input pixels as 13 dense 16-pixel tiles (waves 0-4 two,
//     waves 5-7 one), inputs split once and held in registers;
//   * depthwise (stride 2) + project: the 49 outputs as 4 16-pixel tiles;
//     wave w takes tile w / 2 and half of the 10 output-channel tiles;
//   * the stages loaded at a step's start are stored between its two phases
//     (their buffers' readers finished before the step began), so the staging
//     registers live across one phase only;
//   * LDS: a 15 x 15 bordered hidden grid (the stride-2 windows never reach row
//     or column 15), expand and project stages unpadded with the chunk index
//     XOR-swizzled by row (wsw: every ds_read_b128 lane group on 16 distinct
//     16-byte bank slots); double-buffered: 155 KB.
constexpr int kIrpsG = 15;                    // hidden grid (bordered): cell (y + 1, x + 1)
constexpr int kIrpsCells = kIrpsG * kIrpsG;   // 225

// First cell of hidden channel quad cq's plane in the stride-2 kernels (irps,
// irh S = 2).  A stride-2 window read (lane: output pixel li, quads 2 g + qq)
// reads columns 2 ox + dx, so all of a lane group's addresses have one slot
// parity -- 16 lanes on 8 bank slots, 2-way.  Shifting plane cq by cq / 2
// cells (g = cq / 2) puts a group's two g values on opposite parities:
// conflict-free for irps, 8 -> 4.6 cycles for irh S = 2 (scripts/lds_banks.py).
// The shift only grows with cq, so the planes stay disjoint: 3 cells past the
// 8 planes.
__device__ __forceinline__ int s2_plane(int cq, int cells) { return cq * cells + (cq >> 1); }

template <int CIN, int COUT>
struct IrpsGeom {
  static constexpr int NW = 8, NT = 64 * NW;
  static constexpr int NK32 = CIN / 32, NO16 = COUT / 16, NOH = NO16 / 2;
  static constexpr int WEP = CIN / 8;  // expand weight row pitch (16-B chunks, swizzled: wsw)
  static constexpr size_t hid1 = static_cast<size_t>(8 * kIrpsCells + 3) * 16;  // (+3: s2_plane)
  static constexpr size_t we_w = static_cast<size_t>(3) * 32 * WEP * 16;
  static constexpr size_t we1 = we_w + 32 * 4;
  static constexpr size_t wp_w = static_cast<size_t>(3) * COUT * 4 * 16;
  static constexpr size_t wp1 = wp_w + 10 * 32 * 4;
  static constexpr size_t lds = 2 * (hid1 + we1 + wp1);
  static_assert(lds <= 160 * 1024, "irps: LDS");
  static_assert(NO16 % 2 == 0, "irps: output tiles split in halves");
  static constexpr int WE_CH = 3 * 32 * (CIN / 8) + 8;
  static constexpr int WP_CH = 3 * COUT * 4 + 80;
  static constexpr int WE_IT = (WE_CH + NT - 1) / NT;
  static constexpr int WP_IT = (WP_CH + NT - 1) / NT;
};

// (TERMS: bit 0 = eight-product project, bit 1 = eight-product expand, bit 2 =
// compensated project accumulation (add_comp); A/B of the numerics)
template <int CIN, int COUT, int TERMS = 0>
__global__ void __launch_bounds__(512, 2) irps_x3_kernel(IrBlockF32Args a) {
  using G = IrpsGeom<CIN, COUT>;
  constexpr int NK32 = G::NK32, NO16 = G::NO16, NOH = G::NOH, WEP = G::WEP, NT = G::NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* const base = reinterpret_cast<char*>(smem);
  auto hbuf = [&](int i) { return reinterpret_cast<f32x4_t*>(base + i * G::hid1); };
  auto webuf = [&](int i) { return base + 2 * G::hid1 + i * G::we1; };
  auto wpbuf = [&](int i) { return base + 2 * G::hid1 + 2 * G::we1 + i * G::wp1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const int hid = a.hid, nsteps = hid / 32;
  const int late_e = a.irp_order == 0 ? 0 : (a.irp_order == 2 ? (wave & 1) : ((wave >> 2) & 1));
  // expand tiles of this wave: 2 w, 2 w + 1 (waves 5-7: w + 5 only)
  const bool two = wave < 5;
  const int et0 = two ? 2 * wave : wave + 5;
  // depthwise + project: output tile and the first of its output-channel tiles
  const int dt = wave >> 1;
  const int o0 = (wave & 1) * NOH;
  const int q = 16 * dt + li;  // output pixel of this lane
  const bool qreal = q < 49;
  const int oy = qreal ? q / 7 : 6, ox = qreal ? q - 7 * (q / 7) : 6;

  for (int v = tid; v < static_cast<int>(2 * G::hid1 / 16); v += NT) hbuf(0)[v] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int64_t wes = static_cast<int64_t>(hid) * CIN;
  const int64_t wps = static_cast<int64_t>(COUT) * hid;
  u32x4_t we_st[G::WE_IT], wp_st[G::WP_IT];
  auto we_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.we3 + p * wes + static_cast<int64_t>(32 * s + h) * CIN + kc * 8);
      } else {
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.be + 32 * s + 4 * (v - (G::WE_CH - 8)));
      }
    }
  };
  auto we_store = [&](int i) {
    char* wel = webuf(i);
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        *reinterpret_cast<u32x4_t*>(wel + ((p * 32 + h) * WEP + wsw<WEP>(h, kc)) * 16) = we_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(wel + G::we_w + 16 * (v - (G::WE_CH - 8))) = we_st[it];
      }
    }
  };
  auto wp_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>(a.wp3 + p * wps + static_cast<int64_t>(co) * hid + 32 * s + kc * 8);
      } else {
        const int qq = v - (G::WP_CH - 80), t = qq >> 3, c4 = qq & 7;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>((t < 9 ? a.wd + t * hid : a.bd) + 32 * s + 4 * c4);
      }
    }
  };
  // project stage: [part][row][wsw<4>(row, chunk)]
  auto wp_store = [&](int i) {
    char* wpl = wpbuf(i);
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        *reinterpret_cast<u32x4_t*>(wpl + ((p * COUT + co) * 4 + wsw<4>(co, kc)) * 16) = wp_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(wpl + G::wp_w + 16 * (v - (G::WP_CH - 80))) = wp_st[it];
      }
    }
  };

  // the wave's input pixels, split once (tile et0 + t; pixel 16 e + li)
  X3Frag xin[2][NK32];
  int ecell[2];
  const float* xb = a.x + static_cast<int64_t>(b) * kIrpH * kIrpH * CIN;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int p = 16 * (et0 + t) + li;
    const bool real = p < 196 && (t == 0 || two);
    const int ps = real ? p : 0;
    const int py = ps / 14, px = ps - 14 * (ps / 14);
    ecell[t] = real ? (py + 1) * kIrpsG + px + 1 : -1;
    const int64_t off = static_cast<int64_t>(ps) * CIN + 8 * g;
#pragma unroll
    for (int c = 0; c < NK32; ++c) {
      f32x4_t lo = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c);
      f32x4_t hi = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c + 4);
      if (!real) lo = hi = f32x4_t{0.f, 0.f, 0.f, 0.f};
      xin[t][c] = split_x3(lo, hi);
    }
  }
  const int wcell = 2 * oy * kIrpsG + 2 * ox;  // window origin: input (2 oy - 1, 2 ox - 1)

  auto expand = [&](int s) {
    const char* wel = webuf(s & 1);
    f32x4_t* hb = hbuf(s & 1);
    f32x4_t e[2][2];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
      for (int t = 0; t < 2; ++t) e[ht][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NK32; ++c) {
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        X3Frag wa;
        const char* wr = wel + ((ht * 16 + li) * WEP + wsw<WEP>(li, 4 * c + g)) * 16;
        wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
        wa.m = *reinterpret_cast<const bf16x8_t*>(wr + 32 * WEP * 16);
        wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * 32 * WEP * 16);
        if constexpr (TERMS & 2) {
          e[ht][0] += mfma_x3e(wa, xin[0][c]);
          if (two) e[ht][1] += mfma_x3e(wa, xin[1][c]);
        } else {
          e[ht][0] += mfma_x3(wa, xin[0][c]);
          if (two) e[ht][1] += mfma_x3(wa, xin[1][c]);
        }
      }
    }
    const float* bel = reinterpret_cast<const float*>(wel + G::we_w);
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
      const f32x4_t be4 = *reinterpret_cast<const f32x4_t*>(bel + ht * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (ecell[t] >= 0) hb[s2_plane(ht * 4 + g, kIrpsCells) + ecell[t]] = relu6x4(e[ht][t] + be4);
    }
  };

  f32x4_t acc[NOH], cmp[(TERMS & 4) ? NOH : 1];
#pragma unroll
  for (int o = 0; o < NOH; ++o) acc[o] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < ((TERMS & 4) ? NOH : 1); ++o) cmp[o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto dwproj = [&](int s) {
    const f32x4_t* hb = hbuf(s & 1);
    const char* wpl = wpbuf(s & 1);
    const float* wdl = reinterpret_cast<const float*>(wpl + G::wp_w);
    f32x4_t d[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int qd = 2 * g + qq;
      f32x4_t o = *reinterpret_cast<const f32x4_t*>(wdl + 9 * 32 + 4 * qd);
      const f32x4_t* hp = hb + s2_plane(qd, kIrpsCells) + wcell;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
          o = __builtin_elementwise_fma(hp[dy * kIrpsG + dx],
                                        *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy + dx) * 32 + 4 * qd), o);
      d[qq] = relu6x4(o);
    }
    const X3Frag bf = split_x3(d[0], d[1]);
#pragma unroll
    for (int oi = 0; oi < NOH; ++oi) {
      const int row = (o0 + oi) * 16 + li;
      const char* wr = wpl + (row * 4 + wsw<4>(row, g)) * 16;
      X3Frag wa;
      wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
      wa.m = *reinterpret_cast<const bf16x8_t*>(wr + COUT * 64);
      wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * COUT * 64);
      const f32x4_t tt = (TERMS & 1) ? mfma_x3e(wa, bf) : mfma_x3(wa, bf);
      if constexpr ((TERMS & 4) != 0)
        add_comp(acc[oi], cmp[(TERMS & 4) ? oi : 0], tt);
      else
        acc[oi] += tt;
    }
  };

  we_load(0);
  wp_load(0);
  we_store(0);
  wp_store(0);
  if (nsteps > 1) {
    we_load(1);
    we_store(1);
  }
  __syncthreads();
  expand(0);
  __syncthreads();
  // one barrier per step (irpp_x3_kernel's hazard argument, same buffers);
  // the stages go to LDS between the phases
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps, more2 = s + 2 < nsteps;
    if (more) wp_load(s + 1);
    if (more2) we_load(s + 2);
#pragma nounroll
    for (int ph = 0; ph < 2; ++ph) {
      if (ph == late_e) {
        if (more) expand(s + 1);
      } else {
        dwproj(s);
      }
      if (ph == 0) {
        if (more) wp_store((s + 1) & 1);
        if (more2) we_store(s & 1);
      }
    }
    __syncthreads();
  }

  if (!qreal) return;
  float* yo = a.y + (static_cast<int64_t>(b) * 49 + q) * COUT;
#pragma unroll
  for (int oi = 0; oi < NOH; ++oi) {
    const int co = (o0 + oi) * 16 + 4 * g;
    f32x4_t v = acc[oi];
    if constexpr ((TERMS & 4) != 0) v += cmp[(TERMS & 4) ? oi : 0];
    *reinterpret_cast<f32x4_t*>(yo + co) = v + *reinterpret_cast<const f32x4_t*>(a.bp + co);
  }
}

// ---------------------------------------------------------------------------
// irh: the 28 x 28 blocks (32 -> 192 -> 32 residual; S = 2: 32 -> 192 -> 64 to
// 14 x 14), HALF an image per workgroup (output rows of half h), pipelined like
// irpp.  The expand runs on
// the 15 image rows the half's depthwise windows need (S = 1: its 14 + one halo
// row; 420 pixels, 27 dense 16-pixel tiles) into a 16 x 30 bordered hidden
// grid; the depthwise + project on its outputs (S = 1: 392 pixels, 25 tiles;
// S = 2: 7 x 14 = 98, 7 tiles).  16 waves: waves 0-10 expand two tiles, 11-15
// one; S = 1: waves 7-15 run the depthwise + project of two output tiles, 0-6
// of one -- at most four tile-phases (48 split-bf16 MFMAs) per wave and step;
// S = 2: waves 0-13 one output tile and half its output channels.  cin = 32:
// one k-chunk, held split in registers.
// LDS: hidden 2 x 61 KB, expand / project stages 2 x 7.8 / 2 x 7.3 KB.
constexpr int kIrhW = 28, kIrhGW = 30;   // map width; hidden grid width (bordered)

template <int CIN, int COUT, int S>
struct IrhGeom {
  static constexpr int NW = 16, NT = 64 * NW;
  static constexpr int NK32 = CIN / 32, NO16 = COUT / 16;
  static constexpr int DT = S == 1 ? 2 : 1;             // output tiles per wave (at most)
  static constexpr int NOW = S == 1 ? NO16 : NO16 / 2;  // output-channel tiles per wave
  static constexpr int WO = kIrhW / S;                  // output map width
  // hidden grid rows: S = 1 16 (15 expand rows + a border row); S = 2 15 (the
  // windows never reach the last expand row of the top half)
  static constexpr int GH = S == 1 ? 16 : 15, CELLS = kIrhGW * GH;
  static constexpr int WEP = CIN / 8;  // expand weight row pitch (16-B chunks, swizzled: wsw)
  static constexpr size_t hid1 = static_cast<size_t>(8 * CELLS + (S == 2 ? 3 : 0)) * 16;  // (S = 2: s2_plane)
  static constexpr size_t we_w = static_cast<size_t>(3) * 32 * WEP * 16;
  static constexpr size_t we1 = we_w + 32 * 4;
  static constexpr size_t wp_w = static_cast<size_t>(3) * COUT * 4 * 16;
  static constexpr size_t wp1 = wp_w + 10 * 32 * 4;
  static constexpr size_t lds = 2 * (hid1 + we1 + wp1);
  static_assert(lds <= 160 * 1024, "irh: LDS");
  static constexpr int WE_CH = 3 * 32 * (CIN / 8) + 8;
  static constexpr int WP_CH = 3 * COUT * 4 + 80;
  static constexpr int WE_IT = (WE_CH + NT - 1) / NT;
  static constexpr int WP_IT = (WP_CH + NT - 1) / NT;
};

template <int CIN, int COUT, int S>
__global__ void __launch_bounds__(1024, 1) irh_x3_kernel(IrBlockF32Args a) {
  using G = IrhGeom<CIN, COUT, S>;
  constexpr int NK32 = G::NK32, WEP = G::WEP, NT = G::NT, DT = G::DT, NOW = G::NOW, WO = G::WO;
  constexpr int kIrhCells = G::CELLS;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* const base = reinterpret_cast<char*>(smem);
  auto hbuf = [&](int i) { return reinterpret_cast<f32x4_t*>(base + i * G::hid1); };
  auto webuf = [&](int i) { return base + 2 * G::hid1 + i * G::we1; };
  auto wpbuf = [&](int i) { return base + 2 * G::hid1 + 2 * G::we1 + i * G::wp1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.x >> 1, hh = blockIdx.x & 1;
  const int hid = a.hid, nsteps = hid / 32;
  const int late_e = a.irp_order == 0 ? 0 : (a.irp_order == 2 ? (wave & 1) : ((wave >> 2) & 1));
  // expand tiles (of 27) and depthwise + project tiles of this wave
  const bool e2 = wave < 11;
  const bool d2 = S == 1 && wave >= 7;
  const bool dact = S == 1 || wave < 14;
  const int dt0 = S == 1 ? (d2 ? 7 + 2 * (wave - 7) : wave) : (wave >> 1);
  const int o0 = S == 1 ? 0 : (wave & 1) * NOW;
  const int et0 = e2 ? 2 * wave : wave + 11;
  const int er0 = hh ? 13 : 0;      // first image row of the expand
  const int gro = hh ? 0 : 1;       // grid row of expand row er0

  for (int v = tid; v < static_cast<int>(2 * G::hid1 / 16); v += NT) hbuf(0)[v] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // plane of channel quad cq (S = 2: shifted by cq / 2 cells, s2_plane; S = 1
  // reads consecutive pixels, where the shift would cost: 5.9 -> 8 cycles)
  auto plane = [](int cq) { return S == 2 ? s2_plane(cq, kIrhCells) : cq * kIrhCells; };

  const int64_t wes = static_cast<int64_t>(hid) * CIN;
  const int64_t wps = static_cast<int64_t>(COUT) * hid;
  u32x4_t we_st[G::WE_IT], wp_st[G::WP_IT];
  auto we_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int pp = v / (32 * (CIN / 8)), r = v - pp * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.we3 + pp * wes + static_cast<int64_t>(32 * s + h) * CIN + kc * 8);
      } else {
        we_st[it] = *reinterpret_cast<const u32x4_t*>(a.be + 32 * s + 4 * (v - (G::WE_CH - 8)));
      }
    }
  };
  auto we_store = [&](int i) {
    char* wel = webuf(i);
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int pp = v / (32 * (CIN / 8)), r = v - pp * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        *reinterpret_cast<u32x4_t*>(wel + ((pp * 32 + h) * WEP + wsw<WEP>(h, kc)) * 16) = we_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(wel + G::we_w + 16 * (v - (G::WE_CH - 8))) = we_st[it];
      }
    }
  };
  auto wp_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int pp = v / (COUT * 4), r = v - pp * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>(a.wp3 + pp * wps + static_cast<int64_t>(co) * hid + 32 * s + kc * 8);
      } else {
        const int qq = v - (G::WP_CH - 80), tt = qq >> 3, c4 = qq & 7;
        wp_st[it] = *reinterpret_cast<const u32x4_t*>((tt < 9 ? a.wd + tt * hid : a.bd) + 32 * s + 4 * c4);
      }
    }
  };
  auto wp_store = [&](int i) {
    char* wpl = wpbuf(i);
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * NT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int pp = v / (COUT * 4), r = v - pp * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        *reinterpret_cast<u32x4_t*>(wpl + ((pp * COUT + co) * 4 + wsw<4>(co, kc)) * 16) = wp_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(wpl + G::wp_w + 16 * (v - (G::WP_CH - 80))) = wp_st[it];
      }
    }
  };

  // expand inputs: tile et0 + t, pixel pe = 16 tile + li of the 420 expand pixels
  X3Frag xin[2][NK32];
  int ecell[2];
  const float* xb = a.x + static_cast<int64_t>(b) * kIrhW * kIrhW * CIN;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int pe = 16 * (et0 + t) + li;
    const bool real = pe < 420 && (t == 0 || e2);
    const int ps = real ? pe : 0;
    const int r = ps / kIrhW, c = ps - kIrhW * (ps / kIrhW);
    ecell[t] = real && r + gro < G::GH ? (r + gro) * kIrhGW + c + 1 : -1;
    const int64_t off = (static_cast<int64_t>(er0 + r) * kIrhW + c) * CIN + 8 * g;
#pragma unroll
    for (int k = 0; k < NK32; ++k) {
      f32x4_t lo = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * k);
      f32x4_t hi = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * k + 4);
      if (!real) lo = hi = f32x4_t{0.f, 0.f, 0.f, 0.f};
      xin[t][k] = split_x3(lo, hi);
    }
  }
  // depthwise + project outputs: tile dt0 + t, pixel pd = 16 tile + li of the
  // half's (14 / S) x WO outputs; window origin: grid cell (S r, S c)
  int wcell[DT], opix[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    const int pd = 16 * (dt0 + t) + li;
    const bool real = dact && pd < (14 / S) * WO && (t == 0 || d2);
    const int ps = real ? pd : 0;
    const int r = ps / WO, c = ps - WO * (ps / WO);
    wcell[t] = S * r * kIrhGW + S * c;
    opix[t] = real ? ((14 / S) * hh + r) * WO + c : -1;
  }

  auto expand = [&](int s) {
    const char* wel = webuf(s & 1);
    f32x4_t* hb = hbuf(s & 1);
    f32x4_t e[2][2];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
      for (int t = 0; t < 2; ++t) e[ht][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NK32; ++k) {
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        X3Frag wa;
        const char* wr = wel + ((ht * 16 + li) * WEP + wsw<WEP>(li, 4 * k + g)) * 16;
        wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
        wa.m = *reinterpret_cast<const bf16x8_t*>(wr + 32 * WEP * 16);
        wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * 32 * WEP * 16);
        e[ht][0] += mfma_x3(wa, xin[0][k]);
        if (e2) e[ht][1] += mfma_x3(wa, xin[1][k]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const float* bel = reinterpret_cast<const float*>(wel + G::we_w);
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
      const f32x4_t be4 = *reinterpret_cast<const f32x4_t*>(bel + ht * 16 + 4 * g);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (ecell[t] >= 0) hb[plane(ht * 4 + g) + ecell[t]] = relu6x4(e[ht][t] + be4);
    }
  };

  f32x4_t acc[DT][NOW];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int o = 0; o < NOW; ++o) acc[t][o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto dwproj = [&](int s) {
    const f32x4_t* hb = hbuf(s & 1);
    const char* wpl = wpbuf(s & 1);
    const float* wdl = reinterpret_cast<const float*>(wpl + G::wp_w);
    if (!dact) return;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      if (t == 1 && !d2) break;
      f32x4_t d[2];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int qd = 2 * g + qq;
        f32x4_t o = *reinterpret_cast<const f32x4_t*>(wdl + 9 * 32 + 4 * qd);
        const f32x4_t* hp = hb + plane(qd) + wcell[t];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            o = __builtin_elementwise_fma(hp[dy * kIrhGW + dx],
                                          *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy + dx) * 32 + 4 * qd), o);
        d[qq] = relu6x4(o);
      }
      const X3Frag bf = split_x3(d[0], d[1]);
#pragma unroll
      for (int o = 0; o < NOW; ++o) {
        const int row = (o0 + o) * 16 + li;
        const char* wr = wpl + (row * 4 + wsw<4>(row, g)) * 16;
        X3Frag wa;
        wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
        wa.m = *reinterpret_cast<const bf16x8_t*>(wr + COUT * 64);
        wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * COUT * 64);
        acc[t][o] += mfma_x3(wa, bf);
      }
      // (one tile's operands live at a time: 16 waves need <= 128 VGPRs)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  we_load(0);
  wp_load(0);
  we_store(0);
  wp_store(0);
  if (nsteps > 1) {
    we_load(1);
    we_store(1);
  }
  __syncthreads();
  expand(0);
  __syncthreads();
  // one barrier per step (irpp_x3_kernel's hazard argument, same buffers)
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps, more2 = s + 2 < nsteps;
    if (more) wp_load(s + 1);
    if (more2) we_load(s + 2);
#pragma nounroll
    for (int ph = 0; ph < 2; ++ph) {
      if (ph == late_e) {
        if (more) expand(s + 1);
      } else {
        dwproj(s);
      }
      if (ph == 0) {
        if (more) wp_store((s + 1) & 1);
        if (more2) we_store(s & 1);
      }
    }
    __syncthreads();
  }

#pragma unroll
  for (int t = 0; t < DT; ++t) {
    if (opix[t] < 0) continue;
    const int64_t pix = static_cast<int64_t>(b) * WO * WO + opix[t];
#pragma unroll
    for (int o = 0; o < NOW; ++o) {
      const int co = (o0 + o) * 16 + 4 * g;
      f32x4_t v = acc[t][o] + *reinterpret_cast<const f32x4_t*>(a.bp + co);
      if (S == 1 && a.residual) v += *reinterpret_cast<const f32x4_t*>(a.x + pix * CIN + co);
      *reinterpret_cast<f32x4_t*>(a.y + pix * COUT + co) = v;
    }
  }
}

struct IrpCfg {
  int cin, cout, tpw;
  void (*kernel)(IrBlockF32Args);
  size_t lds;
  int threads;
  bool xl, pipe;
};
#define NNSX_IRP(CI, CO, T, XL) \
  IrpCfg { CI, CO, T, &irp_x3_kernel<CI, CO, T, XL>, IrpGeom<CI, CO, T, XL>::lds, IrpGeom<CI, CO, T, XL>::NT, XL, false }
#define NNSX_IRPP(CI, CO, T) \
  IrpCfg { CI, CO, T, &irpp_x3_kernel<CI, CO, T>, IrppGeom<CI, CO, T>::lds, IrppGeom<CI, CO, T>::NT, false, true }
// (first match per shape is the default; NNSX_IRP_TPW=1|2, NNSX_IRP_XL=0|1 and
// NNSX_IRP_PIPE=0|1 pick a variant).  Batch 512, us per block
// (profiles/r6_irp_layers_b512.txt), wave-split irw_x3 / irp TPW 2 / irp TPW 1 /
// irp TPW 1 XL / irpp TPW 2 (phase order 2):
//   64 -> 384 -> 64   143.9 / 111.0 / 115.7 /   -   / 110.2
//   64 -> 384 -> 96   187.1 / 125.5 / 143.2 /   -   / 131.9
//   96 -> 576 -> 96   315.6 / 309.2 / 279.0 / 248.6 / 223.4
const IrpCfg kIrpCfgs[] = {NNSX_IRP(64, 64, 2, false),  NNSX_IRP(64, 96, 2, false),  NNSX_IRPP(96, 96, 2),
                           NNSX_IRP(96, 96, 1, true),   NNSX_IRP(96, 96, 1, false),  NNSX_IRP(64, 64, 1, false),
                           NNSX_IRP(64, 96, 1, false),  NNSX_IRPP(64, 64, 2),        NNSX_IRPP(64, 96, 2),
                           NNSX_IRPP(64, 64, 1),        NNSX_IRPP(64, 96, 1),        NNSX_IRPP(96, 96, 1)};
#undef NNSX_IRP
#undef NNSX_IRPP

std::atomic<int> g_irp_min_b{[] {
  const char* e = std::getenv("NNSX_IRP_MIN_B");
  return e && *e ? std::atoi(e) : 128;
}()};

const IrpCfg* find_irp(const IrBlockF32Args& a) {
  // one workgroup per image: only batches that fill the chip (small batches keep
  // the wave-split kernels, which spread an image's hidden channels over CUs)
  const int min_b = g_irp_min_b.load(std::memory_order_relaxed);
  if (a.stride != 1 || a.dil != 1 || !a.has_expand || a.H != kIrpH || a.W != kIrpH || a.hid % 32 || !a.we3 ||
      !a.wp3 || a.B < min_b)
    return nullptr;
  // A/B: NNSX_IRP_TPW=1|2 picks that tile count, NNSX_IRP_XL=0|1 the input's place
  static const int tpw = [] {
    const char* e = std::getenv("NNSX_IRP_TPW");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  static const int xl = [] {
    const char* e = std::getenv("NNSX_IRP_XL");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
  }();
  // NNSX_IRP_PIPE=0|1: the two-barrier kernel / the pipelined one (irpp)
  static const int pipe = [] {
    const char* e = std::getenv("NNSX_IRP_PIPE");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
  }();
  for (const IrpCfg& c : kIrpCfgs)
    if (c.cin == a.cin && c.cout == a.cout && (tpw == 0 || c.tpw == tpw) && (xl < 0 || c.xl == (xl == 1)) &&
        (pipe < 0 || c.pipe == (pipe == 1)))
      return &c;
  return nullptr;
}

}  // namespace

// NNSX_IRP=0 turns the image-per-workgroup kernels off (A/B)
static bool irp_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NNSX_IRP");
    return !(e && e[0] == '0');
  }();
  return on;
}

// the stride-2 14 -> 7 block (irps); NNSX_IRPS=0 turns it off (A/B)
static bool irps_match(const IrBlockF32Args& a) {
  static const bool on = [] {
    const char* e = std::getenv("NNSX_IRPS");
    return !(e && e[0] == '0');
  }();
  return on && a.stride == 2 && a.dil == 1 && a.has_expand && a.H == kIrpH && a.W == kIrpH && a.cin == 96 &&
         a.cout == 160 && a.hid % 32 == 0 && a.hid >= 64 && a.we3 && a.wp3 && !a.residual &&
         a.B >= g_irp_min_b.load(std::memory_order_relaxed);
}

// the 28 x 28 32 -> 192 -> 32 block and the 28 -> 14 32 -> 192 -> 64 one, half
// an image per workgroup (irh): 157.5 vs 188 / 109 vs 138 us at batch 512, and
// the sustained pipeline 3.753 vs 3.866 ms per invoke on the same box
// (profiles/r6_host_bound_converter.txt; an earlier A/B that had it slower was
// bound by the converter's per-frame event records, not the GPU).  Mode 2 =
// both (default), 1 = the stride-2 one, 0 = off (NNSX_IRH, or irh_mode() at run time)
std::atomic<int> g_irh_mode{[] {
  const char* e = std::getenv("NNSX_IRH");
  return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 2;
}()};

static bool irh_match(const IrBlockF32Args& a) {
  const int on = g_irh_mode.load(std::memory_order_relaxed);
  const bool s1 = a.stride == 1 && a.cout == 32 && on >= 2;
  const bool s2 = a.stride == 2 && a.cout == 64 && !a.residual && on >= 1;
  return (s1 || s2) && a.dil == 1 && a.has_expand && a.H == kIrhW && a.W == kIrhW && a.cin == 32 &&
         a.hid % 32 == 0 && a.hid >= 64 && a.we3 && a.wp3 && a.B >= g_irp_min_b.load(std::memory_order_relaxed);
}

int irh_set_mode(int m) { return g_irh_mode.exchange(m); }

bool irp_x3_supported(const IrBlockF32Args& a) {
  return irp_enabled() && (irps_match(a) || irh_match(a) || find_irp(a) != nullptr);
}

int irp_x3_set_min_batch(int b) { return g_irp_min_b.exchange(b); }

bool irp_x3(const IrBlockF32Args& args, hipStream_t s) {
  if (irp_enabled() && irps_match(args)) {
    using G = IrpsGeom<96, 160>;
    IrBlockF32Args a = args;
    a.irp_order = 2;
    // NNSX_IRPS_TERMS=0..5: product terms of the project (bit 0) / expand (bit 1),
    // compensated project accumulation (bit 2).  Default 4: with plain fp32 adds
    // of the 18 k-step partials the max error against fp64 exceeded the native
    // kernel's on 2 of 6 seeds (x1.09; mean x0.66); compensated, x0.45-0.61 (mean
    // x0.51) for 30 us more (profiles/r6_irps_numerics.txt); eight-product
    // terms change nothing
    static const int terms = [] {
      const char* e = std::getenv("NNSX_IRPS_TERMS");
      return e && e[0] >= '0' && e[0] <= '5' ? e[0] - '0' : 4;
    }();
    void (*k)(IrBlockF32Args) = terms == 1   ? &irps_x3_kernel<96, 160, 1>
                                : terms == 2 ? &irps_x3_kernel<96, 160, 2>
                                : terms == 3 ? &irps_x3_kernel<96, 160, 3>
                                : terms == 4 ? &irps_x3_kernel<96, 160, 4>
                                : terms == 5 ? &irps_x3_kernel<96, 160, 5>
                                             : &irps_x3_kernel<96, 160, 0>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return false;
    hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(a.B)), dim3(G::NT), G::lds, s, a);
    return true;
  }
  if (irp_enabled() && irh_match(args)) {
    IrBlockF32Args a = args;
    a.irp_order = 2;
    void (*k)(IrBlockF32Args) = a.stride == 2 ? &irh_x3_kernel<32, 64, 2> : &irh_x3_kernel<32, 32, 1>;
    const size_t lds = a.stride == 2 ? IrhGeom<32, 64, 2>::lds : IrhGeom<32, 32, 1>::lds;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return false;
    hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(2 * a.B)), dim3(1024), lds, s, a);
    return true;
  }
  const IrpCfg* c = irp_enabled() ? find_irp(args) : nullptr;
  if (!c) return false;
  IrBlockF32Args a = args;
  // irpp phase order (NNSX_IRP_ORDER: 0 = every wave expand first, 1 = waves with
  // bit 2 set depthwise + project first, 2 = odd waves -- the fastest: 223.4 /
  // 227.4 / 227.8 us on 96 -> 576 -> 96, profiles/r6_irp_layers_b512.txt)
  static const int order = [] {
    const char* e = std::getenv("NNSX_IRP_ORDER");
    return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 2;
  }();
  a.irp_order = order;
  if (c->lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(c->kernel),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
    return false;
  hipLaunchKernelGGL(c->kernel, dim3(static_cast<unsigned>(a.B)), dim3(c->threads), c->lds, s, a);
  return true;
}

}  // namespace kernels
}  // namespace nnsx
