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

namespace nnsx {
namespace kernels {

namespace {

constexpr int kIrpH = 14;           // map size handled (S = 1)
constexpr int kIrpWaves = 7;        // two image rows per wave
constexpr int kIrpNT = 64 * kIrpWaves;
constexpr int kIrpRow = 16;         // hidden grid row pitch (cells): 14 + 2 border
constexpr int kIrpCells = 16 * kIrpRow + 16;  // + one scratch row for the padding lanes

template <int CIN, int COUT>
struct IrpGeom {
  static constexpr int NK32 = CIN / 32;        // expand k-steps
  static constexpr int NO16 = COUT / 16;       // project output tiles
  static constexpr int WEP = CIN / 8 + 1;      // expand weight row pitch (16-B chunks): odd -> conflict-free
  static constexpr int WPP = 32 / 8 + 1;       // project weight row pitch (chunks)
  static constexpr size_t hid_b = static_cast<size_t>(8) * kIrpCells * 16;      // [quad][cell] f32x4
  static constexpr size_t we_b = static_cast<size_t>(3) * 32 * WEP * 16;        // [part][hid row][chunk]
  static constexpr size_t wp_b = static_cast<size_t>(3) * COUT * WPP * 16;      // [part][cout row][chunk]
  static constexpr size_t wd_b = static_cast<size_t>(10) * 32 * 4;              // [tap | bias][ch] f32
  static constexpr size_t be_b = static_cast<size_t>(32) * 4;
  static constexpr size_t lds = hid_b + we_b + wp_b + wd_b + be_b;
  // 16-B chunks staged per step
  static constexpr int WE_CH = 3 * 32 * (CIN / 8) + 8;   // + expand bias (32 f32)
  static constexpr int WP_CH = 3 * COUT * 4 + 80;         // + depthwise taps and bias (10 x 32 f32)
  static constexpr int WE_IT = (WE_CH + kIrpNT - 1) / kIrpNT;
  static constexpr int WP_IT = (WP_CH + kIrpNT - 1) / kIrpNT;
};

template <int CIN, int COUT>
__global__ void __launch_bounds__(kIrpNT, 2) irp_x3_kernel(IrBlockF32Args a) {
  using G = IrpGeom<CIN, COUT>;
  constexpr int NK32 = G::NK32, NO16 = G::NO16, WEP = G::WEP, WPP = G::WPP;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  f32x4_t* hb = reinterpret_cast<f32x4_t*>(smem);                                   // [8][kIrpCells]
  char* wel = reinterpret_cast<char*>(smem) + G::hid_b;                              // expand weights
  char* wpl = wel + G::we_b;                                                         // project weights
  float* wdl = reinterpret_cast<float*>(wpl + G::wp_b);                              // [10][32]
  float* bel = wdl + 320;                                                            // [32]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const int hid = a.hid, nsteps = hid / 32;
  const int r0 = 2 * wave;
  // this lane's pixel slot (both tiles: columns x0 and x0 + 1 of row y)
  const bool real = li < 14;
  const int y = r0 + (li >= 7 ? 1 : 0);
  const int x0 = 2 * (li >= 7 ? li - 7 : li);
  const int ys = real ? y : r0, x0s = real ? x0 : 0;  // (padding lanes read a valid window)

  // ---- zero the hidden image (its border is the depthwise padding) ----
  for (int v = tid; v < 8 * kIrpCells; v += kIrpNT) hb[v] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- weight staging (16-B chunks through registers) ----
  const int64_t wes = static_cast<int64_t>(hid) * CIN;     // we3 part stride (elements)
  const int64_t wps = static_cast<int64_t>(COUT) * hid;    // wp3 part stride (cout multiple of 32)
  u32x4_t we_st[G::WE_IT], wp_st[G::WP_IT];
  auto we_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WE_IT; ++it) {
      const int v = tid + it * kIrpNT;
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
      const int v = tid + it * kIrpNT;
      if (v >= G::WE_CH) break;
      if (v < G::WE_CH - 8) {
        const int p = v / (32 * (CIN / 8)), r = v - p * 32 * (CIN / 8);
        const int h = r / (CIN / 8), kc = r - h * (CIN / 8);
        *reinterpret_cast<u32x4_t*>(wel + ((p * 32 + h) * WEP + kc) * 16) = we_st[it];
      } else {
        *reinterpret_cast<u32x4_t*>(bel + 4 * (v - (G::WE_CH - 8))) = we_st[it];
      }
    }
  };
  auto wp_load = [&](int s) {
#pragma unroll
    for (int it = 0; it < G::WP_IT; ++it) {
      const int v = tid + it * kIrpNT;
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
      const int v = tid + it * kIrpNT;
      if (v >= G::WP_CH) break;
      if (v < G::WP_CH - 80) {
        const int p = v / (COUT * 4), r = v - p * COUT * 4;
        const int co = r >> 2, kc = r & 3;
        *reinterpret_cast<u32x4_t*>(wpl + ((p * COUT + co) * WPP + kc) * 16) = wp_st[it];
      } else {
        const int q = v - (G::WP_CH - 80);
        *reinterpret_cast<u32x4_t*>(wdl + 4 * q) = wp_st[it];
      }
    }
  };
  we_load(0);
  wp_load(0);

  // ---- the wave's input pixels, split once: B fragments of every expand ----
  X3Frag xin[2][NK32];
  {
    const float* xb = a.x + static_cast<int64_t>(b) * kIrpH * kIrpH * CIN;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int64_t off = (static_cast<int64_t>(ys) * kIrpH + x0s + t) * CIN + 8 * g;
#pragma unroll
      for (int c = 0; c < NK32; ++c) {
        f32x4_t lo = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c);
        f32x4_t hi = *reinterpret_cast<const f32x4_t*>(xb + off + 32 * c + 4);
        if (!real) lo = hi = f32x4_t{0.f, 0.f, 0.f, 0.f};
        xin[t][c] = split_x3(lo, hi);
      }
    }
  }
  we_store();
  wp_store();
  __syncthreads();  // zeroed hidden image, step-0 weights

  f32x4_t acc[2][NO16];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int o = 0; o < NO16; ++o) acc[t][o] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // expand output cells of this lane (tile t: column x0 + t); padding lanes -> scratch row
  const int ecell0 = real ? (y + 1) * kIrpRow + x0 + 1 : 16 * kIrpRow + li;
  const int ecell1 = real ? ecell0 + 1 : 16 * kIrpRow + li;
  // depthwise window origin: cell (ys - 1, x0s - 1) of the bordered grid = (ys) * row + x0s
  const int wcell = ys * kIrpRow + x0s;

  // Two barriers per step, single weight buffers: the project / depthwise
  // weights of step s are loaded at the start of its expand phase and stored at
  // its end (their last readers, D(s - 1), finished before the previous B2; B1
  // publishes them to D(s)); the expand weights of step s + 1 are loaded after
  // B1 and stored at the end of D(s) (their readers, E(s), finished before B1;
  // B2 publishes them to E(s + 1)).
  for (int s = 0; s < nsteps; ++s) {
    if (s > 0) wp_load(s);
    // ================= expand (A: weights of hidden rows 16 ht + li) =================
    f32x4_t e[2][2];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
#pragma unroll
      for (int t = 0; t < 2; ++t) e[ht][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NK32; ++c) {
        X3Frag wa;
        const char* wr = wel + ((ht * 16 + li) * WEP + 4 * c + g) * 16;
        wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
        wa.m = *reinterpret_cast<const bf16x8_t*>(wr + 32 * WEP * 16);
        wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * 32 * WEP * 16);
#pragma unroll
        for (int t = 0; t < 2; ++t) e[ht][t] += mfma_x3(wa, xin[t][c]);
      }
    }
    // bias + ReLU6 -> the shared hidden image (lane: pixel slot li, channels 16 ht + 4 g .. + 3)
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) {
      const f32x4_t be4 = *reinterpret_cast<const f32x4_t*>(bel + ht * 16 + 4 * g);
      hb[(ht * 4 + g) * kIrpCells + ecell0] = relu6x4(e[ht][0] + be4);
      hb[(ht * 4 + g) * kIrpCells + ecell1] = relu6x4(e[ht][1] + be4);
    }
    if (s > 0) wp_store();
    __syncthreads();  // B1: hidden image and this step's project weights complete; wel free
    if (s + 1 < nsteps) we_load(s + 1);

    // ================= depthwise 3 x 3 (+ bias, ReLU6): 2 pixels x 8 channels =================
    f32x4_t d[2][2];  // [quad 2g + qq][pixel t]
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int q = 2 * g + qq;
      const f32x4_t bd4 = *reinterpret_cast<const f32x4_t*>(wdl + 9 * 32 + 4 * q);
      f32x4_t o0 = bd4, o1 = bd4;
      const f32x4_t* hp = hb + q * kIrpCells + wcell;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const f32x4_t c0 = hp[dy * kIrpRow], c1 = hp[dy * kIrpRow + 1], c2 = hp[dy * kIrpRow + 2],
                      c3 = hp[dy * kIrpRow + 3];
        const f32x4_t w0 = *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy) * 32 + 4 * q);
        const f32x4_t w1 = *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy + 1) * 32 + 4 * q);
        const f32x4_t w2 = *reinterpret_cast<const f32x4_t*>(wdl + (3 * dy + 2) * 32 + 4 * q);
        o0 = __builtin_elementwise_fma(c0, w0, o0);
        o0 = __builtin_elementwise_fma(c1, w1, o0);
        o0 = __builtin_elementwise_fma(c2, w2, o0);
        o1 = __builtin_elementwise_fma(c1, w0, o1);
        o1 = __builtin_elementwise_fma(c2, w1, o1);
        o1 = __builtin_elementwise_fma(c3, w2, o1);
      }
      d[qq][0] = relu6x4(o0);
      d[qq][1] = relu6x4(o1);
    }
    const X3Frag bf0 = split_x3(d[0][0], d[1][0]);
    const X3Frag bf1 = split_x3(d[0][1], d[1][1]);
    // ================= project (A: weights of output rows 16 o + li, k = this step's 32) =================
#pragma unroll
    for (int o = 0; o < NO16; ++o) {
      X3Frag wa;
      const char* wr = wpl + ((o * 16 + li) * WPP + g) * 16;
      wa.h = *reinterpret_cast<const bf16x8_t*>(wr);
      wa.m = *reinterpret_cast<const bf16x8_t*>(wr + COUT * WPP * 16);
      wa.l = *reinterpret_cast<const bf16x8_t*>(wr + 2 * COUT * WPP * 16);
      acc[0][o] += mfma_x3(wa, bf0);
      acc[1][o] += mfma_x3(wa, bf1);
    }
    if (s + 1 < nsteps) we_store();
    __syncthreads();  // B2: the next expand weights complete; hb, wpl and wdl free
  }

  // ---- epilogue: + bias (+ residual) -> NHWC ----
  if (!real) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int64_t pix = (static_cast<int64_t>(b) * kIrpH + y) * kIrpH + x0 + t;
#pragma unroll
    for (int o = 0; o < NO16; ++o) {
      const int co = o * 16 + 4 * g;
      f32x4_t v = acc[t][o] + *reinterpret_cast<const f32x4_t*>(a.bp + co);
      if (a.residual) v += *reinterpret_cast<const f32x4_t*>(a.x + pix * CIN + co);
      *reinterpret_cast<f32x4_t*>(a.y + pix * COUT + co) = v;
    }
  }
}

struct IrpCfg {
  int cin, cout;
  void (*kernel)(IrBlockF32Args);
  size_t lds;
};
#define NNSX_IRP(CI, CO) IrpCfg{CI, CO, &irp_x3_kernel<CI, CO>, IrpGeom<CI, CO>::lds}
const IrpCfg kIrpCfgs[] = {NNSX_IRP(64, 64), NNSX_IRP(64, 96), NNSX_IRP(96, 96)};
#undef NNSX_IRP

const IrpCfg* find_irp(const IrBlockF32Args& a) {
  if (a.stride != 1 || a.dil != 1 || !a.has_expand || a.H != kIrpH || a.W != kIrpH || a.hid % 32 || !a.we3 ||
      !a.wp3)
    return nullptr;
  for (const IrpCfg& c : kIrpCfgs)
    if (c.cin == a.cin && c.cout == a.cout) return &c;
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

bool irp_x3_supported(const IrBlockF32Args& a) { return irp_enabled() && find_irp(a) != nullptr; }

bool irp_x3(const IrBlockF32Args& a, hipStream_t s) {
  const IrpCfg* c = irp_enabled() ? find_irp(a) : nullptr;
  if (!c) return false;
  if (c->lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(c->kernel),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
    return false;
  hipLaunchKernelGGL(c->kernel, dim3(static_cast<unsigned>(a.B)), dim3(kIrpNT), c->lds, s, a);
  return true;
}

}  // namespace kernels
}  // namespace nnsx
