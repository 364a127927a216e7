// irw_x3: the fused inverted residual on split-bf16 MFMAs, in a translation
// unit of its own built with the MFMA results in VGPRs (kernels/irw_common.h).
#include "kernels/irw_common.h"

namespace nnsx {
namespace kernels {

namespace {

// ------------------------------------------------------------- irw_x3 ----
// The wave-split fused inverted residual with its products on split-bf16
// MFMAs (kernels/x3.h): the same tiles, waves, hidden parts and combine as
// irw_f32, and
//   * the input tile is split once, while it is staged: three bf16 planes
//     [part][k8][cell] (8 channels = 16 B per cell), cells XOR-swizzled by k8
//     within their 16-cell group (the staging writes spread over the banks;
//     a fragment read stays 256 contiguous bytes per 16 lanes);
//   * expand: per 16-channel subtile, six v_mfma_f32_16x16x32_bf16 per 32 input
//     channels (weights pre-split at export: we3 [3][hid][ceil32(cin)] bf16);
//   * depthwise: lane = one pixel of a 32-pixel tile x 8 of the subtile's 16
//     channels -- exactly the B operand of v_mfma_f32_32x32x16_bf16 (k = 8 (l >> 5)
//     + j), split into its three parts in registers;
//   * project: 32 output channels x 32 pixels x the subtile's 16 channels per
//     six 32x32x16 MFMAs (wp3 [3][ceil32(cout)][hid] bf16), the subtile's
//     partial added to the accumulator by the VALU (round to nearest).
// The cross-wave reduction, hidden parts and in-launch combine are irw_f32's.
template <int S, int TY, int TX, int KIN, int NOT, int NW, bool FULL, int DIL = 1>
struct IrwX3Geom {
  using Base = IrwGeom<S, TY, TX, KIN, NOT, NW, FULL, DIL>;
  static constexpr int TIY = Base::TIY, TIX = Base::TIX, PIN = Base::PIN, NC16 = Base::NC16, NBT = Base::NBT;
  static constexpr int PINP = Base::PINP;
  static constexpr int KP = (KIN + 31) / 32 * 32, NK32 = KP / 32, K8 = KP / 8;
  static constexpr int XSP = NC16;                   // cells per plane
  static constexpr int NP32 = (TY * TX + 31) / 32;   // 32-pixel project tiles
  static constexpr int NPX = NP32 * 32;
  static constexpr int NO32 = (NOT * 16 + 31) / 32;  // 32-channel output tiles (rows of wp3)
  static constexpr size_t xs_b = static_cast<size_t>(3) * K8 * XSP * 16;
  static constexpr size_t hid_b = static_cast<size_t>(16) * 4 * NW * PINP;
  static constexpr size_t red_b = static_cast<size_t>(16) * 8 * NW * NPX;  // [wave][cout quad][px]
  // + the depthwise weights and bias of the workgroup's hidden channels, [10][hid]
  // (taps 0-8, bias), staged once: read per subtile just before the depthwise
  static size_t lds_bytes(int hid) {
    return std::max(xs_b + hid_b + static_cast<size_t>(40) * hid, red_b);
  }
  static constexpr int MINB = (NOT > 0 && NO32 * NP32 <= 4) ? 2 : 1;
};

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

template <int S, int TY, int TX, int KIN, int NOT, int NW, bool FULL, int DIL = 1>
__global__ void __launch_bounds__(64 * NW, (IrwX3Geom<S, TY, TX, KIN, NOT, NW, FULL, DIL>::MINB))
    irw_x3_kernel(IrBlockF32Args a) {
  using G = IrwX3Geom<S, TY, TX, KIN, NOT, NW, FULL, DIL>;
  constexpr int NT = 64 * NW;
  constexpr int TIX = G::TIX, PIN = G::PIN, NC16 = G::NC16, NBT = G::NBT, PINP = G::PINP;
  constexpr int KP = G::KP, K8 = G::K8, NK32 = G::NK32, XSP = G::XSP, NP32 = G::NP32, NPX = G::NPX;
  constexpr int NO32 = G::NO32, NOA = NO32 > 0 ? NO32 : 1;
  constexpr int KQP = KP / 4;  // fp32 quads staged per cell (zeros past cin)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  bf16x8_t* xs = reinterpret_cast<bf16x8_t*>(smem);  // [3][K8][XSP], cell swizzled by k8
  f32x4_t* hidw = reinterpret_cast<f32x4_t*>(reinterpret_cast<char*>(smem) + G::xs_b);  // [NW][4][PINP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, l32 = lane & 31, h = lane >> 5;
  const int nparts = a.hsplit;
  const int tiles_img = a.tiles_x * a.tiles_y;

  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int part = wg % nparts, tile = wg / nparts;
  const int b = tile / tiles_img;
  const int tyx = tile - b * tiles_img;
  const int oy0 = (tyx / a.tiles_x) * TY, ox0 = (tyx % a.tiles_x) * TX;
  const int iy0 = oy0 * S - DIL, ix0 = ox0 * S - DIL;
  const int ry0 = max(iy0, 0), ry1 = min(iy0 + G::TIY, a.H);
  const int rx0 = max(ix0, 0), rx1 = min(ix0 + TIX, a.W);
  const int RW = rx1 - rx0, NC = FULL ? PIN : (ry1 - ry0) * RW;
  const float rrw = 1.f / static_cast<float>(RW);

  // ---- stage the input tile, split into its bf16 parts on the way (loads of
  // the whole tile issued first, branch-free, then the LDS stores)
  {
    constexpr int NSV = NC16 * KQP, NSIT = (NSV + NT - 1) / NT;
    f32x4_t sv[NSIT];
    bool sok[NSIT];
    const float* qb = a.x + static_cast<int64_t>(b) * a.H * a.W * a.cin;
#pragma unroll
    for (int it = 0; it < NSIT; ++it) {
      const int v = tid + it * NT;
      const int c = v / KQP, kq = v - c * KQP;
      int yy, xx;
      if constexpr (FULL) {
        yy = iy0 + c / TIX;
        xx = ix0 + c % TIX;
      } else {
        const int cy = static_cast<int>((static_cast<float>(c) + 0.5f) * rrw);
        yy = ry0 + cy;
        xx = rx0 + c - cy * RW;
      }
      const bool ok = (NSV % NT == 0 || v < NSV) && c < NC && kq * 4 < a.cin && yy >= 0 && yy < a.H && xx >= 0 &&
                      xx < a.W;
      const int64_t off = ok ? (static_cast<int64_t>(yy) * a.W + xx) * a.cin + kq * 4 : 0;
      sok[it] = ok;
      sv[it] = *reinterpret_cast<const f32x4_t*>(qb + off);
    }
#pragma unroll
    for (int it = 0; it < NSIT; ++it) {
      const int v = tid + it * NT;
      if (NSV % NT != 0 && v >= NSV) break;
      const int c = v / KQP, kq = v - c * KQP, k8 = kq >> 1;
      if (!sok[it]) sv[it] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      bf16x2_t h0, m0, l0, h1, m1, l1;
      split2(f32x2_t{sv[it][0], sv[it][1]}, h0, m0, l0);
      split2(f32x2_t{sv[it][2], sv[it][3]}, h1, m1, l1);
      char* p = reinterpret_cast<char*>(xs) + (static_cast<size_t>(k8) * XSP + (c ^ (k8 & 15))) * 16 + (kq & 1) * 8;
      constexpr size_t PS = static_cast<size_t>(K8) * XSP * 16;  // part stride (bytes)
      *reinterpret_cast<bf16x4_t*>(p) = __builtin_shufflevector(h0, h1, 0, 1, 2, 3);
      *reinterpret_cast<bf16x4_t*>(p + PS) = __builtin_shufflevector(m0, m1, 0, 1, 2, 3);
      *reinterpret_cast<bf16x4_t*>(p + 2 * PS) = __builtin_shufflevector(l0, l1, 0, 1, 2, 3);
    }
  }
  if (!FULL && (ry0 > iy0 || ry1 < iy0 + G::TIY || rx0 > ix0 || rx1 < ix0 + TIX)) {
    for (int v = tid; v < 4 * NW * PIN; v += NT) {
      const int pl = v / PIN, p = v - pl * PIN;
      const int yy = iy0 + p / TIX, xx = ix0 + p % TIX;
      if (yy < ry0 || yy >= ry1 || xx < rx0 || xx >= rx1) hidw[pl * PINP + p] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  }
  int hcell[NBT];
#pragma unroll
  for (int j = 0; j < NBT; ++j) {
    const int c = j * 16 + li;
    if constexpr (FULL) {
      const int yy = iy0 + c / TIX, xx = ix0 + c % TIX;
      hcell[j] = (c < PIN && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) ? 1 : 0;
    } else {
      const int cy = static_cast<int>((static_cast<float>(c) + 0.5f) * rrw);
      hcell[j] = c < NC ? (ry0 + cy - iy0) * TIX + (rx0 + c - cy * RW - ix0) : PIN;
    }
  }
  int dcell[NP32];
#pragma unroll
  for (int pt = 0; pt < NP32; ++pt) {
    const int q = pt * 32 + l32;
    const int qq = q < TY * TX ? q : 0;
    dcell[pt] = (qq / TX) * S * TIX + (qq % TX) * S;
  }
  const int nbt = (NC + 15) / 16;

  f32x16_t acc[NP32][NOA];
#pragma unroll
  for (int pt = 0; pt < NP32; ++pt)
#pragma unroll
    for (int o = 0; o < NOA; ++o) acc[pt][o] = f32x16_t{};

  const int nsub = a.hid >> 4;
  const int sub0 = part * nsub / nparts, sub1 = (part + 1) * nsub / nparts;
  // the part's depthwise taps + bias into LDS ([10][nch], row 9 = bias)
  const int nch = (sub1 - sub0) * 16, ch0 = sub0 * 16;
  f32x4_t* wdl = reinterpret_cast<f32x4_t*>(reinterpret_cast<char*>(smem) + G::xs_b + G::hid_b);
  for (int v = tid; v < 10 * (nch / 4); v += NT) {
    const int t = v / (nch / 4), q = v - t * (nch / 4);
    wdl[v] = *reinterpret_cast<const f32x4_t*>((t < 9 ? a.wd + t * a.hid : a.bd) + ch0 + 4 * q);
  }
  __syncthreads();  // xs + zeroed halos + depthwise weights

  f32x4_t* myhid = hidw + wave * 4 * PINP;
  const int64_t wes = static_cast<int64_t>(a.hid) * KP;            // we3 part stride
  const int64_t wps = static_cast<int64_t>(NOA * 32) * a.hid;      // wp3 part stride
  // the expand weights + bias of the NEXT subtile are in flight during this
  // subtile's depthwise + project (issued after its expand's last use of them)
  X3Frag ea[NK32];
  f32x4_t be4;
  auto load_ea = [&](int hs) {
#pragma unroll
    for (int c = 0; c < NK32; ++c)
      ea[c] = load_x3(a.we3, wes, static_cast<int64_t>(hs * 16 + li) * KP + 32 * c + 8 * g);
    be4 = *reinterpret_cast<const f32x4_t*>(a.be + hs * 16 + 4 * g);
  };
  int hs = sub0 + wave;
  if (hs < sub1) load_ea(hs);
  for (; hs < sub1; hs += NW) {
    const int ch8 = hs * 16 + 8 * h;  // this lane's 8 depthwise / project channels
    // project weights: in flight during the expand
    X3Frag pa[NOA];
#pragma unroll
    for (int o = 0; o < NO32; ++o) pa[o] = load_x3(a.wp3, wps, static_cast<int64_t>(o * 32 + l32) * a.hid + ch8);

    // ---- expand -> private hidden image (lane: pixel li, channels 4g .. 4g + 3)
#pragma unroll
    for (int j = 0; j < NBT; j += 2) {
      if (FULL || j < nbt) {
        const int j1 = j + 1 < NBT ? j + 1 : j;
        f32x4_t e0 = f32x4_t{0.f, 0.f, 0.f, 0.f}, e1 = e0;
#pragma unroll
        for (int c = 0; c < NK32; ++c) {
          const int k8 = 4 * c + g;
          const bf16x8_t* pl = xs + k8 * XSP;
          X3Frag b0, b1;
          const int c0 = (j * 16 + li) ^ (k8 & 15), c1 = (j1 * 16 + li) ^ (k8 & 15);
          b0.h = pl[c0];
          b0.m = pl[K8 * XSP + c0];
          b0.l = pl[2 * K8 * XSP + c0];
          b1.h = pl[c1];
          b1.m = pl[K8 * XSP + c1];
          b1.l = pl[2 * K8 * XSP + c1];
          e0 += mfma_x3(ea[c], b0);
          e1 += mfma_x3(ea[c], b1);
        }
        if constexpr (FULL) {
          const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
          myhid[g * PINP + j * 16 + li] = hcell[j] ? relu6x4(e0 + be4) : z;
          if (j + 1 < NBT) myhid[g * PINP + j1 * 16 + li] = hcell[j1] ? relu6x4(e1 + be4) : z;
        } else {
          myhid[g * PINP + hcell[j]] = relu6x4(e0 + be4);
          if (j + 1 < NBT) myhid[g * PINP + hcell[j1]] = relu6x4(e1 + be4);
        }
      }
    }
    if (hs + NW < sub1) load_ea(hs + NW);
    wave_sync();

    // ---- depthwise 3x3 + bias + ReLU6 (lane: pixel l32 of tile pt, 8 channels
    // in two halves of 4, the taps from LDS), split -> project
    f32x4_t dA[NP32], dB[NP32];
    const int cl = ch8 - ch0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4_t w[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) w[t] = wdl[(t * nch + cl) / 4 + half];
      const f32x4_t bd = wdl[(9 * nch + cl) / 4 + half];
#pragma unroll
      for (int pt = 0; pt < NP32; ++pt) {
        const f32x4_t* hp = myhid + (2 * h + half) * PINP + dcell[pt];
        f32x4_t d = bd;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) d = __builtin_elementwise_fma(hp[(ky * TIX + kx) * DIL], w[ky * 3 + kx], d);
        if (half == 0)
          dA[pt] = relu6x4(d);
        else
          dB[pt] = relu6x4(d);
      }
    }
#pragma unroll
    for (int pt = 0; pt < NP32; ++pt) {
      if constexpr (NOT == 0) {
        const int q = pt * 32 + l32;
        const int gy = oy0 + q / TX, gx = ox0 + q % TX;
        if (q < TY * TX && gy < a.Ho && gx < a.Wo) {
          float* yp = a.y + ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * a.hid + ch8;
          *reinterpret_cast<f32x4_t*>(yp) = dA[pt];
          *reinterpret_cast<f32x4_t*>(yp + 4) = dB[pt];
        }
        continue;
      }
      const X3Frag bf = split_x3(dA[pt], dB[pt]);
#pragma unroll
      for (int o = 0; o < NO32; ++o) acc[pt][o] += mfma32_x3(pa[o], bf);
    }
    wave_sync();  // this wave's hidden image is read out before the next subtile's expand
  }
  if constexpr (NOT == 0) return;

  // ---- cross-wave reduction (fixed order) + bias + residual -> NHWC
  // acc[pt][o] lane l: pixel pt * 32 + l32, output channels o * 32 + 8 qd + 4 h + r
  // (register 4 qd + r) -> red [wave][cout quad 2 qd + h][pixel]
  f32x4_t* red = reinterpret_cast<f32x4_t*>(smem);
  for (int o = 0; o < NO32; ++o) {
    __syncthreads();  // (o = 0: xs / hidden done; else the previous round's reads)
#pragma unroll
    for (int pt = 0; pt < NP32; ++pt)
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        red[(wave * 8 + 2 * qd + h) * NPX + pt * 32 + l32] =
            f32x4_t{acc[pt][o][4 * qd], acc[pt][o][4 * qd + 1], acc[pt][o][4 * qd + 2], acc[pt][o][4 * qd + 3]};
    __syncthreads();
    for (int v = tid; v < 8 * NPX; v += NT) {
      const int cq = v / NPX, q = v - cq * NPX;
      f32x4_t s = red[cq * NPX + q];
#pragma unroll
      for (int w = 1; w < NW; ++w) s += red[(w * 8 + cq) * NPX + q];
      const int co = o * 32 + 4 * cq;
      if (q >= TY * TX || co >= a.cout) continue;
      const int gy = oy0 + q / TX, gx = ox0 + q % TX;
      if (gy >= a.Ho || gx >= a.Wo) continue;
      const int64_t pix = (static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx;
      if (a.ws) {
        const int64_t plane = static_cast<int64_t>(a.B) * a.Ho * a.Wo * a.cout;
        if (a.tickets) {
          const __amdgpu_buffer_rsrc_t slab = __builtin_amdgcn_make_buffer_rsrc(
              a.ws, 0, static_cast<int>(nparts * plane * sizeof(float)), 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, s), slab,
                                                 static_cast<int>((part * plane + pix * a.cout + co) * 4), 0, 16);
        } else {
          *reinterpret_cast<f32x4_t*>(a.ws + part * plane + pix * a.cout + co) = s;
        }
        continue;
      }
      if (part == 0) {
        s += *reinterpret_cast<const f32x4_t*>(a.bp + co);
        if (a.residual) s += *reinterpret_cast<const f32x4_t*>(a.x + pix * a.cin + co);
      }
      float* yp = a.y + pix * a.cout + co;
      if (nparts > 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(yp + r, s[r]);
      } else {
        *reinterpret_cast<f32x4_t*>(yp) = s;
      }
    }
  }
  if (!a.ws || !a.tickets) return;
  irw_inlaunch_combine<TY, TX, NT>(a, smem, tile, part, nparts, b, oy0, ox0, tid);
}


// the x3 twins (irw_x3_kernel) of the configurations above: same tiles, waves
// and hidden parts, so workspace and tickets size the same way
#define NNSX_IRWX(S, TY, TX, KIN, NOT, NW, F)                                                   \
  IrwCfg {                                                                                      \
    S, TY, TX, KIN, NOT, NW, F, &irw_x3_kernel<S, TY, TX, KIN, NOT, NW, F>,                     \
        &IrwX3Geom<S, TY, TX, KIN, NOT, NW, F>::lds_bytes, 1                                    \
  }
const std::vector<IrwCfg> kIrwX3Cfgs = {
    NNSX_IRWX(2, 4, 8, 16, 2, 3, true),   NNSX_IRWX(1, 8, 8, 24, 2, 3, true),   NNSX_IRWX(2, 4, 4, 24, 2, 3, true),
    NNSX_IRWX(2, 7, 4, 24, 2, 3, true),   NNSX_IRWX(1, 7, 7, 32, 2, 4, false),  NNSX_IRWX(2, 2, 7, 32, 4, 4, false),
    NNSX_IRWX(1, 7, 7, 64, 4, 4, false),  NNSX_IRWX(1, 7, 7, 64, 6, 4, false),  NNSX_IRWX(1, 7, 7, 96, 6, 4, false),
    NNSX_IRWX(1, 7, 7, 160, 10, 4, false), NNSX_IRWX(2, 7, 7, 96, 10, 4, false), NNSX_IRWX(1, 7, 7, 160, 0, 4, false),
    NNSX_IRWX(1, 5, 5, 160, 10, 4, false), NNSX_IRWX(2, 5, 5, 96, 10, 4, false), NNSX_IRWX(1, 5, 5, 160, 0, 4, false),
    NNSX_IRWX(1, 5, 10, 32, 2, 4, false),
};
#undef NNSX_IRWX


}  // namespace

const std::vector<IrwCfg>& x3_irw_cfgs() { return kIrwX3Cfgs; }

}  // namespace kernels
}  // namespace nnsx
