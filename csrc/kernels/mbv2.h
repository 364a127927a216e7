// MobileNet-family CDNA4 kernels (bf16 NHWC).  See mbv2.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace nnsx {
namespace kernels {

// y[M][N] = act(x[M][K] . wt[N][K]^T + bias) (+ res), bf16 in, bf16/f32 out.
// wt is zero-padded to [ceil16(N)][Kpad], Kpad = ceil32(K).  act: 0 none, 1 relu6, 2 relu
// Npad: rows of wt (0 = ceil64(N)); large-M layers run the LDS-staged kernel
void pw_gemm(const void* x, const void* wt, const float* bias, const void* res, void* y, int M, int N, int K, int Kpad,
             int act, bool out_f32, hipStream_t s, int Npad = 0);
// depthwise 3x3, stride 1|2, dilation d (padding d); x [B][H][W][C], w [9][C], C % 8 == 0
void dw3x3(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int C, int stride, int dil,
           int act, hipStream_t s);
// 3x3/2 stem conv 3 -> 32 from an f32 NHWC frame; w f32 [3][3][3][32]
void stem3x3(const float* x, const float* w, const float* bias, void* y, int B, int H, int W, int act, hipStream_t s);
// same from the raw uint8 RGB frame, mapped in-kernel through lut[256] (device,
// f32: the upstream tensor_transform arithmetic folded into a table)
void stem3x3_u8(const uint8_t* x, const float* w, const float* bias, void* y, int B, int H, int W, int act,
                const float* lut, hipStream_t s);
// mean over HW: x [B][HW][C] -> y [B][C] (bf16)
void avgpool(const void* x, void* y, int B, int HW, int C, hipStream_t s);

// Fused inverted-residual block (ir_fused.hip): expand 1x1 + ReLU6 -> dw 3x3 +
// ReLU6 -> project 1x1 (+ residual), hidden activation kept in LDS.
//   we [hid][cin32] (K zero-padded), wd [9][hid], wp [ceil16(cout)][hid]
//   (rows zero-padded); biases fp32.  has_expand = 0: hidden == input (t=1).
struct IrBlockArgs {
  const uint16_t* x = nullptr;
  uint16_t* y = nullptr;
  const uint16_t* we = nullptr;
  const float* be = nullptr;
  const uint16_t* wd = nullptr;
  const float* bd = nullptr;
  const uint16_t* wp = nullptr;
  const float* bp = nullptr;
  int B = 0, H = 0, W = 0, cin = 0, hid = 0, cout = 0, stride = 1;
  int has_expand = 1, residual = 0;
  // derived by ir_block()
  int cin32 = 0, Ho = 0, Wo = 0, tiles_x = 0, tiles_y = 0, tiles_per_wg = 1;
};
bool ir_block_supported(int stride, int cin, int hid, int cout);
// returns false (nothing launched) for unsupported shapes
bool ir_block(const IrBlockArgs& a, hipStream_t s);

// ---------------------------------------------------------------- fp32 ----
// How the fp32 engine computes its GEMM-shaped products: kX3 = split-bf16 MFMAs
// (each operand = three bf16 parts, six cross products, fp32 sums; error vs an
// fp64 oracle below the native fp32 MFMA's), kNative = v_mfma_f32_16x16x4_f32.
// Default from NNSX_F32_MATH (x3 | fp32); x3 unless set.
enum class F32Math { kNative = 0, kX3 = 1 };
F32Math f32_math();
void set_f32_math(F32Math m);
const char* f32_math_name(F32Math m);
// The reference-precision engine (mbv2_f32.hip): fp32 activations, weights
// and accumulation, GEMMs on v_mfma_f32_16x16x4_f32.
// y[M][N] = act(x[M][K] . wt[N][K]^T + bias) (+ res); wt zero-padded [Npad][Kpad]
// (Kpad >= K, Kpad % 4 == 0), K % 4 == 0, N % 4 == 0.
// tile: 0 = auto, else BM * 1000 + BN of an instantiated tile (64064, 128064, 64128, 128128, 128192)
// Output layout of a GEMM writing into a slice of a concatenated tensor: rpb >
// 0 -> row m goes to y + (m / rpb) * bstride + (m % rpb) * ncols, and only the
// first ncols columns are stored (no split-K).  rpb = 0: plain y[M][N].
// brpb > 0: a per-batch bias -- bias is [M / brpb][N] and row m adds row
// m / brpb (a spatially constant branch folded into the GEMM; no split-K).
struct YLayout {
  int rpb = 0;
  int ncols = 0;
  int64_t bstride = 0;
  int brpb = 0;
  // pool > 0 (BN = 64 tiles, pool <= BM, no split-K / residual): y is [M / pool][N],
  // the mean over each image's `pool` rows of act(x . w + bias); the caller zeroes y
  // (an image spans at most two row tiles: two addends, so the sum is order-free)
  int pool = 0;
};
// The weights of an fp32 GEMM already split into their three bf16 parts
// (x3_split_weights), laid out the way a k-stage of the x3 GEMM stages them:
// [stages][rows][3 parts][32 k] bf16 -- a tile's rows of one stage are one
// contiguous block (192 B per row).  rows >= Npad, stages * 32 >= Kpad.  Given,
// the x3 GEMM stages them as they are (no per-tile split of the weight operand);
// absent (p null), it splits the fp32 weights per tile.
struct X3W {
  const uint16_t* p = nullptr;
  int stages = 0, rows = 0;
};
void pw_gemm_f32(const float* x, const float* wt, const float* bias, const float* res, float* y, int M, int N, int K,
                 int Kpad, int Npad, int act, hipStream_t s, int tile = 0, float* ws = nullptr,
                 const YLayout& yl = YLayout{}, X3W w3 = X3W{});
// fp32 weights [rows][cols] -> out [ceil(cols / 32)][x3_split_rows(rows)][3][32]
// bf16 (hi, mid, lo; zero past rows / cols): the X3W layout.  Rows are padded
// to a multiple of every tile width (64, 128, 192), so a tile's weight loads
// need no bounds checks.
int x3_split_rows(int rows);
void x3_split_weights(const float* w, int rows, int cols, uint16_t* out, hipStream_t s);
// Grouped launches (the SSD prediction heads): up to kGroupMax independent
// problems per launch.  pw_gemm_f32_group: 64 x 64 tiles, no split-K, no
// residual, any YLayout but pool.  dw3x3_f32_group: stride 1, dilation 1,
// y [B][H][W][C] (act as dw3x3_f32).
constexpr int kGroupMax = 16;
struct GemmProb {
  const float* x = nullptr;
  const float* wt = nullptr;
  const float* bias = nullptr;
  float* y = nullptr;
  int M = 0, N = 0, K = 0, Kpad = 0, Npad = 0, act = 0;
  YLayout yl;
  X3W w3;  // (the x3 launch stages pre-split weights only if every problem has them)
};
struct DwProb {
  const float* x = nullptr;
  const float* w = nullptr;
  const float* bias = nullptr;
  float* y = nullptr;
  int B = 0, H = 0, W = 0, C = 0, act = 0;
};
void pw_gemm_f32_group(const GemmProb* p, int n, hipStream_t s);
void dw3x3_f32_group(const DwProb* p, int n, hipStream_t s);
// SSDLite prediction heads, all in one launch (heads_f32.hip): per head y =
// pw(relu6(dw3x3(x) + bd)) + bias written into rows of a concatenated output.
struct SepHead {
  const float* x = nullptr;     // [B][H][W][K] feature map (f32 NHWC)
  const float* wd = nullptr;    // [9][K] depthwise weights (BN folded)
  const float* bd = nullptr;    // [K]
  const float* wt = nullptr;    // [Npad][Kpad] predictor weights
  const float* bias = nullptr;  // [>= N rounded to 4]
  float* out = nullptr;         // this head's first row in image 0 of the [B][T][C] output
  int64_t bstride = 0;          // floats between images in the output (T * C; NHWC: Ho * Wo * N)
  int B = 0, H = 0, W = 0, K = 0, Kpad = 0, N = 0, Npad = 0;  // N: outputs per pixel (anchors x C)
  int stride = 1;               // depthwise stride; wd == nullptr: no depthwise (plain 1x1)
  int dil = 1;                  // depthwise dilation (padding = dil)
  const float* res = nullptr;   // residual added before act (NHWC like the output)
  int act = 0;                  // 1: ReLU6 on the output
  int Ho = 0, Wo = 0;           // output map (0: from H, W, stride)
  int ldo = 0;                  // floats between output pixels (0: N)
  int tiles = 0;                // (set by the launcher)
};
constexpr int kSepHeadsMax = 16;
struct SepHeadsArgs {
  int n = 0;
  SepHead h[kSepHeadsMax];
};
// split-K workspace the GEMM wants for this shape (0: no split; without it the
// GEMM runs unsplit)
size_t pw_gemm_f32_workspace_bytes(int M, int N, int Kpad, bool has_res, int tile = 0);
// depthwise 3x3, stride 1|2, dilation d (padding d); w [9][C], C % 4 == 0
void dw3x3_f32(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int C, int stride,
               int dil, int act, hipStream_t s);
// 3x3/2 stem 3 -> 32, w [3][3][3][32]; fp32 output
void stem3x3_f32(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int act,
                 hipStream_t s);
void stem3x3_u8_f32(const uint8_t* x, const float* w, const float* bias, float* y, int B, int H, int W, int act,
                    const float* lut, hipStream_t s);
void avgpool_f32(const float* x, float* y, int B, int HW, int C, hipStream_t s);
// head 1x1 conv + act + global average pool in one launch (small batches):
// x [B][HW][K] -> y [B][N] = mean_p act(x[b][p] . wt^T + bias)
void pw_pool_f32(const float* x, const float* wt, const float* bias, float* y, int B, int HW, int N, int K, int Kpad,
                 int Npad, int act, hipStream_t s, X3W w3 = X3W{});

// fused inverted residual, fp32.  we [hid][KIN] (KIN = ceil8(cin), zero
// padded), wd [9][hid], wp [ceil16(cout)][hid] (rows zero padded); biases
// [hid] / [hid] / [ceil16(cout)].
struct IrBlockF32Args {
  const float* x = nullptr;
  float* y = nullptr;
  const float* we = nullptr;
  const float* be = nullptr;
  const float* wd = nullptr;
  const float* bd = nullptr;
  const float* wp = nullptr;
  const float* bp = nullptr;
  int B = 0, H = 0, W = 0, cin = 0, hid = 0, cout = 0, stride = 1;
  int has_expand = 1, residual = 0;
  int dil = 1;  // depthwise dilation (padding = dil)
  // derived by ir_block_f32()
  int Ho = 0, Wo = 0, tiles_x = 0, tiles_y = 0;
  int hsplit = 1;  // hidden-channel parts per tile (wave-split kernel)
  float* ws = nullptr;  // partial-sum workspace (ir_block_f32_workspace_bytes; small batches)
  // per-tile tickets (ir_block_f32_tickets entries, zeroed once at creation):
  // the hidden parts are added inside the launch instead of by a separate
  // reduce kernel (spread form below by default; NNSX_F32_IRW_INLAUNCH=1: the
  // last part of a tile to finish adds all slabs)
  int* tickets = nullptr;
  // spread = 1: every part of a tile waits at a per-tile arrival counter (64-bit,
  // monotone: tickets[] read as uint64) and then adds its 1/parts share of the
  // tile's outputs from all slabs -- the combine spread over the parts, not left
  // to the last one.  Only launched when every workgroup of the grid is resident
  // at once (the host checks occupancy); the wait is bounded.
  int spread = 0;
  // split-bf16 weights (F32Math::kX3): we3 [3][hid][ceil32(cin)], wp3
  // [3][ceil32(cout)][hid] bf16 (hi, mid, lo parts; zero padded).  Both set and
  // the method x3: the irw_x3 kernel of the same geometry, when there is one
  const uint16_t* we3 = nullptr;
  const uint16_t* wp3 = nullptr;
  int irp_order = 2;  // irpp_x3 phase order (kernels/irp_x3.hip)
};
// Launches enqueued by this thread while a SharedDeviceScope is alive may run
// concurrently with other kernels of the same process (a filter's replay
// lanes), including other launches of the same model: no in-launch combine of
// hidden parts -- the spread form would wait for a residency nothing
// guarantees, and both forms count arrivals in the model's one ticket buffer,
// which concurrent replays of a block would share.  Graph capture bakes the
// choice into the captured kernels.
struct SharedDeviceScope {
  explicit SharedDeviceScope(bool on);
  ~SharedDeviceScope();
  SharedDeviceScope(const SharedDeviceScope&) = delete;
  SharedDeviceScope& operator=(const SharedDeviceScope&) = delete;

 private:
  bool prev_;
};
bool device_shared();
// set this thread's flag directly (tests); returns the previous value
bool set_device_shared(bool on);

bool ir_block_f32_supported(int stride, int H, int W, int cin, int hid, int cout, bool has_expand, int dil = 1,
                            int B = 0);
// device workspace ir_block_f32 needs for these args (0 = none)
size_t ir_block_f32_workspace_bytes(const IrBlockF32Args& a);
// int tickets (zeroed) the in-launch combine of hidden parts wants (0: none)
size_t ir_block_f32_tickets(const IrBlockF32Args& a);
// expand 1x1 + ReLU6 + depthwise 3x3 + ReLU6 in one kernel, the depthwise
// output to y [B][Ho][Wo][hid] (the hidden map never touches HBM; the caller
// runs the project as a GEMM).  wp / bp / cout / residual are unused.
// (B > 0: whether it is the faster path at this batch; B = 0: supported at all)
bool ir_expand_dw_f32_supported(int stride, int H, int W, int cin, int hid, int B = 0, int dil = 1);
bool ir_expand_dw_f32(const IrBlockF32Args& a, hipStream_t s);

// stem (3x3/2 conv 3 -> 32 on the uint8 frame, mapped through lut[256],
// + ReLU6) fused with an expand-free inverted residual 32 -> 32 -> 16
// (dw 3x3 + ReLU6, project).  ws [3][3][3][32], bs [32], wd [9][32], bd [32],
// wp [16][32], bp [16]; y [B][Ho][Wo][16], Ho = (H-1)/2+1.
struct StemIr1F32Args {
  const uint8_t* x = nullptr;
  float* y = nullptr;
  const float* ws = nullptr;
  const float* bs = nullptr;
  const float* wd = nullptr;
  const float* bd = nullptr;
  const float* wp = nullptr;
  const float* bp = nullptr;
  int B = 0, H = 0, W = 0;
  const float* lut = nullptr;  // [256] f32, device
  int mode = -1;               // (unused: one kernel)
  // derived
  int Ho = 0, Wo = 0, tiles_x = 0, tiles_y = 0;
};
bool stem_ir1_f32(const StemIr1F32Args& a, hipStream_t s);
bool ir_block_f32(const IrBlockF32Args& a, hipStream_t s);
// which product method ir_block_f32 uses for this shape under the current
// F32Math with x3 weights given: "x3", "fp32", or "" (unsupported)
const char* ir_block_f32_method(int stride, int H, int W, int cin, int hid, int cout, int B, int dil = 1);
// the 14 x 14 image-per-workgroup kernels' smallest batch (kernels/irp_x3.hip); returns the old value
int irp_x3_set_min_batch(int b);
// the 28 x 28 half-image kernels (kernels/irp_x3.hip): 0 off, 1 stride 2, 2 both; returns the old mode
int irh_set_mode(int m);

}  // namespace kernels
}  // namespace nnsx
