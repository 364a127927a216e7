// torch.ops.nnsx.* -- the CDNA4 kernels exposed as PyTorch operators so that
// TorchScript models (loaded by tensor_filter framework=pytorch) run them,
// and hipGraph capture records them like any other kernel.  CPU
// implementations are the fp32 numerics reference.
#include <algorithm>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "kernels/mbv2.h"
#include "kernels/vision.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

at::Tensor act_ref(at::Tensor v, int64_t act) {
  if (act == 1) return v.clamp(0, 6);
  if (act == 2) return v.clamp_min(0);
  return v;
}

// ------------------------------------------------- pre-split x3 weights ----
// The x3 GEMMs stage weights that are already split into their bf16 parts
// (kernels::X3W): each fp32 weight matrix is split once, at its first GEMM
// outside a graph capture (tensor_filter runs a model eagerly before it
// captures), and kept with a reference to the weights -- so the address cannot
// be reused by another tensor while cached -- and the weights' version, so an
// in-place update is split again.  Entries whose weights nobody else holds any
// more (an unloaded model) are dropped at the next miss.
struct X3Cached {
  at::Tensor src, parts;
  int64_t version = -1;
  nnsx::kernels::X3W w3;
};
std::mutex g_x3_mu;
std::unordered_map<const void*, X3Cached> g_x3;
bool g_x3_cache_on = true;
// parts of replaced / evicted entries: a graph captured on a cache hit baked
// in their address, so they stay alive until the graphs are cleared
// (tensor_filter's clear_graphs -> x3_retire_flush; bounded for direct users)
std::deque<at::Tensor> g_x3_retired;
void x3_retire(at::Tensor parts) {
  g_x3_retired.push_back(std::move(parts));
  while (g_x3_retired.size() > 256) g_x3_retired.pop_front();
}

// tests: off = every x3 GEMM splits its weights per tile (the capture fallback)
bool x3_weight_cache(bool on) {
  std::lock_guard<std::mutex> lk(g_x3_mu);
  const bool prev = g_x3_cache_on;
  g_x3_cache_on = on;
  if (!on) g_x3.clear();
  return prev;
}

nnsx::kernels::X3W x3_weights(const at::Tensor& wt) {
  if (nnsx::kernels::f32_math() != nnsx::kernels::F32Math::kX3 || !wt.is_cuda() || wt.scalar_type() != at::kFloat ||
      wt.dim() != 2 || !wt.is_contiguous() || wt.numel() == 0)
    return {};
  std::lock_guard<std::mutex> lk(g_x3_mu);
  if (!g_x3_cache_on) return {};
  auto it = g_x3.find(wt.data_ptr());
  if (it != g_x3.end() && it->second.src.sizes() == wt.sizes() && it->second.src.device() == wt.device() &&
      it->second.version == wt._version())
    return it->second.w3;
  hipStream_t s = cur_stream();
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return {};  // (per-tile split)
  if (it != g_x3.end()) {  // (in-place updated weights: their old parts)
    x3_retire(std::move(it->second.parts));
    g_x3.erase(it);
  }
  for (auto e = g_x3.begin(); e != g_x3.end();) {
    if (e->second.src.use_count() == 1) {
      x3_retire(std::move(e->second.parts));
      e = g_x3.erase(e);
    } else {
      ++e;
    }
  }
  const int64_t rows = wt.size(0), cols = wt.size(1), stages = (cols + 31) / 32;
  X3Cached c;
  c.src = wt;
  c.version = wt._version();
  const int64_t rows3 = nnsx::kernels::x3_split_rows(static_cast<int>(rows));
  c.parts = at::empty({stages, rows3, 3, 32}, wt.options().dtype(at::kBFloat16));
  nnsx::kernels::x3_split_weights(wt.data_ptr<float>(), static_cast<int>(rows), static_cast<int>(cols),
                                  reinterpret_cast<uint16_t*>(c.parts.data_ptr()), s);
  // other streams (replay lanes) read the parts later: done before first use
  TORCH_CHECK(hipStreamSynchronize(s) == hipSuccess, "x3 weight split");
  c.w3.p = reinterpret_cast<const uint16_t*>(c.parts.data_ptr());
  c.w3.stages = static_cast<int>(stages);
  c.w3.rows = static_cast<int>(rows3);
  const nnsx::kernels::X3W w3 = c.w3;
  g_x3[wt.data_ptr()] = std::move(c);
  return w3;
}

// ------------------------------------------------------------ pw_conv ----
at::Tensor pw_conv_f32_cuda(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias,
                            const c10::optional<at::Tensor>& res, int64_t N, int64_t act, int64_t tile = 0) {
  TORCH_CHECK(x.is_contiguous(), "pw_conv(f32): x must be contiguous");
  TORCH_CHECK(wt.scalar_type() == at::kFloat && wt.is_contiguous() && wt.dim() == 2, "pw_conv(f32): wt [Npad,Kpad] f32");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() >= N, "pw_conv(f32): bias f32 [N]");
  const int64_t K = x.size(-1);
  const int64_t M = x.numel() / K;
  const int64_t Kpad = wt.size(1), Npad = wt.size(0);
  TORCH_CHECK(K % 4 == 0 && N % 4 == 0 && Kpad % 4 == 0 && Kpad >= K && Npad >= N,
              "pw_conv(f32): shape constraints (K%4, N%4, Kpad%4, Kpad >= K, Npad >= N)");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  at::Tensor y = at::empty(sizes, x.options());
  const float* r = nullptr;
  if (res.has_value() && res->defined()) {
    TORCH_CHECK(res->scalar_type() == at::kFloat && res->is_contiguous() && res->numel() == M * N, "pw_conv(f32): residual");
    r = res->data_ptr<float>();
  }
  const size_t wsb = nnsx::kernels::pw_gemm_f32_workspace_bytes(static_cast<int>(M), static_cast<int>(N),
                                                                 static_cast<int>(Kpad), r != nullptr, static_cast<int>(tile));
  at::Tensor ws;
  if (wsb) ws = at::empty({static_cast<int64_t>(wsb / sizeof(float))}, x.options());
  nnsx::kernels::pw_gemm_f32(x.data_ptr<float>(), wt.data_ptr<float>(), bias.data_ptr<float>(), r, y.data_ptr<float>(),
                             static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), static_cast<int>(Kpad),
                             static_cast<int>(Npad), static_cast<int>(act), cur_stream(), static_cast<int>(tile),
                             wsb ? ws.data_ptr<float>() : nullptr, nnsx::kernels::YLayout{}, x3_weights(wt));
  return y;
}

// benchmarking entry: the fp32 GEMM with an explicit tile (BM * 1000 + BN, 0 = auto)
at::Tensor pw_conv_f32_tile_cuda(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias,
                                 const c10::optional<at::Tensor>& res, int64_t N, int64_t act, int64_t tile) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat, "pw_conv_f32_tile: x must be a f32 cuda tensor");
  return pw_conv_f32_cuda(x, wt, bias, res, N, act, tile);
}

at::Tensor pw_conv_cuda(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias,
                        const c10::optional<at::Tensor>& res, int64_t N, int64_t act, bool out_f32) {
  TORCH_CHECK(x.is_cuda(), "pw_conv: x must be a cuda tensor");
  if (x.scalar_type() == at::kFloat) return pw_conv_f32_cuda(x, wt, bias, res, N, act);
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "pw_conv: x must be contiguous bf16 cuda");
  TORCH_CHECK(wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() && wt.dim() == 2, "pw_conv: wt [Npad,Kpad] bf16");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() >= N, "pw_conv: bias f32 [N]");
  const int64_t K = x.size(-1);
  const int64_t M = x.numel() / K;
  const int64_t Kpad = wt.size(1);
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0 && Kpad % 32 == 0 && Kpad >= K && wt.size(0) >= ((N + 63) / 64) * 64,
              "pw_conv: shape constraints (K%8, N%8, Kpad%32, wt rows padded to 64)");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  at::Tensor y = at::empty(sizes, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  const void* r = nullptr;
  if (res.has_value() && res->defined()) {
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->is_contiguous() && res->numel() == M * N, "pw_conv: residual");
    r = res->data_ptr();
  }
  nnsx::kernels::pw_gemm(x.data_ptr(), wt.data_ptr(), bias.data_ptr<float>(), r, y.data_ptr(), static_cast<int>(M),
                         static_cast<int>(N), static_cast<int>(K), static_cast<int>(Kpad), static_cast<int>(act), out_f32,
                         cur_stream(), static_cast<int>(wt.size(0)));
  return y;
}

at::Tensor pw_conv_cpu(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias,
                       const c10::optional<at::Tensor>& res, int64_t N, int64_t act, bool out_f32) {
  const int64_t K = x.size(-1);
  at::Tensor w = wt.slice(0, 0, N).slice(1, 0, K).to(at::kFloat);
  at::Tensor v = at::matmul(x.to(at::kFloat), w.t()) + bias.slice(0, 0, N);
  if (res.has_value() && res->defined()) v = v + res->to(at::kFloat);
  v = act_ref(v, act);
  return v.to(out_f32 || x.scalar_type() == at::kFloat ? at::kFloat : at::kBFloat16);
}

// pw_conv whose output goes straight into a slice of a concatenated tensor:
// out [B, T, C]; the GEMM of x [B, H, W, K] writes rows row0 .. row0 + H*W*n/C
// of every batch (n = the real output width, a multiple of C).  Replaces a
// per-head output + torch.cat (the SSD heads).
void pw_conv_into_cuda(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias, at::Tensor& out,
                       int64_t row0, int64_t n, int64_t act) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
              "pw_conv_into: x [B,H,W,K] f32 contiguous");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 3,
              "pw_conv_into: out [B,T,C] f32 contiguous");
  const int64_t B = x.size(0), HW = x.size(1) * x.size(2), K = x.size(3), C = out.size(2), T = out.size(1);
  const int64_t N = (n + 3) / 4 * 4, Kpad = wt.size(1), Npad = wt.size(0);
  TORCH_CHECK(out.size(0) == B && n % C == 0 && row0 + HW * (n / C) <= T, "pw_conv_into: slice out of range");
  TORCH_CHECK(K % 4 == 0 && Kpad >= K && Npad >= N && bias.numel() >= N && wt.scalar_type() == at::kFloat,
              "pw_conv_into: weights");
  nnsx::kernels::YLayout yl;
  yl.rpb = static_cast<int>(HW);
  yl.ncols = static_cast<int>(n);
  yl.bstride = T * C;
  nnsx::kernels::pw_gemm_f32(x.data_ptr<float>(), wt.data_ptr<float>(), bias.data_ptr<float>(), nullptr,
                             out.data_ptr<float>() + row0 * C, static_cast<int>(B * HW), static_cast<int>(N),
                             static_cast<int>(K), static_cast<int>(Kpad), static_cast<int>(Npad), static_cast<int>(act),
                             cur_stream(), 0, nullptr, yl, x3_weights(wt));
}

void pw_conv_into_cpu(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias, at::Tensor& out,
                      int64_t row0, int64_t n, int64_t act) {
  at::Tensor y = pw_conv_cpu(x, wt, bias, c10::nullopt, (n + 3) / 4 * 4, act, true).slice(-1, 0, n);
  const int64_t B = x.size(0), C = out.size(2);
  y = y.reshape({B, -1, C});
  out.slice(1, row0, row0 + y.size(1)).copy_(y);
}

at::Tensor dw_conv_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t stride, int64_t act,
                       int64_t dilation);

// All SSDLite heads in one launch (kernels::sep_heads_f32): head i reads
// feature xs[i] through its depthwise (wds[i], bds[i]) and predictor (wts[i],
// biases[i], ns[i] outputs per pixel) into out_box (which[i] == 0) or out_cls
// (1), its rows following the previous head's of the same output.
// mode 0: two grouped launches -- every head's depthwise into a scratch map
// (kernels::dw3x3_f32_group), then every predictor GEMM
// (kernels::pw_gemm_f32_group).  (The one-launch form with the depthwise in
// the GEMM's operand staging measured slower and was removed:
// profiles/r4_dwpw_ab.txt.)
void sep_heads_cuda(at::TensorList xs, at::TensorList wds, at::TensorList bds, at::TensorList wts,
                    at::TensorList biases, at::IntArrayRef ns, at::IntArrayRef which, at::Tensor& out_box,
                    at::Tensor& out_cls, int64_t mode) {
  const size_t n = xs.size();
  TORCH_CHECK(n > 0 && n <= static_cast<size_t>(nnsx::kernels::kSepHeadsMax) && wds.size() == n && bds.size() == n &&
                  wts.size() == n && biases.size() == n && ns.size() == n && which.size() == n,
              "sep_heads: 1..16 heads, one entry of every list per head");
  nnsx::kernels::SepHeadsArgs a;
  a.n = static_cast<int>(n);
  int64_t rows[2] = {0, 0};
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor& x = xs[i];
    at::Tensor& o = which[i] ? out_cls : out_box;
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
                "sep_heads: x [B,H,W,K] f32 contiguous");
    TORCH_CHECK(o.is_cuda() && o.scalar_type() == at::kFloat && o.is_contiguous() && o.dim() == 3 && o.size(0) == x.size(0),
                "sep_heads: outputs [B,T,C] f32");
    const int64_t K = x.size(3), C = o.size(2), N = ns[i];
    TORCH_CHECK(N % C == 0 && wds[i].numel() == 9 * K && bds[i].numel() >= K && wts[i].dim() == 2 &&
                    wts[i].size(1) >= K && wts[i].size(0) >= (N + 3) / 4 * 4 && biases[i].numel() >= (N + 3) / 4 * 4,
                "sep_heads: weights");
    const int64_t HW = x.size(1) * x.size(2);
    const int64_t r0 = rows[which[i] ? 1 : 0];
    TORCH_CHECK(r0 + HW * (N / C) <= o.size(1), "sep_heads: output rows");
    auto& h = a.h[i];
    h.x = x.data_ptr<float>();
    h.wd = wds[i].data_ptr<float>();
    h.bd = bds[i].data_ptr<float>();
    h.wt = wts[i].data_ptr<float>();
    h.bias = biases[i].data_ptr<float>();
    h.out = o.data_ptr<float>() + r0 * C;
    h.bstride = o.size(1) * C;
    h.B = static_cast<int>(x.size(0));
    h.H = static_cast<int>(x.size(1));
    h.W = static_cast<int>(x.size(2));
    h.K = static_cast<int>(K);
    h.Kpad = static_cast<int>(wts[i].size(1));
    h.N = static_cast<int>(N);
    h.Npad = static_cast<int>(wts[i].size(0));
    rows[which[i] ? 1 : 0] = r0 + HW * (N / C);
  }
  TORCH_CHECK(mode == 0, "sep_heads: mode 0 (grouped depthwise + grouped GEMM)");
  int64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += xs[i].numel();
  at::Tensor hid = at::empty({total}, xs[0].options());
  // the largest maps first: their blocks start first, the small maps fill the tail
  std::vector<size_t> order(n);
  for (size_t i = 0; i < n; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t p, size_t q) {
    const auto& hp = a.h[p];
    const auto& hq = a.h[q];
    return static_cast<int64_t>(hp.B) * hp.H * hp.W * hp.Kpad > static_cast<int64_t>(hq.B) * hq.H * hq.W * hq.Kpad;
  });
  nnsx::kernels::DwProb dp[nnsx::kernels::kGroupMax];
  nnsx::kernels::GemmProb gp[nnsx::kernels::kGroupMax];
  int64_t off = 0;
  for (size_t j = 0; j < n; ++j) {
    const auto& h = a.h[order[j]];
    float* hb = hid.data_ptr<float>() + off;
    off += static_cast<int64_t>(h.B) * h.H * h.W * h.K;
    dp[j].x = h.x;
    dp[j].w = h.wd;
    dp[j].bias = h.bd;
    dp[j].y = hb;
    dp[j].B = h.B;
    dp[j].H = h.H;
    dp[j].W = h.W;
    dp[j].C = h.K;
    dp[j].act = 1;
    auto& g = gp[j];
    g.x = hb;
    g.wt = h.wt;
    g.bias = h.bias;
    g.y = h.out;
    g.M = h.B * h.H * h.W;
    g.N = (h.N + 3) / 4 * 4;
    g.K = h.K;
    g.Kpad = h.Kpad;
    g.Npad = h.Npad;
    g.act = 0;
    g.yl.rpb = h.H * h.W;
    g.yl.ncols = h.N;
    g.yl.bstride = h.bstride;
    g.w3 = x3_weights(wts[order[j]]);
  }
  nnsx::kernels::dw3x3_f32_group(dp, static_cast<int>(n), cur_stream());
  nnsx::kernels::pw_gemm_f32_group(gp, static_cast<int>(n), cur_stream());
}

// Several pointwise convs in one grouped launch (kernels::pw_gemm_f32_group):
// out[i] = act_i(xs[i] . wts[i]^T + biases[i]), NHWC [B, H, W, ns[i]] with
// exact columns (the PoseNet heatmap + offset heads).
std::vector<at::Tensor> pw_conv_group_cuda(at::TensorList xs, at::TensorList wts, at::TensorList biases,
                                           at::IntArrayRef ns, at::IntArrayRef acts) {
  const size_t n = xs.size();
  TORCH_CHECK(n > 0 && n <= static_cast<size_t>(nnsx::kernels::kGroupMax) && wts.size() == n && biases.size() == n &&
                  ns.size() == n && acts.size() == n,
              "pw_conv_group: 1..16 problems, one entry of every list per problem");
  nnsx::kernels::GemmProb gp[nnsx::kernels::kGroupMax];
  std::vector<at::Tensor> outs;
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor& x = xs[i];
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
                "pw_conv_group: x [B,H,W,K] f32 contiguous");
    const int64_t K = x.size(3), M = x.numel() / K, N = ns[i], N4 = (N + 3) / 4 * 4;
    TORCH_CHECK(K % 4 == 0 && wts[i].scalar_type() == at::kFloat && wts[i].is_contiguous() && wts[i].dim() == 2 &&
                    wts[i].size(1) >= K && wts[i].size(0) >= N4 && biases[i].numel() >= N4 && acts[i] >= 0 &&
                    acts[i] <= 1 && M > 0 && M < (1 << 30),
                "pw_conv_group: weights [Npad >= N rounded to 4][Kpad >= K], bias, act 0|1");
    at::Tensor y = at::empty({x.size(0), x.size(1), x.size(2), N}, x.options());
    auto& g = gp[i];
    g.x = x.data_ptr<float>();
    g.wt = wts[i].data_ptr<float>();
    g.bias = biases[i].data_ptr<float>();
    g.y = y.data_ptr<float>();
    g.M = static_cast<int>(M);
    g.N = static_cast<int>(N4);
    g.K = static_cast<int>(K);
    g.Kpad = static_cast<int>(wts[i].size(1));
    g.Npad = static_cast<int>(wts[i].size(0));
    g.act = static_cast<int>(acts[i]);
    g.yl.rpb = static_cast<int>(M);  // one "batch" of M rows, N exact columns each
    g.yl.ncols = static_cast<int>(N);
    g.yl.bstride = 0;
    g.w3 = x3_weights(wts[i]);
    outs.push_back(y);
  }
  nnsx::kernels::pw_gemm_f32_group(gp, static_cast<int>(n), cur_stream());
  return outs;
}

std::vector<at::Tensor> pw_conv_group_cpu(at::TensorList xs, at::TensorList wts, at::TensorList biases,
                                          at::IntArrayRef ns, at::IntArrayRef acts) {
  std::vector<at::Tensor> outs;
  for (size_t i = 0; i < xs.size(); ++i)
    outs.push_back(pw_conv_cpu(xs[i], wts[i], biases[i], c10::nullopt, (ns[i] + 3) / 4 * 4, acts[i], true)
                       .slice(-1, 0, ns[i])
                       .contiguous());
  return outs;
}

void sep_heads_cpu(at::TensorList xs, at::TensorList wds, at::TensorList bds, at::TensorList wts, at::TensorList biases,
                   at::IntArrayRef ns, at::IntArrayRef which, at::Tensor& out_box, at::Tensor& out_cls, int64_t) {
  int64_t rows[2] = {0, 0};
  for (size_t i = 0; i < xs.size(); ++i) {
    at::Tensor& o = which[i] ? out_cls : out_box;
    at::Tensor h = dw_conv_cpu(xs[i], wds[i], bds[i], 1, 1, 1);
    const int64_t N = ns[i], B = h.size(0), C = o.size(2);
    at::Tensor y = pw_conv_cpu(h, wts[i], biases[i], c10::nullopt, (N + 3) / 4 * 4, 0, true).slice(-1, 0, N);
    y = y.reshape({B, -1, C});
    const int64_t r0 = rows[which[i] ? 1 : 0];
    o.slice(1, r0, r0 + y.size(1)).copy_(y);
    rows[which[i] ? 1 : 0] = r0 + y.size(1);
  }
}


// pw_conv with a per-image bias: bias [B, N] (row b of it for every pixel of
// image b).  project(cat[a, p]) with p constant over space (DeepLab's image
// pooling branch) is W_a . a + (W_p . p + b): one GEMM on a, no concat.
at::Tensor pw_conv_rowbias_cuda(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias, int64_t N,
                                int64_t act) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
              "pw_conv_rowbias: x [B,H,W,K] f32 contiguous");
  const int64_t B = x.size(0), HW = x.size(1) * x.size(2), K = x.size(3);
  const int64_t Kpad = wt.size(1), Npad = wt.size(0);
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.is_contiguous() && bias.numel() == B * N,
              "pw_conv_rowbias: bias [B,N] f32");
  TORCH_CHECK(K % 4 == 0 && N % 4 == 0 && Kpad >= K && Npad >= N && wt.scalar_type() == at::kFloat,
              "pw_conv_rowbias: weights");
  at::Tensor y = at::empty({B, x.size(1), x.size(2), N}, x.options());
  nnsx::kernels::YLayout yl;
  yl.brpb = static_cast<int>(HW);
  nnsx::kernels::pw_gemm_f32(x.data_ptr<float>(), wt.data_ptr<float>(), bias.data_ptr<float>(), nullptr,
                             y.data_ptr<float>(), static_cast<int>(B * HW), static_cast<int>(N), static_cast<int>(K),
                             static_cast<int>(Kpad), static_cast<int>(Npad), static_cast<int>(act), cur_stream(), 0,
                             nullptr, yl, x3_weights(wt));
  return y;
}

at::Tensor pw_conv_rowbias_cpu(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias, int64_t N,
                               int64_t act) {
  const int64_t K = x.size(-1), B = x.size(0);
  at::Tensor w = wt.slice(0, 0, N).slice(1, 0, K).to(at::kFloat);
  at::Tensor v = at::matmul(x.to(at::kFloat), w.t()) + bias.reshape({B, 1, 1, N});
  return act_ref(v, act);
}

// NHWC bilinear resize with align_corners (F.interpolate(..., "bilinear",
// align_corners=True) on channels-last data, without the permutes)
at::Tensor upsample_bilinear_cuda(const at::Tensor& x, int64_t H, int64_t W) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
              "upsample_bilinear: x [B,h,w,C] f32 contiguous");
  TORCH_CHECK(H > 0 && W > 0 && W * x.size(3) < (int64_t{1} << 31), "upsample_bilinear: size");
  at::Tensor y = at::empty({x.size(0), H, W, x.size(3)}, x.options());
  nnsx::kernels::upsample_bilinear_nhwc(x.data_ptr<float>(), static_cast<int>(x.size(0)), static_cast<int>(x.size(1)),
                                        static_cast<int>(x.size(2)), static_cast<int>(x.size(3)), static_cast<int>(H),
                                        static_cast<int>(W), y.data_ptr<float>(), cur_stream());
  return y;
}

at::Tensor upsample_bilinear_cpu(const at::Tensor& x, int64_t H, int64_t W) {
  at::Tensor v = at::upsample_bilinear2d(x.permute({0, 3, 1, 2}), {H, W}, true);
  return v.permute({0, 2, 3, 1}).contiguous();
}

// ------------------------------------------------------------ dw_conv ----
at::Tensor dw_conv_cuda(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t stride, int64_t act,
                        int64_t dilation) {
  if (x.scalar_type() == at::kFloat) {
    TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "dw_conv(f32): x [B,H,W,C] f32");
    const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
    TORCH_CHECK(C % 4 == 0 && w.numel() == 9 * C && w.scalar_type() == at::kFloat && w.is_contiguous(),
                "dw_conv(f32): w [9,C] f32, C%4==0");
    const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
    at::Tensor y = at::empty({B, Ho, Wo, C}, x.options());
    nnsx::kernels::dw3x3_f32(x.data_ptr<float>(), w.data_ptr<float>(), bias.data_ptr<float>(), y.data_ptr<float>(),
                             static_cast<int>(B), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                             static_cast<int>(stride), static_cast<int>(dilation), static_cast<int>(act), cur_stream());
    return y;
  }
  TORCH_CHECK(act < 2, "dw_conv: the deferred input activation (act bit 1) is fp32 only");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 4, "dw_conv: x [B,H,W,C] bf16");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && w.numel() == 9 * C && w.scalar_type() == at::kBFloat16, "dw_conv: w [9,C] bf16, C%8==0");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  at::Tensor y = at::empty({B, Ho, Wo, C}, x.options());
  nnsx::kernels::dw3x3(x.data_ptr(), w.data_ptr(), bias.data_ptr<float>(), y.data_ptr(), static_cast<int>(B),
                       static_cast<int>(H), static_cast<int>(W), static_cast<int>(C), static_cast<int>(stride),
                       static_cast<int>(dilation), static_cast<int>(act), cur_stream());
  return y;
}

at::Tensor dw_conv_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t stride, int64_t act,
                       int64_t dilation) {
  const int64_t C = x.size(3);
  at::Tensor xf = x.to(at::kFloat).permute({0, 3, 1, 2});
  if (act & 2) xf = xf.clamp(0, 6);  // deferred input ReLU6
  act &= 1;
  at::Tensor wf = w.to(at::kFloat).view({3, 3, C}).permute({2, 0, 1}).unsqueeze(1).contiguous();
  at::Tensor v = at::conv2d(xf, wf, bias, {stride, stride}, {dilation, dilation}, {dilation, dilation}, C);
  return act_ref(v, act).permute({0, 2, 3, 1}).contiguous().to(x.scalar_type() == at::kFloat ? at::kFloat : at::kBFloat16);
}

// --------------------------------------------------------------- stem ----
at::Tensor stem_conv_cuda(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t act, bool out_f32) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3,
              "stem_conv: x [B,H,W,3] f32");
  TORCH_CHECK(w.numel() == 27 * 32 && w.scalar_type() == at::kFloat, "stem_conv: w [3,3,3,32] f32");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  at::Tensor y = at::empty({B, Ho, Wo, 32}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  if (out_f32) {
    nnsx::kernels::stem3x3_f32(x.data_ptr<float>(), w.data_ptr<float>(), bias.data_ptr<float>(), y.data_ptr<float>(),
                               static_cast<int>(B), static_cast<int>(H), static_cast<int>(W), static_cast<int>(act),
                               cur_stream());
    return y;
  }
  nnsx::kernels::stem3x3(x.data_ptr<float>(), w.data_ptr<float>(), bias.data_ptr<float>(), y.data_ptr(),
                         static_cast<int>(B), static_cast<int>(H), static_cast<int>(W), static_cast<int>(act), cur_stream());
  return y;
}

at::Tensor stem_conv_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t act, bool out_f32) {
  at::Tensor xf = x.to(at::kFloat).permute({0, 3, 1, 2});
  at::Tensor wf = w.view({3, 3, 3, 32}).permute({3, 2, 0, 1}).contiguous();
  at::Tensor v = at::conv2d(xf, wf, bias, {2, 2}, {1, 1});
  return act_ref(v, act).permute({0, 2, 3, 1}).contiguous().to(out_f32 ? at::kFloat : at::kBFloat16);
}

at::Tensor stem_conv_u8_cuda(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t act,
                             const at::Tensor& lut, bool out_f32) {
  TORCH_CHECK(lut.is_cuda() && lut.scalar_type() == at::kFloat && lut.numel() == 256 && lut.is_contiguous(),
              "stem_conv_u8: lut [256] f32 on the device");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kByte && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3,
              "stem_conv_u8: x [B,H,W,3] uint8");
  TORCH_CHECK(w.numel() == 27 * 32 && w.scalar_type() == at::kFloat, "stem_conv_u8: w [3,3,3,32] f32");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  at::Tensor y = at::empty({B, Ho, Wo, 32}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  if (out_f32) {
    nnsx::kernels::stem3x3_u8_f32(x.data_ptr<uint8_t>(), w.data_ptr<float>(), bias.data_ptr<float>(),
                                  y.data_ptr<float>(), static_cast<int>(B), static_cast<int>(H), static_cast<int>(W),
                                  static_cast<int>(act), lut.data_ptr<float>(), cur_stream());
    return y;
  }
  nnsx::kernels::stem3x3_u8(x.data_ptr<uint8_t>(), w.data_ptr<float>(), bias.data_ptr<float>(), y.data_ptr(),
                            static_cast<int>(B), static_cast<int>(H), static_cast<int>(W), static_cast<int>(act),
                            lut.data_ptr<float>(), cur_stream());
  return y;
}

at::Tensor stem_conv_u8_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t act,
                            const at::Tensor& lut, bool out_f32) {
  at::Tensor xf = lut.to(at::kFloat).index_select(0, x.to(at::kLong).flatten()).view(x.sizes());
  return stem_conv_cpu(xf, w, bias, act, out_f32);
}

// ------------------------------------------------------------ avgpool ----
at::Tensor avgpool_cuda(const at::Tensor& x) {
  if (x.scalar_type() == at::kFloat) {
    TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4 && x.size(3) % 4 == 0, "avgpool(f32): x [B,H,W,C%4]");
    const int64_t B = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
    at::Tensor y = at::empty({B, C}, x.options());
    nnsx::kernels::avgpool_f32(x.data_ptr<float>(), y.data_ptr<float>(), static_cast<int>(B), static_cast<int>(HW),
                               static_cast<int>(C), cur_stream());
    return y;
  }
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 4, "avgpool: x [B,H,W,C] bf16");
  const int64_t B = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0, "avgpool: C % 8");
  at::Tensor y = at::empty({B, C}, x.options());
  nnsx::kernels::avgpool(x.data_ptr(), y.data_ptr(), static_cast<int>(B), static_cast<int>(HW), static_cast<int>(C),
                         cur_stream());
  return y;
}

at::Tensor avgpool_cpu(const at::Tensor& x) { return x.to(at::kFloat).mean({1, 2}).to(x.scalar_type()); }

// head 1x1 conv + act + global average pool, one launch (fp32; the small-batch
// path of the fused MobileNetV2): x [B,H,W,K] -> [B,N]
at::Tensor pw_conv_pool_cuda(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias, int64_t N, int64_t act) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
              "pw_conv_pool: x [B,H,W,K] f32 contiguous");
  TORCH_CHECK(wt.scalar_type() == at::kFloat && wt.is_contiguous() && wt.dim() == 2, "pw_conv_pool: wt [Npad,Kpad] f32");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() >= N, "pw_conv_pool: bias f32 [N]");
  const int64_t B = x.size(0), HW = x.size(1) * x.size(2), K = x.size(3);
  const int64_t Kpad = wt.size(1), Npad = wt.size(0);
  TORCH_CHECK(K % 4 == 0 && N % 4 == 0 && Kpad >= K && Npad >= N, "pw_conv_pool: shape constraints (K%4, N%4)");
  at::Tensor y = at::empty({B, N}, x.options());
  nnsx::kernels::pw_pool_f32(x.data_ptr<float>(), wt.data_ptr<float>(), bias.data_ptr<float>(), y.data_ptr<float>(),
                             static_cast<int>(B), static_cast<int>(HW), static_cast<int>(N), static_cast<int>(K),
                             static_cast<int>(Kpad), static_cast<int>(Npad), static_cast<int>(act), cur_stream(),
                             x3_weights(wt));
  return y;
}

at::Tensor pw_conv_pool_cpu(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& bias, int64_t N, int64_t act) {
  return avgpool_cpu(pw_conv_cpu(x, wt, bias, c10::nullopt, N, act, true));
}

// ----------------------------------------------------------- ir_block ----
// Fused inverted residual.  we [hid, cin32], wd [9, hid], wp [ceil16(cout), hid] bf16; biases f32.
// split-bf16 weight parts [3][rows][cols] bf16 of at least these sizes (else unused)
static const uint16_t* x3_ptr(const c10::optional<at::Tensor>& t, const at::Tensor& x, int64_t rows, int64_t cols) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 3 &&
                  t->size(0) == 3 && t->size(1) == rows && t->size(2) == cols && t->get_device() == x.get_device(),
              "x3 weights: [3, ", rows, ", ", cols, "] bf16 on the input's device");
  return static_cast<const uint16_t*>(t->data_ptr());
}

at::Tensor ir_block_f32_cuda(const at::Tensor& x, const at::Tensor& we, const at::Tensor& be, const at::Tensor& wd,
                             const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, int64_t stride,
                             int64_t cout, bool has_expand, bool residual, int64_t dilation,
                             const c10::optional<at::Tensor>& tickets, const c10::optional<at::Tensor>& we3,
                             const c10::optional<at::Tensor>& wp3) {
  TORCH_CHECK(x.is_contiguous() && x.dim() == 4, "ir_block(f32): x [B,H,W,C] f32");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t hid = wd.size(1);
  for (const auto* t : {&we, &be, &wd, &bd, &wp, &bp})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "ir_block(f32): weights must be contiguous f32");
  TORCH_CHECK(wd.numel() == 9 * hid && bd.numel() >= hid && wp.size(1) == hid && wp.size(0) >= (cout + 15) / 16 * 16 &&
                  bp.numel() >= wp.size(0),
              "ir_block(f32): dw / project weights");
  TORCH_CHECK(!has_expand || (we.size(0) == hid && we.size(1) == (C + 7) / 8 * 8 && be.numel() >= hid),
              "ir_block(f32): expand weights [hid, ceil8(cin)]");
  TORCH_CHECK(!residual || (stride == 1 && C == cout), "ir_block(f32): residual needs stride 1 and cin == cout");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  at::Tensor y = at::empty({B, Ho, Wo, cout}, x.options());
  nnsx::kernels::IrBlockF32Args a;
  a.x = x.data_ptr<float>();
  a.y = y.data_ptr<float>();
  a.we = has_expand ? we.data_ptr<float>() : nullptr;
  a.be = has_expand ? be.data_ptr<float>() : nullptr;
  a.wd = wd.data_ptr<float>();
  a.bd = bd.data_ptr<float>();
  a.wp = wp.data_ptr<float>();
  a.bp = bp.data_ptr<float>();
  a.B = static_cast<int>(B);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.cin = static_cast<int>(C);
  a.hid = static_cast<int>(hid);
  a.cout = static_cast<int>(cout);
  a.stride = static_cast<int>(stride);
  a.has_expand = has_expand ? 1 : 0;
  a.residual = residual ? 1 : 0;
  a.dil = static_cast<int>(dilation);
  if (has_expand) {
    a.we3 = x3_ptr(we3, x, hid, (C + 31) / 32 * 32);
    a.wp3 = x3_ptr(wp3, x, (cout + 31) / 32 * 32, hid);
  }
  at::Tensor ws;
  if (const size_t wsb = nnsx::kernels::ir_block_f32_workspace_bytes(a)) {
    ws = at::empty({static_cast<int64_t>(wsb / sizeof(float))}, x.options());  // caching allocator: graph-capture safe
    a.ws = ws.data_ptr<float>();
  }
  // hidden-part tickets of the in-launch combine: the model's zero-initialised
  // int32 buffer (each launch leaves it zeroed again); without one, or when
  // too small, the parts are added by a separate reduce launch
  if (const size_t nt = nnsx::kernels::ir_block_f32_tickets(a)) {
    if (tickets.has_value() && tickets->defined() && tickets->is_cuda() && tickets->scalar_type() == at::kInt &&
        tickets->is_contiguous() && static_cast<size_t>(tickets->numel()) >= nt &&
        tickets->get_device() == x.get_device())
      a.tickets = tickets->data_ptr<int>();
  }
  TORCH_CHECK(nnsx::kernels::ir_block_f32(a, cur_stream()), "ir_block(f32): unsupported shape (stride ", stride, ", ",
              H, "x", W, ", cin ", C, ", hid ", hid, ", cout ", cout, ")");
  return y;
}

// expand + depthwise (fp32), the depthwise output [B, Ho, Wo, hid]: blocks
// whose project runs as a plain GEMM afterwards
at::Tensor ir_expand_dw_cuda(const at::Tensor& x, const at::Tensor& we, const at::Tensor& be, const at::Tensor& wd,
                             const at::Tensor& bd, int64_t stride, int64_t dilation,
                             const c10::optional<at::Tensor>& we3) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4,
              "ir_expand_dw: x [B,H,W,C] f32");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t hid = wd.size(1);
  for (const auto* t : {&we, &be, &wd, &bd})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "ir_expand_dw: weights must be contiguous f32");
  TORCH_CHECK(wd.numel() == 9 * hid && bd.numel() >= hid && we.size(0) == hid && we.size(1) == (C + 7) / 8 * 8 &&
                  be.numel() >= hid,
              "ir_expand_dw: weights (we [hid, ceil8(cin)], wd [9, hid])");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  at::Tensor y = at::empty({B, Ho, Wo, hid}, x.options());
  nnsx::kernels::IrBlockF32Args a;
  a.x = x.data_ptr<float>();
  a.y = y.data_ptr<float>();
  a.we = we.data_ptr<float>();
  a.be = be.data_ptr<float>();
  a.wd = wd.data_ptr<float>();
  a.bd = bd.data_ptr<float>();
  a.B = static_cast<int>(B);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.cin = static_cast<int>(C);
  a.hid = static_cast<int>(hid);
  a.cout = 0;
  a.stride = static_cast<int>(stride);
  a.has_expand = 1;
  a.dil = static_cast<int>(dilation);
  a.we3 = x3_ptr(we3, x, hid, (C + 31) / 32 * 32);
  TORCH_CHECK(nnsx::kernels::ir_expand_dw_f32(a, cur_stream()), "ir_expand_dw: unsupported shape (stride ", stride,
              ", ", H, "x", W, ", cin ", C, ", hid ", hid, ")");
  return y;
}

at::Tensor ir_expand_dw_cpu(const at::Tensor& x, const at::Tensor& we, const at::Tensor& be, const at::Tensor& wd,
                            const at::Tensor& bd, int64_t stride, int64_t dilation,
                            const c10::optional<at::Tensor>& we3) {
  (void)we3;
  const int64_t hid = wd.size(1);
  at::Tensor h = pw_conv_cpu(x, we, be, c10::nullopt, hid, 1, false);
  return dw_conv_cpu(h, wd, bd, stride, 1, dilation);
}

bool ir_expand_dw_supported_f32(int64_t stride, int64_t H, int64_t W, int64_t cin, int64_t hid, int64_t B,
                                int64_t dilation) {
  return nnsx::kernels::ir_expand_dw_f32_supported(static_cast<int>(stride), static_cast<int>(H), static_cast<int>(W),
                                                   static_cast<int>(cin), static_cast<int>(hid), static_cast<int>(B),
                                                   static_cast<int>(dilation));
}

at::Tensor ir_block_cuda(const at::Tensor& x, const at::Tensor& we, const at::Tensor& be, const at::Tensor& wd,
                         const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, int64_t stride,
                         int64_t cout, bool has_expand, bool residual, int64_t dilation,
                         const c10::optional<at::Tensor>& tickets, const c10::optional<at::Tensor>& we3,
                         const c10::optional<at::Tensor>& wp3) {
  TORCH_CHECK(x.is_cuda(), "ir_block: x must be a cuda tensor");
  if (x.scalar_type() == at::kFloat)
    return ir_block_f32_cuda(x, we, be, wd, bd, wp, bp, stride, cout, has_expand, residual, dilation, tickets, we3,
                             wp3);
  TORCH_CHECK(dilation == 1, "ir_block(bf16): dilation 1 only");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 4,
              "ir_block: x [B,H,W,C] bf16");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t hid = wd.size(1);
  TORCH_CHECK(wd.numel() == 9 * hid && wp.size(1) == hid && wp.size(0) >= (cout + 15) / 16 * 16, "ir_block: weights");
  TORCH_CHECK(!has_expand || (we.size(0) == hid && we.size(1) >= C), "ir_block: expand weights");
  TORCH_CHECK(!residual || (stride == 1 && C == cout), "ir_block: residual needs stride 1 and cin == cout");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  at::Tensor y = at::empty({B, Ho, Wo, cout}, x.options());
  nnsx::kernels::IrBlockArgs a;
  a.x = static_cast<const uint16_t*>(x.data_ptr());
  a.y = static_cast<uint16_t*>(y.data_ptr());
  a.we = has_expand ? static_cast<const uint16_t*>(we.data_ptr()) : nullptr;
  a.be = has_expand ? be.data_ptr<float>() : nullptr;
  a.wd = static_cast<const uint16_t*>(wd.data_ptr());
  a.bd = bd.data_ptr<float>();
  a.wp = static_cast<const uint16_t*>(wp.data_ptr());
  a.bp = bp.data_ptr<float>();
  a.B = static_cast<int>(B);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.cin = static_cast<int>(C);
  a.hid = static_cast<int>(hid);
  a.cout = static_cast<int>(cout);
  a.stride = static_cast<int>(stride);
  a.has_expand = has_expand ? 1 : 0;
  a.residual = residual ? 1 : 0;
  TORCH_CHECK(nnsx::kernels::ir_block(a, cur_stream()), "ir_block: unsupported shape (stride ", stride, ", cin ", C,
              ", hid ", hid, ", cout ", cout, ")");
  return y;
}

at::Tensor ir_block_cpu(const at::Tensor& x, const at::Tensor& we, const at::Tensor& be, const at::Tensor& wd,
                        const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, int64_t stride,
                        int64_t cout, bool has_expand, bool residual, int64_t dilation,
                        const c10::optional<at::Tensor>& tickets, const c10::optional<at::Tensor>& we3,
                        const c10::optional<at::Tensor>& wp3) {
  (void)tickets;
  (void)we3;
  (void)wp3;
  at::Tensor h = x;
  const int64_t hid = wd.size(1);
  if (has_expand) h = pw_conv_cpu(x, we, be, c10::nullopt, hid, 1, false);
  h = dw_conv_cpu(h, wd, bd, stride, 1, dilation);
  c10::optional<at::Tensor> res;
  if (residual) res = x;
  return pw_conv_cpu(h, wp, bp, res, cout, 0, false);  // (dtype follows x: f32 stays f32)
}

// ------------------------------------------------- lowered-graph ops ----
// Composite ops the load-time lowering (filter/torch_lower.cc) emits for a
// plain TorchScript model: each takes the fused kernel when the shape, dtype
// and device allow it and otherwise runs the same arithmetic on the unfused
// nnsx ops, so a lowered graph never fails on a shape the kernels lack.
at::Tensor ir_block_any(const at::Tensor& x, const at::Tensor& we, const at::Tensor& be, const at::Tensor& wd,
                        const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, int64_t stride, int64_t cout,
                        bool has_expand, bool residual, int64_t dilation, const c10::optional<at::Tensor>& tickets,
                        const c10::optional<at::Tensor>& we3, const c10::optional<at::Tensor>& wp3) {
  if (!x.is_cuda() || x.scalar_type() != at::kFloat)
    return ir_block_cpu(x.to(at::kFloat), we, be, wd, bd, wp, bp, stride, cout, has_expand, residual, dilation,
                        tickets, we3, wp3);
  at::Tensor xc = x.contiguous();
  const int64_t B = xc.size(0), H = xc.size(1), W = xc.size(2), C = xc.size(3), hid = wd.size(1);
  if (nnsx::kernels::ir_block_f32_supported(static_cast<int>(stride), static_cast<int>(H), static_cast<int>(W),
                                            static_cast<int>(C), static_cast<int>(hid), static_cast<int>(cout),
                                            has_expand, static_cast<int>(dilation), static_cast<int>(B)))
    return ir_block_f32_cuda(xc, we, be, wd, bd, wp, bp, stride, cout, has_expand, residual, dilation, tickets, we3,
                             wp3);
  at::Tensor h;
  if (has_expand && nnsx::kernels::ir_expand_dw_f32_supported(static_cast<int>(stride), static_cast<int>(H),
                                                             static_cast<int>(W), static_cast<int>(C),
                                                             static_cast<int>(hid), static_cast<int>(B),
                                                             static_cast<int>(dilation))) {
    h = ir_expand_dw_cuda(xc, we, be, wd, bd, stride, dilation, we3);
  } else {
    h = has_expand ? pw_conv_f32_cuda(xc, we, be, c10::nullopt, hid, 1) : xc;
    h = dw_conv_cuda(h, wd, bd, stride, 1, dilation);
  }
  c10::optional<at::Tensor> res;
  if (residual) res = xc;
  return pw_conv_f32_cuda(h, wp, bp, res, cout, 0);
}

// stem conv + act from a uint8 frame (through the input table) or a float one
at::Tensor stem_any(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, const at::Tensor& lut,
                    int64_t act) {
  if (x.scalar_type() == at::kByte)
    return x.is_cuda() ? stem_conv_u8_cuda(x.contiguous(), w, bias, act, lut, true)
                       : stem_conv_u8_cpu(x, w, bias, act, lut, true);
  at::Tensor xf = x.to(at::kFloat).contiguous();
  return xf.is_cuda() ? stem_conv_cuda(xf, w, bias, act, true) : stem_conv_cpu(xf, w, bias, act, true);
}

at::Tensor stem_ir1_cuda(const at::Tensor& x, const at::Tensor& ws, const at::Tensor& bs, const at::Tensor& wd,
                         const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, const at::Tensor& lut,
                         int64_t mode);
at::Tensor stem_ir1_cpu(const at::Tensor& x, const at::Tensor& ws, const at::Tensor& bs, const at::Tensor& wd,
                        const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, const at::Tensor& lut,
                        int64_t mode);

// stem + a t = 1 first block (32 -> dw -> 16): one kernel on a uint8 frame,
// else the stem, depthwise and project ops
at::Tensor stem_ir1_any(const at::Tensor& x, const at::Tensor& ws, const at::Tensor& bs, const at::Tensor& wd,
                        const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, const at::Tensor& lut,
                        int64_t cout) {
  if (x.scalar_type() == at::kByte && x.is_cuda() && cout == 16 && wp.size(0) >= 16 && wp.size(1) == 32)
    return stem_ir1_cuda(x.contiguous(), ws, bs, wd, bd, wp, bp, lut, -1);
  at::Tensor h = stem_any(x, ws, bs, lut, 1);
  if (h.is_cuda()) {
    h = dw_conv_cuda(h, wd, bd, 1, 1, 1);
    return pw_conv_f32_cuda(h, wp, bp, c10::nullopt, cout, 0);
  }
  h = dw_conv_cpu(h, wd, bd, 1, 1, 1);
  return pw_conv_cpu(h, wp, bp, c10::nullopt, cout, 0, true);
}

// stem + first (t = 1) block, fused (fp32): uint8 frame -> [B, Ho, Wo, 16]
at::Tensor stem_ir1_cuda(const at::Tensor& x, const at::Tensor& ws, const at::Tensor& bs, const at::Tensor& wd,
                         const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, const at::Tensor& lut,
                         int64_t mode) {
  TORCH_CHECK(lut.is_cuda() && lut.scalar_type() == at::kFloat && lut.numel() == 256 && lut.is_contiguous(),
              "stem_ir1: lut [256] f32 on the device");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kByte && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3,
              "stem_ir1: x [B,H,W,3] uint8");
  for (const auto* t : {&ws, &bs, &wd, &bd, &wp, &bp})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), "stem_ir1: f32 weights");
  TORCH_CHECK(ws.numel() == 27 * 32 && bs.numel() >= 32 && wd.numel() == 9 * 32 && bd.numel() >= 32 &&
                  wp.size(0) >= 16 && wp.size(1) == 32 && bp.numel() >= 16,
              "stem_ir1: ws [3,3,3,32], wd [9,32], wp [16,32]");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2);
  at::Tensor y = at::empty({B, (H - 1) / 2 + 1, (W - 1) / 2 + 1, 16}, x.options().dtype(at::kFloat));
  nnsx::kernels::StemIr1F32Args a;
  a.x = x.data_ptr<uint8_t>();
  a.y = y.data_ptr<float>();
  a.ws = ws.data_ptr<float>();
  a.bs = bs.data_ptr<float>();
  a.wd = wd.data_ptr<float>();
  a.bd = bd.data_ptr<float>();
  a.wp = wp.data_ptr<float>();
  a.bp = bp.data_ptr<float>();
  a.B = static_cast<int>(B);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.lut = lut.data_ptr<float>();
  a.mode = static_cast<int>(mode);
  TORCH_CHECK(nnsx::kernels::stem_ir1_f32(a, cur_stream()), "stem_ir1: launch failed");
  return y;
}

at::Tensor stem_ir1_cpu(const at::Tensor& x, const at::Tensor& ws, const at::Tensor& bs, const at::Tensor& wd,
                        const at::Tensor& bd, const at::Tensor& wp, const at::Tensor& bp, const at::Tensor& lut,
                        int64_t mode) {
  (void)mode;
  at::Tensor h = stem_conv_u8_cpu(x, ws, bs, 1, lut, true);
  h = dw_conv_cpu(h, wd, bd, 1, 1, 1);
  return pw_conv_cpu(h, wp, bp, c10::nullopt, 16, 0, true);
}

bool ir_supported_f32(int64_t stride, int64_t H, int64_t W, int64_t cin, int64_t hid, int64_t cout, bool has_expand,
                      int64_t dilation, int64_t B) {
  return nnsx::kernels::ir_block_f32_supported(static_cast<int>(stride), static_cast<int>(H), static_cast<int>(W),
                                               static_cast<int>(cin), static_cast<int>(hid), static_cast<int>(cout),
                                               has_expand, static_cast<int>(dilation), static_cast<int>(B));
}

bool ir_supported(int64_t stride, int64_t cin, int64_t hid, int64_t cout) {
  return nnsx::kernels::ir_block_supported(static_cast<int>(stride), static_cast<int>(cin), static_cast<int>(hid),
                                           static_cast<int>(cout));
}

std::string ir_method_f32(int64_t stride, int64_t H, int64_t W, int64_t cin, int64_t hid, int64_t cout, int64_t B,
                          int64_t dilation) {
  return nnsx::kernels::ir_block_f32_method(static_cast<int>(stride), static_cast<int>(H), static_cast<int>(W),
                                            static_cast<int>(cin), static_cast<int>(hid), static_cast<int>(cout),
                                            static_cast<int>(B), static_cast<int>(dilation));
}

bool set_device_shared(bool on) { return nnsx::kernels::set_device_shared(on); }

std::string f32_math() { return nnsx::kernels::f32_math_name(nnsx::kernels::f32_math()); }

// returns the previous method
std::string set_f32_math(const std::string& m) {
  const std::string prev = f32_math();
  if (m == "x3") {
    nnsx::kernels::set_f32_math(nnsx::kernels::F32Math::kX3);
  } else if (m == "fp32" || m == "native") {
    nnsx::kernels::set_f32_math(nnsx::kernels::F32Math::kNative);
  } else {
    TORCH_CHECK(false, "set_f32_math: x3 | fp32, got ", m);
  }
  return prev;
}

}  // namespace

namespace nnsx {
namespace ops {
// tensor_filter (filter/pytorch.cc clear_graphs): no captured graph refers to
// retired x3 weight parts any more
void x3_retire_flush() {
  std::lock_guard<std::mutex> lk(g_x3_mu);
  g_x3_retired.clear();
}
}  // namespace ops
}  // namespace nnsx

TORCH_LIBRARY(nnsx, m) {
  m.def("f32_math() -> str", f32_math);
  m.def("set_device_shared(bool on) -> bool", set_device_shared);
  m.def("x3_weight_cache(bool on) -> bool", x3_weight_cache);
  m.def("ir_method_f32(int stride, int H, int W, int cin, int hid, int cout, int B, int dilation=1) -> str",
        ir_method_f32);
  m.def("set_f32_math(str method) -> str", set_f32_math);
  m.def("irp_min_batch(int b) -> int", [](int64_t b) -> int64_t {
    return nnsx::kernels::irp_x3_set_min_batch(static_cast<int>(b));
  });
  m.def("irh_mode(int m) -> int", [](int64_t m) -> int64_t {
    return nnsx::kernels::irh_set_mode(static_cast<int>(m));
  });
  m.def("pw_conv(Tensor x, Tensor wt, Tensor bias, Tensor? res, int N, int act, bool out_f32) -> Tensor");
  m.def("pw_conv_into(Tensor x, Tensor wt, Tensor bias, Tensor(a!) out, int row0, int n, int act) -> ()");
  m.def("pw_conv_rowbias(Tensor x, Tensor wt, Tensor bias, int N, int act) -> Tensor");
  m.def("upsample_bilinear(Tensor x, int H, int W) -> Tensor");
  m.def("sep_heads(Tensor[] xs, Tensor[] wds, Tensor[] bds, Tensor[] wts, Tensor[] biases, int[] ns, int[] which, "
        "Tensor(a!) out_box, Tensor(b!) out_cls, int mode=0) -> ()");
  m.def("pw_conv_group(Tensor[] xs, Tensor[] wts, Tensor[] biases, int[] ns, int[] acts) -> Tensor[]");
  m.def("dw_conv(Tensor x, Tensor w, Tensor bias, int stride, int act, int dilation=1) -> Tensor");
  m.def("stem_conv(Tensor x, Tensor w, Tensor bias, int act, bool out_f32=False) -> Tensor");
  m.def("stem_conv_u8(Tensor x, Tensor w, Tensor bias, int act, Tensor lut, bool out_f32=False) -> Tensor");
  m.def("avgpool(Tensor x) -> Tensor");
  m.def("pw_conv_pool(Tensor x, Tensor wt, Tensor bias, int N, int act) -> Tensor");
  m.def("stem_ir1(Tensor x, Tensor ws, Tensor bs, Tensor wd, Tensor bd, Tensor wp, Tensor bp, Tensor lut, "
        "int mode=-1) -> Tensor");
  m.def("pw_conv_f32_tile(Tensor x, Tensor wt, Tensor bias, Tensor? res, int N, int act, int tile) -> Tensor");
  m.def("ir_block(Tensor x, Tensor we, Tensor be, Tensor wd, Tensor bd, Tensor wp, Tensor bp, int stride, int cout, "
        "bool has_expand, bool residual, int dilation=1, Tensor(a!)? tickets=None, Tensor? we3=None, "
        "Tensor? wp3=None) -> Tensor");
  m.def("ir_supported(int stride, int cin, int hid, int cout) -> bool", ir_supported);
  // composite ops of the load-time lowering of plain TorchScript models (filter/torch_lower.cc)
  m.def("ir_block_any(Tensor x, Tensor we, Tensor be, Tensor wd, Tensor bd, Tensor wp, Tensor bp, int stride, "
        "int cout, bool has_expand, bool residual, int dilation=1, Tensor(a!)? tickets=None, Tensor? we3=None, "
        "Tensor? wp3=None) -> Tensor", ir_block_any);
  m.def("stem_any(Tensor x, Tensor w, Tensor bias, Tensor lut, int act) -> Tensor", stem_any);
  m.def("stem_ir1_any(Tensor x, Tensor ws, Tensor bs, Tensor wd, Tensor bd, Tensor wp, Tensor bp, Tensor lut, "
        "int cout) -> Tensor", stem_ir1_any);
  m.def("ir_supported_f32(int stride, int H, int W, int cin, int hid, int cout, bool has_expand, int dilation=1, "
        "int B=0) -> bool",
        ir_supported_f32);
  m.def("ir_expand_dw_supported_f32(int stride, int H, int W, int cin, int hid, int B=0, int dilation=1) -> bool",
        ir_expand_dw_supported_f32);
  m.def("ir_expand_dw(Tensor x, Tensor we, Tensor be, Tensor wd, Tensor bd, int stride, int dilation=1, "
        "Tensor? we3=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(nnsx, CUDA, m) {
  m.impl("pw_conv", pw_conv_cuda);
  m.impl("pw_conv_into", pw_conv_into_cuda);
  m.impl("pw_conv_rowbias", pw_conv_rowbias_cuda);
  m.impl("upsample_bilinear", upsample_bilinear_cuda);
  m.impl("sep_heads", sep_heads_cuda);
  m.impl("pw_conv_group", pw_conv_group_cuda);
  m.impl("dw_conv", dw_conv_cuda);
  m.impl("stem_conv", stem_conv_cuda);
  m.impl("stem_conv_u8", stem_conv_u8_cuda);
  m.impl("avgpool", avgpool_cuda);
  m.impl("pw_conv_pool", pw_conv_pool_cuda);
  m.impl("stem_ir1", stem_ir1_cuda);
  m.impl("pw_conv_f32_tile", pw_conv_f32_tile_cuda);
  m.impl("ir_block", ir_block_cuda);
  m.impl("ir_expand_dw", ir_expand_dw_cuda);
}

TORCH_LIBRARY_IMPL(nnsx, CPU, m) {
  m.impl("pw_conv", pw_conv_cpu);
  m.impl("pw_conv_into", pw_conv_into_cpu);
  m.impl("pw_conv_rowbias", pw_conv_rowbias_cpu);
  m.impl("upsample_bilinear", upsample_bilinear_cpu);
  m.impl("sep_heads", sep_heads_cpu);
  m.impl("pw_conv_group", pw_conv_group_cpu);
  m.impl("dw_conv", dw_conv_cpu);
  m.impl("stem_conv", stem_conv_cpu);
  m.impl("stem_conv_u8", stem_conv_u8_cpu);
  m.impl("avgpool", avgpool_cpu);
  m.impl("pw_conv_pool", pw_conv_pool_cpu);
  m.impl("stem_ir1", stem_ir1_cpu);
  m.impl("ir_block", ir_block_cpu);
  m.impl("ir_expand_dw", ir_expand_dw_cpu);
}
