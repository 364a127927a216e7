// tensor_decoder mode=image_segment and mode=pose_estimation.
//
// image_segment -- reference ext/nnstreamer/tensor_decoder/
// tensordec-imagesegment.c: option1 mode (tflite-deeplab: [L:W:H] label
// probabilities, argmax with a 0.5 threshold; snpe-deeplab: [W:H:1] label
// indices; snpe-depth: [1:W:H] grayscale normalised by the frame maximum),
// option2 max labels (default 20).  nnsx extension, option3 = W:H: a
// tflite-deeplab score map smaller than W x H (e.g. DeepLab's 33 x 33 logits at
// output stride 16) is bilinearly resized (align_corners, the rule of
// PyTorch's upsample_bilinear2d) to W x H per label before the argmax, in the
// same device pass -- the model then ships its low-resolution logits and the
// full-resolution score map never exists.  The colour map is the deterministic
// rgb_modifier * label table the reference uses on its vectorised path
// (:200-215); its scalar path draws random colours, which no golden can pin.
// On HBM-resident input the fused argmax + colour kernel writes the RGBA frame
// directly (kernels/vision.hip); trailing batch dims decode B frames at once.
//
// pose_estimation -- reference tensordec-pose.c: option1 output W:H, option2
// input W:H, option3 keypoint/connection file, option4 heatmap-only |
// heatmap-offset; per-keypoint heatmap argmax (first maximum, floor
// FLT_MIN, :780-800), offset refinement, Bresenham skeleton with end dots
// and labels.  For HBM-resident float input the whole decode runs on the GPU
// (argmax kernel, then one raster kernel per batch of frames); otherwise on
// the host.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <fstream>

#include "core/cpu_ops.h"
#include "core/log.h"
#include "decoders/decoders.h"
#include "decoders/font.h"
#include "kernels/vision.h"
#include "runtime/hip_util.h"

namespace nnsx {

namespace {

const uint8_t kFontTable[95][13] = NNSX_FONT8X13_DATA;

bool rest_ones(const Dims& d, int from) {
  for (int i = from; i < kRankLimit; ++i)
    if (d[i] != 1) return false;
  return true;
}

// ============================================================ image_segment ====
class ImageSegment : public DecoderInstance {
 public:
  enum Mode { TFLITE_DEEPLAB = 0, SNPE_DEEPLAB, SNPE_DEPTH, UNKNOWN };

  bool set_option(int idx, const std::string& v) override {
    if (idx == 0) {
      if (v.empty()) return false;
      mode_ = v == "tflite-deeplab" ? TFLITE_DEEPLAB : v == "snpe-deeplab" ? SNPE_DEEPLAB
                                                    : v == "snpe-depth"     ? SNPE_DEPTH
                                                                            : UNKNOWN;
      return true;
    }
    if (idx == 1) {
      uint64_t m = to_uint(v);
      if (m != 0 && m <= UINT32_MAX) max_labels_ = static_cast<unsigned>(m);
    }
    if (idx == 2) {
      out_w_ = out_h_ = 0;
      const size_t c = v.find(':');
      if (c != std::string::npos) {
        const uint64_t ow = to_uint(v.substr(0, c)), oh = to_uint(v.substr(c + 1));
        if (ow > 0 && oh > 0 && ow <= 65535 && oh <= 65535) {
          out_w_ = static_cast<unsigned>(ow);
          out_h_ = static_cast<unsigned>(oh);
        }
      }
    }
    return true;
  }

  bool supports_device() const override { return true; }

  Caps get_out_caps(const TensorsConfig& config) override {
    if (config.info.num_tensors < 1) return Caps();
    unsigned w, h, b;
    if (!geometry(config.info.at(0), &w, &h, &b)) return Caps();
    if (resizes(w, h)) {
      w = out_w_;
      h = out_h_;
    }
    Caps c = Caps::from_string(strfmt("video/x-raw, format=(string)RGBA, width=(int)", w, ", height=(int)", h));
    set_framerate_from_config(c, config);
    return c;
  }

  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext& ctx) override {
    const TensorInfo& ti = config.info.at(0);
    unsigned w, h, batch;
    if (!geometry(ti, &w, &h, &batch) || !sane(ti)) {
      NNSX_LOGE("image_segment", "invalid input data format");
      return FlowReturn::ERROR;
    }
    const uint32_t rgb_mod = 0xFFFFFFu / (max_labels_ + 1);
    ctx.out_frames = batch;
    if (resizes(w, h)) return decode_resized(x_of(in[0], ctx), w, h, batch, rgb_mod, in[0], out, ctx);
    const uint64_t npix = static_cast<uint64_t>(w) * h;
    const size_t fsize = npix * 4;
    if (ctx.device >= 0) {
      const int dev = ctx.device;
      hipStream_t s = ctx.stream;
      const float* x = static_cast<const float*>(in[0]->map_device(dev, s));
      MemoryPtr frames = Memory::alloc_device(fsize * batch, dev, s);
      uint32_t* o = static_cast<uint32_t*>(frames->data());
      if (mode_ == TFLITE_DEEPLAB) {
        kernels::segment_argmax_color(x, static_cast<int>(max_labels_ + 1), npix * batch, rgb_mod, kThreshold, o, s);
      } else if (mode_ == SNPE_DEEPLAB) {
        kernels::segment_index_color(x, npix * batch, static_cast<int>(max_labels_), rgb_mod, o, s);
      } else {
        if (!ws_ || ws_->size() < batch * sizeof(uint32_t) || ws_->device() != dev)
          ws_ = Memory::alloc_device(std::max<size_t>(batch, 64) * sizeof(uint32_t), dev, s);
        kernels::segment_depth_gray(x, npix, static_cast<int>(batch), static_cast<uint32_t*>(ws_->data()), o, s);
        ws_->record_use(s, dev);
      }
      frames->mark_ready(s);
      for (unsigned b = 0; b < batch; ++b) out->mems.push_back(Memory::view(frames, b * fsize, fsize));
      return FlowReturn::OK;
    }
    const float* x = static_cast<const float*>(in[0]->map_host());
    for (unsigned b = 0; b < batch; ++b) {
      auto m = Memory::alloc_host(fsize);
      uint32_t* o = static_cast<uint32_t*>(m->data());
      std::memset(o, 0, fsize);
      if (mode_ == TFLITE_DEEPLAB) {
        const unsigned L = max_labels_ + 1;
        const float* f = x + static_cast<uint64_t>(b) * npix * L;
        for (uint64_t p = 0; p < npix; ++p) {
          const float* v = f + p * L;
          float best = v[0];
          unsigned bi = 0;
          for (unsigned l = 1; l < L; ++l)
            if (v[l] > best) {
              best = v[l];
              bi = l;
            }
          o[p] = best > kThreshold ? color(bi, rgb_mod) : 0u;
        }
      } else if (mode_ == SNPE_DEEPLAB) {
        const float* f = x + static_cast<uint64_t>(b) * npix;
        for (uint64_t p = 0; p < npix; ++p) {
          if (!(f[p] >= 0.f) || f[p] >= static_cast<float>(max_labels_) + 1.f) continue;
          o[p] = color(static_cast<unsigned>(f[p]), rgb_mod);
        }
      } else {
        const float* f = x + static_cast<uint64_t>(b) * npix;
        float mx = 0.f;
        for (uint64_t p = 0; p < npix; ++p) mx = std::max(mx, f[p]);
        if (mx != 0.f) {
          for (uint64_t p = 0; p < npix; ++p) {
            float g = f[p] / mx * 255.f;
            uint32_t gray = g >= 0.f ? static_cast<uint32_t>(g) : 0xffffffffu;
            if (gray > 255u) continue;
            o[p] = gray | (gray << 8) | (gray << 16) | 0xff000000u;
          }
        }
      }
      out->mems.push_back(m);
    }
    return FlowReturn::OK;
  }

 private:
  static constexpr float kThreshold = 0.5f;

 public:
  // ---- device stage (runtime/fusion.h): (resize +) argmax + colour map inside
  // the filter's graph; output = the B RGBA frames [4:W:H:B] ----
  bool stage_prepare(const TensorsConfig& config, int dev, hipStream_t s, TensorsInfo* out) override {
    if (dev < 0 || config.info.num_tensors < 1) return false;
    const TensorInfo& ti = config.info.at(0);
    unsigned w, h, batch;
    if (!geometry(ti, &w, &h, &batch) || !sane(ti)) return false;
    st_w_ = w;
    st_h_ = h;
    st_batch_ = batch;
    if (mode_ == SNPE_DEPTH && (!ws_ || ws_->size() < batch * sizeof(uint32_t) || ws_->device() != dev))
      ws_ = Memory::alloc_device(std::max<size_t>(batch, 64) * sizeof(uint32_t), dev, s);
    const bool rs = resizes(w, h);
    out->resize(1);
    out->at(0).type = DType::UINT8;
    out->at(0).dim = make_dims({4, rs ? out_w_ : w, rs ? out_h_ : h, batch});
    return true;
  }
  // the depth mode reduces through ws_; the label modes write only `out`
  bool stage_lane_safe() const override { return mode_ != SNPE_DEPTH; }
  bool stage_enqueue(const std::vector<const void*>& in, const std::vector<void*>& out, hipStream_t s) override {
    if (in.empty() || out.size() != 1) return false;
    enqueue_device(static_cast<const float*>(in[0]), st_w_, st_h_, st_batch_, static_cast<uint32_t*>(out[0]), s);
    return true;
  }

 private:
  // the device decode of [B] frames of w x h scores into RGBA frames (kernels only)
  void enqueue_device(const float* x, unsigned w, unsigned h, unsigned batch, uint32_t* o, hipStream_t s) {
    const uint32_t rgb_mod = 0xFFFFFFu / (max_labels_ + 1);
    const uint64_t npix = static_cast<uint64_t>(w) * h;
    if (resizes(w, h)) {
      kernels::segment_upsample_argmax_color(x, static_cast<int>(max_labels_ + 1), static_cast<int>(h), static_cast<int>(w),
                                             static_cast<int>(batch), static_cast<int>(out_h_), static_cast<int>(out_w_),
                                             rgb_mod, kThreshold, o, s);
    } else if (mode_ == TFLITE_DEEPLAB) {
      kernels::segment_argmax_color(x, static_cast<int>(max_labels_ + 1), npix * batch, rgb_mod, kThreshold, o, s);
    } else if (mode_ == SNPE_DEEPLAB) {
      kernels::segment_index_color(x, npix * batch, static_cast<int>(max_labels_), rgb_mod, o, s);
    } else {
      kernels::segment_depth_gray(x, npix, static_cast<int>(batch), static_cast<uint32_t*>(ws_->data()), o, s);
    }
  }

  bool resizes(unsigned w, unsigned h) const {
    return mode_ == TFLITE_DEEPLAB && out_w_ && out_h_ && (out_w_ != w || out_h_ != h);
  }
  static const float* x_of(const MemoryPtr& m, InvokeContext& ctx) {
    return static_cast<const float*>(ctx.device >= 0 ? m->map_device(ctx.device, ctx.stream) : m->map_host());
  }

  // option3: [B][h][w][L] scores -> W x H RGBA frames (resize + argmax fused)
  FlowReturn decode_resized(const float* x, unsigned w, unsigned h, unsigned batch, uint32_t rgb_mod,
                            const MemoryPtr& src, Buffer* out, InvokeContext& ctx) {
    (void)src;
    const unsigned W = out_w_, H = out_h_, L = max_labels_ + 1;
    const size_t fsize = static_cast<size_t>(W) * H * 4;
    if (ctx.device >= 0) {
      MemoryPtr frames = Memory::alloc_device(fsize * batch, ctx.device, ctx.stream);
      kernels::segment_upsample_argmax_color(x, static_cast<int>(L), static_cast<int>(h), static_cast<int>(w),
                                             static_cast<int>(batch), static_cast<int>(H), static_cast<int>(W),
                                             rgb_mod, kThreshold, static_cast<uint32_t*>(frames->data()), ctx.stream);
      frames->mark_ready(ctx.stream);
      for (unsigned b = 0; b < batch; ++b) out->mems.push_back(Memory::view(frames, b * fsize, fsize));
      return FlowReturn::OK;
    }
    // host: the same taps and mixing order as the kernel
    auto tap = [](unsigned dst, unsigned in, unsigned outn, unsigned* i0, unsigned* i1, float* l0, float* l1) {
      const float scale = outn > 1 ? static_cast<float>(in - 1) / static_cast<float>(outn - 1) : 0.f;
      const float s = scale * static_cast<float>(dst);
      *i0 = std::min(static_cast<unsigned>(s), in - 1);
      *l1 = s - static_cast<float>(*i0);
      *l0 = 1.f - *l1;
      *i1 = *i0 + (*i0 < in - 1 ? 1 : 0);
    };
    std::vector<unsigned> x0(W), x1(W);
    std::vector<float> lx0(W), lx1(W);
    for (unsigned X = 0; X < W; ++X) tap(X, w, W, &x0[X], &x1[X], &lx0[X], &lx1[X]);
    for (unsigned b = 0; b < batch; ++b) {
      auto m = Memory::alloc_host(fsize);
      uint32_t* o = static_cast<uint32_t*>(m->data());
      const float* f = x + static_cast<uint64_t>(b) * h * w * L;
      for (unsigned Y = 0; Y < H; ++Y) {
        unsigned y0, y1;
        float ly0, ly1;
        tap(Y, h, H, &y0, &y1, &ly0, &ly1);
        const float* r0 = f + static_cast<uint64_t>(y0) * w * L;
        const float* r1 = f + static_cast<uint64_t>(y1) * w * L;
        for (unsigned X = 0; X < W; ++X) {
          const float *a0 = r0 + x0[X] * L, *a1 = r0 + x1[X] * L, *c0 = r1 + x0[X] * L, *c1 = r1 + x1[X] * L;
          float best = 0.f;
          unsigned bi = 0;
          for (unsigned l = 0; l < L; ++l) {
            const float v = ly0 * (lx0[X] * a0[l] + lx1[X] * a1[l]) + ly1 * (lx0[X] * c0[l] + lx1[X] * c1[l]);
            if (l == 0 || v > best) {
              best = v;
              bi = l;
            }
          }
          o[static_cast<uint64_t>(Y) * W + X] = best > kThreshold ? color(bi, rgb_mod) : 0u;
        }
      }
      out->mems.push_back(m);
    }
    return FlowReturn::OK;
  }

  static uint32_t color(unsigned label, uint32_t rgb_mod) {
    return label == 0 ? 0u : ((rgb_mod * label) & 0x00ffffffu) | 0xff000000u;
  }

  bool geometry(const TensorInfo& ti, unsigned* w, unsigned* h, unsigned* b) const {
    const Dims& d = ti.dim;
    if (mode_ == SNPE_DEEPLAB) {
      *w = d[0];
      *h = d[1];
      *b = d[2] * d[3];  // [W:H:1:B]
      return rest_ones(d, 4);
    }
    if (mode_ == UNKNOWN) return false;
    *w = d[1];
    *h = d[2];
    *b = d[3];
    return rest_ones(d, 4);
  }

  bool sane(const TensorInfo& ti) const {
    if (ti.type != DType::FLOAT32) return false;
    if (mode_ == TFLITE_DEEPLAB) return ti.dim[0] == max_labels_ + 1;
    if (mode_ == SNPE_DEPTH) return ti.dim[0] == 1;
    return mode_ == SNPE_DEEPLAB;
  }

  int mode_ = UNKNOWN;
  unsigned max_labels_ = 20;
  unsigned out_w_ = 0, out_h_ = 0;  // option3
  MemoryPtr ws_;
  unsigned st_w_ = 0, st_h_ = 0, st_batch_ = 1;  // the geometry stage_prepare saw
};

class ImageSegmentPlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "image_segment"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<ImageSegment>(); }
};

// ========================================================== pose_estimation ====
struct PoseMeta {
  std::string label;
  std::vector<int> connections;
};

const std::vector<PoseMeta>& default_pose_meta() {
  static const std::vector<PoseMeta> m = {
      {"top", {1}},          {"neck", {0, 2, 5, 8, 11}}, {"r_shoulder", {1, 3}}, {"r_elbow", {2, 4}},
      {"r_wrist", {3}},      {"l_shoulder", {1, 6}},     {"l_elbow", {5, 7}},    {"l_wrist", {6}},
      {"r_hip", {1, 9}},     {"r_knee", {8, 10}},        {"r_ankle", {9}},       {"l_hip", {1, 12}},
      {"l_knee", {11, 13}},  {"l_ankle", {12}}};
  return m;
}

class PoseEstimation : public DecoderInstance {
 public:
  PoseEstimation() : meta_(default_pose_meta()) {}

  bool set_option(int idx, const std::string& v) override {
    if (idx == 0 || idx == 1) {
      unsigned& w = idx == 0 ? width_ : i_width_;
      unsigned& h = idx == 0 ? height_ : i_height_;
      w = h = 0;
      if (v.empty()) return true;
      Dims d;
      if (parse_dimension(v, d) < 2) return true;
      w = d[0];
      h = d[1];
      return true;
    }
    if (idx == 2) return load_meta(v);
    if (idx == 3) {
      if (v == "heatmap-only")
        mode_ = 0;
      else if (v == "heatmap-offset")
        mode_ = 1;
      else
        return false;
    }
    return true;
  }

  bool supports_device() const override { return true; }

  Caps get_out_caps(const TensorsConfig& config) override {
    if (config.info.num_tensors < 1) return Caps();
    for (unsigned i = 1; i < config.info.num_tensors; ++i)
      if (config.info.at(i).type != config.info.at(i - 1).type) return Caps();
    const Dims& d = config.info.at(0).dim;
    if (d[0] != meta_.size() || !rest_ones(d, 4)) return Caps();
    if (mode_ == 1) {
      if (config.info.num_tensors < 2) return Caps();
      const Dims& o = config.info.at(1).dim;
      if (o[0] != 2 * meta_.size() || !rest_ones(o, 4)) return Caps();
    }
    Caps c = Caps::from_string(strfmt("video/x-raw, format=(string)RGBA, width=(int)", width_, ", height=(int)", height_));
    set_framerate_from_config(c, config);
    return c;
  }

  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext& ctx) override {
    const TensorInfo& hi = config.info.at(0);
    const int K = static_cast<int>(meta_.size());
    const int gw = static_cast<int>(hi.dim[1]), gh = static_cast<int>(hi.dim[2]);
    const unsigned batch = hi.dim[3];
    if (width_ == 0 || height_ == 0 || i_width_ == 0 || i_height_ == 0) {
      NNSX_LOGE("pose_estimation", "option1 (output size) and option2 (input size) must be set");
      return FlowReturn::ERROR;
    }
    // per keypoint: (grid x, grid y, score)
    std::vector<float> kp(static_cast<size_t>(batch) * K * 3);
    const bool offsets_ok = mode_ == 0 || (config.info.num_tensors > 1 && config.info.at(1).type == DType::FLOAT32);
    if (ctx.device >= 0 && hi.type == DType::FLOAT32 && offsets_ok && K <= 64) {
      // all on the GPU: heatmap argmax, offset refinement and skeleton raster (no host sync)
      const int dev = ctx.device;
      hipStream_t s = ctx.stream;
      prepare_device(gw, gh, batch, dev, s);
      const size_t fsize = static_cast<size_t>(width_) * height_ * 4;
      MemoryPtr frames = Memory::alloc_device(fsize * batch, dev, s);
      enqueue_device(static_cast<const float*>(in[0]->map_device(dev, s)),
                     mode_ == 1 ? static_cast<const float*>(in[1]->map_device(dev, s)) : nullptr,
                     static_cast<uint32_t*>(frames->data()), s);
      frames->mark_ready(s);
      dev_kp_->record_use(s, dev);
      ctx.out_frames = batch;
      for (unsigned b = 0; b < batch; ++b) out->mems.push_back(Memory::view(frames, b * fsize, fsize));
      return FlowReturn::OK;
    }
    {
      const void* x = in[0]->map_host();
      for (unsigned b = 0; b < batch; ++b)
        for (int k = 0; k < K; ++k) {
          float best = FLT_MIN;
          int bx = 0, by = 0;
          const size_t base = static_cast<size_t>(b) * gw * gh * K;
          for (int j = 0; j < gh; ++j)
            for (int i = 0; i < gw; ++i) {
              float c = static_cast<float>(
                  cpu::read_as_double(x, hi.type, base + static_cast<size_t>(i) * K + static_cast<size_t>(j) * gw * K + k));
              if (mode_ == 1) c = 1.f / (1.f + std::exp(-c));
              if (c > best) {
                best = c;
                bx = i;
                by = j;
              }
            }
          float* o = &kp[(static_cast<size_t>(b) * K + k) * 3];
          o[0] = static_cast<float>(bx);
          o[1] = static_cast<float>(by);
          o[2] = best;
        }
    }
    ctx.out_frames = batch;
    const void* offsets = mode_ == 1 ? in[1]->map_host() : nullptr;
    const DType ot = mode_ == 1 ? config.info.at(1).type : DType::FLOAT32;
    const size_t fsize = static_cast<size_t>(width_) * height_ * 4;
    for (unsigned b = 0; b < batch; ++b) {
      std::vector<Point> pts(static_cast<size_t>(K));
      for (int k = 0; k < K; ++k) {
        const float* o = &kp[(static_cast<size_t>(b) * K + k) * 3];
        const int mx = static_cast<int>(o[0]), my = static_cast<int>(o[1]);
        Point p;
        p.valid = true;
        p.prob = o[2];
        if (mode_ == 1) {
          const size_t oi = static_cast<size_t>(b) * gw * gh * 2 * K + (static_cast<size_t>(my) * gw + mx) * K * 2 + k;
          float offy = static_cast<float>(cpu::read_as_double(offsets, ot, oi));
          float offx = static_cast<float>(cpu::read_as_double(offsets, ot, oi + static_cast<size_t>(K)));
          float px = (static_cast<float>(mx) / (gw - 1)) * i_width_ + offx;
          float py = (static_cast<float>(my) / (gh - 1)) * i_height_ + offy;
          p.x = static_cast<int>(px * width_ / i_width_);
          p.y = static_cast<int>(py * height_ / i_height_);
        } else {
          p.x = static_cast<int>((static_cast<unsigned>(mx) * width_) / i_width_);
          p.y = static_cast<int>((static_cast<unsigned>(my) * height_) / i_height_);
        }
        p.x = static_cast<int>(std::min<unsigned>(width_, static_cast<unsigned>(std::max(0, p.x))));
        p.y = static_cast<int>(std::min<unsigned>(height_, static_cast<unsigned>(std::max(0, p.y))));
        pts[static_cast<size_t>(k)] = p;
      }
      auto m = Memory::alloc_host(fsize);
      std::memset(m->data(), 0, fsize);
      draw(static_cast<uint32_t*>(m->data()), &pts);
      out->mems.push_back(m);
    }
    return FlowReturn::OK;
  }

 private:
  static constexpr uint32_t kPixel = 0xFFFFFFFFu;

  // device decode, split so the enqueue also runs inside the filter's graph
  // capture (stage_enqueue): prepare allocates / uploads, enqueue only launches
  void prepare_device(int gw, int gh, unsigned batch, int dev, hipStream_t s) {
    const size_t kp_bytes = static_cast<size_t>(batch) * meta_.size() * 3 * sizeof(float);
    if (!dev_kp_ || dev_kp_->size() < kp_bytes || dev_kp_->device() != dev) dev_kp_ = Memory::alloc_device(kp_bytes, dev, s);
    ensure_device_meta(dev, s);
    st_gw_ = gw;
    st_gh_ = gh;
    st_batch_ = batch;
  }
  void enqueue_device(const float* x, const float* offsets, uint32_t* frames, hipStream_t s) {
    const int K = static_cast<int>(meta_.size());
    kernels::pose_heatmap_argmax(x, K, st_gw_, st_gh_, static_cast<int>(st_batch_), mode_ == 1,
                                 static_cast<float*>(dev_kp_->data()), s);
    const size_t fsize = static_cast<size_t>(width_) * height_ * 4;
    hip::check(hipMemsetAsync(frames, 0, fsize * st_batch_, s), "pose clear");
    kernels::PoseDrawArgs da;
    da.kp = static_cast<const float*>(dev_kp_->data());
    da.offsets = offsets;
    da.keypoints = K;
    da.gw = st_gw_;
    da.gh = st_gh_;
    da.i_w = static_cast<int>(i_width_);
    da.i_h = static_cast<int>(i_height_);
    da.W = static_cast<int>(width_);
    da.H = static_cast<int>(height_);
    da.edges = static_cast<const int*>(dev_edges_->data());
    da.n_edges = n_edges_;
    da.labels = static_cast<const char*>(dev_labels_->data());
    da.label_offs = static_cast<const int*>(dev_label_offs_->data());
    da.frames = frames;
    kernels::pose_draw(da, static_cast<int>(st_batch_), s);
  }

 public:
  // ---- device stage (runtime/fusion.h): heatmap argmax + offsets + skeleton
  // raster inside the filter's graph; output = the B RGBA frames [4:W:H:B] ----
  bool stage_prepare(const TensorsConfig& config, int dev, hipStream_t s, TensorsInfo* out) override {
    if (dev < 0 || get_out_caps(config).is_empty()) return false;
    const TensorInfo& hi = config.info.at(0);
    const int K = static_cast<int>(meta_.size());
    for (unsigned i = 0; i < config.info.num_tensors; ++i)
      if (config.info.at(i).type != DType::FLOAT32) return false;
    if (K > 64 || width_ == 0 || height_ == 0 || i_width_ == 0 || i_height_ == 0) return false;
    prepare_device(static_cast<int>(hi.dim[1]), static_cast<int>(hi.dim[2]), hi.dim[3], dev, s);
    st_tensors_ = config.info.num_tensors;
    out->resize(1);
    out->at(0).type = DType::UINT8;
    out->at(0).dim = make_dims({4, width_, height_, hi.dim[3]});
    return true;
  }
  bool stage_enqueue(const std::vector<const void*>& in, const std::vector<void*>& out, hipStream_t s) override {
    if (in.size() != st_tensors_ || out.size() != 1) return false;
    enqueue_device(static_cast<const float*>(in[0]), mode_ == 1 ? static_cast<const float*>(in[1]) : nullptr,
                   static_cast<uint32_t*>(out[0]), s);
    return true;
  }

 private:
  struct Point {
    bool valid = false;
    int x = 0, y = 0;
    float prob = 0;
  };

  bool load_meta(const std::string& path) {
    std::ifstream f(path);
    if (!f) {
      NNSX_LOGW("pose_estimation", "labels file ", path, " does not exist");
      return false;
    }
    std::vector<PoseMeta> m;
    std::string line;
    while (std::getline(f, line)) {
      auto toks = split(strip(line), ' ');
      if (toks.empty() || toks[0].empty()) continue;
      if (toks.size() > 8) toks.resize(8);
      PoseMeta pm;
      pm.label = toks[0].substr(0, 15);
      for (size_t j = 1; j < toks.size(); ++j) pm.connections.push_back(static_cast<int>(to_int(toks[j])));
      m.push_back(pm);
    }
    if (m.empty()) return false;
    meta_ = m;
    dev_edges_.reset();
    return true;
  }

  void ensure_device_meta(int dev, hipStream_t s) {
    if (dev_edges_ && dev_edges_->device() == dev) return;
    std::vector<int> edges;
    const int K = static_cast<int>(meta_.size());
    for (int i = 0; i < K; ++i)
      for (int k : meta_[static_cast<size_t>(i)].connections)
        if (k >= 0 && k < K && k >= i) {
          edges.push_back(i);
          edges.push_back(k);
        }
    n_edges_ = static_cast<int>(edges.size() / 2);
    std::string blob;
    std::vector<int> offs;
    for (auto& m : meta_) {
      offs.push_back(static_cast<int>(blob.size()));
      blob += m.label;
      blob.push_back('\0');
    }
    if (edges.empty()) edges.push_back(0);
    dev_edges_ = Memory::alloc_device(edges.size() * sizeof(int), dev, s);
    dev_labels_ = Memory::alloc_device(blob.size(), dev, s);
    dev_label_offs_ = Memory::alloc_device(offs.size() * sizeof(int), dev, s);
    hip::check(hipMemcpyAsync(dev_edges_->data(), edges.data(), edges.size() * sizeof(int), hipMemcpyHostToDevice, s), "pose edges");
    hip::check(hipMemcpyAsync(dev_labels_->data(), blob.data(), blob.size(), hipMemcpyHostToDevice, s), "pose labels");
    hip::check(hipMemcpyAsync(dev_label_offs_->data(), offs.data(), offs.size() * sizeof(int), hipMemcpyHostToDevice, s),
               "pose label offsets");
    hip::check(hipStreamSynchronize(s), "pose meta");
  }

  void set_pixel(uint32_t* f, int x, int y) const {
    const int W = static_cast<int>(width_), H = static_cast<int>(height_);
    if (x < 0 || x >= W || y < 0 || y >= H) return;
    f[y * W + x] = kPixel;
    if (x + 1 < W) f[y * W + x + 1] = kPixel;
    if (y + 1 < H) f[(y + 1) * W + x] = kPixel;
  }

  void line_with_dots(uint32_t* f, int x1, int y1, int x2, int y2) const {
    // round end dot (radius ~4) at both ends, then a 2-px Bresenham line
    static const int dx_[40] = {-4, 0, 4, 0,  -3, -3, -3, -2, -2, -2, -2, -2, -1, -1, -1, -1, -1, -1, -1, 0,
                                0,  0, 0, 0,  0,  1,  1,  1,  1,  1,  1,  1,  2,  2,  2,  2,  2,  3,  3,  3};
    static const int dy_[40] = {0,  -4, 0,  4,  -1, 0,  1,  -2, -1, 0,  1,  2,  -3, -2, -1, 0,  1,  2,  3,  -3,
                                -2, -1, 1,  2,  3,  -3, -2, -1, 0,  1,  2,  3,  -2, -1, 0,  1,  2,  -1, 0,  1};
    const int W = static_cast<int>(width_), H = static_cast<int>(height_);
    int xs = x1, ys = y1, xe = x2, ye = y2;
    if (x1 > x2) {
      xs = x2;
      ys = y2;
      xe = x1;
      ye = y1;
    }
    for (int i = 0; i < 40; ++i) {
      if (ys + dy_[i] >= 0 && ys + dy_[i] < H && xs + dx_[i] >= 0 && xs + dx_[i] < W)
        f[(ys + dy_[i]) * W + xs + dx_[i]] = kPixel;
      if (ye + dy_[i] >= 0 && ye + dy_[i] < H && xe + dx_[i] >= 0 && xe + dx_[i] < W)
        f[(ye + dy_[i]) * W + xe + dx_[i]] = kPixel;
    }
    const int dx = std::abs(xe - xs), sx = xs < xe ? 1 : -1;
    const int dy = std::abs(ye - ys), sy = ys < ye ? 1 : -1;
    int err = (dx > dy ? dx : -dy) / 2;
    while (true) {
      set_pixel(f, xs, ys);
      if (xs == xe && ys == ye) break;
      const int e2 = err;
      if (e2 > -dx) {
        err -= dy;
        xs += sx;
      }
      if (e2 < dy) {
        err += dx;
        ys += sy;
      }
    }
  }

  void draw(uint32_t* f, std::vector<Point>* pts) const {
    const unsigned K = static_cast<unsigned>(meta_.size());
    for (auto& p : *pts)
      if (p.prob < 0.5f) p.valid = false;
    for (unsigned i = 0; i < K; ++i) {
      if (!(*pts)[i].valid) continue;
      for (int k : meta_[i].connections) {
        if (k < 0 || static_cast<unsigned>(k) >= K || static_cast<unsigned>(k) < i) continue;
        if (!(*pts)[static_cast<size_t>(k)].valid) continue;
        line_with_dots(f, (*pts)[i].x, (*pts)[i].y, (*pts)[static_cast<size_t>(k)].x, (*pts)[static_cast<size_t>(k)].y);
      }
    }
    const int W = static_cast<int>(width_), H = static_cast<int>(height_);
    for (unsigned i = 0; i < K; ++i) {
      if (!(*pts)[i].valid) continue;
      int x1 = (*pts)[i].x;
      const int y1 = std::max(0, (*pts)[i].y - font::kAboveBox);
      for (unsigned char ch : meta_[i].label) {
        if (x1 + 8 > W) break;
        for (int r = 0; r < font::kCellH; ++r)
          for (int c = 0; c < font::kCellW; ++c) {
            const int yy = y1 + r, xx = x1 + c;
            if (yy < H && xx < W) f[yy * W + xx] = font::cell_on(kFontTable, ch, r, c) ? kPixel : 0u;
          }
        x1 += font::kAdvance;
      }
    }
  }

  unsigned width_ = 0, height_ = 0, i_width_ = 0, i_height_ = 0;
  int mode_ = 0;
  std::vector<PoseMeta> meta_;
  MemoryPtr dev_kp_, host_kp_, dev_edges_, dev_labels_, dev_label_offs_;
  int n_edges_ = 0;
  int st_gw_ = 0, st_gh_ = 0;  // the geometry prepare_device saw
  unsigned st_batch_ = 1, st_tensors_ = 1;
};

class PosePlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "pose_estimation"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<PoseEstimation>(); }
};

}  // namespace

void register_segment_decoder() { register_decoder(std::make_shared<ImageSegmentPlugin>()); }
void register_pose_decoder() { register_decoder(std::make_shared<PosePlugin>()); }

}  // namespace nnsx
