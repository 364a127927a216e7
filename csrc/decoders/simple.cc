// Simple decoder sub-plugins: image_labeling, direct_video, octet_stream.
//   image_labeling  ext/nnstreamer/tensor_decoder/tensordec-imagelabel.c:148-240
//   direct_video    ext/nnstreamer/tensor_decoder/tensordec-directvideo.c:20-377
//   octet_stream    ext/nnstreamer/tensor_decoder/tensordec-octetstream.c
// image_labeling runs its argmax as a wave64 reduction on the GPU when the
// logits are HBM-resident (only the winning index crosses PCIe).  nnsx
// extension: a [classes:B] tensor yields B labels, one per line.
#include <cstring>
#include <fstream>

#include "core/cpu_ops.h"
#include "core/log.h"
#include "decoders/decoders.h"
#include "kernels/kernels.h"
#include "runtime/hip_util.h"
#include "runtime/video.h"

namespace nnsx {

std::vector<std::string> load_labels(const std::string& path) {
  std::vector<std::string> labels;
  std::ifstream f(path);
  if (!f) {
    NNSX_LOGE("decoder", "Unable to read label file ", path);
    return labels;
  }
  std::string content((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (!content.empty() && content.back() == '\n') content.pop_back();
  labels = split(content, '\n');
  return labels;
}

void set_framerate_from_config(Caps& caps, const TensorsConfig& config) {
  if (config.rate_n < 0 || config.rate_d <= 0) return;
  for (size_t i = 0; i < caps.size(); ++i) caps.at(i).set("framerate", Value::Fraction(config.rate_n, config.rate_d));
}

namespace {

// --------------------------------------------------------- image_labeling ----
class ImageLabeling : public DecoderInstance {
 public:
  bool set_option(int idx, const std::string& v) override {
    if (idx == 0) {
      labels_ = load_labels(v);
      return !labels_.empty();
    }
    return true;
  }
  Caps get_out_caps(const TensorsConfig& config) override {
    if (config.info.num_tensors < 1) return Caps();
    const auto& d = config.info.at(0).dim;
    if (d[0] == 0) return Caps();
    for (int i = 2; i < kRankLimit; ++i)
      if (d[i] != 1) return Caps();
    Caps c = Caps::from_string("text/x-raw, format=(string)utf8");
    set_framerate_from_config(c, config);
    return c;
  }
  bool supports_device() const override { return true; }
  // the producing filter runs the argmax (runtime/fusion.h): int32 [1:B] indices arrive
  bool accept_argmax_input(uint32_t classes) override {
    if (labels_.empty() || classes == 0) return false;
    indices_ = true;
    return true;
  }
  void drop_argmax_input() override { indices_ = false; }

  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext& ctx) override {
    const TensorInfo& ti = config.info.at(0);
    uint64_t n = ti.dim[0];
    uint32_t batch = ti.dim[1];
    std::vector<int32_t> idx(batch, 0);
    if (indices_ && ti.type == DType::INT32 && n == 1) {
      // only the B indices cross to the host
      if (ctx.device >= 0 && in[0]->on_device()) {
        if (!host_idx_ || host_idx_->size() < batch * sizeof(int32_t))
          host_idx_ = Memory::alloc_pinned(batch * sizeof(int32_t));
        hip::check(hipMemcpyAsync(host_idx_->data(), in[0]->map_device(ctx.device, ctx.stream),
                                  batch * sizeof(int32_t), hipMemcpyDeviceToHost, ctx.stream),
                   "D2H indices");
        hip::check(hipStreamSynchronize(ctx.stream), "sync indices");
        std::memcpy(idx.data(), host_idx_->data(), batch * sizeof(int32_t));
      } else {
        std::memcpy(idx.data(), in[0]->map_host(), batch * sizeof(int32_t));
      }
    } else if (ctx.device >= 0) {
      const void* src = in[0]->map_device(ctx.device, ctx.stream);
      if (!dev_idx_ || dev_idx_->size() < batch * sizeof(int32_t)) {
        dev_idx_ = Memory::alloc_device(batch * sizeof(int32_t), ctx.device, ctx.stream);
        host_idx_ = Memory::alloc_pinned(batch * sizeof(int32_t));
      }
      kernels::argmax_rows(src, ti.type, n, batch, static_cast<int32_t*>(dev_idx_->data()), ctx.stream);
      hip::check(hipMemcpyAsync(host_idx_->data(), dev_idx_->data(), batch * sizeof(int32_t), hipMemcpyDeviceToHost,
                                ctx.stream),
                 "D2H argmax");
      hip::check(hipStreamSynchronize(ctx.stream), "sync argmax");
      std::memcpy(idx.data(), host_idx_->data(), batch * sizeof(int32_t));
    } else {
      const void* p = in[0]->map_host();
      for (uint32_t b = 0; b < batch; ++b) {
        double best = 0;
        int32_t bi = 0;
        for (uint64_t i = 0; i < n; ++i) {
          double v = cpu::read_as_double(p, ti.type, b * n + i);
          if (i == 0 || v > best) {
            best = v;
            bi = static_cast<int32_t>(i);
          }
        }
        idx[b] = bi;
      }
    }
    std::string text;
    for (uint32_t b = 0; b < batch; ++b) {
      if (idx[b] < 0 || static_cast<size_t>(idx[b]) >= labels_.size()) {
        NNSX_LOGE("image_labeling", "label index ", idx[b], " out of range (", labels_.size(), " labels)");
        return FlowReturn::ERROR;
      }
      if (b) text += "\n";
      text += labels_[idx[b]];
    }
    if (text.empty()) return FlowReturn::ERROR;
    out->mems.push_back(Memory::from_bytes(text.data(), text.size()));
    last_index_ = idx.empty() ? -1 : idx[0];
    return FlowReturn::OK;
  }

 private:
  std::vector<std::string> labels_;
  bool indices_ = false;  // argmax absorbed upstream
  MemoryPtr dev_idx_, host_idx_;
  int last_index_ = -1;
};

class ImageLabelingPlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "image_labeling"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<ImageLabeling>(); }
};

// ----------------------------------------------------------- direct_video ----
class DirectVideo : public DecoderInstance {
 public:
  bool set_option(int idx, const std::string& v) override {
    if (idx == 0) format_ = strip(v);
    return true;
  }
  Caps get_out_caps(const TensorsConfig& config) override {
    if (config.info.num_tensors < 1) return Caps();
    const auto& d = config.info.at(0).dim;
    if (config.info.at(0).type != DType::UINT8) return Caps();
    for (int i = 3; i < kRankLimit; ++i)
      if (d[i] != 1) return Caps();
    std::string fmt;
    switch (d[0]) {
      case 1: fmt = "GRAY8"; break;
      case 3: fmt = format_.empty() ? "RGB" : format_; break;
      case 4: fmt = format_.empty() ? "BGRx" : format_; break;
      default: return Caps();
    }
    Caps c = Caps::from_string(strfmt("video/x-raw, format=(string)", fmt, ", width=(int)", d[1], ", height=(int)", d[2]));
    set_framerate_from_config(c, config);
    if (config.rate_n < 0) c.at(0).set("framerate", Value::Fraction(0, 1));
    return c;
  }
  bool supports_device() const override { return true; }
  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext& ctx) override {
    const auto& d = config.info.at(0).dim;
    size_t row = static_cast<size_t>(d[0]) * d[1];
    size_t stride = round_up4(row);
    size_t h = d[2];
    if (stride == row) {
      out->mems.push_back(in[0]->on_device() ? Memory::from_bytes(in[0]->map_host(), in[0]->size()) : in[0]);
      return FlowReturn::OK;
    }
    auto m = Memory::alloc_host(stride * h);
    std::memset(m->data(), 0, stride * h);
    if (in[0]->on_device() && ctx.device >= 0) {
      // pitched D2H (K23)
      in[0]->wait_ready(ctx.stream);
      hip::check(hipMemcpy2DAsync(m->data(), stride, in[0]->data(), row, row, h, hipMemcpyDeviceToHost, ctx.stream),
                 "D2H 2D");
      hip::check(hipStreamSynchronize(ctx.stream), "sync");
    } else {
      const uint8_t* src = static_cast<const uint8_t*>(in[0]->map_host());
      for (size_t y = 0; y < h; ++y) std::memcpy(static_cast<uint8_t*>(m->data()) + y * stride, src + y * row, row);
    }
    out->mems.push_back(m);
    return FlowReturn::OK;
  }

 private:
  std::string format_;
};

class DirectVideoPlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "direct_video"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<DirectVideo>(); }
};

// ----------------------------------------------------------- octet_stream ----
class OctetStream : public DecoderInstance {
 public:
  Caps get_out_caps(const TensorsConfig& config) override {
    Caps c = Caps::from_string("application/octet-stream");
    set_framerate_from_config(c, config);
    return c;
  }
  FlowReturn decode(const TensorsConfig&, const std::vector<MemoryPtr>& in, Buffer* out, InvokeContext&) override {
    size_t total = 0;
    for (auto& m : in) total += m->size();
    auto m = Memory::alloc_host(total);
    size_t off = 0;
    for (auto& x : in) {
      std::memcpy(static_cast<char*>(m->data()) + off, x->map_host(), x->size());
      off += x->size();
    }
    out->mems.push_back(m);
    return FlowReturn::OK;
  }
};

class OctetStreamPlugin : public DecoderSubplugin {
 public:
  std::string name() const override { return "octet_stream"; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<OctetStream>(); }
};

}  // namespace

void register_simple_decoders() {
  register_decoder(std::make_shared<ImageLabelingPlugin>());
  register_decoder(std::make_shared<DirectVideoPlugin>());
  register_decoder(std::make_shared<OctetStreamPlugin>());
}

}  // namespace nnsx
