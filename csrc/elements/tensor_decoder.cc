// tensor_decoder: dispatches `mode=` to a decoder sub-plugin; option1..9 are
// forwarded through set_option(idx).  Reference: gst/nnstreamer/elements/
// gsttensor_decoder.c (registry :133-200, props :286-397, transform :666-742,
// caps :750-907, custom register :936-974).
#include <atomic>
#include <mutex>

#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/fusion.h"
#include "runtime/pipeline.h"
#include "runtime/plugin_api.h"

namespace nnsx {

namespace {

class CustomCodeDecoder : public DecoderInstance {
 public:
  explicit CustomCodeDecoder(DecoderCustomFn fn) : fn_(std::move(fn)) {}
  Caps get_out_caps(const TensorsConfig& config) override {
    (void)config;
    return Caps::Any();
  }
  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext&) override {
    return fn_(in, config, out);
  }

 private:
  DecoderCustomFn fn_;
};

// DecodeStage over a decoder instance: prepared on the filter's device, run by
// the filter inside its graph capture (runtime/fusion.h).  It shares ownership
// of the instance (a mode change replaces the decoder's instance while the
// filter may still hold the stage) and goes stale when the decoder's mode or
// options change (revoke()): the filter then re-takes a stage and re-captures.
class InstanceStage : public DecodeStage {
 public:
  InstanceStage(std::shared_ptr<DecoderInstance> inst, TensorsInfo out) : inst_(std::move(inst)), out_(std::move(out)) {}
  const TensorsInfo& out_info() const override { return out_; }
  bool enqueue(const std::vector<const void*>& in, const std::vector<void*>& out, void* stream) override {
    return inst_->stage_enqueue(in, out, static_cast<hipStream_t>(stream));
  }
  bool stale() const override { return stale_.load(); }
  bool lane_safe() const override { return inst_->stage_lane_safe(); }
  void revoke() { stale_.store(true); }

 private:
  std::shared_ptr<DecoderInstance> inst_;
  TensorsInfo out_;
  std::atomic<bool> stale_{false};
};

class TensorDecoder : public BaseTransform, public ArgmaxConsumer, public DecodeStageConsumer {
 public:
  explicit TensorDecoder(const std::string& name)
      : BaseTransform("tensor_decoder", name, Caps::from_string(tensor_caps_template_all()), Caps::Any()) {
    prop_string("mode", &mode_, "Decoder mode", [this] { load_mode(); });
    for (int i = 0; i < 9; ++i) {
      prop_string("option" + std::to_string(i + 1), &options_[i], "Option " + std::to_string(i + 1) + " of the decoder mode",
                  [this, i] {
                    if (i == 0 && mode_ == "custom-code") return load_mode();  // the callback's name
                    revoke_stage();  // (options are baked into a captured stage)
                    if (inst_ && !inst_->set_option(i, options_[i]))
                      throw Error("decoder " + mode_ + " rejected option" + std::to_string(i + 1) + "=" + options_[i]);
                  });
    }
    prop_readonly("sub-plugins", [] { return join(Registry::get().names(SubpluginKind::DECODER), ","); },
                  "Registrable sub-plugins list");
    prop_string("config-file", &config_file_, "Path to a config file holding option1..9 (key=value lines)", [this] {
      load_config_file();
    });
    prop_int("device", &device_, "nnsx: -2 follow input placement, -1 CPU, N run post-processing kernels on GPU N");
    prop_readonly("argmax-by", [this] { return argmax_by_; },
                  "nnsx: the upstream tensor_filter that runs this decoder's argmax inside its device work "
                  "(runtime/fusion.h; empty: the decoder runs it)");
    prop_readonly("stage-by", [this] { return stage_by_; },
                  "nnsx: the upstream tensor_filter that runs this decoder's device post-processing inside its "
                  "hipGraph (runtime/fusion.h DecodeStage; empty: the decoder runs it)");
  }

  // ---- ArgmaxConsumer (runtime/fusion.h) ----
  bool take_argmax(unsigned tensor, uint32_t classes, const std::string& by) override {
    if (tensor != 0 || !inst_ || !inst_->accept_argmax_input(classes)) return false;
    argmax_by_ = by;
    return true;
  }
  void drop_argmax() override {
    if (inst_) inst_->drop_argmax_input();
    argmax_by_.clear();
  }

  // ---- DecodeStageConsumer (runtime/fusion.h) ----
  std::shared_ptr<DecodeStage> take_stage(const TensorsConfig& model_out, int dev, const std::string& by) override {
    if (!inst_ || dev < 0 || !inst_->supports_device() || !model_out.is_static()) return nullptr;
    if (device_ != -2 && device_ != dev) return nullptr;  // pinned to another device / the host
    if (inst_->get_out_caps(model_out).is_empty()) return nullptr;
    TensorsInfo out;
    hip::DeviceGuard g(dev);
    if (!inst_->stage_prepare(model_out, dev, streams_.get(dev), &out) || out.num_tensors != 1 ||
        out.at(0).type != DType::UINT8 || out.at(0).dim[0] != 4)
      return nullptr;
    auto st = std::make_shared<InstanceStage>(inst_, out);
    std::lock_guard<std::mutex> lk(stage_mu_);
    stage_in_ = model_out;
    stage_by_ = by;
    stage_ = st;
    return st;
  }
  void drop_stage() override {
    std::lock_guard<std::mutex> lk(stage_mu_);
    stage_.reset();
    stage_by_.clear();
  }

 protected:
  void revoke_stage() {
    std::lock_guard<std::mutex> lk(stage_mu_);
    if (auto* st = dynamic_cast<InstanceStage*>(stage_.get())) st->revoke();
  }
  // (the filter's thread takes / drops the stage; this element's thread reads it)
  std::shared_ptr<DecodeStage> current_stage() {
    std::lock_guard<std::mutex> lk(stage_mu_);
    return stage_;
  }
  void load_mode() {
    revoke_stage();
    inst_.reset();
    auto parts = split(mode_, ':', 2);
    // mode=custom-code option1=<name> (the reference's spelling, gsttensor_decoder.c:469,763)
    // or mode=custom-code:<name>
    if (mode_ == "custom-code" && options_[0].empty()) return;  // name follows in option1
    if (mode_ == "custom-code") parts = {"custom-code", options_[0]};
    if (parts.size() == 2 && parts[0] == "custom-code") {
      auto fn = Registry::get().find_as<DecoderCustomFn>(SubpluginKind::CUSTOM_DECODER, parts[1], false);
      if (!fn) throw Error("custom-code decoder '" + parts[1] + "' is not registered");
      inst_ = std::make_unique<CustomCodeDecoder>(*fn);
      return;
    }
    auto d = find_decoder(mode_);
    if (!d) throw Error("tensor_decoder: mode '" + mode_ + "' is not available");
    inst_ = d->create();
    for (int i = 0; i < 9; ++i)
      if (!options_[i].empty() && !inst_->set_option(i, options_[i]))
        throw Error("decoder " + mode_ + " rejected option" + std::to_string(i + 1));
  }

  void load_config_file() {
    // "option1=...\noption2=..." style file
    FILE* f = fopen(config_file_.c_str(), "r");
    if (!f) throw Error("cannot open config-file " + config_file_);
    char line[4096];
    while (fgets(line, sizeof(line), f)) {
      std::string t = strip(line);
      auto eq = t.find('=');
      if (eq == std::string::npos) continue;
      std::string k = strip(t.substr(0, eq));
      if (k == "mode")
        set_property("mode", strip(t.substr(eq + 1)));
      else if (starts_with(k, "option"))
        set_property(k, strip(t.substr(eq + 1)));
    }
    fclose(f);
  }

  Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) override {
    if (dir == PadDirection::SRC) {
      Caps r = sink_pad()->template_caps();
      return filter ? r.intersect(*filter) : r;
    }
    Caps r;
    for (size_t i = 0; i < caps.size(); ++i) {
      TensorsConfig cfg;
      if (!inst_ || !config_from_structure(caps.at(i), &cfg)) {
        r = Caps::Any();
        break;
      }
      if (cfg.is_static() && (cfg.info.num_tensors == 0 || !cfg.info.valid())) {
        r = Caps::Any();
        break;
      }
      // staged: the incoming tensors are the stage's RGBA frames; the media caps
      // follow from the model output the stage was prepared for
      Caps o = inst_->get_out_caps(stage_ ? stage_in_ : cfg);
      if (o.is_empty()) continue;
      r.append(o);
      if (o.is_any()) break;
    }
    if (filter) r = r.intersect(*filter);
    return r;
  }

  Caps fixate_caps(PadDirection, const Caps& caps, Caps othercaps) override {
    (void)caps;
    if (othercaps.is_any()) return othercaps;
    return othercaps.fixate();
  }

  bool set_caps(const Caps& incaps, const Caps& outcaps) override {
    (void)outcaps;
    if (!inst_) {
      NNSX_LOGE(name(), "tensor_decoder: mode is not set");
      return false;
    }
    return tensor_config_from_caps(incaps, &config_);
  }

  FlowReturn transform(const BufferPtr& inbuf, BufferPtr* outbuf) override {
    BufferPtr in;
    if (!buffer_from_config(inbuf, config_, &in)) {
      post_error("tensor_decoder: buffer does not match the negotiated caps");
      return FlowReturn::ERROR;
    }
    TensorsConfig cfg = config_;
    std::vector<MemoryPtr> mems;
    if (config_.is_flexible()) {
      cfg.info.format = Format::STATIC;
      cfg.info.resize(static_cast<unsigned>(in->n_memory()));
      for (size_t i = 0; i < in->n_memory(); ++i) {
        MetaInfo meta;
        MemoryPtr payload;
        if (!parse_flexible(in->mems[i], &meta, &payload)) return FlowReturn::ERROR;
        meta.to_info(&cfg.info.at(static_cast<unsigned>(i)));
        mems.push_back(payload);
      }
    } else {
      mems = in->mems;
    }
    if (current_stage()) {
      // the upstream filter ran this decoder's device stage: [4:W:H:B] RGBA
      // frames, one output buffer per frame (views, no copy)
      const TensorInfo& ti = cfg.info.at(0);
      const unsigned n = std::max<uint32_t>(1, ti.dim[3]);
      const size_t fsize = static_cast<size_t>(ti.dim[0]) * ti.dim[1] * ti.dim[2];
      if (mems.size() != 1 || mems[0]->size() != fsize * n) {
        post_error("tensor_decoder: staged input does not match the stage's output");
        return FlowReturn::ERROR;
      }
      auto out = make_buffer();
      out->copy_metadata_from(*in);
      for (unsigned f = 0; f < n; ++f) out->mems.push_back(Memory::view(mems[0], f * fsize, fsize));
      return push_frames(in, out, n, outbuf);
    }
    InvokeContext ctx;
    ctx.device = inst_->supports_device() ? resolve_device(device_, *in) : -1;
    ctx.stream = ctx.device >= 0 ? streams_.get(ctx.device) : nullptr;
    hip::DeviceGuard g(ctx.device);
    auto out = make_buffer();
    out->copy_metadata_from(*in);
    FlowReturn r = inst_->decode(cfg, mems, out.get(), ctx);
    if (r != FlowReturn::OK) {
      if (r == FlowReturn::CUSTOM_SUCCESS) return r;
      post_error("tensor_decoder: decode failed (" + mode_ + ")");
      return r;
    }
    if (ctx.device >= 0)
      for (auto& m : mems) m->record_use(ctx.stream, ctx.device);
    return push_frames(in, out, ctx.out_frames, outbuf);
  }

  FlowReturn push_frames(const BufferPtr& in, const BufferPtr& out, unsigned frames, BufferPtr* outbuf) {
    if (frames > 1 && out->n_memory() == frames) {
      // batched input: one output buffer per frame, timestamps spread over the batch duration
      const unsigned n = frames;
      const int64_t step = in->duration > 0 ? in->duration / n : 0;
      for (unsigned f = 0; f < n; ++f) {
        auto fb = make_buffer();
        fb->copy_metadata_from(*out);
        fb->mems.push_back(out->mems[f]);
        if (in->pts >= 0) fb->pts = in->pts + step * f;
        if (step > 0) fb->duration = step;
        if (f + 1 == n) {
          *outbuf = fb;
          break;
        }
        FlowReturn r = src_pad()->push(fb);
        if (!flow_ok(r)) return r;
      }
      return FlowReturn::OK;
    }
    *outbuf = out;
    return FlowReturn::OK;
  }

  std::string mode_, options_[9], config_file_;
  int device_ = -2;
  std::shared_ptr<DecoderInstance> inst_;
  std::string argmax_by_;
  std::mutex stage_mu_;
  std::shared_ptr<DecodeStage> stage_;  // run upstream by stage_by_ (take_stage)
  TensorsConfig stage_in_;              // the model output the stage was prepared for
  std::string stage_by_;
  TensorsConfig config_;
  StreamSet streams_;
};

}  // namespace

void register_tensor_decoder() {
  register_element("tensor_decoder", "Converter/Tensor", "Converts tensors to media streams via decoder sub-plugins",
                   [](const std::string& n) { return std::make_unique<TensorDecoder>(n); });
}

}  // namespace nnsx
