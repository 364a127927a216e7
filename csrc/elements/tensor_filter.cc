// tensor_filter: runs a framework sub-plugin on every buffer.
// Reference: gst/nnstreamer/tensor_filter/tensor_filter.c (validate :558-626,
// transform :632-894, statistics :354-495, configure :903-1086,
// transform_caps :1099-1215, latency query :1314-1376, model update event
// :1414-1446, QoS throttle :1455-1485) and tensor_filter_common.c
// (properties :899-1017, combinations :1815-1885, shared models :2911-3076,
// accelerator grammar :2495-2800).
//
// nnsx: frameworks receive Memory objects plus the element's HIP stream and
// device; GPU frameworks consume device memories in place and return
// device-resident, allocate-in-invoke outputs (no per-frame PCIe copies).
#include <algorithm>
#include <cmath>
#include <deque>

#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/fusion.h"
#include "runtime/pipeline.h"
#include "runtime/plugin_api.h"

namespace nnsx {

namespace {

// shared-tensor-filter-key table (tensor_filter_common.c:2911-3076)
struct SharedModel {
  std::shared_ptr<FilterInstance> inst;
  std::mutex invoke_mu;
  int refs = 0;
};
std::mutex g_shared_mu;
std::map<std::string, std::shared_ptr<SharedModel>> g_shared;

std::vector<int> field_ranks(const std::string& dims) {
  std::vector<int> v;
  for (auto& d : split_any(dims, ",.")) {
    Dims tmp{};
    v.push_back(static_cast<int>(parse_dimension(d, tmp)));
  }
  return v;
}

std::vector<int> parse_ranks(const std::string& s) {
  std::vector<int> v;
  for (auto& x : split(s, ','))
    if (!strip(x).empty()) v.push_back(static_cast<int>(to_int(x)));
  return v;
}

class TensorFilter : public BaseTransform, public TransformAbsorber {
 public:
  explicit TensorFilter(const std::string& name)
      : BaseTransform("tensor_filter", name, Caps::from_string(tensor_caps_template_all()),
                      Caps::from_string(tensor_caps_template_all())) {
    prop_string("framework", &fw_name_, "Neural network framework", [this] { on_framework_set(); });
    prop_string("model", &model_str_, "File path to the model file. Separated with ',' in case of multiple model files",
                [this] { on_model_set(); });
    prop_string("input", &input_str_, "Input tensor dimension from inner array, up to 8 dimensions ?", [this] {
      unsigned n = props_.input_info.parse_dimensions(input_str_);
      props_.input_info.num_tensors = std::max(props_.input_info.num_tensors, n);
      // the rank of each tensor is the number of fields written (tensor_filter_common.c:1490-1505)
      if (inputranks_str_.empty()) props_.input_ranks = field_ranks(input_str_);
      notify_io(true);
    });
    prop_string("inputtype", &inputtype_str_, "Type of each element of the input tensor ?", [this] {
      unsigned n = props_.input_info.parse_types(inputtype_str_);
      props_.input_info.num_tensors = std::max(props_.input_info.num_tensors, n);
      notify_io(true);
    });
    prop_string("inputname", &inputname_str_, "The Name of Input Tensor", [this] { props_.input_info.parse_names(inputname_str_); });
    prop_string("inputlayout", &props_.input_layout, "Set channel first (NCHW) or channel last layout (NHWC) or None for input data");
    prop_string("inputranks", &inputranks_str_, "The Rank of the Input Tensor", [this] { props_.input_ranks = parse_ranks(inputranks_str_); });
    prop_string("output", &output_str_, "Output tensor dimension from inner array, up to 8 dimensions ?", [this] {
      unsigned n = props_.output_info.parse_dimensions(output_str_);
      props_.output_info.num_tensors = std::max(props_.output_info.num_tensors, n);
      if (outputranks_str_.empty()) props_.output_ranks = field_ranks(output_str_);
      notify_io(false);
    });
    prop_string("outputtype", &outputtype_str_, "Type of each element of the output tensor ?", [this] {
      unsigned n = props_.output_info.parse_types(outputtype_str_);
      props_.output_info.num_tensors = std::max(props_.output_info.num_tensors, n);
      notify_io(false);
    });
    prop_string("outputname", &outputname_str_, "The Name of Output Tensor", [this] { props_.output_info.parse_names(outputname_str_); });
    prop_string("outputlayout", &props_.output_layout, "Set channel first (NCHW) or channel last layout (NHWC) or None for output data");
    prop_string("outputranks", &outputranks_str_, "The Rank of the Out Tensor", [this] { props_.output_ranks = parse_ranks(outputranks_str_); });
    prop_string("custom", &props_.custom_properties, "Custom properties for subplugins ?", [this] {
      // an open framework hears about it (V1 CUSTOM_PROP, tensor_filter_common.c _gtfc_setprop_CUSTOM)
      if (inst_ && !inst_->update_custom(props_.custom_properties))
        NNSX_LOGD(this->name(), "framework did not take the new custom properties");
    });
    prop_readonly("sub-plugins", [] { return join(Registry::get().names(SubpluginKind::FILTER), ","); },
                  "Registrable sub-plugins list");
    prop_string("accelerator", &props_.accl_str, "Set accelerator for the subplugin with format (true/false):(comma separated ACCELERATOR(s)). true/false determines if accelerator is to be used. list of accelerators determines the backend (ignored with false). Example, if GPU, NPU can be used but not CPU - true:npu,gpu,!cpu.",
                [this] {
                  if (inst_ && fw_) {  // V1 SET_ACCELERATOR with the list the framework supports
                    bool use = false;
                    parse_accelerator(props_.accl_str, fw_->accelerators(), &use);
                    if (!inst_->update_accelerator(use ? fw_->accelerators() : std::string("cpu")))
                      NNSX_LOGD(this->name(), "framework did not take the accelerator change");
                  }
                });
    prop_bool("is-updatable", &props_.is_updatable, "Indicate whether a given model to this tensor filter is updatable in runtime. (e.g., with on-device training)");
    {
      PropSpec s;
      s.name = "latency";
      s.type = PropType::INT;
      s.blurb = "The average latency over the recent 10 inferences in microseconds (write 1 to enable, 0 to disable; -1 when disabled)";
      s.set = [this](const std::string& v) { latency_mode_ = static_cast<int>(to_int(v)); };
      s.get = [this] { return std::to_string(latency_mode_ == 1 ? avg_latency_us() : -1); };
      add_prop(s);
    }
    {
      PropSpec s;
      s.name = "throughput";
      s.type = PropType::INT;
      s.blurb = "The average throughput in frames per second x 1000 (write 1 to enable, 0 to disable; -1 when disabled)";
      s.set = [this](const std::string& v) { throughput_mode_ = static_cast<int>(to_int(v)); };
      s.get = [this] { return std::to_string(throughput_mode_ == 1 ? throughput_milli_fps() : -1); };
      add_prop(s);
    }
    prop_string("input-combination", &input_comb_str_, "Select the input tensor(s) to invoke the models", [this] {
      input_comb_.clear();
      for (auto& x : split(input_comb_str_, ','))
        if (!strip(x).empty()) input_comb_.push_back(static_cast<int>(to_int(x)));
    });
    prop_string("output-combination", &output_comb_str_, "Select the output tensor(s) in the input tensor(s) and/or model output (e.g. i0,o0,o1)",
                [this] { parse_output_combination(); });
    prop_string("shared-tensor-filter-key", &props_.shared_key, "Multiple element instances of tensor-filter in a pipeline may share a single resource instance if they share the same framework (subplugin) and neural network model. Designate \"shared-tensor-filter-key\" for such elements.");
    prop_bool("latency-report", &latency_report_, "Report the latency of tensor filter to the pipeline bus (LATENCY message)");
    prop_int("invoke-dynamic", &props_.invoke_dynamic, "Flexible tensors whose shape can change per invoke (output caps become flexible)");
    prop_int("device", &device_prop_, "nnsx: GPU index for GPU frameworks (-2 = follow input placement, else LOCAL_RANK or 0)");
    prop_bool("device-stats", &device_stamps_,
              "nnsx: log every GPU invoke's device time (HIP events); read back with device-stamps");
    prop_readonly("device-stamps", [this] {
      poll_device_stats(true);
      std::lock_guard<std::mutex> lk(stat_mu_);
      std::string r;
      for (auto& e : dev_log_) r += std::to_string(e.first) + ":" + std::to_string(e.second) + ",";
      return r;
    }, "nnsx: per-invoke 'end_ns:latency_ns' on the device clock (relative to the first invoke), comma separated");
    prop_string("config-file", &config_file_, "Path to a key=value file setting any of the properties", [this] { load_config_file(); });
    prop_bool("absorb-transform", &absorb_enabled_,
              "nnsx: fold an adjacent upstream tensor_transform (uint8 -> float32 elementwise arithmetic) into the "
              "model when the model maps uint8 frames through an input table");
    prop_readonly("lowered", [this] { return inst_ ? inst_->info("lowered") : std::string(); },
                  "nnsx (framework=pytorch): what the load-time lowering of a plain model onto the nnsx kernels "
                  "did ('' = not lowered)");
    prop_readonly("model-broadcast", [this] { return inst_ ? inst_->info("model-broadcast") : std::string(); },
                  "nnsx: '<data plane>:<members>:<bytes>' when the model arrived by a rank-group broadcast "
                  "(custom=broadcast:<root>)");
    prop_readonly("absorbed", [this] { return absorbed_from_; },
                  "nnsx: name of the tensor_transform absorbed at caps negotiation (empty: none)");
    prop_bool("absorb-decoder", &absorb_dec_enabled_,
              "nnsx: run an adjacent downstream image_labeling decoder's argmax at the end of the model's device "
              "work (inside its hipGraph); the decoder then receives int32 indices");
    prop_readonly("absorbed-decoder", [this] { return absorbed_decoder_; },
                  "nnsx: name of the tensor_decoder whose argmax this filter runs (empty: none)");
  }

  // V1 SET_INPUT_PROP / SET_OUTPUT_PROP once the framework is open
  void notify_io(bool input) {
    if (!inst_) return;
    const TensorsInfo& ti = input ? props_.input_info : props_.output_info;
    if (ti.num_tensors > 0 && ti.valid() && !inst_->update_io_info(input, ti))
      NNSX_LOGD(name(), "framework did not take the new ", input ? "input" : "output", " info");
  }

  // ---- TransformAbsorber (runtime/fusion.h) ----
  bool absorb_arith(const ArithPrefix& p, const std::string& by) override {
    if (!inst_ || !input_comb_.empty() || p.in_type != DType::UINT8 || p.out_type != DType::FLOAT32) return false;
    // the table belongs to the model instance: rewriting it for an instance shared
    // by key would change the input mapping of every other element using it
    if (shared_) return false;
    if (!inst_->accepts_input_table(p.tensor)) return false;
    std::vector<float> lut;
    if (!arith_table_u8(p.params, p.out_type, &lut)) return false;
    if (!inst_->set_input_table(p.tensor, lut)) return false;
    // the model input is now the transform's input: uint8
    if (props_.input_info.num_tensors > p.tensor) props_.input_info.at(p.tensor).type = DType::UINT8;
    if (model_in_.num_tensors > p.tensor) model_in_.at(p.tensor).type = DType::UINT8;
    absorbed_from_ = by;
    NNSX_LOGI(name(), "absorbed ", by, " into the model's uint8 input table");
    return true;
  }

  // walk upstream through queues to an absorbable element (tensor_transform)
  void attach_absorbable() {
    detach_absorbable();
    if (!absorb_enabled_ || !inst_ || !inst_->accepts_input_table(0)) return;
    Pad* sp = sink_pad(0);
    Element* up = sp && sp->peer() ? sp->peer()->parent() : nullptr;
    while (up && up->factory() == "queue") {
      Pad* s = up->sink_pad(0);
      up = s && s->peer() ? s->peer()->parent() : nullptr;
    }
    if (auto* ab = dynamic_cast<AbsorbableElement*>(up)) {
      ab->set_absorber(this);
      absorbable_up_ = ab;
    }
  }
  void detach_absorbable() {
    if (absorbable_up_) absorbable_up_->set_absorber(nullptr);
    absorbable_up_ = nullptr;
    if (!absorbed_from_.empty()) {
      // undo the absorption: the model's own input table and model-reported
      // input info again, so a restart with another upstream negotiates afresh
      if (inst_ && !inst_->reset_input_table(0))
        NNSX_LOGW(name(), "could not restore the model's input table after releasing ", absorbed_from_);
      absorbed_from_.clear();
      if (inst_) load_model_info();
    }
  }

  ~TensorFilter() override {
    release_timing_events();
    close_fw();
  }

 protected:
  // ------------------------------------------------------------ properties ----
  void on_framework_set() {
    if (inst_) close_fw();
    fw_.reset();
  }

  void on_model_set() {
    std::vector<std::string> models;
    for (auto& m : split(model_str_, ','))
      if (!strip(m).empty()) models.push_back(strip(m));
    bool reload = inst_ && props_.is_updatable && models != props_.model_files;
    props_.model_files = models;
    if (reload) {
      FilterProperties np = props_;
      if (!inst_->reload_model(np)) post_error("tensor_filter: model reload failed");
    }
  }

  void load_config_file() {
    FILE* f = fopen(config_file_.c_str(), "r");
    if (!f) throw Error("cannot open config-file " + config_file_);
    char line[8192];
    while (fgets(line, sizeof(line), f)) {
      std::string t = strip(line);
      if (t.empty() || t[0] == '#') continue;
      auto eq = t.find('=');
      if (eq == std::string::npos) continue;
      set_property(strip(t.substr(0, eq)), strip(t.substr(eq + 1)));
    }
    fclose(f);
  }

  void parse_output_combination() {
    out_comb_.clear();
    for (auto& x : split(output_comb_str_, ',')) {
      std::string t = strip(x);
      if (t.empty()) continue;
      if (t[0] != 'i' && t[0] != 'o') throw Error("output-combination: invalid token " + t);
      out_comb_.emplace_back(t[0] == 'i', static_cast<int>(to_int(t.substr(1))));
    }
  }

  // -------------------------------------------------------------- framework ----
  bool ensure_open() {
    if (inst_) return true;
    std::lock_guard<std::mutex> lk(open_mu_);
    if (inst_) return true;
    std::string err;
    fw_ = resolve_filter_framework(fw_name_, &props_, device_prop_, &err);
    if (!fw_) {
      NNSX_LOGE(name(), "tensor_filter: ", err, " (model '", model_str_, "')");
      return false;
    }
    const std::string fwn = props_.fwname;
    if (!props_.shared_key.empty()) {
      std::lock_guard<std::mutex> lk2(g_shared_mu);
      auto it = g_shared.find(props_.shared_key);
      if (it != g_shared.end()) {
        shared_ = it->second;
        shared_->refs++;
        inst_ = shared_->inst;
        return true;
      }
    }
    try {
      inst_ = std::shared_ptr<FilterInstance>(fw_->open(props_).release());
    } catch (const std::exception& e) {
      NNSX_LOGE(name(), "tensor_filter: failed to open framework ", fwn, ": ", e.what());
      inst_.reset();
      return false;
    }
    if (!inst_) return false;
    if (!props_.shared_key.empty()) {
      std::lock_guard<std::mutex> lk2(g_shared_mu);
      auto sm = std::make_shared<SharedModel>();
      sm->inst = inst_;
      sm->refs = 1;
      g_shared[props_.shared_key] = sm;
      shared_ = sm;
    }
    load_model_info();
    return true;
  }

  void close_fw() {
    if (shared_) {
      std::lock_guard<std::mutex> lk(g_shared_mu);
      if (--shared_->refs == 0) g_shared.erase(props_.shared_key);
      shared_.reset();
    }
    inst_.reset();
  }

  void load_model_info() {
    TensorsInfo in, out;
    model_info_known_ = inst_->get_model_info(&in, &out);
    if (model_info_known_) {
      // properties given by the user must agree with the model (gst_tensor_filter_load_tensor_info)
      if (props_.input_info.num_tensors > 0 && props_.input_info.valid() && !(in == props_.input_info)) {
        NNSX_LOGW(name(), "input property (", props_.input_info.to_string(), ") differs from model (", in.to_string(), ")");
      }
      model_in_ = in;
      model_out_ = out;
    } else {
      model_in_ = props_.input_info;
      model_out_ = props_.output_info;
    }
  }

  // -------------------------------------------------------------------- caps ----
  TensorsInfo combined_in(const TensorsInfo& full) const {
    if (input_comb_.empty()) return full;
    TensorsInfo r;
    r.format = full.format;
    r.resize(static_cast<unsigned>(input_comb_.size()));
    for (size_t i = 0; i < input_comb_.size(); ++i) r.at(static_cast<unsigned>(i)) = full.at(static_cast<unsigned>(input_comb_[i]));
    return r;
  }

  // ---- argmax absorption (runtime/fusion.h ArgmaxConsumer) ----
  // A single float score tensor [classes:B] feeding (through queues) a decoder
  // that starts with an argmax: the framework appends the argmax to its device
  // work and the tensor leaves as int32 indices [1:B].
  void absorb_decoder_argmax(TensorsInfo* mout) {
    if (!argmax_tried_) {
      argmax_tried_ = true;
      const bool fp = mout->num_tensors == 1 &&
                      (mout->at(0).type == DType::FLOAT32 || mout->at(0).type == DType::FLOAT16 ||
                       mout->at(0).type == DType::FLOAT64 || mout->at(0).type == DType::BFLOAT16);
      bool shape_ok = fp && mout->at(0).dim[0] > 1;
      for (int r = 2; shape_ok && r < kRankLimit; ++r) shape_ok = mout->at(0).dim[r] <= 1;
      if (absorb_dec_enabled_ && inst_ && !shared_ && out_comb_.empty() && !props_.invoke_dynamic && shape_ok &&
          inst_->accepts_output_argmax(0)) {
        Pad* sp = src_pad();
        Element* dn = sp && sp->peer() ? sp->peer()->parent() : nullptr;
        while (dn && dn->factory() == "queue") {
          Pad* q = dn->src_pad();
          dn = q && q->peer() ? q->peer()->parent() : nullptr;
        }
        if (auto* c = dynamic_cast<ArgmaxConsumer*>(dn)) {
          if (c->take_argmax(0, mout->at(0).dim[0], name())) {
            if (inst_->set_output_argmax(0, true)) {
              argmax_consumer_ = c;
              absorbed_decoder_ = dn->name();
              NNSX_LOGI(name(), "runs the argmax of ", absorbed_decoder_, " at the end of its device work");
            } else {
              c->drop_argmax();
            }
          }
        }
      }
    }
    if (argmax_consumer_ && mout->num_tensors >= 1) {
      mout->at(0).type = DType::INT32;
      mout->at(0).dim[0] = 1;
    }
  }

  // ---- decode-stage absorption (runtime/fusion.h DecodeStage) ----
  // A downstream decoder whose whole device post-processing can run inside this
  // filter's captured graph (bounding_boxes, image_segment, pose_estimation):
  // the model outputs never leave the graph, the decoded RGBA frames do.
  void absorb_decoder_stage(TensorsInfo* mout, const TensorsConfig& in) {
    if (!stage_tried_) {
      stage_tried_ = true;
      const int dev = inst_ ? inst_->stage_device() : -1;
      if (absorb_dec_enabled_ && inst_ && dev >= 0 && !shared_ && !argmax_consumer_ && out_comb_.empty() &&
          !props_.invoke_dynamic && mout->num_tensors > 0 && mout->valid()) {
        Pad* sp = src_pad();
        Element* dn = sp && sp->peer() ? sp->peer()->parent() : nullptr;
        while (dn && dn->factory() == "queue") {
          Pad* q = dn->src_pad();
          dn = q && q->peer() ? q->peer()->parent() : nullptr;
        }
        if (auto* c = dynamic_cast<DecodeStageConsumer*>(dn)) {
          TensorsConfig mc;
          mc.info = *mout;
          mc.info.format = Format::STATIC;
          mc.rate_n = in.rate_n;
          mc.rate_d = in.rate_d;
          if (auto st = c->take_stage(mc, dev, name())) {
            if (inst_->set_output_stage(st)) {
              stage_consumer_ = c;
              stage_ = st;
              stage_model_out_ = mc;
              absorbed_decoder_ = dn->name();
              NNSX_LOGI(name(), "runs the device post-processing of ", absorbed_decoder_, " inside its graph");
            } else {
              c->drop_stage();
            }
          }
        }
      }
    }
    if (stage_) *mout = stage_->out_info();
  }
  // the decoder's mode / options changed after its stage was captured: take a
  // fresh stage for the same model outputs (the filter re-captures its graphs);
  // false when the decoder no longer offers one with the same output
  bool refresh_decoder_stage() {
    const TensorsConfig mc = stage_model_out_;
    const TensorsInfo old = stage_->out_info();
    const int dev = inst_->stage_device();
    inst_->set_output_stage(nullptr);
    {
      // replays of the old graphs may still read the stage's scratch, which
      // re-preparing the stage replaces (a rare event: a sync is fine)
      hip::DeviceGuard g(dev);
      hip::check(hipDeviceSynchronize(), "decoder stage refresh");
    }
    stage_.reset();
    // (the decoder swaps its stage in take_stage: it never sees none in between)
    auto st = stage_consumer_->take_stage(mc, dev, name());
    if (!st || !(st->out_info() == old) || !inst_->set_output_stage(st)) {
      if (st) stage_consumer_->drop_stage();
      stage_consumer_ = nullptr;
      return false;
    }
    stage_ = st;
    NNSX_LOGI(name(), "re-took the device post-processing of ", absorbed_decoder_, " (decoder options changed)");
    return true;
  }
  void release_decoder_stage() {
    if (stage_consumer_) {
      if (inst_) inst_->set_output_stage(nullptr);
      stage_consumer_->drop_stage();
    }
    stage_consumer_ = nullptr;
    stage_.reset();
    stage_tried_ = false;
  }
  void release_decoder_argmax() {
    if (argmax_consumer_) {
      argmax_consumer_->drop_argmax();
      if (inst_) inst_->set_output_argmax(0, false);
    }
    argmax_consumer_ = nullptr;
    absorbed_decoder_.clear();
    argmax_tried_ = false;
  }

  bool output_info_for(const TensorsConfig& in, TensorsInfo* out) {
    TensorsInfo min = combined_in(in.info);
    TensorsInfo mout;
    if (model_info_known_ && (model_in_ == min || min.format != Format::STATIC)) {
      mout = model_out_;
    } else {
      if (!inst_->set_input_info(min, &mout)) {
        if (model_info_known_) {
          NNSX_LOGE(name(), "tensor_filter: input ", min.to_string(), " does not match model input ", model_in_.to_string());
          return false;
        }
        if (props_.output_info.num_tensors > 0 && props_.output_info.valid()) {
          mout = props_.output_info;
        } else {
          NNSX_LOGE(name(), "tensor_filter: cannot determine output info for ", min.to_string());
          return false;
        }
      }
    }
    if (out_comb_.empty()) {
      absorb_decoder_argmax(&mout);
      absorb_decoder_stage(&mout, in);
      *out = mout;
      return true;
    }
    TensorsInfo r;
    r.resize(static_cast<unsigned>(out_comb_.size()));
    for (size_t i = 0; i < out_comb_.size(); ++i) {
      const auto& c = out_comb_[i];
      r.at(static_cast<unsigned>(i)) = c.first ? in.info.at(static_cast<unsigned>(c.second)) : mout.at(static_cast<unsigned>(c.second));
    }
    *out = r;
    return true;
  }

  Caps transform_caps(PadDirection dir, const Caps& caps, const Caps* filter) override {
    if (!ensure_open()) return Caps();
    Caps r;
    if (dir == PadDirection::SRC) {
      TensorsConfig c;
      c.info = model_in_;
      if (model_in_.num_tensors > 0 && model_in_.valid() && input_comb_.empty()) {
        for (size_t i = 0; i < caps.size(); ++i) {
          TensorsConfig oc;
          if (config_from_structure(caps.at(i), &oc) && oc.rate_n >= 0) {
            c.rate_n = oc.rate_n;
            c.rate_d = oc.rate_d;
          }
        }
        r = caps_from_config(c);
        r.append(Caps::from_string(tensor_caps_template_flexible()));
      } else {
        r = Caps::from_string(tensor_caps_template_all());
      }
    } else {
      for (size_t i = 0; i < caps.size(); ++i) {
        TensorsConfig in;
        if (!config_from_structure(caps.at(i), &in)) continue;
        if (in.is_static() && (in.info.num_tensors == 0 || !in.info.valid())) {
          r.append(Caps::from_string(tensor_caps_template_all()));
          continue;
        }
        TensorsInfo out;
        if (in.is_flexible() && !model_info_known_) {
          r.append(Caps::from_string(tensor_caps_template_flexible()));
          continue;
        }
        if (!output_info_for(in, &out)) continue;
        TensorsConfig oc;
        oc.info = out;
        oc.rate_n = in.rate_n;
        oc.rate_d = in.rate_d;
        if (props_.invoke_dynamic) oc.info.format = Format::FLEXIBLE;
        r.append(caps_from_config(oc, props_.device >= 0));
        if (!props_.invoke_dynamic) {
          TensorsConfig fc = oc;
          fc.info.format = Format::FLEXIBLE;
          r.append(caps_from_config(fc));
        }
      }
    }
    if (filter) r = r.intersect(*filter);
    return r;
  }

  Caps fixate_caps(PadDirection, const Caps& caps, Caps othercaps) override {
    TensorsConfig in;
    if (caps.size() && config_from_structure(caps.at(0), &in) && othercaps.size() > 0) {
      TensorsConfig oc;
      if (config_from_structure(othercaps.at(0), &oc)) {
        Caps peer = src_pad()->peer_query_caps(nullptr);
        return pad_caps_from_config(oc, &peer, props_.device >= 0);
      }
    }
    return othercaps.fixate();
  }

  bool set_caps(const Caps& incaps, const Caps& outcaps) override {
    if (!ensure_open()) return false;
    if (!tensor_config_from_caps(incaps, &in_config_) || !tensor_config_from_caps(outcaps, &out_config_)) return false;
    in_flexible_ = in_config_.is_flexible();
    out_flexible_ = out_config_.is_flexible();
    if (in_flexible_ && out_flexible_ && !model_info_known_ && props_.input_info.num_tensors == 0 &&
        !props_.invoke_dynamic) {
      NNSX_LOGE(name(), "tensor_filter: flexible -> flexible needs the model I/O or input/output properties");
      return false;
    }
    if (!in_flexible_) {
      TensorsInfo out;
      if (!output_info_for(in_config_, &out)) return false;
      model_out_runtime_ = out;
    } else {
      model_out_runtime_ = model_out_;
    }
    configured_ = true;
    return true;
  }

  // ------------------------------------------------------------------ events ----
  bool handle_sink_event(Event& ev) override {
    if (ev.type == EventType::CUSTOM_DOWNSTREAM && ev.data.name() == "evt_update_model") {
      std::string m = ev.data.get_string_or("model", "");
      if (!m.empty() && inst_) {
        props_.model_files = split(m, ',');
        model_str_ = m;
        if (!inst_->reload_model(props_)) post_error("tensor_filter: failed to update the model");
      }
      return false;  // consumed
    }
    return true;
  }

  bool handle_src_event(Event& ev) override {
    if (ev.type == EventType::QOS && ev.qos_type == "throttle") {
      throttle_delay_ = ev.diff > 0 ? ev.diff : 0;
      return true;  // keep propagating upstream like the reference
    }
    return true;
  }


  // ---------------------------------------------------------------- transform ----
  FlowReturn transform(const BufferPtr& inbuf, BufferPtr* outbuf) override {
    if (!configured_ || !inst_) {
      post_error("tensor_filter: not configured");
      return FlowReturn::NOT_NEGOTIATED;
    }
    if (stage_ && stage_->stale() && !refresh_decoder_stage()) {
      post_error("tensor_filter: the absorbed decoder changed its output while playing (" + absorbed_decoder_ +
                 "); restart the pipeline");
      return FlowReturn::ERROR;
    }
    // QoS throttling drop (tensor_filter.c:501-552)
    if (throttle_delay_ > 0 && inbuf->pts >= 0) {
      if (prev_ts_ >= 0 && inbuf->pts - prev_ts_ < throttle_delay_) return FlowReturn::CUSTOM_SUCCESS;
      prev_ts_ = inbuf->pts;
    }
    BufferPtr in;
    if (!buffer_from_config(inbuf, in_config_, &in)) {
      post_error("tensor_filter: input buffer does not match the negotiated caps");
      return FlowReturn::ERROR;
    }
    std::vector<MemoryPtr> all_in;
    if (in_flexible_) {
      for (auto& m : in->mems) {
        MetaInfo meta;
        MemoryPtr payload;
        if (!parse_flexible(m, &meta, &payload)) return FlowReturn::ERROR;
        all_in.push_back(payload);
      }
    } else {
      all_in = in->mems;
    }
    std::vector<MemoryPtr> model_in;
    if (input_comb_.empty()) {
      model_in = all_in;
    } else {
      for (int i : input_comb_) {
        if (i < 0 || static_cast<size_t>(i) >= all_in.size()) return FlowReturn::ERROR;
        model_in.push_back(all_in[i]);
      }
    }
    InvokeContext ctx;
    ctx.device = props_.device;
    if (device_prop_ == -2 && ctx.device >= 0) {
      int d = resolve_device(-2, *in);
      if (d >= 0) ctx.device = d;
    }
    ctx.stream = ctx.device >= 0 ? streams_.get(ctx.device) : nullptr;
    TensorsInfo dyn_out;
    ctx.out_info = &dyn_out;
    std::vector<MemoryPtr> outs;
    int64_t t0 = now_ns();
    int ret;
    // GPU invokes are asynchronous: statistics come from HIP events around
    // the invoke on the element's stream (device time), not host enqueue time
    const bool dev_timing = ctx.device >= 0 && ctx.stream && stats_enabled();
    DevStamp ds;
    {
      hip::DeviceGuard g(ctx.device);
      if (dev_timing) {
        poll_device_stats(false);
        ds = dev_stamp_begin(ctx.device, ctx.stream);
      }
      if (shared_) {
        std::lock_guard<std::mutex> lk(shared_->invoke_mu);
        ret = inst_->invoke(model_in, &outs, ctx);
      } else {
        ret = inst_->invoke(model_in, &outs, ctx);
      }
      if (dev_timing) dev_stamp_end(&ds, ctx.done_stream ? ctx.done_stream : ctx.stream, ret);
    }
    int64_t t1 = now_ns();
    if (!dev_timing) record_stats(t1 - t0, t1);
    if (ret > 0) return FlowReturn::CUSTOM_SUCCESS;  // drop this frame (tensor_filter.c:811-813)
    if (ret < 0) {
      post_error(strfmt("tensor_filter: invoke failed (", ret, ")"));
      return FlowReturn::ERROR;
    }
    auto out = make_buffer();
    out->copy_metadata_from(*in);
    auto add = [&](const MemoryPtr& m, const TensorInfo* ti) {
      if (out_flexible_) {
        TensorInfo info = ti ? *ti : TensorInfo();
        if (!ti || !dimension_valid(info.dim)) {
          info.type = DType::UINT8;
          info.dim = make_dims({static_cast<uint32_t>(m->size())});
        }
        out->mems.push_back(make_flexible(m, MetaInfo::from_info(info)));
      } else {
        out->mems.push_back(m);
      }
    };
    const TensorsInfo& oinfo = dyn_out.num_tensors ? dyn_out : model_out_;
    if (out_comb_.empty()) {
      for (size_t i = 0; i < outs.size(); ++i) add(outs[i], i < oinfo.num_tensors ? &oinfo.at(static_cast<unsigned>(i)) : nullptr);
    } else {
      for (const auto& c : out_comb_) {
        if (c.first) {
          if (static_cast<size_t>(c.second) >= all_in.size()) return FlowReturn::ERROR;
          const TensorInfo* ti = in_flexible_ ? nullptr : &in_config_.info.at(static_cast<unsigned>(c.second));
          add(all_in[c.second], ti);
        } else {
          if (static_cast<size_t>(c.second) >= outs.size()) return FlowReturn::ERROR;
          add(outs[c.second], static_cast<unsigned>(c.second) < oinfo.num_tensors ? &oinfo.at(static_cast<unsigned>(c.second)) : nullptr);
        }
      }
    }
    *outbuf = out;
    return FlowReturn::OK;
  }

  // ---------------------------------------------------------------- stats ----
  // Reference: tensor_filter.c:354-495 (latency = invoke duration, throughput
  // from the invoke timestamps).  On a GPU the invoke only enqueues work, so a
  // pair of timing events brackets it on the element's stream: latency = the
  // device time between them, the "timestamp" of an invoke = its end event on
  // the device clock (relative to the first event this element recorded).
  struct DevStamp {
    hipEvent_t beg = nullptr, end = nullptr;
    int dev = -1;
  };
  bool stats_enabled() const { return latency_mode_ > 0 || throughput_mode_ > 0 || latency_report_ || device_stamps_; }

  hipEvent_t timing_event(int dev) {
    std::lock_guard<std::mutex> lk(stat_mu_);
    if (!ev_free_.empty()) {
      hipEvent_t e = ev_free_.back();
      ev_free_.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    hip::check(hipEventCreate(&e), "hipEventCreate(timing)");
    ev_all_.emplace_back(dev, e);
    return e;
  }

  DevStamp dev_stamp_begin(int dev, hipStream_t s) {
    DevStamp d;
    d.dev = dev;
    d.beg = timing_event(dev);
    d.end = timing_event(dev);
    hip::check(hipEventRecord(d.beg, s), "hipEventRecord(invoke begin)");
    std::lock_guard<std::mutex> lk(stat_mu_);
    if (!ev_base_) {
      ev_base_ = d.beg;
      ev_base_dev_ = dev;
    }
    return d;
  }

  void dev_stamp_end(DevStamp* d, hipStream_t s, int ret) {
    if (ret != 0) {  // dropped / failed invoke: nothing to time
      hip::check(hipEventSynchronize(d->beg), "sync timing event");
      std::lock_guard<std::mutex> lk(stat_mu_);
      if (d->beg != ev_base_) ev_free_.push_back(d->beg);
      ev_free_.push_back(d->end);
      return;
    }
    hip::check(hipEventRecord(d->end, s), "hipEventRecord(invoke end)");
    std::lock_guard<std::mutex> lk(stat_mu_);
    pending_.push_back(*d);
    // bound the number of outstanding timing pairs (the stream is far ahead)
    if (pending_.size() > 4096) drain_locked(true);
  }

  // fold completed timing pairs into the statistics; wait = block on all
  void drain_locked(bool wait) {
    while (!pending_.empty()) {
      DevStamp d = pending_.front();
      if (wait) {
        hip::DeviceGuard g(d.dev);
        if (hipEventSynchronize(d.end) != hipSuccess) break;
      } else if (hipEventQuery(d.end) != hipSuccess) {
        break;
      }
      pending_.pop_front();
      float lat_ms = 0.f, at_ms = 0.f;
      (void)hipEventElapsedTime(&lat_ms, d.beg, d.end);
      if (ev_base_ && ev_base_dev_ == d.dev) (void)hipEventElapsedTime(&at_ms, ev_base_, d.end);
      const int64_t dur = static_cast<int64_t>(static_cast<double>(lat_ms) * 1e6);
      const int64_t at = static_cast<int64_t>(static_cast<double>(at_ms) * 1e6);
      if (device_stamps_) dev_log_.emplace_back(at, dur);
      add_sample_locked(dur, at);
      if (d.beg != ev_base_) ev_free_.push_back(d.beg);
      ev_free_.push_back(d.end);
    }
  }
  void poll_device_stats(bool wait) {
    std::lock_guard<std::mutex> lk(stat_mu_);
    drain_locked(wait);
  }

  void record_stats(int64_t dur_ns, int64_t now) {
    if (!stats_enabled()) return;
    std::lock_guard<std::mutex> lk(stat_mu_);
    add_sample_locked(dur_ns, now);
  }

  // tensor_filter.c:378-455 record_statistics: the first measurement is
  // ignored (latency_ignore_count = 1, tensor_filter_common.c:579); latency =
  // mean of the last 10 invokes (us); throughput = invokes x 1e6 x 1000 /
  // total invoke latency (us), i.e. FPS x 1000; totals are rebased past 2000
  // invokes (cache at 1000) so they never overflow.
  void add_sample_locked(int64_t dur_ns, int64_t now) {
    (void)now;
    ++total_invoke_;
    if (ignore_count_ > 0) {
      --ignore_count_;
      return;
    }
    sum_lat_ns_ += dur_ns;
    sum_num_ += 1;
    lat_.push_back(dur_ns);
    if (lat_.size() > kMaxRecent) lat_.pop_front();
    if (latency_mode_ > 0 || latency_report_) {
      int64_t avg = 0;
      for (auto v : lat_) avg += v;
      avg = avg / static_cast<int64_t>(lat_.size()) / 1000;  // us, like g_get_real_time deltas
      prop_latency_us_ = avg <= INT32_MAX ? avg : -1;
    }
    if (throughput_mode_ > 0) {
      int64_t thr = -1;
      if (sum_lat_ns_ != 0) {
        const double t = static_cast<double>(sum_num_) * 1e12 / static_cast<double>(sum_lat_ns_);
        if (t <= INT32_MAX) thr = static_cast<int64_t>(t);
      }
      prop_throughput_ = thr;
    }
    if (sum_num_ > kDropOld) {
      sum_lat_ns_ -= old_lat_ns_;
      sum_num_ -= old_num_;
      old_lat_ns_ = 0;
      old_num_ = 0;
    } else if (sum_num_ > kCacheOld && old_num_ == 0) {
      old_lat_ns_ = sum_lat_ns_;
      old_num_ = sum_num_;
    }
    if (latency_report_) track_latency_locked();
  }

  // tensor_filter.c:470-495 track_latency: post LATENCY when the estimate
  // exceeds what the last latency query reported, or deviates from it by more
  // than 25 %.  The latency query (query_latency below) stores the reported
  // value with 5 % headroom (tensor_filter.c:1338-1349).
  void track_latency_locked() {
    const double estimated = static_cast<double>(prop_latency_us_) * 1000.0;
    const double reported = static_cast<double>(latency_reported_ns_);
    if (estimated <= 0) return;
    const double deviation = reported > 0 ? std::abs(estimated - reported) / reported : 0.0;
    if (estimated > reported || deviation > kLatencyReportThreshold) {
      ++latency_posts_;
      post_latency();
    }
  }

  bool query_latency(Pad* pad, bool* live, int64_t* min_lat, int64_t* max_lat) override {
    int64_t est;
    {
      std::lock_guard<std::mutex> lk(stat_mu_);
      est = prop_latency_us_;
    }
    bool ok = Element::query_latency(pad, live, min_lat, max_lat);
    if (latency_report_ && est > 0 && ok) {
      const int64_t lat = static_cast<int64_t>(static_cast<double>(est) * 1000.0 * (1.0 + kLatencyReportHeadroom));
      {
        std::lock_guard<std::mutex> lk(stat_mu_);
        latency_reported_ns_ = lat;
      }
      *min_lat += lat;
      if (*max_lat >= 0) *max_lat += lat;
    }
    return ok;
  }

  int64_t avg_latency_us() {
    poll_device_stats(false);
    std::lock_guard<std::mutex> lk(stat_mu_);
    return prop_latency_us_;
  }

  int64_t throughput_milli_fps() {
    poll_device_stats(false);
    std::lock_guard<std::mutex> lk(stat_mu_);
    return prop_throughput_;
  }

  void reset_stats_locked() {
    lat_.clear();
    dev_log_.clear();
    total_invoke_ = 0;
    ignore_count_ = 1;
    sum_lat_ns_ = sum_num_ = old_lat_ns_ = old_num_ = 0;
    prop_latency_us_ = prop_throughput_ = 0;
    latency_reported_ns_ = 0;
  }

  bool start() override {
    prev_ts_ = -1;
    throttle_delay_ = 0;
    {
      std::lock_guard<std::mutex> lk(stat_mu_);
      reset_stats_locked();
    }
    if (!ensure_open()) {
      post_error("tensor_filter: cannot open framework '" + fw_name_ + "' (model '" + model_str_ + "')");
      return false;
    }
    attach_absorbable();
    return true;
  }
  bool stop() override {
    poll_device_stats(true);
    detach_absorbable();
    release_decoder_argmax();
    release_decoder_stage();
    return true;
  }
  void release_timing_events() {
    std::lock_guard<std::mutex> lk(stat_mu_);
    drain_locked(true);
    for (auto& de : ev_all_) {
      hip::DeviceGuard g(de.first);
      (void)hipEventDestroy(de.second);
    }
    ev_all_.clear();
    ev_free_.clear();
    ev_base_ = nullptr;
  }
  void close() override { close_fw(); }

 private:
  static constexpr size_t kMaxRecent = 10;             // GST_TF_STAT_MAX_RECENT
  static constexpr int64_t kDropOld = 2000, kCacheOld = 1000;  // THRESHOLD_DROP_OLD / _CACHE_OLD
  static constexpr double kLatencyReportThreshold = 0.25, kLatencyReportHeadroom = 0.05;
  std::string fw_name_, model_str_, input_str_, inputtype_str_, inputname_str_, inputranks_str_, output_str_,
      outputtype_str_, outputname_str_, outputranks_str_, input_comb_str_, output_comb_str_, config_file_;
  FilterProperties props_;
  std::vector<int> input_comb_;
  std::vector<std::pair<bool, int>> out_comb_;
  bool latency_report_ = false;
  int latency_mode_ = 0, throughput_mode_ = 0;
  bool absorb_enabled_ = true;
  bool absorb_dec_enabled_ = true;
  bool argmax_tried_ = false;
  ArgmaxConsumer* argmax_consumer_ = nullptr;
  bool stage_tried_ = false;
  DecodeStageConsumer* stage_consumer_ = nullptr;
  std::shared_ptr<DecodeStage> stage_;
  TensorsConfig stage_model_out_;  // the model outputs the stage was taken for
  std::string absorbed_decoder_;
  AbsorbableElement* absorbable_up_ = nullptr;
  std::string absorbed_from_;
  int device_prop_ = -1;
  std::shared_ptr<FilterFramework> fw_;
  std::shared_ptr<FilterInstance> inst_;
  std::shared_ptr<SharedModel> shared_;
  std::mutex open_mu_;
  bool model_info_known_ = false;
  TensorsInfo model_in_, model_out_, model_out_runtime_;
  TensorsConfig in_config_, out_config_;
  bool in_flexible_ = false, out_flexible_ = false, configured_ = false;
  int64_t throttle_delay_ = 0, prev_ts_ = -1;
  mutable std::mutex stat_mu_;
  std::deque<int64_t> lat_;
  int64_t total_invoke_ = 0;
  int ignore_count_ = 1;
  int64_t sum_lat_ns_ = 0, sum_num_ = 0, old_lat_ns_ = 0, old_num_ = 0;
  int64_t prop_latency_us_ = 0, prop_throughput_ = 0, latency_reported_ns_ = 0, latency_posts_ = 0;
  bool device_stamps_ = false;
  std::deque<DevStamp> pending_;
  std::vector<hipEvent_t> ev_free_;
  std::vector<std::pair<int, hipEvent_t>> ev_all_;
  hipEvent_t ev_base_ = nullptr;
  int ev_base_dev_ = -1;
  std::vector<std::pair<int64_t, int64_t>> dev_log_;  // (end ns on the device clock, device latency ns)
  StreamSet streams_;
};

}  // namespace

void register_tensor_filter() {
  register_element("tensor_filter", "Filter/Tensor", "Handles NN Frameworks (e.g., pytorch) as Media Filters with other/tensor type stream",
                   [](const std::string& n) { return std::make_unique<TensorFilter>(n); });
}

}  // namespace nnsx
