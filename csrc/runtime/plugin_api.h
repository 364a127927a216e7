// Sub-plugin APIs: tensor_filter frameworks, tensor_decoder modes,
// tensor_converter external converters and tensor_trainer frameworks.
//
// Reference ABIs: GstTensorFilterFramework V0/V1
// (gst/nnstreamer/include/nnstreamer_plugin_api_filter.h:273-495),
// GstTensorDecoderDef (nnstreamer_plugin_api_decoder.h:38-97),
// NNStreamerExternalConverter (nnstreamer_plugin_api_converter.h:41-85),
// GstTensorTrainerFramework (nnstreamer_plugin_api_trainer.h:66-127).
// nnsx redesign: invoke works on Memory objects that may be device-resident;
// the element hands the framework a HIP stream (per-pad stream) and the
// framework returns allocate-in-invoke outputs whose lifetime is tied to the
// output Memory's release (DESTROY_NOTIFY).
#pragma once

#include <hip/hip_runtime_api.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/caps.h"
#include "core/registry.h"
#include "runtime/element.h"
#include "runtime/memory.h"

namespace nnsx {

// ------------------------------------------------------------- filters ----

enum class Accelerator { NONE, AUTO, CPU, GPU, DEFAULT };

class DecodeStage;  // runtime/fusion.h

struct FilterProperties {
  std::string fwname;
  std::vector<std::string> model_files;
  TensorsInfo input_info;       // from properties or model
  TensorsInfo output_info;
  std::string input_layout, output_layout;
  std::vector<int> input_ranks, output_ranks;
  std::string custom_properties;  // custom=...
  std::string accl_str;           // accelerator=...
  Accelerator accl = Accelerator::DEFAULT;
  int device = -1;                // resolved GPU index (-1 = CPU)
  bool is_updatable = false;
  std::string shared_key;
  bool input_configured = false, output_configured = false;
  int invoke_dynamic = 0;         // flexible output shapes
};

struct InvokeContext {
  int device = -1;          // -1: host invoke
  hipStream_t stream = nullptr;
  // set by the framework when outputs' shapes change (flexible / invoke-dynamic)
  TensorsInfo* out_info = nullptr;
  // decoders: >1 when out->mems holds one memory per frame of a batched input;
  // tensor_decoder then pushes them as consecutive buffers
  unsigned out_frames = 1;
  // set by a filter instance whose device work for this invoke ended on another
  // stream than `stream` (pytorch replay lanes): the element's end-of-invoke
  // timing event goes there
  hipStream_t done_stream = nullptr;
};

class FilterInstance {
 public:
  virtual ~FilterInstance() = default;
  // GET_IN_OUT_INFO; return false if the model does not know (needs SET_INPUT_INFO)
  virtual bool get_model_info(TensorsInfo* in, TensorsInfo* out) = 0;
  // SET_INPUT_INFO: given input info, report output info (dynamic shapes)
  virtual bool set_input_info(const TensorsInfo& in, TensorsInfo* out) {
    (void)in;
    (void)out;
    return false;
  }
  // Run the model.  `out` must be filled with one Memory per output tensor.
  // Return 0 on success, >0 to drop this frame silently, <0 on error.
  virtual int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext& ctx) = 0;
  virtual bool reload_model(const FilterProperties& props) {
    (void)props;
    return false;
  }
  virtual bool handle_event(const std::string& name, const std::string& arg) {
    (void)name;
    (void)arg;
    return false;
  }
  // true when input memories must be on the host (CPU frameworks)
  virtual bool wants_host_input() const { return true; }
  // Upstream-arithmetic absorption (runtime/fusion.h): true when the model maps
  // a uint8 input `index` through a 256-entry f32 table it can be given.
  virtual bool accepts_input_table(unsigned index) const {
    (void)index;
    return false;
  }
  // Install that table; the input then arrives as uint8 (the caller updates
  // the negotiated input type).  Must survive a hot reload.
  virtual bool set_input_table(unsigned index, const std::vector<float>& lut) {
    (void)index;
    (void)lut;
    return false;
  }
  // Undo set_input_table: the model's own table again (absorption released)
  virtual bool reset_input_table(unsigned index) {
    (void)index;
    return false;
  }
  // Downstream-argmax absorption (runtime/fusion.h): true when the framework
  // can end its device work with an argmax over the innermost dimension of
  // output `index`, producing int32 indices (that dimension becomes 1)
  virtual bool accepts_output_argmax(unsigned index) const {
    (void)index;
    return false;
  }
  virtual bool set_output_argmax(unsigned index, bool on) {
    (void)index;
    (void)on;
    return false;
  }
  // Downstream decode-stage absorption (runtime/fusion.h DecodeStage): the
  // framework runs `stage` after its forward (inside its captured graph) and
  // hands out the stage's outputs instead of the model's; nullptr removes it.
  // stage_device(): the GPU the outputs are produced on (-1: host framework)
  virtual int stage_device() const { return -1; }
  virtual bool set_output_stage(std::shared_ptr<DecodeStage> stage) {
    (void)stage;
    return false;
  }
  // Property changes after open (reference V1 events CUSTOM_PROP,
  // SET_INPUT_PROP / SET_OUTPUT_PROP, SET_ACCELERATOR): true = applied.
  virtual bool update_custom(const std::string& custom) {
    (void)custom;
    return false;
  }
  virtual bool update_io_info(bool input, const TensorsInfo& info) {
    (void)input;
    (void)info;
    return false;
  }
  virtual bool update_accelerator(const std::string& accelerators) {
    (void)accelerators;
    return false;
  }
  // framework-specific read-only facts for tools / stats (e.g. "model-broadcast")
  virtual std::string info(const std::string& key) const {
    (void)key;
    return std::string();
  }
};

class FilterFramework {
 public:
  virtual ~FilterFramework() = default;
  virtual std::string name() const = 0;
  virtual std::unique_ptr<FilterInstance> open(FilterProperties& props) = 0;
  virtual bool check_availability(Accelerator accl) const {
    return accl == Accelerator::CPU || accl == Accelerator::DEFAULT || accl == Accelerator::AUTO;
  }
  virtual std::vector<std::string> model_extensions() const { return {}; }
  virtual bool run_without_model() const { return false; }
  virtual bool verify_model_path() const { return true; }
  virtual bool allocate_in_invoke() const { return true; }
  virtual std::string accelerators() const { return "cpu"; }
};

bool register_filter_framework(std::shared_ptr<FilterFramework> fw);
std::shared_ptr<FilterFramework> find_filter_framework(const std::string& name);
// framework=auto: detect from model extension honouring [filter] framework_priority_<ext>
std::string detect_framework(const std::vector<std::string>& models);
// accelerator string grammar "true:gpu,cpu" / "false" / "true:!npu" (tensor_filter_common.c:2495-2800)
Accelerator parse_accelerator(const std::string& s, const std::string& supported, bool* use_accel);
// Shared by tensor_filter and the single-shot API: framework=auto detection,
// accelerator parsing and GPU selection (`device` >= 0, else LOCAL_RANK % #GPUs,
// else 0) into props->fwname / accl / device.  nullptr + *err on failure.
std::shared_ptr<FilterFramework> resolve_filter_framework(const std::string& fw_name, FilterProperties* props,
                                                          int device_prop, std::string* err);

// custom-easy (NNS_custom_easy_register)
using CustomEasyFn = std::function<int(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out,
                                       const TensorsInfo& in_info, const TensorsInfo& out_info)>;
bool custom_easy_register(const std::string& name, CustomEasyFn fn, const TensorsInfo& in, const TensorsInfo& out);
bool custom_easy_unregister(const std::string& name);

// -------------------------------------------------------------- decoders ----

class DecoderInstance {
 public:
  virtual ~DecoderInstance() = default;
  virtual bool set_option(int idx, const std::string& value) {
    (void)idx;
    (void)value;
    return true;
  }
  // output caps for the given input config (ANY/empty = cannot decide yet)
  virtual Caps get_out_caps(const TensorsConfig& config) = 0;
  // decode: fill *out (buffer timestamps already copied); may run kernels on ctx.stream
  virtual FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                            InvokeContext& ctx) = 0;
  virtual bool supports_device() const { return false; }
  // Argmax absorption (runtime/fusion.h): a decoder whose first step is an
  // argmax over the innermost dimension of tensor 0 may receive the producer's
  // int32 indices [1:B] instead of the scores [classes:B].  true = from now on
  // decode() takes indices.
  // Device stage (runtime/fusion.h): the decoder's device post-processing of
  // inputs shaped `in` as one capturable enqueue on GPU `dev`.  prepare
  // allocates every buffer the enqueue touches and uploads tables (it may
  // synchronize) and reports the stage's output tensors; enqueue then only
  // launches kernels / memsets on `s`.  Decoders whose stage writes RGBA frames
  // report one uint8 [4:W:H:B] tensor, which the element slices per frame.
  virtual bool stage_prepare(const TensorsConfig& in, int dev, hipStream_t s, TensorsInfo* out) {
    (void)in;
    (void)dev;
    (void)s;
    (void)out;
    return false;
  }
  virtual bool stage_enqueue(const std::vector<const void*>& in, const std::vector<void*>& out, hipStream_t s) {
    (void)in;
    (void)out;
    (void)s;
    return false;
  }
  // stage_enqueue writes only its `out` buffers (no scratch of the instance):
  // the stage may be replayed on several lanes at once (DecodeStage::lane_safe)
  virtual bool stage_lane_safe() const { return false; }
  virtual bool accept_argmax_input(uint32_t classes) {
    (void)classes;
    return false;
  }
  virtual void drop_argmax_input() {}
};

class DecoderSubplugin {
 public:
  virtual ~DecoderSubplugin() = default;
  virtual std::string name() const = 0;
  virtual std::unique_ptr<DecoderInstance> create() = 0;
};

bool register_decoder(std::shared_ptr<DecoderSubplugin> d);
std::shared_ptr<DecoderSubplugin> find_decoder(const std::string& mode);

// custom-code decoder (nnstreamer_decoder_custom_register)
using DecoderCustomFn = std::function<FlowReturn(const std::vector<MemoryPtr>& in, const TensorsConfig& config,
                                                 Buffer* out)>;
bool decoder_custom_register(const std::string& name, DecoderCustomFn fn);
bool decoder_custom_unregister(const std::string& name);

// ------------------------------------------------------------ converters ----

class ConverterSubplugin {
 public:
  virtual ~ConverterSubplugin() = default;
  virtual std::string name() const = 0;
  // media this converter accepts (caps) -- used to pick a converter by input caps
  virtual Caps query_caps() const = 0;
  virtual bool get_out_config(const Caps& in, TensorsConfig* config) {
    (void)in;
    (void)config;
    return false;
  }
  // convert one buffer; sets *config (may change per buffer -> caps update)
  virtual BufferPtr convert(const BufferPtr& in, TensorsConfig* config) = 0;
  virtual bool open(const std::string& script) {
    (void)script;
    return true;
  }
};

bool register_converter(std::shared_ptr<ConverterSubplugin> c);
std::shared_ptr<ConverterSubplugin> find_converter(const std::string& name);
std::shared_ptr<ConverterSubplugin> find_converter_for_caps(const Caps& caps);

using ConverterCustomFn = std::function<BufferPtr(const BufferPtr& in, TensorsConfig* config)>;
bool converter_custom_register(const std::string& name, ConverterCustomFn fn);
bool converter_custom_unregister(const std::string& name);

// Script-backed helpers are provided by the Python bridge (bindings):
// `custom-script:<file>.py` converter / decoder, framework=python3 filter.
using ScriptConverterFactory = std::function<std::shared_ptr<ConverterSubplugin>(const std::string& path)>;
void set_script_converter_factory(ScriptConverterFactory f);
std::shared_ptr<ConverterSubplugin> make_script_converter(const std::string& path);

// tensor_if custom condition (nnstreamer_if_custom_register)
using IfCustomFn = std::function<bool(const TensorsInfo& info, const std::vector<MemoryPtr>& in)>;
bool if_custom_register(const std::string& name, IfCustomFn fn);
bool if_custom_unregister(const std::string& name);
IfCustomFn find_if_custom(const std::string& name);

// -------------------------------------------------------------- trainers ----

struct TrainerProperties {
  std::string model_config, model_save_path, model_load_path;
  TensorsInfo input_info;
  unsigned num_inputs = 1, num_labels = 1;
  unsigned num_training_samples = 0, num_validation_samples = 0;
  unsigned epochs = 1;
  int device = -1;
};

struct TrainerStatus {
  double training_loss = 0, training_accuracy = 0, validation_loss = 0, validation_accuracy = 0;
  unsigned epoch_count = 0;
  bool complete = false;
};

class TrainerInstance {
 public:
  virtual ~TrainerInstance() = default;
  virtual bool start() = 0;
  virtual bool stop() = 0;
  // push one sample (inputs followed by labels); validation samples flagged
  virtual bool push_data(const std::vector<MemoryPtr>& tensors, bool is_validation) = 0;
  virtual TrainerStatus status() = 0;
  virtual bool save(const std::string& path) = 0;
  // block until training completes (or timeout)
  virtual bool wait_complete(int64_t timeout_ns) = 0;
};

class TrainerFramework {
 public:
  virtual ~TrainerFramework() = default;
  virtual std::string name() const = 0;
  virtual std::unique_ptr<TrainerInstance> create(const TrainerProperties& props) = 0;
};

bool register_trainer(std::shared_ptr<TrainerFramework> t);
std::shared_ptr<TrainerFramework> find_trainer(const std::string& name);

}  // namespace nnsx
