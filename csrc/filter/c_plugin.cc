// The public C sub-plugin ABI (include/nnsx/nnsx_plugin_api*.h): adapters
// from the plain-C tables of external shared objects to the runtime's
// FilterFramework / DecoderSubplugin / ConverterSubplugin classes, the host
// table handed to nnsx_subplugin_init(), and the reference-named in-process
// registration entry points (nnstreamer_filter_probe, nnstreamer_decoder_probe,
// registerExternalConverter).
//
// Reference: nnstreamer_plugin_api_filter.h:139-495 (V0 and V1 vtables, the
// seven V1 events), nnstreamer_plugin_api_decoder.h:38-97,
// nnstreamer_plugin_api_converter.h:41-85, nnstreamer_plugin_api_trainer.h
// :31-141 and the dlopen-then-probe flow of nnstreamer_subplugin.c:108-171.
#include <dlfcn.h>

#include <cerrno>
#include <condition_variable>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <nnsx/nnsx_plugin_api.h>

#include "core/log.h"
#include "core/registry.h"
#include "core/util.h"
#include "filter/filter.h"
#include "runtime/hip_util.h"
#include "runtime/plugin_api.h"

namespace nnsx {
namespace {

// ------------------------------------------------------------ conversions ----
void to_c_info(const TensorsInfo& a, NNSX_TensorsInfo* b) {
  std::memset(b, 0, sizeof(*b));
  b->num_tensors = std::min<unsigned>(a.num_tensors, NNSX_SIZE_LIMIT);
  b->format = static_cast<uint32_t>(a.format);
  for (unsigned i = 0; i < b->num_tensors; ++i) {
    b->info[i].type = static_cast<uint32_t>(a.at(i).type);
    for (int d = 0; d < kRankLimit; ++d) b->info[i].dimension[d] = a.at(i).dim[d];
  }
}

// false when the plugin handed back more tensors than the ABI allows
bool from_c_info(const NNSX_TensorsInfo& b, TensorsInfo* a) {
  if (b.num_tensors > NNSX_SIZE_LIMIT) return false;
  *a = TensorsInfo();
  a->resize(b.num_tensors);
  a->format = static_cast<Format>(b.format);
  for (unsigned i = 0; i < b.num_tensors; ++i) {
    a->at(i).type = static_cast<DType>(b.info[i].type);
    for (int d = 0; d < kRankLimit; ++d) a->at(i).dim[d] = b.info[i].dimension[d] ? b.info[i].dimension[d] : 1;
    if (b.info[i].name) a->at(i).name = b.info[i].name;
  }
  return true;
}

void to_c_config(const TensorsConfig& a, NNSX_TensorsConfig* b) {
  to_c_info(a.info, &b->info);
  b->rate_n = a.rate_n;
  b->rate_d = a.rate_d;
}

std::string take_string(char* s) {
  if (!s) return std::string();
  std::string r(s);
  std::free(s);
  return r;
}

MemoryPtr adopt_malloc(void* data, size_t size) {
  return Memory::wrap(data, size, MemPlace::HOST, -1, [](Memory* m) { std::free(m->data()); });
}

// ---------------------------------------------------------------- filters ----
struct CFilterProps {
  // keeps the C view of FilterProperties (and the strings it points at) alive
  explicit CFilterProps(const FilterProperties& p) { set(p); }
  void set(const FilterProperties& p) {
    fw = p.fwname;
    custom = p.custom_properties;
    models = p.model_files;
    ptrs.clear();
    for (auto& m : models) ptrs.push_back(m.c_str());
    std::memset(&c, 0, sizeof(c));
    c.fwname = fw.c_str();
    c.model_files = ptrs.data();
    c.num_models = static_cast<int>(ptrs.size());
    c.custom_properties = custom.c_str();
    to_c_info(p.input_info, &c.input_meta);
    to_c_info(p.output_info, &c.output_meta);
  }
  std::string fw, custom;
  std::vector<std::string> models;
  std::vector<const char*> ptrs;
  NNSX_FilterProperties c;
};

int c_event(const NNSX_FilterFramework* fw, const NNSX_FilterProperties* prop, void* priv, NNSX_FilterEvent ev,
            const NNSX_FilterEventData& d) {
  if (!fw->eventHandler) return -ENOENT;
  return fw->eventHandler(fw, prop, priv, ev, &d);
}

class CFilterInstance : public FilterInstance {
 public:
  CFilterInstance(const NNSX_FilterFramework* fw, FilterProperties& p, bool alloc_in_invoke)
      : fw_(fw), props_(p), cprops_(p), alloc_(alloc_in_invoke) {
    if (fw_->version == NNSX_FILTER_FRAMEWORK_V2) priv_ = fw_->subplugin_data;  // the C++ base's class object
    if (fw_->open && fw_->open(&cprops_.c, &priv_) != 0)
      throw Error("framework " + std::string(fw_->name) + ": open failed");
  }
  ~CFilterInstance() override {
    if (fw_->close) fw_->close(&cprops_.c, &priv_);
  }
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    if (!fw_->getModelInfo) return false;
    NNSX_TensorsInfo a, b;
    std::memset(&a, 0, sizeof(a));
    std::memset(&b, 0, sizeof(b));
    if (fw_->getModelInfo(fw_, &cprops_.c, priv_, NNSX_GET_IN_OUT_INFO, &a, &b) != 0) return false;
    if (!from_c_info(a, in) || !from_c_info(b, out)) return false;
    remember(*in, *out);
    return true;
  }
  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override {
    if (!fw_->getModelInfo) return false;
    NNSX_TensorsInfo a, b;
    to_c_info(in, &a);
    std::memset(&b, 0, sizeof(b));
    if (fw_->getModelInfo(fw_, &cprops_.c, priv_, NNSX_SET_INPUT_INFO, &a, &b) != 0) return false;
    if (!from_c_info(b, out)) return false;
    remember(in, *out);
    return true;
  }
  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext& ctx) override {
    const int dev = device();
    NNSX_TensorMemory ci[NNSX_SIZE_LIMIT], co[NNSX_SIZE_LIMIT];
    std::memset(ci, 0, sizeof(ci));
    std::memset(co, 0, sizeof(co));
    hipStream_t s = ctx.stream;
    if (dev >= 0 && !s) s = hip::thread_copy_stream(dev);
    for (size_t i = 0; i < in.size() && i < NNSX_SIZE_LIMIT; ++i) {
      ci[i].data = dev >= 0 ? const_cast<void*>(in[i]->map_device(dev, s)) : const_cast<void*>(in[i]->map_host());
      ci[i].size = in[i]->size();
    }
    std::vector<MemoryPtr> allocated;
    const unsigned nout = std::min<unsigned>(out_.num_tensors, NNSX_SIZE_LIMIT);
    if (!alloc_) {
      for (unsigned i = 0; i < nout; ++i) {
        const size_t sz = out_.size(static_cast<int>(i));
        auto m = dev >= 0 ? Memory::alloc_device(sz, dev, s) : Memory::alloc_host(sz);
        co[i].data = m->data();
        co[i].size = sz;
        allocated.push_back(m);
      }
    }
    NNSX_InvokeContext c{dev, dev >= 0 ? static_cast<void*>(s) : nullptr};
    const int r = fw_->invoke(fw_, &cprops_.c, priv_, ci, co, &c);
    if (dev >= 0)
      for (auto& m : in) m->record_use(s, dev);
    if (r != 0) return r;
    if (alloc_) {
      for (unsigned i = 0; i < nout; ++i) {
        if (!co[i].data) return -EINVAL;
        const NNSX_FilterFramework* fw = fw_;
        void* priv = priv_;
        auto rel = [fw, priv, s, dev](Memory* m) {
          if (dev >= 0) {
            hip::DeviceGuard g(dev);
            m->wait_uses(s);
            (void)hipStreamSynchronize(s);
          }
          if (fw->destroyNotify) {
            fw->destroyNotify(priv, m->data());
          } else {  // V1 DESTROY_NOTIFY event; not handled (-ENOENT): the runtime frees host data
            NNSX_FilterEventData d{};
            d.data = m->data();
            if (c_event(fw, nullptr, priv, NNSX_EVENT_DESTROY_NOTIFY, d) == -ENOENT && dev < 0) std::free(m->data());
          }
        };
        auto m = Memory::wrap(co[i].data, co[i].size, dev >= 0 ? MemPlace::DEVICE : MemPlace::HOST, dev, rel);
        if (dev >= 0) m->mark_ready(s);
        out->push_back(m);
      }
      return 0;
    }
    if (dev >= 0)
      for (auto& m : allocated) m->mark_ready(s);
    *out = std::move(allocated);
    return 0;
  }
  bool reload_model(const FilterProperties& p) override {
    if (!fw_->eventHandler) return false;
    CFilterProps np(p);
    if (fw_->eventHandler(fw_, &cprops_.c, priv_, NNSX_EVENT_RELOAD_MODEL, &np.c) != 0) return false;
    props_ = p;
    cprops_.set(p);
    return true;
  }
  bool handle_event(const std::string& name, const std::string& arg) override {
    if (!fw_->eventHandler) return false;
    const std::string s = name + "=" + arg;
    return fw_->eventHandler(fw_, &cprops_.c, priv_, NNSX_EVENT_CUSTOM, s.c_str()) == 0;
  }
  bool update_custom(const std::string& custom) override {
    NNSX_FilterEventData d{};
    d.custom_properties = custom.c_str();
    if (c_event(fw_, &cprops_.c, priv_, NNSX_EVENT_CUSTOM_PROP, d) != 0) return false;
    props_.custom_properties = custom;
    cprops_.set(props_);
    return true;
  }
  bool update_io_info(bool input, const TensorsInfo& info) override {
    NNSX_TensorsInfo ci;
    to_c_info(info, &ci);
    NNSX_FilterEventData d{};
    d.info = &ci;
    if (c_event(fw_, &cprops_.c, priv_, input ? NNSX_EVENT_SET_INPUT_PROP : NNSX_EVENT_SET_OUTPUT_PROP, d) != 0)
      return false;
    (input ? props_.input_info : props_.output_info) = info;
    if (!input) out_ = info;
    cprops_.set(props_);
    return true;
  }
  bool update_accelerator(const std::string& accelerators) override {
    NNSX_FilterEventData d{};
    d.accelerators = accelerators.c_str();
    return c_event(fw_, &cprops_.c, priv_, NNSX_EVENT_SET_ACCELERATOR, d) == 0;
  }
  bool wants_host_input() const override { return device() < 0; }

 private:
  int device() const { return props_.device; }
  void remember(const TensorsInfo& in, const TensorsInfo& out) {
    out_ = out;
    props_.input_info = in;
    props_.output_info = out;
    to_c_info(in, &cprops_.c.input_meta);
    to_c_info(out, &cprops_.c.output_meta);
  }
  const NNSX_FilterFramework* fw_;
  FilterProperties props_;
  CFilterProps cprops_;
  bool alloc_;
  void* priv_ = nullptr;
  TensorsInfo out_;
};

class CFilterFramework : public FilterFramework {
 public:
  explicit CFilterFramework(const NNSX_FilterFramework* fw) : fw_(fw) {
    NNSX_FrameworkInfo info;
    std::memset(&info, 0, sizeof(info));
    // static information: queried without an instance (prop / private_data NULL)
    if (fw_->getFrameworkInfo && fw_->getFrameworkInfo(fw_, nullptr, nullptr, &info) == 0) {
      alloc_ = info.allocate_in_invoke != 0;
      without_model_ = info.run_without_model != 0;
      verify_ = info.verify_model_path != 0;
      if (info.accelerators) accl_ = info.accelerators;
      if (info.model_extensions)
        for (auto& e : split(info.model_extensions, ',')) exts_.push_back(strip(e));
    }
  }
  std::string name() const override { return fw_->name; }
  std::unique_ptr<FilterInstance> open(FilterProperties& props) override {
    if (props.device >= 0 && accl_.find("gpu") == std::string::npos) props.device = -1;  // host-only framework
    return std::make_unique<CFilterInstance>(fw_, props, alloc_);
  }
  bool check_availability(Accelerator accl) const override {
    // CHECK_HW_AVAILABILITY (no instance yet: private_data NULL); frameworks
    // without the event answer from their static accelerator list
    if (fw_->eventHandler && (accl == Accelerator::GPU || accl == Accelerator::CPU)) {
      NNSX_FilterEventData d{};
      d.hw = accl == Accelerator::GPU ? "gpu" : "cpu";
      const int r = c_event(fw_, nullptr, nullptr, NNSX_EVENT_CHECK_HW_AVAILABILITY, d);
      if (r != -ENOENT) return r == 0;
    }
    if (accl == Accelerator::GPU) return accl_.find("gpu") != std::string::npos;
    return FilterFramework::check_availability(accl) || accl == Accelerator::NONE;
  }
  std::vector<std::string> model_extensions() const override { return exts_; }
  bool run_without_model() const override { return without_model_; }
  bool verify_model_path() const override { return verify_; }
  bool allocate_in_invoke() const override { return alloc_; }
  std::string accelerators() const override { return accl_; }

 private:
  const NNSX_FilterFramework* fw_;
  bool alloc_ = false, without_model_ = false, verify_ = true;
  std::string accl_ = "cpu";
  std::vector<std::string> exts_;
};

// ------------------------------------------------------ filters: V0 table ----
// The legacy V0 table (invoke_NN, get/set dimensions, reloadModel, handleEvent,
// checkAvailability, allocateInInvoke) adapted to the runtime; V0 frameworks run
// on host memories.
class CFilterInstanceV0 : public FilterInstance {
 public:
  CFilterInstanceV0(const NNSX_FilterFrameworkV0* fw, FilterProperties& p) : fw_(fw), props_(p), cprops_(p) {
    if (fw_->open && fw_->open(&cprops_.c, &priv_) != 0)
      throw Error("framework " + std::string(fw_->name) + ": open failed");
    alloc_ = fw_->allocateInInvoke ? fw_->allocateInInvoke(&priv_) == 0 : fw_->allocate_in_invoke != 0;
  }
  ~CFilterInstanceV0() override {
    if (fw_->close) fw_->close(&cprops_.c, &priv_);
  }
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    if (!fw_->getInputDimension || !fw_->getOutputDimension) return false;
    NNSX_TensorsInfo a, b;
    std::memset(&a, 0, sizeof(a));
    std::memset(&b, 0, sizeof(b));
    if (fw_->getInputDimension(&cprops_.c, &priv_, &a) != 0 || fw_->getOutputDimension(&cprops_.c, &priv_, &b) != 0)
      return false;
    if (!from_c_info(a, in) || !from_c_info(b, out)) return false;
    remember(*in, *out);
    return true;
  }
  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override {
    if (!fw_->setInputDimension) return false;
    NNSX_TensorsInfo a, b;
    to_c_info(in, &a);
    std::memset(&b, 0, sizeof(b));
    if (fw_->setInputDimension(&cprops_.c, &priv_, &a, &b) != 0 || !from_c_info(b, out)) return false;
    remember(in, *out);
    return true;
  }
  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext&) override {
    NNSX_TensorMemory ci[NNSX_SIZE_LIMIT], co[NNSX_SIZE_LIMIT];
    std::memset(ci, 0, sizeof(ci));
    std::memset(co, 0, sizeof(co));
    for (size_t i = 0; i < in.size() && i < NNSX_SIZE_LIMIT; ++i) {
      ci[i].data = const_cast<void*>(in[i]->map_host());
      ci[i].size = in[i]->size();
    }
    const unsigned nout = std::min<unsigned>(out_.num_tensors, NNSX_SIZE_LIMIT);
    std::vector<MemoryPtr> allocated;
    for (unsigned i = 0; i < nout; ++i) {
      co[i].size = out_.size(static_cast<int>(i));
      if (!alloc_) {
        allocated.push_back(Memory::alloc_host(co[i].size));
        co[i].data = allocated.back()->data();
      }
    }
    const int r = fw_->invoke_NN(&cprops_.c, &priv_, ci, co);
    if (r != 0) return r;
    if (!alloc_) {
      *out = std::move(allocated);
      return 0;
    }
    for (unsigned i = 0; i < nout; ++i) {
      if (!co[i].data) return -EINVAL;
      const NNSX_FilterFrameworkV0* fw = fw_;
      auto pv = std::make_shared<void*>(priv_);  // outlives neither the instance's data nor this output
      out->push_back(Memory::wrap(co[i].data, co[i].size, MemPlace::HOST, -1, [fw, pv](Memory* m) {
        if (fw->destroyNotify) fw->destroyNotify(pv.get(), m->data());
        else std::free(m->data());  // the reference's default for V0 allocate-in-invoke
      }));
    }
    return 0;
  }
  bool reload_model(const FilterProperties& p) override {
    if (!fw_->reloadModel) return false;
    CFilterProps np(p);
    if (fw_->reloadModel(&np.c, &priv_) != 0) return false;
    props_ = p;
    cprops_.set(p);
    return true;
  }
  bool handle_event(const std::string& name, const std::string& arg) override {
    if (!fw_->handleEvent) return false;
    const std::string s = name + "=" + arg;
    return fw_->handleEvent(NNSX_EVENT_CUSTOM, &priv_, s.c_str()) == 0;
  }
  bool update_custom(const std::string& custom) override {
    if (!fw_->handleEvent) return false;
    NNSX_FilterEventData d{};
    d.custom_properties = custom.c_str();
    if (fw_->handleEvent(NNSX_EVENT_CUSTOM_PROP, &priv_, &d) != 0) return false;
    props_.custom_properties = custom;
    cprops_.set(props_);
    return true;
  }

 private:
  void remember(const TensorsInfo& in, const TensorsInfo& out) {
    out_ = out;
    props_.input_info = in;
    props_.output_info = out;
    to_c_info(in, &cprops_.c.input_meta);
    to_c_info(out, &cprops_.c.output_meta);
  }
  const NNSX_FilterFrameworkV0* fw_;
  FilterProperties props_;
  CFilterProps cprops_;
  bool alloc_ = false;
  void* priv_ = nullptr;
  TensorsInfo out_;
};

class CFilterFrameworkV0 : public FilterFramework {
 public:
  explicit CFilterFrameworkV0(const NNSX_FilterFrameworkV0* fw) : fw_(fw) {}
  std::string name() const override { return fw_->name; }
  std::unique_ptr<FilterInstance> open(FilterProperties& props) override {
    props.device = -1;  // V0: host memories
    return std::make_unique<CFilterInstanceV0>(fw_, props);
  }
  bool check_availability(Accelerator accl) const override {
    if (fw_->checkAvailability && (accl == Accelerator::GPU || accl == Accelerator::CPU))
      return fw_->checkAvailability(accl == Accelerator::GPU ? "gpu" : "cpu") == 0;
    return FilterFramework::check_availability(accl) || accl == Accelerator::NONE;
  }
  bool run_without_model() const override { return fw_->run_without_model != 0; }
  bool verify_model_path() const override { return fw_->verify_model_path != 0; }
  bool allocate_in_invoke() const override { return fw_->allocate_in_invoke != 0; }

 private:
  const NNSX_FilterFrameworkV0* fw_;
};

// --------------------------------------------------------------- trainers ----
// GstTensorTrainerFramework (nnstreamer_plugin_api_trainer.h:66-127) adapted to
// TrainerInstance; the training-complete GCond becomes the notify callback.
class CTrainerInstance : public TrainerInstance {
 public:
  CTrainerInstance(const NNSX_TrainerFramework* fw, const TrainerProperties& p) : fw_(fw), p_(p) {
    cfg_ = p.model_config;
    save_ = p.model_save_path;
    load_ = p.model_load_path;
    std::memset(&c_, 0, sizeof(c_));
    to_c_info(p.input_info, &c_.input_meta);
    c_.model_config = cfg_.c_str();
    c_.model_save_path = save_.c_str();
    c_.model_load_path = load_.empty() ? nullptr : load_.c_str();
    c_.num_inputs = p.num_inputs;
    c_.num_labels = p.num_labels;
    c_.num_training_samples = p.num_training_samples;
    c_.num_validation_samples = p.num_validation_samples;
    c_.num_epochs = p.epochs;
    c_.device = p.device;
    c_.notify = &CTrainerInstance::notify;
    c_.notify_handle = this;
    if (!fw_->create || fw_->create(fw_, &c_, &priv_) != 0)
      throw Error("trainer " + std::string(fw_->name) + ": create failed");
  }
  ~CTrainerInstance() override {
    if (fw_->destroy) fw_->destroy(fw_, &c_, &priv_);
  }
  bool start() override { return !fw_->start || fw_->start(fw_, &c_, priv_) == 0; }
  bool stop() override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stopped_ = true;
      cv_.notify_all();
    }
    return !fw_->stop || fw_->stop(fw_, &c_, priv_) == 0;
  }
  bool push_data(const std::vector<MemoryPtr>& tensors, bool) override {
    NNSX_TensorMemory in[NNSX_SIZE_LIMIT];
    std::memset(in, 0, sizeof(in));
    for (size_t i = 0; i < tensors.size() && i < NNSX_SIZE_LIMIT; ++i) {
      in[i].data = const_cast<void*>(tensors[i]->map_host());
      in[i].size = tensors[i]->size();
    }
    return fw_->push_data(fw_, &c_, priv_, in) == 0;
  }
  TrainerStatus status() override {
    NNSX_TrainerFrameworkInfo i;
    std::memset(&i, 0, sizeof(i));
    TrainerStatus st;
    if (fw_->getFrameworkInfo(fw_, &c_, priv_, &i) != 0) return st;
    st.training_loss = i.training_loss;
    st.training_accuracy = i.training_accuracy;
    st.validation_loss = i.validation_loss;
    st.validation_accuracy = i.validation_accuracy;
    st.epoch_count = static_cast<unsigned>(i.epoch_cnt);
    std::lock_guard<std::mutex> lk(mu_);
    st.complete = i.is_training_complete != 0 || complete_;
    return st;
  }
  bool save(const std::string& path) override { return fw_->save && fw_->save(fw_, &c_, priv_, path.c_str()) == 0; }
  bool wait_complete(int64_t timeout_ns) override {
    std::unique_lock<std::mutex> lk(mu_);
    auto done = [&] {
      if (complete_ || stopped_) return true;
      NNSX_TrainerFrameworkInfo i;
      std::memset(&i, 0, sizeof(i));
      return fw_->getFrameworkInfo(fw_, &c_, priv_, &i) == 0 && i.is_training_complete != 0;
    };
    if (timeout_ns < 0) {
      // the notify wakes us; a plugin that only sets is_training_complete is polled
      while (!cv_.wait_for(lk, std::chrono::milliseconds(50), done)) {
      }
      return complete_ || !stopped_;
    }
    return cv_.wait_for(lk, std::chrono::nanoseconds(timeout_ns), done);
  }

 private:
  static void notify(void* h, NNSX_TrainerEvent ev) {
    auto* self = static_cast<CTrainerInstance*>(h);
    std::lock_guard<std::mutex> lk(self->mu_);
    if (ev == NNSX_TRAINER_EVENT_TRAINING_COMPLETION) self->complete_ = true;
    ++self->events_;
    self->cv_.notify_all();
  }
  const NNSX_TrainerFramework* fw_;
  TrainerProperties p_;
  std::string cfg_, save_, load_;
  NNSX_TrainerProperties c_;
  void* priv_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  bool complete_ = false, stopped_ = false;
  uint64_t events_ = 0;
};

class CTrainer : public TrainerFramework {
 public:
  explicit CTrainer(const NNSX_TrainerFramework* fw) : fw_(fw) {}
  std::string name() const override { return fw_->name; }
  std::unique_ptr<TrainerInstance> create(const TrainerProperties& props) override {
    return std::make_unique<CTrainerInstance>(fw_, props);
  }

 private:
  const NNSX_TrainerFramework* fw_;
};

// ------------------------------------------------------ framework=cpp ----
// objects of <nnsx/tensor_filter_cpp.hh>, reached through their C thunks
class CppOpsFilter : public CppFilter {
 public:
  CppOpsFilter(void* obj, const NNSX_CppFilterOps* ops) : obj_(obj), ops_(ops) {}
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    NNSX_TensorsInfo a, b;
    std::memset(&a, 0, sizeof(a));
    std::memset(&b, 0, sizeof(b));
    if (ops_->getInputDim(obj_, &a) != 0 || ops_->getOutputDim(obj_, &b) != 0) return false;
    if (!from_c_info(a, in) || !from_c_info(b, out)) return false;
    out_ = *out;
    return true;
  }
  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override {
    NNSX_TensorsInfo a, b;
    to_c_info(in, &a);
    std::memset(&b, 0, sizeof(b));
    if (ops_->setInputDim(obj_, &a, &b) != 0 || !from_c_info(b, out)) return false;
    out_ = *out;
    return true;
  }
  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext&) override {
    NNSX_TensorMemory ci[NNSX_SIZE_LIMIT], co[NNSX_SIZE_LIMIT];
    std::memset(ci, 0, sizeof(ci));
    std::memset(co, 0, sizeof(co));
    for (size_t i = 0; i < in.size() && i < NNSX_SIZE_LIMIT; ++i) {
      ci[i].data = const_cast<void*>(in[i]->map_host());
      ci[i].size = in[i]->size();
    }
    const bool pre = ops_->isAllocatedBeforeInvoke(obj_) != 0;
    const unsigned nout = std::min<unsigned>(out_.num_tensors, NNSX_SIZE_LIMIT);
    std::vector<MemoryPtr> mem;
    for (unsigned i = 0; i < nout; ++i) {
      co[i].size = out_.size(static_cast<int>(i));
      if (pre) {
        mem.push_back(Memory::alloc_host(co[i].size));
        co[i].data = mem.back()->data();
      }
    }
    const int r = ops_->invoke(obj_, ci, co);
    if (r != 0) return r;
    if (!pre) {
      for (unsigned i = 0; i < nout; ++i) {
        if (!co[i].data) return -EINVAL;
        mem.push_back(adopt_malloc(co[i].data, co[i].size));
      }
    }
    *out = std::move(mem);
    return 0;
  }

 private:
  void* obj_;
  const NNSX_CppFilterOps* ops_;
  TensorsInfo out_;
};

int reg_cpp(const char* name, void* obj, const void* ops_v) {
  auto* ops = static_cast<const NNSX_CppFilterOps*>(ops_v);
  if (!name || !*name || !obj || !ops || !ops->invoke || !ops->isAllocatedBeforeInvoke) return -EINVAL;
  return register_cpp_filter(name, [obj, ops](const FilterProperties&) {
           return std::unique_ptr<CppFilter>(new CppOpsFilter(obj, ops));
         }) ? 0 : -EINVAL;
}
int unreg_cpp(const char* name) { return name && unregister_cpp_filter(name) ? 0 : -ENOENT; }

// --------------------------------------------------------------- decoders ----
class CDecoderInstance : public DecoderInstance {
 public:
  explicit CDecoderInstance(const NNSX_Decoder* d) : d_(d) {
    if (d_->init && d_->init(&priv_) != 0) throw Error(std::string("decoder ") + d_->modename + ": init failed");
  }
  ~CDecoderInstance() override {
    if (d_->exit) d_->exit(&priv_);
  }
  bool set_option(int idx, const std::string& value) override {
    return !d_->setOption || d_->setOption(&priv_, idx, value.c_str()) == 0;
  }
  Caps get_out_caps(const TensorsConfig& config) override {
    if (!d_->getOutCaps) return Caps();
    NNSX_TensorsConfig c;
    to_c_config(config, &c);
    const std::string s = take_string(d_->getOutCaps(&priv_, &c));
    return s.empty() ? Caps() : Caps::from_string(s);
  }
  FlowReturn decode(const TensorsConfig& config, const std::vector<MemoryPtr>& in, Buffer* out,
                    InvokeContext&) override {
    NNSX_TensorsConfig c;
    to_c_config(config, &c);
    NNSX_TensorMemory ci[NNSX_SIZE_LIMIT];
    std::memset(ci, 0, sizeof(ci));
    size_t in_size = 0;
    for (size_t i = 0; i < in.size() && i < NNSX_SIZE_LIMIT; ++i) {
      ci[i].data = const_cast<void*>(in[i]->map_host());
      ci[i].size = in[i]->size();
      in_size += ci[i].size;
    }
    NNSX_TensorMemory co{nullptr, 0};
    MemoryPtr pre;
    if (d_->getTransformSize) {
      const size_t n = d_->getTransformSize(&priv_, &c, in_size);
      if (n > 0) {
        pre = Memory::alloc_host(n);
        co.data = pre->data();
        co.size = n;
      }
    }
    if (d_->decode(&priv_, &c, ci, &co) != 0) return FlowReturn::ERROR;
    if (pre && co.data == pre->data()) {
      out->mems.push_back(co.size < pre->size() ? Memory::view(pre, 0, co.size) : pre);
    } else {
      if (!co.data) return FlowReturn::ERROR;
      out->mems.push_back(adopt_malloc(co.data, co.size));
    }
    return FlowReturn::OK;
  }

 private:
  const NNSX_Decoder* d_;
  void* priv_ = nullptr;
};

class CDecoder : public DecoderSubplugin {
 public:
  explicit CDecoder(const NNSX_Decoder* d) : d_(d) {}
  std::string name() const override { return d_->modename; }
  std::unique_ptr<DecoderInstance> create() override { return std::make_unique<CDecoderInstance>(d_); }

 private:
  const NNSX_Decoder* d_;
};

// ------------------------------------------------------------- converters ----
class CConverter : public ConverterSubplugin {
 public:
  explicit CConverter(const NNSX_Converter* c) : c_(c) {}
  std::string name() const override { return c_->name; }
  Caps query_caps() const override {
    if (!c_->query_caps) return Caps();
    const std::string s = take_string(c_->query_caps());
    return s.empty() ? Caps() : Caps::from_string(s);
  }
  bool get_out_config(const Caps& in, TensorsConfig* config) override {
    if (!c_->get_out_config) return false;
    NNSX_TensorsConfig c;
    std::memset(&c, 0, sizeof(c));
    if (c_->get_out_config(in.to_string().c_str(), &c) != 0 || !from_c_info(c.info, &config->info)) return false;
    config->rate_n = c.rate_n;
    config->rate_d = c.rate_d;
    return true;
  }
  BufferPtr convert(const BufferPtr& in, TensorsConfig* config) override {
    std::vector<char> bytes;
    for (auto& m : in->mems) {
      const char* p = static_cast<const char*>(m->map_host());
      bytes.insert(bytes.end(), p, p + m->size());
    }
    NNSX_TensorMemory src{bytes.data(), bytes.size()};
    NNSX_TensorsConfig c;
    std::memset(&c, 0, sizeof(c));
    NNSX_TensorMemory out[NNSX_SIZE_LIMIT];
    std::memset(out, 0, sizeof(out));
    if (c_->convert(&src, &c, out) != 0) return nullptr;
    if (!from_c_info(c.info, &config->info)) {
      NNSX_LOGE("c_plugin", "converter ", c_->name, " returned num_tensors=", c.info.num_tensors);
      for (auto& o : out) std::free(o.data);
      return nullptr;
    }
    config->rate_n = c.rate_n;
    config->rate_d = c.rate_d;
    auto b = make_buffer();
    b->copy_metadata_from(*in);
    for (unsigned i = 0; i < c.info.num_tensors; ++i) b->mems.push_back(adopt_malloc(out[i].data, out[i].size));
    return b;
  }

 private:
  const NNSX_Converter* c_;
};

// ------------------------------------------------------------ registration ----
int reg_filter(const NNSX_FilterFramework* fw) {
  if (fw && fw->version == NNSX_FILTER_FRAMEWORK_V0) {  // the legacy table (same leading version word)
    auto* v0 = reinterpret_cast<const NNSX_FilterFrameworkV0*>(fw);
    if (!v0->name || !v0->invoke_NN) return -EINVAL;
    return register_filter_framework(std::make_shared<CFilterFrameworkV0>(v0)) ? 0 : -EINVAL;
  }
  if (!fw || !fw->name || !fw->invoke) return -EINVAL;
  if (fw->version != NNSX_FILTER_FRAMEWORK_V1 && fw->version != NNSX_FILTER_FRAMEWORK_V2) {
    NNSX_LOGE("c_plugin", "filter framework ", fw->name, ": unsupported ABI version ", fw->version);
    return -EINVAL;
  }
  try {
    return register_filter_framework(std::make_shared<CFilterFramework>(fw)) ? 0 : -EINVAL;
  } catch (const std::exception& e) {
    NNSX_LOGE("c_plugin", "filter framework ", fw->name, ": ", e.what());
    return -EINVAL;
  }
}
int unreg_filter(const char* name) {
  return name && Registry::get().remove(SubpluginKind::FILTER, name) ? 0 : -ENOENT;
}
int reg_decoder(const NNSX_Decoder* d) {
  if (!d || !d->modename || !d->decode) return -EINVAL;
  return register_decoder(std::make_shared<CDecoder>(d)) ? 0 : -EINVAL;
}
int unreg_decoder(const char* name) {
  return name && Registry::get().remove(SubpluginKind::DECODER, name) ? 0 : -ENOENT;
}
int reg_converter(const NNSX_Converter* c) {
  if (!c || !c->name || !c->convert) return -EINVAL;
  return register_converter(std::make_shared<CConverter>(c)) ? 0 : -EINVAL;
}
int unreg_converter(const char* name) {
  return name && Registry::get().remove(SubpluginKind::CONVERTER, name) ? 0 : -ENOENT;
}
int reg_trainer(const NNSX_TrainerFramework* t) {
  if (!t || !t->name || !t->push_data || !t->getFrameworkInfo) return -EINVAL;
  if (t->version != NNSX_TRAINER_FRAMEWORK_V1) {
    NNSX_LOGE("c_plugin", "trainer ", t->name, ": unsupported ABI version ", t->version);
    return -EINVAL;
  }
  return register_trainer(std::make_shared<CTrainer>(t)) ? 0 : -EINVAL;
}
int unreg_trainer(const char* name) {
  return name && Registry::get().remove(SubpluginKind::TRAINER, name) ? 0 : -ENOENT;
}
void host_log(int level, const char* cat, const char* msg) {
  const char* c = cat ? cat : "subplugin";
  const char* m = msg ? msg : "";
  switch (level) {
    case 0: NNSX_LOGE(c, m); break;
    case 1: NNSX_LOGW(c, m); break;
    case 2: NNSX_LOGI(c, m); break;
    default: NNSX_LOGD(c, m); break;
  }
}

const NNSX_PluginHost kHost = {NNSX_PLUGIN_ABI_VERSION, reg_filter, unreg_filter,  reg_decoder,
                               unreg_decoder,           reg_converter, unreg_converter, host_log,
                               reg_trainer,             unreg_trainer, reg_cpp,       unreg_cpp};

// every library the registry loads: run its nnsx_subplugin_init(&host), if any
void on_library(void* handle, const std::string& path) {
  auto init = reinterpret_cast<NNSX_SubpluginInitFunc>(dlsym(handle, NNSX_SUBPLUGIN_INIT_SYMBOL));
  if (!init) return;  // an in-tree style library that registers itself
  const int r = init(&kHost);
  if (r != 0) NNSX_LOGW("c_plugin", path, ": nnsx_subplugin_init returned ", r);
}

struct HookInstaller {
  HookInstaller() { Registry::get().set_library_hook(&on_library); }
} g_hook_installer;

}  // namespace
}  // namespace nnsx

extern "C" {
__attribute__((visibility("default"))) int nnstreamer_filter_probe(const NNSX_FilterFramework* fw) {
  return nnsx::reg_filter(fw);
}
__attribute__((visibility("default"))) int nnstreamer_filter_exit(const char* name) {
  return nnsx::unreg_filter(name);
}
__attribute__((visibility("default"))) int nnstreamer_decoder_probe(const NNSX_Decoder* dec) {
  return nnsx::reg_decoder(dec);
}
__attribute__((visibility("default"))) int nnstreamer_decoder_exit(const char* modename) {
  return nnsx::unreg_decoder(modename);
}
__attribute__((visibility("default"))) int registerExternalConverter(const NNSX_Converter* conv) {
  return nnsx::reg_converter(conv);
}
__attribute__((visibility("default"))) int unregisterExternalConverter(const char* name) {
  return nnsx::unreg_converter(name);
}
__attribute__((visibility("default"))) int nnstreamer_cpp_filter_register(const char* name, void* obj,
                                                                          const void* ops) {
  return nnsx::reg_cpp(name, obj, ops);
}
__attribute__((visibility("default"))) int nnstreamer_cpp_filter_unregister(const char* name) {
  return nnsx::unreg_cpp(name);
}
__attribute__((visibility("default"))) int nnstreamer_trainer_probe(const NNSX_TrainerFramework* ttsp) {
  return nnsx::reg_trainer(ttsp);
}
__attribute__((visibility("default"))) int nnstreamer_trainer_exit(const char* name) {
  return nnsx::unreg_trainer(name);
}
}
