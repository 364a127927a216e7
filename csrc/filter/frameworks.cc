// Built-in host filter frameworks:
//   custom       C shared object exporting NNStreamer_custom
//                (gst/nnstreamer/tensor_filter/tensor_filter_custom.c:64-330)
//   custom-easy  in-process callbacks (tensor_filter_custom_easy.c:73-257)
//   cpp          C++ classes registered by name (ext/.../tensor_filter_cpp.cc)
#include <dlfcn.h>

#include <cstring>

#include "../../include/nnsx/tensor_filter_custom.h"
#include "core/log.h"
#include "filter/filter.h"
#include "runtime/plugin_api.h"

namespace nnsx {

bool custom_easy_lookup(const std::string& name, CustomEasyFn* fn, TensorsInfo* in, TensorsInfo* out);

namespace {

void to_c(const TensorsInfo& a, NNSX_TensorsInfo* b) {
  std::memset(b, 0, sizeof(*b));
  b->num_tensors = std::min<unsigned>(a.num_tensors, NNSX_SIZE_LIMIT);
  b->format = static_cast<uint32_t>(a.format);
  for (unsigned i = 0; i < b->num_tensors; ++i) {
    b->info[i].type = static_cast<uint32_t>(a.at(i).type);
    for (int d = 0; d < kRankLimit; ++d) b->info[i].dimension[d] = a.at(i).dim[d];
    b->info[i].name = nullptr;
  }
}

void from_c(const NNSX_TensorsInfo& b, TensorsInfo* a) {
  // the count comes from a user plugin: never index past info[NNSX_SIZE_LIMIT]
  if (b.num_tensors > NNSX_SIZE_LIMIT)
    throw Error("plugin returned num_tensors=" + std::to_string(b.num_tensors) + " (limit " +
                std::to_string(NNSX_SIZE_LIMIT) + ")");
  *a = TensorsInfo();
  a->resize(b.num_tensors);
  a->format = static_cast<Format>(b.format);
  for (unsigned i = 0; i < b.num_tensors; ++i) {
    a->at(i).type = static_cast<DType>(b.info[i].type);
    for (int d = 0; d < kRankLimit; ++d) a->at(i).dim[d] = b.info[i].dimension[d] ? b.info[i].dimension[d] : 1;
    if (b.info[i].name) a->at(i).name = b.info[i].name;
  }
}

// ---------------------------------------------------------------- custom ----
class CustomSo : public FilterInstance {
 public:
  explicit CustomSo(FilterProperties& p) : props_(p) {
    const std::string& path = p.model_files.at(0);
    handle_ = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!handle_) throw Error("cannot open custom filter " + path + ": " + dlerror());
    auto** cls = reinterpret_cast<NNStreamer_custom_class**>(dlsym(handle_, "NNStreamer_custom"));
    if (!cls || !*cls) throw Error("custom filter " + path + " does not export NNStreamer_custom");
    cls_ = *cls;
    if ((cls_->invoke != nullptr) == (cls_->allocate_invoke != nullptr))
      throw Error("custom filter must define exactly one of invoke / allocate_invoke");
    model_c_ = path;
    models_[0] = model_c_.c_str();
    cprop_.fwname = "custom";
    cprop_.model_files = models_;
    cprop_.num_models = 1;
    cprop_.custom_properties = props_.custom_properties.c_str();
    to_c(p.input_info, &cprop_.input_meta);
    to_c(p.output_info, &cprop_.output_meta);
    priv_ = cls_->initfunc ? cls_->initfunc(&cprop_) : nullptr;
  }
  ~CustomSo() override {
    if (cls_ && cls_->exitfunc) cls_->exitfunc(priv_, &cprop_);
    // keep the handle loaded: allocate-in-invoke outputs may still reference code in it
  }
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    if (!cls_->getInputDim || !cls_->getOutputDim) return false;
    NNSX_TensorsInfo a, b;
    std::memset(&a, 0, sizeof(a));
    std::memset(&b, 0, sizeof(b));
    if (cls_->getInputDim(priv_, &cprop_, &a) != 0 || cls_->getOutputDim(priv_, &cprop_, &b) != 0) return false;
    from_c(a, in);
    from_c(b, out);
    out_ = *out;
    return true;
  }
  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override {
    if (!cls_->setInputDim) return false;
    NNSX_TensorsInfo a, b;
    to_c(in, &a);
    std::memset(&b, 0, sizeof(b));
    if (cls_->setInputDim(priv_, &cprop_, &a, &b) != 0) return false;
    from_c(b, out);
    out_ = *out;
    to_c(in, &cprop_.input_meta);
    to_c(*out, &cprop_.output_meta);
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
    std::vector<MemoryPtr> allocated;
    if (cls_->invoke) {
      for (unsigned i = 0; i < out_.num_tensors; ++i) {
        auto m = Memory::alloc_host(out_.size(static_cast<int>(i)));
        co[i].data = m->data();
        co[i].size = m->size();
        allocated.push_back(m);
      }
      int r = cls_->invoke(priv_, &cprop_, ci, co);
      if (r != 0) return r;
      *out = allocated;
      return 0;
    }
    int r = cls_->allocate_invoke(priv_, &cprop_, ci, co);
    if (r != 0) return r;
    auto dn = cls_->destroy_notify;
    for (unsigned i = 0; i < out_.num_tensors; ++i) {
      void* p = co[i].data;
      size_t sz = co[i].size ? co[i].size : out_.size(static_cast<int>(i));
      out->push_back(Memory::wrap(p, sz, MemPlace::HOST, -1, [dn, p](Memory*) {
        if (dn)
          dn(p);
        else
          free(p);
      }));
    }
    return 0;
  }
  bool reload_model(const FilterProperties& p) override {
    (void)p;
    return false;
  }

 private:
  FilterProperties props_;
  void* handle_ = nullptr;
  NNStreamer_custom_class* cls_ = nullptr;
  void* priv_ = nullptr;
  std::string model_c_;
  const char* models_[1] = {nullptr};
  NNSX_FilterProperties cprop_{};
  TensorsInfo out_;
};

class CustomFw : public FilterFramework {
 public:
  std::string name() const override { return "custom"; }
  std::unique_ptr<FilterInstance> open(FilterProperties& p) override { return std::make_unique<CustomSo>(p); }
  std::vector<std::string> model_extensions() const override { return {".so"}; }
  bool allocate_in_invoke() const override { return false; }
};

// ----------------------------------------------------------- custom-easy ----
class CustomEasy : public FilterInstance {
 public:
  explicit CustomEasy(FilterProperties& p) {
    if (!custom_easy_lookup(p.model_files.at(0), &fn_, &in_, &out_))
      throw Error("custom-easy model '" + p.model_files.at(0) + "' is not registered");
  }
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    *in = in_;
    *out = out_;
    return true;
  }
  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext&) override {
    return fn_(in, out, in_, out_);
  }

 private:
  CustomEasyFn fn_;
  TensorsInfo in_, out_;
};

class CustomEasyFw : public FilterFramework {
 public:
  std::string name() const override { return "custom-easy"; }
  bool verify_model_path() const override { return false; }  // the model is a registered name
  std::unique_ptr<FilterInstance> open(FilterProperties& p) override { return std::make_unique<CustomEasy>(p); }
};

// ------------------------------------------------------------------- cpp ----
std::mutex g_cpp_mu;
std::map<std::string, CppFilterFactory>& cpp_table() {
  static auto* t = new std::map<std::string, CppFilterFactory>();
  return *t;
}

class CppInstance : public FilterInstance {
 public:
  explicit CppInstance(FilterProperties& p) {
    // model = "Name", "Name,lib.so" (the reference order) or "lib.so,Name": the
    // library registers its objects when loaded (nnsx_subplugin_init or a
    // constructor); it is not loaded when Name is already registered
    std::string cls, lib;
    for (const auto& m : p.model_files) {
      if (m.size() > 3 && m.compare(m.size() - 3, 3, ".so") == 0)
        lib = m;
      else
        cls = m;
    }
    auto lookup = [&](CppFilterFactory* f) {
      std::lock_guard<std::mutex> lk(g_cpp_mu);
      auto it = cpp_table().find(cls);
      if (it == cpp_table().end()) return false;
      *f = it->second;
      return true;
    };
    CppFilterFactory f;
    if (!lookup(&f)) {
      if (!lib.empty()) Registry::get().load_library(lib);
      if (!lookup(&f)) throw Error("cpp filter '" + cls + "' is not registered");
    }
    obj_ = f(p);
  }
  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override { return obj_->get_model_info(in, out); }
  bool set_input_info(const TensorsInfo& in, TensorsInfo* out) override { return obj_->set_input_info(in, out); }
  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext& ctx) override {
    return obj_->invoke(in, out, ctx);
  }

 private:
  std::unique_ptr<CppFilter> obj_;
};

class CppFw : public FilterFramework {
 public:
  std::string name() const override { return "cpp"; }
  bool verify_model_path() const override { return false; }  // the model is a registered name
  std::unique_ptr<FilterInstance> open(FilterProperties& p) override { return std::make_unique<CppInstance>(p); }
};

}  // namespace

bool register_cpp_filter(const std::string& name, CppFilterFactory f) {
  std::lock_guard<std::mutex> lk(g_cpp_mu);
  cpp_table()[name] = std::move(f);
  return true;
}

bool unregister_cpp_filter(const std::string& name) {
  std::lock_guard<std::mutex> lk(g_cpp_mu);
  return cpp_table().erase(name) > 0;
}

void register_host_frameworks() {
  register_filter_framework(std::make_shared<CustomFw>());
  register_filter_framework(std::make_shared<CustomEasyFw>());
  register_filter_framework(std::make_shared<CppFw>());
}

}  // namespace nnsx
