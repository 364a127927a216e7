/*
 * tensor_filter framework=cpp: C++ filter objects registered by name.
 * Reference: ext/nnstreamer/tensor_filter/tensor_filter_cpp.hh (class
 * tensor_filter_cpp, __register / __unregister; pipelines use
 * `tensor_filter framework=cpp model=<name>` or `model=<name>,lib.so`).
 *
 * Header-only over the C ABI (NNSX_CppFilterOps thunks): an object lives in
 * the application or in a shared object and registers itself --
 *
 *   class myfilter : public nnsx::tensor_filter_cpp {
 *    public:
 *     myfilter() : tensor_filter_cpp("myfilter01") {}
 *     int getInputDim(NNSX_TensorsInfo *info) override { ... }
 *     ...
 *   };
 *   // in an application linked against the runtime:
 *   static myfilter fx;  fx._register();
 *   // in a shared object loaded through model=myfilter01,libabc.so:
 *   extern "C" int nnsx_subplugin_init(const NNSX_PluginHost *host) {
 *     static myfilter fx;
 *     return fx._register(host);
 *   }
 *
 * Model names must be unique across the objects of a process.
 */
#ifndef NNSX_TENSOR_FILTER_CPP_HH
#define NNSX_TENSOR_FILTER_CPP_HH

#include <dlfcn.h>
#include <nnsx/nnsx_plugin_api.h>

#include <cerrno>
#include <string>

namespace nnsx {

class tensor_filter_cpp {
 public:
  explicit tensor_filter_cpp(const char *modelName) : name_(modelName ? modelName : "") {}
  virtual ~tensor_filter_cpp() = default;

  /* fill {getInputDim and getOutputDim} and/or setInputDim; return -EINVAL if unsupported */
  virtual int getInputDim(NNSX_TensorsInfo *info) = 0;
  virtual int getOutputDim(NNSX_TensorsInfo *info) = 0;
  virtual int setInputDim(const NNSX_TensorsInfo *in, NNSX_TensorsInfo *out) = 0;
  /* host memories; when !isAllocatedBeforeInvoke() out[i].data is malloc()ed here */
  virtual int invoke(const NNSX_TensorMemory *in, NNSX_TensorMemory *out) = 0;
  /* true: the runtime allocates the outputs before invoke (must not change) */
  virtual bool isAllocatedBeforeInvoke() = 0;

  const char *model_name() const { return name_.c_str(); }

  /* register / unregister through a sub-plugin host table, or (host == null)
   * through the runtime's exported nnstreamer_cpp_filter_register */
  int _register(const NNSX_PluginHost *host = nullptr) {
    if (host) {
      if (host->abi_version < 2 || !host->register_cpp_filter) return -ENOTSUP;
      return host->register_cpp_filter(name_.c_str(), this, &ops());
    }
    auto f = reinterpret_cast<int (*)(const char *, void *, const void *)>(
        dlsym(RTLD_DEFAULT, "nnstreamer_cpp_filter_register"));  // (no link-time dependency)
    return f ? f(name_.c_str(), this, &ops()) : -ENOSYS;
  }
  int _unregister(const NNSX_PluginHost *host = nullptr) {
    if (host) return host->abi_version >= 2 ? host->unregister_cpp_filter(name_.c_str()) : -ENOTSUP;
    auto f = reinterpret_cast<int (*)(const char *)>(dlsym(RTLD_DEFAULT, "nnstreamer_cpp_filter_unregister"));
    return f ? f(name_.c_str()) : -ENOSYS;
  }
  static int __register(tensor_filter_cpp *filter, const NNSX_PluginHost *host = nullptr) {
    return filter ? filter->_register(host) : -EINVAL;
  }

 private:
  static tensor_filter_cpp *self_of(void *o) { return static_cast<tensor_filter_cpp *>(o); }
  static int t_in(void *o, NNSX_TensorsInfo *i) { return self_of(o)->getInputDim(i); }
  static int t_out(void *o, NNSX_TensorsInfo *i) { return self_of(o)->getOutputDim(i); }
  static int t_set(void *o, const NNSX_TensorsInfo *a, NNSX_TensorsInfo *b) { return self_of(o)->setInputDim(a, b); }
  static int t_alloc(void *o) { return self_of(o)->isAllocatedBeforeInvoke() ? 1 : 0; }
  static int t_invoke(void *o, const NNSX_TensorMemory *a, NNSX_TensorMemory *b) { return self_of(o)->invoke(a, b); }
  static const NNSX_CppFilterOps &ops() {
    static const NNSX_CppFilterOps k = {&t_in, &t_out, &t_set, &t_alloc, &t_invoke};
    return k;
  }

  std::string name_;
};

}  // namespace nnsx

#endif /* NNSX_TENSOR_FILTER_CPP_HH */
