/*
 * C++ base for tensor_filter framework sub-plugins.  Reference:
 * gst/nnstreamer/include/nnstreamer_cppplugin_api_filter.hh:67-198
 * (nnstreamer::tensor_filter_subplugin, register_subplugin<T>()).
 *
 * Header-only over the C ABI (<nnsx/nnsx_plugin_api.h>, a V2
 * NNSX_FilterFramework table whose subplugin_data is the class's "empty"
 * object): a sub-plugin built with any C++11 compiler needs no link-time
 * dependency on the runtime.  A framework is a class derived from
 * nnsx::tensor_filter_subplugin; its shared object registers it from
 * nnsx_subplugin_init():
 *
 *   class my_fw : public nnsx::tensor_filter_subplugin { ... };
 *   static my_fw *reg;
 *   extern "C" int nnsx_subplugin_init(const NNSX_PluginHost *host) {
 *     reg = nnsx::tensor_filter_subplugin::register_subplugin<my_fw>(host);
 *     return reg ? 0 : -1;
 *   }
 *
 * Each opened tensor_filter gets its own object from getEmptyInstance(),
 * configured by configure_instance(); exceptions thrown by the virtual
 * methods become -EINVAL returns.
 */
#ifndef NNSX_CPPPLUGIN_API_FILTER_HH
#define NNSX_CPPPLUGIN_API_FILTER_HH

#include <dlfcn.h>
#include <nnsx/nnsx_plugin_api.h>

#include <cerrno>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace nnsx {

class tensor_filter_subplugin {
 public:
  tensor_filter_subplugin() { std::memset(&fwdesc_, 0, sizeof(fwdesc_)); }
  virtual ~tensor_filter_subplugin() = default;

  /* ---- to be implemented by sub-plugin authors ---- */
  // a newly created non-functional ("empty") object of the derived class
  virtual tensor_filter_subplugin &getEmptyInstance() = 0;
  // make an empty object a functional one for these properties (throw on failure)
  virtual void configure_instance(const NNSX_FilterProperties *prop) = 0;
  // host invoke (throw on failure)
  virtual void invoke(const NNSX_TensorMemory *input, NNSX_TensorMemory *output) = 0;
  // nnsx: device-aware invoke; ctx.device >= 0 means device pointers ordered on
  // ctx.stream.  The default serves host invokes only.
  virtual void invoke(const NNSX_TensorMemory *input, NNSX_TensorMemory *output, const NNSX_InvokeContext &ctx) {
    if (ctx.device >= 0) throw std::invalid_argument("this framework has no device invoke");
    invoke(input, output);
  }
  // static info; an empty object answers with its defaults.  name must not change.
  virtual void getFrameworkInfo(NNSX_FrameworkInfo &info) = 0;
  // -ENOENT: op not available; -EINVAL: invalid request
  virtual int getModelInfo(NNSX_ModelInfoOps ops, NNSX_TensorsInfo &in_info, NNSX_TensorsInfo &out_info) = 0;
  // optional; -ENOENT = not handled (DESTROY_NOTIFY: the runtime frees with free())
  virtual int eventHandler(NNSX_FilterEvent ops, const void *data) {
    (void)ops;
    (void)data;
    return -ENOENT;
  }

  /* ---- registration ---- */
  // creates the class's empty object, fills its C table and registers it
  // (through `host`, or the runtime's exported nnstreamer_filter_probe when null)
  template <typename T>
  static T *register_subplugin(const NNSX_PluginHost *host = nullptr) {
    static_assert(std::is_base_of<tensor_filter_subplugin, T>::value, "T must derive from tensor_filter_subplugin");
    T *empty = new T();
    NNSX_FrameworkInfo info;
    std::memset(&info, 0, sizeof(info));
    empty->getFrameworkInfo(info);
    if (!info.name) {
      delete empty;
      return nullptr;
    }
    empty->name_ = info.name;
    NNSX_FilterFramework &d = empty->fwdesc_;
    d.version = NNSX_FILTER_FRAMEWORK_V2;
    d.name = empty->name_.c_str();
    d.open = &tensor_filter_subplugin::c_open;
    d.close = &tensor_filter_subplugin::c_close;
    d.getFrameworkInfo = &tensor_filter_subplugin::c_info;
    d.getModelInfo = &tensor_filter_subplugin::c_model;
    d.invoke = &tensor_filter_subplugin::c_invoke;
    d.destroyNotify = nullptr;  // DESTROY_NOTIFY goes through eventHandler
    d.eventHandler = &tensor_filter_subplugin::c_event;
    d.subplugin_data = static_cast<tensor_filter_subplugin *>(empty);
    const int r = host ? host->register_filter(&d) : runtime_call<int (*)(const NNSX_FilterFramework *)>(
                                                          "nnstreamer_filter_probe", &d);
    if (r != 0) {
      delete empty;
      return nullptr;
    }
    return empty;
  }
  template <typename T>
  static void unregister_subplugin(T *empty, const NNSX_PluginHost *host = nullptr) {
    if (!empty) return;
    if (host)
      host->unregister_filter(empty->name_.c_str());
    else
      runtime_call<int (*)(const char *)>("nnstreamer_filter_exit", empty->name_.c_str());
    delete empty;
  }

 private:
  // the runtime's exported entry points, looked up when called (no link-time
  // dependency: a shared object that only uses the host table loads anywhere)
  template <typename F, typename A>
  static int runtime_call(const char *sym, A arg) {
    F f = reinterpret_cast<F>(dlsym(RTLD_DEFAULT, sym));
    return f ? f(arg) : -ENOSYS;
  }
  static tensor_filter_subplugin *self_of(void *p) { return static_cast<tensor_filter_subplugin *>(p); }

  // *pd arrives as the class's empty object (V2 subplugin_data); leaves as the instance
  static int c_open(const NNSX_FilterProperties *prop, void **pd) {
    tensor_filter_subplugin *obj = nullptr;
    try {
      obj = &self_of(*pd)->getEmptyInstance();
      obj->configure_instance(prop);
    } catch (const std::exception &) {
      delete obj;
      return -EINVAL;
    }
    *pd = obj;
    return 0;
  }
  static void c_close(const NNSX_FilterProperties *prop, void **pd) {
    (void)prop;
    delete self_of(*pd);
    *pd = nullptr;
  }
  static int c_info(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd,
                    NNSX_FrameworkInfo *info) {
    (void)prop;
    try {
      self_of(pd ? pd : self->subplugin_data)->getFrameworkInfo(*info);
    } catch (const std::exception &) {
      return -EINVAL;
    }
    return 0;
  }
  static int c_model(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd,
                     NNSX_ModelInfoOps ops, NNSX_TensorsInfo *in, NNSX_TensorsInfo *out) {
    (void)self;
    (void)prop;
    try {
      return self_of(pd)->getModelInfo(ops, *in, *out);
    } catch (const std::exception &) {
      return -EINVAL;
    }
  }
  static int c_invoke(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd,
                      const NNSX_TensorMemory *in, NNSX_TensorMemory *out, const NNSX_InvokeContext *ctx) {
    (void)self;
    (void)prop;
    try {
      self_of(pd)->invoke(in, out, *ctx);
    } catch (const std::exception &) {
      return -EINVAL;
    }
    return 0;
  }
  static int c_event(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd, NNSX_FilterEvent ev,
                     const void *data) {
    (void)prop;
    try {
      return self_of(pd ? pd : self->subplugin_data)->eventHandler(ev, data);
    } catch (const std::exception &) {
      return -EINVAL;
    }
  }

  NNSX_FilterFramework fwdesc_;
  std::string name_;
};

}  // namespace nnsx

#endif /* NNSX_CPPPLUGIN_API_FILTER_HH */
