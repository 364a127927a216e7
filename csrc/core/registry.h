// Sub-plugin registry (filters, decoders, converters, trainers) and the
// configuration system.
//
// Lookup order follows gst/nnstreamer/nnstreamer_subplugin.c:71-171: an
// in-process registration wins; on a miss the registry dlopen()s
// `lib<prefix><name>.so` from the configured search paths and retries (the
// .so registers itself from a static constructor).  "any"/"auto" are reserved.
// Configuration (.ini + env) follows gst/nnstreamer/nnstreamer_conf.c.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace nnsx {

enum class SubpluginKind { FILTER = 0, DECODER, CONVERTER, TRAINER, CUSTOM_DECODER, CUSTOM_CONVERTER, CUSTOM_IF };
const char* subplugin_kind_name(SubpluginKind k);
const char* subplugin_prefix(SubpluginKind k);  // "libnnstreamer_filter_" style file prefix

class Registry {
 public:
  static Registry& get();
  // obj: type-erased shared object (FilterFramework, DecoderSubplugin, ...)
  bool add(SubpluginKind kind, const std::string& name, std::shared_ptr<void> obj);
  bool remove(SubpluginKind kind, const std::string& name);
  std::shared_ptr<void> find(SubpluginKind kind, const std::string& name, bool try_load = true);
  std::vector<std::string> names(SubpluginKind kind, bool scan_paths = false);
  // dlopen a shared object explicitly
  bool load_library(const std::string& path, std::string* err = nullptr);
  // called after every successful load_library() (outside the registry lock):
  // the C sub-plugin ABI uses it to run the library's nnsx_subplugin_init()
  using LibraryHook = void (*)(void* handle, const std::string& path);
  void set_library_hook(LibraryHook h) { hook_ = h; }

  template <typename T>
  std::shared_ptr<T> find_as(SubpluginKind kind, const std::string& name, bool try_load = true) {
    return std::static_pointer_cast<T>(find(kind, name, try_load));
  }

 private:
  Registry() = default;
  std::mutex mu_;
  std::map<int, std::map<std::string, std::shared_ptr<void>>> tables_;
  std::vector<void*> handles_;
  LibraryHook hook_ = nullptr;
};

// -------------------------------------------------------------- config ----
class Config {
 public:
  static Config& get();
  // reload from $NNSTREAMER_CONF / $NNSX_CONF / /etc/nnstreamer.ini
  void load(const std::string& explicit_path = "");
  std::string path() const;
  // [common] enable_envvar etc.
  bool envvar_enabled() const;
  // Search paths for a sub-plugin kind (env NNSTREAMER_FILTERS etc. first when enabled)
  std::vector<std::string> paths(SubpluginKind kind) const;
  // Custom key: env NNSTREAMER_<group>_<key> first, then the ini.
  std::string custom_value(const std::string& group, const std::string& key, const std::string& def = "") const;
  bool custom_bool(const std::string& group, const std::string& key, bool def) const;
  void set_value(const std::string& group, const std::string& key, const std::string& value);
  std::string dump() const;  // nnsx-check style dump

 private:
  Config();
  mutable std::mutex mu_;
  std::string path_;
  std::map<std::string, std::map<std::string, std::string>> ini_;
};

}  // namespace nnsx
