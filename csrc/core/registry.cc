#include "core/registry.h"

#include <dirent.h>
#include <dlfcn.h>
#include <sys/stat.h>

#include <cstdlib>
#include <fstream>

#include "core/log.h"
#include "core/util.h"

namespace nnsx {

const char* subplugin_kind_name(SubpluginKind k) {
  switch (k) {
    case SubpluginKind::FILTER: return "filter";
    case SubpluginKind::DECODER: return "decoder";
    case SubpluginKind::CONVERTER: return "converter";
    case SubpluginKind::TRAINER: return "trainer";
    case SubpluginKind::CUSTOM_DECODER: return "custom-decoder";
    case SubpluginKind::CUSTOM_CONVERTER: return "custom-converter";
    case SubpluginKind::CUSTOM_IF: return "custom-if";
  }
  return "?";
}

const char* subplugin_prefix(SubpluginKind k) {
  switch (k) {
    case SubpluginKind::FILTER: return "libnnstreamer_filter_";
    case SubpluginKind::DECODER: return "libnnstreamer_decoder_";
    case SubpluginKind::CONVERTER: return "libnnstreamer_converter_";
    case SubpluginKind::TRAINER: return "libnnstreamer_trainer_";
    default: return "libnnstreamer_custom_";
  }
}

Registry& Registry::get() {
  static Registry* r = new Registry();
  return *r;
}

bool Registry::add(SubpluginKind kind, const std::string& name, std::shared_ptr<void> obj) {
  if (name.empty() || name == "any" || name == "auto") {
    NNSX_LOGE("registry", "cannot register sub-plugin with reserved name '", name, "'");
    return false;
  }
  std::lock_guard<std::mutex> lk(mu_);
  auto& t = tables_[static_cast<int>(kind)];
  if (t.count(name)) NNSX_LOGW("registry", "sub-plugin ", name, " (", subplugin_kind_name(kind), ") is overridden");
  t[name] = std::move(obj);
  return true;
}

bool Registry::remove(SubpluginKind kind, const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  return tables_[static_cast<int>(kind)].erase(name) > 0;
}

bool Registry::load_library(const std::string& path, std::string* err) {
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    if (err) *err = dlerror();
    return false;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    handles_.push_back(h);
  }
  if (hook_) hook_(h, path);
  return true;
}

std::shared_ptr<void> Registry::find(SubpluginKind kind, const std::string& name, bool try_load) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto& t = tables_[static_cast<int>(kind)];
    auto it = t.find(name);
    if (it != t.end()) return it->second;
  }
  if (!try_load) return nullptr;
  for (const auto& dir : Config::get().paths(kind)) {
    std::string fn = dir + "/" + subplugin_prefix(kind) + name + ".so";
    struct stat sb;
    if (stat(fn.c_str(), &sb) != 0) continue;
    std::string err;
    if (!load_library(fn, &err)) {
      NNSX_LOGW("registry", "dlopen ", fn, " failed: ", err);
      continue;
    }
    std::lock_guard<std::mutex> lk(mu_);
    auto& t = tables_[static_cast<int>(kind)];
    auto it = t.find(name);
    if (it != t.end()) return it->second;
  }
  return nullptr;
}

std::vector<std::string> Registry::names(SubpluginKind kind, bool scan_paths) {
  if (scan_paths) {
    std::string prefix = subplugin_prefix(kind);
    for (const auto& dir : Config::get().paths(kind)) {
      DIR* d = opendir(dir.c_str());
      if (!d) continue;
      while (dirent* e = readdir(d)) {
        std::string fn = e->d_name;
        if (starts_with(fn, prefix) && ends_with(fn, ".so")) {
          std::string nm = fn.substr(prefix.size(), fn.size() - prefix.size() - 3);
          find(kind, nm, true);
        }
      }
      closedir(d);
    }
  }
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> v;
  for (auto& kv : tables_[static_cast<int>(kind)]) v.push_back(kv.first);
  return v;
}

// --------------------------------------------------------------- Config ----

Config& Config::get() {
  static Config* c = new Config();
  return *c;
}

Config::Config() { load(); }

void Config::load(const std::string& explicit_path) {
  std::lock_guard<std::mutex> lk(mu_);
  ini_.clear();
  std::vector<std::string> cands;
  if (!explicit_path.empty()) cands.push_back(explicit_path);
  if (const char* e = std::getenv("NNSX_CONF")) cands.push_back(e);
  if (const char* e = std::getenv("NNSTREAMER_CONF")) cands.push_back(e);
  cands.push_back("/etc/nnstreamer.ini");
  path_.clear();
  for (const auto& c : cands) {
    std::ifstream f(c);
    if (!f) continue;
    path_ = c;
    std::string line, section;
    while (std::getline(f, line)) {
      std::string t = strip(line);
      if (t.empty() || t[0] == '#' || t[0] == ';') continue;
      if (t.front() == '[' && t.back() == ']') {
        section = strip(t.substr(1, t.size() - 2));
        continue;
      }
      auto eq = t.find('=');
      if (eq == std::string::npos) continue;
      ini_[section][strip(t.substr(0, eq))] = strip(t.substr(eq + 1));
    }
    break;
  }
  // defaults
  if (!ini_["common"].count("enable_envvar")) ini_["common"]["enable_envvar"] = "True";
  if (!ini_["pytorch"].count("enable_use_gpu")) ini_["pytorch"]["enable_use_gpu"] = "True";
}

std::string Config::path() const {
  std::lock_guard<std::mutex> lk(mu_);
  return path_;
}

bool Config::envvar_enabled() const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = ini_.find("common");
  if (it == ini_.end()) return true;
  auto jt = it->second.find("enable_envvar");
  return jt == it->second.end() ? true : to_bool(jt->second, true);
}

std::vector<std::string> Config::paths(SubpluginKind kind) const {
  std::vector<std::string> out;
  static const char* env_names[] = {"NNSTREAMER_FILTERS",    "NNSTREAMER_DECODERS", "NNSTREAMER_CONVERTERS",
                                    "NNSTREAMER_TRAINERS",   "NNSTREAMER_CUSTOMFILTERS",
                                    "NNSTREAMER_CUSTOMFILTERS", "NNSTREAMER_CUSTOMFILTERS"};
  static const char* keys[] = {"filters", "decoders", "converters", "trainers", "customfilters", "customfilters",
                               "customfilters"};
  static const char* sections[] = {"filter", "decoder", "converter", "trainer", "filter", "filter", "filter"};
  int k = static_cast<int>(kind);
  if (envvar_enabled()) {
    if (const char* e = std::getenv(env_names[k]))
      for (auto& p : split(e, ':'))
        if (!strip(p).empty()) out.push_back(strip(p));
    if (const char* e = std::getenv("NNSX_SUBPLUGIN_PATH"))
      for (auto& p : split(e, ':'))
        if (!strip(p).empty()) out.push_back(strip(p));
  }
  std::lock_guard<std::mutex> lk(mu_);
  auto it = ini_.find(sections[k]);
  if (it != ini_.end()) {
    auto jt = it->second.find(keys[k]);
    if (jt != it->second.end())
      for (auto& p : split(jt->second, ':'))
        if (!strip(p).empty()) out.push_back(strip(p));
  }
  return out;
}

std::string Config::custom_value(const std::string& group, const std::string& key, const std::string& def) const {
  if (envvar_enabled()) {
    std::string env = "NNSTREAMER_" + group + "_" + key;
    if (const char* e = std::getenv(env.c_str())) return e;
  }
  std::lock_guard<std::mutex> lk(mu_);
  auto it = ini_.find(group);
  if (it == ini_.end()) return def;
  auto jt = it->second.find(key);
  return jt == it->second.end() ? def : jt->second;
}

bool Config::custom_bool(const std::string& group, const std::string& key, bool def) const {
  std::string v = custom_value(group, key, "");
  return v.empty() ? def : to_bool(v, def);
}

void Config::set_value(const std::string& group, const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> lk(mu_);
  ini_[group][key] = value;
}

std::string Config::dump() const {
  std::string r = "nnsx configuration\n  conf file: " + path() + "\n";
  std::lock_guard<std::mutex> lk(mu_);
  for (const auto& s : ini_) {
    r += "  [" + s.first + "]\n";
    for (const auto& kv : s.second) r += "    " + kv.first + " = " + kv.second + "\n";
  }
  return r;
}

}  // namespace nnsx
