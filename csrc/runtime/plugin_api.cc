#include "runtime/plugin_api.h"

#include <cstdlib>
#include <regex>

#include "core/log.h"
#include "core/util.h"
#include "runtime/hip_util.h"

namespace nnsx {

bool register_filter_framework(std::shared_ptr<FilterFramework> fw) {
  std::string n = fw->name();
  return Registry::get().add(SubpluginKind::FILTER, n, std::static_pointer_cast<void>(fw));
}

std::shared_ptr<FilterFramework> find_filter_framework(const std::string& name) {
  // [filter-aliases] section maps alias -> framework name
  std::string real = Config::get().custom_value("filter-aliases", name, name);
  return Registry::get().find_as<FilterFramework>(SubpluginKind::FILTER, real);
}

std::string detect_framework(const std::vector<std::string>& models) {
  if (models.empty()) return "";
  const std::string& m = models[0];
  auto dot = m.rfind('.');
  std::string ext = dot == std::string::npos ? "" : lower(m.substr(dot + 1));
  if (m.size() > 3 && ends_with(m, ".so")) ext = "so";
  // ini priority: [filter] framework_priority_<ext> = a,b,c
  std::string prio = Config::get().custom_value("filter", "framework_priority_" + ext, "");
  for (auto& cand : split(prio, ',')) {
    std::string c = strip(cand);
    if (!c.empty() && find_filter_framework(c)) return c;
  }
  for (const auto& n : Registry::get().names(SubpluginKind::FILTER)) {
    auto fw = find_filter_framework(n);
    if (!fw) continue;
    for (const auto& e : fw->model_extensions())
      if (lower(e) == ext || lower(e) == "." + ext) return n;
  }
  return "";
}

Accelerator parse_accelerator(const std::string& s, const std::string& supported, bool* use_accel) {
  // grammar: (true|false)[:accl(,accl)*] with `!accl` to exclude
  std::string t = lower(strip(s));
  *use_accel = false;
  if (t.empty()) return Accelerator::DEFAULT;
  auto parts = split(t, ':', 2);
  *use_accel = to_bool(parts[0], false);
  if (!*use_accel) return Accelerator::CPU;
  if (parts.size() < 2) return Accelerator::AUTO;
  std::vector<std::string> sup = split(lower(supported), ',');
  for (auto& a : split(parts[1], ',')) {
    std::string x = strip(a);
    if (x.empty() || x[0] == '!') continue;
    bool ok = supported.empty();
    for (auto& ss : sup)
      if (strip(ss) == x) ok = true;
    if (!ok) continue;
    if (x == "gpu") return Accelerator::GPU;
    if (x == "cpu") return Accelerator::CPU;
    if (x == "auto") return Accelerator::AUTO;
    if (x == "default") return Accelerator::DEFAULT;
  }
  return Accelerator::AUTO;
}

std::shared_ptr<FilterFramework> resolve_filter_framework(const std::string& fw_name, FilterProperties* props,
                                                          int device_prop, std::string* err) {
  std::string fwn = fw_name;
  if (fwn.empty() || fwn == "auto") {
    fwn = detect_framework(props->model_files);
    if (fwn.empty()) {
      *err = "cannot detect the framework for the model";
      return nullptr;
    }
  }
  auto fw = find_filter_framework(fwn);
  if (!fw) {
    *err = "framework '" + fwn + "' is not available";
    return nullptr;
  }
  props->fwname = fw->name();
  if (props->model_files.empty() && !fw->run_without_model()) {
    *err = "model property is not set";
    return nullptr;
  }
  bool use_accl = false;
  props->accl = parse_accelerator(props->accl_str, fw->accelerators(), &use_accl);
  props->device = -1;
  if ((props->accl == Accelerator::GPU || props->accl == Accelerator::AUTO ||
       (props->accl == Accelerator::DEFAULT && fw->accelerators().find("gpu") != std::string::npos &&
        Config::get().custom_bool("pytorch", "enable_use_gpu", true))) &&
      fw->check_availability(Accelerator::GPU) && hip::available()) {
    int dev = device_prop;
    if (dev < 0) {
      const char* lr = getenv("LOCAL_RANK");
      dev = lr ? static_cast<int>(to_int(lr)) % hip::device_count() : 0;
    }
    props->device = dev;
  }
  return fw;
}

// ------------------------------------------------------------ custom-easy ----
namespace {
struct CustomEasyEntry {
  CustomEasyFn fn;
  TensorsInfo in, out;
};
}  // namespace

bool custom_easy_register(const std::string& name, CustomEasyFn fn, const TensorsInfo& in, const TensorsInfo& out) {
  auto e = std::make_shared<CustomEasyEntry>(CustomEasyEntry{std::move(fn), in, out});
  // custom-easy entries live in the custom table under a "custom-easy:" prefix
  return Registry::get().add(SubpluginKind::CUSTOM_IF, "custom-easy:" + name, std::static_pointer_cast<void>(e));
}

bool custom_easy_unregister(const std::string& name) {
  return Registry::get().remove(SubpluginKind::CUSTOM_IF, "custom-easy:" + name);
}

// used by filter/custom_easy.cc
bool custom_easy_lookup(const std::string& name, CustomEasyFn* fn, TensorsInfo* in, TensorsInfo* out) {
  auto e = Registry::get().find_as<CustomEasyEntry>(SubpluginKind::CUSTOM_IF, "custom-easy:" + name, false);
  if (!e) return false;
  *fn = e->fn;
  *in = e->in;
  *out = e->out;
  return true;
}

// --------------------------------------------------------------- decoders ----
bool register_decoder(std::shared_ptr<DecoderSubplugin> d) {
  std::string n = d->name();
  return Registry::get().add(SubpluginKind::DECODER, n, std::static_pointer_cast<void>(d));
}

std::shared_ptr<DecoderSubplugin> find_decoder(const std::string& mode) {
  return Registry::get().find_as<DecoderSubplugin>(SubpluginKind::DECODER, mode);
}

bool decoder_custom_register(const std::string& name, DecoderCustomFn fn) {
  return Registry::get().add(SubpluginKind::CUSTOM_DECODER, name, std::make_shared<DecoderCustomFn>(std::move(fn)));
}

bool decoder_custom_unregister(const std::string& name) {
  return Registry::get().remove(SubpluginKind::CUSTOM_DECODER, name);
}

// ------------------------------------------------------------- converters ----
bool register_converter(std::shared_ptr<ConverterSubplugin> c) {
  std::string n = c->name();
  return Registry::get().add(SubpluginKind::CONVERTER, n, std::static_pointer_cast<void>(c));
}

std::shared_ptr<ConverterSubplugin> find_converter(const std::string& name) {
  return Registry::get().find_as<ConverterSubplugin>(SubpluginKind::CONVERTER, name);
}

std::shared_ptr<ConverterSubplugin> find_converter_for_caps(const Caps& caps) {
  // NNS_SEARCH_GETALL: every converter library is loaded up-front
  for (const auto& n : Registry::get().names(SubpluginKind::CONVERTER, true)) {
    auto c = find_converter(n);
    if (c && c->query_caps().can_intersect(caps)) return c;
  }
  return nullptr;
}

bool converter_custom_register(const std::string& name, ConverterCustomFn fn) {
  return Registry::get().add(SubpluginKind::CUSTOM_CONVERTER, name, std::make_shared<ConverterCustomFn>(std::move(fn)));
}

bool converter_custom_unregister(const std::string& name) {
  return Registry::get().remove(SubpluginKind::CUSTOM_CONVERTER, name);
}

namespace {
ScriptConverterFactory& script_factory() {
  static ScriptConverterFactory* f = new ScriptConverterFactory();
  return *f;
}
}  // namespace

void set_script_converter_factory(ScriptConverterFactory f) { script_factory() = std::move(f); }

std::shared_ptr<ConverterSubplugin> make_script_converter(const std::string& path) {
  if (!script_factory()) {
    NNSX_LOGE("converter", "custom-script converters need the Python bridge (import nnstreamer_amd)");
    return nullptr;
  }
  return script_factory()(path);
}

bool if_custom_register(const std::string& name, IfCustomFn fn) {
  return Registry::get().add(SubpluginKind::CUSTOM_IF, name, std::make_shared<IfCustomFn>(std::move(fn)));
}

bool if_custom_unregister(const std::string& name) { return Registry::get().remove(SubpluginKind::CUSTOM_IF, name); }

IfCustomFn find_if_custom(const std::string& name) {
  auto f = Registry::get().find_as<IfCustomFn>(SubpluginKind::CUSTOM_IF, name, false);
  return f ? *f : IfCustomFn();
}

// --------------------------------------------------------------- trainers ----
bool register_trainer(std::shared_ptr<TrainerFramework> t) {
  std::string n = t->name();
  return Registry::get().add(SubpluginKind::TRAINER, n, std::static_pointer_cast<void>(t));
}

std::shared_ptr<TrainerFramework> find_trainer(const std::string& name) {
  return Registry::get().find_as<TrainerFramework>(SubpluginKind::TRAINER, name);
}

}  // namespace nnsx
