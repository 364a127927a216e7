// nnsx-check: what this installation provides -- version, GPUs, elements,
// sub-plugins per kind (scanning the sub-plugin paths) and the effective
// configuration.  Reference: tools/development/confchk/confchk.c:20-105
// (nnstreamer-check).  `--json` prints one machine-readable object.
#include <cstdio>
#include <string>
#include <vector>

#include "core/registry.h"
#include "core/types.h"
#include "runtime/hip_util.h"
#include "runtime/pipeline.h"

using namespace nnsx;

namespace {

std::string jstr(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if (static_cast<unsigned char>(c) < 0x20) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o + "\"";
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int nnsx_check_main(int argc, char** argv) {
  bool json = argc > 1 && std::string(argv[1]) == "--json";
  const std::pair<const char*, SubpluginKind> kinds[] = {{"filter", SubpluginKind::FILTER},
                                                         {"decoder", SubpluginKind::DECODER},
                                                         {"converter", SubpluginKind::CONVERTER},
                                                         {"trainer", SubpluginKind::TRAINER}};
  const int ngpu = hip::device_count();
  auto elems = list_elements();
  if (json) {
    std::printf("{\n  \"version\": %s,\n  \"gpus\": [", jstr(version_string()).c_str());
    for (int d = 0; d < ngpu; ++d)
      std::printf("%s{\"index\": %d, \"arch\": %s}", d ? ", " : "", d, jstr(hip::device_arch(d)).c_str());
    std::printf("],\n  \"elements\": [");
    for (size_t i = 0; i < elems.size(); ++i) std::printf("%s%s", i ? ", " : "", jstr(elems[i].name).c_str());
    std::printf("],\n  \"subplugins\": {");
    bool first = true;
    for (auto& k : kinds) {
      auto names = Registry::get().names(k.second, true);
      std::printf("%s%s: [", first ? "" : ", ", jstr(k.first).c_str());
      for (size_t i = 0; i < names.size(); ++i) std::printf("%s%s", i ? ", " : "", jstr(names[i]).c_str());
      std::printf("]");
      first = false;
    }
    std::printf("},\n  \"config\": %s\n}\n", jstr(Config::get().dump()).c_str());
    return 0;
  }
  std::printf("%s\n", version_string());
  std::printf("GPUs: %d\n", ngpu);
  for (int d = 0; d < ngpu; ++d) std::printf("  [%d] %s\n", d, hip::device_arch(d).c_str());
  std::printf("Elements (%zu):\n", elems.size());
  for (auto& e : elems) std::printf("  %-24s %s\n", e.name.c_str(), e.description.c_str());
  for (auto& k : kinds) {
    auto names = Registry::get().names(k.second, true);
    std::printf("%s sub-plugins:", k.first);
    if (names.empty()) std::printf(" (none)");
    for (auto& n : names) std::printf(" %s", n.c_str());
    std::printf("\n");
  }
  std::printf("%s\n", Config::get().dump().c_str());
  return 0;
}
