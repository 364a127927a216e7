// Filter framework registration and the C++ custom-filter class API
// (framework=cpp; nnstreamer_cppplugin_api_filter.hh / tensor_filter_cpp.hh).
#pragma once

#include <functional>
#include <memory>
#include <string>

#include "runtime/plugin_api.h"

namespace nnsx {

class CppFilter {
 public:
  virtual ~CppFilter() = default;
  virtual bool get_model_info(TensorsInfo* in, TensorsInfo* out) = 0;
  virtual bool set_input_info(const TensorsInfo& in, TensorsInfo* out) {
    (void)in;
    (void)out;
    return false;
  }
  virtual int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext& ctx) = 0;
};
using CppFilterFactory = std::function<std::unique_ptr<CppFilter>(const FilterProperties&)>;
bool register_cpp_filter(const std::string& name, CppFilterFactory f);
bool unregister_cpp_filter(const std::string& name);

void register_host_frameworks();   // custom, custom-easy, cpp
void register_lua_framework();     // lua (built-in Lua 5.1 subset, filter/lua_vm.h)
void register_torch_frameworks();  // pytorch (libtorch, ROCm) -- torch TU
void register_torch_trainer();     // tensor_trainer framework=pytorch -- torch TU

}  // namespace nnsx
