// tensor_filter framework=lua: the model is a Lua script (a file path, or the
// script text itself when no such file exists) that declares
//
//   inputTensorsInfo  = { num = N, type = {'uint8', ...}, dim = {{d0, d1, ...}, ...} }
//   outputTensorsInfo = { ... }
//   function nnstreamer_invoke() ... end
//
// and reads / writes tensors through input_tensor(i) / output_tensor(i)
// (1-based tensor index; 1-based element index; values are numbers).
// Behaviour follows ext/nnstreamer/tensor_filter/tensor_filter_lua.cc:
//   script vs file mode, model files joined with ","      :439-475
//   TensorsInfo parsing, missing trailing dims = 1        :366-435
//   input_tensor / output_tensor index range 1..16        :255-290
//   element get / set, bounds check, type conversion      :110-240
//   nnstreamer_invoke called per frame                    :495-512
// Differences, on purpose: a FLOAT64 element store writes the double (the
// reference stores `(uint8_t) value` there, :230); integer stores wrap modulo
// the type width instead of relying on an out-of-range C cast; input tensors
// are read-only (they can be shared with other branches of a tee); a tensor
// handle kept past its invoke raises an error instead of dangling.
//
// The interpreter is the built-in Lua 5.1 subset in filter/lua_vm.{h,cc}: the
// image ships no liblua.
#include <sys/stat.h>

#include <cmath>
#include <cstring>
#include <mutex>

#include "core/cpu_ops.h"
#include "core/log.h"
#include "filter/filter.h"
#include "filter/lua_vm.h"
#include "runtime/plugin_api.h"

namespace nnsx {
namespace {

using lua::LuaError;
using lua::Value;
using cpu::bf16_to_float;
using cpu::float_to_bf16;
using cpu::float_to_half;
using cpu::half_to_float;

// one tensor seen from the script; `live` is cleared when the invoke ends
struct TensorUD : lua::Userdata {
  uint8_t* data = nullptr;
  DType type = DType::END;
  size_t count = 0;
  bool writable = false;
  bool live = true;
  std::string what;

  size_t slot(const Value& k) const {
    if (!live) throw LuaError(what + " was used after nnstreamer_invoke() returned");
    double d;
    if (!lua::tonumber(k, &d) || d != std::floor(d)) throw LuaError("Invalid index for tensor");
    if (d < 1 || d > static_cast<double>(count)) throw LuaError("Invalid index for tensor");
    return static_cast<size_t>(d) - 1;
  }

  Value index(const Value& k) override {
    const size_t i = slot(k);
    const uint8_t* p = data + i * dtype_size(type);
    double v = 0;
    switch (type) {
      case DType::INT8: v = *reinterpret_cast<const int8_t*>(p); break;
      case DType::UINT8: v = *p; break;
      case DType::INT16: v = *reinterpret_cast<const int16_t*>(p); break;
      case DType::UINT16: v = *reinterpret_cast<const uint16_t*>(p); break;
      case DType::INT32: v = *reinterpret_cast<const int32_t*>(p); break;
      case DType::UINT32: v = *reinterpret_cast<const uint32_t*>(p); break;
      case DType::INT64: v = static_cast<double>(*reinterpret_cast<const int64_t*>(p)); break;
      case DType::UINT64: v = static_cast<double>(*reinterpret_cast<const uint64_t*>(p)); break;
      case DType::FLOAT32: v = *reinterpret_cast<const float*>(p); break;
      case DType::FLOAT64: v = *reinterpret_cast<const double*>(p); break;
      case DType::FLOAT16: v = half_to_float(*reinterpret_cast<const uint16_t*>(p)); break;
      case DType::BFLOAT16: v = bf16_to_float(*reinterpret_cast<const uint16_t*>(p)); break;
      default: throw LuaError("Error occurred during get tensor value");
    }
    return Value::number(v);
  }

  template <typename T>
  static void store_int(uint8_t* p, double v) {
    // truncate toward zero, then wrap modulo 2^bits
    const double t = std::trunc(v);
    uint64_t u;
    if (!std::isfinite(t))
      u = 0;
    else if (t >= 0)
      u = t < 18446744073709551616.0 ? static_cast<uint64_t>(t) : 0;
    else
      u = t > -9223372036854775808.0 ? static_cast<uint64_t>(static_cast<int64_t>(t)) : 0;
    const T x = static_cast<T>(u);
    std::memcpy(p, &x, sizeof(T));
  }

  void newindex(const Value& k, const Value& val) override {
    const size_t i = slot(k);
    if (!writable) throw LuaError(what + " is read-only");
    double v;
    if (!lua::tonumber(val, &v)) throw LuaError("Error occurred during set tensor value: number expected, got " + val.type_name());
    uint8_t* p = data + i * dtype_size(type);
    switch (type) {
      case DType::INT8: store_int<int8_t>(p, v); break;
      case DType::UINT8: store_int<uint8_t>(p, v); break;
      case DType::INT16: store_int<int16_t>(p, v); break;
      case DType::UINT16: store_int<uint16_t>(p, v); break;
      case DType::INT32: store_int<int32_t>(p, v); break;
      case DType::UINT32: store_int<uint32_t>(p, v); break;
      case DType::INT64: store_int<int64_t>(p, v); break;
      case DType::UINT64: store_int<uint64_t>(p, v); break;
      case DType::FLOAT32: *reinterpret_cast<float*>(p) = static_cast<float>(v); break;
      case DType::FLOAT64: *reinterpret_cast<double*>(p) = v; break;
      case DType::FLOAT16: *reinterpret_cast<uint16_t*>(p) = float_to_half(static_cast<float>(v)); break;
      case DType::BFLOAT16: *reinterpret_cast<uint16_t*>(p) = float_to_bf16(static_cast<float>(v)); break;
      default: throw LuaError("Error occurred during set tensor value");
    }
  }

  size_t length() const override { return live ? count : 0; }
  std::string type_name() const override { return "tensor"; }
};

// tensor_filter_lua.cc:366-435
TensorsInfo parse_tensors_info(const lua::VM& vm, const char* global) {
  const Value g = vm.global(global);
  if (g.t != Value::TABLE)
    throw Error(std::string("Failed to parse global variable `") + global + "`. Please check the script");
  const lua::Table* t = g.tab();
  double num;
  if (!lua::tonumber(t->get(Value::string("num")), &num) || num != std::floor(num))
    throw Error("Failed to parse `num`. Please check the script");
  if (num <= 0 || num > kSizeLimit)
    throw Error("The number of tensors required by the given model exceeds the nnstreamer tensor limit (" +
                std::to_string(kSizeLimit) + " by default).");
  TensorsInfo info;
  info.resize(static_cast<unsigned>(num));
  const Value types = t->get(Value::string("type"));
  if (types.t != Value::TABLE) throw Error("Failed to parse `type`. Please check the script");
  const Value dims = t->get(Value::string("dim"));
  if (dims.t != Value::TABLE) throw Error("Failed to parse `dim`. Please check the script");
  for (unsigned j = 0; j < info.num_tensors; ++j) {
    const Value ty = types.tab()->get(Value::number(j + 1));
    const DType dt = ty.t == Value::STR ? dtype_from_string(ty.str()) : DType::END;
    if (dt == DType::END) throw Error("Failed to parse `type`. Possible types are int32, uint32, int16, uint16, int8, uint8, float64, float32, int64, uint64, float16");
    info.at(j).type = dt;
    const Value d = dims.tab()->get(Value::number(j + 1));
    if (d.t != Value::TABLE) throw Error("Failed to parse `dim`. Please check the script");
    const size_t len = d.tab()->length();
    if (len > static_cast<size_t>(kRankLimit)) throw Error("Failed to parse `dim`: rank above " + std::to_string(kRankLimit));
    for (int r = 0; r < kRankLimit; ++r) {
      double v = 1;
      if (static_cast<size_t>(r) < len) {
        if (!lua::tonumber(d.tab()->get(Value::number(r + 1)), &v) || v != std::floor(v) || v < 1 || v > 4294967295.0)
          throw Error("Failed to parse `dim`. Please check the script");
      }
      info.at(j).dim[r] = static_cast<uint32_t>(v);
    }
  }
  return info;
}

bool file_exists(const std::string& p) {
  struct stat st;
  return !p.empty() && ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

class LuaInstance : public FilterInstance {
 public:
  explicit LuaInstance(FilterProperties& p) { load(p); }

  bool get_model_info(TensorsInfo* in, TensorsInfo* out) override {
    std::lock_guard<std::mutex> lk(mu_);
    *in = in_;
    *out = out_;
    return true;
  }

  int invoke(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, InvokeContext&) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (in.size() < in_.num_tensors) {
      NNSX_LOGE("lua", "%zu input tensors for a script that declares %u", in.size(), in_.num_tensors);
      return -1;
    }
    std::vector<MemoryPtr> outs;
    for (unsigned i = 0; i < out_.num_tensors; ++i) {
      auto m = Memory::alloc_host(out_.size(static_cast<int>(i)));
      std::memset(m->data(), 0, m->size());
      outs.push_back(m);
    }
    std::vector<std::shared_ptr<TensorUD>> uds;
    auto make = [&](bool input, unsigned i) {
      auto u = std::make_shared<TensorUD>();
      const TensorInfo& ti = input ? in_.at(i) : out_.at(i);
      u->type = ti.type;
      u->count = element_count(ti.dim);
      if (input) {
        u->data = static_cast<uint8_t*>(const_cast<void*>(in[i]->map_host()));
        const size_t need = u->count * dtype_size(ti.type);
        if (in[i]->size() < need) throw LuaError("input tensor " + std::to_string(i + 1) + " is smaller than declared");
      } else {
        u->data = static_cast<uint8_t*>(outs[i]->data());
      }
      u->writable = !input;
      u->what = std::string(input ? "input_tensor(" : "output_tensor(") + std::to_string(i + 1) + ")";
      uds.push_back(u);
      return Value::userdata(u);
    };
    auto accessor = [&](bool input) {
      return Value::native(input ? "input_tensor" : "output_tensor", [&, input](std::vector<Value>& a) {
        double d = 0;
        const unsigned n = input ? in_.num_tensors : out_.num_tensors;
        if (a.empty() || !lua::tonumber(a[0], &d) || d != std::floor(d) || d <= 0 || d > kSizeLimit)
          throw LuaError(std::string("Invalid idx for `") + (input ? "input" : "output") + "_tensor(idx)`");
        if (d > n)
          throw LuaError(std::string(input ? "input" : "output") + "_tensor(" + lua::fmt_number(d) +
                         "): the script declares " + std::to_string(n) + " tensors");
        return std::vector<Value>{make(input, static_cast<unsigned>(d) - 1)};
      });
    };
    vm_->set_global("input_tensor", accessor(true));
    vm_->set_global("output_tensor", accessor(false));
    int rc = 0;
    try {
      const Value fn = vm_->global("nnstreamer_invoke");
      if (fn.t != Value::FUNC) throw LuaError("Error while loading function `nnstreamer_invoke` in lua script");
      vm_->call(fn, {});
    } catch (const std::exception& e) {
      NNSX_LOGE("lua", "error while calling nnstreamer_invoke: %s", e.what());
      rc = -1;
    }
    for (auto& u : uds) u->live = false;
    // the accessors capture this frame's locals: replace them until the next invoke
    vm_->set_global("input_tensor", Value());
    vm_->set_global("output_tensor", Value());
    if (rc == 0) *out = std::move(outs);
    return rc;
  }

  bool reload_model(const FilterProperties& p) override {
    try {
      FilterProperties q = p;
      load(q);
      return true;
    } catch (const std::exception& e) {
      NNSX_LOGE("lua", "reload failed: %s", e.what());
      return false;
    }
  }

 private:
  void load(FilterProperties& p) {
    if (p.model_files.empty()) throw Error("lua: no model (a script file or the script text)");
    // tensor_filter_lua.cc:439-475: a path that exists is a file, otherwise
    // the property was the script itself, which tensor_filter split at ','
    std::string src, chunk;
    if (p.model_files.size() == 1 && file_exists(p.model_files[0])) {
      FILE* f = std::fopen(p.model_files[0].c_str(), "rb");
      if (!f) throw Error("lua: cannot open " + p.model_files[0]);
      char buf[65536];
      size_t n;
      while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) src.append(buf, n);
      std::fclose(f);
      chunk = p.model_files[0];
    } else {
      for (size_t i = 0; i < p.model_files.size(); ++i) src += (i ? "," : "") + p.model_files[i];
      chunk = "[script]";
    }
    auto vm = std::make_unique<lua::VM>();
    vm->set_step_limit(step_limit(p.custom_properties));
    try {
      vm->run(src, chunk);
    } catch (const LuaError& e) {
      throw Error(std::string(file_exists(chunk) ? "Failed to run given Lua script file. Error message: "
                                                  : "Failed to run given Lua script. Error message: ") +
                  e.what());
    }
    TensorsInfo in = parse_tensors_info(*vm, "inputTensorsInfo");
    TensorsInfo out = parse_tensors_info(*vm, "outputTensorsInfo");
    if (vm->global("nnstreamer_invoke").t != Value::FUNC)
      throw Error("Error while loading function `nnstreamer_invoke` in lua script");
    std::lock_guard<std::mutex> lk(mu_);
    vm_ = std::move(vm);
    in_ = in;
    out_ = out;
  }

  // custom=max_steps:N caps the statements one invoke may execute (0 = no cap)
  static uint64_t step_limit(const std::string& custom) {
    const std::string key = "max_steps:";
    const size_t at = custom.find(key);
    if (at == std::string::npos) return 0;
    return std::strtoull(custom.c_str() + at + key.size(), nullptr, 10);
  }

  std::mutex mu_;
  std::unique_ptr<lua::VM> vm_;
  TensorsInfo in_, out_;
};

class LuaFw : public FilterFramework {
 public:
  std::string name() const override { return "lua"; }
  std::unique_ptr<FilterInstance> open(FilterProperties& p) override { return std::make_unique<LuaInstance>(p); }
  std::vector<std::string> model_extensions() const override { return {".lua"}; }
  bool verify_model_path() const override { return false; }  // the model may be the script text
  bool allocate_in_invoke() const override { return false; }
};

}  // namespace

void register_lua_framework() { register_filter_framework(std::make_shared<LuaFw>()); }

}  // namespace nnsx
