// C entry points of include/nnsx/nnstreamer_custom.h: C callbacks behind the
// C++ custom-code registries (custom-easy filter, converter, decoder,
// tensor_if).  Reference names: NNS_custom_easy_register
// (tensor_filter_custom_easy.c:73-257), nnstreamer_converter_custom_register
// (gsttensor_converter.c:2385-2420), nnstreamer_decoder_custom_register
// (gsttensor_decoder.c:936-974), nnstreamer_if_custom_register
// (gsttensor_if.c:1010-1055).
#include <nnsx/nnstreamer_custom.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "core/log.h"
#include "core/registry.h"
#include "runtime/plugin_api.h"

namespace nnsx {

bool custom_easy_lookup(const std::string& name, CustomEasyFn* fn, TensorsInfo* in, TensorsInfo* out);

namespace {

// the reference refuses a name that is already registered (register_subplugin,
// nnstreamer_subplugin.c:223-276) and the reserved names "any" / "auto"
bool name_taken(SubpluginKind kind, const char* name) {
  const std::string n = name;
  if (n == "any" || n == "auto") return true;
  return Registry::get().find(kind, n, false) != nullptr;
}

void info_to_c(const TensorsInfo& a, NNSX_TensorsInfo* b) {
  std::memset(b, 0, sizeof(*b));
  b->num_tensors = std::min<unsigned>(a.num_tensors, NNSX_SIZE_LIMIT);
  b->format = static_cast<uint32_t>(a.format);
  for (unsigned i = 0; i < b->num_tensors; ++i) {
    b->info[i].type = static_cast<uint32_t>(a.at(i).type);
    for (int d = 0; d < kRankLimit; ++d) b->info[i].dimension[d] = a.at(i).dim[d];
  }
}

// counts come from user code: never index past info[NNSX_SIZE_LIMIT]
bool info_ok(const NNSX_TensorsInfo& b) { return b.num_tensors <= NNSX_SIZE_LIMIT; }

void info_from_c(const NNSX_TensorsInfo& b, TensorsInfo* a) {
  *a = TensorsInfo();
  if (!info_ok(b)) return;
  a->resize(b.num_tensors);
  a->format = static_cast<Format>(b.format);
  for (unsigned i = 0; i < b.num_tensors; ++i) {
    a->at(i).type = static_cast<DType>(b.info[i].type);
    for (int d = 0; d < kRankLimit; ++d) a->at(i).dim[d] = b.info[i].dimension[d] ? b.info[i].dimension[d] : 1;
    if (b.info[i].name) a->at(i).name = b.info[i].name;
  }
}

void config_to_c(const TensorsConfig& a, NNSX_TensorsConfig* b) {
  info_to_c(a.info, &b->info);
  b->rate_n = a.rate_n;
  b->rate_d = a.rate_d;
}

// host views of the inputs (device memories are mapped)
std::vector<NNSX_TensorMemory> host_views(const std::vector<MemoryPtr>& in) {
  std::vector<NNSX_TensorMemory> v(in.size());
  for (size_t i = 0; i < in.size(); ++i) {
    v[i].data = const_cast<void*>(in[i]->map_host());
    v[i].size = in[i]->size();
  }
  return v;
}

// a malloc()ed block handed over by a C callback
MemoryPtr adopt(const NNSX_TensorMemory& m) {
  return Memory::wrap(m.data, m.size, MemPlace::HOST, -1, [](Memory* mm) { std::free(mm->data()); });
}

}  // namespace
}  // namespace nnsx

using namespace nnsx;

extern "C" {

int NNS_custom_easy_register(const char* modelname, NNS_custom_easy_invoke func, void* data,
                             const NNSX_TensorsInfo* in_info, const NNSX_TensorsInfo* out_info) {
  if (!modelname || !func || !in_info || !out_info) return -22;  // -EINVAL
  if (!info_ok(*in_info) || !info_ok(*out_info)) return -22;
  {
    CustomEasyFn f;
    TensorsInfo a, b;
    if (custom_easy_lookup(modelname, &f, &a, &b)) return -17;  // -EEXIST
  }
  TensorsInfo in, out;
  info_from_c(*in_info, &in);
  info_from_c(*out_info, &out);
  auto fn = [func, data](const std::vector<MemoryPtr>& inm, std::vector<MemoryPtr>* outm, const TensorsInfo& ii,
                         const TensorsInfo& oi) -> int {
    NNSX_FilterProperties prop;
    std::memset(&prop, 0, sizeof(prop));
    prop.fwname = "custom-easy";
    info_to_c(ii, &prop.input_meta);
    info_to_c(oi, &prop.output_meta);
    std::vector<NNSX_TensorMemory> iv = host_views(inm);
    std::vector<NNSX_TensorMemory> ov(oi.num_tensors);
    std::vector<MemoryPtr> outs;
    for (unsigned i = 0; i < oi.num_tensors; ++i) {
      outs.push_back(Memory::alloc_host(oi.size(static_cast<int>(i))));
      ov[i].data = outs.back()->data();
      ov[i].size = outs.back()->size();
    }
    const int r = func(data, &prop, iv.data(), ov.data());
    if (r == 0) *outm = std::move(outs);
    return r;
  };
  return custom_easy_register(modelname, fn, in, out) ? 0 : -17;  // -EEXIST
}

int NNS_custom_easy_unregister(const char* modelname) {
  return modelname && custom_easy_unregister(modelname) ? 0 : -22;
}

int nnstreamer_converter_custom_register(const char* name, tensor_converter_custom func, void* data) {
  if (!name || !func) return -22;
  if (name_taken(SubpluginKind::CUSTOM_CONVERTER, name)) return -17;
  auto fn = [func, data](const BufferPtr& in, TensorsConfig* config) -> BufferPtr {
    // the raw input as one contiguous host block
    std::vector<char> bytes;
    for (auto& m : in->mems) {
      const char* p = static_cast<const char*>(m->map_host());
      bytes.insert(bytes.end(), p, p + m->size());
    }
    NNSX_TensorsConfig c;
    std::memset(&c, 0, sizeof(c));
    NNSX_TensorMemory out[NNSX_SIZE_LIMIT];
    std::memset(out, 0, sizeof(out));
    if (func(bytes.data(), bytes.size(), data, &c, out) != 0) return nullptr;
    if (!info_ok(c.info)) {
      NNSX_LOGE("c_api", "custom converter returned num_tensors=%u (limit %d)", c.info.num_tensors, NNSX_SIZE_LIMIT);
      return nullptr;
    }
    info_from_c(c.info, &config->info);
    config->rate_n = c.rate_n;
    config->rate_d = c.rate_d;
    auto b = make_buffer();
    for (unsigned i = 0; i < c.info.num_tensors && i < NNSX_SIZE_LIMIT; ++i) b->mems.push_back(adopt(out[i]));
    return b;
  };
  return converter_custom_register(name, fn) ? 0 : -17;
}

int nnstreamer_converter_custom_unregister(const char* name) {
  return name && converter_custom_unregister(name) ? 0 : -22;
}

int nnstreamer_decoder_custom_register(const char* name, tensor_decoder_custom func, void* data) {
  if (!name || !func) return -22;
  if (name_taken(SubpluginKind::CUSTOM_DECODER, name)) return -17;
  auto fn = [func, data](const std::vector<MemoryPtr>& in, const TensorsConfig& config, Buffer* out) -> FlowReturn {
    NNSX_TensorsConfig c;
    config_to_c(config, &c);
    std::vector<NNSX_TensorMemory> iv = host_views(in);
    NNSX_TensorMemory o{nullptr, 0};
    if (func(iv.data(), &c, data, &o) != 0 || !o.data) return FlowReturn::ERROR;
    out->mems.push_back(adopt(o));
    return FlowReturn::OK;
  };
  return decoder_custom_register(name, fn) ? 0 : -17;
}

int nnstreamer_decoder_custom_unregister(const char* name) {
  return name && decoder_custom_unregister(name) ? 0 : -22;
}

int nnstreamer_if_custom_register(const char* name, tensor_if_custom func, void* data) {
  if (!name || !func) return -22;
  if (name_taken(SubpluginKind::CUSTOM_IF, name)) return -17;
  auto fn = [func, data](const TensorsInfo& info, const std::vector<MemoryPtr>& in) -> bool {
    NNSX_TensorsInfo ci;
    info_to_c(info, &ci);
    std::vector<NNSX_TensorMemory> iv = host_views(in);
    int result = 0;
    if (func(&ci, iv.data(), data, &result) != 0) {
      NNSX_LOGW("tensor_if", "custom condition callback failed: treated as false");
      return false;
    }
    return result != 0;
  };
  return if_custom_register(name, fn) ? 0 : -17;
}

int nnstreamer_if_custom_unregister(const char* name) { return name && if_custom_unregister(name) ? 0 : -22; }

}  // extern "C"
