#include "elements/tensor_common.h"

namespace nnsx {

StreamSet::~StreamSet() {
  for (auto& kv : streams_) hip::stream_destroy(kv.first, kv.second);
}

hipStream_t StreamSet::get(int dev) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = streams_.find(dev);
  if (it != streams_.end()) return it->second;
  hipStream_t s = hip::stream_create(dev);
  streams_[dev] = s;
  return s;
}

int resolve_device(int prop, const MemoryPtr& m) {
  if (prop >= 0) return hip::available() ? prop : -1;
  if (prop == -1) return -1;
  return (m && m->on_device()) ? m->device() : -1;
}

int resolve_device(int prop, const Buffer& in) {
  if (prop >= 0) return hip::available() ? prop : -1;
  if (prop == -1) return -1;
  for (auto& m : in.mems)
    if (m->on_device()) return m->device();
  return -1;
}

bool tensor_config_from_caps(const Caps& caps, TensorsConfig* config) {
  if (caps.size() == 0) return false;
  return config_from_structure(caps.at(0), config);
}

Caps tensor_src_caps(Pad* srcpad, const TensorsConfig& config, bool device) {
  Caps peer = srcpad->peer_query_caps(nullptr);
  Caps c = pad_caps_from_config(config, &peer, device);
  Caps i = c.intersect(srcpad->template_caps());
  if (i.is_empty()) return c;
  return c;
}

bool pad_caps_is_flexible(Pad* pad) {
  if (!pad->has_current_caps()) return false;
  TensorsConfig c;
  if (!tensor_config_from_caps(pad->current_caps(), &c)) return false;
  return c.is_flexible();
}

MemoryPtr alloc_output(size_t size, int dev, hipStream_t s) {
  if (dev >= 0) return Memory::alloc_device(size, dev, s);
  return Memory::alloc_host(size);
}

}  // namespace nnsx
