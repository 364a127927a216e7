// Helpers shared by the tensor_* elements: per-element HIP stream, device
// placement, and config <-> caps plumbing.
#pragma once

#include <hip/hip_runtime_api.h>

#include "core/caps.h"
#include "runtime/element.h"
#include "runtime/hip_util.h"

namespace nnsx {

// One non-blocking stream per element instance and device ("per-pad HIP
// streams": consecutive GPU elements overlap through event dependencies).
class StreamSet {
 public:
  ~StreamSet();
  hipStream_t get(int dev);

 private:
  std::mutex mu_;
  std::map<int, hipStream_t> streams_;
};

// device property semantics shared by GPU-capable elements:
//   -2 auto: follow the input memory placement
//   -1 cpu:  force host processing
//   >=0:     force that GPU (inputs are uploaded on demand)
int resolve_device(int prop, const Buffer& in);
int resolve_device(int prop, const MemoryPtr& in);

// Read the static/flexible config of a tensor pad's caps.
bool tensor_config_from_caps(const Caps& caps, TensorsConfig* config);
// Caps of a src pad from config, consulting the peer (flexible wins).
Caps tensor_src_caps(Pad* srcpad, const TensorsConfig& config, bool device = false);
// Does the negotiated caps of this pad say flexible?
bool pad_caps_is_flexible(Pad* pad);

// Allocate an output memory on the element's stream (device) or host.
MemoryPtr alloc_output(size_t size, int dev, hipStream_t s);

}  // namespace nnsx
