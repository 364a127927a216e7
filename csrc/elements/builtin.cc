// Registration of every built-in element, decoder and framework
// (gst/nnstreamer/registerer/nnstreamer.c:91-122 equivalent).
#include <mutex>

#include "decoders/decoders.h"
#include "elements/elements.h"
#include "filter/filter.h"
#include "runtime/pipeline.h"

namespace nnsx {

void register_tensor_converter();
void register_tensor_transform();
void register_tensor_sink();
void register_tensor_decoder();
void register_tensor_filter();
void register_tensor_stream_elements();  // mux/demux/merge/split/aggregator
void register_extra_elements();

void ensure_builtin_elements() {
  static std::once_flag once;
  std::call_once(once, [] {
    register_basic_elements();
    register_tensor_converter();
    register_tensor_transform();
    register_tensor_sink();
    register_tensor_decoder();
    register_tensor_filter();
    register_tensor_stream_elements();
    register_extra_elements();
    register_comm_elements();
    register_mqtt_elements();
    register_fault_inject();
    register_grpc_elements();
    register_host_frameworks();
    register_lua_framework();
    register_torch_frameworks();
    register_torch_trainer();
    register_simple_decoders();
    register_bbox_decoder();
    register_segment_decoder();
    register_pose_decoder();
    register_serial_decoders();
  });
}

}  // namespace nnsx
