// Decoder sub-plugins shipped with nnsx.
#pragma once

#include <string>
#include <vector>

#include "runtime/plugin_api.h"

namespace nnsx {

std::vector<std::string> load_labels(const std::string& path);
void set_framerate_from_config(Caps& caps, const TensorsConfig& config);

void register_simple_decoders();     // image_labeling, direct_video, octet_stream
void register_bbox_decoder();        // bounding_boxes
void register_segment_decoder();     // image_segment
void register_pose_decoder();        // pose_estimation
void register_serial_decoders();     // protobuf / flexbuf / flatbuf wire formats

}  // namespace nnsx
