// gst-launch pipeline <-> MediaPipe-style pbtxt (tools/development/parser).
#pragma once

#include <string>

#include "runtime/pipeline.h"

namespace nnsx {

// with_options: add node_options with the properties that differ from the
// factory defaults (and the caps filter feeding the node), enough for
// pbtxt_to_launch() to rebuild the pipeline.
std::string pipeline_to_pbtxt(const Pipeline& pipeline, bool with_options = false);
// "" + *err on a malformed graph
std::string pbtxt_to_launch(const std::string& pbtxt, std::string* err);

}  // namespace nnsx
