// Host (de)serializers of a tensors frame for the wire-format decoders /
// converters and the gRPC elements (optional host path,
// never on the GPU hot loop).
//
//   protobuf : nnstreamer.protobuf.Tensors (ext/nnstreamer/include/nnstreamer.proto)
//   flatbuf  : nnstreamer.flatbuf.Tensors  (ext/nnstreamer/include/nnstreamer.fbs)
//   flexbuf  : schema-less FlexBuffers map {num_tensors, rate_n, rate_d,
//              format, tensor_<i>: [name, type, dims[8], blob]}
//              (tensordec-flexbuf.cc / tensor_converter_flexbuf.cc)
//
// No protobuf / flatbuffers library is linked: the three wire formats are
// written and parsed directly (proto3 canonical field order, defaults
// omitted; FlatBuffers tables with vtables; FlexBuffers with 8-byte slots).
// Readers accept any valid encoding (other builders' layouts and widths).
// For flexible streams the per-tensor 128-byte header travels inside `data`
// and supplies name-less info, as in the reference.
#pragma once

#include <string>
#include <vector>

#include "core/types.h"
#include "runtime/memory.h"

namespace nnsx {
namespace serial {

enum class Wire { PROTOBUF, FLATBUF, FLEXBUF };

const char* wire_name(Wire w);
const char* wire_caps(Wire w);  // other/protobuf-tensor, other/flatbuf-tensor, other/flexbuf

// tensors -> one serialized blob (host memory)
MemoryPtr encode(Wire w, const TensorsConfig& config, const std::vector<MemoryPtr>& tensors);
// serialized blob -> tensors (+ config); false on a malformed buffer
bool decode(Wire w, const void* data, size_t size, TensorsConfig* config, std::vector<MemoryPtr>* tensors);

}  // namespace serial
}  // namespace nnsx
