// dtype/shape conversions between the nnsx tensor model and ATen, shared by
// the libtorch filter and trainer translation units.
#pragma once

#include <ATen/ATen.h>

#include "core/types.h"
#include "core/util.h"

namespace nnsx {

inline at::ScalarType to_torch(DType t) {
  switch (t) {
    case DType::INT32: return at::kInt;
    case DType::UINT32: return at::kUInt32;
    case DType::INT16: return at::kShort;
    case DType::UINT16: return at::kUInt16;
    case DType::INT8: return at::kChar;
    case DType::UINT8: return at::kByte;
    case DType::FLOAT64: return at::kDouble;
    case DType::FLOAT32: return at::kFloat;
    case DType::INT64: return at::kLong;
    case DType::UINT64: return at::kUInt64;
    case DType::FLOAT16: return at::kHalf;
    case DType::BFLOAT16: return at::kBFloat16;
    default: throw Error("pytorch: unsupported tensor type");
  }
}

inline DType from_torch(at::ScalarType t) {
  switch (t) {
    case at::kInt: return DType::INT32;
    case at::kUInt32: return DType::UINT32;
    case at::kShort: return DType::INT16;
    case at::kUInt16: return DType::UINT16;
    case at::kChar: return DType::INT8;
    case at::kByte: return DType::UINT8;
    case at::kBool: return DType::UINT8;
    case at::kDouble: return DType::FLOAT64;
    case at::kFloat: return DType::FLOAT32;
    case at::kLong: return DType::INT64;
    case at::kUInt64: return DType::UINT64;
    case at::kHalf: return DType::FLOAT16;
    case at::kBFloat16: return DType::BFLOAT16;
    default: return DType::END;
  }
}

// nnsx dims are innermost-first; torch sizes are outermost-first
inline std::vector<int64_t> torch_shape(const TensorInfo& ti, int rank) {
  std::vector<int64_t> s;
  for (int i = rank - 1; i >= 0; --i) s.push_back(ti.dim[i]);
  return s;
}

}  // namespace nnsx
