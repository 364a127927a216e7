// nnsx core data model: tensor element types, dimensions, formats, tensor
// info/config and the 128-byte flexible-tensor meta header.
//
// Behaviour parity targets (reference paths relative to /root/reference):
//   limits          gst/nnstreamer/include/tensor_typedef.h:34-46
//   type enum order gst/nnstreamer/include/tensor_typedef.h:133-148 (ABI: int32=0 .. float16=10)
//   names / sizes   gst/nnstreamer/nnstreamer_plugin_api_util_impl.c:20-51
//   dim parse/print gst/nnstreamer/nnstreamer_plugin_api_util_impl.c:922-1016
//   meta header     gst/nnstreamer/nnstreamer_plugin_api_util_impl.c:1215-1470
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace nnsx {

constexpr int kRankLimit = 8;         // NNS_TENSOR_RANK_LIMIT
constexpr int kRankLimitPrev = 4;     // NNS_TENSOR_RANK_LIMIT_PREV (legacy caps spelling)
constexpr int kSizeLimit = 16;        // tensors per buffer (GstBuffer memory limit)
constexpr int kSizeExtraLimit = 200;  // extra tensors packed in the 16th memory
constexpr int kMetaRankLimit = 16;    // rank inside the flexible meta header
constexpr size_t kMetaHeaderSize = 128;

enum class DType : uint32_t {
  INT32 = 0,
  UINT32,
  INT16,
  UINT16,
  INT8,
  UINT8,
  FLOAT64,
  FLOAT32,
  INT64,
  UINT64,
  FLOAT16,
  END,           // == _NNS_END (11); invalid / unknown
  BFLOAT16 = 12  // nnsx extension (not in the reference); compute dtype on MI355X
};

enum class Format : uint32_t { STATIC = 0, FLEXIBLE, SPARSE, END };

enum class MediaType : int32_t {
  INVALID = -1,
  VIDEO = 0,
  AUDIO = 1,
  TEXT = 2,
  OCTET = 3,
  TENSOR = 4,
  ANY = 0x1000,
};

using Dims = std::array<uint32_t, kRankLimit>;

const char* dtype_name(DType t);           // nullptr for END
size_t dtype_size(DType t);                // 0 for END
DType dtype_from_string(const std::string& s);  // END if unrecognized (case-insensitive)
bool dtype_valid(DType t);
const char* format_name(Format f);
Format format_from_string(const std::string& s);

// "d1:d2:..." innermost first; unspecified trailing dims are 1.  Returns rank
// (number of parsed fields), 0 on error.
unsigned parse_dimension(const std::string& s, Dims& dim);
std::string dimension_string(const Dims& dim);                 // always 8 fields
std::string rank_dimension_string(const Dims& dim, unsigned rank);  // rank fields (0 -> 8)
bool dimension_valid(const Dims& dim);                         // every entry > 0
bool dimension_string_equal(const std::string& a, const std::string& b);
uint64_t element_count(const Dims& dim);
Dims make_dims(std::initializer_list<uint32_t> v);

struct TensorInfo {
  std::string name;
  DType type = DType::END;
  Dims dim{};  // all 0 == unset (gst_tensor_info_init)

  size_t size() const { return dimension_valid(dim) ? element_count(dim) * dtype_size(type) : 0; }
  bool valid() const { return dtype_valid(type) && dimension_valid(dim); }
  int rank() const;  // trailing 1s ignored, minimum 1
  bool operator==(const TensorInfo& o) const;  // type + dims (names ignored, like the reference)
  bool operator!=(const TensorInfo& o) const { return !(*this == o); }
};

struct TensorsInfo {
  unsigned num_tensors = 0;
  Format format = Format::STATIC;
  std::vector<TensorInfo> info;  // size >= num_tensors

  TensorInfo& at(unsigned i);
  const TensorInfo& at(unsigned i) const;
  void resize(unsigned n);
  bool valid() const;
  bool operator==(const TensorsInfo& o) const;
  bool operator!=(const TensorsInfo& o) const { return !(*this == o); }
  size_t size(int index = -1) const;  // -1 = total

  // "d:d:d:d,d:d:d:d" etc.  parse_* return count parsed.
  unsigned parse_dimensions(const std::string& s);
  unsigned parse_types(const std::string& s);
  unsigned parse_names(const std::string& s);
  std::string dimensions_string() const;
  std::string rank_dimensions_string(unsigned rank) const;
  std::string types_string() const;
  std::string names_string() const;
  std::string to_string() const;
};

struct TensorsConfig {
  TensorsInfo info;
  int rate_n = -1;
  int rate_d = -1;

  bool valid() const;
  bool operator==(const TensorsConfig& o) const;
  bool operator!=(const TensorsConfig& o) const { return !(*this == o); }
  std::string to_string() const;
  bool is_flexible() const { return info.format == Format::FLEXIBLE; }
  bool is_sparse() const { return info.format == Format::SPARSE; }
  bool is_static() const { return info.format == Format::STATIC; }
};

// Flexible / sparse per-tensor header (GstTensorMetaInfo, 128 bytes on the wire).
struct MetaInfo {
  uint32_t version = 0;
  uint32_t type = static_cast<uint32_t>(DType::END);
  uint32_t dimension[kMetaRankLimit] = {0};
  uint32_t format = static_cast<uint32_t>(Format::STATIC);
  uint32_t media_type = static_cast<uint32_t>(MediaType::TENSOR);
  uint32_t nnz = 0;  // sparse only

  static constexpr uint32_t make_version(uint32_t major, uint32_t minor) {
    return (major << 12) | minor | 0xDE000000u;
  }
  static constexpr uint32_t kVersion = (1u << 12) | 0u | 0xDE000000u;  // make_version(1, 0)

  MetaInfo() { version = kVersion; }
  static MetaInfo from_info(const TensorInfo& info, Format fmt = Format::FLEXIBLE,
                            MediaType media = MediaType::TENSOR);
  bool valid() const;
  size_t header_size() const;  // 128 for v1, 0 if invalid version
  size_t data_size() const;
  void write(void* header) const;  // writes kMetaHeaderSize bytes
  static bool parse(const void* header, size_t avail, MetaInfo* out);
  bool to_info(TensorInfo* info) const;
};

// Version API (nnstreamer_version_string / fetch)
const char* version_string();
void version_fetch(unsigned* major, unsigned* minor, unsigned* micro);

}  // namespace nnsx
