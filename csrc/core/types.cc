#include "core/types.h"

#include <cstring>

#include "core/util.h"

namespace nnsx {

namespace {
const char* kTypeNames[] = {"int32", "uint32", "int16",   "uint16", "int8",   "uint8",
                            "float64", "float32", "int64", "uint64", "float16"};
const size_t kTypeSizes[] = {4, 4, 2, 2, 1, 1, 8, 4, 8, 8, 2};
const char* kFormatNames[] = {"static", "flexible", "sparse"};
}  // namespace

bool dtype_valid(DType t) { return static_cast<uint32_t>(t) < static_cast<uint32_t>(DType::END) || t == DType::BFLOAT16; }

const char* dtype_name(DType t) {
  if (t == DType::BFLOAT16) return "bfloat16";
  auto i = static_cast<uint32_t>(t);
  return i < static_cast<uint32_t>(DType::END) ? kTypeNames[i] : nullptr;
}

size_t dtype_size(DType t) {
  if (t == DType::BFLOAT16) return 2;
  auto i = static_cast<uint32_t>(t);
  return i < static_cast<uint32_t>(DType::END) ? kTypeSizes[i] : 0;
}

DType dtype_from_string(const std::string& s) {
  std::string t = lower(strip(s));
  if (t.empty()) return DType::END;
  auto num = [&](size_t off) -> int {
    std::string d = t.substr(off);
    if (d.empty()) return -1;
    for (char c : d)
      if (c < '0' || c > '9') return -1;
    return static_cast<int>(to_int(d));
  };
  if (starts_with(t, "uint")) {
    switch (num(4)) {
      case 8: return DType::UINT8;
      case 16: return DType::UINT16;
      case 32: return DType::UINT32;
      case 64: return DType::UINT64;
    }
  } else if (starts_with(t, "int")) {
    switch (num(3)) {
      case 8: return DType::INT8;
      case 16: return DType::INT16;
      case 32: return DType::INT32;
      case 64: return DType::INT64;
    }
  } else if (starts_with(t, "float")) {
    switch (num(5)) {
      case 16: return DType::FLOAT16;
      case 32: return DType::FLOAT32;
      case 64: return DType::FLOAT64;
    }
  } else if (t == "bfloat16" || t == "bf16") {
    return DType::BFLOAT16;
  }
  return DType::END;
}

const char* format_name(Format f) {
  auto i = static_cast<uint32_t>(f);
  return i < 3 ? kFormatNames[i] : nullptr;
}

Format format_from_string(const std::string& s) {
  std::string t = strip(s);
  for (uint32_t i = 0; i < 3; ++i)
    if (t == kFormatNames[i]) return static_cast<Format>(i);
  return Format::END;
}

unsigned parse_dimension(const std::string& s, Dims& dim) {
  std::string t = strip(s);
  auto parts = split(t, ':', kRankLimit);
  unsigned rank = 0;
  size_t i = 0;
  for (; i < parts.size(); ++i) {
    std::string p = strip(parts[i]);
    if (p.empty()) break;
    dim[i] = static_cast<uint32_t>(to_uint(p, 0));
    rank = static_cast<unsigned>(i + 1);
  }
  for (; i < static_cast<size_t>(kRankLimit); ++i) dim[i] = 1;
  return rank;
}

std::string dimension_string(const Dims& dim) { return rank_dimension_string(dim, kRankLimit); }

std::string rank_dimension_string(const Dims& dim, unsigned rank) {
  unsigned r = (rank == 0 || rank > static_cast<unsigned>(kRankLimit)) ? kRankLimit : rank;
  std::string out;
  for (unsigned i = 0; i < r; ++i) {
    if (i) out += ':';
    out += std::to_string(dim[i]);
  }
  return out;
}

bool dimension_valid(const Dims& dim) {
  for (auto d : dim)
    if (d == 0) return false;
  return true;
}

bool dimension_string_equal(const std::string& a, const std::string& b) {
  auto sa = split_any(a, ",.");
  auto sb = split_any(b, ",.");
  if (sa.size() != sb.size()) return false;
  for (size_t i = 0; i < sa.size(); ++i) {
    Dims d1{}, d2{};
    if (!parse_dimension(sa[i], d1) || !parse_dimension(sb[i], d2)) return false;
    if (d1 != d2) return false;
  }
  return true;
}

uint64_t element_count(const Dims& dim) {
  uint64_t c = 1;
  for (auto d : dim) c *= d;
  return c;
}

Dims make_dims(std::initializer_list<uint32_t> v) {
  Dims d;
  d.fill(1);
  size_t i = 0;
  for (auto x : v) {
    if (i >= d.size()) break;
    d[i++] = x;
  }
  return d;
}

int TensorInfo::rank() const {
  int idx;
  for (idx = kRankLimit - 1; idx > 0; --idx)
    if (dim[idx] != 1) break;
  return idx + 1;
}

bool TensorInfo::operator==(const TensorInfo& o) const {
  if (!valid() || !o.valid()) return false;
  return type == o.type && dim == o.dim;
}

TensorInfo& TensorsInfo::at(unsigned i) {
  if (i >= info.size()) info.resize(i + 1);
  return info[i];
}

const TensorInfo& TensorsInfo::at(unsigned i) const {
  static const TensorInfo kEmpty;
  return i < info.size() ? info[i] : kEmpty;
}

void TensorsInfo::resize(unsigned n) {
  num_tensors = n;
  if (info.size() < n) info.resize(n);
}

bool TensorsInfo::valid() const {
  if (format == Format::END) return false;
  if (format != Format::STATIC) return true;
  if (num_tensors < 1) return false;
  for (unsigned i = 0; i < num_tensors; ++i)
    if (!at(i).valid()) return false;
  return true;
}

bool TensorsInfo::operator==(const TensorsInfo& o) const {
  if (format != o.format || format == Format::END) return false;
  if (format != Format::STATIC) return true;
  if (!valid() || !o.valid()) return false;
  if (num_tensors != o.num_tensors) return false;
  for (unsigned i = 0; i < num_tensors; ++i)
    if (at(i) != o.at(i)) return false;
  return true;
}

size_t TensorsInfo::size(int index) const {
  if (index >= 0) return at(static_cast<unsigned>(index)).size();
  size_t total = 0;
  for (unsigned i = 0; i < num_tensors; ++i) total += at(i).size();
  return total;
}

unsigned TensorsInfo::parse_dimensions(const std::string& s) {
  auto parts = split_any(s, ",.");
  unsigned n = static_cast<unsigned>(parts.size());
  if (n > static_cast<unsigned>(kSizeLimit + kSizeExtraLimit)) n = kSizeLimit + kSizeExtraLimit;
  for (unsigned i = 0; i < n; ++i) parse_dimension(parts[i], at(i).dim);
  return n;
}

unsigned TensorsInfo::parse_types(const std::string& s) {
  auto parts = split_any(s, ",.");
  unsigned n = static_cast<unsigned>(parts.size());
  if (n > static_cast<unsigned>(kSizeLimit + kSizeExtraLimit)) n = kSizeLimit + kSizeExtraLimit;
  for (unsigned i = 0; i < n; ++i) at(i).type = dtype_from_string(parts[i]);
  return n;
}

unsigned TensorsInfo::parse_names(const std::string& s) {
  auto parts = split(s, ',');
  unsigned n = static_cast<unsigned>(parts.size());
  if (n > static_cast<unsigned>(kSizeLimit + kSizeExtraLimit)) n = kSizeLimit + kSizeExtraLimit;
  for (unsigned i = 0; i < n; ++i) at(i).name = strip(parts[i]);
  return n;
}

std::string TensorsInfo::dimensions_string() const { return rank_dimensions_string(kRankLimit); }

std::string TensorsInfo::rank_dimensions_string(unsigned rank) const {
  std::string out;
  for (unsigned i = 0; i < num_tensors; ++i) {
    if (i) out += ',';
    out += rank_dimension_string(at(i).dim, rank);
  }
  return out;
}

std::string TensorsInfo::types_string() const {
  std::string out;
  for (unsigned i = 0; i < num_tensors; ++i) {
    const char* n = dtype_name(at(i).type);
    if (!n) continue;
    if (!out.empty()) out += ',';
    out += n;
  }
  return out;
}

std::string TensorsInfo::names_string() const {
  std::string out;
  for (unsigned i = 0; i < num_tensors; ++i) {
    if (i) out += ',';
    out += at(i).name;
  }
  return out;
}

std::string TensorsInfo::to_string() const {
  std::string out = strfmt("Format = ", format_name(format) ? format_name(format) : "(null)",
                           ", Num_Tensors = ", num_tensors);
  if (format == Format::STATIC) {
    out += ", Tensors = [";
    for (unsigned i = 0; i < num_tensors; ++i) {
      const auto& t = at(i);
      if (i) out += ", ";
      out += strfmt("{", t.name.empty() ? "" : t.name + ", ", dtype_name(t.type) ? dtype_name(t.type) : "(null)", ", ",
                    rank_dimension_string(t.dim, t.rank()), "}");
    }
    out += "]";
  }
  return out;
}

bool TensorsConfig::valid() const {
  if (rate_n < 0 || rate_d <= 0) return false;
  return info.valid();
}

bool TensorsConfig::operator==(const TensorsConfig& o) const {
  // framerate compared as a rational (0/x == 0/y)
  bool rate_eq = (rate_n == 0 && o.rate_n == 0) ||
                 (static_cast<int64_t>(rate_n) * o.rate_d == static_cast<int64_t>(o.rate_n) * rate_d);
  return rate_eq && info == o.info;
}

std::string TensorsConfig::to_string() const {
  return strfmt(info.to_string(), ", Framerate = ", rate_n, "/", rate_d);
}

MetaInfo MetaInfo::from_info(const TensorInfo& info, Format fmt, MediaType media) {
  MetaInfo m;
  m.type = static_cast<uint32_t>(info.type);
  for (int i = 0; i < kRankLimit; ++i) {
    if (info.dim[i] > 0)
      m.dimension[i] = info.dim[i];
    else
      break;
  }
  m.format = static_cast<uint32_t>(fmt);
  m.media_type = static_cast<uint32_t>(media);
  return m;
}

bool MetaInfo::valid() const {
  if ((version & 0xDE000000u) != 0xDE000000u) return false;
  if (!dtype_valid(static_cast<DType>(type))) return false;
  if (dimension[0] == 0) return false;
  if (format >= static_cast<uint32_t>(Format::END)) return false;
  if (static_cast<int32_t>(media_type) > static_cast<int32_t>(MediaType::TENSOR) &&
      static_cast<int32_t>(media_type) != static_cast<int32_t>(MediaType::ANY))
    return false;
  return true;
}

size_t MetaInfo::header_size() const {
  if ((version & 0xDE000000u) != 0xDE000000u) return 0;
  if ((version & 0x00FFF000u) & kVersion) return kMetaHeaderSize;
  return 0;
}

size_t MetaInfo::data_size() const {
  if ((version & 0xDE000000u) != 0xDE000000u) return 0;
  size_t es = dtype_size(static_cast<DType>(type));
  if (format == static_cast<uint32_t>(Format::SPARSE)) return nnz * (es + sizeof(uint32_t));
  size_t ds = es;
  int i = 0;
  for (; i < kMetaRankLimit; ++i) {
    if (dimension[i] == 0) break;
    ds *= dimension[i];
  }
  return i > 0 ? ds : 0;
}

void MetaInfo::write(void* header) const {
  uint32_t v[kMetaHeaderSize / 4];
  std::memset(v, 0, sizeof(v));
  v[0] = version;
  v[1] = type;
  std::memcpy(&v[2], dimension, sizeof(dimension));
  v[18] = format;
  v[19] = media_type;
  v[20] = nnz;
  std::memcpy(header, v, kMetaHeaderSize);
}

bool MetaInfo::parse(const void* header, size_t avail, MetaInfo* out) {
  if (!header || avail < kMetaHeaderSize) return false;
  uint32_t v[21];
  std::memcpy(v, header, sizeof(v));
  MetaInfo m;
  m.version = v[0];
  m.type = v[1];
  std::memcpy(m.dimension, &v[2], sizeof(m.dimension));
  m.format = v[18];
  m.media_type = v[19];
  m.nnz = (m.format == static_cast<uint32_t>(Format::SPARSE)) ? v[20] : 0;
  *out = m;
  return m.valid();
}

bool MetaInfo::to_info(TensorInfo* info) const {
  if (!valid()) return false;
  *info = TensorInfo();
  info->type = static_cast<DType>(type);
  for (int i = 0; i < kMetaRankLimit; ++i) {
    if (i >= kRankLimit) {
      if (dimension[i] > 0) return false;
      break;
    }
    info->dim[i] = dimension[i] > 0 ? dimension[i] : 1;
  }
  return true;
}

const char* version_string() { return "nnsx 2.3.0 (MI355X-native NNStreamer-compatible runtime)"; }

void version_fetch(unsigned* major, unsigned* minor, unsigned* micro) {
  if (major) *major = 2;
  if (minor) *minor = 3;
  if (micro) *micro = 0;
}

}  // namespace nnsx
