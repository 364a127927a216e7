#include "serial/serial.h"

#include <algorithm>
#include <cstring>
#include <map>

#include "core/log.h"

namespace nnsx {
namespace serial {

namespace {

struct Item {
  std::string name;
  uint32_t type = 0;
  uint32_t dims[kRankLimit] = {0};
  const uint8_t* data = nullptr;
  size_t size = 0;
};

// per-tensor wire fields; flexible payloads keep their header in `data` and
// take type / dims from it (the reference's gst_tensor_meta_info_convert)
std::vector<Item> items_of(const TensorsConfig& c, const std::vector<MemoryPtr>& t) {
  std::vector<Item> r;
  const size_t n = std::min<size_t>(c.info.num_tensors ? c.info.num_tensors : t.size(), t.size());
  for (size_t i = 0; i < n; ++i) {
    Item it;
    TensorInfo ti = i < c.info.num_tensors ? c.info.at(static_cast<unsigned>(i)) : TensorInfo();
    it.data = static_cast<const uint8_t*>(t[i]->map_host());
    it.size = t[i]->size();
    if (c.is_flexible()) {
      MetaInfo meta;
      if (MetaInfo::parse(it.data, it.size, &meta)) meta.to_info(&ti);
    }
    it.name = ti.name;
    it.type = static_cast<uint32_t>(ti.type);
    for (int k = 0; k < kRankLimit; ++k) it.dims[k] = ti.dim[k];
    r.push_back(std::move(it));
  }
  return r;
}

TensorInfo info_of(const std::string& name, uint32_t type, const uint32_t* dims, int ndims) {
  TensorInfo ti;
  ti.name = name;
  ti.type = static_cast<DType>(type);
  for (int k = 0; k < kRankLimit; ++k) ti.dim[k] = k < ndims && dims[k] ? dims[k] : 1;  // 0 = unused rank
  return ti;
}

MemoryPtr host_copy(const uint8_t* p, size_t n) {
  auto m = Memory::alloc_host(n);
  if (n) std::memcpy(m->data(), p, n);
  return m;
}

// ================================================================ protobuf ====
size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

struct PbWriter {
  uint8_t* p;
  void varint(uint64_t v) {
    while (v >= 0x80) {
      *p++ = static_cast<uint8_t>(v | 0x80);
      v >>= 7;
    }
    *p++ = static_cast<uint8_t>(v);
  }
  void tag(int field, int wt) { varint(static_cast<uint64_t>(field) << 3 | static_cast<uint64_t>(wt)); }
  void raw(const void* d, size_t n) {
    if (n) std::memcpy(p, d, n);
    p += n;
  }
};

// int32 fields are sign-extended to 64-bit varints (protobuf wire rule)
uint64_t pb_int32(int32_t v) { return static_cast<uint64_t>(static_cast<int64_t>(v)); }

size_t pb_dims_len(const Item& it) {
  size_t n = 0;
  for (uint32_t d : it.dims) n += varint_len(d);
  return n;
}

size_t pb_tensor_len(const Item& it) {
  size_t n = 0;
  if (!it.name.empty()) n += 1 + varint_len(it.name.size()) + it.name.size();
  if (it.type) n += 1 + varint_len(it.type);
  const size_t dl = pb_dims_len(it);
  n += 1 + varint_len(dl) + dl;  // packed repeated uint32 (proto3 default)
  if (it.size) n += 1 + varint_len(it.size) + it.size;
  return n;
}

MemoryPtr pb_encode(const TensorsConfig& c, const std::vector<Item>& items) {
  const uint32_t num = static_cast<uint32_t>(items.size());
  const size_t fr_len = (c.rate_n ? 1 + varint_len(pb_int32(c.rate_n)) : 0) + (c.rate_d ? 1 + varint_len(pb_int32(c.rate_d)) : 0);
  size_t total = (num ? 1 + varint_len(num) : 0) + 1 + varint_len(fr_len) + fr_len;
  std::vector<size_t> tl;
  for (auto& it : items) {
    tl.push_back(pb_tensor_len(it));
    total += 1 + varint_len(tl.back()) + tl.back();
  }
  const uint32_t fmt = static_cast<uint32_t>(c.info.format);
  if (fmt) total += 1 + varint_len(fmt);
  auto m = Memory::alloc_host(total);
  PbWriter w{static_cast<uint8_t*>(m->data())};
  if (num) {
    w.tag(1, 0);
    w.varint(num);
  }
  w.tag(2, 2);  // fr is always set (mutable_fr in the reference)
  w.varint(fr_len);
  if (c.rate_n) {
    w.tag(1, 0);
    w.varint(pb_int32(c.rate_n));
  }
  if (c.rate_d) {
    w.tag(2, 0);
    w.varint(pb_int32(c.rate_d));
  }
  for (size_t i = 0; i < items.size(); ++i) {
    const Item& it = items[i];
    w.tag(3, 2);
    w.varint(tl[i]);
    if (!it.name.empty()) {
      w.tag(1, 2);
      w.varint(it.name.size());
      w.raw(it.name.data(), it.name.size());
    }
    if (it.type) {
      w.tag(2, 0);
      w.varint(it.type);
    }
    w.tag(3, 2);
    w.varint(pb_dims_len(it));
    for (uint32_t d : it.dims) w.varint(d);
    if (it.size) {
      w.tag(4, 2);
      w.varint(it.size);
      w.raw(it.data, it.size);
    }
  }
  if (fmt) {
    w.tag(4, 0);
    w.varint(fmt);
  }
  return m;
}

struct PbReader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  bool varint(uint64_t* v) {
    *v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= end) return ok = false;
      const uint8_t b = *p++;
      *v |= static_cast<uint64_t>(b & 0x7f) << s;
      if (!(b & 0x80)) return true;
    }
    return ok = false;
  }
  // next field: number, wire type; LEN fields give [*d, *d + *n)
  bool field(int* num, int* wt, uint64_t* v, const uint8_t** d, size_t* n) {
    uint64_t key;
    if (p >= end || !varint(&key)) return false;
    *num = static_cast<int>(key >> 3);
    *wt = static_cast<int>(key & 7);
    switch (*wt) {
      case 0: return varint(v);
      case 1:
        if (end - p < 8) return ok = false;
        std::memcpy(v, p, 8);
        p += 8;
        return true;
      case 5: {
        if (end - p < 4) return ok = false;
        uint32_t x;
        std::memcpy(&x, p, 4);
        *v = x;
        p += 4;
        return true;
      }
      case 2: {
        uint64_t len;
        if (!varint(&len) || len > static_cast<uint64_t>(end - p)) return ok = false;
        *d = p;
        *n = static_cast<size_t>(len);
        p += len;
        return true;
      }
      default: return ok = false;
    }
  }
};

bool pb_decode(const uint8_t* data, size_t size, TensorsConfig* c, std::vector<MemoryPtr>* out) {
  PbReader r{data, data + size};
  uint64_t num = 0, fmt = 0;
  int64_t rate_n = 0, rate_d = 0;
  std::vector<std::pair<const uint8_t*, size_t>> tensors;
  int f, wt;
  uint64_t v = 0;
  const uint8_t* d = nullptr;
  size_t n = 0;
  while (r.field(&f, &wt, &v, &d, &n)) {
    if (f == 1 && wt == 0) num = v;
    else if (f == 4 && wt == 0) fmt = v;
    else if (f == 3 && wt == 2) tensors.emplace_back(d, n);
    else if (f == 2 && wt == 2) {
      PbReader fr{d, d + n};
      int g, gw;
      uint64_t x = 0;
      const uint8_t* dd;
      size_t nn;
      while (fr.field(&g, &gw, &x, &dd, &nn)) {
        if (g == 1 && gw == 0) rate_n = static_cast<int32_t>(x);
        if (g == 2 && gw == 0) rate_d = static_cast<int32_t>(x);
      }
      if (!fr.ok) return false;
    }
  }
  if (!r.ok || num > static_cast<uint64_t>(kSizeLimit) || tensors.size() < num) return false;
  c->info.num_tensors = static_cast<unsigned>(num);
  c->info.format = static_cast<Format>(std::min<uint64_t>(fmt, static_cast<uint64_t>(Format::SPARSE)));
  c->rate_n = static_cast<int>(rate_n);
  c->rate_d = static_cast<int>(rate_d);
  out->clear();
  for (unsigned i = 0; i < num; ++i) {
    PbReader t{tensors[i].first, tensors[i].first + tensors[i].second};
    std::string name;
    uint64_t type = 0;
    uint32_t dims[kRankLimit] = {0};
    int nd = 0;
    const uint8_t* payload = nullptr;
    size_t plen = 0;
    while (t.field(&f, &wt, &v, &d, &n)) {
      if (f == 1 && wt == 2) name.assign(reinterpret_cast<const char*>(d), n);
      else if (f == 2 && wt == 0) type = v;
      else if (f == 3 && wt == 2) {  // packed
        PbReader pk{d, d + n};
        uint64_t x;
        while (pk.p < pk.end && pk.varint(&x))
          if (nd < kRankLimit) dims[nd++] = static_cast<uint32_t>(x);
        if (!pk.ok) return false;
      } else if (f == 3 && wt == 0) {
        if (nd < kRankLimit) dims[nd++] = static_cast<uint32_t>(v);
      } else if (f == 4 && wt == 2) {
        payload = d;
        plen = n;
      }
    }
    if (!t.ok) return false;
    c->info.at(i) = info_of(name, static_cast<uint32_t>(type), dims, nd);
    out->push_back(host_copy(payload, plen));
  }
  return true;
}

// ================================================================= flatbuf ====
struct FbWriter {
  std::string b;
  size_t here() const { return b.size(); }
  void pad(size_t a) {
    while (b.size() % a) b.push_back('\0');
  }
  size_t u32(uint32_t v) {
    size_t p = b.size();
    b.append(reinterpret_cast<const char*>(&v), 4);
    return p;
  }
  size_t u16(uint16_t v) {
    size_t p = b.size();
    b.append(reinterpret_cast<const char*>(&v), 2);
    return p;
  }
  void set32(size_t at, uint32_t v) { std::memcpy(&b[at], &v, 4); }
  // vtable (4 + 2 * n bytes) then the table; returns the table position
  size_t table(const std::vector<uint16_t>& field_off, uint16_t inline_size) {
    pad(4);
    const size_t vt = u16(static_cast<uint16_t>(4 + 2 * field_off.size()));
    u16(inline_size);
    for (auto o : field_off) u16(o);
    pad(4);
    const size_t t = here();
    u32(static_cast<uint32_t>(t - vt));  // soffset: vtable = table - soffset
    return t;
  }
};

constexpr uint32_t kFbTypeDefault = 10;  // NNS_END

MemoryPtr fb_encode(const TensorsConfig& c, const std::vector<Item>& items) {
  FbWriter w;
  const size_t root = w.u32(0);
  const uint32_t fmt = static_cast<uint32_t>(c.info.format);
  const uint32_t num = static_cast<uint32_t>(items.size());
  // Tensors: [soff][num_tensor][fr.rate_n][fr.rate_d][tensor uoffset][format]
  std::vector<uint16_t> fo = {static_cast<uint16_t>(num ? 4 : 0), 8, 16, static_cast<uint16_t>(fmt ? 20 : 0)};
  const size_t t = w.table(fo, static_cast<uint16_t>(fmt ? 24 : 20));
  w.set32(root, static_cast<uint32_t>(t - root));
  w.u32(num);
  w.u32(static_cast<uint32_t>(c.rate_n));
  w.u32(static_cast<uint32_t>(c.rate_d));
  const size_t vec_field = w.u32(0);
  if (fmt) w.u32(fmt);
  // tensor vector of table offsets
  w.pad(4);
  const size_t vec = w.u32(num);
  w.set32(vec_field, static_cast<uint32_t>(vec - vec_field));
  std::vector<size_t> slots;
  for (uint32_t i = 0; i < num; ++i) slots.push_back(w.u32(0));
  for (uint32_t i = 0; i < num; ++i) {
    const Item& it = items[i];
    // Tensor: [soff][name uoff][type][dimension uoff][data uoff]
    const bool has_type = it.type != kFbTypeDefault;
    std::vector<uint16_t> to = {4, static_cast<uint16_t>(has_type ? 8 : 0), 12, 16};
    const size_t tt = w.table(to, 20);
    w.set32(slots[i], static_cast<uint32_t>(tt - slots[i]));
    const size_t f_name = w.u32(0);
    w.u32(has_type ? it.type : 0);
    const size_t f_dims = w.u32(0);
    const size_t f_data = w.u32(0);
    w.pad(4);
    const size_t s = w.u32(static_cast<uint32_t>(it.name.size()));
    w.b.append(it.name);
    w.b.push_back('\0');
    w.set32(f_name, static_cast<uint32_t>(s - f_name));
    w.pad(4);
    const size_t dv = w.u32(kRankLimit);
    for (uint32_t dd : it.dims) w.u32(dd);
    w.set32(f_dims, static_cast<uint32_t>(dv - f_dims));
    const size_t bv = w.u32(static_cast<uint32_t>(it.size));
    w.b.append(reinterpret_cast<const char*>(it.data), it.size);
    w.set32(f_data, static_cast<uint32_t>(bv - f_data));
  }
  w.pad(4);
  return host_copy(reinterpret_cast<const uint8_t*>(w.b.data()), w.b.size());
}

struct FbReader {
  const uint8_t* b;
  size_t n;
  bool ok = true;
  uint32_t u32(size_t at) {
    if (at + 4 > n) {
      ok = false;
      return 0;
    }
    uint32_t v;
    std::memcpy(&v, b + at, 4);
    return v;
  }
  uint16_t u16(size_t at) {
    if (at + 2 > n) {
      ok = false;
      return 0;
    }
    uint16_t v;
    std::memcpy(&v, b + at, 2);
    return v;
  }
  // position of field `id` of the table at `t`, 0 if absent
  size_t field(size_t t, int id) {
    const int32_t so = static_cast<int32_t>(u32(t));
    const size_t vt = static_cast<size_t>(static_cast<int64_t>(t) - so);
    if (!ok || vt + 4 > n) return ok = false, 0;
    const uint16_t vsz = u16(vt);
    const size_t at = 4 + 2 * static_cast<size_t>(id);
    if (at + 2 > vsz) return 0;
    const uint16_t o = u16(vt + at);
    return o ? t + o : 0;
  }
  size_t deref(size_t at) { return at + u32(at); }
};

bool fb_decode(const uint8_t* data, size_t size, TensorsConfig* c, std::vector<MemoryPtr>* out) {
  FbReader r{data, size};
  const size_t t = r.deref(0);
  if (!r.ok || t >= size) return false;
  size_t f;
  const uint32_t num = (f = r.field(t, 0)) ? r.u32(f) : 0;
  c->rate_n = c->rate_d = 0;
  if ((f = r.field(t, 1))) {
    c->rate_n = static_cast<int32_t>(r.u32(f));
    c->rate_d = static_cast<int32_t>(r.u32(f + 4));
  }
  const uint32_t fmt = (f = r.field(t, 3)) ? r.u32(f) : 0;
  if (num > static_cast<uint32_t>(kSizeLimit)) return false;
  size_t vec = 0;
  uint32_t count = 0;
  if ((f = r.field(t, 2))) {
    vec = r.deref(f);
    count = r.u32(vec);
  }
  if (!r.ok || count < num) return false;
  c->info.num_tensors = num;
  c->info.format = static_cast<Format>(std::min<uint32_t>(fmt, static_cast<uint32_t>(Format::SPARSE)));
  out->clear();
  for (uint32_t i = 0; i < num; ++i) {
    const size_t tt = r.deref(vec + 4 + 4 * static_cast<size_t>(i));
    std::string name;
    if ((f = r.field(tt, 0))) {
      const size_t s = r.deref(f);
      const uint32_t len = r.u32(s);
      if (s + 4 + len > size) return false;
      name.assign(reinterpret_cast<const char*>(data + s + 4), len);
    }
    const uint32_t type = (f = r.field(tt, 1)) ? r.u32(f) : kFbTypeDefault;
    uint32_t dims[kRankLimit] = {0};
    int nd = 0;
    if ((f = r.field(tt, 2))) {
      const size_t dv = r.deref(f);
      const uint32_t cnt = r.u32(dv);
      for (uint32_t k = 0; k < cnt && nd < kRankLimit; ++k) dims[nd++] = r.u32(dv + 4 + 4 * static_cast<size_t>(k));
    }
    const uint8_t* payload = nullptr;
    uint32_t plen = 0;
    if ((f = r.field(tt, 3))) {
      const size_t bv = r.deref(f);
      plen = r.u32(bv);
      if (bv + 4 + plen > size) return false;
      payload = data + bv + 4;
    }
    if (!r.ok) return false;
    c->info.at(i) = info_of(name, type, dims, nd);
    out->push_back(host_copy(payload, plen));
  }
  return true;
}

// ================================================================= flexbuf ====
enum FlexType : uint8_t {
  FX_NULL = 0, FX_INT = 1, FX_UINT = 2, FX_FLOAT = 3, FX_KEY = 4, FX_STRING = 5, FX_INDIRECT_INT = 6,
  FX_INDIRECT_UINT = 7, FX_INDIRECT_FLOAT = 8, FX_MAP = 9, FX_VECTOR = 10, FX_VECTOR_INT = 11, FX_VECTOR_UINT = 12,
  FX_VECTOR_FLOAT = 13, FX_VECTOR_KEY = 14, FX_VECTOR_INT2 = 16, FX_VECTOR_UINT4 = 23, FX_BLOB = 25, FX_BOOL = 26,
};
constexpr uint8_t kW = 8;                 // every slot written 8 bytes wide
constexpr uint8_t packed(uint8_t t) { return static_cast<uint8_t>(t << 2 | 3); }

struct FxWriter {
  std::string b;
  void pad() {
    while (b.size() % kW) b.push_back('\0');
  }
  void u64(uint64_t v) { b.append(reinterpret_cast<const char*>(&v), 8); }
  size_t key(const std::string& k) {
    size_t p = b.size();
    b.append(k);
    b.push_back('\0');
    return p;
  }
  size_t sized(const void* d, size_t n, bool nul) {  // string / blob: [size][bytes](\0)
    pad();
    u64(n);
    size_t p = b.size();
    b.append(static_cast<const char*>(d), n);
    if (nul) b.push_back('\0');
    return p;
  }
  // slot value for an offset child at `target` from slot position `slot`
  static uint64_t rel(size_t slot, size_t target) { return static_cast<uint64_t>(slot - target); }
};

MemoryPtr fx_encode(const TensorsConfig& c, const std::vector<Item>& items) {
  FxWriter w;
  struct Val {
    std::string key;
    uint8_t type;
    uint64_t v;  // inline value or target position
    bool offset;
  };
  std::vector<Val> vals;
  vals.push_back({"num_tensors", FX_UINT, items.size(), false});
  vals.push_back({"rate_n", FX_INT, static_cast<uint64_t>(static_cast<int64_t>(c.rate_n)), false});
  vals.push_back({"rate_d", FX_INT, static_cast<uint64_t>(static_cast<int64_t>(c.rate_d)), false});
  vals.push_back({"format", FX_INT, static_cast<uint64_t>(c.info.format), false});
  for (size_t i = 0; i < items.size(); ++i) {
    const Item& it = items[i];
    const size_t name = w.sized(it.name.data(), it.name.size(), true);
    w.pad();
    w.u64(kRankLimit);
    const size_t dims = w.b.size();
    for (uint32_t d : it.dims) w.u64(d);
    const size_t blob = w.sized(it.data, it.size, false);
    // [name, type, dims, blob] untyped vector
    w.pad();
    w.u64(4);
    const size_t vec = w.b.size();
    w.u64(FxWriter::rel(vec, name));
    w.u64(static_cast<uint64_t>(static_cast<int64_t>(it.type)));
    w.u64(FxWriter::rel(vec + 16, dims));
    w.u64(FxWriter::rel(vec + 24, blob));
    w.b.push_back(static_cast<char>(packed(FX_STRING)));
    w.b.push_back(static_cast<char>(packed(FX_INT)));
    w.b.push_back(static_cast<char>(packed(FX_VECTOR_UINT)));
    w.b.push_back(static_cast<char>(packed(FX_BLOB)));
    vals.push_back({"tensor_" + std::to_string(i), FX_VECTOR, vec, true});
  }
  std::sort(vals.begin(), vals.end(), [](const Val& a, const Val& b) { return a.key < b.key; });  // strcmp order
  std::vector<size_t> keys;
  for (auto& v : vals) keys.push_back(w.key(v.key));
  w.pad();
  w.u64(vals.size());
  const size_t kv = w.b.size();
  for (size_t i = 0; i < keys.size(); ++i) w.u64(FxWriter::rel(kv + 8 * i, keys[i]));
  // map: [keys offset][keys width][size][values][types]
  w.pad();
  const size_t kslot = w.b.size();
  w.u64(FxWriter::rel(kslot, kv));
  w.u64(kW);
  w.u64(vals.size());
  const size_t map = w.b.size();
  for (size_t i = 0; i < vals.size(); ++i) w.u64(vals[i].offset ? FxWriter::rel(map + 8 * i, vals[i].v) : vals[i].v);
  for (auto& v : vals) w.b.push_back(static_cast<char>(packed(v.type)));
  w.pad();
  const size_t root = w.b.size();
  w.u64(FxWriter::rel(root, map));
  w.b.push_back(static_cast<char>(packed(FX_MAP)));
  w.b.push_back(static_cast<char>(kW));
  return host_copy(reinterpret_cast<const uint8_t*>(w.b.data()), w.b.size());
}

struct FxRef {
  const uint8_t* b = nullptr;
  size_t n = 0;
  size_t slot = 0;         // where the value (or its offset) sits
  uint8_t parent_w = 1;    // width of that slot
  uint8_t type = FX_NULL;  // FlexType
  uint8_t child_w = 1;     // width of the pointed-to data
  bool ok = true;

  uint64_t rdu(size_t at, uint8_t w) {
    if (at + w > n) {
      ok = false;
      return 0;
    }
    uint64_t v = 0;
    std::memcpy(&v, b + at, w);  // little endian
    return v;
  }
  int64_t rdi(size_t at, uint8_t w) {
    uint64_t v = rdu(at, w);
    if (w < 8) {
      const uint64_t sign = 1ull << (8 * w - 1);
      v = (v ^ sign) - sign;
    }
    return static_cast<int64_t>(v);
  }
  size_t target() {
    const uint64_t o = rdu(slot, parent_w);
    if (o > slot) return ok = false, 0;
    return slot - static_cast<size_t>(o);
  }
  int64_t as_int() {
    switch (type) {
      case FX_INT: return rdi(slot, parent_w);
      case FX_UINT: case FX_BOOL: return static_cast<int64_t>(rdu(slot, parent_w));
      case FX_INDIRECT_INT: return rdi(target(), child_w);
      case FX_INDIRECT_UINT: return static_cast<int64_t>(rdu(target(), child_w));
      default: return 0;
    }
  }
  FxRef child(size_t s, uint8_t pw, uint8_t packed_type) const {
    FxRef r{b, n, s, pw, static_cast<uint8_t>(packed_type >> 2), static_cast<uint8_t>(1u << (packed_type & 3)), true};
    return r;
  }
  // vectors / maps: element count and the i-th element
  size_t size() {
    const size_t d = target();
    if (type == FX_VECTOR_INT2 || type == FX_VECTOR_INT2 + 1 || type == FX_VECTOR_INT2 + 2) return 2;
    if (type >= FX_VECTOR_INT2 + 3 && type <= FX_VECTOR_INT2 + 5) return 3;
    if (type >= FX_VECTOR_INT2 + 6 && type <= FX_VECTOR_INT2 + 8) return 4;
    if (d < child_w) return ok = false, 0;
    return static_cast<size_t>(rdu(d - child_w, child_w));
  }
  FxRef at(size_t i) {
    const size_t d = target();
    const size_t cnt = size();
    if (i >= cnt) {
      FxRef r = *this;
      r.ok = false;
      return r;
    }
    if (type == FX_VECTOR || type == FX_MAP) {
      const uint8_t pt = static_cast<uint8_t>(rdu(d + cnt * child_w + i, 1));
      return child(d + i * child_w, child_w, pt);
    }
    // typed vectors: element type from the vector type, inline scalars
    uint8_t et = FX_INT;
    if (type == FX_VECTOR_UINT || (type >= FX_VECTOR_INT2 && (type - FX_VECTOR_INT2) % 3 == 1)) et = FX_UINT;
    if (type == FX_VECTOR_KEY) et = FX_KEY;
    return child(d + i * child_w, child_w, static_cast<uint8_t>(et << 2));
  }
  std::string as_string() {  // STRING / KEY / BLOB contents
    const size_t d = target();
    if (type == FX_KEY) {
      size_t e = d;
      while (e < n && b[e]) ++e;
      return std::string(reinterpret_cast<const char*>(b + d), e - d);
    }
    const size_t len = static_cast<size_t>(rdu(d - child_w, child_w));
    if (!ok || d + len > n) return ok = false, std::string();
    return std::string(reinterpret_cast<const char*>(b + d), len);
  }
  bool blob(const uint8_t** p, size_t* len) {
    const size_t d = target();
    *len = static_cast<size_t>(rdu(d - child_w, child_w));
    if (!ok || d + *len > n) return ok = false;
    *p = b + d;
    return true;
  }
  FxRef lookup(const std::string& key) {
    const size_t d = target();
    const size_t ks = d - 3 * static_cast<size_t>(child_w);
    FxRef keys = child(ks, child_w, static_cast<uint8_t>(FX_VECTOR_KEY << 2 | 0));
    keys.child_w = static_cast<uint8_t>(rdu(d - 2 * static_cast<size_t>(child_w), child_w));
    const size_t cnt = size();
    for (size_t i = 0; i < cnt && ok; ++i) {
      FxRef k = keys.at(i);
      if (k.as_string() == key) return at(i);
    }
    FxRef none = *this;
    none.type = FX_NULL;
    return none;
  }
};

bool fx_decode(const uint8_t* data, size_t size, TensorsConfig* c, std::vector<MemoryPtr>* out) {
  if (size < 3) return false;
  const uint8_t w = data[size - 1];
  if (w != 1 && w != 2 && w != 4 && w != 8) return false;
  FxRef root{data, size, size - 2 - w, w, FX_NULL, 1, true};
  root = root.child(size - 2 - w, w, data[size - 2]);
  if (root.type != FX_MAP) return false;
  const int64_t num = root.lookup("num_tensors").as_int();
  if (num < 0 || num > kSizeLimit) return false;
  c->info.num_tensors = static_cast<unsigned>(num);
  c->rate_n = static_cast<int>(root.lookup("rate_n").as_int());
  c->rate_d = static_cast<int>(root.lookup("rate_d").as_int());
  c->info.format = static_cast<Format>(std::clamp<int64_t>(root.lookup("format").as_int(), 0, 2));
  out->clear();
  for (int64_t i = 0; i < num; ++i) {
    FxRef t = root.lookup("tensor_" + std::to_string(i));
    if (t.type != FX_VECTOR || t.size() < 4) return false;
    FxRef nm = t.at(0), ty = t.at(1), dv = t.at(2), bl = t.at(3);
    uint32_t dims[kRankLimit] = {0};
    const size_t nd = std::min<size_t>(dv.size(), kRankLimit);
    for (size_t k = 0; k < nd; ++k) dims[k] = static_cast<uint32_t>(dv.at(k).as_int());
    const uint8_t* p = nullptr;
    size_t len = 0;
    if (!bl.blob(&p, &len)) return false;
    if (!(t.ok && nm.ok && ty.ok && dv.ok && root.ok)) return false;
    c->info.at(static_cast<unsigned>(i)) =
        info_of(nm.as_string(), static_cast<uint32_t>(ty.as_int()), dims, static_cast<int>(nd));
    out->push_back(host_copy(p, len));
  }
  return root.ok;
}

}  // namespace

const char* wire_name(Wire w) {
  switch (w) {
    case Wire::PROTOBUF: return "protobuf";
    case Wire::FLATBUF: return "flatbuf";
    default: return "flexbuf";
  }
}

const char* wire_caps(Wire w) {
  switch (w) {
    case Wire::PROTOBUF: return "other/protobuf-tensor";
    case Wire::FLATBUF: return "other/flatbuf-tensor";
    default: return "other/flexbuf";
  }
}

MemoryPtr encode(Wire w, const TensorsConfig& config, const std::vector<MemoryPtr>& tensors) {
  auto items = items_of(config, tensors);
  switch (w) {
    case Wire::PROTOBUF: return pb_encode(config, items);
    case Wire::FLATBUF: return fb_encode(config, items);
    default: return fx_encode(config, items);
  }
}

bool decode(Wire w, const void* data, size_t size, TensorsConfig* config, std::vector<MemoryPtr>* tensors) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  config->info.resize(kSizeLimit);
  switch (w) {
    case Wire::PROTOBUF: return pb_decode(p, size, config, tensors);
    case Wire::FLATBUF: return fb_decode(p, size, config, tensors);
    default: return fx_decode(p, size, config, tensors);
  }
}

}  // namespace serial
}  // namespace nnsx
