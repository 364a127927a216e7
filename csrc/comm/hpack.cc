// HPACK (RFC 7541): see hpack.h.
#include "comm/hpack.h"

#include <array>

namespace nnsx {
namespace hpack {
namespace {

// RFC 7541 Appendix A
const char* const kStatic[61][2] = {
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""}, {"cache-control", ""},
    {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""}, {"content-length", ""},
    {"content-location", ""}, {"content-range", ""}, {"content-type", ""}, {"cookie", ""}, {"date", ""},
    {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""}, {"if-match", ""},
    {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""}, {"if-unmodified-since", ""},
    {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""}, {"proxy-authenticate", ""},
    {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""}, {"retry-after", ""},
    {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""}, {"transfer-encoding", ""},
    {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""}};

// Huffman code lengths of symbols 0..255 and EOS (256), RFC 7541 Appendix B.
// The code is canonical: ordering symbols by (length, symbol) and counting up
// reproduces the appendix's code words, so the lengths define it completely.
constexpr uint8_t kHuffLen[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 30, 28, 28, 28,
    28, 28, 28, 28, 28, 28, 6,  10, 10, 12, 13, 6,  8,  11, 10, 10, 8,  11, 8,  6,  6,  6,  5,  5,  5,  6,
    6,  6,  6,  6,  6,  6,  7,  8,  15, 6,  12, 10, 13, 6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,
    7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8,  13, 19, 13, 14, 6,  15, 5,  6,  5,  6,  5,  6,  6,
    6,  5,  7,  7,  6,  6,  6,  5,  6,  7,  6,  5,  5,  6,  7,  7,  7,  7,  7,  15, 11, 14, 13, 28, 20, 22,
    20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23,
    22, 23, 23, 24, 22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22,
    23, 23, 20, 22, 22, 22, 23, 22, 22, 23, 26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27, 20, 24, 20, 21, 22, 21, 21, 23, 22, 22,
    25, 25, 24, 24, 26, 23, 26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26, 30};

struct Huffman {
  uint32_t code[257];
  // canonical decoding: per length, the first code and the index of its first
  // symbol in `sorted`
  uint32_t first[31] = {};
  int count[31] = {}, base[31] = {};
  uint16_t sorted[257];
  Huffman() {
    int n = 0;
    for (int len = 1; len <= 30; ++len)
      for (int s = 0; s < 257; ++s)
        if (kHuffLen[s] == len) sorted[n++] = static_cast<uint16_t>(s);
    uint32_t c = 0;
    int prev = kHuffLen[sorted[0]];
    for (int i = 0; i < 257; ++i) {
      const int len = kHuffLen[sorted[i]];
      if (i) c = (c + 1) << (len - prev);
      prev = len;
      code[sorted[i]] = c;
      if (count[len]++ == 0) {
        first[len] = c;
        base[len] = i;
      }
    }
  }
};
const Huffman& huff() {
  static const Huffman h;
  return h;
}

// integer with an N-bit prefix (RFC 7541 5.1)
bool read_int(const uint8_t*& p, const uint8_t* end, int prefix_bits, uint64_t* v) {
  if (p >= end) return false;
  const uint64_t mask = (1u << prefix_bits) - 1;
  uint64_t x = *p++ & mask;
  if (x < mask) {
    *v = x;
    return true;
  }
  int shift = 0;
  while (p < end && shift < 56) {
    const uint8_t b = *p++;
    x += static_cast<uint64_t>(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;
}

void write_int(std::string* out, uint8_t first_bits, int prefix_bits, uint64_t v) {
  const uint64_t mask = (1u << prefix_bits) - 1;
  if (v < mask) {
    out->push_back(static_cast<char>(first_bits | v));
    return;
  }
  out->push_back(static_cast<char>(first_bits | mask));
  v -= mask;
  while (v >= 0x80) {
    out->push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  out->push_back(static_cast<char>(v));
}

bool read_string(const uint8_t*& p, const uint8_t* end, std::string* s) {
  if (p >= end) return false;
  const bool huffman = (*p & 0x80) != 0;
  uint64_t len;
  if (!read_int(p, end, 7, &len) || len > static_cast<uint64_t>(end - p)) return false;
  if (huffman) {
    if (!huffman_decode(p, len, s)) return false;
  } else {
    s->assign(reinterpret_cast<const char*>(p), len);
  }
  p += len;
  return true;
}

}  // namespace

std::string huffman_encode(const std::string& s) {
  const Huffman& h = huff();
  std::string out;
  uint64_t acc = 0;
  int bits = 0;
  for (unsigned char c : s) {
    acc = (acc << kHuffLen[c]) | h.code[c];
    bits += kHuffLen[c];
    while (bits >= 8) {
      bits -= 8;
      out.push_back(static_cast<char>(acc >> bits));
    }
  }
  if (bits) out.push_back(static_cast<char>((acc << (8 - bits)) | (0xff >> bits)));  // EOS-prefix padding
  return out;
}

bool huffman_decode(const uint8_t* p, size_t n, std::string* out) {
  const Huffman& h = huff();
  out->clear();
  uint32_t code = 0;
  int len = 0;
  for (size_t i = 0; i < n; ++i) {
    for (int b = 7; b >= 0; --b) {
      code = (code << 1) | ((p[i] >> b) & 1);
      ++len;
      if (len > 30) return false;
      if (h.count[len] && code >= h.first[len] && code - h.first[len] < static_cast<uint32_t>(h.count[len])) {
        const int sym = h.sorted[h.base[len] + static_cast<int>(code - h.first[len])];
        if (sym == 256) return false;  // EOS inside a string is an error (5.2)
        out->push_back(static_cast<char>(sym));
        code = 0;
        len = 0;
      }
    }
  }
  // padding: at most 7 bits, all ones (the most significant bits of EOS)
  return len <= 7 && code == (1u << len) - 1;
}

bool Decoder::lookup(uint64_t index, Header* h) const {
  if (index == 0) return false;
  if (index <= 61) {
    *h = {kStatic[index - 1][0], kStatic[index - 1][1]};
    return true;
  }
  const uint64_t d = index - 62;
  if (d >= dyn_.size()) return false;
  *h = dyn_[d];
  return true;
}

void Decoder::evict() {
  while (size_ > limit_ && !dyn_.empty()) {
    size_ -= dyn_.back().first.size() + dyn_.back().second.size() + 32;
    dyn_.pop_back();
  }
}

void Decoder::insert(Header h) {
  const size_t sz = h.first.size() + h.second.size() + 32;
  if (sz > limit_) {  // larger than the table: empties it (4.4)
    dyn_.clear();
    size_ = 0;
    return;
  }
  size_ += sz;
  dyn_.push_front(std::move(h));
  evict();
}

bool Decoder::decode(const uint8_t* p, size_t n, Headers* out, std::string* err) {
  const uint8_t* end = p + n;
  while (p < end) {
    const uint8_t b = *p;
    if (b & 0x80) {  // indexed field (6.1)
      uint64_t idx;
      Header h;
      if (!read_int(p, end, 7, &idx) || !lookup(idx, &h)) {
        *err = "hpack: bad index";
        return false;
      }
      out->push_back(std::move(h));
    } else if ((b & 0xe0) == 0x20) {  // dynamic table size update (6.3)
      uint64_t sz;
      if (!read_int(p, end, 5, &sz) || sz > max_) {
        *err = "hpack: bad table size update";
        return false;
      }
      limit_ = sz;
      evict();
    } else {
      // literal: with incremental indexing (01), without (0000) or never indexed (0001)
      const bool incremental = (b & 0xc0) == 0x40;
      const int prefix = incremental ? 6 : 4;
      uint64_t idx;
      if (!read_int(p, end, prefix, &idx)) {
        *err = "hpack: truncated literal";
        return false;
      }
      Header h;
      if (idx) {
        if (!lookup(idx, &h)) {
          *err = "hpack: bad name index";
          return false;
        }
      } else if (!read_string(p, end, &h.first)) {
        *err = "hpack: bad name";
        return false;
      }
      if (!read_string(p, end, &h.second)) {
        *err = "hpack: bad value";
        return false;
      }
      if (incremental) insert(h);
      out->push_back(std::move(h));
    }
  }
  return true;
}

void Encoder::encode(const Headers& hs, std::string* out) const {
  for (const auto& h : hs) {
    write_int(out, 0x00, 4, 0);  // literal without indexing, new name
    write_int(out, 0x00, 7, h.first.size());
    out->append(h.first);
    write_int(out, 0x00, 7, h.second.size());
    out->append(h.second);
  }
}

}  // namespace hpack
}  // namespace nnsx
