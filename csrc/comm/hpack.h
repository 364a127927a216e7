// HPACK (RFC 7541) header compression for the native HTTP/2 gRPC transport
// (comm/grpc_native.cc).  The decoder is complete -- static + dynamic table,
// all five representations, table size updates, Huffman-coded strings -- so
// any peer's header blocks decode; the encoder emits literal fields without
// indexing and without Huffman coding (always valid, never touches the peer's
// dynamic table).
#pragma once

#include <cstdint>
#include <deque>
#include <string>
#include <utility>
#include <vector>

namespace nnsx {
namespace hpack {

using Header = std::pair<std::string, std::string>;
using Headers = std::vector<Header>;

class Decoder {
 public:
  // the SETTINGS_HEADER_TABLE_SIZE this side advertised (the peer's encoder may
  // resize its table up to it)
  explicit Decoder(size_t max_table = 4096) : limit_(max_table), max_(max_table) {}
  // one complete header block (HEADERS + CONTINUATION payloads)
  bool decode(const uint8_t* p, size_t n, Headers* out, std::string* err);

 private:
  bool lookup(uint64_t index, Header* h) const;
  void insert(Header h);
  void evict();
  std::deque<Header> dyn_;  // newest first
  size_t size_ = 0, limit_, max_;
};

class Encoder {
 public:
  void encode(const Headers& h, std::string* out) const;
};

// Huffman code of RFC 7541 Appendix B (canonical; exposed for tests)
std::string huffman_encode(const std::string& s);
bool huffman_decode(const uint8_t* p, size_t n, std::string* out);

}  // namespace hpack
}  // namespace nnsx
