// Native gRPC transport of tensor_src_grpc / tensor_sink_grpc: HTTP/2 over
// cleartext TCP ("h2c" with prior knowledge, RFC 9113) + HPACK (comm/hpack.h)
// + the gRPC length-prefixed message framing -- wire-compatible with grpc++
// (the reference, ext/nnstreamer/extra/nnstreamer_grpc_common.cc:83-200) and
// grpcio peers.  The service is the reference's TensorService:
//   /nnstreamer.<idl>.TensorService/SendTensors  client -> server stream,
//                                                  replies google.protobuf.Empty
//   /nnstreamer.<idl>.TensorService/RecvTensors  server -> client stream
// Roles (GrpcOptions): sink+client calls SendTensors, src+server serves it
// (messages from any client are queued), sink+server serves RecvTensors (every
// subscribed call receives each buffer), src+client calls RecvTensors.
//
// One reader thread per connection dispatches frames; writers hold the
// connection's write lock per frame and block on the peer's flow-control
// windows (connection + stream).  Received DATA is credited back right away
// (WINDOW_UPDATE per frame), so a peer is never stalled by us.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>

#include "comm/grpc_bridge.h"
#include "comm/hpack.h"
#include "core/log.h"

namespace nnsx {
namespace comm {
namespace {

enum FrameType : uint8_t { DATA = 0, HEADERS = 1, PRIORITY = 2, RST_STREAM = 3, SETTINGS = 4, PUSH_PROMISE = 5,
                           PING = 6, GOAWAY = 7, WINDOW_UPDATE = 8, CONTINUATION = 9 };
constexpr uint8_t F_END_STREAM = 0x1, F_ACK = 0x1, F_END_HEADERS = 0x4, F_PADDED = 0x8, F_PRIORITY = 0x20;
constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr size_t kPrefaceLen = 24;
constexpr uint32_t kOurMaxFrame = 1 << 20;  // what we accept (SETTINGS_MAX_FRAME_SIZE)
constexpr uint32_t kMaxHeaderList = 64 << 10;  // SETTINGS_MAX_HEADER_LIST_SIZE: a header block larger than this
                                               // (HEADERS + CONTINUATION) ends the connection
constexpr uint32_t kMaxStreams = 128;          // SETTINGS_MAX_CONCURRENT_STREAMS (peer-opened)
// google.protobuf.Empty / nnstreamer.flatbuf.Empty as serialized messages: protobuf
// encodes an empty message as 0 bytes; flatbuffers' builder emits a finished
// buffer for the empty root table (root uoffset 8, vtable {4, 4}, soffset 4),
// what CreateEmpty + Finish produce in the reference (nnstreamer_grpc_flatbuf.cc
// :269-276, :397-402) and what its verifier expects
const std::string kFlatbufEmpty("\x08\x00\x00\x00\x04\x00\x04\x00\x04\x00\x00\x00", 12);
constexpr int64_t kOurWindow = (1u << 30);  // stream + connection receive windows we advertise

bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    c += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

bool read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t r = ::recv(fd, c, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    c += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
void put32(std::string* s, uint32_t v) {
  for (int i = 3; i >= 0; --i) s->push_back(static_cast<char>((v >> (8 * i)) & 0xff));
}

std::string grpc_frame(const std::string& msg) {
  std::string f;
  f.reserve(msg.size() + 5);
  f.push_back(0);  // not compressed
  put32(&f, static_cast<uint32_t>(msg.size()));
  f.append(msg);
  return f;
}

const std::string* find_header(const hpack::Headers& h, const char* name) {
  for (const auto& kv : h)
    if (kv.first == name) return &kv.second;
  return nullptr;
}

// ------------------------------------------------------------------ H2Conn --
class H2Conn {
 public:
  struct Events {
    virtual ~Events() = default;
    virtual void on_headers(H2Conn* c, uint32_t sid, hpack::Headers&& h, bool end_stream) = 0;
    virtual void on_message(H2Conn* c, uint32_t sid, std::string&& msg) = 0;
    virtual void on_end(H2Conn* c, uint32_t sid) = 0;  // peer half-closed (END_STREAM) or reset
    virtual void on_closed(H2Conn* c) = 0;
    // a message whose gRPC length prefix exceeds the receive limit: its stream
    // no longer delivers data (the endpoint ends the call)
    virtual void on_oversize(H2Conn* c, uint32_t sid, uint64_t bytes) = 0;
  };

  H2Conn(int fd, bool server, Events* ev, int64_t max_msg)
      : fd_(fd), server_(server), ev_(ev), max_msg_(max_msg) {
    int one = 1;
    (void)setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  ~H2Conn() {
    close();
    if (reader_.joinable()) reader_.join();
    if (fd_ >= 0) ::close(fd_);
  }

  bool start() {
    std::string out;
    if (!server_) out.append(kPreface, kPrefaceLen);
    // our SETTINGS: no server push, large frames and windows, no dynamic HPACK
    // table limit change (the decoder keeps the default 4096)
    std::string s;
    auto setting = [&s](uint16_t id, uint32_t v) {
      s.push_back(static_cast<char>(id >> 8));
      s.push_back(static_cast<char>(id & 0xff));
      put32(&s, v);
    };
    setting(0x2, 0);  // ENABLE_PUSH
    setting(0x4, static_cast<uint32_t>(kOurWindow));  // INITIAL_WINDOW_SIZE
    setting(0x5, kOurMaxFrame);  // MAX_FRAME_SIZE
    setting(0x6, kMaxHeaderList);  // MAX_HEADER_LIST_SIZE
    if (server_) setting(0x3, kMaxStreams);  // MAX_CONCURRENT_STREAMS
    append_frame(&out, SETTINGS, 0, 0, s);
    std::string wu;
    put32(&wu, static_cast<uint32_t>(kOurWindow - 65535));
    append_frame(&out, WINDOW_UPDATE, 0, 0, wu);  // connection window
    {
      std::lock_guard<std::mutex> lk(wmu_);
      if (!write_all(fd_, out.data(), out.size())) return false;
    }
    reader_ = std::thread([this] { read_loop(); });
    return true;
  }

  void close() {
    if (closed_.exchange(true)) return;
    ::shutdown(fd_, SHUT_RDWR);
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_all();
  }
  bool alive() const { return !closed_.load(); }

  uint32_t open_stream() {
    std::lock_guard<std::mutex> lk(mu_);
    const uint32_t sid = next_sid_;
    next_sid_ += 2;
    streams_[sid].send_window = peer_init_window_;
    return sid;
  }

  bool send_headers(uint32_t sid, const hpack::Headers& h, bool end_stream) {
    std::string block;
    enc_.encode(h, &block);
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto& st = streams_[sid];
      if (!st.opened) {
        st.opened = true;
        st.send_window = peer_init_window_ + st.window_delta;
      }
    }
    std::string out;
    size_t off = 0;
    const size_t maxf = peer_max_frame_.load();
    bool first = true;
    do {
      const size_t n = std::min(maxf, block.size() - off);
      const bool last = off + n == block.size();
      uint8_t flags = last ? F_END_HEADERS : 0;
      if (first && end_stream) flags |= F_END_STREAM;
      append_frame(&out, first ? HEADERS : CONTINUATION, flags, sid, block.substr(off, n));
      off += n;
      first = false;
    } while (off < block.size());
    std::lock_guard<std::mutex> lk(wmu_);
    return !closed_.load() && write_all(fd_, out.data(), out.size());
  }

  // DATA within the peer's flow-control windows (blocks until credited)
  bool send_data(uint32_t sid, const std::string& payload, bool end_stream) {
    size_t off = 0;
    do {
      size_t n = 0;
      {
        std::unique_lock<std::mutex> lk(mu_);
        auto it = streams_.find(sid);
        if (it == streams_.end()) return false;
        const size_t want = payload.size() - off;
        if (want > 0) {
          cv_.wait(lk, [&] {
            auto s = streams_.find(sid);
            return closed_.load() || s == streams_.end() || s->second.reset ||
                   (conn_send_window_ > 0 && s->second.send_window > 0);
          });
          it = streams_.find(sid);
          if (closed_.load() || it == streams_.end() || it->second.reset) return false;
          n = std::min<size_t>({want, static_cast<size_t>(conn_send_window_),
                                static_cast<size_t>(it->second.send_window), peer_max_frame_.load()});
          conn_send_window_ -= static_cast<int64_t>(n);
          it->second.send_window -= static_cast<int64_t>(n);
        }
      }
      const bool last = off + n == payload.size();
      std::string out;
      append_frame(&out, DATA, (last && end_stream) ? F_END_STREAM : 0, sid, payload.substr(off, n));
      {
        std::lock_guard<std::mutex> lk(wmu_);
        if (closed_.load() || !write_all(fd_, out.data(), out.size())) return false;
      }
      off += n;
    } while (off < payload.size());
    return true;
  }

  bool send_message(uint32_t sid, const std::string& msg, bool end_stream) {
    return send_data(sid, grpc_frame(msg), end_stream);
  }

  void send_rst(uint32_t sid, uint32_t code) {
    std::string p, out;
    put32(&p, code);
    append_frame(&out, RST_STREAM, 0, sid, p);
    std::lock_guard<std::mutex> lk(wmu_);
    (void)write_all(fd_, out.data(), out.size());
  }

  void goaway(uint32_t code = 0) {
    std::string p, out;
    put32(&p, last_peer_sid_.load());
    put32(&p, code);  // NO_ERROR unless given
    append_frame(&out, GOAWAY, 0, 0, p);
    std::lock_guard<std::mutex> lk(wmu_);
    (void)write_all(fd_, out.data(), out.size());
  }

  void forget(uint32_t sid) {
    std::lock_guard<std::mutex> lk(mu_);
    streams_.erase(sid);
    cv_.notify_all();
  }
  bool is_reset(uint32_t sid) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = streams_.find(sid);
    return it != streams_.end() && it->second.reset;
  }
  size_t stream_count() {
    std::lock_guard<std::mutex> lk(mu_);
    return streams_.size();
  }

 private:
  struct Stream {
    int64_t send_window = 65535;
    int64_t window_delta = 0;  // SETTINGS changes before the stream opened on our side
    bool opened = false, reset = false;
    bool discard = false;  // an oversize message was refused: drop the rest of the stream's data
    std::string rx;  // gRPC message reassembly
  };

  static void append_frame(std::string* out, uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload) {
    const uint32_t n = static_cast<uint32_t>(payload.size());
    out->push_back(static_cast<char>((n >> 16) & 0xff));
    out->push_back(static_cast<char>((n >> 8) & 0xff));
    out->push_back(static_cast<char>(n & 0xff));
    out->push_back(static_cast<char>(type));
    out->push_back(static_cast<char>(flags));
    put32(out, sid & 0x7fffffffu);
    out->append(payload);
  }

  void write_frame(uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload) {
    std::string out;
    append_frame(&out, type, flags, sid, payload);
    std::lock_guard<std::mutex> lk(wmu_);
    if (!closed_.load()) (void)write_all(fd_, out.data(), out.size());
  }

  void credit(uint32_t sid, uint32_t n) {
    if (!n) return;
    std::string p;
    put32(&p, n);
    std::string out;
    append_frame(&out, WINDOW_UPDATE, 0, 0, p);
    if (sid) append_frame(&out, WINDOW_UPDATE, 0, sid, p);
    std::lock_guard<std::mutex> lk(wmu_);
    if (!closed_.load()) (void)write_all(fd_, out.data(), out.size());
  }

  void read_loop() {
    bool ok = true;
    if (server_) {
      char pre[kPrefaceLen];
      ok = read_all(fd_, pre, kPrefaceLen) && std::memcmp(pre, kPreface, kPrefaceLen) == 0;
      if (!ok) NNSX_LOGW("grpc", "connection without the HTTP/2 client preface (not an h2c gRPC client?)");
    }
    std::string block;  // header block being assembled
    uint32_t block_sid = 0;
    bool block_end_stream = false;
    std::vector<uint8_t> buf;
    while (ok && !closed_.load()) {
      uint8_t h[9];
      if (!read_all(fd_, h, 9)) break;
      const uint32_t len = (uint32_t(h[0]) << 16) | (uint32_t(h[1]) << 8) | h[2];
      const uint8_t type = h[3], flags = h[4];
      const uint32_t sid = be32(h + 5) & 0x7fffffffu;
      if (len > kOurMaxFrame) {
        NNSX_LOGW("grpc", "frame of ", len, " bytes exceeds MAX_FRAME_SIZE");
        break;
      }
      buf.resize(len);
      if (len && !read_all(fd_, buf.data(), len)) break;
      const uint8_t* p = buf.data();
      size_t n = len;
      // strip padding / priority fields
      if ((type == DATA || type == HEADERS) && (flags & F_PADDED)) {
        if (!n || p[0] >= n) break;
        const size_t pad = p[0];
        ++p;
        n -= 1 + pad;
      }
      if (type == HEADERS && (flags & F_PRIORITY)) {
        if (n < 5) break;
        p += 5;
        n -= 5;
      }
      switch (type) {
        case DATA: {
          bool end = (flags & F_END_STREAM) != 0;
          std::vector<std::string> msgs;
          uint64_t oversize = 0;
          bool known = false;
          {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = streams_.find(sid);
            // data for a stream that was never opened (or already ended): flow
            // control is still credited, nothing is buffered
            known = it != streams_.end() && !it->second.reset;
            if (known && !it->second.discard) {
              Stream& st = it->second;
              st.rx.append(reinterpret_cast<const char*>(p), n);
              size_t off = 0;
              while (st.rx.size() - off >= 5) {
                const uint32_t ml = be32(reinterpret_cast<const uint8_t*>(st.rx.data()) + off + 1);
                if (max_msg_ >= 0 && ml > static_cast<uint64_t>(max_msg_)) {  // refused before buffering it
                  oversize = ml;
                  st.discard = true;
                  st.rx.clear();
                  off = 0;
                  break;
                }
                if (st.rx.size() - off - 5 < ml) break;
                if (st.rx[off] != 0) NNSX_LOGW("grpc", "compressed gRPC message (no codec negotiated) passed through");
                msgs.emplace_back(st.rx.substr(off + 5, ml));
                off += 5 + ml;
              }
              st.rx.erase(0, off);
            }
          }
          credit(known ? sid : 0, len);
          for (auto& m : msgs) ev_->on_message(this, sid, std::move(m));
          if (oversize) ev_->on_oversize(this, sid, oversize);
          if (known && end) ev_->on_end(this, sid);
          break;
        }
        case HEADERS:
        case CONTINUATION: {
          if (type == HEADERS) {
            block.clear();
            block_sid = sid;
            block_end_stream = (flags & F_END_STREAM) != 0;
            if (server_) {
              uint32_t prev = last_peer_sid_.load();
              if (sid > prev) last_peer_sid_.store(sid);
            }
          } else if (sid != block_sid) {
            ok = false;
            break;
          }
          if (block.size() + n > kMaxHeaderList) {  // unbounded CONTINUATION chains end here
            NNSX_LOGW("grpc", "header block above ", kMaxHeaderList, " bytes: closing the connection");
            goaway(0xb);  // ENHANCE_YOUR_CALM
            ok = false;
            break;
          }
          block.append(reinterpret_cast<const char*>(p), n);
          if (flags & F_END_HEADERS) {
            hpack::Headers hs;
            std::string err;
            if (!dec_.decode(reinterpret_cast<const uint8_t*>(block.data()), block.size(), &hs, &err)) {
              NNSX_LOGW("grpc", err);
              ok = false;
              break;
            }
            bool refuse = false, fresh = false;
            {
              std::lock_guard<std::mutex> lk(mu_);
              fresh = streams_.find(block_sid) == streams_.end();
              if (fresh && server_ && streams_.size() >= kMaxStreams) {
                refuse = true;
              } else {
                auto& st = streams_[block_sid];
                if (!st.opened) {
                  st.opened = true;
                  st.send_window = peer_init_window_ + st.window_delta;
                }
              }
            }
            if (refuse) {
              send_rst(block_sid, 0x7);  // REFUSED_STREAM
              break;
            }
            ev_->on_headers(this, block_sid, std::move(hs), block_end_stream);
            if (block_end_stream) ev_->on_end(this, block_sid);
          }
          break;
        }
        case SETTINGS: {
          if (flags & F_ACK) break;
          for (size_t i = 0; i + 6 <= n; i += 6) {
            const uint16_t id = static_cast<uint16_t>((p[i] << 8) | p[i + 1]);
            const uint32_t v = be32(p + i + 2);
            if (id == 0x4) {  // INITIAL_WINDOW_SIZE: applies to every stream window (6.9.2)
              std::lock_guard<std::mutex> lk(mu_);
              const int64_t delta = static_cast<int64_t>(v) - peer_init_window_;
              peer_init_window_ = v;
              for (auto& kv : streams_) {
                if (kv.second.opened) kv.second.send_window += delta;
              }
              cv_.notify_all();
            } else if (id == 0x5) {
              peer_max_frame_.store(std::max<uint32_t>(16384, std::min<uint32_t>(v, 1u << 24)));
            }
          }
          write_frame(SETTINGS, F_ACK, 0, "");
          break;
        }
        case PING:
          if (!(flags & F_ACK) && n == 8) write_frame(PING, F_ACK, 0, std::string(reinterpret_cast<const char*>(p), 8));
          break;
        case WINDOW_UPDATE: {
          if (n < 4) break;
          const uint32_t inc = be32(p) & 0x7fffffffu;
          std::lock_guard<std::mutex> lk(mu_);
          if (sid == 0) {
            conn_send_window_ += inc;
          } else {
            auto it = streams_.find(sid);  // (never opened / already ended: ignored)
            if (it != streams_.end()) {
              if (it->second.opened) it->second.send_window += inc;
              else it->second.window_delta += inc;
            }
          }
          cv_.notify_all();
          break;
        }
        case RST_STREAM: {
          bool known;
          {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = streams_.find(sid);
            known = it != streams_.end();
            if (known) it->second.reset = true;  // erased by the endpoint (forget) once it is done with it
            cv_.notify_all();
          }
          if (known) ev_->on_end(this, sid);
          break;
        }
        case GOAWAY:
          ok = false;
          break;
        default:
          break;  // PRIORITY, PUSH_PROMISE (disabled), unknown types: ignored
      }
    }
    close();
    ev_->on_closed(this);
  }

  int fd_;
  bool server_;
  Events* ev_;
  int64_t max_msg_;
  std::thread reader_;
  std::mutex wmu_;  // frame writes
  std::mutex mu_;   // streams + windows
  std::condition_variable cv_;
  std::map<uint32_t, Stream> streams_;
  int64_t conn_send_window_ = 65535;
  int64_t peer_init_window_ = 65535;
  std::atomic<size_t> peer_max_frame_{16384};
  uint32_t next_sid_ = 1;
  std::atomic<uint32_t> last_peer_sid_{0};
  std::atomic<bool> closed_{false};
  hpack::Decoder dec_;
  hpack::Encoder enc_;
};

// --------------------------------------------------------------- endpoint --
constexpr int kUnimplemented = 12;

class NativeGrpcEndpoint : public GrpcEndpoint, public H2Conn::Events {
 public:
  explicit NativeGrpcEndpoint(const GrpcOptions& o) : o_(o) {
    std::string idl = o.idl;
    for (auto& c : idl) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    service_ = "/nnstreamer." + idl + ".TensorService/";
    empty_ = idl == "flatbuf" ? kFlatbufEmpty : std::string();
  }
  ~NativeGrpcEndpoint() override { stop(); }

  bool start(std::string* err) override { return o_.server ? start_server(err) : start_client(err); }

  bool send(const std::string& msg) override {
    if (stopped_.load()) return false;
    if (o_.server) {
      std::vector<std::pair<std::shared_ptr<H2Conn>, uint32_t>> subs;
      {
        std::lock_guard<std::mutex> lk(mu_);
        subs = subs_;
      }
      for (auto& s : subs)
        if (!s.first->send_message(s.second, msg, false)) drop_sub(s.first.get(), s.second);
      return true;
    }
    if (failed_.load() || !conn_ || !conn_->alive()) return false;
    return conn_->send_message(sid_, msg, false);
  }

  int recv(std::string* msg, int timeout_ms) override {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait_for(lk, std::chrono::milliseconds(std::max(0, timeout_ms)),
                 [&] { return !q_.empty() || stopped_.load() || finished_; });
    if (!q_.empty()) {
      *msg = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      cv_.notify_all();  // room in the queue
      return 1;
    }
    return (stopped_.load() || finished_) ? -1 : 0;
  }

  void stop() override {
    if (stopped_.exchange(true)) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      cv_.notify_all();
    }
    if (o_.server) {
      listening_.store(false);
      if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
      if (acceptor_.joinable()) acceptor_.join();
      if (lfd_ >= 0) ::close(lfd_);
      lfd_ = -1;
      std::vector<std::pair<std::shared_ptr<H2Conn>, uint32_t>> subs;
      std::vector<std::shared_ptr<H2Conn>> conns;
      {
        std::lock_guard<std::mutex> lk(mu_);
        subs.swap(subs_);
        conns = conns_;
      }
      for (auto& s : subs) finish_call(s.first.get(), s.second, 0, "");  // RecvTensors streams end OK
      for (auto& c : conns) c->goaway();
      for (auto& c : conns) c->close();
      {
        std::lock_guard<std::mutex> lk(mu_);
        conns.insert(conns.end(), conns_.begin(), conns_.end());
        conns_.clear();
        dead_.clear();
      }
      // destroyed here, outside mu_: each destructor joins a reader that may be
      // waiting for mu_ in on_closed()
      subs.clear();
      conns.clear();
      return;
    }
    if (conn_) {
      if (o_.sending && !failed_.load() && conn_->alive()) {
        // half-close the SendTensors call and wait for the server's status
        conn_->send_data(sid_, "", true);
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait_for(lk, std::chrono::seconds(10), [&] { return finished_ || !conn_->alive(); });
      }
      conn_->close();
      conn_.reset();
    }
  }

  int port() override { return bound_port_; }

  // ---- H2Conn::Events
  void on_headers(H2Conn* c, uint32_t sid, hpack::Headers&& h, bool end_stream) override {
    if (!o_.server) {
      // response headers / trailers of our call: a non-OK grpc-status fails it
      const std::string* st = find_header(h, "grpc-status");
      if (st && *st != "0") {
        const std::string* m = find_header(h, "grpc-message");
        NNSX_LOGW("grpc", "call failed: grpc-status ", *st, m ? " (" + *m + ")" : std::string());
        failed_.store(true);
      }
      (void)end_stream;
      return;
    }
    const std::string* path = find_header(h, ":path");
    const std::string method = path && path->compare(0, service_.size(), service_) == 0 ? path->substr(service_.size())
                                                                                        : std::string();
    if (method == "SendTensors" && !o_.sending) {
      std::lock_guard<std::mutex> lk(mu_);
      calls_[{c, sid}] = Call::SEND;
      return;
    }
    if (method == "RecvTensors" && o_.sending) {
      if (!c->send_headers(sid, response_headers(), false)) return;
      std::lock_guard<std::mutex> lk(mu_);
      calls_[{c, sid}] = Call::RECV;
      subs_.emplace_back(find_conn(c), sid);
      return;
    }
    // not served by this endpoint: trailers-only UNIMPLEMENTED
    hpack::Headers t = response_headers();
    t.emplace_back("grpc-status", std::to_string(kUnimplemented));
    t.emplace_back("grpc-message", "method not served by this tensor_" + std::string(o_.sending ? "sink" : "src") +
                                       "_grpc: " + (path ? *path : std::string("?")));
    c->send_headers(sid, t, true);
    c->forget(sid);
  }

  void on_oversize(H2Conn* c, uint32_t sid, uint64_t bytes) override {
    const std::string msg = "Received message larger than max (" + std::to_string(bytes) + " vs. " +
                            std::to_string(o_.max_recv_bytes) + ")";
    NNSX_LOGW("grpc", msg);
    if (!o_.server) {  // our call's incoming stream: give up on it
      failed_.store(true);
      c->send_rst(sid, 0x8);  // CANCEL
      std::lock_guard<std::mutex> lk(mu_);
      finished_ = true;
      cv_.notify_all();
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      calls_.erase({c, sid});
    }
    hpack::Headers t = response_headers();
    t.emplace_back("grpc-status", "8");  // RESOURCE_EXHAUSTED
    t.emplace_back("grpc-message", msg);
    c->send_headers(sid, t, true);
    c->send_rst(sid, 0x0);  // NO_ERROR: the rest of the request is not read
    c->forget(sid);
  }

  void on_message(H2Conn* c, uint32_t sid, std::string&& m) override {
    std::unique_lock<std::mutex> lk(mu_);
    if (o_.server) {
      auto it = calls_.find({c, sid});
      if (it == calls_.end() || it->second != Call::SEND) return;  // RecvTensors' Empty request
    } else if (o_.sending) {
      return;  // SendTensors' Empty reply
    }
    // bounded queue: the reader (and so the peer, through flow control) waits
    cv_.wait(lk, [&] { return q_.size() < 64 || stopped_.load(); });
    if (stopped_.load()) return;
    q_.push_back(std::move(m));
    cv_.notify_all();
  }

  void on_end(H2Conn* c, uint32_t sid) override {
    if (!o_.server) {
      std::lock_guard<std::mutex> lk(mu_);
      if (sid == sid_) finished_ = true;
      cv_.notify_all();
      return;
    }
    Call kind;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = calls_.find({c, sid});
      if (it == calls_.end()) return;
      kind = it->second;
      if (kind == Call::SEND) calls_.erase(it);
    }
    if (kind == Call::SEND) {
      // client finished its stream: reply Empty (per IDL) + OK status
      if (c->send_headers(sid, response_headers(), false) && c->send_message(sid, empty_, false)) {
        hpack::Headers t{{"grpc-status", "0"}};
        c->send_headers(sid, t, true);
      }
      c->forget(sid);
      return;
    }
    // RecvTensors: the client half-closed after its request; keep streaming
    // unless it reset the stream
    if (c->is_reset(sid)) {
      drop_sub(c, sid);
      {
        std::lock_guard<std::mutex> lk(mu_);
        calls_.erase({c, sid});
      }
      c->forget(sid);
    }
  }

  void on_closed(H2Conn* c) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (!o_.server) {
      finished_ = true;
      cv_.notify_all();
      return;
    }
    for (auto it = subs_.begin(); it != subs_.end();)
      it = it->first.get() == c ? subs_.erase(it) : it + 1;
    for (auto it = calls_.begin(); it != calls_.end();)
      it = it->first.first == c ? calls_.erase(it) : std::next(it);
    dead_.push_back(c);
  }

 private:
  enum class Call { SEND, RECV };

  hpack::Headers response_headers() const { return {{":status", "200"}, {"content-type", "application/grpc"}}; }

  std::shared_ptr<H2Conn> find_conn(H2Conn* c) {
    for (auto& x : conns_)
      if (x.get() == c) return x;
    return nullptr;
  }

  void drop_sub(H2Conn* c, uint32_t sid) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = subs_.begin(); it != subs_.end(); ++it)
      if (it->first.get() == c && it->second == sid) {
        subs_.erase(it);
        break;
      }
    calls_.erase({c, sid});
  }

  void finish_call(H2Conn* c, uint32_t sid, int status, const std::string& msg) {
    hpack::Headers t{{"grpc-status", std::to_string(status)}};
    if (!msg.empty()) t.emplace_back("grpc-message", msg);
    c->send_headers(sid, t, true);
    c->forget(sid);
  }

  bool start_server(std::string* err) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    const std::string host = o_.host.empty() ? std::string("0.0.0.0") : o_.host;
    const std::string port = std::to_string(o_.port);
    if (getaddrinfo(host == "localhost" ? "127.0.0.1" : host.c_str(), port.c_str(), &hints, &res) != 0 || !res) {
      *err = "cannot resolve " + host;
      return false;
    }
    int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
    int one = 1;
    (void)setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (fd < 0 || ::bind(fd, res->ai_addr, res->ai_addrlen) != 0 || ::listen(fd, 16) != 0) {
      *err = "cannot bind " + host + ":" + port + ": " + std::strerror(errno);
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
      return false;
    }
    freeaddrinfo(res);
    sockaddr_storage ss{};
    socklen_t sl = sizeof(ss);
    if (getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl) == 0)
      bound_port_ = ntohs(ss.ss_family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port
                                                   : reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    lfd_ = fd;
    listening_.store(true);
    acceptor_ = std::thread([this] { accept_loop(); });
    return true;
  }

  void accept_loop() {
    while (listening_.load()) {
      pollfd pf{lfd_, POLLIN, 0};
      const int r = ::poll(&pf, 1, 100);
      reap();
      if (r <= 0 || !(pf.revents & POLLIN)) continue;
      const int cfd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (cfd < 0) continue;
      auto conn = std::make_shared<H2Conn>(cfd, true, this, o_.max_recv_bytes);
      {
        std::lock_guard<std::mutex> lk(mu_);
        conns_.push_back(conn);
      }
      if (!conn->start()) conn->close();
    }
  }

  // connections whose reader ended: dropped outside their own reader thread
  void reap() {
    std::vector<std::shared_ptr<H2Conn>> gone;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (H2Conn* d : dead_)
        for (auto it = conns_.begin(); it != conns_.end(); ++it)
          if (it->get() == d) {
            gone.push_back(*it);
            conns_.erase(it);
            break;
          }
      dead_.clear();
    }
    gone.clear();  // joins the finished readers
  }

  bool start_client(std::string* err) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    const std::string host = o_.host.empty() ? std::string("localhost") : o_.host;
    const std::string port = std::to_string(o_.port);
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) {
      *err = "cannot resolve " + host;
      return false;
    }
    int fd = -1;
    for (addrinfo* a = res; a; a = a->ai_next) {
      fd = ::socket(a->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (fd >= 0 && ::connect(fd, a->ai_addr, a->ai_addrlen) == 0) break;
      if (fd >= 0) ::close(fd);
      fd = -1;
    }
    freeaddrinfo(res);
    if (fd < 0) {
      *err = "cannot connect to " + host + ":" + port;
      return false;
    }
    conn_ = std::make_shared<H2Conn>(fd, false, this, o_.max_recv_bytes);
    if (!conn_->start()) {
      *err = "HTTP/2 handshake failed";
      return false;
    }
    sid_ = conn_->open_stream();
    hpack::Headers h{{":method", "POST"},
                     {":scheme", "http"},
                     {":path", service_ + (o_.sending ? "SendTensors" : "RecvTensors")},
                     {":authority", host + ":" + port},
                     {"content-type", "application/grpc"},
                     {"te", "trailers"},
                     {"user-agent", "nnstreamer-amd-grpc/1"}};
    if (!conn_->send_headers(sid_, h, false)) {
      *err = "cannot open the call";
      return false;
    }
    // RecvTensors: the Empty request (per IDL), then half-close
    if (!o_.sending && !conn_->send_message(sid_, empty_, true)) {
      *err = "cannot send the RecvTensors request";
      return false;
    }
    return true;
  }

  GrpcOptions o_;
  std::string service_;
  std::string empty_;  // the IDL's serialized Empty message
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> q_;
  std::atomic<bool> stopped_{false}, failed_{false}, listening_{false};
  bool finished_ = false;
  // server
  int lfd_ = -1, bound_port_ = 0;
  std::thread acceptor_;
  std::vector<std::shared_ptr<H2Conn>> conns_;
  std::vector<H2Conn*> dead_;
  std::vector<std::pair<std::shared_ptr<H2Conn>, uint32_t>> subs_;
  std::map<std::pair<H2Conn*, uint32_t>, Call> calls_;
  // client
  std::shared_ptr<H2Conn> conn_;
  uint32_t sid_ = 1;
};

}  // namespace

std::shared_ptr<GrpcEndpoint> make_native_grpc_endpoint(const GrpcOptions& o) {
  return std::make_shared<NativeGrpcEndpoint>(o);
}

}  // namespace comm
}  // namespace nnsx
