// Message transport for the among-device elements (tensor_query_*, edgesrc /
// edgesink).
//
// Reference behaviour: nnstreamer-edge carries a list of <=16 blobs plus
// string key/values (client_id, caps) per message (tensor_query_client.c:
// 673-690, edge_sink.c:305-345).  nnsx frames the same information as one
// length-prefixed message on a TCP stream:
//
//   u32 magic 'NNSX' | u32 version | u32 type | u32 nblobs
//   u64 client_id | u64 seq | i64 pts | i64 dts | i64 duration
//   u32 caps_len | u32 flags | u64 blob_size[nblobs] | caps bytes | blobs
//
// HBM-resident blobs are staged through pinned memory on send; receivers
// may upload into HBM (element `device` property).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "runtime/memory.h"

namespace nnsx {
namespace comm {

enum class MsgType : uint32_t { HELLO = 1, CAPS = 2, DATA = 3, EOS = 4, ERROR = 5, BYE = 6 };

struct Message {
  MsgType type = MsgType::DATA;
  uint64_t client_id = 0;
  uint64_t seq = 0;
  int64_t pts = -1, dts = -1, duration = -1;
  uint32_t flags = 0;
  std::string caps;
  std::vector<MemoryPtr> blobs;
};

class Connection {
 public:
  explicit Connection(int fd, std::string peer);
  ~Connection();
  // connect with retries until timeout_ms (0 = one attempt)
  static std::shared_ptr<Connection> connect(const std::string& host, int port, int timeout_ms, std::string* err);

  bool send(const Message& m);
  // returns false on timeout (timed_out = true) or on a closed/broken stream
  bool recv(Message* m, int timeout_ms, bool* timed_out = nullptr);
  void close();
  bool alive() const { return alive_.load(); }
  const std::string& peer() const { return peer_; }
  uint64_t id = 0;  // server-assigned client id

 private:
  bool write_all(const void* p, size_t n);
  bool read_all(void* p, size_t n, int timeout_ms, bool* timed_out);
  int fd_;
  std::string peer_;
  std::mutex send_mu_;
  std::atomic<bool> alive_{true};
};

class Listener {
 public:
  ~Listener();
  // bind + listen; port 0 picks an ephemeral port (see port())
  bool listen(const std::string& host, int port, std::string* err);
  // nullptr on timeout or after close()
  std::shared_ptr<Connection> accept(int timeout_ms);
  void close();
  int port() const { return port_; }

 private:
  int fd_ = -1;
  int port_ = 0;
  std::atomic<bool> closed_{false};
};

// Blocking FIFO of messages with flush support (the element unlock path).
class MessageQueue {
 public:
  void push(Message m);
  // false when flushing or on timeout (timeout_ms < 0 waits forever)
  bool pop(Message* m, int timeout_ms);
  void set_flushing(bool f);
  size_t size();

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Message> q_;
  bool flushing_ = false;
};

}  // namespace comm
}  // namespace nnsx
