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
//
// Device-direct path (connect-type=HIPIPC, same host): each sending end owns
// a hipMalloc'd staging ring in HBM exported once with hipIpcGetMemHandle.
// A device blob is copied D2D (or peer, over xGMI) into a ring slot and only
// {offset, size} travels on the socket; the receiver maps the ring once
// (hipIpcOpenMemHandle, lazily peer-enabled) and hands the slot downstream
// zero-copy as a device Memory whose release sends IPC_ACK back, which frees
// the slot.  Both ends announce the capability (IPC_HELLO with the kernel
// boot id, so a cross-host peer never tries), and a full ring falls back to
// the TCP byte path for that blob instead of blocking.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "runtime/memory.h"

namespace nnsx {
namespace comm {

enum class MsgType : uint32_t {
  HELLO = 1, CAPS = 2, DATA = 3, EOS = 4, ERROR = 5, BYE = 6,
  IPC_HELLO = 7,  // caps: "boot=<id>;pid=<n>" -- the sender can receive ring blobs
  IPC_RING = 8,   // caps: ring description (handle, size, PCI bus id); precedes its first use
  IPC_ACK = 9,    // seq = ring offset, duration = bytes: the receiver released a slot
  SHM_HELLO = 10,  // caps: "boot=<id>": the sender maps shared-memory segments of this host
  SHM_SEG = 11,    // caps: "id=<n>;name=<shm path>;size=<bytes>": a segment, before its first blob
  SHM_ACK = 12,    // seq = blob reference: the receiver released a shared-memory blob
};

struct IpcRing;      // transport.cc
struct PeerRing;     // transport.cc

struct Message {
  MsgType type = MsgType::DATA;
  uint64_t client_id = 0;
  uint64_t seq = 0;
  int64_t pts = -1, dts = -1, duration = -1;
  uint32_t flags = 0;
  std::string caps;
  std::vector<MemoryPtr> blobs;
};

class Connection;
std::shared_ptr<Connection> make_connection(int fd, std::string peer);

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
  // wakes a recv() blocked in another thread (shutdown only: that thread still
  // owns the descriptor, which the destructor closes)
  void shutdown();
  bool alive() const { return alive_.load(); }
  const std::string& peer() const { return peer_; }
  std::string local_ip() const;  // this end's IPv4 address (what peers can reach us at)
  uint64_t id = 0;  // server-assigned client id

  // device-direct path: announce that this end takes ring blobs (and will
  // export its own ring, sized `ring_bytes`, when it first sends a device blob)
  bool send_ipc_hello(size_t ring_bytes = 0);
  // the peer announced IPC and lives on this host: device blobs go through the ring
  bool peer_ipc() const { return peer_ipc_.load(); }
  // blobs sent through the ring / inline since the connection opened (tests, stats)
  uint64_t ipc_blobs_sent() const { return ipc_sent_.load(); }
  uint64_t ipc_blobs_received() const { return ipc_recv_.load(); }

  // same-host shared memory (connect-type=SHM): announce that this end maps the
  // peer's POSIX shared-memory segments (comm/shm.h).  The peer then sends a
  // host blob that lies in one of its segments as a reference (segment, offset)
  // instead of its bytes and holds the blob until this end releases it
  bool send_shm_hello();
  bool peer_shm() const { return peer_shm_.load(); }
  uint64_t shm_blobs_sent() const { return shm_sent_.load(); }
  uint64_t shm_blobs_received() const { return shm_recv_.load(); }

 private:
  bool send_locked(const Message& m, const std::vector<uint64_t>* offsets, bool shm = false);
  bool handle_control(const Message& m);  // IPC_* messages, consumed inside recv()
  void send_ack(uint64_t off, uint64_t bytes);
  std::weak_ptr<Connection> self_;  // for the ACK-on-release closures
  friend std::shared_ptr<Connection> make_connection(int fd, std::string peer);
  std::atomic<bool> peer_ipc_{false}, hello_sent_{false}, peer_shm_{false};
  std::atomic<uint64_t> shm_sent_{0}, shm_recv_{0};
  std::mutex shm_mu_;
  std::map<std::string, uint32_t> shm_ids_;              // sender: our segments announced to the peer
  std::multimap<uint64_t, MemoryPtr> shm_held_;          // sender: blobs the peer still reads
  std::map<uint32_t, std::shared_ptr<void>> shm_peer_;   // receiver: the peer's segments, mapped
  std::atomic<uint64_t> ipc_sent_{0}, ipc_recv_{0};
  size_t ring_bytes_ = 0;
  std::shared_ptr<IpcRing> ring_;      // ours (sending side)
  std::shared_ptr<PeerRing> peer_ring_;  // theirs, mapped (receiving side)

  bool write_all(const void* p, size_t n);
  bool read_all(void* p, size_t n, int timeout_ms, bool* timed_out);
  int fd_;
  std::string peer_;
  std::mutex send_mu_, ipc_mu_;
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
  void release();     // ::close the socket (no accept() may still be running)
  std::atomic<int> fd_{-1};
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
