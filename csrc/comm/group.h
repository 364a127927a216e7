// Rank groups: the intra-node multi-GPU data plane (RCCL over xGMI) plus the
// host control plane (a TCP key/value store) that every among-GPU element
// uses -- one process per GPU, exactly like torch.distributed.
//
// The reference has no collectives at all: tensors
// leave a process only through nnstreamer-edge / MQTT / gRPC sockets
// (tensor_query_client.c:673-700, edge_sink.c:305-345).  nnsx keeps those
// element semantics and maps them onto collectives when the peers are GPUs
// of the same node:
//
//   pub/sub 1->N (edgesink/edgesrc)        -> ncclBroadcast(root = publisher)
//   demux 1->N   (edgesink mode=scatter)   -> grouped ncclSend / ncclRecv
//   N-source mux (tensor_allgather)        -> ncclAllGather (equal sizes) or
//                                              grouped ncclBroadcast per root
//   request/reply (tensor_query_*)         -> ncclSend / ncclRecv pairs
//
// Rendezvous: a small key/value store hosted by the group's first member
// (TCPStore analogue: set / blocking get / add; a key written with
// `readers = n` is erased after n gets) -- used to join, to exchange the RCCL
// unique id and the members' link addresses, and for element handshakes.
// Per-message headers (pts, caps, blob sizes, flexible meta, EOS) travel on
// direct member-to-member TCP links (Mesh): one message, no store round trip.
// Payloads travel on the group's RCCL communicator and its own high-priority
// HIP stream, ordered against producers / consumers with the Memory ready /
// use events -- never a host sync on the data path.
//
// Without GPUs (or backend=tcp) the payload rides on the same direct link
// behind its header (host bytes), so the same elements and tests run on
// CPU-only boxes.
//
// Point-to-point payloads ride on per-direction links: for each ordered pair
// (sender -> receiver) a two-rank RCCL communicator with its own stream on
// both sides, all created when the group opens (pairs in lexicographic order,
// so the creation itself cannot deadlock and no send waits for its peer to
// reach recv()).  A send kernel then waits
// only for receives of the SAME direction, which its own earlier sends
// already matched, so no cycle of GPU waits can form -- a ring or a
// bidirectional exchange of frame-sized messages cannot deadlock the way one
// shared comm stream does (each rank's send kernel queued ahead of the
// receive its peer's send waits for).  Collectives keep the group
// communicator and stream.
//
// Threading rule: collectives are driven by one thread at a time (RCCL
// communicators are not thread-safe); send() and recv() use disjoint links
// and may run on two threads (one sender, one receiver).
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "comm/transport.h"
#include "runtime/memory.h"

namespace nnsx {
namespace comm {

// ------------------------------------------------------------ store ----
class StoreClient {
 public:
  static std::shared_ptr<StoreClient> connect(const std::string& host, int port, int timeout_ms, std::string* err);
  // readers > 0: the key is erased after that many successful get()s
  bool set(const std::string& key, const std::string& val, int readers = 0);
  // false on timeout / lost connection
  // timed_out: set when the server's wait expired (false on a lost connection)
  bool get(const std::string& key, std::string* val, int timeout_ms, bool* timed_out = nullptr);
  // atomic add on a decimal counter (missing = 0); returns the new value, INT64_MIN on error
  int64_t add(const std::string& key, int64_t delta);
  bool del(const std::string& key);
  void close();
  std::string local_ip() const;  // this process's address on the store's network

 private:
  bool call(const std::string& op, const std::string& key, const std::string* val, int64_t arg, int wait_ms,
            std::string* out, int64_t* iout, int* status = nullptr);
  std::shared_ptr<Connection> conn_;
  std::mutex mu_;
};

// Host a store server on host:port inside this process (refcounted: several
// groups may share it).  Returns a handle that keeps it alive, or nullptr
// with *in_use=true when another process already listens there.
std::shared_ptr<void> host_store(const std::string& host, int port, bool* in_use, std::string* err);

// ------------------------------------------------------------- mesh ----
// Direct member-to-member links of a group: every member listens on an
// ephemeral port (address published once in the store), a sender connects to
// a receiver on first use and keeps the connection.  One message = one
// transport Message (comm/transport.h) carrying a tag (p2p or the collective
// sequence), the encoded packet header and -- on the tcp backend -- the payload
// blobs.  An acceptor thread and one reader thread per inbound connection fill
// a single inbox that receives match by (tag, source).
class Mesh {
 public:
  ~Mesh();
  bool start(StoreClient* store, const std::string& prefix, int grank, int n, int timeout_ms, std::string* err);
  bool send(int peer, uint64_t tag, Message m, std::string* err);
  void deliver_local(uint64_t tag, Message m);  // a member's message to itself
  // next message with this tag from `src` (-1: any member), FIFO per source.
  // false: *timed_out on timeout, else the mesh is closed or the awaited
  // member's link broke without its goodbye (*err says which)
  bool recv(uint64_t tag, int src, Message* m, int* from, int timeout_ms, bool* timed_out, std::string* err);
  void close();

 private:
  struct Item {
    int src;
    uint64_t tag;
    Message m;
  };
  void reader(std::shared_ptr<Connection> c);
  StoreClient* store_ = nullptr;
  std::string prefix_;
  int grank_ = 0, n_ = 1, timeout_ms_ = 60000;
  Listener lis_;
  std::thread acceptor_;
  std::vector<std::thread> readers_;
  std::vector<std::shared_ptr<Connection>> in_, out_;
  std::vector<std::mutex> out_mu_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> inbox_;
  std::vector<int> lost_;  // per member: 1 = its link broke without a goodbye, 2 = that was reported
  std::atomic<bool> closed_{false};
};

// ------------------------------------------------------------ group ----
struct GroupSpec {
  std::string name;            // channel name (same on every member)
  int rank = -1;               // global rank (-1: $RANK or 0)
  int world = -1;              // global world size (-1: $WORLD_SIZE or 1)
  std::vector<int> members;    // global ranks in the group (empty: all)
  std::string store;           // "host:port" ("": ini [rccl] store, $NNSX_STORE, else $MASTER_ADDR:$MASTER_PORT+17)
  int device = -1;             // GPU of this member (-1: host only)
  std::string backend = "auto";  // auto | rccl | tcp ("auto": ini [rccl] backend, default auto)
  int timeout_ms = 0;          // rendezvous timeout (0: ini [rccl] timeout_ms, default 60000)
};

// One message: what an element hands to / gets from the group.
struct Packet {
  int src = -1;  // group rank of the sender (filled on receive)
  int64_t pts = -1, dts = -1, duration = -1;
  uint64_t client_id = 0;
  uint32_t flags = 0;
  bool eos = false;
  std::string caps;  // optional caps string riding with the header
  std::vector<MemoryPtr> blobs;
};

class Group {
 public:
  ~Group();
  static std::shared_ptr<Group> open(const GroupSpec& spec, std::string* err);

  int rank() const { return grank_; }
  int size() const { return static_cast<int>(members_.size()); }
  int global_rank(int group_rank) const { return members_.at(static_cast<size_t>(group_rank)); }
  int device() const { return device_; }
  bool rccl() const { return comm_ != nullptr; }
  const char* backend_name() const { return comm_ ? "rccl" : "tcp"; }
  hipStream_t stream() const { return stream_; }
  const std::string& name() const { return spec_.name; }

  // ---- collectives: every member calls them in the same order ----
  // all[r] = member r's packet (own packet is passed through).  stacked
  // (optional): when every member sends exactly one blob of the same size,
  // the n*size buffer holding them in member order (one ncclAllGather output,
  // no extra copy); nullptr otherwise.
  bool allgather(const Packet& mine, std::vector<Packet>* all, std::string* err, MemoryPtr* stacked = nullptr);
  // root: *pkt is sent; others: *pkt receives it
  bool broadcast(int root, Packet* pkt, std::string* err);
  // root: parts[r] goes to member r (parts[root] stays local); others receive their part
  bool scatter(int root, const std::vector<Packet>* parts, Packet* mine, std::string* err);

  // ---- point to point (FIFO per sender -> receiver) ----
  bool send(int peer, const Packet& p, std::string* err);
  // from any member; false + *timed_out on timeout
  bool recv(Packet* p, int timeout_ms, bool* timed_out, std::string* err);

  // ---- control-plane access for element handshakes (keys are group-scoped) ----
  bool put(const std::string& key, const std::string& val, int readers = 0);
  bool get(const std::string& key, std::string* val, int timeout_ms);

  // abort blocking control-plane waits (element unlock / shutdown)
  void cancel();

  // bytes moved on the data plane (stats / tests)
  uint64_t bytes_sent() const { return bytes_sent_; }
  uint64_t bytes_received() const { return bytes_recv_; }

 private:
  Group() = default;
  bool init(const GroupSpec& spec, std::string* err);
  std::string key(const std::string& k) const { return prefix_ + "/" + k; }
  std::string encode(const Packet& p, bool inline_payload);
  bool decode(const std::string& s, Packet* p, bool inline_payload, std::vector<size_t>* sizes,
              std::vector<std::string>* metas);
  // device pointer of a blob for the data plane (uploads host blobs)
  void* dev_ptr(const MemoryPtr& m);
  std::vector<MemoryPtr> alloc_recv(const std::vector<size_t>& sizes, const std::vector<std::string>& metas);
  Message to_message(const Packet& p);
  bool from_message(Message&& m, Packet* p, std::vector<size_t>* sizes, std::vector<std::string>* metas);
  bool recv_from(uint64_t tag, int src, Packet* p, std::vector<size_t>* sizes, std::vector<std::string>* metas,
                 std::string* err, const char* what);
  void finish_inputs(const std::vector<MemoryPtr>& in, hipStream_t s = nullptr);
  void* dev_ptr_on(const MemoryPtr& m, hipStream_t s);
  // per-direction p2p links (see the header comment): the link carrying this
  // member's messages to `peer` (tx) or `peer`'s messages to this member (rx)
  struct Link {
    void* comm = nullptr;  // ncclComm_t of the two-rank pair (sender = rank 0)
    hipStream_t stream = nullptr;
  };
  bool link(int peer, bool tx, Link** out, std::string* err);
  // a group of one on forced RCCL: the blobs copied through a grouped
  // ncclSend / ncclRecv to itself (the data plane's p2p kernels, on one GPU)
  bool self_copy(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, std::string* err);

  GroupSpec spec_;
  std::vector<int> members_;
  int grank_ = 0;
  int device_ = -1;
  std::string prefix_;
  std::shared_ptr<void> store_host_;
  std::shared_ptr<StoreClient> store_;
  std::unique_ptr<Mesh> mesh_;  // member-to-member links (headers; tcp payloads)
  void* comm_ = nullptr;  // ncclComm_t
  hipStream_t stream_ = nullptr;
  std::vector<Link> tx_, rx_;  // per peer (group rank): send side / receive side
  uint64_t seq_ = 0;            // collective sequence
  std::deque<Message> local_;   // a group of one: its messages to itself
  std::mutex local_mu_;
  std::condition_variable local_cv_;
  std::atomic<bool> cancelled_{false};
  uint64_t bytes_sent_ = 0, bytes_recv_ = 0;
};

// Process-wide cache so elements of one pipeline share a channel by name.
// (opened outside the cache lock: opening waits for the other members)
std::shared_ptr<Group> group_get(const GroupSpec& spec, std::string* err);

}  // namespace comm
}  // namespace nnsx
