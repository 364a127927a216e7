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
//   demux 1->N   (edgesink mode=scatter)   -> ncclSend / ncclRecv
//   N-source mux (tensor_allgather)        -> ncclAllGather (equal sizes) or
//                                              grouped ncclBroadcast per root
//   request/reply (tensor_query_*)         -> ncclSend / ncclRecv pairs
//
// Rendezvous: a small key/value store hosted by the group's first member
// (TCPStore analogue: set / blocking get / add; a key written with
// `readers = n` is erased after n gets) -- used to join, to exchange the RCCL
// unique id and the members' link addresses, and for element handshakes.
//
// ---- Rounds: why the data plane cannot deadlock ----
// Every operation of a group -- collectives AND point-to-point messages --
// is executed by ONE progress thread per member, in numbered ROUNDS.  Each
// round, every member sends every other member a manifest over the direct
// member-to-member TCP links (Mesh): its pending collectives (sequence number,
// kind, root, packet header) and the headers of the p2p messages it sends to
// that member in this round.  Once a member holds all manifests of round r it
// knows exactly which operations run in round r on EVERY member:
//   * a collective runs when every member has listed it (members submit
//     collectives in the same order, so the runnable set is the same prefix
//     of the sequence everywhere);
//   * every p2p message listed by its sender runs (the receiver allocates the
//     buffer in the round itself -- no wait for a recv() call).
// The member then issues round r on the group's single communicator and
// single comm stream: one ncclGroupStart/End per collective in sequence
// order, then one ncclGroupStart/End holding all of its p2p sends and
// receives of the round.  So every member's comm stream carries the same
// sequence of NCCL groups G_1, G_2, ..., and the operations of G_k on one
// member are matched exactly by the operations of G_k on the others.  By
// induction on k each G_k completes: G_1..G_{k-1} complete everywhere, so
// every member's G_k is at the head of its stream, and an NCCL group whose
// counterpart groups are all issued completes.  No send kernel can sit in
// front of a receive its peer's send waits for (the hang of free-running
// send/recv on one stream), and no cycle through several communicators and
// hardware queues can form inside a group.  The one rule left to callers is
// NCCL's own: two DIFFERENT groups on the same GPUs must not be driven in
// opposite orders by a blocking dependency (each group has its own
// communicator; elements never make one group's progress wait on another's).
//
// Backpressure: a receiver grants each sender a window of kWindow unconsumed
// messages in its manifests; a sender lists no more than the grant, and
// send() blocks while kWindow messages to that peer wait for a round.
//
// Bounded failure: manifests are awaited with the group timeout (a member
// that stops answering fails the round with an error naming it); each
// issued round records an event, and a round not complete on the device
// within the operation deadline (ini [rccl] op_timeout_ms, default the group
// timeout) calls ncclCommAbort -- RCCL's kernels then exit -- and every
// pending and later operation fails with an error naming the round's
// peers.  A member that leaves (its Group destroyed: an orderly goodbye on
// its links) is dropped from later rounds: p2p among the others continues,
// collectives fail ("member k left the group").
//
// Without GPUs (or backend=tcp) the same rounds run and the payload rides
// inline behind its header on the direct links (host bytes), so the same
// elements and tests exercise the same round logic on CPU-only boxes.
//
// Threading: any number of threads may call send() / recv(); collectives are
// called in the same order on every member (from one thread per group, as
// with NCCL).  Only the progress thread touches the communicator.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
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
  // open the outbound link to every other member now (so a member that leaves
  // before it ever sent anything still says goodbye on every link)
  bool connect_all(std::string* err);
  bool send(int peer, uint64_t tag, Message m, std::string* err);
  // next message with this tag from `src`, FIFO per source.  false:
  // *timed_out on timeout; else the mesh is closed or the member is gone --
  // *gone = 3 when it left with a goodbye, 1 when its link broke without one
  bool recv(uint64_t tag, int src, Message* m, int timeout_ms, bool* timed_out, int* gone, std::string* err);
  // wait until a message with this tag is queued (1), wake() holds or the
  // time runs out (0), or the mesh is closed (-1); wake() is evaluated under
  // the mesh lock, so a poke() after its condition became true is never lost
  int wait_tag(uint64_t tag, const std::function<bool()>& wake, int timeout_ms);
  void poke();
  void close();

 private:
  struct Item {
    int src;
    uint64_t tag;
    Message m;
  };
  void reader(std::shared_ptr<Connection> c);
  bool ensure_link(int peer, std::string* err);  // out_mu_[peer] held
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
  std::vector<int> lost_;  // per member: 1 = its link broke without a goodbye, 3 = it said goodbye
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
  // queued for the next round (blocks while kOutbox messages to the peer
  // wait); a message to oneself is handed over in-process
  bool send(int peer, const Packet& p, std::string* err);
  // from any member; false + *timed_out on timeout
  bool recv(Packet* p, int timeout_ms, bool* timed_out, std::string* err);

  // ---- control-plane access for element handshakes (keys are group-scoped) ----
  bool put(const std::string& key, const std::string& val, int readers = 0);
  bool get(const std::string& key, std::string* val, int timeout_ms);

  // abort blocking waits (element unlock / shutdown): pending and later
  // operations fail; the round in progress still completes on every member
  void cancel();

  // bytes moved on the data plane (stats / tests)
  uint64_t bytes_sent() const { return bytes_sent_.load(); }
  uint64_t bytes_received() const { return bytes_recv_.load(); }

  // why the group failed ("" while healthy)
  std::string failure() const;

 private:
  // one collective handed to the progress thread; its results are written
  // before `done` is published under mu_
  struct CollOp {
    enum Kind : uint32_t { kAllGather = 1, kBroadcast = 2, kScatter = 3 };
    Kind kind = kAllGather;
    uint64_t seq = 0;
    int root = 0;
    Packet mine;                // allgather: own packet; broadcast: the root's packet
    std::vector<Packet> parts;  // scatter root: one per member
    bool want_stacked = false;
    bool done = false, ok = false;
    std::string err;
    std::vector<Packet> all;  // allgather
    MemoryPtr stacked;
    Packet out;  // broadcast / scatter
    static const char* name(uint32_t k) {
      return k == kAllGather ? "allgather" : k == kBroadcast ? "broadcast" : k == kScatter ? "scatter" : "?";
    }
  };
  // what one member told this member in one round
  struct ManifestEntry {
    Packet hdr;  // header (+ inline blobs on tcp)
    std::vector<size_t> sizes;
    std::vector<std::string> metas;
  };
  struct ManifestColl {
    uint64_t seq = 0;
    uint32_t kind = 0;
    int root = 0;
    bool has_hdr = false;
    ManifestEntry e;
  };
  struct Manifest {
    uint32_t grant = 0;                // messages this member may still send it
    std::vector<ManifestColl> colls;   // its pending collectives (sequence order)
    std::vector<ManifestEntry> sends;  // its p2p messages to this member, in order
  };
  struct Inflight {
    hipEvent_t ev = nullptr;
    int64_t t0 = 0;
    uint64_t round = 0;
    std::string what;  // the round's operations and peers (deadline errors)
  };
  static constexpr int kWindow = 8;       // unconsumed messages a receiver grants each sender
  static constexpr int kOutbox = 8;       // queued sends per peer before send() blocks
  static constexpr size_t kInflight = 4;  // issued rounds not yet complete on the device

  Group() = default;
  bool init(const GroupSpec& spec, std::string* err);
  std::string key(const std::string& k) const { return prefix_ + "/" + k; }
  std::string encode(const Packet& p);
  bool decode(const std::string& s, Packet* p, std::vector<size_t>* sizes, std::vector<std::string>* metas);
  void* dev_ptr(const MemoryPtr& m);
  std::vector<MemoryPtr> alloc_recv(const std::vector<size_t>& sizes, const std::vector<std::string>& metas);
  void finish_inputs(const std::vector<MemoryPtr>& in);
  // ---- round engine ----
  bool collective(const std::shared_ptr<CollOp>& op, std::string* err);
  void progress();
  bool wait_trigger();
  // stopping (not cancelled): messages still queued for a member that is in
  // the group -- the engine runs rounds until they are out (bounded), so an
  // orderly close never drops what send() accepted
  bool pending_out();
  bool run_round(std::string* err);
  Message manifest_for(int d, uint32_t grant, const std::vector<std::shared_ptr<CollOp>>& colls,
                       const std::vector<Packet>& sends);
  bool parse_manifest(Message&& m, Manifest* out);
  bool issue_collective(CollOp& op, const std::vector<const ManifestColl*>& ent, std::string* what,
                        std::string* err);
  bool issue_p2p(std::vector<std::vector<Packet>>& sends, const std::vector<Manifest>& man,
                 std::vector<Packet>* got, std::string* what, std::string* err);
  bool reap(bool need_room, std::string* err);
  void fail(const std::string& why);       // fatal: every pending and later operation fails
  void drop_member(int m, bool orderly);   // a member left: later rounds run without it
  void poke();                             // wake the progress thread
  void stop_engine();

  GroupSpec spec_;
  std::vector<int> members_;
  int grank_ = 0;
  int device_ = -1;
  std::string prefix_;
  std::shared_ptr<void> store_host_;
  std::shared_ptr<StoreClient> store_;
  std::unique_ptr<Mesh> mesh_;  // member-to-member links (manifests; tcp payloads)
  void* comm_ = nullptr;        // ncclComm_t
  hipStream_t stream_ = nullptr;
  bool engine_ = false;         // rounds on a progress thread (n > 1, or forced RCCL)
  int op_timeout_ms_ = 60000;   // device completion deadline of an issued round
  std::thread thr_;
  std::atomic<bool> work_{false}, stop_{false}, cancelled_{false}, aborted_{false};
  int64_t drain_deadline_ = 0;  // stopping with queued sends: the flush rounds end by then
  std::vector<int> recvd_since_grant_;  // per sender: messages received since this member's last grant
  mutable std::mutex mu_;       // everything below, shared by callers and the progress thread
  std::condition_variable cv_;  // collective completion, inbox, outbox room
  std::string failed_;          // fatal error ("" while healthy)
  std::string coll_dead_;       // collectives no longer possible (a member left / a collective timed out)
  uint64_t coll_seq_ = 0;       // next collective sequence number
  std::deque<std::shared_ptr<CollOp>> colls_;  // submitted, not yet run (sequence order)
  std::vector<std::deque<Packet>> outbox_;     // per peer: sends waiting for a round
  std::deque<Packet> inbox_;                   // received p2p messages
  std::vector<int> unconsumed_;                // per sender: received, not taken by recv()
  std::vector<int> allowed_;                   // per peer: messages the next round may list
  std::vector<int> granted_;                   // per sender: last grant advertised to it
  std::vector<char> active_;                   // per member: still in the group's rounds
  std::vector<uint64_t> listed_upto_;          // per member: collectives listed in its last manifest
  uint64_t round_ = 0;                         // (progress thread only)
  std::deque<Inflight> inflight_;              // (progress thread only)
  std::atomic<uint64_t> bytes_sent_{0}, bytes_recv_{0};
};

// Process-wide cache so elements of one pipeline share a channel by name.
// (opened outside the cache lock: opening waits for the other members)
std::shared_ptr<Group> group_get(const GroupSpec& spec, std::string* err);

}  // namespace comm
}  // namespace nnsx
