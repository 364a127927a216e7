// Among-device elements over the nnsx TCP transport (comm/transport.h):
//   tensor_query_serversrc / tensor_query_serversink / tensor_query_client
//   (request/reply offload, replies routed by client_id) and edgesink /
//   edgesrc (publish/subscribe).
//
// Reference: gst/nnstreamer/tensor_query/tensor_query_client.c (props
// :99-165, caps handshake :421-500, chain :657-746), tensor_query_serversrc.c
// (:299-466), tensor_query_serversink.c (:237-293, `limit` of meta-less
// frames), tensor_query_server.c (id -> server registry, waits for the sink's
// caps before answering clients), gst/edge/edge_sink.c / edge_src.c.  The
// reference rides on the external nnstreamer-edge library (TCP / MQTT-hybrid
// / AITT); nnsx implements TCP and HYBRID (endpoint discovery through an MQTT
// broker, comm/mqtt.h) natively, MQTT / AITT for edgesink / edgesrc (the
// frames themselves travel through the broker on the topic: pub/sub without
// a direct socket, what nnstreamer-edge's MQTT and AITT types give an
// application; AITT's own library is not in the image), plus HIPIPC: the same framing with
// HBM-resident tensors handed over through an exported device ring
// (zero-copy on the same GPU, one xGMI peer copy across GPUs; see
// comm/transport.h), and RCCL: rank groups over xGMI (comm/group.h).
#include <algorithm>
#include <cstring>
#include <atomic>
#include <map>
#include <thread>

#include <unistd.h>

#include "comm/group.h"
#include "comm/mqtt.h"
#include "comm/transport.h"
#include "core/log.h"
#include "elements/elements.h"
#include "elements/rank_props.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/hip_util.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

const std::vector<std::string> kConnectTypes = {"TCP", "HYBRID", "MQTT", "AITT", "HIPIPC", "RCCL", "SHM"};
constexpr int kHipIpc = 4;
constexpr int kRccl = 5;
// same-host processes: TCP carries the headers, host frames that live in a
// shared-memory segment (videotestsrc pool-shm) travel by reference (comm/shm.h)
constexpr int kShm = 6;
const std::vector<std::string> kRcclModes = {"broadcast", "scatter", "allgather"};
constexpr int kRcclAllGather = 2;
constexpr uint32_t kPktCaps = 1;  // packet carries only a caps string

constexpr int kHybrid = 1;
constexpr int kMqtt = 2;
constexpr int kAitt = 3;

// broker-carried pub/sub (edgesink / edgesrc only)
bool via_broker(int type) { return type == kMqtt || type == kAitt; }

bool check_connect_type(Element* e, int type, bool pubsub = false) {
  if (type == 0 || type == kHybrid || type == kHipIpc || type == kRccl) return true;
  if (pubsub && type == kShm) return true;
  if (pubsub && via_broker(type)) return true;
  e->post_error("connect-type " + kConnectTypes[static_cast<size_t>(type)] + " is not supported by " + e->name() +
                (pubsub ? " (nnsx implements TCP, HYBRID, MQTT, AITT, HIPIPC, RCCL and SHM)"
                        : " (nnsx implements TCP, HYBRID, HIPIPC and RCCL; MQTT / AITT are pub/sub: edgesink / edgesrc)"));
  return false;
}

// ---- connect-type=MQTT / AITT: every message is one PUBLISH on
// nnsx/<type>/<topic>/data (QoS 0, in order over the broker connection); the
// current caps are also retained on .../caps for subscribers that join late.
//   u32 magic 'NXBK' | u32 type | u32 nblobs | u32 caps_len
//   i64 pts | i64 dts | i64 duration | u64 blob_size[nblobs] | caps | blobs
constexpr uint32_t kBrokerMagic = 0x4e58424bu;

std::string broker_topic(int type, const std::string& topic, const char* leaf) {
  return strfmt("nnsx/", type == kAitt ? "aitt" : "mqtt", "/", topic.empty() ? "default" : topic, "/", leaf);
}

std::string broker_header(const comm::Message& m) {
  std::string h;
  auto put = [&](const void* p, size_t n) { h.append(static_cast<const char*>(p), n); };
  const uint32_t w[4] = {kBrokerMagic, static_cast<uint32_t>(m.type), static_cast<uint32_t>(m.blobs.size()),
                         static_cast<uint32_t>(m.caps.size())};
  put(w, sizeof(w));
  const int64_t t[3] = {m.pts, m.dts, m.duration};
  put(t, sizeof(t));
  for (auto& b : m.blobs) {
    const uint64_t n = b->size();
    put(&n, sizeof(n));
  }
  h += m.caps;
  return h;
}

bool broker_publish(comm::MqttClient& cli, const std::string& topic, const comm::Message& m) {
  const std::string h = broker_header(m);
  if (m.blobs.empty()) return cli.publish(topic, h.data(), h.size(), 0, false);
  if (m.blobs.size() == 1) {
    const void* p = m.blobs[0]->map_host();
    return cli.publish2(topic, h.data(), h.size(), p, m.blobs[0]->size(), 0, false);
  }
  std::string body;
  for (auto& b : m.blobs) body.append(static_cast<const char*>(b->map_host()), b->size());
  return cli.publish2(topic, h.data(), h.size(), body.data(), body.size(), 0, false);
}

bool broker_parse(const std::string& pl, comm::Message* m) {
  size_t at = 0;
  auto get = [&](void* p, size_t n) {
    if (pl.size() - at < n) return false;
    std::memcpy(p, pl.data() + at, n);
    at += n;
    return true;
  };
  uint32_t w[4];
  int64_t t[3];
  if (!get(w, sizeof(w)) || w[0] != kBrokerMagic || w[2] > static_cast<uint32_t>(kSizeLimit + kSizeExtraLimit) ||
      !get(t, sizeof(t)))
    return false;
  std::vector<uint64_t> sizes(w[2]);
  for (auto& n : sizes)
    if (!get(&n, sizeof(n))) return false;
  if (pl.size() - at < w[3]) return false;
  m->type = static_cast<comm::MsgType>(w[1]);
  m->caps = pl.substr(at, w[3]);
  at += w[3];
  m->pts = t[0];
  m->dts = t[1];
  m->duration = t[2];
  m->blobs.clear();
  for (uint64_t n : sizes) {
    if (pl.size() - at < n) return false;
    auto b = Memory::alloc_host(static_cast<size_t>(n));
    if (n) std::memcpy(b->data(), pl.data() + at, static_cast<size_t>(n));
    at += static_cast<size_t>(n);
    m->blobs.push_back(b);
  }
  return true;
}

// ---- connect-type=HYBRID: the MQTT broker at dest-host:dest-port only
// carries each server's / publisher's TCP endpoint, retained on
// nnsx/edge/<topic>/<id>; data flows over TCP (nnstreamer-edge HYBRID:
// tensor_query_client.c:366-384 reconnects to another server on failure).
std::string hybrid_topic(const std::string& topic) { return "nnsx/edge/" + (topic.empty() ? "default" : topic); }

class HybridAnnouncer {
 public:
  ~HybridAnnouncer() { withdraw(); }
  bool announce(const std::string& broker, int broker_port, const std::string& topic, const std::string& host,
                int port, std::string* err) {
    static std::atomic<unsigned> seq{0};
    key_ = strfmt(hybrid_topic(topic), "/", getpid(), "-", seq++);
    if (!cli_.connect(broker, broker_port, key_, 60, true, 5000, err)) return false;
    const std::string ep = strfmt(host == "localhost" || host.empty() ? "127.0.0.1" : host, ":", port);
    return cli_.publish(key_, ep.data(), ep.size(), 1, true);
  }
  void withdraw() {
    if (!cli_.connected()) return;
    cli_.publish(key_, "", 0, 1, true);  // empty retained payload clears the entry
    cli_.close();
  }

 private:
  comm::MqttClient cli_;
  std::string key_;
};

// every endpoint announced on the topic (retained), in announcement-key order
std::vector<std::pair<std::string, int>> hybrid_discover(const std::string& broker, int broker_port,
                                                         const std::string& topic, int timeout_ms, std::string* err) {
  comm::MqttClient cli;
  std::vector<std::pair<std::string, int>> out;
  if (!cli.connect(broker, broker_port, strfmt("nnsx-discover-", getpid(), "-", now_ns()), 0, true, 5000, err) ||
      !cli.subscribe(hybrid_topic(topic) + "/+", 1)) {
    if (err && err->empty()) *err = "HYBRID: broker subscription failed";
    return out;
  }
  std::map<std::string, std::string> found;
  const int64_t deadline = now_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  while (now_ns() < deadline) {
    comm::MqttMessage m;
    // after the first answer only the rest of the retained burst is awaited
    if (!cli.recv(&m, found.empty() ? 100 : 50)) {
      if (!found.empty()) break;
      continue;
    }
    if (m.payload.empty())
      found.erase(m.topic);
    else
      found[m.topic] = m.payload;
  }
  cli.close();
  for (auto& kv : found) {
    const size_t c = kv.second.rfind(':');
    if (c != std::string::npos) out.emplace_back(kv.second.substr(0, c), std::atoi(kv.second.c_str() + c + 1));
  }
  if (out.empty() && err) *err = "HYBRID: no server announced on " + hybrid_topic(topic);
  return out;
}

// connect to the first reachable endpoint (TCP / HYBRID)
std::shared_ptr<comm::Connection> connect_endpoint(int type, const std::string& host, unsigned port,
                                                   const std::string& topic, int timeout_ms, std::string* err,
                                                   const std::string& avoid = std::string()) {
  if (type != kHybrid) return comm::Connection::connect(host, static_cast<int>(port), timeout_ms, err);
  auto eps = hybrid_discover(host, static_cast<int>(port), topic, timeout_ms, err);
  std::shared_ptr<comm::Connection> c;
  for (int pass = 0; pass < 2 && !c; ++pass)
    for (auto& ep : eps) {
      if (pass == 0 && strfmt(ep.first, ":", ep.second) == avoid) continue;  // prefer another server
      if ((c = comm::Connection::connect(ep.first, ep.second, timeout_ms, err))) break;
    }
  return c;
}

// channel name shared by the two ends of a connect-type=RCCL link
std::string rccl_channel(const char* kind, const std::string& topic, unsigned port) {
  return strfmt(kind, ":", topic.empty() ? std::to_string(port) : topic);
}

std::vector<MemoryPtr> place_blobs(std::vector<MemoryPtr> blobs, int device, StreamSet& streams);

// ---------------------------------------------------------------- EdgeHub ----
// connect-type=RCCL rccl-mode=allgather: N->N pub/sub on one topic.  Every
// member's edgesink publishes its stream and every member subscribes to the
// others' with one edgesrc per source (peer-rank); a round is ONE collective
// (comm::Group::allgather -> ncclAllGather over xGMI for equal-size frames)
// instead of one broadcast per publisher.  The hub is the process-local
// meeting point: the publishing edgesink runs the rounds and deals each
// member's packet to the queue of the local edgesrc subscribed to it (sources
// nobody subscribed to are dropped); a full queue holds the publisher back
// (bounded, cancellable), so a slow consumer throttles the whole round.
// Reference pub/sub: gst/edge/edge_sink.c:305-345, edge_src.c:255-412.
class EdgeHub {
 public:
  static std::shared_ptr<EdgeHub> get(const std::string& key) {
    static std::mutex mu;
    static std::map<std::string, std::weak_ptr<EdgeHub>> hubs;
    std::lock_guard<std::mutex> lk(mu);
    auto h = hubs[key].lock();
    if (!h) hubs[key] = h = std::make_shared<EdgeHub>();
    return h;
  }
  void subscribe(int global_rank) {
    std::lock_guard<std::mutex> lk(mu_);
    auto& q = subs_[global_rank].q;
    // a subscriber that starts after the caps round still gets the caps (sticky)
    auto c = caps_.find(global_rank);
    if (q.empty() && c != caps_.end()) q.push_back(c->second);
  }
  void unsubscribe(int global_rank) {
    std::lock_guard<std::mutex> lk(mu_);
    subs_.erase(global_rank);
    cv_.notify_all();
  }
  // one round: every member's packet, dealt to the subscribed queues.  false:
  // the round failed, or cancel_publish() ended this call's wait for room
  bool publish(comm::Group& g, const comm::Packet& mine, std::string* err) {
    std::vector<comm::Packet> all;
    if (!g.allgather(mine, &all, err)) return false;
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t gen = pub_gen_;
    for (size_t r = 0; r < all.size(); ++r) {
      const int src = g.global_rank(static_cast<int>(r));
      if (all[r].flags & kPktCaps) {
        caps_[src] = all[r];
        caps_[src].src = src;
      }
      auto it = subs_.find(src);
      if (it == subs_.end()) continue;
      cv_.wait(lk, [&] {
        auto i = subs_.find(src);
        return pub_gen_ != gen || i == subs_.end() || i->second.q.size() < kDepth;
      });
      if (pub_gen_ != gen) return false;
      it = subs_.find(src);
      if (it == subs_.end()) continue;
      all[r].src = src;
      it->second.q.push_back(std::move(all[r]));
    }
    cv_.notify_all();
    return true;
  }
  // next packet of member `global_rank` (false + *timed_out on timeout; false:
  // unsubscribed, or cancel_take(global_rank) ended this call's wait)
  bool take(int global_rank, comm::Packet* p, int timeout_ms, bool* timed_out) {
    std::unique_lock<std::mutex> lk(mu_);
    *timed_out = false;
    auto it0 = subs_.find(global_rank);
    if (it0 == subs_.end()) return false;
    const uint64_t gen = it0->second.cancel_gen;
    auto ready = [&] {
      auto it = subs_.find(global_rank);
      return it == subs_.end() || it->second.cancel_gen != gen || !it->second.q.empty();
    };
    if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) {
      *timed_out = true;
      return false;
    }
    auto it = subs_.find(global_rank);
    if (it == subs_.end() || it->second.cancel_gen != gen) return false;
    *p = std::move(it->second.q.front());
    it->second.q.pop_front();
    cv_.notify_all();
    return true;
  }
  // Cancellation is per waiter: it ends the waits in progress of ONE party --
  // the publishing edgesink's publish() (its unlock / flush), or one
  // subscriber's take() (its edgesrc's unlock) -- and nothing later, so one
  // element stopping never fails the other elements of the topic.
  void cancel_publish() {
    std::lock_guard<std::mutex> lk(mu_);
    ++pub_gen_;
    cv_.notify_all();
  }
  void cancel_take(int global_rank) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = subs_.find(global_rank);
    if (it != subs_.end()) ++it->second.cancel_gen;
    cv_.notify_all();
  }

 private:
  static constexpr size_t kDepth = 4;
  struct Sub {
    std::deque<comm::Packet> q;
    uint64_t cancel_gen = 0;
  };
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int, Sub> subs_;           // per subscribed source (global rank)
  std::map<int, comm::Packet> caps_;  // latest caps packet per source
  uint64_t pub_gen_ = 0;
};

comm::Packet packet_of(const Buffer& b) {
  comm::Packet p;
  p.pts = b.pts;
  p.dts = b.dts;
  p.duration = b.duration;
  p.blobs = b.mems;
  return p;
}

BufferPtr buffer_of(comm::Packet& p, int device, StreamSet& streams) {
  auto b = make_buffer();
  b->mems = place_blobs(std::move(p.blobs), device, streams);
  b->pts = p.pts;
  b->dts = p.dts;
  b->duration = p.duration;
  return b;
}

// received host blobs -> memories on the requested device (-1: keep them in
// pinned host memory); ring blobs already live in HBM and stay zero-copy
std::vector<MemoryPtr> place_blobs(std::vector<MemoryPtr> blobs, int device, StreamSet& streams) {
  if (device < 0) return blobs;
  hip::DeviceGuard g(device);
  hipStream_t s = streams.get(device);
  std::vector<MemoryPtr> out;
  for (auto& b : blobs) {
    if (b->on_device()) {
      out.push_back(b);
      continue;
    }
    auto d = Memory::alloc_device(b->size(), device, s);
    if (b->size())
      hip::check(hipMemcpyAsync(d->data(), b->data(), b->size(), hipMemcpyHostToDevice, s), "comm H2D");
    d->mark_ready(s);
    b->record_use(s, device);
    out.push_back(d);
  }
  return out;
}

// ============================================================ query server ====
class QueryServer {
 public:
  bool start(const std::string& host, int port, std::string* err) {
    std::lock_guard<std::mutex> lk(life_mu_);
    if (users_++ > 0) return true;
    if (!listener_.listen(host, port, err)) {
      users_ = 0;
      return false;
    }
    running_ = true;
    incoming.set_flushing(false);
    accept_thr_ = std::thread([this] { accept_loop(); });
    return true;
  }

  void stop() {
    std::lock_guard<std::mutex> lk(life_mu_);
    if (users_ == 0 || --users_ > 0) return;
    running_ = false;
    listener_.close();
    {
      std::lock_guard<std::mutex> l2(mu_);
      for (auto& c : conns_) c.second->close();
      cv_.notify_all();
    }
    if (accept_thr_.joinable()) accept_thr_.join();
    std::vector<std::thread> rs;
    {
      std::lock_guard<std::mutex> l2(mu_);
      rs.swap(readers_);
      conns_.clear();
      sink_caps_.clear();
    }
    for (auto& t : rs)
      if (t.joinable()) t.join();
    incoming.set_flushing(true);
  }

  int port() const { return listener_.port(); }

  void set_sink_caps(const std::string& caps) {
    std::lock_guard<std::mutex> lk(mu_);
    sink_caps_ = caps;
    cv_.notify_all();
  }

  bool reply(uint64_t client_id, const comm::Message& m) {
    std::shared_ptr<comm::Connection> c;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = conns_.find(client_id);
      if (it == conns_.end()) return false;
      c = it->second;
    }
    return c->send(m);
  }

  size_t clients() {
    std::lock_guard<std::mutex> lk(mu_);
    return conns_.size();
  }

  comm::MessageQueue incoming;

  // connect-type=RCCL: the serversrc's rank settings + channel, read by the
  // paired serversink (requests and replies ride one group per direction)
  std::mutex rank_mu;
  RankProps rank;
  std::string channel;

 private:
  void accept_loop() {
    while (running_) {
      auto c = listener_.accept(100);
      if (!c) continue;
      std::lock_guard<std::mutex> lk(mu_);
      c->id = next_id_++;
      conns_[c->id] = c;
      readers_.emplace_back([this, c] { reader(c); });
    }
  }

  void reader(std::shared_ptr<comm::Connection> c) {
    {
      // answer only once the server pipeline negotiated its output (serversink caps)
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !sink_caps_.empty() || !running_; });
      if (!running_) return;
      comm::Message hello;
      hello.type = comm::MsgType::HELLO;
      hello.client_id = c->id;
      hello.caps = sink_caps_;
      lk.unlock();
      if (!c->send(hello)) return;
    }
    while (running_ && c->alive()) {
      comm::Message m;
      bool timed_out = false;
      if (!c->recv(&m, 100, &timed_out)) {
        if (timed_out) continue;
        break;
      }
      if (m.type == comm::MsgType::DATA) {
        m.client_id = c->id;
        incoming.push(std::move(m));
      } else if (m.type == comm::MsgType::BYE || m.type == comm::MsgType::EOS) {
        break;
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    conns_.erase(c->id);
  }

  std::mutex life_mu_;
  int users_ = 0;
  comm::Listener listener_;
  std::atomic<bool> running_{false};
  std::thread accept_thr_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<uint64_t, std::shared_ptr<comm::Connection>> conns_;
  std::vector<std::thread> readers_;
  std::string sink_caps_;
  uint64_t next_id_ = 1;
};

std::shared_ptr<QueryServer> query_server(int id) {
  static std::mutex mu;
  static std::map<int, std::shared_ptr<QueryServer>> servers;
  std::lock_guard<std::mutex> lk(mu);
  auto& s = servers[id];
  if (!s) s = std::make_shared<QueryServer>();
  return s;
}

// --------------------------------------------------------- serversrc ----
class QueryServerSrc : public BaseSrc {
 public:
  explicit QueryServerSrc(const std::string& name)
      : BaseSrc("tensor_query_serversrc", name, Caps::from_string(tensor_caps_template_all())) {
    prop_string("host", &host_, "The hostname to listen as");
    PropSpec p;
    p.name = "port";
    p.type = PropType::UINT;
    p.blurb = "The port to listen to (0 = ephemeral; reads back the bound port)";
    p.set = [this](const std::string& v) { port_ = static_cast<int>(to_uint(v)); };
    p.get = [this] { return std::to_string(server_ && server_->port() ? server_->port() : port_); };
    add_prop(p);
    prop_string("dest-host", &dest_host_, "The hostname of the broker (HYBRID/MQTT; unused over TCP)");
    prop_uint("dest-port", &dest_port_, "The port of the broker (HYBRID/MQTT; unused over TCP)");
    prop_enum("connect-type", &connect_type_, kConnectTypes, "The connection type");
    prop_uint("timeout", &timeout_ms_, "The timeout (ms) to wait for the first client message (0 = forever)");
    prop_string("topic", &topic_, "The main topic of the host (HYBRID/MQTT)");
    prop_uint("id", &id_, "ID shared with the paired tensor_query_serversink");
    prop_int("device", &device_, "nnsx: upload received tensors to this GPU (-1 = keep in pinned host memory)");
    rp_.install([this](PropSpec p) -> PropSpec& { return add_prop(p); }, false);
    is_live_ = true;
  }

 protected:
  bool on_start() override {
    if (!check_connect_type(this, connect_type_)) return false;
    server_ = query_server(static_cast<int>(id_));
    if (connect_type_ == kRccl) {
      rp_.device = device_;
      std::lock_guard<std::mutex> lk(server_->rank_mu);
      server_->rank = rp_;
      server_->channel = rccl_channel("query", topic_, static_cast<unsigned>(port_));
      return true;
    }
    std::string err;
    if (!server_->start(host_, port_, &err)) {
      post_error("tensor_query_serversrc: " + err);
      server_.reset();
      return false;
    }
    if (connect_type_ == kHybrid) {
      announcer_ = std::make_unique<HybridAnnouncer>();
      if (!announcer_->announce(dest_host_, static_cast<int>(dest_port_), topic_, host_, server_->port(), &err)) {
        post_error("tensor_query_serversrc: HYBRID announce: " + err);
        return false;
      }
    }
    return true;
  }
  void on_stop() override {
    announcer_.reset();
    if (server_ && connect_type_ != kRccl) server_->stop();
    req_.reset();
  }
  void on_unlock() override {
    if (server_) server_->incoming.set_flushing(true);
    if (auto g = req_) g->cancel();
  }

  FlowReturn create(BufferPtr* out) override {
    if (connect_type_ == kRccl) {
      if (!req_ && !(req_ = rp_.open(this, server_->channel))) return FlowReturn::ERROR;
      comm::Packet p;
      std::string err;
      const int64_t t0 = now_ns();
      while (true) {
        bool to = false;
        if (req_->recv(&p, 100, &to, &err)) break;
        if (flushing_.load()) return FlowReturn::FLUSHING;
        if (!to) {
          post_error("tensor_query_serversrc: " + err);
          return FlowReturn::ERROR;
        }
        if (timeout_ms_ > 0 && now_ns() - t0 > static_cast<int64_t>(timeout_ms_) * 1000000) return FlowReturn::EOS;
      }
      if (p.eos) return create(out);  // a client left; keep serving the others
      const uint64_t cid = static_cast<uint64_t>(p.src) + 1;
      *out = buffer_of(p, device_, streams_);
      (*out)->meta.client_id = cid;
      return FlowReturn::OK;
    }
    comm::Message m;
    const int64_t t0 = now_ns();
    while (true) {
      if (server_->incoming.pop(&m, 100)) break;
      if (flushing_.load()) return FlowReturn::FLUSHING;
      if (timeout_ms_ > 0 && now_ns() - t0 > static_cast<int64_t>(timeout_ms_) * 1000000) return FlowReturn::EOS;
    }
    auto b = make_buffer();
    b->mems = place_blobs(std::move(m.blobs), device_, streams_);
    b->pts = m.pts;
    b->dts = m.dts;
    b->duration = m.duration;
    b->meta.client_id = m.client_id;
    *out = b;
    return FlowReturn::OK;
  }

 private:
  std::string host_ = "localhost", dest_host_ = "localhost", topic_;
  int port_ = 3000;
  unsigned dest_port_ = 1883, timeout_ms_ = 0, id_ = 0;
  int connect_type_ = 0, device_ = -1;
  std::shared_ptr<QueryServer> server_;
  StreamSet streams_;
  RankProps rp_;
  std::shared_ptr<comm::Group> req_;
  std::unique_ptr<HybridAnnouncer> announcer_;
};

// -------------------------------------------------------- serversink ----
class QueryServerSink : public BaseSink {
 public:
  explicit QueryServerSink(const std::string& name)
      : BaseSink("tensor_query_serversink", name, Caps::from_string(tensor_caps_template_all())) {
    prop_enum("connect-type", &connect_type_, kConnectTypes, "The connection type");
    prop_uint("timeout", &timeout_ms_, "The timeout (ms) for sending a reply");
    prop_uint("id", &id_, "ID shared with the paired tensor_query_serversrc");
    prop_uint("limit", &limit_, "Consecutive frames without a client id tolerated before erroring out");
    PropSpec a;
    a.name = "async";
    a.type = PropType::BOOL;
    a.blurb = "Accepted for gst-launch compatibility";
    a.set = [](const std::string&) {};
    a.get = [] { return std::string("false"); };
    add_prop(a);
  }

 protected:
  bool start() override {
    BaseSink::start();
    metaless_ = 0;
    server_ = query_server(static_cast<int>(id_));
    return check_connect_type(this, connect_type_);
  }
  bool set_caps(const Caps& caps) override {
    if (connect_type_ == kRccl) {
      if (!open_rep()) return false;
      // clients read the server's output caps from the group store
      return rep_->put("caps", caps.to_string());
    }
    server_->set_sink_caps(caps.to_string());
    return true;
  }
  bool stop() override {
    rep_.reset();
    return true;
  }
  void unlock() override {
    if (auto g = rep_) g->cancel();
  }
  bool open_rep() {
    if (rep_) return true;
    RankProps rp;
    std::string ch;
    {
      std::lock_guard<std::mutex> lk(server_->rank_mu);
      rp = server_->rank;
      ch = server_->channel;
    }
    if (ch.empty()) {
      post_error("tensor_query_serversink: no connect-type=RCCL tensor_query_serversrc with the same id");
      return false;
    }
    return (rep_ = rp.open(this, ch)) != nullptr;  // (the serversrc's group: one per query channel)
  }
  FlowReturn render(const BufferPtr& buf) override {
    const uint64_t cid = buf->meta.client_id;
    if (connect_type_ == kRccl && cid != 0) {
      metaless_ = 0;
      std::string err;
      if (!open_rep() || !rep_->send(static_cast<int>(cid - 1), packet_of(*buf), &err)) {
        post_error("tensor_query_serversink: " + err);
        return FlowReturn::ERROR;
      }
      return FlowReturn::OK;
    }
    if (cid == 0) {
      if (++metaless_ > limit_) {
        post_error("tensor_query_serversink: too many frames without a query client id");
        return FlowReturn::ERROR;
      }
      return FlowReturn::OK;
    }
    metaless_ = 0;
    comm::Message m;
    m.type = comm::MsgType::DATA;
    m.client_id = cid;
    m.pts = buf->pts;
    m.dts = buf->dts;
    m.duration = buf->duration;
    m.blobs = buf->mems;
    if (!server_->reply(cid, m)) NNSX_LOGW(name(), "client ", cid, " is gone; reply dropped");
    return FlowReturn::OK;
  }

 private:
  int connect_type_ = 0;
  unsigned timeout_ms_ = 0, id_ = 0, limit_ = 1, metaless_ = 0;
  std::shared_ptr<QueryServer> server_;
  std::shared_ptr<comm::Group> rep_;
};

// ------------------------------------------------------------ client ----
class QueryClient : public Element {
 public:
  explicit QueryClient(const std::string& name) : Element("tensor_query_client", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_all()));
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_all()));
    prop_string("host", &host_, "A host address to receive the results (unused over TCP: replies share the socket)");
    prop_uint("port", &port_, "A port to receive the results (unused over TCP)");
    prop_string("dest-host", &dest_host_, "A server host address to connect to");
    prop_uint("dest-port", &dest_port_, "A server port to connect to");
    prop_bool("silent", &silent_, "Produce verbose output");
    prop_enum("connect-type", &connect_type_, kConnectTypes, "The connection type");
    prop_string("topic", &topic_, "The main topic of the host and option if necessary");
    prop_uint("timeout", &timeout_ms_, "The timeout (ms) for a server reply (0 = wait forever)");
    prop_uint("max-request", &max_request_, "Requests kept in flight before waiting for a reply");
    prop_int("device", &device_, "nnsx: upload replies to this GPU (-1 = pinned host memory)");
    prop_readonly("client-id", [this] { return std::to_string(conn_ ? conn_->id : 0); }, "Client id assigned by the server");
    prop_readonly(
        "ipc-blobs",
        [this] { return conn_ ? strfmt(conn_->ipc_blobs_sent(), ":", conn_->ipc_blobs_received()) : std::string("0:0"); },
        "nnsx: tensors sent:received through the HIPIPC device ring");
    rp_.install([this](PropSpec p) -> PropSpec& { return add_prop(p); }, false);
  }

  bool start() override {
    if (!check_connect_type(this, connect_type_)) return false;
    pending_.clear();
    seq_ = 0;
    if (connect_type_ == kRccl) return true;
    std::string err;
    if (!connect_server(std::string(), &err)) {
      post_error("tensor_query_client: " + err);
      return false;
    }
    return true;
  }

  // TCP / HYBRID / HIPIPC: connect + HELLO handshake (HYBRID: `avoid` = the
  // server that just failed; another announced one is preferred)
  bool connect_server(const std::string& avoid, std::string* err) {
    conn_ = connect_endpoint(connect_type_, dest_host_, dest_port_, topic_,
                             timeout_ms_ ? static_cast<int>(timeout_ms_) : 10000, err, avoid);
    if (!conn_) return false;
    comm::Message hello;
    if (!conn_->recv(&hello, 30000) || hello.type != comm::MsgType::HELLO) {
      *err = "no handshake from the server";
      return false;
    }
    conn_->id = hello.client_id;
    if (connect_type_ == kHipIpc && !conn_->send_ipc_hello())
      NNSX_LOGW(name(), "HIPIPC: no GPU here, requests travel as bytes");
    server_caps_ = hello.caps.empty() ? Caps::from_string(tensor_caps_template_all()) : Caps::from_string(hello.caps);
    return true;
  }

  comm::Message request_of(const Buffer& b) {
    comm::Message m;
    m.type = comm::MsgType::DATA;
    m.client_id = conn_->id;
    m.seq = seq_++;
    m.pts = b.pts;
    m.dts = b.dts;
    m.duration = b.duration;
    m.blobs = b.mems;
    return m;
  }

  // HYBRID failover (tensor_query_client.c:366-384): reconnect to another
  // announced server and re-send every request still waiting for a reply
  bool failover() {
    if (connect_type_ != kHybrid) return false;
    const std::string failed = conn_ ? conn_->peer() : std::string();
    if (conn_) conn_->close();
    std::string err;
    if (!connect_server(failed, &err)) {
      NNSX_LOGW(name(), "HYBRID failover: ", err);
      return false;
    }
    NNSX_LOGI(name(), "HYBRID failover: ", failed, " -> ", conn_->peer());
    for (auto& b : pending_)
      if (!conn_->send(request_of(*b))) return false;
    return true;
  }
  bool stop() override {
    if (conn_) {
      comm::Message bye;
      bye.type = comm::MsgType::BYE;
      conn_->send(bye);
      conn_->close();
      conn_.reset();
    }
    req_.reset();
    rep_.reset();
    have_server_caps_ = false;
    return true;
  }
  void unlock() override {
    if (conn_) conn_->close();
    if (auto g = req_) g->cancel();
    if (auto g = rep_) g->cancel();
  }

  // connect-type=RCCL: join the request / reply groups and read the server's caps
  bool open_rccl() {
    if (req_) return true;
    rp_.device = device_;
    const std::string ch = rccl_channel("query", topic_, dest_port_);
    // requests and replies share ONE group (one round sequence: a reply can
    // never queue on the device behind a request of another group's round)
    if (!(rep_ = rp_.open(this, ch))) return false;
    req_ = rep_;
    server_ = rp_.peer_in(*req_);
    if (server_ < 0 || server_ == req_->rank()) {
      post_error("tensor_query_client: peer-rank is not another member of the group");
      return false;
    }
    std::string caps;
    if (!rep_->get("caps", &caps, static_cast<int>(rp_.timeout_ms))) {
      post_error("tensor_query_client: the server published no caps");
      return false;
    }
    server_caps_ = Caps::from_string(caps);
    have_server_caps_ = true;
    return true;
  }

  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS && connect_type_ == kRccl) {
      if (!open_rccl()) return false;
      return src_pad()->push_event(Event::make_caps(server_caps_));
    }
    if (ev.type == EventType::EOS && connect_type_ == kRccl && req_) {
      if (!flow_ok(drain(0))) return false;
      // tell the server this client is done (it keeps serving the others)
      comm::Packet bye;
      bye.eos = true;
      std::string err;
      req_->send(server_, bye, &err);
      return forward_event_downstream(ev);
    }
    if (ev.type == EventType::CAPS) {
      comm::Message m;
      m.type = comm::MsgType::CAPS;
      m.caps = ev.caps.to_string();
      if (conn_) conn_->send(m);
      return src_pad()->push_event(Event::make_caps(server_caps_));
    }
    if (ev.type == EventType::EOS) {
      if (!flow_ok(drain(0))) return false;
    }
    return forward_event_downstream(ev);
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->direction() == PadDirection::SRC && (conn_ || have_server_caps_) ? server_caps_ : pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    if (connect_type_ == kRccl) {
      std::string err;
      if (!open_rccl()) return FlowReturn::ERROR;
      if (!req_->send(server_, packet_of(*buf), &err)) {
        post_error("tensor_query_client: " + err);
        return FlowReturn::ERROR;
      }
      pending_.push_back(buf);
      return drain(std::max(1u, max_request_) - 1);
    }
    if (!conn_) return FlowReturn::ERROR;
    if (!conn_->send(request_of(*buf))) {
      const std::string peer = conn_->peer();
      if (!failover() || !conn_->send(request_of(*buf))) {
        post_error("tensor_query_client: failed to send a request to " + peer);
        return FlowReturn::ERROR;
      }
    }
    pending_.push_back(buf);
    return drain(std::max(1u, max_request_) - 1);
  }

 private:
  // receive replies until at most `keep` requests remain in flight
  FlowReturn drain(size_t keep) {
    while (rep_ && pending_.size() > keep) {
      comm::Packet r;
      bool timed_out = false;
      std::string err;
      const int t = timeout_ms_ ? static_cast<int>(timeout_ms_) : -1;
      if (!rep_->recv(&r, t, &timed_out, &err)) {
        post_error(timed_out ? "tensor_query_client: timed out waiting for the server"
                             : "tensor_query_client: " + err);
        return FlowReturn::ERROR;
      }
      BufferPtr in = pending_.front();
      pending_.pop_front();
      auto out = buffer_of(r, device_, streams_);
      out->copy_metadata_from(*in);
      FlowReturn fr = src_pad()->push(out);
      if (!flow_ok(fr)) return fr;
    }
    while (pending_.size() > keep) {
      comm::Message r;
      bool timed_out = false;
      const int t = timeout_ms_ ? static_cast<int>(timeout_ms_) : -1;
      if (!conn_ || !conn_->recv(&r, t, &timed_out)) {
        if (!timed_out && failover()) continue;
        post_error(timed_out ? "tensor_query_client: timed out waiting for the server"
                             : "tensor_query_client: connection to the server lost");
        return FlowReturn::ERROR;
      }
      if (r.type != comm::MsgType::DATA) continue;
      BufferPtr in = pending_.front();
      pending_.pop_front();
      auto out = make_buffer();
      out->copy_metadata_from(*in);
      out->mems = place_blobs(std::move(r.blobs), device_, streams_);
      FlowReturn fr = src_pad()->push(out);
      if (!flow_ok(fr)) return fr;
    }
    return FlowReturn::OK;
  }

  std::string host_ = "localhost", dest_host_ = "localhost", topic_;
  unsigned port_ = 0, dest_port_ = 3000, timeout_ms_ = 0, max_request_ = 1;
  bool silent_ = true;
  int connect_type_ = 0, device_ = -1;
  std::shared_ptr<comm::Connection> conn_;
  Caps server_caps_;
  std::deque<BufferPtr> pending_;
  uint64_t seq_ = 0;
  StreamSet streams_;
  RankProps rp_;
  std::shared_ptr<comm::Group> req_, rep_;
  int server_ = 0;  // server's rank inside the request / reply groups
  bool have_server_caps_ = false;
};

// ============================================================== edgesink ====
class EdgeSink : public BaseSink {
 public:
  explicit EdgeSink(const std::string& name) : BaseSink("edgesink", name, Caps::Any()) {
    prop_string("host", &host_, "The hostname of the pipeline");
    PropSpec p;
    p.name = "port";
    p.type = PropType::UINT;
    p.blurb = "The port of the pipeline (0 = ephemeral; reads back the bound port)";
    p.set = [this](const std::string& v) { port_ = static_cast<int>(to_uint(v)); };
    p.get = [this] { return std::to_string(listener_.port() ? listener_.port() : port_); };
    add_prop(p);
    prop_enum("connect-type", &connect_type_, kConnectTypes, "The connections type between edgesink and edgesrc");
    prop_string("dest-host", &dest_host_, "The hostname of the broker (HYBRID/MQTT)");
    prop_uint("dest-port", &dest_port_, "The port of the broker (HYBRID/MQTT)");
    prop_string("topic", &topic_, "The main topic of the host");
    prop_uint("wait-connection", &wait_subscribers_,
              "nnsx: block the first frame until this many subscribers are connected");
    prop_uint("connection-timeout", &wait_timeout_ms_, "nnsx: max wait (ms) for wait-connection");
    PropSpec a;
    a.name = "async";
    a.type = PropType::BOOL;
    a.blurb = "Accepted for gst-launch compatibility";
    a.set = [](const std::string&) {};
    a.get = [] { return std::string("false"); };
    add_prop(a);
    prop_readonly("subscribers", [this] { return std::to_string(subscribers()); }, "Connected subscribers");
    rp_.install([this](PropSpec p) -> PropSpec& { return add_prop(p); });
    prop_enum("rccl-mode", &rccl_mode_, kRcclModes,
              "nnsx (connect-type=RCCL): broadcast every frame to all subscribers, scatter frames round-robin, "
              "or allgather (every member publishes on the topic; one collective per round)");
    prop_readonly("comm-bytes", [this] { return std::to_string(g_ ? g_->bytes_sent() : 0); },
                  "nnsx: payload bytes published on the rank group");

    prop_readonly("comm-group", [this] { return g_ ? strfmt(g_->backend_name(), ":", g_->size()) : std::string(); },
                  "nnsx: data plane and member count of the rank group (e.g. rccl:8)");
  }

 protected:
  bool start() override {
    BaseSink::start();
    if (!check_connect_type(this, connect_type_, true)) return false;
    if (connect_type_ == kRccl) {
      running_ = true;
      return true;
    }
    std::string err;
    if (via_broker(connect_type_)) {
      static std::atomic<unsigned> seq{0};
      broker_ = std::make_unique<comm::MqttClient>();
      if (!broker_->connect(dest_host_, static_cast<int>(dest_port_), strfmt("nnsx-edgesink-", getpid(), "-", seq++),
                            60, true, 5000, &err)) {
        post_error("edgesink: broker " + dest_host_ + ":" + std::to_string(dest_port_) + ": " + err);
        return false;
      }
      running_ = true;
      return true;
    }
    if (!listener_.listen(host_, port_, &err)) {
      post_error("edgesink: " + err);
      return false;
    }
    if (connect_type_ == kHybrid) {
      announcer_ = std::make_unique<HybridAnnouncer>();
      if (!announcer_->announce(dest_host_, static_cast<int>(dest_port_), topic_, host_, listener_.port(), &err)) {
        post_error("edgesink: HYBRID announce: " + err);
        return false;
      }
    }
    running_ = true;
    accept_thr_ = std::thread([this] {
      while (running_) {
        auto c = listener_.accept(100);
        if (!c) continue;
        comm::Message hello;
        hello.type = comm::MsgType::HELLO;
        std::lock_guard<std::mutex> lk(mu_);
        hello.caps = caps_str_;
        if (c->send(hello)) {
          subs_.push_back(c);
          // subscribers only talk control traffic (IPC handshake, ring ACKs): drain it
          readers_.emplace_back([this, c] {
            comm::Message m;
            bool to = false;
            while (running_ && c->alive()) (void)c->recv(&m, 100, &to);
          });
        }
        cv_.notify_all();
      }
    });
    return true;
  }
  bool stop() override {
    running_ = false;
    g_.reset();
    hub_.reset();
    announcer_.reset();
    if (broker_) {
      if (broker_->connected()) broker_->publish(broker_topic(connect_type_, topic_, "caps"), "", 0, 1, true);
      broker_->close();
      broker_.reset();
    }
    listener_.close();
    if (accept_thr_.joinable()) accept_thr_.join();
    std::vector<std::thread> rs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& c : subs_) c->close();
      subs_.clear();
      rs.swap(readers_);
    }
    for (auto& t : rs)
      if (t.joinable()) t.join();
    return true;
  }
  void unlock() override {
    running_ = false;
    cv_.notify_all();
    if (auto h = hub_) h->cancel_publish();
    if (auto g = g_) g->cancel();
  }
  bool set_caps(const Caps& caps) override {
    if (connect_type_ == kRccl) {
      if (!g_ && !(g_ = rp_.open(this, rccl_channel("edge", topic_, static_cast<unsigned>(port_))))) return false;
      comm::Packet p;
      p.caps = caps.to_string();
      p.flags = kPktCaps;
      return publish_rccl(p, true);
    }
    comm::Message m;
    m.type = comm::MsgType::CAPS;
    std::lock_guard<std::mutex> lk(mu_);
    caps_str_ = caps.to_string();
    m.caps = caps_str_;
    if (broker_) {
      const std::string h = broker_header(m);
      return broker_->publish(broker_topic(connect_type_, topic_, "caps"), h.data(), h.size(), 1, true) &&
             broker_publish(*broker_, broker_topic(connect_type_, topic_, "data"), m);
    }
    for (auto& c : subs_) c->send(m);
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
    if (connect_type_ == kRccl) {
      if (!g_) return FlowReturn::NOT_NEGOTIATED;
      return publish_rccl(packet_of(*buf), false) ? FlowReturn::OK : FlowReturn::ERROR;
    }
    if (wait_subscribers_ > 0 && !waited_) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_for(lk, std::chrono::milliseconds(wait_timeout_ms_),
                   [&] { return subs_.size() >= wait_subscribers_ || !running_; });
      waited_ = true;
    }
    comm::Message m;
    m.type = comm::MsgType::DATA;
    m.pts = buf->pts;
    m.dts = buf->dts;
    m.duration = buf->duration;
    m.blobs = buf->mems;
    publish(m);
    return FlowReturn::OK;
  }
  void on_eos() override {
    if (connect_type_ == kRccl) {
      if (!g_) return;
      comm::Packet p;
      p.eos = true;
      publish_rccl(p, true);
      return;
    }
    comm::Message m;
    m.type = comm::MsgType::EOS;
    publish(m);
  }

 private:
  // broadcast: one collective per frame, root = this publisher; scatter:
  // frames round-robin over the other members, control packets to all
  bool publish_rccl(comm::Packet p, bool control) {
    std::string err;
    bool ok = true;
    if (rccl_mode_ == 0) {
      ok = g_->broadcast(g_->rank(), &p, &err);
    } else if (rccl_mode_ == kRcclAllGather) {
      if (!hub_) hub_ = EdgeHub::get(g_->name());
      ok = hub_->publish(*g_, p, &err);
    } else if (control) {
      for (int r = 0; r < g_->size() && ok; ++r)
        if (r != g_->rank()) ok = g_->send(r, p, &err);
    } else if (g_->size() > 1) {
      int r = static_cast<int>(rr_++ % static_cast<unsigned>(g_->size() - 1));
      if (r >= g_->rank()) ++r;
      ok = g_->send(r, p, &err);
    }
    if (!ok && running_) post_error("edgesink: " + err);
    return ok;
  }

  void publish(const comm::Message& m) {
    if (broker_) {
      if (!broker_publish(*broker_, broker_topic(connect_type_, topic_, "data"), m) && running_)
        post_error("edgesink: lost the broker connection");
      return;
    }
    std::vector<std::shared_ptr<comm::Connection>> subs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      subs = subs_;
    }
    for (auto& c : subs) c->send(m);
    std::lock_guard<std::mutex> lk(mu_);
    subs_.erase(std::remove_if(subs_.begin(), subs_.end(), [](auto& c) { return !c->alive(); }), subs_.end());
  }
  size_t subscribers() {
    std::lock_guard<std::mutex> lk(mu_);
    return subs_.size();
  }

  std::string host_ = "localhost", dest_host_ = "localhost", topic_;
  int port_ = 3000, connect_type_ = 0;
  unsigned dest_port_ = 1883, wait_subscribers_ = 0, wait_timeout_ms_ = 10000;
  comm::Listener listener_;
  std::atomic<bool> running_{false};
  bool waited_ = false;
  std::thread accept_thr_;
  std::vector<std::thread> readers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::shared_ptr<comm::Connection>> subs_;
  std::string caps_str_;
  RankProps rp_;
  int rccl_mode_ = 0;
  unsigned rr_ = 0;
  std::shared_ptr<comm::Group> g_;
  std::shared_ptr<EdgeHub> hub_;  // rccl-mode=allgather
  std::unique_ptr<HybridAnnouncer> announcer_;
  std::unique_ptr<comm::MqttClient> broker_;  // connect-type=MQTT / AITT
};

// =============================================================== edgesrc ====
class EdgeSrc : public BaseSrc {
 public:
  explicit EdgeSrc(const std::string& name) : BaseSrc("edgesrc", name, Caps::Any()) {
    prop_string("host", &host_, "The hostname of the pipeline");
    prop_uint("port", &port_, "The port of the pipeline (unused over TCP)");
    prop_string("dest-host", &dest_host_, "The hostname of the publishing edgesink");
    prop_uint("dest-port", &dest_port_, "The port of the publishing edgesink");
    prop_enum("connect-type", &connect_type_, kConnectTypes, "The connections type between edgesink and edgesrc");
    prop_string("topic", &topic_, "The main topic of the host");
    prop_int("device", &device_, "nnsx: upload received tensors to this GPU (-1 = pinned host memory)");
    prop_readonly("ipc-blobs", [this] { return std::to_string(conn_ ? conn_->ipc_blobs_received() : 0); },
                  "nnsx: tensors received through the HIPIPC device ring");
    prop_readonly("shm-blobs", [this] { return std::to_string(conn_ ? conn_->shm_blobs_received() : 0); },
                  "nnsx: tensors received by reference into the publisher's shared memory (connect-type=SHM)");
    rp_.install([this](PropSpec p) -> PropSpec& { return add_prop(p); }, false);
    prop_enum("rccl-mode", &rccl_mode_, kRcclModes, "nnsx (connect-type=RCCL): must match the publishing edgesink");
    prop_readonly("comm-bytes", [this] { return std::to_string(g_ ? g_->bytes_received() : 0); },
                  "nnsx: payload bytes received on the rank group");
    prop_readonly("comm-group", [this] { return g_ ? strfmt(g_->backend_name(), ":", g_->size()) : std::string(); },
                  "nnsx: data plane and member count of the rank group (e.g. rccl:8)");
    is_live_ = true;
  }

 protected:
  bool on_start() override {
    if (!check_connect_type(this, connect_type_, true)) return false;
    caps_str_.clear();
    if (connect_type_ == kRccl) return true;
    std::string err;
    if (via_broker(connect_type_)) {
      static std::atomic<unsigned> seq{0};
      broker_ = std::make_unique<comm::MqttClient>();
      if (!broker_->connect(dest_host_, static_cast<int>(dest_port_), strfmt("nnsx-edgesrc-", getpid(), "-", seq++), 60,
                            true, 5000, &err) ||
          !broker_->subscribe(broker_topic(connect_type_, topic_, "caps"), 1) ||
          !broker_->subscribe(broker_topic(connect_type_, topic_, "data"), 0)) {
        post_error("edgesrc: broker " + dest_host_ + ":" + std::to_string(dest_port_) + ": " +
                   (err.empty() ? "subscription failed" : err));
        return false;
      }
      return true;
    }
    conn_ = connect_endpoint(connect_type_, dest_host_, dest_port_, topic_, 10000, &err);
    if (!conn_) {
      post_error("edgesrc: " + err);
      return false;
    }
    caps_str_.clear();
    return true;
  }
  void on_stop() override {
    if (conn_) conn_->close();
    if (broker_) broker_->close();
    if (hub_) hub_->unsubscribe(hub_src_);
    hub_.reset();
    g_.reset();
  }
  void on_unlock() override {
    if (conn_) conn_->close();
    if (auto h = hub_) h->cancel_take(hub_src_);
    if (auto g = g_) g->cancel();
  }

  // connect-type=MQTT / AITT: next message from the topic (false: timeout / lost)
  bool recv_broker(comm::Message* m, int timeout_ms, bool* timed_out) {
    comm::MqttMessage mm;
    *timed_out = false;
    while (broker_->recv(&mm, timeout_ms, timed_out)) {
      if (mm.payload.empty()) continue;  // a withdrawn retained caps entry
      if (broker_parse(mm.payload, m)) return true;
      NNSX_LOGW(name(), "dropping a malformed message on ", mm.topic);
    }
    return false;
  }

  // connect-type=RCCL: next packet from the publisher (false: cancelled / lost)
  bool recv_rccl(comm::Packet* p) {
    std::string err;
    if (rccl_mode_ == kRcclAllGather) {
      // the local edgesink of the topic runs the rounds (EdgeHub); this source
      // takes its publisher's share
      while (!flushing_.load()) {
        bool to = false;
        if (hub_->take(hub_src_, p, 100, &to)) return true;
        if (!to) break;
      }
      return false;
    }
    if (rccl_mode_ == 0) {
      const int root = rp_.peer_in(*g_);
      if (root < 0 || root == g_->rank()) {
        post_error("edgesrc: peer-rank is not another member of the group");
        return false;
      }
      *p = comm::Packet();
      if (g_->broadcast(root, p, &err)) return true;
    } else {
      while (!flushing_.load()) {
        bool to = false;
        if (g_->recv(p, 100, &to, &err)) return true;
        if (!to) break;
      }
    }
    if (!flushing_.load() && !err.empty()) post_error("edgesrc: " + err);
    return false;
  }

  // the publisher's caps arrive with HELLO (or a later CAPS message)
  bool negotiate() override {
    if (connect_type_ == kRccl && rccl_mode_ == kRcclAllGather) {
      // no group of its own: subscribe to the topic's hub (fed by the local edgesink)
      if (rp_.peer < 0) {
        post_error("edgesrc: rccl-mode=allgather needs peer-rank (the publishing member)");
        return false;
      }
      if (!hub_) {
        hub_src_ = rp_.peer;
        hub_ = EdgeHub::get(rccl_channel("edge", topic_, dest_port_));
        hub_->subscribe(hub_src_);
      }
      while (caps_str_.empty()) {
        comm::Packet p;
        if (!recv_rccl(&p) || p.eos) return false;
        if (!p.caps.empty()) caps_str_ = p.caps;
      }
      return BaseSrc::negotiate();
    }
    if (connect_type_ == kRccl) {
      rp_.device = device_;
      if (!g_ && !(g_ = rp_.open(this, rccl_channel("edge", topic_, dest_port_)))) return false;
      while (caps_str_.empty()) {
        comm::Packet p;
        if (!recv_rccl(&p) || p.eos) return false;
        if (!p.caps.empty()) caps_str_ = p.caps;
      }
      return BaseSrc::negotiate();
    }
    while (caps_str_.empty()) {
      comm::Message m;
      bool timed_out = false;
      if (!(broker_ ? recv_broker(&m, 100, &timed_out) : conn_->recv(&m, 100, &timed_out))) {
        if (timed_out && !flushing_.load()) continue;
        return false;
      }
      if (m.type == comm::MsgType::HELLO && connect_type_ == kHipIpc) conn_->send_ipc_hello();
      if (m.type == comm::MsgType::HELLO && connect_type_ == kShm) conn_->send_shm_hello();
      if ((m.type == comm::MsgType::HELLO || m.type == comm::MsgType::CAPS) && !m.caps.empty()) caps_str_ = m.caps;
      if (m.type == comm::MsgType::EOS) return false;
    }
    return BaseSrc::negotiate();
  }
  Caps get_caps(const Caps* filter) override {
    Caps c = caps_str_.empty() ? Caps::Any() : Caps::from_string(caps_str_);
    return filter ? c.intersect(*filter) : c;
  }

  FlowReturn create(BufferPtr* out) override {
    while (connect_type_ == kRccl) {
      comm::Packet p;
      if (!recv_rccl(&p)) return flushing_.load() ? FlowReturn::FLUSHING : FlowReturn::ERROR;
      if (p.eos) return FlowReturn::EOS;
      if (p.flags & kPktCaps) {
        if (p.caps != caps_str_) {
          caps_str_ = p.caps;
          src_pad()->push_event(Event::make_caps(Caps::from_string(caps_str_)));
        }
        continue;
      }
      *out = buffer_of(p, device_, streams_);
      return FlowReturn::OK;
    }
    while (true) {
      comm::Message m;
      bool timed_out = false;
      if (!(broker_ ? recv_broker(&m, 100, &timed_out) : conn_->recv(&m, 100, &timed_out))) {
        if (timed_out && !flushing_.load()) continue;
        return flushing_.load() ? FlowReturn::FLUSHING : FlowReturn::EOS;
      }
      if (m.type == comm::MsgType::EOS) return FlowReturn::EOS;
      if (m.type == comm::MsgType::CAPS && m.caps != caps_str_) {
        caps_str_ = m.caps;
        src_pad()->push_event(Event::make_caps(Caps::from_string(caps_str_)));
        continue;
      }
      if (m.type != comm::MsgType::DATA) continue;
      auto b = make_buffer();
      b->mems = place_blobs(std::move(m.blobs), device_, streams_);
      b->pts = m.pts;
      b->dts = m.dts;
      b->duration = m.duration;
      *out = b;
      return FlowReturn::OK;
    }
  }

 private:
  std::string host_ = "localhost", dest_host_ = "localhost", topic_;
  unsigned port_ = 0, dest_port_ = 3000;
  int connect_type_ = 0, device_ = -1;
  std::shared_ptr<comm::Connection> conn_;
  std::string caps_str_;
  StreamSet streams_;
  RankProps rp_;
  int rccl_mode_ = 0;
  std::shared_ptr<comm::Group> g_;
  std::shared_ptr<EdgeHub> hub_;  // rccl-mode=allgather: the topic's hub
  int hub_src_ = -1;              // the publishing member (global rank) this source takes
  std::unique_ptr<comm::MqttClient> broker_;  // connect-type=MQTT / AITT
};

// ====================================================== tensor_allgather ====
// N-rank fan-in with every rank receiving every stream (nnsx; the reference
// has no cross-process mux -- tensor_mux over edge/query sockets is the
// closest: nnstreamer_plugin_api_impl.c:266-441).  Each member contributes
// its frame; the output carries all members' tensors in member order:
//   mode=concat: num_tensors adds up (like tensor_mux),
//   mode=stack:  one tensor per member, joined along `axis` (like
//                tensor_merge); the joined tensor IS the ncclAllGather output.
// Caps, frames and EOS are one collective each, so members stay in lock step;
// the first EOS of any member ends the stream on every member.
class TensorAllGather : public Element {
 public:
  explicit TensorAllGather(const std::string& name) : Element("tensor_allgather", name) {
    add_template("sink", PadDirection::SINK, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_static()));
    add_template("src", PadDirection::SRC, PadPresence::ALWAYS, Caps::from_string(tensor_caps_template_static()));
    rp_.install([this](PropSpec p) -> PropSpec& { return add_prop(p); });
    prop_string("channel", &channel_, "nnsx: group name shared by the members");
    prop_enum("mode", &mode_, {"concat", "stack"}, "concat: append every member's tensors; stack: join along axis");
    prop_int("axis", &axis_, "stack: axis to join along (every dim above it must be 1)");
    prop_readonly("comm-bytes",
                  [this] { return g_ ? strfmt(g_->bytes_sent(), ":", g_->bytes_received()) : std::string("0:0"); },
                  "nnsx: payload bytes sent:received on the rank group");
    prop_readonly("comm-group", [this] { return g_ ? strfmt(g_->backend_name(), ":", g_->size()) : std::string(); },
                  "nnsx: data plane and member count of the rank group (e.g. rccl:8)");
  }

  bool stop() override {
    g_.reset();
    done_ = false;
    return true;
  }
  void unlock() override {
    if (auto g = g_) g->cancel();
  }

  Caps query_caps(Pad* pad, const Caps* filter) override {
    Caps c = pad->direction() == PadDirection::SRC && have_out_ ? out_caps_ : pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

  bool sink_event(Pad*, Event& ev) override {
    if (ev.type == EventType::CAPS) {
      TensorsConfig in;
      if (!tensor_config_from_caps(ev.caps, &in) || !in.is_static()) {
        post_error("tensor_allgather: static tensor caps required");
        return false;
      }
      if (!g_ && !(g_ = rp_.open(this, "allgather:" + channel_))) return false;
      comm::Packet p;
      p.caps = ev.caps.to_string();
      p.flags = kPktCaps;
      std::vector<comm::Packet> all;
      std::string err;
      if (!g_->allgather(p, &all, &err)) {
        post_error("tensor_allgather: " + err);
        return false;
      }
      TensorsConfig out;
      if (!merge_configs(all, &out)) return false;
      out_caps_ = tensor_src_caps(src_pad(), out);
      have_out_ = true;
      return src_pad()->push_event(Event::make_caps(out_caps_));
    }
    if (ev.type == EventType::EOS) {
      if (g_ && !done_) {
        comm::Packet p;
        p.eos = true;
        std::vector<comm::Packet> all;
        std::string err;
        g_->allgather(p, &all, &err);
        done_ = true;
      }
      return forward_event_downstream(ev);
    }
    return forward_event_downstream(ev);
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    if (done_) return FlowReturn::EOS;
    if (!g_) return FlowReturn::NOT_NEGOTIATED;
    std::vector<comm::Packet> all;
    std::string err;
    MemoryPtr stacked;
    if (!g_->allgather(packet_of(*buf), &all, &err, mode_ == 1 ? &stacked : nullptr)) {
      post_error("tensor_allgather: " + err);
      return FlowReturn::ERROR;
    }
    for (auto& p : all)
      if (p.eos) {
        // another member finished: end here too (its EOS round is this one)
        done_ = true;
        Event eos = Event::make_eos();
        src_pad()->push_event(eos);
        return FlowReturn::EOS;
      }
    auto out = make_buffer();
    out->copy_metadata_from(*buf);
    if (mode_ == 1) {
      if (!stacked) {
        post_error("tensor_allgather: mode=stack needs one equal-size tensor per member");
        return FlowReturn::ERROR;
      }
      out->mems.push_back(stacked);
    } else {
      for (auto& p : all)
        for (auto& m : p.blobs) out->mems.push_back(m);
    }
    return src_pad()->push(out);
  }

 private:
  bool merge_configs(const std::vector<comm::Packet>& all, TensorsConfig* out) {
    std::vector<TensorsConfig> cfgs;
    for (auto& p : all) {
      TensorsConfig c;
      if (!tensor_config_from_caps(Caps::from_string(p.caps), &c) || !c.is_static()) {
        post_error("tensor_allgather: member " + std::to_string(p.src) + " has no static tensor caps");
        return false;
      }
      cfgs.push_back(c);
    }
    out->rate_n = cfgs[0].rate_n;
    out->rate_d = cfgs[0].rate_d;
    if (mode_ == 0) {
      unsigned n = 0;
      for (auto& c : cfgs) n += c.info.num_tensors;
      if (n > static_cast<unsigned>(kSizeLimit)) {
        post_error("tensor_allgather: more than 16 tensors in total; use mode=stack");
        return false;
      }
      out->info.resize(n);
      unsigned k = 0;
      for (auto& c : cfgs)
        for (unsigned i = 0; i < c.info.num_tensors; ++i) out->info.at(k++) = c.info.at(i);
      return true;
    }
    if (axis_ < 0 || axis_ >= kRankLimit) {
      post_error("tensor_allgather: axis out of range");
      return false;
    }
    TensorInfo o = cfgs[0].info.at(0);
    for (auto& c : cfgs) {
      const TensorInfo& t = c.info.at(0);
      bool ok = c.info.num_tensors == 1 && t.type == o.type;
      for (int d = 0; d < kRankLimit && ok; ++d) {
        if (d > axis_) ok = t.dim[d] == 1;
        else if (d < axis_) ok = t.dim[d] == o.dim[d];
      }
      ok = ok && t.dim[axis_] == o.dim[axis_];
      if (!ok) {
        post_error("tensor_allgather: mode=stack needs one tensor per member, equal shape and type, "
                   "and dims above `axis` equal to 1");
        return false;
      }
    }
    o.dim[axis_] *= static_cast<uint32_t>(cfgs.size());
    out->info.resize(1);
    out->info.at(0) = o;
    return true;
  }

  RankProps rp_;
  std::string channel_ = "default";
  int mode_ = 0, axis_ = 3;
  std::shared_ptr<comm::Group> g_;
  bool done_ = false, have_out_ = false;
  Caps out_caps_;
};

}  // namespace

void register_comm_elements() {
  register_element("tensor_allgather", "Muxer/Tensor/Rank", "Gathers every rank's tensors on every rank (RCCL all-gather)",
                   [](const std::string& n) { return std::make_unique<TensorAllGather>(n); });
  register_element("tensor_query_serversrc", "Source/Tensor/Query", "Receives tensors from query clients",
                   [](const std::string& n) { return std::make_unique<QueryServerSrc>(n); });
  register_element("tensor_query_serversink", "Sink/Tensor/Query", "Sends results back to the query clients",
                   [](const std::string& n) { return std::make_unique<QueryServerSink>(n); });
  register_element("tensor_query_client", "Filter/Tensor/Query", "Offloads tensors to a query server",
                   [](const std::string& n) { return std::make_unique<QueryClient>(n); });
  register_element("edgesink", "Sink/Edge", "Publishes tensors to edgesrc subscribers",
                   [](const std::string& n) { return std::make_unique<EdgeSink>(n); });
  register_element("edgesrc", "Source/Edge", "Subscribes to an edgesink publisher",
                   [](const std::string& n) { return std::make_unique<EdgeSrc>(n); });
}

}  // namespace nnsx
