// Rank groups over RCCL (data) + a TCP key/value store (control).  See group.h.
#include "comm/group.h"

#include <rccl/rccl.h>

#include <climits>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>

#include "core/log.h"
#include "core/registry.h"
#include "core/util.h"
#include "runtime/hip_util.h"

namespace nnsx {
namespace comm {

namespace {

// ================================================================ store ====
// Request:  Message{type DATA, caps "op\nkey", seq = arg, duration = wait ms, blobs[0] = value}
// Response: Message{type DATA, flags = status (0 ok, 1 timeout, 2 error), pts = integer result, blobs[0] = value}
class StoreServer {
 public:
  ~StoreServer() { stop(); }

  bool start(const std::string& host, int port, bool* in_use, std::string* err) {
    std::string e;
    if (!listener_.listen(host, port, &e)) {
      if (in_use) *in_use = e.find("in use") != std::string::npos;
      if (err) *err = e;
      return false;
    }
    running_ = true;
    acc_ = std::thread([this] {
      while (running_) {
        auto c = listener_.accept(100);
        if (!c) continue;
        std::lock_guard<std::mutex> lk(thr_mu_);
        workers_.emplace_back([this, c] { serve(c); });
      }
    });
    return true;
  }

  void stop() {
    if (!running_.exchange(false)) return;
    listener_.close();
    cv_.notify_all();
    if (acc_.joinable()) acc_.join();
    std::vector<std::thread> ws;
    {
      std::lock_guard<std::mutex> lk(thr_mu_);
      ws.swap(workers_);
    }
    for (auto& t : ws)
      if (t.joinable()) t.join();
  }

 private:
  struct Entry {
    std::string val;
    int readers = 0;  // 0: persistent
  };

  void serve(std::shared_ptr<Connection> c) {
    while (running_ && c->alive()) {
      Message m;
      bool to = false;
      if (!c->recv(&m, 100, &to)) {
        if (to) continue;
        break;
      }
      const size_t nl = m.caps.find('\n');
      if (nl == std::string::npos) break;
      const std::string op = m.caps.substr(0, nl), key = m.caps.substr(nl + 1);
      std::string val;
      if (!m.blobs.empty() && m.blobs[0]->size())
        val.assign(static_cast<const char*>(m.blobs[0]->map_host()), m.blobs[0]->size());
      Message r;
      r.type = MsgType::DATA;
      r.flags = 0;
      const int64_t arg = static_cast<int64_t>(m.seq);
      if (op == "set") {
        std::lock_guard<std::mutex> lk(mu_);
        kv_[key] = Entry{std::move(val), static_cast<int>(arg)};
        cv_.notify_all();
      } else if (op == "get") {
        const int64_t wait_ms = m.duration;
        const int64_t deadline = now_ns() + wait_ms * 1000000;
        std::unique_lock<std::mutex> lk(mu_);
        while (true) {
          auto it = kv_.find(key);
          if (it != kv_.end()) {
            r.blobs.push_back(Memory::from_bytes(it->second.val.data(), it->second.val.size()));
            if (it->second.readers > 0 && --it->second.readers == 0) kv_.erase(it);
            break;
          }
          if (!running_ || (wait_ms >= 0 && now_ns() >= deadline)) {
            r.flags = 1;
            break;
          }
          // bounded waits so a stopping server is noticed
          cv_.wait_for(lk, std::chrono::milliseconds(50));
        }
      } else if (op == "add") {
        std::lock_guard<std::mutex> lk(mu_);
        auto& e = kv_[key];
        const int64_t v = (e.val.empty() ? 0 : std::strtoll(e.val.c_str(), nullptr, 10)) + arg;
        e.val = std::to_string(v);
        r.pts = v;
        cv_.notify_all();
      } else if (op == "del") {
        std::lock_guard<std::mutex> lk(mu_);
        kv_.erase(key);
      } else {
        r.flags = 2;
      }
      if (!c->send(r)) break;
    }
  }

  Listener listener_;
  std::atomic<bool> running_{false};
  std::thread acc_;
  std::mutex thr_mu_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, Entry> kv_;
};

std::mutex g_store_mu;
std::map<int, std::weak_ptr<StoreServer>> g_stores;

bool split_hostport(const std::string& s, std::string* host, int* port) {
  const size_t c = s.rfind(':');
  if (c == std::string::npos) return false;
  *host = c ? s.substr(0, c) : "127.0.0.1";
  *port = std::atoi(s.c_str() + c + 1);
  return *port > 0;
}

int env_int(const char* name, int def) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : def;
}

bool nccl_ok(ncclResult_t r, const char* what, std::string* err) {
  if (r == ncclSuccess || r == ncclInProgress) return true;
  if (err) *err = strfmt(what, ": ", ncclGetErrorString(r));
  return false;
}

// ---- header codec ----
void put_u32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
void put_u64(std::string& s, uint64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }
struct Reader {
  const std::string& s;
  size_t off = 0;
  bool ok = true;
  template <typename T>
  T get() {
    T v{};
    if (off + sizeof(T) > s.size()) {
      ok = false;
      return v;
    }
    std::memcpy(&v, s.data() + off, sizeof(T));
    off += sizeof(T);
    return v;
  }
  std::string bytes(size_t n) {
    if (off + n > s.size()) {
      ok = false;
      return {};
    }
    std::string r = s.substr(off, n);
    off += n;
    return r;
  }
};
constexpr uint32_t kPktMagic = 0x4b50584eu;  // "NXPK"

std::mutex g_groups_mu;
std::map<std::string, std::weak_ptr<Group>> g_groups;

// Process-local hand-off for point-to-point sends to oneself (a query client
// and server in the same process): the header still goes through the store so
// the FIFO order is shared with remote senders; the blobs stay zero-copy.
constexpr uint64_t kTagP2P = 0;  // mesh tags: p2p messages; collectives use 1 + their sequence

}  // namespace

// ================================================================ client ====
std::shared_ptr<StoreClient> StoreClient::connect(const std::string& host, int port, int timeout_ms, std::string* err) {
  auto c = Connection::connect(host, port, timeout_ms, err);
  if (!c) return nullptr;
  auto s = std::make_shared<StoreClient>();
  s->conn_ = c;
  return s;
}

bool StoreClient::call(const std::string& op, const std::string& key, const std::string* val, int64_t arg, int wait_ms,
                       std::string* out, int64_t* iout, int* status) {
  // status: 0 ok, 1 the server's own wait expired (a timeout: retryable),
  // 2 anything else (lost or failed connection, server error: not retryable)
  int st_local = 2;
  int& st = status ? *status : st_local;
  st = 2;
  std::lock_guard<std::mutex> lk(mu_);
  if (!conn_ || !conn_->alive()) return false;
  Message m;
  m.type = MsgType::DATA;
  m.caps = op + "\n" + key;
  m.seq = static_cast<uint64_t>(arg);
  m.duration = wait_ms;
  if (val) m.blobs.push_back(Memory::from_bytes(val->data(), val->size()));
  if (!conn_->send(m)) return false;
  Message r;
  // the server answers a timed get itself; allow slack for the round trip
  const int t = wait_ms < 0 ? -1 : wait_ms + 30000;
  if (!conn_->recv(&r, t)) return false;
  if (r.flags != 0) {
    st = r.flags == 1 ? 1 : 2;
    return false;
  }
  st = 0;
  if (out) {
    out->clear();
    if (!r.blobs.empty() && r.blobs[0]->size())
      out->assign(static_cast<const char*>(r.blobs[0]->map_host()), r.blobs[0]->size());
  }
  if (iout) *iout = r.pts;
  return true;
}

bool StoreClient::set(const std::string& key, const std::string& val, int readers) {
  return call("set", key, &val, readers, 0, nullptr, nullptr);
}
bool StoreClient::get(const std::string& key, std::string* val, int timeout_ms, bool* timed_out) {
  int st = 2;
  const bool ok = call("get", key, nullptr, 0, timeout_ms, val, nullptr, &st);
  if (timed_out) *timed_out = st == 1;
  return ok;
}
int64_t StoreClient::add(const std::string& key, int64_t delta) {
  int64_t v = INT64_MIN;
  if (!call("add", key, nullptr, delta, 0, nullptr, &v)) return INT64_MIN;
  return v;
}
bool StoreClient::del(const std::string& key) { return call("del", key, nullptr, 0, 0, nullptr, nullptr); }
// no lock: unblocks a call() waiting inside recv (conn_ is set once at connect)
void StoreClient::close() {
  if (conn_) conn_->close();
}
std::string StoreClient::local_ip() const { return conn_ ? conn_->local_ip() : std::string("127.0.0.1"); }

// ================================================================== mesh ====
Mesh::~Mesh() { close(); }

bool Mesh::start(StoreClient* store, const std::string& prefix, int grank, int n, int timeout_ms, std::string* err) {
  store_ = store;
  prefix_ = prefix;
  grank_ = grank;
  n_ = n;
  timeout_ms_ = timeout_ms;
  out_.assign(static_cast<size_t>(n), nullptr);
  out_mu_ = std::vector<std::mutex>(static_cast<size_t>(n));
  lost_.assign(static_cast<size_t>(n), 0);
  if (!lis_.listen("0.0.0.0", 0, err)) return false;
  const std::string addr = strfmt(store->local_ip(), ":", lis_.port());
  if (!store->set(strfmt(prefix_, "/mesh/", grank_), addr)) {
    if (err) *err = "mesh: cannot publish the link address";
    return false;
  }
  acceptor_ = std::thread([this] {
    while (!closed_.load()) {
      auto c = lis_.accept(100);
      if (!c) continue;
      std::lock_guard<std::mutex> lk(mu_);
      if (closed_.load()) {
        c->close();
        break;
      }
      in_.push_back(c);
      readers_.emplace_back([this, c] { reader(c); });
    }
  });
  return true;
}

void Mesh::reader(std::shared_ptr<Connection> c) {
  Message hello;
  if (!c->recv(&hello, timeout_ms_, nullptr) || hello.type != MsgType::HELLO) return;
  const int src = static_cast<int>(hello.client_id);
  if (src < 0 || src >= n_) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    lost_[static_cast<size_t>(src)] = 0;  // (re)connected
  }
  while (true) {
    Message m;
    if (!c->recv(&m, -1, nullptr)) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!closed_.load()) lost_[static_cast<size_t>(src)] = 1;  // broke without a goodbye
      cv_.notify_all();
      return;
    }
    if (m.type == MsgType::BYE) return;
    std::lock_guard<std::mutex> lk(mu_);
    const uint64_t tag = m.seq;
    inbox_.push_back(Item{src, tag, std::move(m)});
    cv_.notify_all();
  }
}

bool Mesh::send(int peer, uint64_t tag, Message m, std::string* err) {
  std::lock_guard<std::mutex> lk(out_mu_[static_cast<size_t>(peer)]);
  auto& c = out_[static_cast<size_t>(peer)];
  if (!c) {
    std::string addr, host;
    int port = 0;
    if (!store_->get(strfmt(prefix_, "/mesh/", peer), &addr, timeout_ms_) || !split_hostport(addr, &host, &port)) {
      if (err) *err = strfmt("mesh: no link address of member ", peer);
      return false;
    }
    c = Connection::connect(host, port, timeout_ms_, err);
    if (!c) return false;
    Message h;
    h.type = MsgType::HELLO;
    h.client_id = static_cast<uint64_t>(grank_);
    if (!c->send(h)) {
      c.reset();
      if (err) *err = strfmt("mesh: cannot greet member ", peer);
      return false;
    }
  }
  m.type = MsgType::DATA;
  m.seq = tag;
  if (!c->send(m)) {
    if (err) *err = strfmt("mesh: the link to member ", peer, " broke");
    return false;
  }
  return true;
}

void Mesh::deliver_local(uint64_t tag, Message m) {
  std::lock_guard<std::mutex> lk(mu_);
  inbox_.push_back(Item{grank_, tag, std::move(m)});
  cv_.notify_all();
}

bool Mesh::recv(uint64_t tag, int src, Message* m, int* from, int timeout_ms, bool* timed_out, std::string* err) {
  if (timed_out) *timed_out = false;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(0, timeout_ms));
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    for (auto it = inbox_.begin(); it != inbox_.end(); ++it)
      if (it->tag == tag && (src < 0 || it->src == src)) {
        *m = std::move(it->m);
        if (from) *from = it->src;
        inbox_.erase(it);
        return true;
      }
    if (closed_.load()) {
      if (err) *err = "mesh: closed";
      return false;
    }
    if (src >= 0) {
      if (lost_[static_cast<size_t>(src)]) {
        if (err) *err = strfmt("lost the link to member ", src);
        return false;
      }
    } else {
      // any-source: one member's broken link must not stop the traffic of the
      // live ones (a query server keeps serving its other clients).  The loss
      // is reported once per member; the receive fails only when no other
      // member is left that could still send.
      int alive = 0;
      for (int r = 0; r < n_; ++r) {
        if (r == grank_) continue;
        if (!lost_[static_cast<size_t>(r)]) {
          ++alive;
        } else if (lost_[static_cast<size_t>(r)] == 1) {
          lost_[static_cast<size_t>(r)] = 2;  // reported
          NNSX_LOGW("mesh", "lost the link to member ", r, " (any-source receives continue with the others)");
        }
      }
      if (alive == 0 && n_ > 1) {
        if (err) *err = "mesh: lost the links to every other member";
        return false;
      }
    }
    if (timeout_ms < 0) {
      cv_.wait(lk);
    } else if (cv_.wait_until(lk, deadline) == std::cv_status::timeout) {
      if (timed_out) *timed_out = true;
      return false;
    }
  }
}

void Mesh::close() {
  if (closed_.exchange(true)) return;
  lis_.close();
  if (acceptor_.joinable()) acceptor_.join();
  for (size_t r = 0; r < out_.size(); ++r) {
    std::lock_guard<std::mutex> lk(out_mu_[r]);
    if (!out_[r]) continue;
    Message bye;
    bye.type = MsgType::BYE;
    (void)out_[r]->send(bye);  // orderly goodbye: the peer's reader ends without a "lost" mark
    out_[r]->close();
  }
  std::vector<std::thread> readers;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& c : in_) c->shutdown();  // the readers own their descriptors until joined
    readers.swap(readers_);
    cv_.notify_all();
  }
  for (auto& t : readers)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> lk(mu_);
  in_.clear();
}

std::shared_ptr<void> host_store(const std::string& host, int port, bool* in_use, std::string* err) {
  std::lock_guard<std::mutex> lk(g_store_mu);
  if (in_use) *in_use = false;
  if (auto s = g_stores[port].lock()) return s;
  auto s = std::make_shared<StoreServer>();
  if (!s->start(host, port, in_use, err)) return nullptr;
  g_stores[port] = s;
  return s;
}

// ================================================================= group ====
Group::~Group() {
  mesh_.reset();  // goodbyes first: peers see an orderly end of our links
  for (auto* links : {&tx_, &rx_})
    for (auto& l : *links) {
      if (!l.comm) continue;
      hip::DeviceGuard g(device_);
      if (l.stream) (void)hipStreamSynchronize(l.stream);
      ncclCommDestroy(static_cast<ncclComm_t>(l.comm));
      if (l.stream) hip::stream_destroy(device_, l.stream);
    }
  if (comm_) {
    hip::DeviceGuard g(device_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    ncclCommDestroy(static_cast<ncclComm_t>(comm_));
  }
  if (stream_) hip::stream_destroy(device_, stream_);
  if (store_) store_->close();
}

std::shared_ptr<Group> Group::open(const GroupSpec& spec, std::string* err) {
  std::shared_ptr<Group> g(new Group());
  if (!g->init(spec, err)) return nullptr;
  return g;
}

bool Group::init(const GroupSpec& in, std::string* err) {
  spec_ = in;
  const int rank = spec_.rank >= 0 ? spec_.rank : env_int("RANK", 0);
  const int world = spec_.world > 0 ? spec_.world : env_int("WORLD_SIZE", 1);
  members_ = spec_.members;
  if (members_.empty())
    for (int r = 0; r < world; ++r) members_.push_back(r);
  grank_ = -1;
  for (size_t i = 0; i < members_.size(); ++i)
    if (members_[i] == rank) grank_ = static_cast<int>(i);
  if (grank_ < 0) {
    if (err) *err = strfmt("rank ", rank, " is not a member of group ", spec_.name);
    return false;
  }
  device_ = spec_.device;
  // [rccl] section (ini / NNSTREAMER_rccl_<key>): job-wide defaults for what
  // an element or spec leaves unset -- backend (auto|rccl|tcp), store
  // (host:port of the control-plane store), timeout_ms (rendezvous and
  // control-plane waits)
  const Config& cfg = Config::get();
  if (spec_.backend.empty() || spec_.backend == "auto") spec_.backend = cfg.custom_value("rccl", "backend", "auto");
  if (spec_.timeout_ms <= 0)
    spec_.timeout_ms = static_cast<int>(to_int(cfg.custom_value("rccl", "timeout_ms", "60000"), 60000));
  // ---- control plane ----
  std::string addr = spec_.store;
  if (addr.empty()) addr = cfg.custom_value("rccl", "store", "");
  if (addr.empty()) {
    if (const char* e = std::getenv("NNSX_STORE")) addr = e;
  }
  if (addr.empty()) {
    const char* ma = std::getenv("MASTER_ADDR");
    const char* mp = std::getenv("MASTER_PORT");
    addr = (ma && mp) ? strfmt(ma, ":", std::atoi(mp) + 17) : std::string("127.0.0.1:29587");
  }
  std::string host;
  int port = 0;
  if (!split_hostport(addr, &host, &port)) {
    if (err) *err = "bad store address '" + addr + "' (want host:port)";
    return false;
  }
  if (rank == members_[0]) {
    bool in_use = false;
    std::string e;
    store_host_ = host_store(host == "localhost" ? "127.0.0.1" : host, port, &in_use, &e);
    if (!store_host_ && !in_use) {
      if (err) *err = "store: " + e;
      return false;
    }
  }
  store_ = StoreClient::connect(host, port, spec_.timeout_ms, err);
  if (!store_) return false;
  // ---- join: generation-scoped prefix so a restarted pipeline never sees stale keys ----
  const int n = size();
  const int64_t j = store_->add(spec_.name + "/join", 1);
  if (j == INT64_MIN) {
    if (err) *err = "store: join failed";
    return false;
  }
  const int64_t gen = (j - 1) / n;
  prefix_ = strfmt(spec_.name, "#", gen);
  if (n > 1) {
    std::string v;
    if (j % n == 0) {
      store_->set(key("ready"), "1", n - 1);
    } else if (!store_->get(key("ready"), &v, spec_.timeout_ms)) {
      if (err) *err = strfmt("group ", spec_.name, ": timed out waiting for ", n, " members");
      return false;
    }
  }
  tx_.assign(static_cast<size_t>(n), Link{});
  rx_.assign(static_cast<size_t>(n), Link{});
  // ---- member-to-member links (headers; payloads too on the tcp backend) ----
  if (n > 1) {
    mesh_ = std::make_unique<Mesh>();
    if (!mesh_->start(store_.get(), prefix_, grank_, n, spec_.timeout_ms, err)) return false;
  }
  // ---- data plane: RCCL when every member holds a GPU ----
  bool all_dev = device_ >= 0 && hip::available();
  if (n > 1) {
    put(strfmt("dev/", grank_), all_dev ? "1" : "0", n - 1);
    for (int r = 0; r < n; ++r) {
      if (r == grank_) continue;
      std::string v;
      if (!get(strfmt("dev/", r), &v, spec_.timeout_ms)) {
        if (err) *err = "group " + spec_.name + ": member placement exchange timed out";
        return false;
      }
      all_dev = all_dev && v == "1";
    }
  }
  // a group of one has no peers: "auto" skips the communicator (and RCCL's proxy
  // thread) and the collectives stay local
  const bool want_rccl = spec_.backend == "rccl" || (spec_.backend == "auto" && all_dev && n > 1);
  if (want_rccl) {
    if (!all_dev) {
      if (err) *err = "backend=rccl needs a GPU (device >= 0) on every member";
      return false;
    }
    ncclUniqueId id;
    if (grank_ == 0) {
      if (!nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId", err)) return false;
      if (n > 1) put("ncclid", std::string(reinterpret_cast<const char*>(&id), sizeof(id)), n - 1);
    } else {
      std::string v;
      if (!get("ncclid", &v, spec_.timeout_ms) || v.size() != sizeof(id)) {
        if (err) *err = "group " + spec_.name + ": no RCCL unique id from member 0";
        return false;
      }
      std::memcpy(&id, v.data(), sizeof(id));
    }
    hip::DeviceGuard dg(device_);
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    stream_ = hip::stream_create(device_, hi);  // comm traffic ahead of bulk compute
    ncclComm_t c = nullptr;
    if (!nccl_ok(ncclCommInitRank(&c, n, id, grank_), "ncclCommInitRank", err)) return false;
    comm_ = c;
    // every per-direction p2p link, now: member pairs (a < b) in lexicographic
    // order, a -> b then b -> a.  Each member walks its own pairs in that order,
    // so the smallest pair not yet linked always has both members waiting on it
    // and the walk cannot deadlock; created lazily at a pair's first message
    // instead, a sender blocked until its peer reached recv(), and members that
    // all send before they receive waited on each other until the timeout.
    for (int a = 0; a < n; ++a)
      for (int b = a + 1; b < n; ++b) {
        if (grank_ != a && grank_ != b) continue;
        const int peer = grank_ == a ? b : a;
        Link* l = nullptr;
        if (!link(peer, grank_ == a, &l, err) || !link(peer, grank_ == b, &l, err)) return false;
      }
  }
  NNSX_LOGD("comm", "group ", spec_.name, " rank ", grank_, "/", n, " backend ", backend_name(), " store ", addr);
  return true;
}

void Group::cancel() {
  if (store_) store_->close();
  if (mesh_) mesh_->close();
  std::lock_guard<std::mutex> lk(local_mu_);
  cancelled_.store(true);
  local_cv_.notify_all();
}

bool Group::put(const std::string& k, const std::string& v, int readers) { return store_->set(key(k), v, readers); }
bool Group::get(const std::string& k, std::string* v, int timeout_ms) { return store_->get(key(k), v, timeout_ms); }

std::string Group::encode(const Packet& p, bool inline_payload) {
  std::string s;
  put_u32(s, kPktMagic);
  put_u32(s, static_cast<uint32_t>(p.blobs.size()));
  put_u64(s, static_cast<uint64_t>(p.pts));
  put_u64(s, static_cast<uint64_t>(p.dts));
  put_u64(s, static_cast<uint64_t>(p.duration));
  put_u64(s, p.client_id);
  put_u32(s, p.flags);
  put_u32(s, p.eos ? 1u : 0u);
  put_u32(s, static_cast<uint32_t>(grank_));
  put_u32(s, static_cast<uint32_t>(p.caps.size()));
  s += p.caps;
  for (auto& b : p.blobs) {
    put_u64(s, b->size());
    put_u32(s, b->has_meta() ? 1u : 0u);
    if (b->has_meta()) {
      char h[kMetaHeaderSize];
      b->meta().write(h);
      s.append(h, kMetaHeaderSize);
    }
  }
  if (inline_payload)
    for (auto& b : p.blobs) {
      if (b->size()) s.append(static_cast<const char*>(b->map_host()), b->size());
      bytes_sent_ += b->size();
    }
  return s;
}

bool Group::decode(const std::string& s, Packet* p, bool inline_payload, std::vector<size_t>* sizes,
                   std::vector<std::string>* metas) {
  Reader r{s};
  if (r.get<uint32_t>() != kPktMagic) return false;
  const uint32_t nb = r.get<uint32_t>();
  p->pts = static_cast<int64_t>(r.get<uint64_t>());
  p->dts = static_cast<int64_t>(r.get<uint64_t>());
  p->duration = static_cast<int64_t>(r.get<uint64_t>());
  p->client_id = r.get<uint64_t>();
  p->flags = r.get<uint32_t>();
  p->eos = r.get<uint32_t>() != 0;
  p->src = static_cast<int>(r.get<uint32_t>());
  p->caps = r.bytes(r.get<uint32_t>());
  sizes->clear();
  metas->clear();
  for (uint32_t i = 0; i < nb && r.ok; ++i) {
    sizes->push_back(static_cast<size_t>(r.get<uint64_t>()));
    metas->push_back(r.get<uint32_t>() ? r.bytes(kMetaHeaderSize) : std::string());
  }
  p->blobs.clear();
  if (inline_payload) {
    for (uint32_t i = 0; i < nb && r.ok; ++i) {
      auto m = Memory::alloc_pinned((*sizes)[i]);
      const std::string b = r.bytes((*sizes)[i]);
      if (!b.empty()) std::memcpy(m->data(), b.data(), b.size());
      if (!(*metas)[i].empty()) {
        MetaInfo mi;
        if (MetaInfo::parse((*metas)[i].data(), (*metas)[i].size(), &mi)) m->set_meta(mi);
      }
      bytes_recv_ += m->size();
      p->blobs.push_back(m);
    }
  }
  return r.ok;
}

void* Group::dev_ptr(const MemoryPtr& m) { return dev_ptr_on(m, stream_); }

void* Group::dev_ptr_on(const MemoryPtr& m, hipStream_t s) {
  if (m->on_device() && m->device() == device_) {
    m->wait_ready(s);
    return m->data();
  }
  // host blob (or another GPU's): stage it onto ours, ordered on the comm stream
  return const_cast<void*>(m->map_device(device_, s));
}

std::vector<MemoryPtr> Group::alloc_recv(const std::vector<size_t>& sizes, const std::vector<std::string>& metas) {
  std::vector<MemoryPtr> out;
  for (size_t i = 0; i < sizes.size(); ++i) {
    auto m = sizes[i] ? Memory::alloc_device(sizes[i], device_, stream_) : Memory::alloc_host(0);
    if (!metas[i].empty()) {
      MetaInfo mi;
      if (MetaInfo::parse(metas[i].data(), metas[i].size(), &mi)) m->set_meta(mi);
    }
    bytes_recv_ += sizes[i];
    out.push_back(m);
  }
  return out;
}

void Group::finish_inputs(const std::vector<MemoryPtr>& in, hipStream_t s) {
  for (auto& m : in)
    if (m->size()) m->record_use(s ? s : stream_, device_);
}

// Per-direction pair communicator (created for every pair at init, in a fixed
// order; see Group::init).  The sender publishes a unique id and waits
// (bounded, cancellable: the store) until the receiver has fetched it; only
// then do both enter the blocking ncclCommInitRank, so a member that never
// joins costs its peer a timeout, not a hang.
bool Group::link(int peer, bool tx, Link** out, std::string* err) {
  Link& l = (tx ? tx_ : rx_).at(static_cast<size_t>(peer));
  *out = &l;
  if (l.comm) return true;
  const int src = tx ? grank_ : peer, dst = tx ? peer : grank_;
  const std::string k = strfmt("p2p/", src, ">", dst);
  ncclUniqueId id;
  if (tx) {
    if (!nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId", err)) return false;
    std::string v;
    if (!put(k + "/id", std::string(reinterpret_cast<const char*>(&id), sizeof(id)), 1) ||
        !get(k + "/joined", &v, spec_.timeout_ms)) {
      if (err) *err = strfmt("p2p link to member ", peer, ": the receiver did not join");
      return false;
    }
  } else {
    std::string v;
    if (!get(k + "/id", &v, spec_.timeout_ms) || v.size() != sizeof(id)) {
      if (err) *err = strfmt("p2p link from member ", peer, ": no RCCL unique id");
      return false;
    }
    std::memcpy(&id, v.data(), sizeof(id));
    if (!put(k + "/joined", "1", 1)) {
      if (err) *err = "p2p link: store lost";
      return false;
    }
  }
  hip::DeviceGuard dg(device_);
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  ncclComm_t c = nullptr;
  if (!nccl_ok(ncclCommInitRank(&c, 2, id, tx ? 0 : 1), "ncclCommInitRank(p2p)", err)) return false;
  l.stream = hip::stream_create(device_, hi);
  l.comm = c;
  NNSX_LOGD("comm", "group ", spec_.name, ": p2p link ", src, " -> ", dst, " up");
  return true;
}

bool Group::self_copy(const std::vector<MemoryPtr>& in, std::vector<MemoryPtr>* out, std::string* err) {
  hip::DeviceGuard dg(device_);
  auto comm = static_cast<ncclComm_t>(comm_);
  out->clear();
  std::vector<void*> src;
  for (auto& b : in) {
    src.push_back(b->size() ? dev_ptr(b) : nullptr);
    auto m = b->size() ? Memory::alloc_device(b->size(), device_, stream_) : Memory::alloc_host(0);
    if (b->has_meta()) m->set_meta(b->meta());
    out->push_back(m);
  }
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (size_t i = 0; i < in.size(); ++i) {
    if (!in[i]->size()) continue;
    if (!nccl_ok(ncclSend(src[i], in[i]->size(), ncclUint8, grank_, comm, stream_), "ncclSend", err) ||
        !nccl_ok(ncclRecv((*out)[i]->data(), in[i]->size(), ncclUint8, grank_, comm, stream_), "ncclRecv", err)) {
      ncclGroupEnd();
      return false;
    }
    bytes_sent_ += in[i]->size();
    bytes_recv_ += in[i]->size();
  }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& m : *out)
    if (m->size()) m->mark_ready(stream_);
  finish_inputs(in);
  return true;
}

// ------------------------------------------------------------ messages ----
// packet -> mesh message: the encoded header rides in `caps`; on the tcp
// backend the payload blobs follow it on the same link
Message Group::to_message(const Packet& p) {
  Message m;
  m.caps = encode(p, false);
  if (!rccl()) {
    m.blobs = p.blobs;
    for (auto& b : p.blobs) bytes_sent_ += b->size();
  }
  return m;
}

// mesh message -> packet header (+ payload on the tcp backend)
bool Group::from_message(Message&& m, Packet* p, std::vector<size_t>* sizes, std::vector<std::string>* metas) {
  if (!decode(m.caps, p, false, sizes, metas)) return false;
  if (rccl()) return true;
  if (m.blobs.size() != sizes->size()) return false;
  for (size_t i = 0; i < m.blobs.size(); ++i) {
    if (!(*metas)[i].empty()) {
      MetaInfo mi;
      if (MetaInfo::parse((*metas)[i].data(), (*metas)[i].size(), &mi)) m.blobs[i]->set_meta(mi);
    }
    bytes_recv_ += m.blobs[i]->size();
  }
  p->blobs = std::move(m.blobs);
  return true;
}

bool Group::recv_from(uint64_t tag, int src, Packet* p, std::vector<size_t>* sizes, std::vector<std::string>* metas,
                      std::string* err, const char* what) {
  Message m;
  bool to = false;
  std::string e;
  if (!mesh_->recv(tag, src, &m, nullptr, spec_.timeout_ms, &to, &e) || !from_message(std::move(m), p, sizes, metas)) {
    if (err) *err = strfmt(what, ": no message from member ", src, to ? " (timed out)" : (e.empty() ? "" : " (" + e + ")"));
    return false;
  }
  return true;
}

// ----------------------------------------------------------- allgather ----
bool Group::allgather(const Packet& mine, std::vector<Packet>* all, std::string* err, MemoryPtr* stacked) {
  const int n = size();
  const uint64_t seq = seq_++;
  all->assign(static_cast<size_t>(n), Packet());
  (*all)[grank_] = mine;
  (*all)[grank_].src = grank_;
  if (stacked) *stacked = nullptr;
  // a group of one: nothing to exchange -- unless RCCL was forced, then the
  // real ncclAllGather runs (one rank: a copy into the gathered buffer)
  if (n == 1 && !rccl()) {
    if (stacked && mine.blobs.size() == 1) *stacked = mine.blobs[0];
    return true;
  }
  const uint64_t tag = 1 + seq;
  for (int r = 0; r < n; ++r)
    if (r != grank_ && !mesh_->send(r, tag, to_message(mine), err)) return false;
  std::vector<std::vector<size_t>> sizes(n);
  std::vector<std::vector<std::string>> metas(n);
  for (int r = 0; r < n; ++r) {
    if (r == grank_) {
      for (auto& b : mine.blobs) {
        sizes[r].push_back(b->size());
        metas[r].push_back(std::string());
      }
      continue;
    }
    if (!recv_from(tag, r, &(*all)[r], &sizes[r], &metas[r], err, "allgather")) return false;
  }
  bool one_uniform = true;
  for (int r = 0; r < n; ++r)
    one_uniform = one_uniform && sizes[r].size() == 1 && sizes[r][0] == sizes[0][0] && sizes[0][0] > 0;
  if (!rccl()) {
    if (stacked && one_uniform) {
      const size_t s = sizes[0][0];
      auto out = Memory::alloc_pinned(s * n);
      for (int r = 0; r < n; ++r)
        std::memcpy(static_cast<char*>(out->data()) + static_cast<size_t>(r) * s, (*all)[r].blobs[0]->map_host(), s);
      *stacked = out;
    }
    return true;
  }
  // ---- RCCL payload ----
  hip::DeviceGuard dg(device_);
  size_t nb = 0;
  for (auto& s : sizes) nb = std::max(nb, s.size());
  std::vector<MemoryPtr> outs;
  for (int r = 0; r < n; ++r)
    if (r != grank_) (*all)[r].blobs.assign(sizes[r].size(), nullptr);
  std::vector<void*> srcs(mine.blobs.size());
  for (size_t j = 0; j < mine.blobs.size(); ++j) srcs[j] = mine.blobs[j]->size() ? dev_ptr(mine.blobs[j]) : nullptr;
  auto comm = static_cast<ncclComm_t>(comm_);
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (size_t j = 0; j < nb; ++j) {
    bool uniform = true;
    for (int r = 0; r < n; ++r) uniform = uniform && j < sizes[r].size() && sizes[r][j] == sizes[0][j];
    if (uniform && sizes[0][j] > 0) {
      const size_t s = sizes[0][j];
      auto out = Memory::alloc_device(s * n, device_, stream_);
      outs.push_back(out);
      if (stacked && one_uniform) *stacked = out;
      if (!nccl_ok(ncclAllGather(srcs[j], out->data(), s, ncclUint8, comm, stream_), "ncclAllGather", err)) {
        ncclGroupEnd();
        return false;
      }
      if (n == 1) (*all)[grank_].blobs[j] = out;  // (forced RCCL: the gathered copy)
      for (int r = 0; r < n; ++r) {
        if (r == grank_) continue;
        auto v = Memory::view(out, static_cast<size_t>(r) * s, s);
        if (!metas[r][j].empty()) {
          MetaInfo mi;
          if (MetaInfo::parse(metas[r][j].data(), metas[r][j].size(), &mi)) v->set_meta(mi);
        }
        (*all)[r].blobs[j] = v;
        bytes_recv_ += s;
      }
      bytes_sent_ += s;
      continue;
    }
    // ragged: one broadcast per owner of blob j
    for (int r = 0; r < n; ++r) {
      if (j >= sizes[r].size() || sizes[r][j] == 0) {
        if (r != grank_ && j < sizes[r].size()) (*all)[r].blobs[j] = Memory::alloc_host(0);
        continue;
      }
      const size_t s = sizes[r][j];
      if (r == grank_) {
        if (!nccl_ok(ncclBroadcast(srcs[j], srcs[j], s, ncclUint8, r, comm, stream_), "ncclBroadcast", err)) {
          ncclGroupEnd();
          return false;
        }
        bytes_sent_ += s;
        continue;
      }
      auto out = alloc_recv({s}, {metas[r][j]})[0];
      outs.push_back(out);
      (*all)[r].blobs[j] = out;
      if (!nccl_ok(ncclBroadcast(out->data(), out->data(), s, ncclUint8, r, comm, stream_), "ncclBroadcast", err)) {
        ncclGroupEnd();
        return false;
      }
    }
  }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& o : outs) o->mark_ready(stream_);
  finish_inputs(mine.blobs);
  return true;
}

// ----------------------------------------------------------- broadcast ----
bool Group::broadcast(int root, Packet* pkt, std::string* err) {
  const int n = size();
  const uint64_t seq = seq_++;
  if (n == 1 && !rccl()) return true;  // (forced RCCL: the one-rank ncclBroadcast runs)
  const uint64_t tag = 1 + seq;
  std::vector<size_t> sizes;
  std::vector<std::string> metas;
  if (grank_ == root) {
    for (int r = 0; r < n; ++r)
      if (r != root && !mesh_->send(r, tag, to_message(*pkt), err)) return false;
    for (auto& b : pkt->blobs) sizes.push_back(b->size());
  } else if (!recv_from(tag, root, pkt, &sizes, &metas, err, "broadcast")) {
    return false;
  }
  if (!rccl()) return true;
  hip::DeviceGuard dg(device_);
  auto comm = static_cast<ncclComm_t>(comm_);
  std::vector<MemoryPtr> outs;
  std::vector<void*> ptrs;
  if (grank_ == root) {
    for (auto& b : pkt->blobs) ptrs.push_back(b->size() ? dev_ptr(b) : nullptr);
  } else {
    pkt->blobs = alloc_recv(sizes, metas);
    for (auto& b : pkt->blobs) ptrs.push_back(b->size() ? b->data() : nullptr);
    outs = pkt->blobs;
  }
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (size_t j = 0; j < sizes.size(); ++j) {
    if (!sizes[j]) continue;
    if (!nccl_ok(ncclBroadcast(ptrs[j], ptrs[j], sizes[j], ncclUint8, root, comm, stream_), "ncclBroadcast", err)) {
      ncclGroupEnd();
      return false;
    }
    if (grank_ == root) bytes_sent_ += sizes[j];
  }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& o : outs)
    if (o->size()) o->mark_ready(stream_);
  if (grank_ == root) finish_inputs(pkt->blobs);
  return true;
}

// ------------------------------------------------------------- scatter ----
bool Group::scatter(int root, const std::vector<Packet>* parts, Packet* mine, std::string* err) {
  const int n = size();
  const uint64_t seq = seq_++;
  const uint64_t tag = 1 + seq;
  if (grank_ == root) {
    if (!parts || static_cast<int>(parts->size()) != n) {
      if (err) *err = "scatter: the root needs one part per member";
      return false;
    }
    *mine = (*parts)[root];
    mine->src = root;
    for (int r = 0; r < n; ++r)
      if (r != root && !mesh_->send(r, tag, to_message((*parts)[r]), err)) return false;
    if (!rccl() || n == 1) return true;
    hip::DeviceGuard dg(device_);
    auto comm = static_cast<ncclComm_t>(comm_);
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
    for (int r = 0; r < n; ++r) {
      if (r == root) continue;
      for (auto& b : (*parts)[r].blobs) {
        if (!b->size()) continue;
        if (!nccl_ok(ncclSend(dev_ptr(b), b->size(), ncclUint8, r, comm, stream_), "ncclSend", err)) {
          ncclGroupEnd();
          return false;
        }
        bytes_sent_ += b->size();
      }
    }
    if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
    for (int r = 0; r < n; ++r)
      if (r != root) finish_inputs((*parts)[r].blobs);
    return true;
  }
  std::vector<size_t> sizes;
  std::vector<std::string> metas;
  if (!recv_from(tag, root, mine, &sizes, &metas, err, "scatter")) return false;
  if (!rccl()) return true;
  hip::DeviceGuard dg(device_);
  mine->blobs = alloc_recv(sizes, metas);
  auto comm = static_cast<ncclComm_t>(comm_);
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (auto& b : mine->blobs)
    if (b->size() && !nccl_ok(ncclRecv(b->data(), b->size(), ncclUint8, root, comm, stream_), "ncclRecv", err)) {
      ncclGroupEnd();
      return false;
    }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& b : mine->blobs)
    if (b->size()) b->mark_ready(stream_);
  return true;
}

// -------------------------------------------------------- point to point ----
// header (and tcp payload) on the direct link to the peer; a member's message
// to itself goes straight into its own inbox with the blobs as they are
bool Group::send(int peer, const Packet& p, std::string* err) {
  if (peer < 0 || peer >= size()) {
    if (err) *err = strfmt("send: no member ", peer);
    return false;
  }
  if (peer == grank_) {
    Message m;
    m.caps = encode(p, false);
    m.blobs = p.blobs;
    m.flags = 1;  // in-process: blobs handed over as they are
    // a group of one on forced RCCL: the payload goes through RCCL's p2p path
    // (grouped ncclSend / ncclRecv to itself) like a peer's would
    if (size() == 1 && rccl() && !self_copy(p.blobs, &m.blobs, err)) return false;
    if (!mesh_) {
      std::lock_guard<std::mutex> lk(local_mu_);
      local_.push_back(std::move(m));
      local_cv_.notify_all();
    } else {
      mesh_->deliver_local(kTagP2P, std::move(m));
    }
    return true;
  }
  if (!mesh_->send(peer, kTagP2P, to_message(p), err)) return false;
  if (!rccl()) return true;
  hip::DeviceGuard dg(device_);
  Link* l = nullptr;
  if (!link(peer, true, &l, err)) return false;
  auto comm = static_cast<ncclComm_t>(l->comm);
  std::vector<void*> src;
  for (auto& b : p.blobs) src.push_back(b->size() ? dev_ptr_on(b, l->stream) : nullptr);
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (size_t i = 0; i < p.blobs.size(); ++i) {
    const size_t sz = p.blobs[i]->size();
    if (!sz) continue;
    if (!nccl_ok(ncclSend(src[i], sz, ncclUint8, 1, comm, l->stream), "ncclSend", err)) {
      ncclGroupEnd();
      return false;
    }
    bytes_sent_ += sz;
  }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  finish_inputs(p.blobs, l->stream);
  return true;
}

bool Group::recv(Packet* p, int timeout_ms, bool* timed_out, std::string* err) {
  if (timed_out) *timed_out = false;
  Message m;
  if (!mesh_) {  // a group of one: only its own messages
    std::unique_lock<std::mutex> lk(local_mu_);
    auto ready = [&] { return !local_.empty() || cancelled_.load(); };
    if (timeout_ms < 0) {
      local_cv_.wait(lk, ready);
    } else {
      local_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
    }
    if (local_.empty()) {
      if (timed_out) *timed_out = !cancelled_.load();
      if (err && cancelled_.load()) *err = "recv: cancelled";
      return false;
    }
    m = std::move(local_.front());
    local_.pop_front();
  } else {
    bool to = false;
    std::string e;
    if (!mesh_->recv(kTagP2P, -1, &m, nullptr, timeout_ms, &to, &e)) {
      // only the wait running out is a timeout; a broken link (the member died)
      // or a closed mesh is an error, so callers stop instead of retrying
      if (timed_out) *timed_out = to;
      if (err && !to) *err = "recv: " + e;
      return false;
    }
  }
  std::vector<size_t> sizes;
  std::vector<std::string> metas;
  if (m.flags & 1) {  // in-process
    if (!decode(m.caps, p, false, &sizes, &metas)) return false;
    p->blobs = std::move(m.blobs);
    return true;
  }
  if (!from_message(std::move(m), p, &sizes, &metas)) {
    if (err) *err = "recv: bad header";
    return false;
  }
  if (!rccl()) return true;
  hip::DeviceGuard dg(device_);
  Link* l = nullptr;
  if (!link(p->src, false, &l, err)) return false;
  auto comm = static_cast<ncclComm_t>(l->comm);
  p->blobs.clear();
  for (size_t i = 0; i < sizes.size(); ++i) {
    auto m = sizes[i] ? Memory::alloc_device(sizes[i], device_, l->stream) : Memory::alloc_host(0);
    if (!metas[i].empty()) {
      MetaInfo mi;
      if (MetaInfo::parse(metas[i].data(), metas[i].size(), &mi)) m->set_meta(mi);
    }
    bytes_recv_ += sizes[i];
    p->blobs.push_back(m);
  }
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (auto& b : p->blobs)
    if (b->size() && !nccl_ok(ncclRecv(b->data(), b->size(), ncclUint8, 0, comm, l->stream), "ncclRecv", err)) {
      ncclGroupEnd();
      return false;
    }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& b : p->blobs)
    if (b->size()) b->mark_ready(l->stream);
  return true;
}

// ------------------------------------------------------------- registry ----
std::shared_ptr<Group> group_get(const GroupSpec& spec, std::string* err) {
  const int rank = spec.rank >= 0 ? spec.rank : env_int("RANK", 0);
  const std::string k = strfmt(spec.name, "@", rank);
  {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    if (auto g = g_groups[k].lock()) return g;
  }
  auto g = Group::open(spec, err);
  if (!g) return nullptr;
  std::lock_guard<std::mutex> lk(g_groups_mu);
  g_groups[k] = g;
  return g;
}

}  // namespace comm
}  // namespace nnsx
