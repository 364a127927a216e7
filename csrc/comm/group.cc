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

// manifests of round r travel with mesh tag r + 1
constexpr uint32_t kRoundMagic = 0x44525851u;  // "QXRD"

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
    const bool got = c->recv(&m, -1, nullptr);
    std::lock_guard<std::mutex> lk(mu_);
    if (!got || m.type == MsgType::BYE) {
      // everything the member sent before is already queued (one ordered stream)
      if (!closed_.load()) lost_[static_cast<size_t>(src)] = got ? 3 : 1;
      cv_.notify_all();
      return;
    }
    inbox_.push_back(Item{src, m.seq, std::move(m)});
    cv_.notify_all();
  }
}

bool Mesh::ensure_link(int peer, std::string* err) {
  auto& c = out_[static_cast<size_t>(peer)];
  if (c) return true;
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
  return true;
}

bool Mesh::connect_all(std::string* err) {
  for (int r = 0; r < n_; ++r) {
    if (r == grank_) continue;
    std::lock_guard<std::mutex> lk(out_mu_[static_cast<size_t>(r)]);
    if (!ensure_link(r, err)) return false;
  }
  return true;
}

bool Mesh::send(int peer, uint64_t tag, Message m, std::string* err) {
  std::lock_guard<std::mutex> lk(out_mu_[static_cast<size_t>(peer)]);
  if (!ensure_link(peer, err)) return false;
  m.type = MsgType::DATA;
  m.seq = tag;
  if (!out_[static_cast<size_t>(peer)]->send(m)) {
    if (err) *err = strfmt("mesh: the link to member ", peer, " broke");
    return false;
  }
  return true;
}

bool Mesh::recv(uint64_t tag, int src, Message* m, int timeout_ms, bool* timed_out, int* gone, std::string* err) {
  if (timed_out) *timed_out = false;
  if (gone) *gone = 0;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(0, timeout_ms));
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    for (auto it = inbox_.begin(); it != inbox_.end(); ++it)
      if (it->tag == tag && it->src == src) {
        *m = std::move(it->m);
        inbox_.erase(it);
        return true;
      }
    if (closed_.load()) {
      if (err) *err = "mesh: closed";
      return false;
    }
    if (const int l = lost_[static_cast<size_t>(src)]) {
      if (gone) *gone = l;
      if (err) *err = l == 3 ? strfmt("member ", src, " left") : strfmt("lost the link to member ", src);
      return false;
    }
    if (timeout_ms < 0) {
      cv_.wait(lk);
    } else if (cv_.wait_until(lk, deadline) == std::cv_status::timeout) {
      if (timed_out) *timed_out = true;
      return false;
    }
  }
}

int Mesh::wait_tag(uint64_t tag, const std::function<bool()>& wake, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(0, timeout_ms));
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    if (closed_.load()) return -1;
    for (auto& it : inbox_)
      if (it.tag == tag) return 1;
    if (wake()) return 0;
    if (cv_.wait_until(lk, deadline) == std::cv_status::timeout) return 0;
  }
}

void Mesh::poke() {
  std::lock_guard<std::mutex> lk(mu_);
  cv_.notify_all();
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
    (void)out_[r]->send(bye);  // orderly goodbye: the peer drops us from later rounds
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
namespace {
void set_metas(std::vector<MemoryPtr>* blobs, const std::vector<std::string>& metas) {
  for (size_t i = 0; i < blobs->size() && i < metas.size(); ++i)
    if (!metas[i].empty()) {
      MetaInfo mi;
      if (MetaInfo::parse(metas[i].data(), metas[i].size(), &mi)) (*blobs)[i]->set_meta(mi);
    }
}
}  // namespace

Group::~Group() {
  stop_engine();
  mesh_.reset();  // (already closed by the progress thread: goodbyes)
  if (comm_) {
    hip::DeviceGuard g(device_);
    // the issued rounds must finish before the communicator goes; one that
    // cannot (a member died mid-round) is aborted instead of hanging here
    const int64_t deadline = now_ns() + static_cast<int64_t>(op_timeout_ms_) * 1000000;
    while (!inflight_.empty() && !aborted_.load()) {
      const hipError_t q = hipEventQuery(inflight_.front().ev);
      if (q == hipErrorNotReady && now_ns() < deadline) {
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        continue;
      }
      if (q != hipSuccess) {
        NNSX_LOGE("comm", "group ", spec_.name, ": round ", inflight_.front().round,
                  " did not complete before the group closed; aborting the communicator");
        ncclCommAbort(static_cast<ncclComm_t>(comm_));
        aborted_ = true;
        break;
      }
      hip::event_put(device_, inflight_.front().ev);
      inflight_.pop_front();
    }
    if (!aborted_.load()) {
      if (stream_) (void)hipStreamSynchronize(stream_);
      ncclCommDestroy(static_cast<ncclComm_t>(comm_));
    }
  }
  for (auto& f : inflight_) (void)hipEventDestroy(f.ev);
  if (stream_ && !aborted_.load()) hip::stream_destroy(device_, stream_);
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
  // (host:port of the control-plane store), timeout_ms (rendezvous, manifest
  // and collective waits), op_timeout_ms (device completion of a round)
  const Config& cfg = Config::get();
  if (spec_.backend.empty() || spec_.backend == "auto") spec_.backend = cfg.custom_value("rccl", "backend", "auto");
  if (spec_.timeout_ms <= 0)
    spec_.timeout_ms = static_cast<int>(to_int(cfg.custom_value("rccl", "timeout_ms", "60000"), 60000));
  op_timeout_ms_ = static_cast<int>(to_int(cfg.custom_value("rccl", "op_timeout_ms", ""), spec_.timeout_ms));
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
  // ---- member-to-member links (manifests; payloads too on the tcp backend) ----
  if (n > 1) {
    mesh_ = std::make_unique<Mesh>();
    if (!mesh_->start(store_.get(), prefix_, grank_, n, spec_.timeout_ms, err) || !mesh_->connect_all(err))
      return false;
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
  }
  outbox_.assign(static_cast<size_t>(n), {});
  unconsumed_.assign(static_cast<size_t>(n), 0);
  allowed_.assign(static_cast<size_t>(n), kWindow);
  granted_.assign(static_cast<size_t>(n), kWindow);
  recvd_since_grant_.assign(static_cast<size_t>(n), 0);
  active_.assign(static_cast<size_t>(n), 1);
  listed_upto_.assign(static_cast<size_t>(n), 0);
  engine_ = n > 1 || rccl();
  if (engine_) thr_ = std::thread([this] { progress(); });
  NNSX_LOGD("comm", "group ", spec_.name, " rank ", grank_, "/", n, " backend ", backend_name(), " store ", addr);
  return true;
}

std::string Group::failure() const {
  std::lock_guard<std::mutex> lk(mu_);
  return failed_;
}

void Group::poke() {
  if (mesh_) {
    mesh_->poke();
  } else {
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_all();
  }
}

void Group::stop_engine() {
  stop_ = true;
  poke();
  if (thr_.joinable()) thr_.join();
}

void Group::cancel() {
  if (store_) store_->close();
  cancelled_ = true;
  stop_ = true;  // the progress thread finishes the round it is in, then says goodbye
  {
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_all();
  }
  poke();
}

bool Group::put(const std::string& k, const std::string& v, int readers) { return store_->set(key(k), v, readers); }
bool Group::get(const std::string& k, std::string* v, int timeout_ms) { return store_->get(key(k), v, timeout_ms); }

std::string Group::encode(const Packet& p) {
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
  return s;
}

bool Group::decode(const std::string& s, Packet* p, std::vector<size_t>* sizes, std::vector<std::string>* metas) {
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
  return r.ok;
}

void* Group::dev_ptr(const MemoryPtr& m) {
  if (m->on_device() && m->device() == device_) {
    m->wait_ready(stream_);
    return m->data();
  }
  // host blob (or another GPU's): stage it onto ours, ordered on the comm stream
  return const_cast<void*>(m->map_device(device_, stream_));
}

std::vector<MemoryPtr> Group::alloc_recv(const std::vector<size_t>& sizes, const std::vector<std::string>& metas) {
  std::vector<MemoryPtr> out;
  for (size_t i = 0; i < sizes.size(); ++i) {
    out.push_back(sizes[i] ? Memory::alloc_device(sizes[i], device_, stream_) : Memory::alloc_host(0));
    bytes_recv_ += sizes[i];
  }
  set_metas(&out, metas);
  return out;
}

void Group::finish_inputs(const std::vector<MemoryPtr>& in) {
  for (auto& m : in)
    if (m->size()) m->record_use(stream_, device_);
}

// ------------------------------------------------------------ manifests ----
// u32 magic | u64 round | u32 grant | u32 ncoll | per collective: u64 seq,
// u32 kind, u32 root, u32 has_header, [u32 len, header] | u32 nsend | per
// message: u32 len, header.  On tcp the payload blobs follow in the same
// order (collective headers first, then the messages).
Message Group::manifest_for(int d, uint32_t grant, const std::vector<std::shared_ptr<CollOp>>& colls,
                            const std::vector<Packet>& sends) {
  Message m;
  std::string s;
  put_u32(s, kRoundMagic);
  put_u64(s, round_);
  put_u32(s, grant);
  put_u32(s, static_cast<uint32_t>(colls.size()));
  for (auto& op : colls) {
    put_u64(s, op->seq);
    put_u32(s, op->kind);
    put_u32(s, static_cast<uint32_t>(op->root));
    const Packet* h = nullptr;
    if (op->kind == CollOp::kAllGather || (op->kind == CollOp::kBroadcast && op->root == grank_)) h = &op->mine;
    if (op->kind == CollOp::kScatter && op->root == grank_) h = &op->parts.at(static_cast<size_t>(d));
    put_u32(s, h ? 1u : 0u);
    if (!h) continue;
    const std::string e = encode(*h);
    put_u32(s, static_cast<uint32_t>(e.size()));
    s += e;
    if (!rccl()) m.blobs.insert(m.blobs.end(), h->blobs.begin(), h->blobs.end());
  }
  put_u32(s, static_cast<uint32_t>(sends.size()));
  for (auto& p : sends) {
    const std::string e = encode(p);
    put_u32(s, static_cast<uint32_t>(e.size()));
    s += e;
    if (!rccl()) m.blobs.insert(m.blobs.end(), p.blobs.begin(), p.blobs.end());
  }
  m.caps = std::move(s);
  return m;
}

bool Group::parse_manifest(Message&& m, Manifest* out) {
  Reader r{m.caps};
  if (r.get<uint32_t>() != kRoundMagic || r.get<uint64_t>() != round_) return false;
  out->grant = r.get<uint32_t>();
  size_t next_blob = 0;
  auto take = [&](ManifestEntry* e) {
    if (!decode(r.bytes(r.get<uint32_t>()), &e->hdr, &e->sizes, &e->metas)) return false;
    if (rccl()) return true;
    if (next_blob + e->sizes.size() > m.blobs.size()) return false;
    e->hdr.blobs.assign(m.blobs.begin() + static_cast<std::ptrdiff_t>(next_blob),
                        m.blobs.begin() + static_cast<std::ptrdiff_t>(next_blob + e->sizes.size()));
    next_blob += e->sizes.size();
    for (size_t i = 0; i < e->sizes.size(); ++i)
      if (e->hdr.blobs[i]->size() != e->sizes[i]) return false;
    set_metas(&e->hdr.blobs, e->metas);
    return true;
  };
  const uint32_t nc = r.get<uint32_t>();
  for (uint32_t i = 0; i < nc && r.ok; ++i) {
    ManifestColl c;
    c.seq = r.get<uint64_t>();
    c.kind = r.get<uint32_t>();
    c.root = static_cast<int>(r.get<uint32_t>());
    c.has_hdr = r.get<uint32_t>() != 0;
    if (c.has_hdr && !take(&c.e)) return false;
    out->colls.push_back(std::move(c));
  }
  const uint32_t ns = r.get<uint32_t>();
  for (uint32_t i = 0; i < ns && r.ok; ++i) {
    ManifestEntry e;
    if (!take(&e)) return false;
    out->sends.push_back(std::move(e));
  }
  return r.ok;
}

// ---------------------------------------------------------- the engine ----
void Group::progress() {
  if (rccl()) (void)hipSetDevice(device_);
  while (wait_trigger()) {
    std::string e;
    if (!reap(true, &e) || !run_round(&e)) {
      fail(e);
      break;
    }
  }
  // leaving (stop / cancel / failure): an orderly goodbye on every link, so
  // the other members drop this one from their next round
  if (mesh_) mesh_->close();
  std::lock_guard<std::mutex> lk(mu_);
  const std::string why = !failed_.empty() ? failed_ : cancelled_.load() ? "cancelled" : "the group closed";
  for (auto& op : colls_) {
    op->done = true;
    op->ok = false;
    op->err = why;
  }
  colls_.clear();
  cv_.notify_all();
}

bool Group::pending_out() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!failed_.empty()) return false;
  for (int d = 0; d < size(); ++d)
    if (d != grank_ && active_[static_cast<size_t>(d)] && !outbox_[static_cast<size_t>(d)].empty()) return true;
  return false;
}

bool Group::wait_trigger() {
  while (true) {
    if (stop_.load()) {
      // an orderly close flushes what send() accepted: rounds go on while a
      // queued message has a member to go to (members that leave are dropped
      // with theirs), for at most min(timeout, 10 s); a cancel does not wait
      if (cancelled_.load() || !mesh_ || !pending_out()) return false;
      const int64_t now = now_ns();
      if (drain_deadline_ == 0)
        drain_deadline_ = now + static_cast<int64_t>(std::min(spec_.timeout_ms, 10000)) * 1000000;
      if (now > drain_deadline_) {
        NNSX_LOGW("comm", "group ", spec_.name, " (member ", grank_, "): closing with undelivered messages");
        return false;
      }
      // (a receiver that does not consume grants nothing: do not spin)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      return true;
    }
    if (work_.load()) return true;
    if (mesh_) {
      const int st = mesh_->wait_tag(round_ + 1, [this] { return work_.load() || stop_.load(); }, 100);
      if (st < 0) return false;
      if (st == 1) return true;
    } else {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_for(lk, std::chrono::milliseconds(100), [this] { return work_.load() || stop_.load(); });
    }
    std::string e;
    if (!reap(false, &e)) {
      fail(e);
      return false;
    }
  }
  return false;
}

// Completion of issued rounds, oldest first.  need_room: wait (bounded by the
// operation deadline) until fewer than kInflight rounds are outstanding.  A
// round past its deadline aborts the communicator: RCCL's kernels exit, and
// the group fails with the round's operations and peers in the error.
bool Group::reap(bool need_room, std::string* err) {
  while (!inflight_.empty()) {
    Inflight& f = inflight_.front();
    const hipError_t q = hipEventQuery(f.ev);
    if (q == hipSuccess) {
      hip::event_put(device_, f.ev);
      inflight_.pop_front();
      continue;
    }
    if (q != hipErrorNotReady) {
      *err = strfmt("round ", f.round, " (", f.what, "): ", hipGetErrorString(q));
      return false;
    }
    if (now_ns() - f.t0 > static_cast<int64_t>(op_timeout_ms_) * 1000000) {
      ncclCommAbort(static_cast<ncclComm_t>(comm_));
      aborted_ = true;
      *err = strfmt("round ", f.round, " (", f.what, ") did not complete on the device within ", op_timeout_ms_,
                    " ms: a member stopped progressing; the communicator was aborted");
      return false;
    }
    if (!need_room || inflight_.size() < kInflight) break;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  return true;
}

void Group::fail(const std::string& why) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!failed_.empty()) return;
  failed_ = why.empty() ? std::string("the group failed") : why;
  NNSX_LOGE("comm", "group ", spec_.name, " (member ", grank_, "): ", failed_);
  for (auto& op : colls_) {
    op->done = true;
    op->ok = false;
    op->err = failed_;
  }
  colls_.clear();
  for (auto& q : outbox_) q.clear();
  cv_.notify_all();
}

void Group::drop_member(int m, bool orderly) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!active_[static_cast<size_t>(m)]) return;
  active_[static_cast<size_t>(m)] = 0;
  const std::string why = strfmt("member ", m, " (rank ", global_rank(m), ") left the group",
                                 orderly ? "" : " without a goodbye");
  if (orderly)
    NNSX_LOGD("comm", "group ", spec_.name, ": ", why);
  else
    NNSX_LOGW("comm", "group ", spec_.name, ": ", why, " (p2p with the other members continues)");
  if (coll_dead_.empty()) coll_dead_ = why;
  for (auto& op : colls_) {
    op->done = true;
    op->ok = false;
    op->err = coll_dead_;
  }
  colls_.clear();
  if (!outbox_[static_cast<size_t>(m)].empty())
    NNSX_LOGW("comm", "group ", spec_.name, ": dropping ", outbox_[static_cast<size_t>(m)].size(),
              " queued message(s) to member ", m);
  outbox_[static_cast<size_t>(m)].clear();
  cv_.notify_all();
}

bool Group::run_round(std::string* err) {
  const int n = size();
  const uint64_t r = round_;
  work_ = false;  // work arriving from now on triggers the next round
  std::vector<std::shared_ptr<CollOp>> colls;
  std::vector<std::vector<Packet>> sends(static_cast<size_t>(n));
  std::vector<uint32_t> grant(static_cast<size_t>(n), 0);
  std::vector<char> act;
  {
    std::lock_guard<std::mutex> lk(mu_);
    act = active_;
    if (coll_dead_.empty()) colls.assign(colls_.begin(), colls_.end());
    for (int d = 0; d < n; ++d) {
      auto& q = outbox_[static_cast<size_t>(d)];
      while (!q.empty() && static_cast<int>(sends[static_cast<size_t>(d)].size()) < allowed_[static_cast<size_t>(d)]) {
        sends[static_cast<size_t>(d)].push_back(std::move(q.front()));
        q.pop_front();
      }
      if (d != grank_) {
        grant[static_cast<size_t>(d)] = static_cast<uint32_t>(std::max(0, kWindow - unconsumed_[static_cast<size_t>(d)]));
        granted_[static_cast<size_t>(d)] = static_cast<int>(grant[static_cast<size_t>(d)]);
        recvd_since_grant_[static_cast<size_t>(d)] = 0;  // (this round's messages count against it)
      }
    }
  }
  cv_.notify_all();  // room in the outboxes
  // ---- manifests out, then in ----
  std::vector<Manifest> man(static_cast<size_t>(n));
  for (int d = 0; d < n; ++d) {
    if (d == grank_ || !act[static_cast<size_t>(d)]) continue;
    std::string e;
    if (!mesh_->send(d, r + 1, manifest_for(d, grant[static_cast<size_t>(d)], colls, sends[static_cast<size_t>(d)]), &e)) {
      drop_member(d, false);
      act[static_cast<size_t>(d)] = 0;
    }
  }
  const int64_t deadline = now_ns() + static_cast<int64_t>(spec_.timeout_ms) * 1000000;
  for (int d = 0; d < n; ++d) {
    if (d == grank_ || !act[static_cast<size_t>(d)]) continue;
    Message m;
    bool to = false;
    int gone = 0;
    std::string e;
    const int left_ms = static_cast<int>(std::max<int64_t>(0, (deadline - now_ns()) / 1000000));
    if (!mesh_->recv(r + 1, d, &m, left_ms, &to, &gone, &e)) {
      if (gone) {
        drop_member(d, gone == 3);
        act[static_cast<size_t>(d)] = 0;
        continue;
      }
      *err = to ? strfmt("round ", r, ": member ", d, " (rank ", global_rank(d), ") sent no manifest within ",
                         spec_.timeout_ms, " ms")
                : strfmt("round ", r, ": ", e);
      return false;
    }
    if (!parse_manifest(std::move(m), &man[static_cast<size_t>(d)])) {
      *err = strfmt("round ", r, ": malformed manifest from member ", d);
      return false;
    }
  }
  for (int d = 0; d < n; ++d)
    if (!act[static_cast<size_t>(d)]) sends[static_cast<size_t>(d)].clear();  // (dropped with the member)
  // ---- the collectives every member listed (a common prefix of the sequence) ----
  bool everyone = true;
  for (int d = 0; d < n; ++d) everyone = everyone && act[static_cast<size_t>(d)];
  std::vector<std::shared_ptr<CollOp>> run;
  std::vector<std::vector<const ManifestColl*>> ents;
  std::string mismatch;
  std::vector<size_t> pos(static_cast<size_t>(n), 0);
  for (auto& op : colls) {
    if (!everyone) break;
    std::vector<const ManifestColl*> ent(static_cast<size_t>(n), nullptr);
    bool listed = true;
    for (int d = 0; d < n && listed; ++d) {
      if (d == grank_) continue;
      const auto& cs = man[static_cast<size_t>(d)].colls;
      size_t& k = pos[static_cast<size_t>(d)];
      while (k < cs.size() && cs[k].seq < op->seq) ++k;
      if (k >= cs.size() || cs[k].seq != op->seq) {
        listed = false;
        break;
      }
      if (cs[k].kind != op->kind || cs[k].root != op->root) {
        mismatch = strfmt("collective ", op->seq, ": member ", d, " called ", CollOp::name(cs[k].kind), "(root ",
                          cs[k].root, ") where member ", grank_, " called ", CollOp::name(op->kind), "(root ", op->root,
                          ")");
        listed = false;
        break;
      }
      ent[static_cast<size_t>(d)] = &cs[k];
    }
    if (!listed) break;
    run.push_back(op);
    ents.push_back(std::move(ent));
  }
  // ---- data plane: the collectives in sequence order, then the p2p group ----
  std::string what;
  std::vector<Packet> got;
  if (rccl()) hip::check(hipSetDevice(device_), "hipSetDevice");
  for (size_t i = 0; i < run.size(); ++i)
    if (!issue_collective(*run[i], ents[i], &what, err)) return false;
  if (!issue_p2p(sends, man, &got, &what, err)) return false;
  if (rccl() && !what.empty()) {
    Inflight f;
    f.ev = hip::event_get(device_);
    hip::check(hipEventRecord(f.ev, stream_), "hipEventRecord(round)");
    f.t0 = now_ns();
    f.round = r;
    f.what = what;
    inflight_.push_back(std::move(f));
  }
  // ---- publish ----
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& op : run) {
      op->done = true;
      op->ok = op->err.empty();
      colls_.erase(std::remove(colls_.begin(), colls_.end(), op), colls_.end());
    }
    if (!mismatch.empty() && coll_dead_.empty()) {
      coll_dead_ = mismatch;
      for (auto& op : colls_) {
        op->done = true;
        op->ok = false;
        op->err = mismatch;
      }
      colls_.clear();
    }
    for (auto& p : got) {
      if (p.src != grank_) {
        ++unconsumed_[static_cast<size_t>(p.src)];
        ++recvd_since_grant_[static_cast<size_t>(p.src)];
      }
      inbox_.push_back(std::move(p));
    }
    for (int d = 0; d < n; ++d) {
      if (d == grank_) {
        allowed_[static_cast<size_t>(d)] = kWindow;  // (forced RCCL group of one: the round receives its own)
      } else if (act[static_cast<size_t>(d)]) {
        const auto& mm = man[static_cast<size_t>(d)];
        allowed_[static_cast<size_t>(d)] =
            std::max(0, static_cast<int>(mm.grant) - static_cast<int>(sends[static_cast<size_t>(d)].size()));
        listed_upto_[static_cast<size_t>(d)] = mm.colls.empty() ? 0 : mm.colls.back().seq + 1;
      }
      if (!outbox_[static_cast<size_t>(d)].empty() && allowed_[static_cast<size_t>(d)] > 0) work_ = true;
    }
  }
  cv_.notify_all();
  ++round_;
  return true;
}

// One collective of the round.  ent[m]: member m's manifest entry for it
// (nullptr for this member).  RCCL: one ncclGroupStart/End on the comm
// stream; tcp: the payloads came inline with the manifests.
bool Group::issue_collective(CollOp& op, const std::vector<const ManifestColl*>& ent, std::string* what,
                             std::string* err) {
  const int n = size();
  what->append(strfmt(what->empty() ? "" : ", ", CollOp::name(op.kind), "#", op.seq));
  auto comm = static_cast<ncclComm_t>(comm_);
  auto header_of = [&](int m) -> const ManifestEntry* {
    const ManifestColl* c = ent[static_cast<size_t>(m)];
    return c && c->has_hdr ? &c->e : nullptr;
  };
  if (op.kind == CollOp::kAllGather) {
    op.all.assign(static_cast<size_t>(n), Packet());
    std::vector<std::vector<size_t>> sizes(static_cast<size_t>(n));
    for (int m = 0; m < n; ++m) {
      if (m == grank_) {
        op.all[static_cast<size_t>(m)] = op.mine;
        for (auto& b : op.mine.blobs) sizes[static_cast<size_t>(m)].push_back(b->size());
        continue;
      }
      const ManifestEntry* h = header_of(m);
      if (!h) {
        op.err = strfmt("allgather: no packet from member ", m);
        return true;
      }
      op.all[static_cast<size_t>(m)] = h->hdr;
      op.all[static_cast<size_t>(m)].src = m;
      sizes[static_cast<size_t>(m)] = h->sizes;
    }
    bool one_uniform = true;
    for (int m = 0; m < n; ++m)
      one_uniform = one_uniform && sizes[static_cast<size_t>(m)].size() == 1 &&
                    sizes[static_cast<size_t>(m)][0] == sizes[0][0] && sizes[0][0] > 0;
    if (!rccl()) {
      for (int m = 0; m < n; ++m)
        if (m != grank_)
          for (auto& b : op.all[static_cast<size_t>(m)].blobs) bytes_recv_ += b->size();
      if (op.want_stacked && one_uniform) {
        const size_t s = sizes[0][0];
        auto out = Memory::alloc_pinned(s * static_cast<size_t>(n));
        for (int m = 0; m < n; ++m)
          std::memcpy(static_cast<char*>(out->data()) + static_cast<size_t>(m) * s,
                      op.all[static_cast<size_t>(m)].blobs[0]->map_host(), s);
        op.stacked = out;
      }
      for (auto& b : op.mine.blobs) bytes_sent_ += b->size() * static_cast<size_t>(n - 1);
      return true;
    }
    size_t nb = 0;
    for (auto& s : sizes) nb = std::max(nb, s.size());
    std::vector<MemoryPtr> outs;
    for (int m = 0; m < n; ++m)
      if (m != grank_) op.all[static_cast<size_t>(m)].blobs.assign(sizes[static_cast<size_t>(m)].size(), nullptr);
    std::vector<void*> srcs(op.mine.blobs.size());
    for (size_t j = 0; j < op.mine.blobs.size(); ++j)
      srcs[j] = op.mine.blobs[j]->size() ? dev_ptr(op.mine.blobs[j]) : nullptr;
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
    for (size_t j = 0; j < nb; ++j) {
      bool uniform = true;
      for (int m = 0; m < n; ++m)
        uniform = uniform && j < sizes[static_cast<size_t>(m)].size() && sizes[static_cast<size_t>(m)][j] == sizes[0][j];
      if (uniform && sizes[0][j] > 0) {
        const size_t s = sizes[0][j];
        auto out = Memory::alloc_device(s * static_cast<size_t>(n), device_, stream_);
        outs.push_back(out);
        if (op.want_stacked && one_uniform) op.stacked = out;
        if (!nccl_ok(ncclAllGather(srcs[j], out->data(), s, ncclUint8, comm, stream_), "ncclAllGather", err)) {
          ncclGroupEnd();
          return false;
        }
        if (n == 1) op.all[static_cast<size_t>(grank_)].blobs[j] = out;  // (forced RCCL: the gathered copy)
        for (int m = 0; m < n; ++m) {
          if (m == grank_) continue;
          auto v = Memory::view(out, static_cast<size_t>(m) * s, s);
          const std::string& meta = header_of(m)->metas[j];
          if (!meta.empty()) {
            MetaInfo mi;
            if (MetaInfo::parse(meta.data(), meta.size(), &mi)) v->set_meta(mi);
          }
          op.all[static_cast<size_t>(m)].blobs[j] = v;
          bytes_recv_ += s;
        }
        bytes_sent_ += s;
        continue;
      }
      // ragged: one broadcast per owner of blob j
      for (int m = 0; m < n; ++m) {
        const auto& sm = sizes[static_cast<size_t>(m)];
        if (j >= sm.size() || sm[j] == 0) {
          if (m != grank_ && j < sm.size()) op.all[static_cast<size_t>(m)].blobs[j] = Memory::alloc_host(0);
          continue;
        }
        const size_t s = sm[j];
        if (m == grank_) {
          if (!nccl_ok(ncclBroadcast(srcs[j], srcs[j], s, ncclUint8, m, comm, stream_), "ncclBroadcast", err)) {
            ncclGroupEnd();
            return false;
          }
          bytes_sent_ += s;
          continue;
        }
        auto out = alloc_recv({s}, {header_of(m)->metas[j]})[0];
        outs.push_back(out);
        op.all[static_cast<size_t>(m)].blobs[j] = out;
        if (!nccl_ok(ncclBroadcast(out->data(), out->data(), s, ncclUint8, m, comm, stream_), "ncclBroadcast", err)) {
          ncclGroupEnd();
          return false;
        }
      }
    }
    if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
    for (auto& o : outs) o->mark_ready(stream_);
    finish_inputs(op.mine.blobs);
    return true;
  }
  if (op.kind == CollOp::kBroadcast) {
    const int root = op.root;
    if (root == grank_) {
      op.out = op.mine;
    } else {
      const ManifestEntry* h = header_of(root);
      if (!h) {
        op.err = "broadcast: no packet from the root";
        return true;
      }
      op.out = h->hdr;
      op.out.src = root;
      if (!rccl()) {
        for (auto& b : op.out.blobs) bytes_recv_ += b->size();
        return true;
      }
      op.out.blobs = alloc_recv(h->sizes, h->metas);
    }
    if (!rccl()) {
      for (auto& b : op.out.blobs) bytes_sent_ += b->size() * static_cast<size_t>(n - 1);
      return true;
    }
    std::vector<void*> ptrs;
    for (auto& b : op.out.blobs) ptrs.push_back(!b->size() ? nullptr : root == grank_ ? dev_ptr(b) : b->data());
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
    for (size_t j = 0; j < op.out.blobs.size(); ++j) {
      const size_t s = op.out.blobs[j]->size();
      if (!s) continue;
      if (!nccl_ok(ncclBroadcast(ptrs[j], ptrs[j], s, ncclUint8, root, comm, stream_), "ncclBroadcast", err)) {
        ncclGroupEnd();
        return false;
      }
      if (root == grank_) bytes_sent_ += s;
    }
    if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
    if (root == grank_) {
      finish_inputs(op.out.blobs);
    } else {
      for (auto& b : op.out.blobs)
        if (b->size()) b->mark_ready(stream_);
    }
    return true;
  }
  // scatter
  const int root = op.root;
  if (root == grank_) {
    op.out = op.parts.at(static_cast<size_t>(root));
    op.out.src = root;
    if (!rccl()) {
      for (int m = 0; m < n; ++m)
        if (m != root)
          for (auto& b : op.parts[static_cast<size_t>(m)].blobs) bytes_sent_ += b->size();
      return true;
    }
    if (n == 1) return true;
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
    for (int m = 0; m < n; ++m) {
      if (m == root) continue;
      for (auto& b : op.parts[static_cast<size_t>(m)].blobs) {
        if (!b->size()) continue;
        if (!nccl_ok(ncclSend(dev_ptr(b), b->size(), ncclUint8, m, comm, stream_), "ncclSend", err)) {
          ncclGroupEnd();
          return false;
        }
        bytes_sent_ += b->size();
      }
    }
    if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
    for (int m = 0; m < n; ++m)
      if (m != root) finish_inputs(op.parts[static_cast<size_t>(m)].blobs);
    return true;
  }
  const ManifestEntry* h = header_of(root);
  if (!h) {
    op.err = "scatter: no part from the root";
    return true;
  }
  op.out = h->hdr;
  op.out.src = root;
  if (!rccl()) {
    for (auto& b : op.out.blobs) bytes_recv_ += b->size();
    return true;
  }
  op.out.blobs = alloc_recv(h->sizes, h->metas);
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (auto& b : op.out.blobs)
    if (b->size() && !nccl_ok(ncclRecv(b->data(), b->size(), ncclUint8, root, comm, stream_), "ncclRecv", err)) {
      ncclGroupEnd();
      return false;
    }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& b : op.out.blobs)
    if (b->size()) b->mark_ready(stream_);
  return true;
}

// Every p2p message of the round, in ONE ncclGroupStart/End: this member's
// sends (peer order, FIFO per peer) and the receives of every message the
// other members listed for it (sender order, FIFO per sender).
bool Group::issue_p2p(std::vector<std::vector<Packet>>& sends, const std::vector<Manifest>& man,
                      std::vector<Packet>* got, std::string* what, std::string* err) {
  const int n = size();
  size_t nsend = 0, nrecv = 0;
  for (auto& s : sends) nsend += s.size();
  for (int m = 0; m < n; ++m)
    if (m != grank_) nrecv += man[static_cast<size_t>(m)].sends.size();
  if (nsend + nrecv == 0) return true;
  if (!rccl()) {
    for (auto& s : sends)
      for (auto& p : s)
        for (auto& b : p.blobs) bytes_sent_ += b->size();
    for (int m = 0; m < n; ++m) {
      if (m == grank_) continue;
      for (auto& e : man[static_cast<size_t>(m)].sends) {
        Packet p = e.hdr;
        p.src = m;
        for (auto& b : p.blobs) bytes_recv_ += b->size();
        got->push_back(std::move(p));
      }
    }
    return true;
  }
  std::string peers;
  for (int m = 0; m < n; ++m) {
    const size_t k = sends[static_cast<size_t>(m)].size() + (m == grank_ ? 0 : man[static_cast<size_t>(m)].sends.size());
    if (k) peers += strfmt(peers.empty() ? "" : ",", m, "(rank ", global_rank(m), ")");
  }
  what->append(strfmt(what->empty() ? "" : ", ", "p2p ", nsend, " out / ", nrecv, " in with members ", peers));
  auto comm = static_cast<ncclComm_t>(comm_);
  std::vector<std::vector<void*>> src(static_cast<size_t>(n));
  for (int d = 0; d < n; ++d)
    for (auto& p : sends[static_cast<size_t>(d)])
      for (auto& b : p.blobs) src[static_cast<size_t>(d)].push_back(b->size() ? dev_ptr(b) : nullptr);
  // receive buffers: a group of one (forced RCCL) receives its own messages
  for (int m = 0; m < n; ++m) {
    if (m == grank_) {
      for (auto& p : sends[static_cast<size_t>(m)]) {
        Packet q = p;
        q.src = m;
        q.blobs.clear();
        for (auto& b : p.blobs) {
          auto o = b->size() ? Memory::alloc_device(b->size(), device_, stream_) : Memory::alloc_host(0);
          if (b->has_meta()) o->set_meta(b->meta());
          bytes_recv_ += b->size();
          q.blobs.push_back(o);
        }
        got->push_back(std::move(q));
      }
      continue;
    }
    for (auto& e : man[static_cast<size_t>(m)].sends) {
      Packet q = e.hdr;
      q.src = m;
      q.blobs = alloc_recv(e.sizes, e.metas);
      got->push_back(std::move(q));
    }
  }
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
  for (int d = 0; d < n; ++d) {
    size_t k = 0;
    for (auto& p : sends[static_cast<size_t>(d)])
      for (auto& b : p.blobs) {
        void* ptr = src[static_cast<size_t>(d)][k++];
        if (!b->size()) continue;
        if (!nccl_ok(ncclSend(ptr, b->size(), ncclUint8, d, comm, stream_), "ncclSend", err)) {
          ncclGroupEnd();
          return false;
        }
        bytes_sent_ += b->size();
      }
  }
  for (auto& q : *got)
    for (auto& b : q.blobs)
      if (b->size() && !nccl_ok(ncclRecv(b->data(), b->size(), ncclUint8, q.src, comm, stream_), "ncclRecv", err)) {
        ncclGroupEnd();
        return false;
      }
  if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  for (auto& q : *got)
    for (auto& b : q.blobs)
      if (b->size()) b->mark_ready(stream_);
  for (auto& s : sends)
    for (auto& p : s) finish_inputs(p.blobs);
  return true;
}

// ------------------------------------------------------------ callers ----
bool Group::collective(const std::shared_ptr<CollOp>& op, std::string* err) {
  std::unique_lock<std::mutex> lk(mu_);
  auto bail = [&](const std::string& why) {
    colls_.erase(std::remove(colls_.begin(), colls_.end(), op), colls_.end());
    if (err) *err = why;
    return false;
  };
  if (!failed_.empty()) return bail(failed_);
  if (!coll_dead_.empty()) return bail(coll_dead_);
  if (cancelled_.load()) return bail("cancelled");
  op->seq = coll_seq_++;
  colls_.push_back(op);
  work_ = true;
  lk.unlock();
  poke();
  lk.lock();
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(spec_.timeout_ms);
  while (!op->done) {
    if (!failed_.empty()) return bail(failed_);
    if (!coll_dead_.empty()) return bail(coll_dead_);
    if (cancelled_.load()) return bail("cancelled");
    if (cv_.wait_until(lk, deadline) == std::cv_status::timeout && !op->done) {
      std::string who;
      for (int m = 0; m < size(); ++m)
        if (m != grank_ && active_[static_cast<size_t>(m)] && listed_upto_[static_cast<size_t>(m)] <= op->seq)
          who += strfmt(who.empty() ? "" : ",", m);
      coll_dead_ = strfmt(CollOp::name(op->kind), " (collective ", op->seq, "): member(s) ",
                          who.empty() ? std::string("?") : who, " did not enter it within ", spec_.timeout_ms, " ms");
      for (auto& o : colls_)
        if (o != op) {
          o->done = true;
          o->ok = false;
          o->err = coll_dead_;
        }
      colls_.clear();
      cv_.notify_all();
      if (err) *err = coll_dead_;
      return false;
    }
  }
  if (!op->ok) {
    if (err) *err = op->err;
    return false;
  }
  return true;
}

bool Group::allgather(const Packet& mine, std::vector<Packet>* all, std::string* err, MemoryPtr* stacked) {
  if (stacked) *stacked = nullptr;
  if (!engine_) {  // a group of one: nothing to exchange
    all->assign(1, mine);
    (*all)[0].src = grank_;
    if (stacked && mine.blobs.size() == 1) *stacked = mine.blobs[0];
    return true;
  }
  auto op = std::make_shared<CollOp>();
  op->kind = CollOp::kAllGather;
  op->mine = mine;
  op->mine.src = grank_;
  op->want_stacked = stacked != nullptr;
  if (!collective(op, err)) return false;
  *all = std::move(op->all);
  if (stacked) *stacked = op->stacked;
  return true;
}

bool Group::broadcast(int root, Packet* pkt, std::string* err) {
  if (root < 0 || root >= size()) {
    if (err) *err = strfmt("broadcast: no member ", root);
    return false;
  }
  if (!engine_) return true;  // (forced RCCL: the one-rank ncclBroadcast runs)
  auto op = std::make_shared<CollOp>();
  op->kind = CollOp::kBroadcast;
  op->root = root;
  if (root == grank_) op->mine = *pkt;
  if (!collective(op, err)) return false;
  *pkt = std::move(op->out);
  return true;
}

bool Group::scatter(int root, const std::vector<Packet>* parts, Packet* mine, std::string* err) {
  const int n = size();
  if (root < 0 || root >= n) {
    if (err) *err = strfmt("scatter: no member ", root);
    return false;
  }
  if (grank_ == root && (!parts || static_cast<int>(parts->size()) != n)) {
    if (err) *err = "scatter: the root needs one part per member";
    return false;
  }
  if (!engine_) {
    *mine = (*parts)[static_cast<size_t>(root)];
    mine->src = root;
    return true;
  }
  auto op = std::make_shared<CollOp>();
  op->kind = CollOp::kScatter;
  op->root = root;
  if (grank_ == root) op->parts = *parts;
  if (!collective(op, err)) return false;
  *mine = std::move(op->out);
  return true;
}

bool Group::send(int peer, const Packet& p, std::string* err) {
  if (peer < 0 || peer >= size()) {
    if (err) *err = strfmt("send: no member ", peer);
    return false;
  }
  std::unique_lock<std::mutex> lk(mu_);
  if (!failed_.empty()) {
    if (err) *err = failed_;
    return false;
  }
  if (cancelled_.load()) {
    if (err) *err = "send: cancelled";
    return false;
  }
  Packet q = p;
  q.src = grank_;
  // to oneself: handed over in-process, blobs as they are -- except in a group
  // of one on forced RCCL, whose round runs the grouped ncclSend / ncclRecv to
  // itself (the data plane's p2p kernels, on one GPU)
  if (peer == grank_ && !(engine_ && size() == 1)) {
    inbox_.push_back(std::move(q));
    cv_.notify_all();
    return true;
  }
  auto& box = outbox_[static_cast<size_t>(peer)];
  while (box.size() >= static_cast<size_t>(kOutbox)) {  // backpressure: the peer has not taken its window
    if (!failed_.empty() || cancelled_.load() || !active_[static_cast<size_t>(peer)]) break;
    cv_.wait_for(lk, std::chrono::milliseconds(100));
  }
  if (!failed_.empty() || cancelled_.load()) {
    if (err) *err = !failed_.empty() ? failed_ : std::string("send: cancelled");
    return false;
  }
  if (!active_[static_cast<size_t>(peer)]) {
    if (err) *err = strfmt("send: member ", peer, " (rank ", global_rank(peer), ") left the group");
    return false;
  }
  box.push_back(std::move(q));
  work_ = true;
  lk.unlock();
  poke();
  return true;
}

bool Group::recv(Packet* p, int timeout_ms, bool* timed_out, std::string* err) {
  if (timed_out) *timed_out = false;
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return !inbox_.empty() || cancelled_.load() || !failed_.empty(); };
  if (timeout_ms < 0) {
    cv_.wait(lk, ready);
  } else {
    cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
  }
  if (!failed_.empty()) {
    if (err) *err = "recv: " + failed_;
    return false;
  }
  if (inbox_.empty()) {
    if (cancelled_.load()) {
      if (err) *err = "recv: cancelled";
    } else if (timed_out) {
      *timed_out = true;
    }
    return false;
  }
  *p = std::move(inbox_.front());
  inbox_.pop_front();
  bool wake = false;
  const int s = p->src;
  if (engine_ && s != grank_ && s >= 0 && s < size()) {
    --unconsumed_[static_cast<size_t>(s)];
    // the sender may be held back by the last grant: advertise the room.  A
    // partial grant can grow now; a full one the sender has used up (its credit
    // is the grant minus what arrived since) leaves it unable to send until
    // some member runs a round -- this one must
    const size_t si = static_cast<size_t>(s);
    wake = granted_[si] < kWindow || granted_[si] - recvd_since_grant_[si] <= 0;
  }
  lk.unlock();
  if (wake) {
    work_ = true;
    poke();
  }
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
