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
// / AITT); nnsx implements the TCP connect-type natively, plus HIPIPC: the
// same framing with HBM-resident tensors handed over through an exported
// device ring (zero-copy on the same GPU, one xGMI peer copy across GPUs;
// see comm/transport.h).
#include <algorithm>
#include <atomic>
#include <map>
#include <thread>

#include "comm/transport.h"
#include "core/log.h"
#include "elements/elements.h"
#include "elements/tensor_common.h"
#include "runtime/base.h"
#include "runtime/hip_util.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

const std::vector<std::string> kConnectTypes = {"TCP", "HYBRID", "MQTT", "AITT", "HIPIPC"};
constexpr int kHipIpc = 4;

bool check_connect_type(Element* e, int type) {
  if (type == 0 || type == kHipIpc) return true;
  e->post_error("connect-type " + kConnectTypes[static_cast<size_t>(type)] +
                " is not supported (nnsx implements TCP and HIPIPC)");
  return false;
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
    is_live_ = true;
  }

 protected:
  bool on_start() override {
    if (!check_connect_type(this, connect_type_)) return false;
    server_ = query_server(static_cast<int>(id_));
    std::string err;
    if (!server_->start(host_, port_, &err)) {
      post_error("tensor_query_serversrc: " + err);
      server_.reset();
      return false;
    }
    return true;
  }
  void on_stop() override {
    if (server_) server_->stop();
  }
  void on_unlock() override {
    if (server_) server_->incoming.set_flushing(true);
  }

  FlowReturn create(BufferPtr* out) override {
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
    server_->set_sink_caps(caps.to_string());
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
    const uint64_t cid = buf->meta.client_id;
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
  }

  bool start() override {
    if (!check_connect_type(this, connect_type_)) return false;
    std::string err;
    conn_ = comm::Connection::connect(dest_host_, static_cast<int>(dest_port_),
                                      timeout_ms_ ? static_cast<int>(timeout_ms_) : 10000, &err);
    if (!conn_) {
      post_error("tensor_query_client: " + err);
      return false;
    }
    comm::Message hello;
    if (!conn_->recv(&hello, 30000) || hello.type != comm::MsgType::HELLO) {
      post_error("tensor_query_client: no handshake from the server");
      return false;
    }
    conn_->id = hello.client_id;
    if (connect_type_ == kHipIpc && !conn_->send_ipc_hello())
      NNSX_LOGW(name(), "HIPIPC: no GPU here, requests travel as bytes");
    server_caps_ = hello.caps.empty() ? Caps::from_string(tensor_caps_template_all()) : Caps::from_string(hello.caps);
    pending_.clear();
    seq_ = 0;
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
    return true;
  }
  void unlock() override {
    if (conn_) conn_->close();
  }

  bool sink_event(Pad*, Event& ev) override {
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
    Caps c = pad->direction() == PadDirection::SRC && conn_ ? server_caps_ : pad->template_caps();
    return filter ? c.intersect(*filter) : c;
  }

  FlowReturn chain(Pad*, BufferPtr buf) override {
    if (!conn_) return FlowReturn::ERROR;
    comm::Message m;
    m.type = comm::MsgType::DATA;
    m.client_id = conn_->id;
    m.seq = seq_++;
    m.pts = buf->pts;
    m.dts = buf->dts;
    m.duration = buf->duration;
    m.blobs = buf->mems;
    if (!conn_->send(m)) {
      post_error("tensor_query_client: failed to send a request to " + conn_->peer());
      return FlowReturn::ERROR;
    }
    pending_.push_back(buf);
    return drain(std::max(1u, max_request_) - 1);
  }

 private:
  // receive replies until at most `keep` requests remain in flight
  FlowReturn drain(size_t keep) {
    while (pending_.size() > keep) {
      comm::Message r;
      bool timed_out = false;
      const int t = timeout_ms_ ? static_cast<int>(timeout_ms_) : -1;
      if (!conn_ || !conn_->recv(&r, t, &timed_out)) {
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
  }

 protected:
  bool start() override {
    BaseSink::start();
    if (!check_connect_type(this, connect_type_)) return false;
    std::string err;
    if (!listener_.listen(host_, port_, &err)) {
      post_error("edgesink: " + err);
      return false;
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
  }
  bool set_caps(const Caps& caps) override {
    comm::Message m;
    m.type = comm::MsgType::CAPS;
    std::lock_guard<std::mutex> lk(mu_);
    caps_str_ = caps.to_string();
    m.caps = caps_str_;
    for (auto& c : subs_) c->send(m);
    return true;
  }
  FlowReturn render(const BufferPtr& buf) override {
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
    comm::Message m;
    m.type = comm::MsgType::EOS;
    publish(m);
  }

 private:
  void publish(const comm::Message& m) {
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
    is_live_ = true;
  }

 protected:
  bool on_start() override {
    if (!check_connect_type(this, connect_type_)) return false;
    std::string err;
    conn_ = comm::Connection::connect(dest_host_, static_cast<int>(dest_port_), 10000, &err);
    if (!conn_) {
      post_error("edgesrc: " + err);
      return false;
    }
    caps_str_.clear();
    return true;
  }
  void on_stop() override {
    if (conn_) conn_->close();
  }
  void on_unlock() override {
    if (conn_) conn_->close();
  }

  // the publisher's caps arrive with HELLO (or a later CAPS message)
  bool negotiate() override {
    while (caps_str_.empty()) {
      comm::Message m;
      bool timed_out = false;
      if (!conn_->recv(&m, 100, &timed_out)) {
        if (timed_out && !flushing_.load()) continue;
        return false;
      }
      if (m.type == comm::MsgType::HELLO && connect_type_ == kHipIpc) conn_->send_ipc_hello();
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
    while (true) {
      comm::Message m;
      bool timed_out = false;
      if (!conn_->recv(&m, 100, &timed_out)) {
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
};

}  // namespace

void register_comm_elements() {
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
