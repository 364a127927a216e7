// MQTT 3.1.1 client + in-process broker.  See mqtt.h.
#include "comm/mqtt.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "core/log.h"
#include "core/util.h"

namespace nnsx {
namespace comm {

namespace {

enum : uint8_t {
  CONNECT = 1,
  CONNACK = 2,
  PUBLISH = 3,
  PUBACK = 4,
  SUBSCRIBE = 8,
  SUBACK = 9,
  UNSUBSCRIBE = 10,
  UNSUBACK = 11,
  PINGREQ = 12,
  PINGRESP = 13,
  DISCONNECT = 14,
};

bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

// 0 = ok, 1 = timeout (nothing read yet), -1 = closed / error
int read_all(int fd, void* p, size_t n, int timeout_ms, const std::atomic<bool>* stop) {
  char* c = static_cast<char*>(p);
  size_t got = 0;
  while (got < n) {
    pollfd pf{fd, POLLIN, 0};
    const int wait = timeout_ms < 0 ? 200 : std::min(timeout_ms, 200);
    const int r = ::poll(&pf, 1, wait);
    if (r < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    if (r == 0) {
      if (stop && stop->load()) return -1;
      if (got == 0 && timeout_ms >= 0) {
        timeout_ms -= wait;
        if (timeout_ms <= 0) return 1;
      }
      continue;
    }
    const ssize_t k = ::recv(fd, c + got, n - got, 0);
    if (k <= 0) {
      if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
      return -1;
    }
    got += static_cast<size_t>(k);
  }
  return 0;
}

void put_u16(std::string& s, uint16_t v) {
  s.push_back(static_cast<char>(v >> 8));
  s.push_back(static_cast<char>(v & 0xff));
}
void put_str(std::string& s, const std::string& v) {
  put_u16(s, static_cast<uint16_t>(v.size()));
  s += v;
}
uint16_t get_u16(const std::string& s, size_t off) {
  return static_cast<uint16_t>((static_cast<uint8_t>(s[off]) << 8) | static_cast<uint8_t>(s[off + 1]));
}

std::string fixed_header(uint8_t type_flags, size_t remaining) {
  std::string h;
  h.push_back(static_cast<char>(type_flags));
  do {
    uint8_t b = remaining % 128;
    remaining /= 128;
    if (remaining) b |= 0x80;
    h.push_back(static_cast<char>(b));
  } while (remaining);
  return h;
}

// one packet: type/flags byte + body.  0 ok, 1 timeout, -1 closed
int read_packet(int fd, uint8_t* tf, std::string* body, int timeout_ms, const std::atomic<bool>* stop) {
  uint8_t b0;
  int r = read_all(fd, &b0, 1, timeout_ms, stop);
  if (r) return r;
  size_t len = 0, mult = 1;
  for (int i = 0; i < 4; ++i) {
    uint8_t b;
    if (read_all(fd, &b, 1, -1, stop)) return -1;
    len += (b & 0x7f) * mult;
    mult *= 128;
    if (!(b & 0x80)) break;
  }
  body->resize(len);
  if (len && read_all(fd, &(*body)[0], len, -1, stop)) return -1;
  *tf = b0;
  return 0;
}

int tcp_connect(const std::string& host, int port, int timeout_ms, std::string* err) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  const std::string h = host == "localhost" ? "127.0.0.1" : host;
  if (getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    if (err) *err = "mqtt: cannot resolve " + host;
    return -1;
  }
  int fd = -1;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype, a->ai_protocol);
    if (fd < 0) continue;
    const int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int rc = ::connect(fd, a->ai_addr, a->ai_addrlen);
    if (rc < 0 && errno == EINPROGRESS) {
      pollfd pf{fd, POLLOUT, 0};
      rc = ::poll(&pf, 1, timeout_ms) == 1 ? 0 : -1;
      int soerr = 0;
      socklen_t sl = sizeof(soerr);
      if (rc == 0 && (getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) < 0 || soerr != 0)) rc = -1;
    }
    if (rc == 0) {
      fcntl(fd, F_SETFL, fl);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      break;
    }
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0 && err) *err = strfmt("mqtt: cannot connect to broker ", host, ":", port);
  return fd;
}

}  // namespace

bool mqtt_topic_matches(const std::string& filter, const std::string& topic) {
  const auto f = split(filter, '/');
  const auto t = split(topic, '/');
  size_t i = 0;
  for (; i < f.size(); ++i) {
    if (f[i] == "#") return true;
    if (i >= t.size()) return false;
    if (f[i] != "+" && f[i] != t[i]) return false;
  }
  return i == t.size();
}

// ================================================================ client ====
MqttClient::~MqttClient() { close(); }

bool MqttClient::connect(const std::string& host, int port, const std::string& client_id, int keepalive_s,
                         bool clean_session, int timeout_ms, std::string* err) {
  fd_ = tcp_connect(host, port, timeout_ms, err);
  if (fd_ < 0) return false;
  std::string var;
  put_str(var, "MQTT");
  var.push_back(4);                                            // protocol level 3.1.1
  var.push_back(static_cast<char>(clean_session ? 0x02 : 0));  // connect flags
  put_u16(var, static_cast<uint16_t>(std::max(0, keepalive_s)));
  put_str(var, client_id);
  const std::string h = fixed_header(CONNECT << 4, var.size());
  if (!write_all(fd_, h.data(), h.size()) || !write_all(fd_, var.data(), var.size())) {
    if (err) *err = "mqtt: CONNECT failed";
    return false;
  }
  uint8_t tf = 0;
  std::string body;
  if (read_packet(fd_, &tf, &body, timeout_ms, nullptr) != 0 || (tf >> 4) != CONNACK || body.size() < 2 || body[1] != 0) {
    if (err) *err = "mqtt: broker refused the connection";
    ::close(fd_);
    fd_ = -1;
    return false;
  }
  alive_ = true;
  stop_ = false;
  reader_ = std::thread([this] { reader(); });
  if (keepalive_s > 0) pinger_ = std::thread([this, keepalive_s] { pinger(keepalive_s); });
  return true;
}

bool MqttClient::send_packet(uint8_t type_flags, const std::string& var, const void* p1, size_t n1, const void* p2,
                             size_t n2) {
  const std::string h = fixed_header(type_flags, var.size() + n1 + n2);
  std::lock_guard<std::mutex> lk(wmu_);
  if (!alive_) return false;
  bool ok = write_all(fd_, h.data(), h.size()) && write_all(fd_, var.data(), var.size()) &&
            (!n1 || write_all(fd_, p1, n1)) && (!n2 || write_all(fd_, p2, n2));
  if (!ok) alive_ = false;
  return ok;
}

bool MqttClient::wait_ack(uint16_t id, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  const bool ok = cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return acks_.count(id) || !alive_; });
  const bool got = ok && acks_.count(id);
  acks_.erase(id);
  return got;
}

bool MqttClient::publish(const std::string& topic, const void* data, size_t len, int qos, bool retain, int timeout_ms) {
  return publish2(topic, data, len, nullptr, 0, qos, retain, timeout_ms);
}

bool MqttClient::publish2(const std::string& topic, const void* hdr, size_t hlen, const void* body, size_t blen, int qos,
                          bool retain, int timeout_ms) {
  qos = std::min(qos, 1);  // QoS 2 is served as QoS 1 (at-least-once)
  std::string var;
  put_str(var, topic);
  uint16_t id = 0;
  if (qos > 0) {
    std::lock_guard<std::mutex> lk(mu_);
    id = next_id_++;
    if (next_id_ == 0) next_id_ = 1;
    put_u16(var, id);
  }
  const uint8_t tf = static_cast<uint8_t>(PUBLISH << 4 | (qos << 1) | (retain ? 1 : 0));
  if (!send_packet(tf, var, hdr, hlen, body, blen)) return false;
  return qos == 0 || wait_ack(id, timeout_ms);
}

bool MqttClient::subscribe(const std::string& filter, int qos, int timeout_ms) {
  std::string var;
  uint16_t id;
  {
    std::lock_guard<std::mutex> lk(mu_);
    id = next_id_++;
    if (next_id_ == 0) next_id_ = 1;
  }
  put_u16(var, id);
  put_str(var, filter);
  var.push_back(static_cast<char>(std::min(qos, 1)));
  if (!send_packet(SUBSCRIBE << 4 | 0x2, var, nullptr, 0, nullptr, 0)) return false;
  return wait_ack(id, timeout_ms);
}

bool MqttClient::recv(MqttMessage* m, int timeout_ms, bool* timed_out) {
  if (timed_out) *timed_out = false;
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return !inbox_.empty() || !alive_; };
  if (timeout_ms < 0)
    cv_.wait(lk, ready);
  else
    cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
  if (!inbox_.empty()) {
    *m = std::move(inbox_.front());
    inbox_.pop_front();
    return true;
  }
  if (timed_out) *timed_out = alive_.load();
  return false;
}

void MqttClient::reader() {
  while (!stop_) {
    uint8_t tf;
    std::string body;
    const int r = read_packet(fd_, &tf, &body, 200, &stop_);
    if (r == 1) continue;
    if (r < 0) break;
    const uint8_t type = tf >> 4;
    if (type == PUBLISH) {
      if (body.size() < 2) break;
      MqttMessage m;
      const uint16_t tl = get_u16(body, 0);
      size_t off = 2 + tl;
      if (off > body.size()) break;
      m.topic = body.substr(2, tl);
      m.qos = (tf >> 1) & 3;
      m.retain = tf & 1;
      if (m.qos > 0) {
        if (off + 2 > body.size()) break;
        const uint16_t id = get_u16(body, off);
        off += 2;
        std::string ack;
        put_u16(ack, id);
        send_packet(PUBACK << 4, ack, nullptr, 0, nullptr, 0);
      }
      m.payload = body.substr(off);
      std::lock_guard<std::mutex> lk(mu_);
      inbox_.push_back(std::move(m));
      cv_.notify_all();
    } else if (type == PUBACK || type == SUBACK || type == UNSUBACK) {
      if (body.size() < 2) continue;
      std::lock_guard<std::mutex> lk(mu_);
      acks_[get_u16(body, 0)] = true;
      cv_.notify_all();
    }
    // PINGRESP: nothing to do
  }
  std::lock_guard<std::mutex> lk(mu_);
  alive_ = false;
  cv_.notify_all();
}

void MqttClient::pinger(int keepalive_s) {
  const auto period = std::chrono::milliseconds(std::max(100, keepalive_s * 1000 / 2));
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_ && alive_) {
    if (cv_.wait_for(lk, period, [&] { return stop_.load() || !alive_; })) break;
    lk.unlock();
    send_packet(PINGREQ << 4, std::string(), nullptr, 0, nullptr, 0);
    lk.lock();
  }
}

void MqttClient::close() {
  if (fd_ < 0) return;
  if (alive_) send_packet(DISCONNECT << 4, std::string(), nullptr, 0, nullptr, 0);
  stop_ = true;
  {
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_all();
  }
  ::shutdown(fd_, SHUT_RDWR);
  if (reader_.joinable()) reader_.join();
  if (pinger_.joinable()) pinger_.join();
  ::close(fd_);
  fd_ = -1;
  alive_ = false;
}

// ================================================================ broker ====
struct MqttBroker::Client {
  int fd = -1;
  std::string id;
  std::mutex wmu;
  std::vector<std::string> filters;
  std::atomic<bool> alive{true};
  bool send(const std::string& h, const std::string& var, const std::string& payload) {
    std::lock_guard<std::mutex> lk(wmu);
    if (!alive) return false;
    if (!write_all(fd, h.data(), h.size()) || !write_all(fd, var.data(), var.size()) ||
        (!payload.empty() && !write_all(fd, payload.data(), payload.size()))) {
      alive = false;
      return false;
    }
    return true;
  }
};

bool MqttBroker::start(const std::string& host, int port, std::string* err) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd_ < 0) {
    if (err) *err = "mqtt broker: socket() failed";
    return false;
  }
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  const std::string h = host.empty() || host == "localhost" ? "127.0.0.1" : host;
  if (inet_pton(AF_INET, h.c_str(), &addr.sin_addr) != 1) addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) < 0 || ::listen(lfd_, 64) < 0) {
    if (err) *err = strfmt("mqtt broker: cannot listen on ", h, ":", port, " (", std::strerror(errno), ")");
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  socklen_t sl = sizeof(addr);
  getsockname(lfd_, reinterpret_cast<sockaddr*>(&addr), &sl);
  port_ = ntohs(addr.sin_port);
  running_ = true;
  acc_ = std::thread([this] { accept_loop(); });
  return true;
}

void MqttBroker::stop() {
  if (!running_.exchange(false)) return;
  ::shutdown(lfd_, SHUT_RDWR);
  ::close(lfd_);
  if (acc_.joinable()) acc_.join();
  std::vector<std::thread> ws;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& c : clients_) {
      std::lock_guard<std::mutex> cl(c->wmu);
      if (c->fd >= 0) ::shutdown(c->fd, SHUT_RDWR);
    }
    ws.swap(workers_);
  }
  for (auto& t : ws)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> lk(mu_);
  clients_.clear();
}

size_t MqttBroker::clients() {
  std::lock_guard<std::mutex> lk(mu_);
  size_t n = 0;
  for (auto& c : clients_) n += c->alive ? 1 : 0;
  return n;
}

void MqttBroker::accept_loop() {
  while (running_) {
    pollfd pf{lfd_, POLLIN, 0};
    if (::poll(&pf, 1, 100) <= 0) continue;
    const int fd = ::accept(lfd_, nullptr, nullptr);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    auto c = std::make_shared<Client>();
    c->fd = fd;
    std::lock_guard<std::mutex> lk(mu_);
    clients_.erase(std::remove_if(clients_.begin(), clients_.end(), [](auto& x) { return !x->alive; }), clients_.end());
    clients_.push_back(c);
    workers_.emplace_back([this, c] { serve(c); });
  }
}

void MqttBroker::route(const MqttMessage& m) {
  ++published_;
  std::vector<std::shared_ptr<Client>> targets;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (m.retain) {
      if (m.payload.empty())
        retained_.erase(m.topic);
      else
        retained_[m.topic] = m;
    }
    for (auto& c : clients_)
      if (c->alive)
        for (auto& f : c->filters)
          if (mqtt_topic_matches(f, m.topic)) {
            targets.push_back(c);
            break;
          }
  }
  // fan-out at QoS 0 (the broker keeps no in-flight state per subscriber)
  std::string var;
  put_str(var, m.topic);
  const std::string h = fixed_header(PUBLISH << 4, var.size() + m.payload.size());
  for (auto& c : targets) c->send(h, var, m.payload);
}

void MqttBroker::serve(std::shared_ptr<Client> c) {
  while (running_ && c->alive) {
    uint8_t tf;
    std::string body;
    const int r = read_packet(c->fd, &tf, &body, 200, nullptr);
    if (r == 1) continue;
    if (r < 0) break;
    const uint8_t type = tf >> 4;
    if (type == CONNECT) {
      if (body.size() >= 12) {
        const uint16_t pl = get_u16(body, 0);
        const size_t idoff = 2 + pl + 4;
        if (idoff + 2 <= body.size()) c->id = body.substr(idoff + 2, get_u16(body, idoff));
      }
      std::string ack("\0\0", 2);
      c->send(fixed_header(CONNACK << 4, 2), ack, std::string());
    } else if (type == PUBLISH) {
      if (body.size() < 2) break;
      MqttMessage m;
      const uint16_t tl = get_u16(body, 0);
      size_t off = 2 + tl;
      if (off > body.size()) break;
      m.topic = body.substr(2, tl);
      m.qos = (tf >> 1) & 3;
      m.retain = tf & 1;
      if (m.qos > 0 && off + 2 <= body.size()) {
        std::string id = body.substr(off, 2);
        off += 2;
        c->send(fixed_header(PUBACK << 4, 2), id, std::string());
      }
      m.payload = body.substr(off);
      route(m);
    } else if (type == SUBSCRIBE) {
      if (body.size() < 2) break;
      std::string var = body.substr(0, 2);  // packet id
      std::vector<std::string> added;
      size_t off = 2;
      std::string codes;
      while (off + 2 <= body.size()) {
        const uint16_t fl = get_u16(body, off);
        if (off + 2 + fl + 1 > body.size()) break;
        added.push_back(body.substr(off + 2, fl));
        codes.push_back(std::min<char>(body[off + 2 + fl], 1));
        off += 2 + fl + 1;
      }
      std::vector<MqttMessage> retained;
      {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto& f : added) {
          c->filters.push_back(f);
          for (auto& kv : retained_)
            if (mqtt_topic_matches(f, kv.first)) retained.push_back(kv.second);
        }
      }
      c->send(fixed_header(SUBACK << 4, var.size() + codes.size()), var, codes);
      for (auto& m : retained) {
        std::string v;
        put_str(v, m.topic);
        c->send(fixed_header(PUBLISH << 4 | 1, v.size() + m.payload.size()), v, m.payload);
      }
    } else if (type == UNSUBSCRIBE) {
      if (body.size() < 2) break;
      size_t off = 2;
      {
        std::lock_guard<std::mutex> lk(mu_);
        while (off + 2 <= body.size()) {
          const uint16_t fl = get_u16(body, off);
          const std::string f = body.substr(off + 2, fl);
          c->filters.erase(std::remove(c->filters.begin(), c->filters.end(), f), c->filters.end());
          off += 2 + fl;
        }
      }
      c->send(fixed_header(UNSUBACK << 4, 2), body.substr(0, 2), std::string());
    } else if (type == PINGREQ) {
      c->send(fixed_header(PINGRESP << 4, 0), std::string(), std::string());
    } else if (type == DISCONNECT) {
      break;
    }
  }
  std::lock_guard<std::mutex> lk(c->wmu);  // no fan-out write may race the close
  c->alive = false;
  ::close(c->fd);
  c->fd = -1;
}

std::shared_ptr<MqttBroker> mqtt_broker_start(const std::string& host, int port, std::string* err) {
  auto b = std::make_shared<MqttBroker>();
  if (!b->start(host, port, err)) return nullptr;
  return b;
}

}  // namespace comm
}  // namespace nnsx
