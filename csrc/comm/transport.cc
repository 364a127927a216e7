// TCP framing for the comm elements (see transport.h).
#include "comm/transport.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <thread>

#include "core/log.h"
#include "core/util.h"

namespace nnsx {
namespace comm {

namespace {

constexpr uint32_t kMagic = 0x58534e4e;  // "NNSX"
constexpr uint32_t kVersion = 1;
constexpr uint32_t kMaxBlobs = 256;

#pragma pack(push, 1)
struct WireHeader {
  uint32_t magic, version, type, nblobs;
  uint64_t client_id, seq;
  int64_t pts, dts, duration;
  uint32_t caps_len, flags;
};
#pragma pack(pop)

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

bool resolve(const std::string& host, int port, sockaddr_in* out) {
  std::memset(out, 0, sizeof(*out));
  out->sin_family = AF_INET;
  out->sin_port = htons(static_cast<uint16_t>(port));
  std::string h = host.empty() || host == "localhost" ? "127.0.0.1" : host;
  if (inet_pton(AF_INET, h.c_str(), &out->sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(h.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
  out->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

}  // namespace

Connection::Connection(int fd, std::string peer) : fd_(fd), peer_(std::move(peer)) { tune(fd_); }

Connection::~Connection() { close(); }

std::shared_ptr<Connection> Connection::connect(const std::string& host, int port, int timeout_ms, std::string* err) {
  sockaddr_in addr;
  if (!resolve(host, port, &addr)) {
    if (err) *err = "cannot resolve " + host;
    return nullptr;
  }
  const int64_t deadline = now_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
      if (err) *err = std::string("socket: ") + std::strerror(errno);
      return nullptr;
    }
    if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) == 0)
      return std::make_shared<Connection>(fd, strfmt(host, ":", port));
    const int e = errno;
    ::close(fd);
    if (now_ns() >= deadline) {
      if (err) *err = strfmt("connect ", host, ":", port, ": ", std::strerror(e));
      return nullptr;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

bool Connection::write_all(const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    ssize_t w = ::send(fd_, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      alive_ = false;
      return false;
    }
    c += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

bool Connection::read_all(void* p, size_t n, int timeout_ms, bool* timed_out) {
  char* c = static_cast<char*>(p);
  bool first = true;
  while (n > 0) {
    pollfd pfd{fd_, POLLIN, 0};
    // the timeout only applies before the first byte of a message
    int pr = ::poll(&pfd, 1, first ? timeout_ms : 30000);
    if (pr == 0) {
      if (first && timed_out) *timed_out = true;
      if (!first) alive_ = false;  // a stalled half-message is a broken stream
      return false;
    }
    if (pr < 0) {
      if (errno == EINTR) continue;
      alive_ = false;
      return false;
    }
    ssize_t r = ::recv(fd_, c, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      alive_ = false;
      return false;
    }
    first = false;
    c += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool Connection::send(const Message& m) {
  if (!alive_) return false;
  if (m.blobs.size() > kMaxBlobs) return false;
  WireHeader h{kMagic, kVersion, static_cast<uint32_t>(m.type), static_cast<uint32_t>(m.blobs.size()),
               m.client_id, m.seq, m.pts, m.dts, m.duration, static_cast<uint32_t>(m.caps.size()), m.flags};
  std::vector<uint64_t> sizes;
  std::vector<const void*> ptrs;
  for (const auto& b : m.blobs) {
    sizes.push_back(b->size());
    ptrs.push_back(b->map_host());  // HBM blobs: staged through a host mirror
  }
  std::lock_guard<std::mutex> lk(send_mu_);
  if (!write_all(&h, sizeof(h))) return false;
  if (!sizes.empty() && !write_all(sizes.data(), sizes.size() * sizeof(uint64_t))) return false;
  if (!m.caps.empty() && !write_all(m.caps.data(), m.caps.size())) return false;
  for (size_t i = 0; i < ptrs.size(); ++i)
    if (sizes[i] && !write_all(ptrs[i], sizes[i])) return false;
  return true;
}

bool Connection::recv(Message* m, int timeout_ms, bool* timed_out) {
  if (timed_out) *timed_out = false;
  if (!alive_) return false;
  WireHeader h;
  if (!read_all(&h, sizeof(h), timeout_ms, timed_out)) return false;
  if (h.magic != kMagic || h.version != kVersion || h.nblobs > kMaxBlobs) {
    NNSX_LOGE("comm", "bad message header from ", peer_);
    alive_ = false;
    return false;
  }
  m->type = static_cast<MsgType>(h.type);
  m->client_id = h.client_id;
  m->seq = h.seq;
  m->pts = h.pts;
  m->dts = h.dts;
  m->duration = h.duration;
  m->flags = h.flags;
  std::vector<uint64_t> sizes(h.nblobs);
  if (h.nblobs && !read_all(sizes.data(), sizes.size() * sizeof(uint64_t), -1, nullptr)) return false;
  m->caps.assign(h.caps_len, '\0');
  if (h.caps_len && !read_all(&m->caps[0], h.caps_len, -1, nullptr)) return false;
  m->blobs.clear();
  for (uint64_t sz : sizes) {
    auto mem = Memory::alloc_pinned(sz);  // pinned: a later H2D is a DMA
    if (sz && !read_all(mem->data(), sz, -1, nullptr)) return false;
    m->blobs.push_back(mem);
  }
  return true;
}

void Connection::close() {
  bool was = alive_.exchange(false);
  if (fd_ >= 0) {
    if (was) ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  }
}

Listener::~Listener() { close(); }

bool Listener::listen(const std::string& host, int port, std::string* err) {
  sockaddr_in addr;
  if (!resolve(host.empty() ? "0.0.0.0" : host, port, &addr)) {
    if (err) *err = "cannot resolve " + host;
    return false;
  }
  fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (::bind(fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(fd_, 64) != 0) {
    if (err) *err = strfmt("bind/listen ", host, ":", port, ": ", std::strerror(errno));
    ::close(fd_);
    fd_ = -1;
    return false;
  }
  socklen_t len = sizeof(addr);
  getsockname(fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  closed_ = false;
  return true;
}

std::shared_ptr<Connection> Listener::accept(int timeout_ms) {
  if (fd_ < 0 || closed_) return nullptr;
  pollfd pfd{fd_, POLLIN, 0};
  if (::poll(&pfd, 1, timeout_ms) <= 0 || closed_) return nullptr;
  sockaddr_in peer;
  socklen_t len = sizeof(peer);
  int fd = ::accept(fd_, reinterpret_cast<sockaddr*>(&peer), &len);
  if (fd < 0) return nullptr;
  char buf[64];
  inet_ntop(AF_INET, &peer.sin_addr, buf, sizeof(buf));
  return std::make_shared<Connection>(fd, strfmt(buf, ":", ntohs(peer.sin_port)));
}

void Listener::close() {
  closed_ = true;
  if (fd_ >= 0) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  }
}

void MessageQueue::push(Message m) {
  std::lock_guard<std::mutex> lk(mu_);
  q_.push_back(std::move(m));
  cv_.notify_one();
}

bool MessageQueue::pop(Message* m, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return !q_.empty() || flushing_; };
  if (timeout_ms < 0)
    cv_.wait(lk, ready);
  else if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready))
    return false;
  if (flushing_ || q_.empty()) return false;
  *m = std::move(q_.front());
  q_.pop_front();
  return true;
}

void MessageQueue::set_flushing(bool f) {
  std::lock_guard<std::mutex> lk(mu_);
  flushing_ = f;
  if (f) q_.clear();
  cv_.notify_all();
}

size_t MessageQueue::size() {
  std::lock_guard<std::mutex> lk(mu_);
  return q_.size();
}

}  // namespace comm
}  // namespace nnsx
