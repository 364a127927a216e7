// TCP framing for the comm elements (see transport.h).
#include "comm/transport.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <map>
#include <thread>

#include "comm/shm.h"
#include "core/log.h"
#include "core/util.h"
#include "runtime/hip_util.h"

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

constexpr uint32_t kFlagIpc = 1u << 31;       // DATA: a u64 ring offset per blob follows the sizes
constexpr uint32_t kFlagShm = 1u << 30;       // DATA: a u64 shared-memory reference per blob follows the sizes
constexpr uint64_t kInline = ~0ull;           // offset of a blob that travels as bytes
constexpr uint64_t kMinIpcBytes = 4096;       // smaller device blobs are cheaper inline
constexpr size_t kDefaultRing = 256ull << 20;  // per sending end; HBM is 288 GB
constexpr int kRingWaitMs = 200;              // then the blob goes inline

const std::string& boot_id() {
  static const std::string id = [] {
    std::ifstream f("/proc/sys/kernel/random/boot_id");
    std::string v;
    std::getline(f, v);
    return strip(v);
  }();
  return id;
}

std::map<std::string, std::string> parse_kv(const std::string& s) {
  std::map<std::string, std::string> kv;
  for (auto& t : split(s, ';')) {
    auto eq = t.find('=');
    if (eq != std::string::npos) kv[t.substr(0, eq)] = t.substr(eq + 1);
  }
  return kv;
}

std::string to_hex(const void* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string r;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t b = static_cast<const uint8_t*>(p)[i];
    r.push_back(d[b >> 4]);
    r.push_back(d[b & 15]);
  }
  return r;
}

bool from_hex(const std::string& h, void* out, size_t n) {
  if (h.size() != 2 * n) return false;
  auto v = [](char c) { return c <= '9' ? c - '0' : c - 'a' + 10; };
  for (size_t i = 0; i < n; ++i) static_cast<uint8_t*>(out)[i] = static_cast<uint8_t>(v(h[2 * i]) << 4 | v(h[2 * i + 1]));
  return true;
}

uint64_t align_up(uint64_t n) { return (n + 255) & ~255ull; }

}  // namespace

// Sending end's HBM staging ring with an out-of-order slot allocator.
struct IpcRing {
  int dev = 0;
  char* base = nullptr;
  size_t size = 0;
  hipStream_t stream = nullptr;
  std::string desc;  // IPC_RING payload
  std::mutex mu;
  std::condition_variable cv;
  std::map<uint64_t, uint64_t> used;  // offset -> bytes
  uint64_t head = 0;

  static std::shared_ptr<IpcRing> create(int dev, size_t bytes);
  ~IpcRing() {
    hip::DeviceGuard g(dev);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    if (base) (void)hipFree(base);
  }
  // first fit at/after `head`, then from 0; waits for releases up to wait_ms
  bool alloc(uint64_t n, int wait_ms, uint64_t* off) {
    std::unique_lock<std::mutex> lk(mu);
    auto fit = [&](uint64_t from, uint64_t limit, uint64_t* o) {
      uint64_t cand = from;
      for (auto it = used.upper_bound(from); ; ++it) {
        if (it != used.begin()) {
          auto p = std::prev(it);
          cand = std::max(cand, p->first + p->second);
        }
        const uint64_t next = it == used.end() ? limit : std::min<uint64_t>(it->first, limit);
        if (cand + n <= next) {
          *o = cand;
          return true;
        }
        if (it == used.end() || it->first >= limit) return false;
      }
    };
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(wait_ms);
    while (true) {
      if (n <= size && (fit(head, size, off) || fit(0, head, off))) {
        used[*off] = n;
        head = *off + n;
        return true;
      }
      if (n > size || cv.wait_until(lk, deadline) == std::cv_status::timeout) return false;
    }
  }
  void release(uint64_t off) {
    std::lock_guard<std::mutex> lk(mu);
    used.erase(off);
    cv.notify_all();
  }
};

namespace {
// same-process peers reach a ring by its pointer: keep it alive while mapped
std::mutex g_rings_mu;
std::map<uintptr_t, std::weak_ptr<IpcRing>> g_rings;
}  // namespace

std::shared_ptr<IpcRing> IpcRing::create(int dev, size_t bytes) {
  hip::DeviceGuard g(dev);
  auto r = std::make_shared<IpcRing>();
  r->dev = dev;
  r->size = bytes;
  void* p = nullptr;
  hip::check(hipMalloc(&p, bytes), "IPC ring hipMalloc");  // IPC needs hipMalloc, not the async pool
  r->base = static_cast<char*>(p);
  hipIpcMemHandle_t h;
  hip::check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  char pci[64] = {0};
  hip::check(hipDeviceGetPCIBusId(pci, sizeof(pci), dev), "hipDeviceGetPCIBusId");
  r->stream = hip::stream_create(dev);
  r->desc = strfmt("boot=", boot_id(), ";pid=", static_cast<long>(getpid()), ";pci=", pci, ";size=", bytes,
                   ";ptr=", reinterpret_cast<uintptr_t>(p), ";handle=", to_hex(&h, sizeof(h)));
  std::lock_guard<std::mutex> lk(g_rings_mu);
  g_rings[reinterpret_cast<uintptr_t>(p)] = r;
  return r;
}

// Receiving end's mapping of the peer's ring.
struct PeerRing {
  char* base = nullptr;
  size_t size = 0;
  int dev = 0;
  bool opened = false;           // hipIpcOpenMemHandle (other process)
  std::shared_ptr<IpcRing> own;  // same process: the ring itself
  ~PeerRing() {
    if (opened) {
      hip::DeviceGuard g(dev);
      (void)hipIpcCloseMemHandle(base);
    }
  }
};

std::shared_ptr<Connection> make_connection(int fd, std::string peer) {
  auto c = std::make_shared<Connection>(fd, std::move(peer));
  c->self_ = c;
  return c;
}

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
      return make_connection(fd, strfmt(host, ":", port));
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

bool Connection::send_ipc_hello(size_t ring_bytes) {
  if (!hip::available() || boot_id().empty()) return false;
  ring_bytes_ = ring_bytes ? ring_bytes : kDefaultRing;
  hello_sent_ = true;
  Message m;
  m.type = MsgType::IPC_HELLO;
  m.caps = strfmt("boot=", boot_id(), ";pid=", static_cast<long>(getpid()));
  return send(m);
}

bool Connection::send_shm_hello() {
  if (boot_id().empty()) return false;
  Message m;
  m.type = MsgType::SHM_HELLO;
  m.caps = strfmt("boot=", boot_id());
  return send(m);
}

void Connection::send_ack(uint64_t off, uint64_t bytes) {
  Message m;
  m.type = MsgType::IPC_ACK;
  m.seq = off;
  m.duration = static_cast<int64_t>(bytes);
  (void)send(m);
}

bool Connection::handle_control(const Message& m) {
  switch (m.type) {
    case MsgType::IPC_HELLO: {
      auto kv = parse_kv(m.caps);
      if (kv["boot"] == boot_id() && hip::available()) {
        peer_ipc_ = true;
        if (!hello_sent_) send_ipc_hello(ring_bytes_);  // answer: we take ring blobs too
      }
      return true;
    }
    case MsgType::IPC_RING: {
      auto kv = parse_kv(m.caps);
      auto pr = std::make_shared<PeerRing>();
      pr->size = static_cast<size_t>(to_uint(kv["size"]));
      if (hipDeviceGetByPCIBusId(&pr->dev, kv["pci"].c_str()) != hipSuccess) {
        NNSX_LOGE("comm", "IPC ring on an unknown GPU (", kv["pci"], ") from ", peer_);
        return false;
      }
      if (static_cast<long>(to_int(kv["pid"])) == static_cast<long>(getpid())) {
        std::lock_guard<std::mutex> lk(g_rings_mu);
        auto it = g_rings.find(static_cast<uintptr_t>(to_uint(kv["ptr"])));
        pr->own = it == g_rings.end() ? nullptr : it->second.lock();
        if (!pr->own) return false;
        pr->base = pr->own->base;
      } else {
        hipIpcMemHandle_t h;
        if (!from_hex(kv["handle"], &h, sizeof(h))) return false;
        hip::DeviceGuard g(pr->dev);
        void* p = nullptr;
        if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
          NNSX_LOGE("comm", "hipIpcOpenMemHandle failed for the ring of ", peer_);
          return false;
        }
        pr->base = static_cast<char*>(p);
        pr->opened = true;
      }
      peer_ring_ = pr;
      return true;
    }
    case MsgType::IPC_ACK:
      if (ring_) ring_->release(m.seq);
      return true;
    case MsgType::SHM_HELLO:
      if (parse_kv(m.caps)["boot"] == boot_id()) peer_shm_ = true;
      return true;
    case MsgType::SHM_SEG: {
      auto kv = parse_kv(m.caps);
      std::string e;
      auto seg = ShmSegment::open(kv["name"], static_cast<size_t>(to_uint(kv["size"])), &e);
      if (!seg) {
        NNSX_LOGE("comm", "cannot map the shared segment of ", peer_, ": ", e);
        return false;
      }
      std::lock_guard<std::mutex> lk(shm_mu_);
      shm_peer_[static_cast<uint32_t>(to_uint(kv["id"]))] = seg;
      return true;
    }
    case MsgType::SHM_ACK: {
      std::lock_guard<std::mutex> lk(shm_mu_);
      auto it = shm_held_.find(m.seq);
      if (it != shm_held_.end()) shm_held_.erase(it);
      return true;
    }
    default:
      return true;
  }
}

bool Connection::send(const Message& m) {
  if (!alive_) return false;
  if (m.blobs.size() > kMaxBlobs) return false;
  std::vector<uint64_t> offs;
  bool announce = false;
  if (m.type == MsgType::DATA && peer_ipc_) {
    std::lock_guard<std::mutex> lk(ipc_mu_);
    for (size_t i = 0; i < m.blobs.size(); ++i) {
      const MemoryPtr& b = m.blobs[i];
      if (!b->on_device() || b->size() < kMinIpcBytes) continue;
      if (offs.empty()) offs.assign(m.blobs.size(), kInline);
      if (!ring_) {
        try {
          ring_ = IpcRing::create(b->device(), std::max<size_t>(ring_bytes_ ? ring_bytes_ : kDefaultRing, 2 * b->size()));
          announce = true;
        } catch (const std::exception& e) {
          NNSX_LOGW("comm", "device-direct path unavailable (", e.what(), "); sending bytes");
          peer_ipc_ = false;
          offs.clear();
          break;
        }
      }
      uint64_t off;
      if (!ring_->alloc(align_up(b->size()), kRingWaitMs, &off)) continue;  // full: inline
      hip::DeviceGuard g(ring_->dev);
      b->wait_ready(ring_->stream);
      hip::check(hipMemcpyAsync(ring_->base + off, b->data(), b->size(), hipMemcpyDefault, ring_->stream),
                 "IPC ring copy");
      offs[i] = off;
    }
    if (!offs.empty()) {
      // the receiver reads the slot as soon as the header lands: the copy must be done
      hip::DeviceGuard g(ring_->dev);
      hip::check(hipStreamSynchronize(ring_->stream), "IPC ring sync");
      bool any = false;
      for (auto o : offs) any |= o != kInline;
      if (!any) offs.clear();
    }
  }
  // same-host shared memory: host blobs inside one of our segments go as
  // references, held until the peer releases them
  std::vector<Message> segs;
  bool shm = false;
  if (m.type == MsgType::DATA && peer_shm_ && offs.empty()) {
    std::lock_guard<std::mutex> lk(shm_mu_);
    for (size_t i = 0; i < m.blobs.size(); ++i) {
      const MemoryPtr& b = m.blobs[i];
      size_t off = 0;
      std::shared_ptr<ShmSegment> seg;
      if (b->on_device() || !b->size() || !(seg = ShmSegment::find(b->data(), b->size(), &off))) continue;
      auto id = shm_ids_.find(seg->name());
      if (id == shm_ids_.end()) {
        id = shm_ids_.emplace(seg->name(), static_cast<uint32_t>(shm_ids_.size())).first;
        Message r;
        r.type = MsgType::SHM_SEG;
        r.caps = strfmt("id=", id->second, ";name=", seg->name(), ";size=", seg->size());
        segs.push_back(std::move(r));
      }
      if (offs.empty()) offs.assign(m.blobs.size(), kInline);
      offs[i] = (static_cast<uint64_t>(id->second) << 48) | static_cast<uint64_t>(off);
      shm_held_.emplace(offs[i], b);
      shm = true;
    }
  }
  std::lock_guard<std::mutex> lk(send_mu_);
  for (auto& r : segs)
    if (!send_locked(r, nullptr)) return false;
  if (announce) {
    Message r;
    r.type = MsgType::IPC_RING;
    r.caps = ring_->desc;
    if (!send_locked(r, nullptr)) return false;
  }
  if (!send_locked(m, offs.empty() ? nullptr : &offs, shm)) return false;
  if (!offs.empty())
    for (auto o : offs) (shm ? shm_sent_ : ipc_sent_) += o != kInline;
  return true;
}

bool Connection::send_locked(const Message& m, const std::vector<uint64_t>* offs, bool shm) {
  const uint32_t flags = m.flags & ~(kFlagIpc | kFlagShm);
  WireHeader h{kMagic, kVersion, static_cast<uint32_t>(m.type), static_cast<uint32_t>(m.blobs.size()),
               m.client_id, m.seq, m.pts, m.dts, m.duration, static_cast<uint32_t>(m.caps.size()),
               offs ? (flags | (shm ? kFlagShm : kFlagIpc)) : flags};
  std::vector<uint64_t> sizes;
  std::vector<const void*> ptrs;
  for (size_t i = 0; i < m.blobs.size(); ++i) {
    const auto& b = m.blobs[i];
    sizes.push_back(b->size());
    const bool inline_bytes = !offs || (*offs)[i] == kInline;
    ptrs.push_back(inline_bytes ? b->map_host() : nullptr);  // HBM blobs inline: staged through a host mirror
  }
  if (!write_all(&h, sizeof(h))) return false;
  if (!sizes.empty() && !write_all(sizes.data(), sizes.size() * sizeof(uint64_t))) return false;
  if (offs && !write_all(offs->data(), offs->size() * sizeof(uint64_t))) return false;
  if (!m.caps.empty() && !write_all(m.caps.data(), m.caps.size())) return false;
  for (size_t i = 0; i < ptrs.size(); ++i)
    if (ptrs[i] && sizes[i] && !write_all(ptrs[i], sizes[i])) return false;
  return true;
}

bool Connection::recv(Message* m, int timeout_ms, bool* timed_out) {
  if (timed_out) *timed_out = false;
  while (true) {
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
    m->flags = h.flags & ~(kFlagIpc | kFlagShm);
    std::vector<uint64_t> sizes(h.nblobs), offs;
    if (h.nblobs && !read_all(sizes.data(), sizes.size() * sizeof(uint64_t), -1, nullptr)) return false;
    const bool shm = (h.flags & kFlagShm) != 0;
    if (h.flags & (kFlagIpc | kFlagShm)) {
      offs.resize(h.nblobs);
      if (h.nblobs && !read_all(offs.data(), offs.size() * sizeof(uint64_t), -1, nullptr)) return false;
    }
    m->caps.assign(h.caps_len, '\0');
    if (h.caps_len && !read_all(&m->caps[0], h.caps_len, -1, nullptr)) return false;
    m->blobs.clear();
    for (size_t i = 0; i < sizes.size(); ++i) {
      const uint64_t sz = sizes[i];
      if (shm && offs[i] != kInline) {
        const uint64_t ref = offs[i];
        std::shared_ptr<ShmSegment> seg;
        {
          std::lock_guard<std::mutex> lk(shm_mu_);
          auto it = shm_peer_.find(static_cast<uint32_t>(ref >> 48));
          if (it != shm_peer_.end()) seg = std::static_pointer_cast<ShmSegment>(it->second);
        }
        const uint64_t off = ref & ((1ull << 48) - 1);
        if (!seg || off + sz > seg->size()) {
          NNSX_LOGE("comm", "shared-memory blob outside a mapped segment from ", peer_);
          alive_ = false;
          return false;
        }
        std::weak_ptr<Connection> w = self_;
        // zero-copy: downstream reads the producer's frame in place; releasing it hands it back
        m->blobs.push_back(seg->view(off, sz, [w, ref, sz](Memory*) {
          if (auto c = w.lock()) {
            Message a;
            a.type = MsgType::SHM_ACK;
            a.seq = ref;
            a.duration = static_cast<int64_t>(sz);
            (void)c->send(a);
          }
        }));
        ++shm_recv_;
        continue;
      }
      if (!offs.empty() && offs[i] != kInline) {
        auto pr = peer_ring_;
        if (!pr || offs[i] + sz > pr->size) {
          NNSX_LOGE("comm", "ring blob without a mapped ring from ", peer_);
          alive_ = false;
          return false;
        }
        const uint64_t off = offs[i];
        std::weak_ptr<Connection> w = self_;
        // zero-copy: downstream reads the peer's slot; releasing it hands the slot back
        m->blobs.push_back(Memory::wrap(pr->base + off, sz, MemPlace::DEVICE, pr->dev, [pr, w, off, sz](Memory* mm) {
          mm->sync_uses();
          if (auto c = w.lock()) c->send_ack(off, sz);
        }));
        ++ipc_recv_;
        continue;
      }
      auto mem = Memory::alloc_pinned(sz);  // pinned: a later H2D is a DMA
      if (sz && !read_all(mem->data(), sz, -1, nullptr)) return false;
      m->blobs.push_back(mem);
    }
    if (m->type == MsgType::IPC_HELLO || m->type == MsgType::IPC_RING || m->type == MsgType::IPC_ACK ||
        m->type == MsgType::SHM_HELLO || m->type == MsgType::SHM_SEG || m->type == MsgType::SHM_ACK) {
      if (!handle_control(*m)) {
        alive_ = false;
        return false;
      }
      continue;  // control traffic is invisible to the elements
    }
    return true;
  }
}

void Connection::shutdown() {
  if (alive_.exchange(false) && fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
}

void Connection::close() {
  {
    std::lock_guard<std::mutex> lk(shm_mu_);
    shm_held_.clear();  // (the peer can no longer release them)
  }
  bool was = alive_.exchange(false);
  if (fd_ >= 0) {
    if (was) ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  }
}

Listener::~Listener() {
  close();
  release();
}

void Listener::release() {
  const int fd = fd_.exchange(-1);
  if (fd >= 0) ::close(fd);
}

std::string Connection::local_ip() const {
  sockaddr_in addr{};
  socklen_t len = sizeof(addr);
  if (getsockname(fd_, reinterpret_cast<sockaddr*>(&addr), &len) != 0) return "127.0.0.1";
  char buf[64];
  inet_ntop(AF_INET, &addr.sin_addr, buf, sizeof(buf));
  return buf;
}

bool Listener::listen(const std::string& host, int port, std::string* err) {
  release();  // a previous socket: its accept loop was joined after close()
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
  const int lfd = fd_.load();
  if (lfd < 0 || closed_) return nullptr;
  pollfd pfd{lfd, POLLIN, 0};
  if (::poll(&pfd, 1, timeout_ms) <= 0 || closed_) return nullptr;
  sockaddr_in peer;
  socklen_t len = sizeof(peer);
  int fd = ::accept(lfd, reinterpret_cast<sockaddr*>(&peer), &len);
  if (fd < 0) return nullptr;
  char buf[64];
  inet_ntop(AF_INET, &peer.sin_addr, buf, sizeof(buf));
  return make_connection(fd, strfmt(buf, ":", ntohs(peer.sin_port)));
}

// wakes a blocked accept(); the descriptor itself stays open until release()
// (destructor / next listen) so a concurrent accept() never polls a closed --
// possibly already reused -- descriptor number (found by scripts/tsan_check.sh)
void Listener::close() {
  closed_ = true;
  const int fd = fd_.load();
  if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
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
