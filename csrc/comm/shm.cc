// Named POSIX shared-memory segments (see shm.h).
#include "comm/shm.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <cerrno>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "core/log.h"
#include "core/util.h"
#include "runtime/hip_util.h"

namespace nnsx {
namespace comm {

namespace {
std::mutex g_mu;
std::vector<std::weak_ptr<ShmSegment>> g_mapped;            // every live segment of this process
std::map<std::string, std::weak_ptr<ShmSegment>> g_opened;  // peers' segments by name

std::string shm_path(const std::string& name) { return name.empty() || name[0] != '/' ? "/" + name : name; }
}  // namespace

bool ShmSegment::map(int fd, size_t bytes, std::string* err) {
  void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    if (err) *err = strfmt("mmap ", name_, ": ", std::strerror(errno));
    return false;
  }
  base_ = static_cast<char*>(p);
  size_ = bytes;
  // registered in every process that DMAs from / into it (pinned rate, no
  // bounce through the runtime's staging buffers)
  if (hip::available()) {
    hipError_t e = hipHostRegister(base_, size_, hipHostRegisterDefault);
    registered_ = e == hipSuccess;
    if (!registered_) NNSX_LOGW("comm", "hipHostRegister(", name_, "): ", hipGetErrorString(e), "; DMA goes through staging");
  }
  return true;
}

std::shared_ptr<ShmSegment> ShmSegment::create(const std::string& name, size_t bytes, std::string* err) {
  std::shared_ptr<ShmSegment> s(new ShmSegment());
  s->name_ = shm_path(name);
  ::shm_unlink(s->name_.c_str());  // a stale segment of a crashed run
  const int fd = ::shm_open(s->name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) {
    if (err) *err = strfmt("shm_open ", s->name_, ": ", std::strerror(errno));
    return nullptr;
  }
  if (::ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
    if (err) *err = strfmt("ftruncate ", s->name_, ": ", std::strerror(errno));
    ::close(fd);
    ::shm_unlink(s->name_.c_str());
    return nullptr;
  }
  s->owner_ = true;
  const bool ok = s->map(fd, bytes, err);
  ::close(fd);
  if (!ok) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  g_mapped.push_back(s);
  return s;
}

std::shared_ptr<ShmSegment> ShmSegment::open(const std::string& name, size_t bytes, std::string* err) {
  const std::string path = shm_path(name);
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_opened.find(path);
  if (it != g_opened.end())
    if (auto s = it->second.lock()) return s;
  // (the owner in this very process: its own mapping)
  for (auto& w : g_mapped)
    if (auto s = w.lock())
      if (s->name_ == path && s->size_ >= bytes) return s;
  std::shared_ptr<ShmSegment> s(new ShmSegment());
  s->name_ = path;
  const int fd = ::shm_open(path.c_str(), O_RDWR, 0600);
  if (fd < 0) {
    if (err) *err = strfmt("shm_open ", path, ": ", std::strerror(errno));
    return nullptr;
  }
  struct stat st;
  if (::fstat(fd, &st) != 0 || static_cast<size_t>(st.st_size) < bytes) {
    if (err) *err = strfmt("shm segment ", path, " is smaller than ", bytes, " bytes");
    ::close(fd);
    return nullptr;
  }
  const bool ok = s->map(fd, static_cast<size_t>(st.st_size), err);
  ::close(fd);
  if (!ok) return nullptr;
  g_opened[path] = s;
  g_mapped.push_back(s);
  return s;
}

std::shared_ptr<ShmSegment> ShmSegment::find(const void* p, size_t n, size_t* off) {
  const char* c = static_cast<const char*>(p);
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto it = g_mapped.begin(); it != g_mapped.end();) {
    auto s = it->lock();
    if (!s) {
      it = g_mapped.erase(it);
      continue;
    }
    if (c >= s->base_ && c + n <= s->base_ + s->size_) {
      if (off) *off = static_cast<size_t>(c - s->base_);
      return s;
    }
    ++it;
  }
  return nullptr;
}

ShmSegment::~ShmSegment() {
  if (base_) {
    if (registered_) (void)hipHostUnregister(base_);
    ::munmap(base_, size_);
  }
  if (owner_) ::shm_unlink(name_.c_str());
}

MemoryPtr ShmSegment::view(size_t off, size_t n, Memory::Release release) {
  auto self = shared_from_this();
  // (the release runs after the memory's readers -- a DMA may still read the
  // frame -- on the deferred-release thread: runtime/memory.h)
  auto m = Memory::wrap(base_ + off, n, registered_ ? MemPlace::PINNED : MemPlace::HOST, -1,
                        [self, release](Memory*) {
                          if (release) release(nullptr);
                        });
  m->set_allocation(base_);
  m->set_deferred_release();
  return m;
}

}  // namespace comm
}  // namespace nnsx
