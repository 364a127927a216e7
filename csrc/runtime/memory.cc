#include "runtime/memory.h"

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <iterator>
#include <set>
#include <thread>

#include "core/log.h"
#include "core/util.h"
#include "runtime/hip_util.h"

namespace nnsx {

bool Memory::check_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NNSX_MEM_CHECK");
    return e && e[0] == '1';
  }();
  return on;
}

namespace {

// fill a host block with the poison pattern (MEM_CHECK)
void poison_host(void* p, size_t n) {
  uint32_t* w = static_cast<uint32_t*>(p);
  for (size_t i = 0; i < n / 4; ++i) w[i] = Memory::kPoison;
}

// Deferred host releases: the last reference to a host / pinned block that an
// asynchronous copy still reads (H2D: recorded uses) or writes (D2H: the ready
// event) drops on some pipeline thread -- a source, the converter -- which must
// not stall on that copy.  The block goes to this thread instead, which waits
// for the copies' events and then frees it (pinned: back to the shared pool,
// where the next frame may pick it up).  FIFO, one thread per process.
class DeferredRelease {
 public:
  struct Item {
    std::vector<std::pair<int, hipEvent_t>> events;
    void* data;
    size_t size;
    MemPlace place;
    std::function<void()> fn;  // instead of a free: a wrapped memory's release (set_deferred_release)
    uint64_t seq = 0;          // (queue order)
  };
  // backpressure: past this many queued blocks / bytes (the GPU has fallen
  // behind its copies) the releasing thread frees the block itself, after the
  // copies' events -- the pinned pool cannot grow without bound
  static constexpr size_t kMaxItems = 256;
  static constexpr size_t kMaxBytes = size_t{1} << 30;
  static DeferredRelease& get() {
    static DeferredRelease* d = [] {
      auto* r = new DeferredRelease();  // (never destroyed: process-lifetime thread)
      std::atexit([] { get().shutdown(); });
      return r;
    }();
    return *d;
  }
  void push(Item it) {
    std::unique_lock<std::mutex> lk(mu_);
    if (stopping_ || q_.size() >= kMaxItems || bytes_ + it.size > kMaxBytes) {
      lk.unlock();
      release(it);
      return;
    }
    bytes_ += it.size;
    it.seq = ++queued_;
    pending_.insert(it.seq);
    q_.push_back(std::move(it));
    cv_.notify_all();
  }
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t target = queued_;
    done_cv_.wait(lk, [&] { return pending_.empty() || *pending_.begin() > target; });
  }
  // process exit (atexit, before the HIP runtime's own teardown): the queue is
  // worked off -- bounded, the copies it waits for are already issued -- and
  // later releases are done in place
  void shutdown() {
    std::unique_lock<std::mutex> lk(mu_);
    stopping_ = true;
    const uint64_t target = queued_;
    done_cv_.wait_for(lk, std::chrono::seconds(5), [&] { return pending_.empty() || *pending_.begin() > target; });
  }

 private:
  DeferredRelease() {
    std::thread([this] { run(); }).detach();
  }
  static void release(Item& it) {
    for (auto& e : it.events) {
      (void)hipEventSynchronize(e.second);
      hip::event_put(e.first, e.second);
    }
    if (it.fn) {
      it.fn();
      return;
    }
    if (Memory::check_enabled() && it.size) poison_host(it.data, it.size);
    if (it.place == MemPlace::PINNED)
      hip::pinned_free(it.data, it.size);
    else
      hip::host_free(it.data);
  }
  void run() {
    // Out of order: the first queued item whose events have all completed goes
    // first, so one block read by a long job (a frame ring a slow consumer
    // holds) does not hold back the frees queued behind it; while nothing is
    // complete the thread polls every 50 us (only while items are pending).
    for (;;) {
      Item it;
      bool found = false;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        for (auto i = q_.begin(); i != q_.end(); ++i) {
          bool done = true;
          for (auto& e : i->events)
            if (hipEventQuery(e.second) != hipSuccess) {
              done = false;
              break;
            }
          if (done) {
            it = std::move(*i);
            q_.erase(i);
            found = true;
            break;
          }
        }
        if (!found) {
          cv_.wait_for(lk, std::chrono::microseconds(50));
          continue;
        }
      }
      release(it);
      std::lock_guard<std::mutex> lk(mu_);
      bytes_ -= it.size;
      pending_.erase(it.seq);
      done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Item> q_;
  std::set<uint64_t> pending_;  // queued, not yet released (drain / shutdown)
  uint64_t queued_ = 0;
  size_t bytes_ = 0;
  bool stopping_ = false;
};

}  // namespace

void Memory::drain_deferred() {
  if (hip::available()) DeferredRelease::get().drain();
}

// lifetime self-test support (runtime/selftest.cc): undo one fix at run time so
// the test that pins it can be shown to fail without it
namespace {
std::atomic<int> g_mutation{0};
std::atomic<const void*> g_watch{nullptr};  // test_watch_free: the block whose free is watched
std::atomic<bool> g_watch_freed{false};
}  // namespace
int Memory::set_test_mutation(int m) { return g_mutation.exchange(m); }
void Memory::test_watch_free(const void* p) {
  g_watch_freed.store(false);
  g_watch.store(p);
}
bool Memory::test_watched_freed() { return g_watch_freed.load(); }

Memory::Memory(void* data, size_t size, MemPlace place, int device, Release release)
    : data_(data), size_(size), place_(place), device_(device), release_(std::move(release)) {}

Memory::~Memory() {
  state_.store(1);
  if (deferrable_) {
    // alloc_host / alloc_pinned: a pending D2H may still be landing here (pinned:
    // the producer's ready event) and pending H2Ds may still read it (recorded
    // uses); the block may be handed out again at once by malloc or the pinned
    // pool, so it is freed only after them -- by the deferred-release thread,
    // never by blocking the thread that dropped the last reference
    std::vector<std::pair<int, hipEvent_t>> evs;
    for (auto& u : uses_) evs.emplace_back(u.dev, u.event);
    uses_.clear();
    if (ready_ && place_ == MemPlace::PINNED) {
      evs.emplace_back(ready_dev_, ready_);
      ready_ = nullptr;
    }
    if (!evs.empty()) {
      DeferredRelease::get().push({std::move(evs), data_, size_, place_});
    } else {
      if (check_enabled() && size_) poison_host(data_, size_);
      if (place_ == MemPlace::PINNED)
        hip::pinned_free(data_, size_);
      else
        hip::host_free(data_);
    }
  } else {
    // other host memory (wrapped buffers with their own release) read by an
    // asynchronous H2D copy: released only after that copy ran -- by the
    // deferred-release thread when the release does not need this object
    // (set_deferred_release: shared-memory frames handed back to their producer)
    if (place_ != MemPlace::DEVICE && !uses_.empty() && defer_wrap_ && release_) {
      std::vector<std::pair<int, hipEvent_t>> evs;
      for (auto& u : uses_) evs.emplace_back(u.dev, u.event);
      uses_.clear();
      Release rel = std::move(release_);
      DeferredRelease::get().push({std::move(evs), nullptr, 0, place_, [rel] { rel(nullptr); }});
    } else {
      if (place_ != MemPlace::DEVICE && !uses_.empty()) sync_uses();
      if (release_) release_(this);
    }
  }
  if (ready_) hip::event_put(ready_dev_, ready_);
  for (auto& u : uses_) hip::event_put(u.dev, u.event);
}

void Memory::check_live(const char* what) const {
  if (!check_enabled()) return;
  for (const Memory* m = this; m; m = m->parent_.get())
    if (m->state_.load() != 0) {
      NNSX_LOGE("memcheck", what, " of a memory whose release has begun (", data_, ", ", size_, " bytes)");
      throw Error(std::string("NNSX_MEM_CHECK: ") + what + " of a released memory");
    }
}

MemoryPtr Memory::alloc_host(size_t size) {
  void* p = hip::host_alloc(size);
  auto m = std::make_shared<Memory>(p, size, MemPlace::HOST, -1, nullptr);
  m->deferrable_ = hip::available();  // (no GPU: nothing is ever in flight)
  if (!m->deferrable_) m->release_ = [](Memory* mm) { hip::host_free(mm->data()); };
  return m;
}

MemoryPtr Memory::alloc_pinned(size_t size) {
  if (!hip::available()) return alloc_host(size);
  void* p = hip::pinned_alloc(size);
  auto m = std::make_shared<Memory>(p, size, MemPlace::PINNED, -1, nullptr);
  m->deferrable_ = true;
  return m;
}

MemoryPtr Memory::alloc_device(size_t size, int dev, hipStream_t stream) {
  void* p = hip::device_alloc(dev, size, stream);
  return std::make_shared<Memory>(p, size, MemPlace::DEVICE, dev, [dev](Memory* m) {
    // the block returns to the stream-ordered pool only after the producer and
    // every recorded reader: the free is ordered on a process-lifetime stream
    hipStream_t rs = hip::release_stream(dev);
    m->wait_ready(rs);
    m->wait_uses(rs);
    hip::DeviceGuard g(dev);
    if (check_enabled() && m->size() >= 4)
      (void)hipMemsetD32Async(m->data(), static_cast<int>(kPoisonDevice), m->size() / 4, rs);
    // The pool hands a block freed on rs to an allocation on another stream
    // before rs has reached the free (measured: a filter input's device mirror,
    // freed on rs behind the wait for the filter's replay, came back at the same
    // address for the next frame's mirror on the filter's stream while the wait
    // and the poison were still pending -- profiles/r6_memcheck_mirror_open.txt;
    // with the pool's cross-stream reuse switched off too).  So the free is
    // issued only once rs has passed the waits: by the deferred-release thread,
    // after an event recorded here.
    // (NNSX_DEVICE_FREE=direct: the free straight on rs, as before -- A/B only)
    static const bool direct = [] {
      const char* v = std::getenv("NNSX_DEVICE_FREE");
      return v && std::string(v) == "direct";
    }();
    void* p = m->data();
    if (direct) {
      hip::device_free(dev, p, rs);
      return;
    }
    hipEvent_t e = hip::event_get(dev);
    hip::check(hipEventRecord(e, rs), "hipEventRecord(release)");
    DeferredRelease::get().push({{{dev, e}}, nullptr, 0, MemPlace::DEVICE, [dev, p] {
      hip::device_free(dev, p, hip::release_stream(dev));
      if (p == g_watch.load()) g_watch_freed.store(true);
    }});
  });
}

MemoryPtr Memory::device_mirror(int dev) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = dev_mirror_.find(dev);
  return it == dev_mirror_.end() ? nullptr : it->second;
}

// ------------------------------------------------------- DeviceBufferPool ----
namespace {
std::mutex& pool_registry_mu() {
  static std::mutex m;
  return m;
}
std::map<uint64_t, std::weak_ptr<DeviceBufferPool>>& pool_registry() {
  static std::map<uint64_t, std::weak_ptr<DeviceBufferPool>> r;
  return r;
}
}  // namespace

std::shared_ptr<DeviceBufferPool> DeviceBufferPool::create(int dev, size_t size, size_t max_blocks) {
  auto p = std::shared_ptr<DeviceBufferPool>(new DeviceBufferPool(dev, size, max_blocks));
  std::lock_guard<std::mutex> lk(pool_registry_mu());
  auto& r = pool_registry();
  for (auto it = r.begin(); it != r.end();) it = it->second.expired() ? r.erase(it) : std::next(it);
  r[p->id()] = p;
  return p;
}

std::shared_ptr<DeviceBufferPool> DeviceBufferPool::find(uint64_t id) {
  std::lock_guard<std::mutex> lk(pool_registry_mu());
  auto it = pool_registry().find(id);
  return it == pool_registry().end() ? nullptr : it->second.lock();
}

void DeviceBufferPool::preallocate(hipStream_t stream) {
  std::lock_guard<std::mutex> lk(mu_);
  while (blocks_.size() < max_) {
    Block b;
    b.ptr = hip::device_alloc(dev_, size_, stream);
    blocks_.push_back(b);
  }
}

std::vector<void*> DeviceBufferPool::block_addresses() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<void*> v;
  for (const auto& b : blocks_) v.push_back(b.ptr);
  return v;
}

DeviceBufferPool::DeviceBufferPool(int dev, size_t size, size_t max_blocks) : dev_(dev), size_(size), max_(max_blocks) {
  static std::atomic<uint64_t> next{1};
  id_ = next++;
}

DeviceBufferPool::~DeviceBufferPool() {
  // blocks still out are owned by their Memory (freed on release); free ones go now,
  // ordered after their last readers
  hip::DeviceGuard g(dev_);
  hipStream_t rs = hip::release_stream(dev_);
  for (auto& b : blocks_) {
    if (!b.free) continue;
    if (b.released) {
      (void)hipStreamWaitEvent(rs, b.released, 0);
      hip::event_put(dev_, b.released);
    }
    hip::device_free(dev_, b.ptr, rs);
  }
}

size_t DeviceBufferPool::blocks() const {
  std::lock_guard<std::mutex> lk(mu_);
  return blocks_.size();
}

MemoryPtr DeviceBufferPool::acquire(hipStream_t stream) {
  int slot = -1;
  void* p = nullptr;
  hipEvent_t wait = nullptr;
  bool poisoned = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    hip::DeviceGuard g(dev_);
    // 1. a free block whose previous readers are done -- the most recently
    // returned one, so the steady state cycles through as few addresses as it
    // needs (a consumer keying per-address state, e.g. an in-place hipGraph
    // instance per block, then sees every address during warm-up)
    int oldest = -1;
    for (size_t i = 0; i < blocks_.size(); ++i) {
      Block& b = blocks_[i];
      if (!b.free) continue;
      if (!b.released || hipEventQuery(b.released) == hipSuccess) {
        if (slot < 0 || b.seq > blocks_[static_cast<size_t>(slot)].seq) slot = static_cast<int>(i);
      } else if (oldest < 0 || b.seq < blocks_[static_cast<size_t>(oldest)].seq) {
        oldest = static_cast<int>(i);
      }
    }
    // 2. grow the pool
    if (slot < 0 && blocks_.size() < max_) {
      Block b;
      b.ptr = hip::device_alloc(dev_, size_, stream);
      blocks_.push_back(b);
      slot = static_cast<int>(blocks_.size()) - 1;
    }
    // 3. the oldest free block, once its readers are done (host wait below)
    if (slot < 0 && oldest >= 0) {
      slot = oldest;
      wait = blocks_[static_cast<size_t>(oldest)].released;
    }
    if (slot >= 0) {
      Block& b = blocks_[static_cast<size_t>(slot)];
      poisoned = pool_poisoned_.erase(slot) > 0;
      b.free = false;
      wait = b.released;  // complete (case 1) or waited for below (case 3); then recycled
      b.released = nullptr;
      p = b.ptr;
    }
  }
  if (slot < 0) return Memory::alloc_device(size_, dev_, stream);  // all blocks out: no pooling
  if (wait) {
    hip::DeviceGuard g(dev_);
    hip::check(hipEventSynchronize(wait), "pool acquire wait");
    hip::event_put(dev_, wait);
  }
  if (poisoned) {
    // the block was poisoned when its previous use was released: it must still
    // hold the pattern, else something wrote to it after the release
    hip::DeviceGuard g(dev_);
    uint32_t head = 0, tail = 0;
    hip::check(hipMemcpy(&head, p, 4, hipMemcpyDeviceToHost), "memcheck head");
    hip::check(hipMemcpy(&tail, static_cast<char*>(p) + (size_ / 4 - 1) * 4, 4, hipMemcpyDeviceToHost),
               "memcheck tail");
    if (head != Memory::kPoison || tail != Memory::kPoison) {
      NNSX_LOGE("memcheck", "pool block ", p, " (", size_, " bytes) was written after its release");
      throw Error("NNSX_MEM_CHECK: pooled device block written after its release");
    }
  }
  std::weak_ptr<DeviceBufferPool> wp = shared_from_this();
  const int dev = dev_;
  const size_t size = size_;
  auto m = std::make_shared<Memory>(p, size, MemPlace::DEVICE, dev, [wp, slot, dev](Memory* mm) {
    hip::DeviceGuard g(dev);
    hipStream_t rs = hip::release_stream(dev);
    mm->wait_ready(rs);
    mm->wait_uses(rs);
    const bool poison = Memory::check_enabled() && mm->size() >= 4;
    if (poison) (void)hipMemsetD32Async(mm->data(), static_cast<int>(Memory::kPoison), mm->size() / 4, rs);
    if (auto pool = wp.lock()) {
      if (poison) pool->mark_poisoned(slot);
      hipEvent_t e = hip::event_get(dev);
      hip::check(hipEventRecord(e, rs), "pool release");
      pool->put_back(slot, e);
    } else {
      hip::device_free(dev, mm->data(), rs);  // the pool is gone: the block goes with its last user
    }
  });
  (void)size;
  m->tags()[kPoolTag] = static_cast<int64_t>(id_);
  m->tags()[kSlotTag] = slot;
  return m;
}

void DeviceBufferPool::mark_poisoned(int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  pool_poisoned_.insert(slot);
}

void DeviceBufferPool::put_back(int slot, hipEvent_t released) {
  std::lock_guard<std::mutex> lk(mu_);
  Block& b = blocks_.at(static_cast<size_t>(slot));
  if (b.released) hip::event_put(dev_, b.released);
  b.released = released;
  b.free = true;
  b.seq = ++seq_;
}

MemoryPtr Memory::wrap(void* data, size_t size, MemPlace place, int device, Release release) {
  return std::make_shared<Memory>(data, size, place, device, std::move(release));
}

MemoryPtr Memory::view(const MemoryPtr& parent, size_t offset, size_t size) {
  if (offset + size > parent->size()) throw Error("Memory::view out of range");
  auto m = std::make_shared<Memory>(static_cast<char*>(parent->data()) + offset, size, parent->place(),
                                    parent->device(), nullptr);
  m->parent_ = parent;
  return m;
}

MemoryPtr Memory::from_bytes(const void* src, size_t size) {
  auto m = alloc_host(size);
  if (size) std::memcpy(m->data(), src, size);
  return m;
}

void Memory::mark_ready(hipStream_t stream) {
  Memory* r = root();
  if (r->place_ == MemPlace::HOST) return;
  // pinned host memory has no device of its own: the event belongs to the
  // producing stream's device (the caller's current device)
  int dev = r->device_;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(r->ev_mu_);
  if (r->ready_ && r->ready_dev_ != dev) {
    hip::event_put(r->ready_dev_, r->ready_);
    r->ready_ = nullptr;
  }
  if (!r->ready_) {
    r->ready_ = hip::event_get(dev);
    r->ready_dev_ = dev;
  }
  hip::check(hipEventRecord(r->ready_, stream), "hipEventRecord(ready)");
  ++r->ready_gen_;
}

void Memory::wait_ready(hipStream_t stream) const {
  const Memory* r = root();
  std::lock_guard<std::mutex> lk(r->ev_mu_);
  if (r->ready_) hip::check(hipStreamWaitEvent(stream, r->ready_, 0), "hipStreamWaitEvent(ready)");
}

void Memory::sync_ready() const {
  const Memory* r = root();
  hipEvent_t e;
  uint64_t gen;
  {
    std::lock_guard<std::mutex> lk(r->ev_mu_);
    if (r->ready_gen_ == r->synced_gen_) return;  // already waited for this recording
    e = r->ready_;
    gen = r->ready_gen_;
  }
  if (e) hip::check(hipEventSynchronize(e), "hipEventSynchronize(ready)");
  // views of one batch share the root: the first frame waits, the rest return here
  std::lock_guard<std::mutex> lk(r->ev_mu_);
  if (r->synced_gen_ < gen) r->synced_gen_ = gen;
}

void Memory::record_use(hipStream_t stream, int dev) {
  // a read on device `dev` of a memory that lives elsewhere read its device
  // mirror (map_device): the mirror is freed / recycled in the order of the
  // stream that mapped it, so a reader on another stream (a filter's replay
  // lane) must hold it too
  MemoryPtr mirror;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = dev_mirror_.find(dev);
    if (it != dev_mirror_.end()) mirror = it->second;
  }
  if (mirror && g_mutation.load() != kMutMirrorNotHeld) mirror->record_use(stream, dev);
  record_use_self(stream, dev);
}

void Memory::record_use_self(hipStream_t stream, int dev) {
  Memory* r = root();
  std::lock_guard<std::mutex> lk(r->ev_mu_);
  // one event per reading stream: work on a stream completes in order, so the
  // latest record there covers every earlier read (a ring frame read by every
  // pass keeps one event instead of one per frame)
  for (auto& u : r->uses_)
    if (u.stream == stream && u.dev == dev) {
      hip::check(hipEventRecord(u.event, stream), "hipEventRecord(use)");
      return;
    }
  hipEvent_t e = hip::event_get(dev);
  hip::check(hipEventRecord(e, stream), "hipEventRecord(use)");
  r->uses_.push_back({dev, stream, e});
}

void Memory::wait_uses(hipStream_t stream) const {
  const Memory* r = root();
  std::lock_guard<std::mutex> lk(r->ev_mu_);
  for (auto& u : r->uses_) (void)hipStreamWaitEvent(stream, u.event, 0);
}

void Memory::sync_uses() const {
  const Memory* r = root();
  std::lock_guard<std::mutex> lk(r->ev_mu_);
  for (auto& u : r->uses_) (void)hipEventSynchronize(u.event);
}

const void* Memory::map_host() {
  check_live("map_host");
  if (place_ != MemPlace::DEVICE) {
    if (place_ == MemPlace::PINNED) sync_ready();  // a D2H may be landing here
    return data_;
  }
  std::lock_guard<std::mutex> lk(mu_);
  if (!host_mirror_) {
    auto mirror = alloc_pinned(size_);
    hip::DeviceGuard g(device_);
    hipStream_t s = hip::thread_copy_stream(device_);
    wait_ready(s);  // producer first, then copy, then block: the caller wants bytes now
    if (size_) hip::check(hipMemcpyAsync(mirror->data(), data_, size_, hipMemcpyDeviceToHost, s), "D2H");
    hip::check(hipStreamSynchronize(s), "hipStreamSynchronize(map_host)");
    host_mirror_ = mirror;
  }
  return host_mirror_->data();
}

const void* Memory::map_device(int dev, hipStream_t stream) {
  check_live("map_device");
  if (place_ == MemPlace::DEVICE && device_ == dev) {
    wait_ready(stream);
    return data_;
  }
  std::lock_guard<std::mutex> lk(mu_);
  auto it = dev_mirror_.find(dev);
  if (it != dev_mirror_.end()) {
    it->second->wait_ready(stream);
    return it->second->data();
  }
  auto mirror = alloc_device(size_, dev, stream);
  hip::DeviceGuard g(dev);
  if (place_ == MemPlace::DEVICE) {
    wait_ready(stream);  // peer copy over xGMI after the producer
    if (size_) hip::check(hipMemcpyPeerAsync(mirror->data(), dev, data_, device_, size_, stream), "P2P");
    record_use_self(stream, dev);  // (mu_ is held: not record_use, which looks up the mirrors)
  } else {
    if (size_) hip::check(hipMemcpyAsync(mirror->data(), data_, size_, hipMemcpyHostToDevice, stream), "H2D");
    // the source may be read asynchronously (pinned always; pageable too, for the
    // runtime's own staging): it must not be freed / recycled before the copy ran
    // (a pageable frame freed at once came back from malloc holding the next
    // frame, and the queued copy read that: test_hipgraph_static_outputs_...)
    if (size_ && g_mutation.load() != kMutHostFreedEarly) record_use_self(stream, dev);
  }
  mirror->mark_ready(stream);
  dev_mirror_[dev] = mirror;
  return mirror->data();
}

// ------------------------------------------------------------ helpers ----

bool buffer_from_config(const BufferPtr& in, const TensorsConfig& config, BufferPtr* out) {
  auto b = make_buffer();
  b->copy_metadata_from(*in);
  if (config.is_static()) {
    unsigned n = config.info.num_tensors;
    if (in->n_memory() == n) {
      b->mems = in->mems;
      for (unsigned i = 0; i < n; ++i)
        if (in->mems[i]->size() != config.info.at(i).size()) return false;
    } else if (in->n_memory() >= 1) {
      // one (or more) contiguous chunk(s): concatenate views across memories
      size_t total = in->total_size();
      if (total != config.info.size()) return false;
      size_t mi = 0, moff = 0;
      for (unsigned i = 0; i < n; ++i) {
        size_t need = config.info.at(i).size();
        if (mi >= in->n_memory()) return false;
        if (moff + need <= in->mems[mi]->size()) {
          b->mems.push_back(Memory::view(in->mems[mi], moff, need));
          moff += need;
          if (moff == in->mems[mi]->size()) {
            ++mi;
            moff = 0;
          }
        } else {
          return false;  // tensor straddles memories: unsupported
        }
      }
    } else {
      return false;
    }
  } else {
    // flexible/sparse: one tensor per memory, or headers walked inside one memory
    for (auto& m : in->mems) {
      if (m->has_meta()) {
        b->mems.push_back(m);
        continue;
      }
      const uint8_t* p = static_cast<const uint8_t*>(m->map_host());
      size_t off = 0;
      while (off < m->size()) {
        MetaInfo meta;
        if (!MetaInfo::parse(p + off, m->size() - off, &meta)) return false;
        size_t sz = meta.header_size() + meta.data_size();
        if (off + sz > m->size()) return false;
        b->mems.push_back(Memory::view(m, off, sz));
        off += sz;
      }
    }
  }
  *out = b;
  return true;
}

MemoryPtr make_flexible(const MemoryPtr& mem, const MetaInfo& meta) {
  if (mem->on_device()) {
    auto v = Memory::view(mem, 0, mem->size());
    v->set_meta(meta);
    return v;
  }
  auto m = Memory::alloc_host(kMetaHeaderSize + mem->size());
  meta.write(m->data());
  if (mem->size()) std::memcpy(static_cast<char*>(m->data()) + kMetaHeaderSize, mem->map_host(), mem->size());
  return m;
}

bool parse_flexible(const MemoryPtr& mem, MetaInfo* meta, MemoryPtr* payload) {
  if (mem->has_meta()) {
    *meta = mem->meta();
    if (payload) *payload = mem;
    return meta->valid();
  }
  if (mem->size() < kMetaHeaderSize) return false;
  const void* p = mem->on_device() ? nullptr : mem->map_host();
  MetaInfo m;
  if (p) {
    if (!MetaInfo::parse(p, mem->size(), &m)) return false;
  } else {
    // device memory with in-band header: read the 128 bytes only
    uint8_t hdr[kMetaHeaderSize];
    hip::DeviceGuard g(mem->device());
    hipStream_t s = hip::thread_copy_stream(mem->device());
    mem->wait_ready(s);
    hip::check(hipMemcpyAsync(hdr, mem->data(), kMetaHeaderSize, hipMemcpyDeviceToHost, s), "D2H hdr");
    hip::check(hipStreamSynchronize(s), "sync hdr");
    if (!MetaInfo::parse(hdr, kMetaHeaderSize, &m)) return false;
  }
  size_t hs = m.header_size();
  size_t ds = m.data_size();
  if (hs + ds > mem->size()) return false;
  *meta = m;
  if (payload) *payload = Memory::view(mem, hs, ds);
  return true;
}

std::vector<uint8_t> serialize_with_header(const MemoryPtr& mem) {
  std::vector<uint8_t> out;
  const uint8_t* p = static_cast<const uint8_t*>(mem->map_host());
  if (mem->has_meta()) {
    out.resize(kMetaHeaderSize + mem->size());
    mem->meta().write(out.data());
    std::memcpy(out.data() + kMetaHeaderSize, p, mem->size());
  } else {
    out.assign(p, p + mem->size());
  }
  return out;
}

namespace {
// Byte layout of the reference's GstTensorExtraInfo on LP64
// (nnstreamer_plugin_api_impl.c:1477-1490, tensor_typedef.h GstTensorInfo):
// u32 magic, u32 version, u32 num_extra_tensors, (pad), u64 reserved (= size
// of the 16th tensor), then 200 GstTensorInfo {char* name; tensor_type type;
// uint32 dimension[8]} of 48 bytes each (name is a pointer in the writer's
// process: written as 0, ignored on read).  The 16th tensor's bytes follow the
// header, then each extra tensor's.
struct ExtraHeader {
  uint32_t magic;
  uint32_t version;
  uint32_t num_extra;
  uint32_t pad;
  uint64_t reserved;
};
struct ExtraEntry {
  uint64_t name;
  uint32_t type;
  uint32_t dim[kRankLimit];
  uint32_t pad;
};
static_assert(sizeof(ExtraHeader) == 24 && sizeof(ExtraEntry) == 48, "GstTensorExtraInfo layout");
constexpr size_t kExtraInfoSize = sizeof(ExtraHeader) + sizeof(ExtraEntry) * kSizeExtraLimit;  // 9624
}  // namespace

std::vector<MemoryPtr> pack_extra(const std::vector<MemoryPtr>& mems, const TensorsInfo& info) {
  if (mems.size() <= static_cast<size_t>(kSizeLimit)) return mems;
  std::vector<MemoryPtr> out(mems.begin(), mems.begin() + (kSizeLimit - 1));
  size_t total = kExtraInfoSize;
  for (size_t i = kSizeLimit - 1; i < mems.size(); ++i) total += mems[i]->size();
  auto blk = Memory::alloc_host(total);
  std::memset(blk->data(), 0, kExtraInfoSize);
  auto* h = static_cast<ExtraHeader*>(blk->data());
  h->magic = kExtraMagic;
  h->num_extra = static_cast<uint32_t>(mems.size() - kSizeLimit);
  h->reserved = mems[kSizeLimit - 1]->size();
  auto* ent = reinterpret_cast<ExtraEntry*>(h + 1);
  for (int i = 0; i < kSizeExtraLimit; ++i) ent[i].type = static_cast<uint32_t>(DType::END);  // gst_tensor_info_init
  for (size_t i = kSizeLimit; i < mems.size(); ++i) {
    const auto& ti = info.at(static_cast<unsigned>(i));
    ent[i - kSizeLimit].type = static_cast<uint32_t>(ti.type);
    for (int d = 0; d < kRankLimit; ++d) ent[i - kSizeLimit].dim[d] = ti.dim[d];
  }
  size_t off = kExtraInfoSize;
  for (size_t i = kSizeLimit - 1; i < mems.size(); ++i) {
    std::memcpy(static_cast<char*>(blk->data()) + off, mems[i]->map_host(), mems[i]->size());
    off += mems[i]->size();
  }
  out.push_back(blk);
  return out;
}

std::vector<MemoryPtr> unpack_extra(const std::vector<MemoryPtr>& mems, TensorsInfo* info) {
  if (mems.size() != static_cast<size_t>(kSizeLimit)) return mems;
  const auto& last = mems.back();
  if (last->size() < kExtraInfoSize) return mems;
  const auto* h = static_cast<const ExtraHeader*>(last->map_host());
  if (h->magic != kExtraMagic) return mems;
  std::vector<MemoryPtr> out(mems.begin(), mems.end() - 1);
  size_t off = kExtraInfoSize;
  out.push_back(Memory::view(last, off, h->reserved));
  off += h->reserved;
  const auto* ent = reinterpret_cast<const ExtraEntry*>(h + 1);
  for (uint32_t i = 0; i < h->num_extra; ++i) {
    TensorInfo ti;
    ti.type = static_cast<DType>(ent[i].type);
    for (int d = 0; d < kRankLimit; ++d) ti.dim[d] = ent[i].dim[d];
    size_t sz = ti.size();
    out.push_back(Memory::view(last, off, sz));
    off += sz;
    if (info) info->at(kSizeLimit + i) = ti;
  }
  if (info && info->num_tensors < out.size()) info->num_tensors = static_cast<unsigned>(out.size());
  return out;
}

}  // namespace nnsx

