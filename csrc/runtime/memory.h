// Memory / Buffer: the payload model that replaces GstMemory / GstBuffer.
//
// A Memory is one tensor chunk.  It lives on the host (plain or pinned) or on
// a GPU.  Device memories carry a `ready` event recorded on the producer's
// stream: consumers make their own stream wait on it (never a host sync), and
// record `uses` so the block is only recycled once every reader finished.
// `map_host` / `map_device` are the caps-boundary copies: a host<->device
// transfer happens only where a host-only element meets device data (or the
// reverse); adjacent GPU elements exchange device pointers zero-copy.
//
// Reference: gst_tensor_buffer_from_config / append/get nth memory
// (gst/nnstreamer/nnstreamer_plugin_api_impl.c:452-556,1477-1768).
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "core/types.h"

namespace nnsx {

enum class MemPlace { HOST = 0, PINNED = 1, DEVICE = 2 };

class Memory;
using MemoryPtr = std::shared_ptr<Memory>;

class Memory : public std::enable_shared_from_this<Memory> {
 public:
  using Release = std::function<void(Memory*)>;

  Memory(void* data, size_t size, MemPlace place, int device, Release release);
  ~Memory();
  Memory(const Memory&) = delete;
  Memory& operator=(const Memory&) = delete;

  static MemoryPtr alloc_host(size_t size);
  static MemoryPtr alloc_pinned(size_t size);
  static MemoryPtr alloc_device(size_t size, int dev, hipStream_t stream);
  // Wrap external memory.  `release` runs when the last reference drops.
  static MemoryPtr wrap(void* data, size_t size, MemPlace place, int device, Release release = nullptr);
  // Sub-view sharing the parent's storage (zero-copy slice / split / demux).
  static MemoryPtr view(const MemoryPtr& parent, size_t offset, size_t size);
  // Host copy of bytes.
  static MemoryPtr from_bytes(const void* src, size_t size);

  void* data() const { return data_; }
  size_t size() const { return size_; }
  MemPlace place() const { return place_; }
  int device() const { return device_; }
  bool on_device() const { return place_ == MemPlace::DEVICE; }
  bool host_accessible() const { return place_ != MemPlace::DEVICE; }

  // --- producer side (device memories) ---
  // Record the ready event on `stream` (after the producing work is enqueued).
  void mark_ready(hipStream_t stream);
  // --- consumer side ---
  // Make `stream` wait until the producer's writes are visible.
  void wait_ready(hipStream_t stream) const;
  // Host wait for the producer (map paths).
  void sync_ready() const;
  // Record that work enqueued on `stream` reads this memory.
  void record_use(hipStream_t stream, int dev);
  // Events of every recorded reader (used when releasing the block).
  void wait_uses(hipStream_t stream) const;
  void sync_uses() const;

  // Host-visible pointer.  Device memories are copied into a cached pinned
  // mirror (one D2H per memory, however many host readers).
  const void* map_host();
  // Device pointer on `dev`, ordered on `stream`.  Host memories are uploaded
  // into a cached device mirror (one H2D per memory and device).
  const void* map_device(int dev, hipStream_t stream);

  // Typed metadata carried per memory.
  std::map<std::string, int64_t>& tags() { return tags_; }

  // Flexible/sparse meta attached out-of-band (device memories keep the
  // 128-byte header off the payload so no payload copy is needed; host
  // memories carry it in-band like the reference).
  bool has_meta() const { return has_meta_; }
  const MetaInfo& meta() const { return meta_; }
  void set_meta(const MetaInfo& m) { meta_ = m; has_meta_ = true; }

  Memory* root() { return parent_ ? parent_->root() : this; }
  const Memory* root() const { return parent_ ? parent_->root() : this; }
  // the allocation this memory lies in (one copy may span several memories of
  // the same allocation -- e.g. the frames of one capture ring): the root's
  // own block unless set_allocation named a larger one (a shared segment)
  const void* allocation() const {
    const Memory* r = root();
    return r->alloc_ ? r->alloc_ : r->data_;
  }
  void set_allocation(const void* a) { alloc_ = a; }
  // wrapped memory whose release callback does not touch the Memory (it gets
  // nullptr): after pending readers it runs on the deferred-release thread
  // instead of blocking the thread that drops the last reference
  void set_deferred_release() { defer_wrap_ = true; }

  // the device mirror of this memory on `dev` (map_device), if any
  MemoryPtr device_mirror(int dev);

  // NNSX_MEM_CHECK=1 (debug builds of a run, read once): released blocks are
  // filled with kPoison (device: on the release stream, after every reader;
  // host / pinned: after the deferred free's waits), a pooled block handed out
  // again must still hold the poison (else something wrote to it after its
  // release: the acquire throws), and map_host / map_device of a memory whose
  // destruction has begun throws.  Stale reads of a recycled block then read
  // NaNs (0x7FBADBAD as fp32) instead of plausible old data.
  static bool check_enabled();
  // lifetime self-tests only: 0 none, kMutHostFreedEarly = a host source's
  // async H2D is not recorded as a use (pageable: the fix of 7ba8684 undone;
  // pinned: the rule it extended to pageable sources),
  // kMutMirrorNotHeld = a reader of a host memory does not hold its device
  // mirror (ee80b24 undone); returns the previous mutation
  static constexpr int kMutHostFreedEarly = 1, kMutMirrorNotHeld = 2;
  static int set_test_mutation(int m);
  // lifetime self-tests: watch one device block's free (issued by the deferred-release thread)
  static void test_watch_free(const void* p);
  static bool test_watched_freed();
  static constexpr uint32_t kPoison = 0x7FBADBADu;
  // released alloc_device blocks (not pooled ones) get their own NaN pattern, so a
  // stale read tells a released device block from a released host one
  static constexpr uint32_t kPoisonDevice = 0x7FDE7ADEu;
  // Wait until every deferred host / pinned release queued so far has run (tests).
  static void drain_deferred();

 private:
  void record_use_self(hipStream_t stream, int dev);  // record_use without the device mirror
  void check_live(const char* what) const;
  // alloc_host / alloc_pinned blocks: the last release hands pending copies'
  // events to the deferred-release thread instead of waiting on them
  bool deferrable_ = false;
  std::atomic<uint32_t> state_{0};  // 0 live, 1 destroying
  void* data_;
  size_t size_;
  MemPlace place_;
  int device_;
  Release release_;
  const void* alloc_ = nullptr;  // set_allocation
  bool defer_wrap_ = false;      // set_deferred_release
  MemoryPtr parent_;  // for views
  hipEvent_t ready_ = nullptr;
  int ready_dev_ = 0;
  uint64_t ready_gen_ = 0;           // mark_ready() count
  mutable uint64_t synced_gen_ = 0;  // last ready_gen_ known complete on the host
  mutable std::mutex ev_mu_;  // ready_ / uses_ (only the root's is used)
  mutable std::mutex mu_;     // mirrors
  struct Use {
    int dev;
    hipStream_t stream;
    hipEvent_t event;  // re-recorded per use: the stream's latest read covers earlier ones
  };
  std::vector<Use> uses_;
  MemoryPtr host_mirror_;
  std::map<int, MemoryPtr> dev_mirror_;
  std::map<std::string, int64_t> tags_;
  MetaInfo meta_;
  bool has_meta_ = false;
};

// A pool of equal-size device blocks (the GstBufferPool of a device-producing
// element): acquire() hands out a free block whose previous readers are done
// (their release event has completed), else grows the pool, else waits on the
// HOST for the oldest free block -- the acquiring stream never carries a
// cross-queue wait.  (Measured: an SDMA upload queued behind a hipStreamWaitEvent
// on the compute queue's event blocked the uploading thread inside
// hipMemcpyAsync for ~7.8 ms and stalled a running kernel by ~0.9 ms; see
// profiles/r3_step_stall_trace.txt.)  The
// block returns to the pool when its last Memory reference drops, instead of
// a hipFreeAsync per buffer (a 77 MB batch free costs milliseconds of host
// time).  Acquired memories are tagged kPoolTag = pool id and kSlotTag = block
// index: a consumer may key per-address state (a hipGraph instance reading the
// block in place) on a pooled address, because a pooled block stays allocated
// for the pool's lifetime and only recurs once its previous use is released.
class DeviceBufferPool : public std::enable_shared_from_this<DeviceBufferPool> {
 public:
  static constexpr const char* kPoolTag = "nnsx.pool";
  static constexpr const char* kSlotTag = "nnsx.pool_slot";
  static std::shared_ptr<DeviceBufferPool> create(int dev, size_t size, size_t max_blocks);
  // the live pool with this id (kPoolTag), or null
  static std::shared_ptr<DeviceBufferPool> find(uint64_t id);
  ~DeviceBufferPool();
  // allocate every block now (ordered on `stream`): the set of addresses is
  // then fixed and known (block_addresses) before the first frame
  void preallocate(hipStream_t stream);
  std::vector<void*> block_addresses() const;
  // a block ordered on `stream`; past max_blocks outstanding: an unpooled alloc_device
  MemoryPtr acquire(hipStream_t stream);
  int device() const { return dev_; }
  size_t block_size() const { return size_; }
  size_t blocks() const;     // allocated so far
  uint64_t id() const { return id_; }

 private:
  DeviceBufferPool(int dev, size_t size, size_t max_blocks);
  void put_back(int slot, hipEvent_t released);
  void mark_poisoned(int slot);  // MEM_CHECK: the block's release filled it with kPoison
  struct Block {
    void* ptr = nullptr;
    hipEvent_t released = nullptr;  // recorded after the last reader of the previous use
    bool free = true;
    uint64_t seq = 0;  // put_back order (oldest free block = smallest)
  };
  int dev_;
  size_t size_, max_;
  uint64_t id_;
  mutable std::mutex mu_;
  std::vector<Block> blocks_;
  uint64_t seq_ = 0;
  std::set<int> pool_poisoned_;  // MEM_CHECK: slots poisoned at release
};

// Meta a buffer carries across elements.
struct BufferMeta {
  int64_t client_id = -1;  // GstMetaQuery client id (tensor_query routing)
  std::map<std::string, std::string> extra;
};

enum BufferFlags : uint32_t {
  BUF_FLAG_NONE = 0,
  BUF_FLAG_DISCONT = 1u << 0,
  BUF_FLAG_GAP = 1u << 1,
  BUF_FLAG_DELTA = 1u << 2,
};

struct Buffer {
  std::vector<MemoryPtr> mems;
  int64_t pts = -1;
  int64_t dts = -1;
  int64_t duration = -1;
  int64_t offset = -1;
  int64_t offset_end = -1;
  uint32_t flags = 0;
  BufferMeta meta;
  int64_t origin_ns = -1;  // tracer: time of the first push at its source (interlatency)

  size_t n_memory() const { return mems.size(); }
  MemoryPtr& mem(size_t i) { return mems.at(i); }
  size_t total_size() const {
    size_t s = 0;
    for (auto& m : mems) s += m->size();
    return s;
  }
  void copy_metadata_from(const Buffer& o) {
    pts = o.pts;
    dts = o.dts;
    duration = o.duration;
    offset = o.offset;
    offset_end = o.offset_end;
    flags = o.flags;
    meta = o.meta;
    origin_ns = o.origin_ns;
  }
};
using BufferPtr = std::shared_ptr<Buffer>;

inline BufferPtr make_buffer() { return std::make_shared<Buffer>(); }

// ---- tensor <-> buffer helpers ----
// Split one contiguous memory into per-tensor chunks of a static config, or walk
// flexible headers.  Views share storage (zero-copy).
bool buffer_from_config(const BufferPtr& in, const TensorsConfig& config, BufferPtr* out);
// Make a flexible-format memory: host memories get the 128B header prepended
// (byte-compatible with the reference); device memories get it attached.
MemoryPtr make_flexible(const MemoryPtr& mem, const MetaInfo& meta);
// Read the meta of a flexible memory and return the payload (zero-copy view).
bool parse_flexible(const MemoryPtr& mem, MetaInfo* meta, MemoryPtr* payload);
// Serialize a memory to host bytes with an in-band header when it carries meta.
std::vector<uint8_t> serialize_with_header(const MemoryPtr& mem);
// nnsx buffers are not limited to 16 memories (no GstBuffer memory cap), so
// >16 tensors are held as plain extra memories.  For wire/file formats that
// must stay within 16 chunks the reference's "extra tensors" packing
// (nnstreamer_plugin_api_impl.c:1477-1768) is available explicitly:
// memories [15..] are concatenated behind an ExtraInfo header.
std::vector<MemoryPtr> pack_extra(const std::vector<MemoryPtr>& mems, const TensorsInfo& info);
std::vector<MemoryPtr> unpack_extra(const std::vector<MemoryPtr>& mems, TensorsInfo* info);

// "Extra tensors" header in the 16th memory (magic 0xf00dc0de).
constexpr uint32_t kExtraMagic = 0xf00dc0deu;

}  // namespace nnsx
