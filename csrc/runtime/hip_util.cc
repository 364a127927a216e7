#include "runtime/hip_util.h"

#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <thread>

#include "core/registry.h"
#include "core/util.h"

namespace nnsx {
namespace hip {

int device_count() {
  static int count = [] {
    if (const char* e = std::getenv("NNSX_DISABLE_GPU")) {
      if (to_bool(e)) return 0;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return n;
  }();
  return count;
}

bool available() { return device_count() > 0; }

int numa_node(int dev) {
  if (!available()) return -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return -1;
  std::string id(bus);
  for (auto& c : id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int node = -1;
  if (!(f >> node)) return -1;
  return node;
}

std::string bind_numa(int dev) {
  const int node = numa_node(dev);
  if (node < 0) return "no NUMA node for the device";
  // CPUs of the node, intersected with what this process may use (cgroups)
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(f, list)) return "no cpulist for node " + std::to_string(node);
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return "sched_getaffinity failed";
  int n = 0;
  std::stringstream ss(list);
  std::string range;
  while (std::getline(ss, range, ',')) {
    int a = -1, b = -1;
    if (std::sscanf(range.c_str(), "%d-%d", &a, &b) == 1) b = a;
    for (int c = a; c >= 0 && c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) {
        CPU_SET(c, &want);
        ++n;
      }
  }
  std::string what;
  if (n > 0 && sched_setaffinity(0, sizeof(want), &want) == 0) what = strfmt(n, " CPUs");
  // prefer the node for new pages (pinned staging rings, pools): MPOL_PREFERRED = 1
  unsigned long mask[16] = {0};
  if (node < 16 * 64) {
    mask[node / 64] = 1ul << (node % 64);
    if (syscall(SYS_set_mempolicy, 1, mask, 16 * 64 + 1) == 0) what += what.empty() ? "memory" : " + memory";
  }
  return what.empty() ? "binding refused" : strfmt("node ", node, ": ", what);
}

std::string device_arch(int dev) {
  if (!available()) return "";
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return "";
  return prop.gcnArchName;
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    int dev = -1;
    (void)hipGetDevice(&dev);
    throw Error(strfmt("HIP error ", hipGetErrorName(e), " (", hipGetErrorString(e), ") at ", what, " on device ", dev));
  }
}

DeviceGuard::DeviceGuard(int dev) {
  if (dev < 0 || !available()) return;
  if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
  if (prev_ != dev) {
    check(hipSetDevice(dev), "hipSetDevice");
    changed_ = true;
  }
}

DeviceGuard::~DeviceGuard() {
  if (changed_ && prev_ >= 0) (void)hipSetDevice(prev_);
}

namespace {
struct EventPool {
  std::mutex mu;
  std::unordered_map<int, std::vector<hipEvent_t>> free;
};
EventPool& event_pool() {
  static EventPool* p = new EventPool();  // leaked on purpose: outlives static dtors
  return *p;
}
}  // namespace

hipEvent_t event_get(int dev) {
  auto& pool = event_pool();
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    auto& v = pool.free[dev];
    if (!v.empty()) {
      hipEvent_t e = v.back();
      v.pop_back();
      return e;
    }
  }
  DeviceGuard g(dev);
  hipEvent_t e;
  check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreateWithFlags");
  return e;
}

void event_put(int dev, hipEvent_t ev) {
  if (!ev) return;
  auto& pool = event_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  pool.free[dev].push_back(ev);
}

// [hip] stream_priority (ini / NNSTREAMER_hip_stream_priority): priority of the
// element streams (0 = normal; lower = more urgent, clamped to the device range)
int configured_stream_priority(int dev) {
  static const int prio = static_cast<int>(to_int(Config::get().custom_value("hip", "stream_priority", "0"), 0));
  if (prio == 0) return 0;
  int lo = 0, hi = 0;  // hi = greatest priority (numerically lowest)
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return 0;
  (void)dev;
  return std::min(std::max(prio, hi), lo);
}

hipStream_t stream_create(int dev, int priority) {
  DeviceGuard g(dev);
  if (priority == kConfiguredPriority) priority = configured_stream_priority(dev);
  hipStream_t s;
  check(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority), "hipStreamCreateWithPriority");
  return s;
}

void stream_destroy(int dev, hipStream_t s) {
  if (!s) return;
  DeviceGuard g(dev);
  (void)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
}

hipStream_t release_stream(int dev) {
  static std::mutex mu;
  static std::map<int, hipStream_t>* streams = new std::map<int, hipStream_t>();
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams->find(dev);
  if (it != streams->end()) return it->second;
  hipStream_t s = stream_create(dev);
  (*streams)[dev] = s;
  return s;
}

hipStream_t thread_copy_stream(int dev) {
  thread_local std::map<int, hipStream_t> streams;  // leaked at thread exit (driver reclaims at exit)
  auto it = streams.find(dev);
  if (it != streams.end()) return it->second;
  hipStream_t s = stream_create(dev);
  streams[dev] = s;
  return s;
}

namespace {
std::once_flag g_pool_once[64];
void configure_pool(int dev) {
  std::call_once(g_pool_once[dev & 63], [dev] {
    DeviceGuard g(dev);
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
      // [hip] pool_release_threshold: bytes the stream-ordered pool keeps cached
      // after a sync ("max" = everything: 288 GB of HBM per GPU leaves no reason
      // to give memory back; lower it when several processes share a GPU)
      const std::string v = lower(Config::get().custom_value("hip", "pool_release_threshold", "max"));
      uint64_t thr = UINT64_MAX;
      if (v != "max" && !v.empty()) thr = static_cast<uint64_t>(std::strtoull(v.c_str(), nullptr, 10));
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
    (void)hipGetLastError();
  });
}
}  // namespace

void* device_alloc(int dev, size_t bytes, hipStream_t s) {
  configure_pool(dev);
  DeviceGuard g(dev);
  void* p = nullptr;
  check(hipMallocAsync(&p, bytes ? bytes : 1, s), "hipMallocAsync");
  return p;
}

void device_free(int dev, void* p, hipStream_t s) {
  if (!p) return;
  DeviceGuard g(dev);
  (void)hipFreeAsync(p, s);
}

namespace {
struct PinnedPool {
  std::mutex mu;
  std::map<size_t, std::vector<void*>> free;  // bucket size -> blocks
};
PinnedPool& pinned_pool() {
  static PinnedPool* p = new PinnedPool();
  return *p;
}
size_t bucket(size_t n) {
  size_t b = 256;
  while (b < n) b <<= 1;
  return b;
}
}  // namespace

void* pinned_alloc(size_t bytes) {
  if (!available()) return host_alloc(bytes);
  size_t b = bucket(bytes);
  auto& pool = pinned_pool();
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    auto& v = pool.free[b];
    if (!v.empty()) {
      void* p = v.back();
      v.pop_back();
      return p;
    }
  }
  void* p = nullptr;
  check(hipHostMalloc(&p, b, hipHostMallocDefault), "hipHostMalloc");
  return p;
}

void pinned_free(void* p, size_t bytes) {
  if (!p) return;
  if (!available()) {
    host_free(p);
    return;
  }
  auto& pool = pinned_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  pool.free[bucket(bytes)].push_back(p);
}

void* host_alloc(size_t bytes) {
  void* p = nullptr;
  size_t n = (bytes + 63) & ~static_cast<size_t>(63);
  if (posix_memalign(&p, 64, n ? n : 64) != 0) throw Error("host_alloc: out of memory");
  return p;
}

void host_free(void* p) { std::free(p); }

}  // namespace hip
}  // namespace nnsx
