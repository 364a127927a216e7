// Deterministic regression tests of the runtime's device-memory lifetime rules
// (exposed to Python as nnstreamer_amd._C.memory_selftest, run by
// tests/test_gpu_memcheck.py).  Each case holds a stream busy with a bounded
// spin kernel (kernels::spin_us) so that an asynchronous copy or read is still
// queued when the Memory that owns its source is released, then re-allocates
// the same storage with other bytes and checks what the delayed copy saw.  A
// lifetime rule that frees too early fails every time, not by chance.
//
// Cases (the fixes they pin):
//   pageable_h2d       a pageable host frame released while its H2D copy is
//                      queued (7ba8684: freed at once, malloc handed the
//                      address to the next frame, the copy read that frame)
//   pinned_h2d         the same for a pinned block (the pinned pool recycles it)
//   mirror_other_stream a host memory's device mirror read on a second stream
//                      (a filter replay lane) that recorded its use on the
//                      host memory (ee80b24: the mirror went back to the pool
//                      ordered only on the mapping stream)
//   device_reader      a device block read on another stream while released
//                      (the release waits for every recorded reader)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kernels/kernels.h"
#include "runtime/hip_util.h"
#include "runtime/memory.h"

namespace nnsx {

namespace {

constexpr size_t kBytes = 8u << 20;  // 8 MB: a few frames; one copy takes ~0.2 ms
constexpr int kSpinUs = 20000;       // 20 ms: every release below happens inside this window

std::string check_bytes(const std::vector<uint8_t>& got, uint8_t want, const char* what) {
  size_t bad = 0;
  for (uint8_t v : got) bad += v != want;
  if (!bad) return "";
  return std::string(what) + ": " + std::to_string(bad) + " of " + std::to_string(got.size()) +
         " bytes differ from the pattern the released source held (first byte " + std::to_string(got[0]) + ")";
}

std::vector<uint8_t> d2h(const void* p, size_t n, hipStream_t s) {
  std::vector<uint8_t> h(n);
  hip::check(hipMemcpyAsync(h.data(), p, n, hipMemcpyDeviceToHost, s), "selftest D2H");
  hip::check(hipStreamSynchronize(s), "selftest sync");
  return h;
}

// host frame (pageable or pinned) -> H2D on s behind a spin; the frame is
// released at once, its storage reused for other frames; the mirror must hold
// the first frame's bytes.  Several sizes: malloc hands a freed small block
// (below its mmap threshold) back at once, a large one through mmap; the HIP
// runtime stages pageable copies differently by size.  NNSX_SELFTEST_VERBOSE=1
// prints how long each map_device call blocked the host (a copy the runtime
// completes inside the call cannot read a recycled frame).
std::string host_h2d_one(int dev, bool pinned, size_t bytes) {
  hip::DeviceGuard g(dev);
  hipStream_t s = nullptr;
  hip::check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "selftest stream");
  MemoryPtr h = pinned ? Memory::alloc_pinned(bytes) : Memory::alloc_host(bytes);
  std::memset(h->data(), 0x11, bytes);
  kernels::spin_us(s, kSpinUs);
  const auto t0 = std::chrono::steady_clock::now();
  (void)h->map_device(dev, s);  // queued behind the spin
  const double blocked_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  MemoryPtr mirror = h->device_mirror(dev);
  h.reset();  // the last reference: the copy has not run yet
  // the next frames take the freed storage (malloc / the pinned pool hand it out again)
  std::vector<MemoryPtr> next;
  for (int i = 0; i < 4; ++i) {
    next.push_back(pinned ? Memory::alloc_pinned(bytes) : Memory::alloc_host(bytes));
    std::memset(next.back()->data(), 0x22, bytes);
  }
  const std::string what = std::string(pinned ? "pinned_h2d" : "pageable_h2d") + "[" + std::to_string(bytes) + " B]";
  std::string r = check_bytes(d2h(mirror->data(), bytes, s), 0x11, what.c_str());
  if (const char* v = std::getenv("NNSX_SELFTEST_VERBOSE"); v && v[0] == '1')
    std::fprintf(stderr, "%s: map_device blocked the host %.3f ms (spin %d ms): %s\n", what.c_str(), blocked_ms,
                 kSpinUs / 1000, r.empty() ? "bytes intact" : r.c_str());
  mirror.reset();
  next.clear();
  hip::check(hipStreamSynchronize(s), "selftest sync");
  (void)hipStreamDestroy(s);
  return r;
}

std::string host_h2d(int dev, bool pinned) {
  std::string r;
  for (size_t bytes : {size_t(4) << 10, size_t(64) << 10, size_t(1) << 20, kBytes}) {
    std::string e = host_h2d_one(dev, pinned, bytes);
    if (!e.empty()) r += (r.empty() ? "" : "; ") + e;
  }
  return r;
}

// the mirror of a host memory is read on a second stream (spinning first),
// which records its use on the HOST memory (what a filter's replay lane does);
// the host memory and so its mirror are released; a new device block of the
// same size, written on the release stream, must not reach the reader
std::string mirror_other_stream(int dev) {
  hip::DeviceGuard g(dev);
  // start from an idle release stream and an empty deferred queue: earlier
  // releases (other cases' 20 ms spins) queued there would delay this case's
  // free past the reader and hide the undone fix
  Memory::drain_deferred();
  hip::check(hipStreamSynchronize(hip::release_stream(dev)), "selftest sync");
  hipStream_t s1 = nullptr, s2 = nullptr;
  hip::check(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking), "selftest stream");
  hip::check(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking), "selftest stream");
  // (pageable: its release does not wait for readers on the host -- the mirror's
  // own release must order itself after them)
  MemoryPtr h = Memory::alloc_host(kBytes);
  std::memset(h->data(), 0x33, kBytes);
  const void* mp = h->map_device(dev, s1);
  hip::check(hipStreamSynchronize(s1), "selftest sync");
  MemoryPtr out = Memory::alloc_device(kBytes, dev, s2);
  kernels::spin_us(s2, kSpinUs);
  MemoryPtr mirror = h->device_mirror(dev);
  mirror->wait_ready(s2);
  hip::check(hipMemcpyAsync(out->data(), mp, kBytes, hipMemcpyDeviceToDevice, s2), "selftest D2D");
  h->record_use(s2, dev);  // the reader holds the host memory (and, through it, the mirror)
  Memory::test_watch_free(mp);
  mirror.reset();
  h.reset();  // mirror released: ordered on the release stream after its recorded readers
  hipStream_t rs = hip::release_stream(dev);
  // device frees are issued by the deferred-release thread once their waits have
  // passed (memory.cc alloc_device): give the mirror's free time to be issued --
  // within microseconds when nothing holds the mirror (the fix undone), only
  // after the reader's 20 ms spin otherwise
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  // the free issued while the reader has not run: the failure, whichever block
  // the pool hands out next (after other tests it may split a larger free block)
  const bool freed_early = Memory::test_watched_freed() && hipStreamQuery(s2) != hipSuccess;
  Memory::test_watch_free(nullptr);
  // allocate on the release stream until the pool hands out the mirror's block
  // (after earlier tests the pool holds other free blocks of this size), each
  // written at once; at most 64 blocks (512 MB).  Getting the block back while
  // the reader has not run is itself the failure.
  std::vector<MemoryPtr> again;
  bool early = false;
  for (int i = 0; i < 64; ++i) {
    again.push_back(Memory::alloc_device(kBytes, dev, rs));
    hip::check(hipMemsetAsync(again.back()->data(), 0x44, kBytes, rs), "selftest memset");
    if (again.back()->data() == mp) {
      early = hipStreamQuery(s2) != hipSuccess;
      break;
    }
  }
  std::string r = check_bytes(d2h(out->data(), kBytes, s2), 0x33, "mirror_other_stream");
  if (r.empty() && early)
    r = "mirror_other_stream: the mirror's block was handed out again while its reader on another stream had not run";
  if (r.empty() && freed_early)
    r = "mirror_other_stream: the mirror's free was issued while its reader on another stream had not run";
  again.clear();
  out.reset();
  hip::check(hipDeviceSynchronize(), "selftest sync");
  (void)hipStreamDestroy(s1);
  (void)hipStreamDestroy(s2);
  return r;
}

// a device block read on another stream (spinning first) that recorded its use
// is released; a new block written on the release stream must not reach the reader
std::string device_reader(int dev) {
  hip::DeviceGuard g(dev);
  hipStream_t s1 = nullptr, s2 = nullptr;
  hip::check(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking), "selftest stream");
  hip::check(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking), "selftest stream");
  MemoryPtr d = Memory::alloc_device(kBytes, dev, s1);
  hip::check(hipMemsetAsync(d->data(), 0x55, kBytes, s1), "selftest memset");
  d->mark_ready(s1);
  MemoryPtr out = Memory::alloc_device(kBytes, dev, s2);
  kernels::spin_us(s2, kSpinUs);
  d->wait_ready(s2);
  hip::check(hipMemcpyAsync(out->data(), d->data(), kBytes, hipMemcpyDeviceToDevice, s2), "selftest D2D");
  d->record_use(s2, dev);
  const void* dp = d->data();
  d.reset();
  hipStream_t rs = hip::release_stream(dev);
  std::this_thread::sleep_for(std::chrono::milliseconds(3));  // (as in mirror_other_stream)
  std::vector<MemoryPtr> again;
  bool early = false;
  for (int i = 0; i < 64; ++i) {
    again.push_back(Memory::alloc_device(kBytes, dev, rs));
    hip::check(hipMemsetAsync(again.back()->data(), 0x66, kBytes, rs), "selftest memset");
    if (again.back()->data() == dp) {
      early = hipStreamQuery(s2) != hipSuccess;
      break;
    }
  }
  std::string r = check_bytes(d2h(out->data(), kBytes, s2), 0x55, "device_reader");
  if (r.empty() && early) r = "device_reader: the block was handed out again while its reader had not run";
  again.clear();
  out.reset();
  hip::check(hipDeviceSynchronize(), "selftest sync");
  (void)hipStreamDestroy(s1);
  (void)hipStreamDestroy(s2);
  return r;
}

}  // namespace

// "" = pass, else what went wrong
std::string memory_selftest(const std::string& name, int dev) {
  if (!hip::available() || dev < 0 || dev >= hip::device_count()) return "memory_selftest: no such GPU";
  if (name == "pageable_h2d") return host_h2d(dev, false);
  if (name == "pinned_h2d") return host_h2d(dev, true);
  if (name == "mirror_other_stream") return mirror_other_stream(dev);
  if (name == "device_reader") return device_reader(dev);
  return "memory_selftest: unknown case " + name;
}

}  // namespace nnsx
