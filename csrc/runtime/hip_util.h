// HIP runtime helpers: device discovery, error checks, per-device event
// pools, stream-ordered device allocation (hipMallocAsync on a per-device
// hipMemPool with a high release threshold -> allocation-free steady state)
// and a pinned-host block pool for H2D/D2H staging.
//
// Replaces the reference's aligned sysmem allocator
// (gst/nnstreamer/tensor_allocator.c:45-128) and its hw_accel probe
// (gst/nnstreamer/hw_accel.c:43-64).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace nnsx {
namespace hip {

int device_count();              // 0 when no GPU / no driver (never throws)
bool available();                // device_count() > 0
// NUMA node of the GPU's PCIe root (-1: unknown)
int numa_node(int dev);
// pin this process's future threads to the GPU's NUMA node CPUs and prefer
// that node for new memory (pinned upload rings); returns what was done
std::string bind_numa(int dev);
std::string device_arch(int dev);  // e.g. "gfx950"
void check(hipError_t e, const char* what);  // throws nnsx::Error
#define NNSX_HIP_CHECK(x) ::nnsx::hip::check((x), #x)

// RAII device selection
class DeviceGuard {
 public:
  explicit DeviceGuard(int dev);
  ~DeviceGuard();

 private:
  int prev_ = -1;
  bool changed_ = false;
};

// Events are recycled: creating one costs a driver call.
hipEvent_t event_get(int dev);
void event_put(int dev, hipEvent_t ev);

// A non-blocking stream owned by the caller (released with stream_destroy).
// priority kConfiguredPriority: the ini's [hip] stream_priority (default 0)
constexpr int kConfiguredPriority = -1000000;
hipStream_t stream_create(int dev, int priority = kConfiguredPriority);
void stream_destroy(int dev, hipStream_t s);
// Process-lifetime stream on which pooled device blocks are returned.
hipStream_t release_stream(int dev);
// Per-thread helper stream for ad-hoc copies (map_host / map_device).
hipStream_t thread_copy_stream(int dev);

// Stream-ordered device memory (hipMallocAsync from the device's default pool,
// release threshold raised so freed blocks are cached, not returned to the OS).
void* device_alloc(int dev, size_t bytes, hipStream_t s);
void device_free(int dev, void* p, hipStream_t s);

// Pinned host memory pool (size-bucketed free lists).
void* pinned_alloc(size_t bytes);
void pinned_free(void* p, size_t bytes);

// Host allocation aligned for 16B vector copies (plain memory when no GPU).
void* host_alloc(size_t bytes);
void host_free(void* p);

}  // namespace hip
}  // namespace nnsx
