// Debug kernels: a bounded device-side busy wait that holds a stream for a set
// time, so tests can make an asynchronous-copy / replay race window
// deterministic (runtime/selftest.cc).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels/kernels.h"

namespace nnsx {
namespace kernels {

namespace {

// one wave spins on the 100 MHz constant clock (wall_clock64) for `ticks`;
// every wave reaches the exit (bounded by the tick count, at most 0.2 s)
__global__ void __launch_bounds__(64) spin_kernel(unsigned long long ticks, unsigned* out) {
  const unsigned long long t0 = wall_clock64();
  unsigned n = 0;
  while (wall_clock64() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    ++n;
  }
  if (threadIdx.x == 0 && out) out[0] = n;
}

}  // namespace

void spin_us(hipStream_t s, int us) {
  const unsigned long long ticks = static_cast<unsigned long long>(std::min(std::max(us, 0), 200000)) * 100ull;
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, ticks, static_cast<unsigned*>(nullptr));
}

}  // namespace kernels
}  // namespace nnsx
