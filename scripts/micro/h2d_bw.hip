// H2D upload bandwidth of one bench batch (512 x 224x224x3 uint8 = 77 MB) from
// pinned host memory: one hipMemcpyAsync, the same bytes split over 2/4/8
// streams (separate SDMA queues), and a zero-copy copy kernel reading the pinned
// pages over PCIe.  Each variant also runs beside a busy compute stream (an
// fp32 FMA loop on every CU) -- the situation of the pipeline, where the next
// batch uploads while the model runs.
//
//   hipcc --offload-arch=gfx950 -O3 h2d_bw.hip -o h2d_bw && ./h2d_bw
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void __launch_bounds__(256) copy_kernel(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n) v[u] = s[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n) d[i + u * stride] = v[u];
  }
}

__global__ void __launch_bounds__(256) busy_kernel(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 0.5f;
  for (int i = 0; i < iters; ++i) {
    a = fmaf(a, 0.999f, b);
    b = fmaf(b, 0.998f, a);
  }
  out[blockIdx.x * 256 + threadIdx.x] = a + b;
}

int main() {
  const size_t B = 512ull * 224 * 224 * 3;
  char* h;
  CK(hipHostMalloc(&h, B, 0));
  std::memset(h, 7, B);
  char* d;
  CK(hipMalloc(&d, B));
  float* junk;
  CK(hipMalloc(&junk, 4096 * 256 * sizeof(float)));
  hipStream_t st[8], busy;
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&busy, hipStreamNonBlocking));
  hipEvent_t a, b, join[8];
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 8; ++i) CK(hipEventCreate(&join[i]));

  auto run = [&](const char* name, int nstreams, bool kernel, int wgs, bool loaded) {
    for (int rep = -2; rep < 6; ++rep) {
      if (rep == 0) {
        if (loaded) hipLaunchKernelGGL(busy_kernel, dim3(4096), dim3(256), 0, busy, junk, 400000);
        hipStreamSynchronize(st[0]);
      }
      if (rep == 0) hipEventRecord(a, st[0]);
      const size_t chunk = (B / nstreams + 4095) / 4096 * 4096;
      for (int i = 0; i < nstreams; ++i) {
        if (i > 0 && rep == 0) hipStreamWaitEvent(st[i], a, 0);
        const size_t off = i * chunk, n = off < B ? std::min(chunk, B - off) : 0;
        if (!n) continue;
        if (kernel)
          hipLaunchKernelGGL(copy_kernel, dim3(wgs / nstreams), dim3(256), 0, st[i],
                             reinterpret_cast<const uint4*>(h + off), reinterpret_cast<uint4*>(d + off), n / 16);
        else
          hipMemcpyAsync(d + off, h + off, n, hipMemcpyHostToDevice, st[i]);
      }
      for (int i = 1; i < nstreams; ++i) {
        hipEventRecord(join[i], st[i]);
        hipStreamWaitEvent(st[0], join[i], 0);
      }
    }
    hipEventRecord(b, st[0]);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipDeviceSynchronize();
    printf("%-34s %s %8.3f ms/batch  %6.1f GB/s\n", name, loaded ? "[beside compute]" : "[idle GPU]      ", ms / 6,
           6 * B / (ms * 1e-3) / 1e9);
  };
  for (int loaded = 0; loaded < 2; ++loaded) {
    run("hipMemcpyAsync x1", 1, false, 0, loaded);
    run("hipMemcpyAsync x2 streams", 2, false, 0, loaded);
    run("hipMemcpyAsync x4 streams", 4, false, 0, loaded);
    run("hipMemcpyAsync x8 streams", 8, false, 0, loaded);
    run("copy kernel 64 WG", 1, true, 64, loaded);
    run("copy kernel 256 WG", 1, true, 256, loaded);
    run("copy kernel 1024 WG", 1, true, 1024, loaded);
    run("copy kernel 2x128 WG (2 streams)", 2, true, 256, loaded);
  }
  return 0;
}
