// H2D batch upload micro-benchmark: 128 pinned 270 KB frames -> one device
// buffer via (a) a zero-copy gather kernel with varying grid sizes,
// (b) per-frame hipMemcpyAsync (SDMA), (c) hipMemcpyBatchAsync.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Seg { const char* src; unsigned long off, bytes; };

__global__ void __launch_bounds__(256) gather(const Seg* segs, int nseg, char* dst, int wgs_per_seg) {
  const int sgi = blockIdx.x / wgs_per_seg, part = blockIdx.x % wgs_per_seg;
  if (sgi >= nseg) return;
  const Seg sg = segs[sgi];
  const uint4* s4 = reinterpret_cast<const uint4*>(sg.src);
  uint4* d4 = reinterpret_cast<uint4*>(dst + sg.off);
  const unsigned long n = sg.bytes / 16, stride = (unsigned long)wgs_per_seg * 256;
  for (unsigned long i = (unsigned long)part * 256 + threadIdx.x; i < n; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) v[u] = s4[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) d4[i + u * stride] = v[u];
  }
}

int main() {
  const int N = 128;
  const size_t B = 300 * 300 * 3;
  std::vector<char*> h(N);
  for (int i = 0; i < N; ++i) { CK(hipHostMalloc(&h[i], 512 << 10, 0)); std::memset(h[i], i, B); }
  char* d; CK(hipMalloc(&d, N * B));
  std::vector<Seg> segs(N);
  for (int i = 0; i < N; ++i) segs[i] = {h[i], i * B, B};
  Seg* dsegs; CK(hipMalloc(&dsegs, N * sizeof(Seg)));
  CK(hipMemcpy(dsegs, segs.data(), N * sizeof(Seg), hipMemcpyHostToDevice));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto fn) {
    for (int w = 0; w < 3; ++w) fn();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    hipEventRecord(a, s);
    for (int r = 0; r < 10; ++r) fn();
    hipEventRecord(b, s);
    auto t1 = std::chrono::steady_clock::now();
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double cpu = std::chrono::duration<double, std::micro>(t1 - t0).count() / 10;
    printf("%-28s %8.1f us/batch  %6.1f GB/s  cpu %7.1f us/batch\n", name, ms * 100, N * B / (ms / 10 * 1e-3) / 1e9, cpu);
  };
  for (int w : {1, 2, 4, 8, 16, 34}) {
    char nm[64]; snprintf(nm, sizeof nm, "gather kernel %d WG/frame", w);
    run(nm, [&] { hipLaunchKernelGGL(gather, dim3(N * w), dim3(256), 0, s, dsegs, N, d, w); });
  }
  run("hipMemcpyAsync x128", [&] { for (int i = 0; i < N; ++i) hipMemcpyAsync(d + i * B, h[i], B, hipMemcpyHostToDevice, s); });
  std::vector<void*> dsts(N), srcs(N); std::vector<size_t> sz(N, B);
  for (int i = 0; i < N; ++i) { dsts[i] = d + i * B; srcs[i] = h[i]; }
  hipMemcpyAttributes attr{}; attr.srcAccessOrder = hipMemcpySrcAccessOrderStream;
  size_t attrIdx = 0, fail = 0;
  run("hipMemcpyBatchAsync", [&] {
    hipError_t e = hipMemcpyBatchAsync(dsts.data(), srcs.data(), sz.data(), N, &attr, &attrIdx, 1, &fail, s);
    if (e != hipSuccess) { static bool once = false; if (!once) printf("batch err %s\n", hipGetErrorString(e)); once = true; }
  });
  return 0;
}
