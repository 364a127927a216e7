// fp32 VALU issue-rate probe for gfx950: scalar v_fma_f32 vs packed
// v_pk_fma_f32, at 1/2/4/8 waves per SIMD.  Settles whether the depthwise
// phases of the fp32 engine need packed math to reach the 157 TF/s vector
// peak (256 FLOP/clk/CU).  Each lane runs NCH independent accumulator chains
// of NIT fused multiply-adds; inline asm keeps the compiler from packing or
// unpacking them.
//
//   hipcc --offload-arch=gfx950 -O3 fma_rate.hip -o fma_rate && ./fma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int NCH = 16;    // independent chains per lane
constexpr int NIT = 4096;  // iterations

__global__ void scalar_fma(float* out, float a, float b) {
  float acc[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) acc[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < NIT; ++it) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void packed_fma(float* out, float a, float b) {
  f32x2 acc[NCH / 2];
  const f32x2 av = {a, a}, bv = {b, b};
#pragma unroll
  for (int i = 0; i < NCH / 2; ++i) acc[i] = f32x2{threadIdx.x * 1e-3f + i, 1.f + i};
  for (int it = 0; it < NIT; ++it) {
#pragma unroll
    for (int i = 0; i < NCH / 2; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(av), "v"(bv));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH / 2; ++i) s += acc[i][0] + acc[i][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, sizeof(float) * cus * 2048);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("CUs %d, %d fma per lane per launch (%d chains)\n", cus, NCH * NIT, NCH);
  for (int wps : {1, 2, 4, 8}) {       // waves per SIMD
    const int threads = wps > 4 ? 1024 : 256 * wps;  // 4 SIMDs x wps waves per CU
    const int blocks = cus * (256 * wps / threads);
    for (int packed = 0; packed < 2; ++packed) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        if (packed)
          hipLaunchKernelGGL(packed_fma, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 1e-4f);
        else
          hipLaunchKernelGGL(scalar_fma, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 1e-4f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double flop = 2.0 * NCH * NIT * double(threads) * blocks;
      printf("waves/SIMD %d  %-14s %8.3f ms  %7.1f TF/s  (%.1f FLOP/clk/CU at 2.4 GHz)\n", wps,
             packed ? "v_pk_fma_f32" : "v_fma_f32", best, flop / best * 1e-9, flop / (best * 1e-3) / 2.4e9 / cus);
    }
  }
  hipFree(out);
  return 0;
}
