// MFMA throughput probe for gfx950: cycles per instruction of the fp32 and
// bf16 MFMA shapes the fp32 engine can use (v_mfma_f32_16x16x4_f32,
// v_mfma_f32_16x16x16_bf16, v_mfma_f32_16x16x32_bf16,
// v_mfma_f32_32x32x16_bf16), one wave per SIMD on every CU, 4 independent
// accumulators per wave; plus FLOP/s.  Decides the x3 operand layout: a
// 16x16x16 bf16 MFMA at the 16x16x32 rate takes the fp32 kernels' k4 lane
// layout unchanged.
//
//   hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate && ./mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int NIT = 4096;

__global__ void k_f32(float* out, float a, float b) {
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < NIT; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
  }
  f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ void k_bf16_16(float* out, float a) {
  bf16x4 x;
  for (int j = 0; j < 4; ++j) x[j] = (__bf16)(a + j);
  s16x4 xs = __builtin_bit_cast(s16x4, x);
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < NIT; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(xs, xs, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(xs, xs, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(xs, xs, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(xs, xs, c3, 0, 0, 0);
  }
  f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ void k_bf16_32(float* out, float a) {
  bf16x8 x;
  for (int j = 0; j < 8; ++j) x[j] = (__bf16)(a + j);
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < NIT; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c3, 0, 0, 0);
  }
  f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ void k_bf16_3216(float* out, float a) {
  bf16x8 x;
  for (int j = 0; j < 8; ++j) x[j] = (__bf16)(a + j);
  f32x16 c0 = {}, c1 = {};
  for (int i = 0; i < NIT; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c1, 0, 0, 0);
  }
  f32x16 s = c0 + c1;
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[5] + s[15];
}

int main() {
  int cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  float* out;
  hipMalloc(&out, static_cast<size_t>(cus) * 256 * 4 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K {
    const char* name;
    double flop_per_mfma;
    int mfma_per_it;
    int which;
  } ks[] = {{"v_mfma_f32_16x16x4_f32", 2.0 * 16 * 16 * 4, 4, 0},
            {"v_mfma_f32_16x16x16_bf16", 2.0 * 16 * 16 * 16, 4, 1},
            {"v_mfma_f32_16x16x32_bf16", 2.0 * 16 * 16 * 32, 4, 2},
            {"v_mfma_f32_32x32x16_bf16", 2.0 * 32 * 32 * 16, 2, 3}};
  printf("# %d CUs, peak clock %d MHz; one wave per SIMD (256 threads per CU), %d iterations\n", cus, clk / 1000, NIT);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& k : ks) {
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) {
        if (k.which == 0) hipLaunchKernelGGL(k_f32, dim3(cus), dim3(256), 0, 0, out, 1.f, 2.f);
        if (k.which == 1) hipLaunchKernelGGL(k_bf16_16, dim3(cus), dim3(256), 0, 0, out, 1.f);
        if (k.which == 2) hipLaunchKernelGGL(k_bf16_32, dim3(cus), dim3(256), 0, 0, out, 1.f);
        if (k.which == 3) hipLaunchKernelGGL(k_bf16_3216, dim3(cus), dim3(256), 0, 0, out, 1.f);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double n_mfma = 5.0 * cus * 4 * NIT * k.mfma_per_it;  // per SIMD-wave
      const double s = ms / 1e3;
      const double per_simd = 5.0 * NIT * k.mfma_per_it;
      printf("%-28s %8.3f ms  %7.1f TF/s  %6.1f ns per MFMA per SIMD (%5.1f cycles at peak clock)\n", k.name, ms,
             n_mfma * k.flop_per_mfma / s / 1e12, s / per_simd * 1e9, s / per_simd * clk * 1e3);
    }
  return 0;
}
