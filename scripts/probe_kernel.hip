#include <hip/hip_runtime.h>
__global__ void add_one(float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += 1.0f;
}
extern "C" int probe_add_one(float* x, int n, hipStream_t s) {
  hipLaunchKernelGGL(add_one, dim3((n + 255) / 256), dim3(256), 0, s, x, n);
  return (int)hipGetLastError();
}
