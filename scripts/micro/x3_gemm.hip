// Split-bf16 ("x3") fp32 GEMM probe for gfx950.
//
// Each fp32 operand is split exactly into three bf16 parts, x = hi + mid + lo
// (round-to-nearest-even at each step: |mid| <= 2^-9 |x|, |lo| <= 2^-17 |x|),
// and the six significant cross products hi.hi, hi.mid, mid.hi, mid.mid,
// hi.lo, lo.hi are accumulated in fp32 on v_mfma_f32_16x16x32_bf16 (16x the
// fp32 MFMA rate per instruction).  This probe answers two questions before
// the engine uses it:
//   1. accuracy: error against an fp64 host reference, side by side with the
//      native fp32 MFMA (v_mfma_f32_16x16x4_f32) on the same data, for
//      MobileNet-like operand distributions (ReLU6 activations, N(0, 1/K)
//      weights) and K = 16 .. 1280;
//   2. the bf16 MFMA's own accumulation: does it keep small products that
//      fall below the accumulator's ulp (a truncating adder would drop them)?
//
//   hipcc --offload-arch=gfx950 -O3 x3_gemm.hip -o x3_gemm && ./x3_gemm
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Split8 {
  bf16x8 h, m, l;
};

// 8 consecutive floats -> three bf16x8 parts (RNE each step; the residuals
// x - hi and r - mid are exact in fp32)
__device__ __forceinline__ Split8 split8(const float* v) {
  Split8 s;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f32x2 x = {v[j], v[j + 1]};
    const bf16x2 h = __builtin_convertvector(x, bf16x2);
    const f32x2 r = x - __builtin_convertvector(h, f32x2);
    const bf16x2 m = __builtin_convertvector(r, bf16x2);
    const f32x2 r2 = r - __builtin_convertvector(m, f32x2);
    const bf16x2 l = __builtin_convertvector(r2, bf16x2);
    s.h[j] = h[0];
    s.h[j + 1] = h[1];
    s.m[j] = m[0];
    s.m[j + 1] = m[1];
    s.l[j] = l[0];
    s.l[j + 1] = l[1];
  }
  return s;
}

// D[m][n] = sum_k X[m][k] W[n][k]; one wave per 16x16 tile, operands straight
// from global memory (accuracy only).  mode 0: native fp32 MFMA; 1: x3 six
// products, small terms first into one accumulator; 2: x3 with the small terms
// in a second accumulator added at the end; 3: bf16 hi.hi only (reference
// for "plain bf16")
__global__ void gemm_probe(const float* X, const float* W, float* D, int M, int N, int K, int mode) {
  const int lane = threadIdx.x & 63;
  const int m0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
  if (mode == 0) {
    const int li = lane & 15, g = lane >> 4;
    for (int k = 0; k < K; k += 4) {
      // A = W rows (n), B = X rows (m): C[row n][col m]
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(W[(n0 + li) * K + k + g], X[(m0 + li) * K + k + g], acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) D[(m0 + li) * N + n0 + 4 * g + r] = acc[r];
    return;
  }
  const int li = lane & 15, g = lane >> 4;
  for (int k = 0; k < K; k += 32) {
    float wa[8], xb[8];
    for (int j = 0; j < 8; ++j) {
      const int kk = k + 8 * g + j;
      wa[j] = kk < K ? W[(n0 + li) * K + kk] : 0.f;
      xb[j] = kk < K ? X[(m0 + li) * K + kk] : 0.f;
    }
    const Split8 a = split8(wa), b = split8(xb);
    if (mode == 3) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, acc, 0, 0, 0);
    } else if (mode == 1) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, acc, 0, 0, 0);
    } else if (mode == 4 || mode == 5) {
      // per-32k partial from zero (corrections first, then hi.hi), added to the
      // running sum with an RNE VALU add (mode 4); mode 5: corrections from zero,
      // hi.hi into the running sum, then the correction added by the VALU
      f32x4 t = {0, 0, 0, 0};
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, t, 0, 0, 0);
      if (mode == 4) {
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, t, 0, 0, 0);
        acc += t;
      } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, acc, 0, 0, 0);
        acc += t;
      }
    } else {
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, acc2, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, acc, 0, 0, 0);
    }
  }
  acc += acc2;
  // C/D: col = lane & 15 (= m), row = 4 g + r (= n)
  for (int r = 0; r < 4; ++r) D[(m0 + li) * N + n0 + 4 * g + r] = acc[r];
}

// accumulation probe: one 16x16x32 MFMA with A row 0 = [1, e, e, ..., e]
// (31 copies of e), B column 0 = all ones.  The exact sum is 1 + 31 e.  A
// fully-precise adder (round once) returns fl(1 + 31e); an adder that aligns
// every product to the largest one's exponent and truncates at fp32 width
// drops each e < 2^-24.
__global__ void accum_probe(float e, float c_in, float* out) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g + j;
    a[j] = (__bf16)(li == 0 ? (k == 0 ? 1.f : e) : 0.f);
    b[j] = (__bf16)(li == 0 ? 1.f : 0.f);
  }
  f32x4 c = {c_in, 0, 0, 0};
  if (g != 0) c[0] = 0.f;
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  if (lane == 0) out[0] = c[0];
}

static double run(int M, int N, int K, int dist, int mode, std::vector<double>* err_out) {
  std::mt19937 rng(1234 + K);
  std::uniform_real_distribution<float> u01(0.f, 1.f);
  std::normal_distribution<float> nrm(0.f, 1.f);
  std::vector<float> X(static_cast<size_t>(M) * K), W(static_cast<size_t>(N) * K);
  for (auto& v : X) {
    if (dist == 0) {
      const float t = nrm(rng) * 2.f;  // ReLU6 of N(0, 2): about half zeros, some clamped at 6
      v = t < 0 ? 0.f : (t > 6 ? 6.f : t);
    } else {
      v = nrm(rng);
    }
  }
  for (auto& v : W) v = nrm(rng) / std::sqrt(static_cast<float>(K));
  float *dX, *dW, *dD;
  CK(hipMalloc(&dX, X.size() * 4));
  CK(hipMalloc(&dW, W.size() * 4));
  CK(hipMalloc(&dD, static_cast<size_t>(M) * N * 4));
  CK(hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  gemm_probe<<<dim3(M / 16, N / 16), 64>>>(dX, dW, dD, M, N, K, mode);
  CK(hipDeviceSynchronize());
  std::vector<float> D(static_cast<size_t>(M) * N);
  CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
  double maxrel = 0, sumrel = 0, maxnorm = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double s = 0, sa = 0;
      for (int k = 0; k < K; ++k) {
        const double p = static_cast<double>(X[static_cast<size_t>(m) * K + k]) * W[static_cast<size_t>(n) * K + k];
        s += p;
        sa += std::fabs(p);
      }
      const double e = std::fabs(D[static_cast<size_t>(m) * N + n] - s);
      const double rel = e / std::max(std::fabs(s), 1e-30);
      if (std::fabs(s) > 1e-3 * sa) {  // skip near-cancelled outputs for the plain relative error
        maxrel = std::max(maxrel, rel);
      }
      sumrel += e / std::max(sa, 1e-30);
      maxnorm = std::max(maxnorm, e / std::max(sa, 1e-30));
    }
  if (err_out) {
    err_out->push_back(maxrel);
    err_out->push_back(sumrel / (static_cast<double>(M) * N));
    err_out->push_back(maxnorm);
  }
  CK(hipFree(dX));
  CK(hipFree(dW));
  CK(hipFree(dD));
  return maxrel;
}

int main() {
  float* dout;
  CK(hipMalloc(&dout, 4));
  printf("# bf16 MFMA accumulation probe: 1 + 31 e in one v_mfma_f32_16x16x32_bf16 (C = 0 or C = c)\n");
  const float es[] = {0x1p-20f, 0x1p-23f, 0x1p-24f, 0x1p-25f, 0x1p-26f, 0x1p-30f};
  for (float c : {0.f, 1.f}) {
    for (float e : es) {
      accum_probe<<<1, 64>>>(e, c, dout);
      float r;
      CK(hipMemcpy(&r, dout, 4, hipMemcpyDeviceToHost));
      const double exact = 1.0 + 31.0 * e + c;
      printf("  C=%g e=2^%d: got %.9g (%a), exact %.12g, fl(exact) %a\n", c, static_cast<int>(std::log2(e)), r, r, exact,
             static_cast<float>(exact));
    }
  }
  const char* names[] = {"fp32 MFMA 16x16x4", "x3 one acc", "x3 two acc", "bf16 hi only", "x3 blocked 32k", "x3 corr-add"};
  printf("\n# error vs fp64: max rel (|ref| > 1e-3 sum|ab|), mean and max of |err| / sum|ab|\n");
  printf("%-18s %5s %5s %5s %5s  %12s %12s %12s\n", "method", "dist", "M", "N", "K", "max_rel", "mean_norm", "max_norm");
  for (int dist = 0; dist < 2; ++dist)
    for (int K : {16, 32, 96, 144, 320, 576, 960, 1280}) {
      for (int mode = 0; mode < 6; ++mode) {
        if (mode == 3) continue;
        std::vector<double> e;
        run(256, 64, K, dist, mode, &e);
        printf("%-18s %5s %5d %5d %5d  %12.3e %12.3e %12.3e\n", names[mode], dist ? "N01" : "relu6", 256, 64, K, e[0],
               e[1], e[2]);
      }
    }
  return 0;
}
