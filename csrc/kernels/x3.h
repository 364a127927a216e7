// Split-bf16 ("x3") fp32 products for gfx950 MFMA kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace nnsx {
namespace kernels {

// ---- split-bf16 ("x3") fp32 products ----------------------------------------
// An fp32 value splits into three bf16 parts, x = hi + mid + lo, rounding to
// nearest at each step (v_cvt_pk_bf16_f32; the residuals x - hi and
// (x - hi) - mid are exact in fp32, |mid| <= 2^-9 |x|, |lo| <= 2^-17 |x|).  A
// 32-deep dot product is then the six significant cross products hi.hi,
// hi.mid, mid.hi, mid.mid, hi.lo, lo.hi (the dropped ones are <= 2^-25 of
// |a.b|), each one v_mfma_f32_16x16x32_bf16: 6 x 16 cycles per 16 x 16 x 32
// against 8 x 32 cycles on v_mfma_f32_16x16x4_f32 -- 2.67x the fp32 MFMA
// rate.  The six products of one 32-k step are summed from zero (small terms
// first) and that partial is added to the running fp32 sum by a
// round-to-nearest VALU add: the bf16 MFMA's adder truncates (probe:
// scripts/micro/x3_gemm.hip), so the running sum never goes through it.
// Measured against an fp64 oracle on MobileNet-shaped operands (K = 16 ..
// 1280, ReLU6 / normal activations): mean |err| / sum|a.b| 4-8.5e-9 against
// 2.0e-8 for the native fp32 MFMA, max 4-8e-8 against 2-3e-7
// (profiles/r5_x3_accuracy_probe.txt).  Operand layout of a 32-k step: lane
// (li, g) holds k = 8g + j in element j of each part (rows li of A and B) --
// in mbv2_f32.hip's k4-major fp32 LDS images, k-quads 2g and 2g + 1.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
struct X3Frag {
  bf16x8_t h, m, l;
};

__device__ __forceinline__ void split2(f32x2_t x, bf16x2_t& h, bf16x2_t& m, bf16x2_t& l) {
  h = __builtin_convertvector(x, bf16x2_t);
  const f32x2_t r = x - __builtin_convertvector(h, f32x2_t);
  m = __builtin_convertvector(r, bf16x2_t);
  l = __builtin_convertvector(r - __builtin_convertvector(m, f32x2_t), bf16x2_t);
}

// 8 consecutive k (lo = k 0..3, hi = k 4..7) -> the three bf16 parts
__device__ __forceinline__ X3Frag split_x3(f32x4_t lo, f32x4_t hi) {
  bf16x2_t h0, m0, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
  split2(f32x2_t{lo[0], lo[1]}, h0, m0, l0);
  split2(f32x2_t{lo[2], lo[3]}, h1, m1, l1);
  split2(f32x2_t{hi[0], hi[1]}, h2, m2, l2);
  split2(f32x2_t{hi[2], hi[3]}, h3, m3, l3);
  X3Frag f;
  f.h = __builtin_shufflevector(__builtin_shufflevector(h0, h1, 0, 1, 2, 3), __builtin_shufflevector(h2, h3, 0, 1, 2, 3),
                                0, 1, 2, 3, 4, 5, 6, 7);
  f.m = __builtin_shufflevector(__builtin_shufflevector(m0, m1, 0, 1, 2, 3), __builtin_shufflevector(m2, m3, 0, 1, 2, 3),
                                0, 1, 2, 3, 4, 5, 6, 7);
  f.l = __builtin_shufflevector(__builtin_shufflevector(l0, l1, 0, 1, 2, 3), __builtin_shufflevector(l2, l3, 0, 1, 2, 3),
                                0, 1, 2, 3, 4, 5, 6, 7);
  return f;
}

__device__ __forceinline__ f32x4_t mfma_bf16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// the 32-k partial a . b of the six products, summed from zero (small first)
__device__ __forceinline__ f32x4_t mfma_x3(const X3Frag& a, const X3Frag& b) {
  f32x4_t t = mfma_bf16(a.l, b.h, f32x4_t{0.f, 0.f, 0.f, 0.f});
  t = mfma_bf16(a.h, b.l, t);
  t = mfma_bf16(a.m, b.m, t);
  t = mfma_bf16(a.m, b.h, t);
  t = mfma_bf16(a.h, b.m, t);
  return mfma_bf16(a.h, b.h, t);
}

// the same with the two mid x low products too (eight MFMAs): every product
// term above 2^-32 relative kept
__device__ __forceinline__ f32x4_t mfma_x3e(const X3Frag& a, const X3Frag& b) {
  f32x4_t t = mfma_bf16(a.l, b.m, f32x4_t{0.f, 0.f, 0.f, 0.f});
  t = mfma_bf16(a.m, b.l, t);
  t = mfma_bf16(a.l, b.h, t);
  t = mfma_bf16(a.h, b.l, t);
  t = mfma_bf16(a.m, b.m, t);
  t = mfma_bf16(a.m, b.h, t);
  t = mfma_bf16(a.h, b.m, t);
  return mfma_bf16(a.h, b.h, t);
}

// acc += t with the rounding error of the add carried in c (Knuth's TwoSum:
// exact for any magnitudes); acc + c at the end is the sum of the partials to
// within one final rounding, whatever the number of k-steps
__device__ __forceinline__ void add_comp(f32x4_t& acc, f32x4_t& c, f32x4_t t) {
  const f32x4_t s = acc + t;
  const f32x4_t bb = s - acc;
  c += (acc - (s - bb)) + (t - bb);
  acc = s;
}

// 32 x 32 x 16 form (project phases whose k-step is one 16-channel subtile):
// lane l holds k = 8 (l >> 5) + j of row / column l & 31; the result lane l
// holds column l & 31, rows (r & 3) + 8 (r >> 2) + 4 (l >> 5)
__device__ __forceinline__ f32x16_t mfma32_bf16(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16_t mfma32_x3(const X3Frag& a, const X3Frag& b) {
  f32x16_t t = mfma32_bf16(a.l, b.h, f32x16_t{});
  t = mfma32_bf16(a.h, b.l, t);
  t = mfma32_bf16(a.m, b.m, t);
  t = mfma32_bf16(a.m, b.h, t);
  t = mfma32_bf16(a.h, b.m, t);
  return mfma32_bf16(a.h, b.h, t);
}

// three pre-split parts of 8 consecutive k from a [3][rows][ld] bf16 weight
// buffer (part stride = rows * ld elements)
__device__ __forceinline__ X3Frag load_x3(const uint16_t* __restrict__ w, int64_t part_stride, int64_t off) {
  X3Frag f;
  f.h = *reinterpret_cast<const bf16x8_t*>(w + off);
  f.m = *reinterpret_cast<const bf16x8_t*>(w + part_stride + off);
  f.l = *reinterpret_cast<const bf16x8_t*>(w + 2 * part_stride + off);
  return f;
}

}  // namespace kernels
}  // namespace nnsx
