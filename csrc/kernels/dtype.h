// Device-side scalar type helpers shared by the CDNA4 kernels.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "core/types.h"

namespace nnsx {
namespace kernels {

// float16 / bfloat16 carried as raw 16-bit storage; arithmetic in fp32 with a
// rounding step after every op (matches per-op _Float16 arithmetic).
struct f16s {
  uint16_t bits;
};
struct bf16s {
  uint16_t bits;
};

__device__ __forceinline__ float to_f32(f16s v) {
  return __half2float(__ushort_as_half(v.bits));
}
__device__ __forceinline__ float to_f32(bf16s v) {
  return __uint_as_float(static_cast<uint32_t>(v.bits) << 16);
}
__device__ __forceinline__ f16s make_f16(float f) {
  return f16s{__half_as_ushort(__float2half_rn(f))};
}
__device__ __forceinline__ bf16s make_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return bf16s{static_cast<uint16_t>((u >> 16) | 0x40)};  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return bf16s{static_cast<uint16_t>(u >> 16)};
}

template <typename T>
struct Num {
  // cast any scalar to T with C semantics
  template <typename S>
  __device__ static __forceinline__ T from(S v) { return static_cast<T>(v); }
  __device__ static __forceinline__ T from(f16s v) { return static_cast<T>(to_f32(v)); }
  __device__ static __forceinline__ T from(bf16s v) { return static_cast<T>(to_f32(v)); }
  __device__ static __forceinline__ double as_double(T v) { return static_cast<double>(v); }
};
template <>
struct Num<f16s> {
  template <typename S>
  __device__ static __forceinline__ f16s from(S v) { return make_f16(static_cast<float>(v)); }
  __device__ static __forceinline__ f16s from(f16s v) { return v; }
  __device__ static __forceinline__ f16s from(bf16s v) { return make_f16(to_f32(v)); }
  __device__ static __forceinline__ double as_double(f16s v) { return to_f32(v); }
};
template <>
struct Num<bf16s> {
  template <typename S>
  __device__ static __forceinline__ bf16s from(S v) { return make_bf16(static_cast<float>(v)); }
  __device__ static __forceinline__ bf16s from(bf16s v) { return v; }
  __device__ static __forceinline__ bf16s from(f16s v) { return make_bf16(to_f32(v)); }
  __device__ static __forceinline__ double as_double(bf16s v) { return to_f32(v); }
};

template <typename T>
struct is_intlike {
  static constexpr bool value = false;
};
#define NNSX_INTLIKE(T) \
  template <>           \
  struct is_intlike<T> { static constexpr bool value = true; };
NNSX_INTLIKE(int8_t)
NNSX_INTLIKE(uint8_t)
NNSX_INTLIKE(int16_t)
NNSX_INTLIKE(uint16_t)
NNSX_INTLIKE(int32_t)
NNSX_INTLIKE(uint32_t)
NNSX_INTLIKE(int64_t)
NNSX_INTLIKE(uint64_t)
#undef NNSX_INTLIKE

template <typename T>
struct is_unsigned_int {
  static constexpr bool value = false;
};
template <> struct is_unsigned_int<uint8_t> { static constexpr bool value = true; };
template <> struct is_unsigned_int<uint16_t> { static constexpr bool value = true; };
template <> struct is_unsigned_int<uint32_t> { static constexpr bool value = true; };
template <> struct is_unsigned_int<uint64_t> { static constexpr bool value = true; };

// Host-side dtype switch helper: calls F::template run<T>(args...)
#define NNSX_DTYPE_CASES(DT, MACRO)                     \
  switch (DT) {                                         \
    case DType::INT32: MACRO(int32_t); break;           \
    case DType::UINT32: MACRO(uint32_t); break;         \
    case DType::INT16: MACRO(int16_t); break;           \
    case DType::UINT16: MACRO(uint16_t); break;         \
    case DType::INT8: MACRO(int8_t); break;             \
    case DType::UINT8: MACRO(uint8_t); break;           \
    case DType::FLOAT64: MACRO(double); break;          \
    case DType::FLOAT32: MACRO(float); break;           \
    case DType::INT64: MACRO(int64_t); break;           \
    case DType::UINT64: MACRO(uint64_t); break;         \
    case DType::FLOAT16: MACRO(f16s); break;            \
    case DType::BFLOAT16: MACRO(bf16s); break;          \
    default: break;                                     \
  }

}  // namespace kernels
}  // namespace nnsx
