// Host (CPU) reference implementations of the tensor ops: the numerics
// oracle of the HIP kernels and the `device=-1` path of the elements.
// Semantics mirror gst/nnstreamer/elements/gsttensor_transform.c
// (C-path arithmetic, not the saturating ORC path -- see SURVEY.md §2.4).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <type_traits>

#include "core/types.h"

namespace nnsx {
namespace cpu {

struct half_t {
  uint16_t bits;
};
struct bhalf_t {
  uint16_t bits;
};

inline float half_to_float(uint16_t h) {
  uint32_t sign = (h >> 15) & 1u, exp = (h >> 10) & 0x1fu, man = h & 0x3ffu;
  uint32_t f;
  if (exp == 0) {
    if (man == 0) {
      f = sign << 31;
    } else {
      exp = 127 - 15 + 1;
      while (!(man & 0x400u)) {
        man <<= 1;
        --exp;
      }
      man &= 0x3ffu;
      f = (sign << 31) | (exp << 23) | (man << 13);
    }
  } else if (exp == 0x1f) {
    f = (sign << 31) | 0x7f800000u | (man << 13);
  } else {
    f = (sign << 31) | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float r;
  std::memcpy(&r, &f, 4);
  return r;
}

inline uint16_t float_to_half(float v) {
  uint32_t f;
  std::memcpy(&f, &v, 4);
  uint32_t sign = (f >> 16) & 0x8000u;
  int32_t exp = static_cast<int32_t>((f >> 23) & 0xffu) - 127 + 15;
  uint32_t man = f & 0x7fffffu;
  if (((f >> 23) & 0xffu) == 0xffu) return static_cast<uint16_t>(sign | 0x7c00u | (man ? 0x200u : 0));
  if (exp >= 0x1f) return static_cast<uint16_t>(sign | 0x7c00u);
  if (exp <= 0) {
    if (exp < -10) return static_cast<uint16_t>(sign);
    man |= 0x800000u;
    uint32_t shift = static_cast<uint32_t>(14 - exp);
    uint32_t h = man >> shift;
    uint32_t rem = man & ((1u << shift) - 1);
    uint32_t halfway = 1u << (shift - 1);
    if (rem > halfway || (rem == halfway && (h & 1u))) ++h;
    return static_cast<uint16_t>(sign | h);
  }
  uint32_t h = sign | (static_cast<uint32_t>(exp) << 10) | (man >> 13);
  uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return static_cast<uint16_t>(h);
}

inline float bf16_to_float(uint16_t b) {
  uint32_t f = static_cast<uint32_t>(b) << 16;
  float r;
  std::memcpy(&r, &f, 4);
  return r;
}

inline uint16_t float_to_bf16(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <typename T>
inline double as_double(T v) {
  return static_cast<double>(v);
}
template <>
inline double as_double(half_t v) {
  return half_to_float(v.bits);
}
template <>
inline double as_double(bhalf_t v) {
  return bf16_to_float(v.bits);
}

template <typename T>
struct Cast {
  template <typename S>
  static T from(S v) {
    return static_cast<T>(v);
  }
  static T from(half_t v) { return static_cast<T>(half_to_float(v.bits)); }
  static T from(bhalf_t v) { return static_cast<T>(bf16_to_float(v.bits)); }
};
template <>
struct Cast<half_t> {
  template <typename S>
  static half_t from(S v) {
    return half_t{float_to_half(static_cast<float>(v))};
  }
  static half_t from(half_t v) { return v; }
  static half_t from(bhalf_t v) { return half_t{float_to_half(bf16_to_float(v.bits))}; }
};
template <>
struct Cast<bhalf_t> {
  template <typename S>
  static bhalf_t from(S v) {
    return bhalf_t{float_to_bf16(static_cast<float>(v))};
  }
  static bhalf_t from(bhalf_t v) { return v; }
  static bhalf_t from(half_t v) { return bhalf_t{float_to_bf16(half_to_float(v.bits))}; }
};

#define NNSX_CPU_DTYPE_CASES(DT, MACRO)       \
  switch (DT) {                               \
    case DType::INT32: MACRO(int32_t); break; \
    case DType::UINT32: MACRO(uint32_t); break; \
    case DType::INT16: MACRO(int16_t); break; \
    case DType::UINT16: MACRO(uint16_t); break; \
    case DType::INT8: MACRO(int8_t); break;   \
    case DType::UINT8: MACRO(uint8_t); break; \
    case DType::FLOAT64: MACRO(double); break; \
    case DType::FLOAT32: MACRO(float); break; \
    case DType::INT64: MACRO(int64_t); break; \
    case DType::UINT64: MACRO(uint64_t); break; \
    case DType::FLOAT16: MACRO(::nnsx::cpu::half_t); break; \
    case DType::BFLOAT16: MACRO(::nnsx::cpu::bhalf_t); break; \
    default: break;                           \
  }

// read element i of a typed buffer as double
double read_as_double(const void* p, DType t, uint64_t i);
void write_from_double(void* p, DType t, uint64_t i, double v);

}  // namespace cpu
}  // namespace nnsx
