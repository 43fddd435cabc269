/*!
 * \file half.h
 * \brief 16-bit floating types of the extended dtype enum (mpi::kHalf = IEEE binary16,
 *        mpi::kBFloat16 = bfloat16): storage types with float arithmetic, usable in host code
 *        (g++) and in gfx950 kernels (hipcc).
 *
 * The reference has no 16-bit types (`include/rabit/internal/engine.h:230-239` stops at
 * kULongLong).  Mixed-precision training on MI355X keeps gradients in bf16, so the engine takes
 * them directly: RCCL reduces them natively, the gfx950 kernels accumulate each element over all
 * peers in fp32 and round once, the host path converts per element.  Conversions round to
 * nearest even; NaN stays NaN.
 */
#ifndef RABIT_INTERNAL_HALF_H_
#define RABIT_INTERNAL_HALF_H_

#include <cstdint>
#include <cstring>

#ifdef __HIPCC__
#define XRABIT_HD __host__ __device__ __forceinline__
#else
#define XRABIT_HD inline
#endif

namespace rabit {
namespace detail {
XRABIT_HD uint32_t FloatBits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}
XRABIT_HD float BitsFloat(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
}  // namespace detail

/*! \brief bfloat16: the upper 16 bits of an IEEE float */
struct bf16_t {
  uint16_t bits;
  bf16_t() = default;
  XRABIT_HD explicit bf16_t(float f) : bits(FromFloat(f)) {}
  XRABIT_HD explicit bf16_t(double f) : bits(FromFloat(static_cast<float>(f))) {}
  XRABIT_HD explicit bf16_t(int i) : bits(FromFloat(static_cast<float>(i))) {}
  XRABIT_HD float f() const { return detail::BitsFloat(static_cast<uint32_t>(bits) << 16); }
  XRABIT_HD static uint16_t FromFloat(float f) {
    const uint32_t u = detail::FloatBits(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);  // NaN
    const uint32_t rounding = 0x7fffu + ((u >> 16) & 1u);                              // RNE
    return static_cast<uint16_t>((u + rounding) >> 16);
  }
};

/*! \brief IEEE 754 binary16 */
struct half_t {
  uint16_t bits;
  half_t() = default;
  XRABIT_HD explicit half_t(float f) : bits(FromFloat(f)) {}
  XRABIT_HD explicit half_t(double f) : bits(FromFloat(static_cast<float>(f))) {}
  XRABIT_HD explicit half_t(int i) : bits(FromFloat(static_cast<float>(i))) {}
  XRABIT_HD float f() const {
    const uint32_t sign = static_cast<uint32_t>(bits & 0x8000u) << 16;
    uint32_t exp = (bits >> 10) & 0x1fu;
    uint32_t man = bits & 0x3ffu;
    if (exp == 0x1fu) return detail::BitsFloat(sign | 0x7f800000u | (man << 13));  // inf / NaN
    if (exp == 0) {
      if (man == 0) return detail::BitsFloat(sign);
      // subnormal: normalise
      int e = -1;
      do {
        man <<= 1;
        ++e;
      } while ((man & 0x400u) == 0);
      man &= 0x3ffu;
      exp = static_cast<uint32_t>(112 - e);  // 127 - 15 - e
      return detail::BitsFloat(sign | (exp << 23) | (man << 13));
    }
    return detail::BitsFloat(sign | ((exp + 112u) << 23) | (man << 13));
  }
  XRABIT_HD static uint16_t FromFloat(float f) {
    const uint32_t u = detail::FloatBits(f);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const uint32_t absu = u & 0x7fffffffu;
    if (absu > 0x7f800000u) return static_cast<uint16_t>(sign | 0x7e00u);  // NaN
    if (absu >= 0x477ff000u) return static_cast<uint16_t>(sign | 0x7c00u);  // overflow -> inf
    if (absu < 0x33000001u) return static_cast<uint16_t>(sign);  // below half the min subnormal
    const int exp = static_cast<int>(absu >> 23) - 127;
    uint32_t man = (absu & 0x7fffffu) | 0x800000u;
    int shift;
    uint32_t base;
    if (exp < -14) {  // subnormal result
      shift = 13 + (-14 - exp);
      base = 0;
    } else {
      shift = 13;
      base = static_cast<uint32_t>(exp + 15) << 10;
      man &= 0x7fffffu;
    }
    uint32_t q = man >> shift;
    const uint32_t rem = man & ((1u << shift) - 1u);
    const uint32_t halfway = 1u << (shift - 1);
    if (rem > halfway || (rem == halfway && (q & 1u))) ++q;  // RNE (a carry bumps the exponent)
    return static_cast<uint16_t>(sign | (base + q));
  }
};

// arithmetic in float, result rounded back (the reducers' a + b, max, min, prepare ops)
#define XRABIT_HALF_OPS(T)                                                             \
  XRABIT_HD T operator+(T a, T b) { return T(a.f() + b.f()); }                         \
  XRABIT_HD T operator*(T a, T b) { return T(a.f() * b.f()); }                         \
  XRABIT_HD T operator-(T a, T b) { return T(a.f() - b.f()); }                         \
  XRABIT_HD T &operator+=(T &a, T b) { return a = a + b; }                             \
  XRABIT_HD bool operator<(T a, T b) { return a.f() < b.f(); }                         \
  XRABIT_HD bool operator>(T a, T b) { return a.f() > b.f(); }
XRABIT_HALF_OPS(bf16_t)
XRABIT_HALF_OPS(half_t)
#undef XRABIT_HALF_OPS

template <typename T>
struct IsHalfType {
  static constexpr bool value = false;
};
template <>
struct IsHalfType<bf16_t> {
  static constexpr bool value = true;
};
template <>
struct IsHalfType<half_t> {
  static constexpr bool value = true;
};
}  // namespace rabit
#endif  // RABIT_INTERNAL_HALF_H_
