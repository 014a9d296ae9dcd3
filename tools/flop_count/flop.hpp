// flop.hpp -- an FP64 value type that counts the arithmetic done on it, so
// that the device functions of lfg_device.hpp can be compiled for the host
// (tools/flop_count/count.cpp, `#define double F64`) and their work counted
// operation by operation (MODEL_SPEC.md section 11).  Tooling only: nothing
// here is on the product path.
//
// Counting rules (the FP64 peak's own: one FMA = 2 FLOP):
//   add, sub, mul                1
//   fma                          2
//   div                          1   (IEEE quotient)
//   sqrt, rsqrt, rcp (v_rsq/v_rcp)  1
//   transcendental (sin, cos, atan2, acos, log, exp, pow, cbrt)  1 each,
//                                counted separately as well
//   negation, fabs, fmin, fmax, compares, selects, conversions  0
#pragma once
#include <cmath>
#include <type_traits>

struct FlopCtr {
    long long add = 0, mul = 0, fma = 0, div = 0, sqrt = 0, trans = 0;
    long long flops() const { return add + mul + 2 * fma + div + sqrt + trans; }
};
inline FlopCtr g_ctr;

#define LFG_CNT(f)                               \
    do {                                         \
        if (!std::is_constant_evaluated()) g_ctr.f++; \
    } while (0)

struct F64 {
    double v;
    constexpr F64() : v(0.0) {}
    template <class T, class = std::enable_if_t<std::is_arithmetic_v<T>>>
    constexpr F64(T x) : v(static_cast<double>(x)) {}
    template <class T, class = std::enable_if_t<std::is_arithmetic_v<T>>>
    explicit constexpr operator T() const { return static_cast<T>(v); }
    constexpr F64 operator-() const { return F64(-v); }
    constexpr F64& operator+=(F64 o);
    constexpr F64& operator-=(F64 o);
    constexpr F64& operator*=(F64 o);
    constexpr F64& operator/=(F64 o);
};

constexpr F64 operator+(F64 a, F64 b) { LFG_CNT(add); return F64(a.v + b.v); }
constexpr F64 operator-(F64 a, F64 b) { LFG_CNT(add); return F64(a.v - b.v); }
constexpr F64 operator*(F64 a, F64 b) { LFG_CNT(mul); return F64(a.v * b.v); }
constexpr F64 operator/(F64 a, F64 b) { LFG_CNT(div); return F64(a.v / b.v); }
constexpr F64& F64::operator+=(F64 o) { *this = *this + o; return *this; }
constexpr F64& F64::operator-=(F64 o) { *this = *this - o; return *this; }
constexpr F64& F64::operator*=(F64 o) { *this = *this * o; return *this; }
constexpr F64& F64::operator/=(F64 o) { *this = *this / o; return *this; }
constexpr bool operator<(F64 a, F64 b) { return a.v < b.v; }
constexpr bool operator>(F64 a, F64 b) { return a.v > b.v; }
constexpr bool operator<=(F64 a, F64 b) { return a.v <= b.v; }
constexpr bool operator>=(F64 a, F64 b) { return a.v >= b.v; }
constexpr bool operator==(F64 a, F64 b) { return a.v == b.v; }
constexpr bool operator!=(F64 a, F64 b) { return a.v != b.v; }

inline F64 fma(F64 a, F64 b, F64 c) { LFG_CNT(fma); return F64(std::fma(a.v, b.v, c.v)); }
inline F64 sqrt(F64 a) { LFG_CNT(sqrt); return F64(std::sqrt(a.v)); }
inline F64 rsqrt(F64 a) { LFG_CNT(sqrt); return F64(1.0 / std::sqrt(a.v)); }
inline F64 lfg_rsq(F64 a) { LFG_CNT(sqrt); return F64(1.0 / std::sqrt(a.v)); }
inline F64 lfg_rcp(F64 a) { LFG_CNT(sqrt); return F64(1.0 / a.v); }
inline F64 cbrt(F64 a) { LFG_CNT(trans); return F64(std::cbrt(a.v)); }
inline F64 log(F64 a) { LFG_CNT(trans); return F64(std::log(a.v)); }
inline F64 exp(F64 a) { LFG_CNT(trans); return F64(std::exp(a.v)); }
inline F64 pow(F64 a, F64 b) { LFG_CNT(trans); return F64(std::pow(a.v, b.v)); }
inline F64 acos(F64 a) { LFG_CNT(trans); return F64(std::acos(a.v)); }
inline F64 atan2(F64 a, F64 b) { LFG_CNT(trans); return F64(std::atan2(a.v, b.v)); }
inline F64 cos(F64 a) { LFG_CNT(trans); return F64(std::cos(a.v)); }
inline F64 sin(F64 a) { LFG_CNT(trans); return F64(std::sin(a.v)); }
inline void sincos(F64 a, F64* s, F64* c)
{
    LFG_CNT(trans);
    LFG_CNT(trans);
    *s = F64(std::sin(a.v));
    *c = F64(std::cos(a.v));
}
inline F64 fabs(F64 a) { return F64(std::fabs(a.v)); }
inline F64 fmin(F64 a, F64 b) { return F64(std::fmin(a.v, b.v)); }
inline F64 fmax(F64 a, F64 b) { return F64(std::fmax(a.v, b.v)); }
inline F64 floor(F64 a) { return F64(std::floor(a.v)); }
inline bool isfinite(F64 a) { return std::isfinite(a.v); }
inline bool isnan(F64 a) { return std::isnan(a.v); }
