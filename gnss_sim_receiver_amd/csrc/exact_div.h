// exact_div.h — quotients by a divisor fixed for the run and the remainder mod 2π, bit-identical to
// the IEEE division and fmod the reference's loop code performs (tracking_loop / update_tracking_vars
// divide by fs_in, by the carrier frequency and by TWO_PI, and take fmod(·, TWO_PI)), in a few FMAs
// instead of the f64 division and fmod sequences.
//   * x / d with inv = RN(1/d): q0 = RN(x·inv), r = x − q0·d (exact in one FMA), q = RN(q0 + r·inv)
//     — Markstein's correction, which returns the correctly rounded quotient for a correctly rounded
//     reciprocal;
//   * fmod(x, c) for c ∈ [4, 8) and |x| < 2^40: n = trunc(x/c) (off by one at most near a multiple of
//     c, then corrected), r = x − n·c in one FMA — exact: r is a multiple of min(ulp(x), ulp(c)) below
//     8 in magnitude; larger |x| take fmod itself.
// Pinned by tests/test_exact_div.py (tests/cpp/exact_div_check.cpp) against the host's division and
// fmod: 10^9 quotients over the engines' divisors and random ones, every float below 2^23 and
// 4·10^8 random doubles below 2^40 for the remainder.
#pragma once
#include <cmath>

#ifndef GNSSHIP_HD
#define GNSSHIP_HD __host__ __device__
#endif

namespace gnsship {

GNSSHIP_HD inline double div_by(double x, double d, double inv)
{
    const double q0 = x * inv;
    if (q0 == 0.0 || !(q0 - q0 == 0.0)) return q0;  // ±0 keeps x's sign; inf / NaN pass through
    const double r = __builtin_fma(-q0, d, x);
    return __builtin_fma(r, inv, q0);
}

GNSSHIP_HD inline double fmod_by(double x, double c, double inv)
{
    if (!(__builtin_fabs(x) < 0x1p40)) return fmod(x, c);
    const double n = __builtin_trunc(x * inv);
    double r = __builtin_fma(-n, c, x);
    if (x >= 0.0) {
        if (r < 0.0) r = __builtin_fma(-(n - 1.0), c, x);
        else if (r >= c) r = __builtin_fma(-(n + 1.0), c, x);
    } else {
        if (r > 0.0) r = __builtin_fma(-(n + 1.0), c, x);
        else if (r <= -c) r = __builtin_fma(-(n - 1.0), c, x);
    }
    return r == 0.0 ? __builtin_copysign(0.0, x) : r;
}

}  // namespace gnsship
