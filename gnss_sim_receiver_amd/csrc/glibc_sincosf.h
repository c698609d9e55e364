// glibc_sincosf.h — glibc's single-precision sin/cos (sysdeps/ieee754/flt-32/s_sincosf.c,
// s_sincosf.h, s_sincosf_data.c: the ARM optimized-routines implementation glibc has shipped since
// 2.28), restated operation for operation so that the tracking engines' carrier phasors are the
// reference's own.
//
// Why: Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler forms
//   phase_offset = (std::cos(rem), −std::sin(rem))          (cpu_multicorrelator_real_codes.cc:115)
//   phase_inc    = std::exp(std::complex<float>(0, −step))  (:123)
// i.e. glibc cosf / sinf, and cexpf → __sincosf (s_cexp_template.c: exp(0) = 1 times the sincos
// pair; |im| ≤ FLT_MIN gives (1, im), which is also __sincosf's tiny-argument branch).  On x86-64
// glibc dispatches (ifunc) the same C source built with -mfma -mavx2 on any FMA host (every AVX2
// server, the GPU box's EPYC included), so GCC's contraction of the `a + b * c` forms into single
// FMAs is part of the result: it is spelled out below.  The non-FMA build differs on rare
// arguments; it is not what the reference runs on such hosts.
//
// The arithmetic is all double: a reduction (|y| < 120: one FMA against π/2 with the quadrant from
// a 2^24-scaled product; larger: the 192-bit 4/π table), then the degree-5/6 even/odd polynomials,
// rounded once to float.  sin and cos of one argument come out bit-identical to separate sinf /
// cosf calls (sinf_poly and sincosf_poly evaluate the same expressions).
//
// Pinned by tests/test_glibc_sincosf.py: the host-compiled restatement against the host's own
// sinf / cosf / sincosf on ≥ 20 M arguments (the NCO's phase and step ranges, the C5 IF steps,
// every float in chosen binades and a random sweep of the whole line).
#pragma once
#include <cstdint>

#ifndef GNSSHIP_HD
#define GNSSHIP_HD __host__ __device__
#endif

namespace gnsship {
namespace gsf {

// __sincosf_table[0] (s_sincosf_data.c); entry 1 negates the cosine polynomial (c0..c4)
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;  // 2/π · 2^24 (TOINT_INTRINSICS is 0 on x86-64)
constexpr double kHpi = 0x1.921FB54442D18p0;       // π/2
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5, kC3 = -0x1.6c087e89a359dp-10,
                 kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;
constexpr double kPi63 = 0x1.921FB54442D18p-62;  // π · 2^-64

GNSSHIP_HD inline double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

GNSSHIP_HD inline uint32_t abstop12(float x) { return (__builtin_bit_cast(uint32_t, x) >> 20) & 0x7ff; }

// sincosf_poly (s_sincosf.h) with the FMA build's contractions; neg: table entry 1 (n & 2)
GNSSHIP_HD inline void poly(double x, double x2, bool neg, int n, float* sinp, float* cosp)
{
#pragma clang fp contract(off)
    const double c0 = neg ? -kC0 : kC0, c1 = neg ? -kC1 : kC1, c2c = neg ? -kC2 : kC2, c3 = neg ? -kC3 : kC3, c4 = neg ? -kC4 : kC4;
    const double x4 = x2 * x2;
    const double x3 = x2 * x;
    const double c2 = fma_d(x2, c4, c3);
    const double s1 = fma_d(x2, kS3, kS2);
    const double cc1 = fma_d(x2, c1, c0);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = fma_d(x3, kS1, x);
    const double c = fma_d(x4, c2c, cc1);
    const float sv = static_cast<float>(fma_d(x5, s1, s));
    const float cv = static_cast<float>(fma_d(x6, c2, c));
    // n odd: the sine and cosine results swap places
    *sinp = (n & 1) ? cv : sv;
    *cosp = (n & 1) ? sv : cv;
}

// reduce_large (s_sincosf.h): |y| ≥ 120 against the 4/π bits (__inv_pio4, s_sincosf_data.c: the
// 32-bit windows of 2/π at byte steps)
GNSSHIP_HD inline uint32_t inv_pio4(int i)
{
    constexpr uint32_t kT[24] = {0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
        0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0, 0x34ddc0db,
        0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
    return kT[i];
}

GNSSHIP_HD inline double reduce_large(uint32_t xi, int* np)
{
#pragma clang fp contract(off)
    const int base = (xi >> 26) & 15;
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = static_cast<uint32_t>(xi * inv_pio4(base));
    const uint64_t res1 = static_cast<uint64_t>(xi) * inv_pio4(base + 4);
    const uint64_t res2 = static_cast<uint64_t>(xi) * inv_pio4(base + 8);
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    const double x = static_cast<double>(static_cast<int64_t>(res0));
    *np = static_cast<int>(n);
    return x * kPi63;
}

}  // namespace gsf

// __sincosf (s_sincosf.c), the FMA build: *s = sinf(y), *c = cosf(y) bit for bit.
GNSSHIP_HD inline void glibc_sincosf(float y, float* sinp, float* cosp)
{
#pragma clang fp contract(off)
    using namespace gsf;
    double x = y;
    const uint32_t top = abstop12(y);
    if (top < abstop12(0x1.921FB6p-1f)) {  // |y| < π/4 (abstop12 of the double pio4 rounded to float)
        if (top < abstop12(0x1p-12f)) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
        poly(x, x * x, false, 0, sinp, cosp);
    } else if (top < abstop12(120.0f)) {
        // reduce_fast: the quadrant in bits 24..31 of a 2^24-scaled product, then x − n·π/2 as one FMA
        const double r = x * kHpiInv;
        const int n = (static_cast<int32_t>(r) + 0x800000) >> 24;
        x = fma_d(-static_cast<double>(n), kHpi, x);
        const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;  // sign[4] = {1, −1, −1, 1}
        poly(x * s, x * x, (n & 2) != 0, n, sinp, cosp);
    } else if (top < abstop12(__builtin_inff())) {
        const uint32_t xi = __builtin_bit_cast(uint32_t, y);
        const int sign = static_cast<int>(xi >> 31);
        int n;
        x = reduce_large(xi, &n);
        const int q = (n + sign) & 3;
        const double s = (q == 1 || q == 2) ? -1.0 : 1.0;
        poly(x * s, x * x, (q & 2) != 0, n, sinp, cosp);
    } else {
        const float nan = y - y;  // ±inf, NaN → NaN (glibc: __math_invalidf)
        *sinp = nan;
        *cosp = nan;
    }
}

}  // namespace gnsship
