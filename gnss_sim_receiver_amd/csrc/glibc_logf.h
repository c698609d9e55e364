// glibc_logf.h — glibc's single-precision logf and log10f, restated operation for operation for the
// lock detector's CN0 estimate: cn0_m2m4_estimator ends in
//   SNR_dB_Hz = 10.0F * std::log10(SNR) - 10.0F * std::log10(coh_integration_time_s)
// (lock_detectors.cc:119), std::log10(float) = log10f.
//   * log10f: sysdeps/ieee754/flt-32/e_log10f.c, the fdlibm routine (float arithmetic, no FMA: it is
//     not one of x86-64's multiarch builds) — the exponent split off, then
//     z = y·log10_2lo + ivln10·logf(m), result z + y·log10_2hi;
//   * logf: sysdeps/ieee754/flt-32/e_logf.c + e_logf_data.c (the ARM optimized-routines logf glibc
//     has shipped since 2.28): a 16-entry table of (1/c, log c) around [0x3f330000, 2·0x3f330000),
//     r = z/c − 1 in double, a degree-3 polynomial — and the FMA build glibc's ifunc picks on any
//     FMA host (every AVX2 server, the GPU box's EPYC included), whose contractions are written out.
// The table and polynomial are the published e_logf_data.c values.  Pinned by
// tests/test_glibc_sincosf.py against the host's logf / log10f (every positive float).
#pragma once
#include <cstdint>

#ifndef GNSSHIP_HD
#define GNSSHIP_HD __host__ __device__
#endif

namespace gnsship {
namespace glog {

// __logf_data.tab[i] = {invc, logc} (e_logf_data.c)
GNSSHIP_HD inline double invc(int i)
{
    constexpr double kT[16] = {0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
                               0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
                               0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
                               0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
    return kT[i];
}
GNSSHIP_HD inline double logc(int i)
{
    constexpr double kT[16] = {-0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
                               -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3,   -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4,
                               -0x1.252f438e10c1ep-5, 0x0p+0,                0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
                               0x1.526e57720db08p-3,  0x1.bc2860d22477p-3,   0x1.1058bc8a07ee1p-2,  0x1.4043057b6ee09p-2};
    return kT[i];
}
constexpr double kLn2 = 0x1.62e42fefa39efp-1;
constexpr double kA0 = -0x1.00ea348b88334p-2, kA1 = 0x1.5575b0be00b6ap-2, kA2 = -0x1.ffffef20a4123p-2;

}  // namespace glog

// __logf (e_logf.c), FMA build
GNSSHIP_HD inline float glibc_logf(float x)
{
#pragma clang fp contract(off)
    using namespace glog;
    uint32_t ix = __builtin_bit_cast(uint32_t, x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {  // x < 0x1p-126, inf or nan
        if (ix * 2 == 0) return -__builtin_inff();
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
        ix = __builtin_bit_cast(uint32_t, x * 0x1p23f);  // subnormal: normalise
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = static_cast<int>((tmp >> (23 - 4)) % 16);
    const int k = static_cast<int32_t>(tmp) >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double z = static_cast<double>(__builtin_bit_cast(float, iz));
    const double r = __builtin_fma(z, invc(i), -1.0);                    // z·invc − 1
    const double y0 = __builtin_fma(static_cast<double>(k), kLn2, logc(i));  // logc + k·Ln2
    const double r2 = r * r;
    double y = __builtin_fma(kA1, r, kA2);
    y = __builtin_fma(kA0, r2, y);
    y = __builtin_fma(y, r2, y0 + r);
    return static_cast<float>(y);
}

// __ieee754_log10f (e_log10f.c)
GNSSHIP_HD inline float glibc_log10f(float x)
{
#pragma clang fp contract(off)
    const float two25 = 0x1p25f;
    const float ivln10 = __builtin_bit_cast(float, 0x3ede5bd9u), log10_2hi = __builtin_bit_cast(float, 0x3e9a2080u),
                log10_2lo = __builtin_bit_cast(float, 0x355427dbu);
    int32_t hx = __builtin_bit_cast(int32_t, x);
    int32_t k = 0;
    if (hx < 0x00800000) {  // x < 2^-126
        if ((hx & 0x7fffffff) == 0) return -__builtin_inff();
        if (hx < 0) return __builtin_nanf("");
        k -= 25;
        x *= two25;  // subnormal: scale up
        hx = __builtin_bit_cast(int32_t, x);
    }
    if (hx >= 0x7f800000) return x + x;
    k += (hx >> 23) - 127;
    const int32_t i = static_cast<int32_t>((static_cast<uint32_t>(k) & 0x80000000u) >> 31);
    hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
    const float y = static_cast<float>(k + i);
    const float z = y * log10_2lo + ivln10 * glibc_logf(__builtin_bit_cast(float, hx));
    return z + y * log10_2hi;
}

}  // namespace gnsship
