// glibc_atanf.h — glibc's single-precision atanf and atan2f (sysdeps/ieee754/flt-32/s_atanf.c and
// e_atan2f.c, the fdlibm float routines: float arithmetic throughout, built without FMA on x86-64),
// restated operation for operation for the tracking loop's discriminators:
//   pll_cloop_two_quadrant_atan  std::atan(Q / I)                 (tracking_discriminators.cc:99-104)
//   fll_diff_atan                std::atan of two prompt ratios   (:68-76)
//   pll_four_quadrant_atan       gr::fast_atan2f(Q, I)            (:86-89; GNU Radio is absent here, so
//                                the oracle and the engine both use atan2f in its place)
// With these, the device's loop and the oracle loop (oracle/trk_oracle.c, host glibc) see the same
// discriminator bits.  Pinned by tests/test_glibc_sincosf.py against the host's atanf / atan2f.
#pragma once
#include <cstdint>

#ifndef GNSSHIP_HD
#define GNSSHIP_HD __host__ __device__
#endif

namespace gnsship {
namespace gatan {

// atan(0.5), atan(1), atan(1.5), atan(inf) as hi + lo, and the polynomial (s_atanf.c)
GNSSHIP_HD inline float hi(int i)
{
    return i == 0 ? __builtin_bit_cast(float, 0x3eed6338u) : i == 1 ? __builtin_bit_cast(float, 0x3f490fdau) : i == 2 ? __builtin_bit_cast(float, 0x3f7b985eu)
                                                                                                               : __builtin_bit_cast(float, 0x3fc90fdau);
}
GNSSHIP_HD inline float lo(int i)
{
    return i == 0 ? __builtin_bit_cast(float, 0x31ac3769u) : i == 1 ? __builtin_bit_cast(float, 0x33222168u) : i == 2 ? __builtin_bit_cast(float, 0x33140fb4u)
                                                                                                               : __builtin_bit_cast(float, 0x33a22168u);
}
constexpr uint32_t kAT[11] = {0x3eaaaaab, 0xbe4ccccd, 0x3e124925, 0xbde38e38, 0x3dba2e6e, 0xbd9d8795,
                              0x3d886b35, 0xbd6ef16b, 0x3d4bda59, 0xbd15a221, 0x3c8569d7};
GNSSHIP_HD inline float aT(int i) { return __builtin_bit_cast(float, kAT[i]); }

}  // namespace gatan

// __atanf (s_atanf.c)
GNSSHIP_HD inline float glibc_atanf(float x)
{
#pragma clang fp contract(off)
    using namespace gatan;
    const int32_t hx = __builtin_bit_cast(int32_t, x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;  // NaN
        return hx > 0 ? hi(3) + lo(3) : -hi(3) - lo(3);
    }
    if (ix < 0x3ee00000) {  // |x| < 0.4375
        if (ix < 0x31000000) return x;  // |x| < 2^-29
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {    // |x| < 1.1875
            if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {  // 11/16 <= |x| < 19/16
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else {
            if (ix < 0x401c0000) {  // |x| < 2.4375
                id = 2;
                x = (x - 1.5f) / (1.0f + 1.5f * x);
            } else {  // 2.4375 <= |x| < 2^25
                id = 3;
                x = -1.0f / x;
            }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT(0) + w * (aT(2) + w * (aT(4) + w * (aT(6) + w * (aT(8) + w * aT(10))))));
    const float s2 = w * (aT(1) + w * (aT(3) + w * (aT(5) + w * (aT(7) + w * aT(9)))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = hi(id) - ((x * (s1 + s2) - lo(id)) - x);
    return hx < 0 ? -r : r;
}

// __ieee754_atan2f (e_atan2f.c)
GNSSHIP_HD inline float glibc_atan2f(float y, float x)
{
#pragma clang fp contract(off)
    const float pi_o_4 = __builtin_bit_cast(float, 0x3f490fdbu), pi_o_2 = __builtin_bit_cast(float, 0x3fc90fdbu);
    const float pi = __builtin_bit_cast(float, 0x40490fdbu), pi_lo = __builtin_bit_cast(float, 0xb3bbbd2eu);
    const float tiny = 1.0e-30f;
    const int32_t hx = __builtin_bit_cast(int32_t, x), ix = hx & 0x7fffffff;
    const int32_t hy = __builtin_bit_cast(int32_t, y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;  // NaN
    if (hx == 0x3f800000) return glibc_atanf(y);           // x = 1.0
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      // 2·sign(x) + sign(y)
    if (iy == 0) {  // y = 0
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;  // x = 0
    if (ix == 0x7f800000) {  // x = ±inf
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0f * pi_o_4 + tiny;
            default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;  // y = ±inf
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 26)
        z = pi_o_2 + 0.5f * pi_lo;  // |y / x| > 2^26
    else if (hx < 0 && k < -26)
        z = 0.0f;  // |y| / x < −2^26
    else
        z = glibc_atanf(__builtin_fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

}  // namespace gnsship
