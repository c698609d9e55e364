// nco_math.h — device helpers shared by the correlator kernels: complex products and magnitudes
// rounded exactly like the reference's generic C (every operation rounded on its own, no FMA).
#pragma once
#include <hip/hip_runtime.h>

namespace gnsship {

__device__ __forceinline__ float2 cmul_rn(float ar, float ai, float br, float bi)
{
    return make_float2(__fsub_rn(__fmul_rn(ar, br), __fmul_rn(ai, bi)), __fadd_rn(__fmul_rn(ar, bi), __fmul_rn(ai, br)));
}

// std::abs(std::complex<float>) / C hypotf → glibc hypotf, which evaluates sqrt(x²+y²) in double and
// rounds once.
__device__ __forceinline__ float hypotf_glibc(float x, float y)
{
    const double dx = x, dy = y;
    return static_cast<float>(__dsqrt_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy))));
}

// cos / sin of a float argument as the double-precision result rounded once to float: the
// correctly rounded value except at rare double-rounding ties.  The reference's phasors come from
// glibc cosf/sinf (std::cos(float), cexpf), which agree with this in ~99 % of arguments (glibc's
// float routines are not correctly rounded, and its FMA and non-FMA variants differ between
// hosts); the device's own single-precision cosf/sinf agree far less often.
__device__ __forceinline__ float cos_f32_rn(float x) { return static_cast<float>(cos(static_cast<double>(x))); }
__device__ __forceinline__ float sin_f32_rn(float x) { return static_cast<float>(sin(static_cast<double>(x))); }

}  // namespace gnsship
