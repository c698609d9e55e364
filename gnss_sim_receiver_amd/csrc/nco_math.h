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

}  // namespace gnsship
