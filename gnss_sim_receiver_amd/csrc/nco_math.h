// nco_math.h — device helpers shared by the correlator kernels: complex products and magnitudes
// rounded exactly like the reference's generic C (every operation rounded on its own, no FMA).
#pragma once
#include <hip/hip_runtime.h>

#include "glibc_atanf.h"
#include "glibc_logf.h"
#include "glibc_sincosf.h"

namespace gnsship {

__device__ __forceinline__ float2 cmul_rn(float ar, float ai, float br, float bi)
{
    return make_float2(__fsub_rn(__fmul_rn(ar, br), __fmul_rn(ai, bi)), __fadd_rn(__fmul_rn(ar, bi), __fmul_rn(ai, br)));
}

// IEEE single square root, correctly rounded (sqrtf / _mm256_sqrt_ps).  On gfx950 __fsqrt_rn and
// sqrtf lower to V_SQRT_F32 alone, which is only 1-ulp accurate (the AVX rotator's dz =
// normalise(inc^16) then differs by an ulp in a few epochs, and the phase error grows over the
// 16-lane chain); the hardware result is corrected by the sign of the residuals x − s⁻·s and
// x − s⁺·s of its neighbours (the lowering LLVM uses for correctly rounded f32 sqrt).  Inputs are
// normal and positive here (|z|² ≈ 1, power sums); ±0, +inf and NaN pass through V_SQRT_F32.
__device__ __forceinline__ float sqrt_rn_f32(float x)
{
    float s;
    asm("v_sqrt_f32 %0, %1" : "=v"(s) : "v"(x));
    const float dn = __int_as_float(__float_as_int(s) - 1), up = __int_as_float(__float_as_int(s) + 1);
    const float r_dn = __builtin_fmaf(-dn, s, x), r_up = __builtin_fmaf(-up, s, x);
    const bool finite_pos = x > 0.0f && x < __int_as_float(0x7f800000) && x >= 1.17549435e-38f;
    float r = s;
    if (r_dn <= 0.0f) r = dn;
    if (r_up > 0.0f) r = up;
    return finite_pos ? r : s;
}

// std::abs(std::complex<float>) / C hypotf → glibc hypotf, which evaluates sqrt(x²+y²) in double and
// rounds once.
__device__ __forceinline__ float hypotf_glibc(float x, float y)
{
    const double dx = x, dy = y;
    return static_cast<float>(__dsqrt_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy))));
}

}  // namespace gnsship
