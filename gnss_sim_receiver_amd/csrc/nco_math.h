// nco_math.h — device helpers shared by the correlator kernels: complex products and magnitudes
// rounded exactly like the reference's generic C (every operation rounded on its own, no FMA).
#pragma once
#include <hip/hip_runtime.h>

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

// cos / sin of a float argument as the double-precision result rounded once to float: the
// correctly rounded value except at rare double-rounding ties.  The reference's phasors come from
// glibc cosf/sinf (std::cos(float), cexpf), which agree with this in ~99 % of arguments (glibc's
// float routines are not correctly rounded, and its FMA and non-FMA variants differ between
// hosts); the device's own single-precision cosf/sinf agree far less often.
__device__ __forceinline__ float cos_f32_rn(float x) { return static_cast<float>(cos(static_cast<double>(x))); }
__device__ __forceinline__ float sin_f32_rn(float x) { return static_cast<float>(sin(static_cast<double>(x))); }


// sin / cos in double of a small argument (|x| below ~1e5; the tracking NCO's phase and step are
// within ±2π): the fdlibm scheme — Cody-Waite reduction by π/2 in three parts, then __kernel_sin /
// __kernel_cos with the reduction's tail — with explicit FMAs, ≤ 1 ulp in double.  Rounded to float
// it agreed with glibc's double sin/cos on 20 M arguments in ±7 rad and ±1e-3 rad (once-rounded
// float cos/sin, as cos_f32_rn / sin_f32_rn); about a sixth of ocml's general sincos on the chain.
__device__ __forceinline__ void sincos_f64_small(double x, double* s, double* c)
{
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00;
    const double pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
    const double k = rint(x * invpio2);
    const double r0 = __fma_rn(-k, pio2_1, x);  // exact: k small, pio2_1 has 33 bits
    const double w = __dmul_rn(k, pio2_2);      // exact: pio2_2 has 33 bits
    const double r1 = __dsub_rn(r0, w);
    const double wt = __fma_rn(k, pio2_2t, -__dsub_rn(__dsub_rn(r0, r1), w));
    const double y0 = __dsub_rn(r1, wt);
    const double y1 = __dsub_rn(__dsub_rn(r1, y0), wt);
    const double z = __dmul_rn(y0, y0), v = __dmul_rn(z, y0);
    // __kernel_sin(y0, y1)
    const double rs = __fma_rn(z, __fma_rn(z, __fma_rn(z, __fma_rn(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08), 2.75573137070700676789e-06),
                                   -1.98412698298579493134e-04), 8.33333333332248946124e-03);
    const double sn = __dsub_rn(y0, __dsub_rn(__dsub_rn(__dmul_rn(z, __dsub_rn(__dmul_rn(0.5, y1), __dmul_rn(v, rs))), y1), __dmul_rn(v, -1.66666666666666324348e-01)));
    // __kernel_cos(y0, y1)
    const double rc = __dmul_rn(z, __fma_rn(z, __fma_rn(z, __fma_rn(z, __fma_rn(z, __fma_rn(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                                              -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                                       -1.38888888888741095749e-03), 4.16666666666666019037e-02));
    const double hz = __dmul_rn(0.5, z), ww = __dsub_rn(1.0, hz);
    const double cs = __dadd_rn(ww, __dadd_rn(__dsub_rn(__dsub_rn(1.0, ww), hz), __dsub_rn(__dmul_rn(z, rc), __dmul_rn(y0, y1))));
    const int q = static_cast<int>(k) & 3;
    *s = q == 0 ? sn : q == 1 ? cs : q == 2 ? -sn : -cs;
    *c = q == 0 ? cs : q == 1 ? -sn : q == 2 ? -cs : sn;
}

}  // namespace gnsship
