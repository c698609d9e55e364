/*
 * oracle/ref_volk_harness.c — exports C entry points around the REFERENCE's own volk_gnsssdr
 * generic kernels, compiled from the headers where they lie under /root/reference (see
 * oracle/Makefile; nothing is copied).  TEST INFRASTRUCTURE ONLY: used by tests/ to pin the
 * restatement in oracle/gnss_oracle.c.  Only kernels whose headers need no generated files are
 * built here: the resamplers, the sincos wipeoff generator and index_max.  The rotator
 * dot-products include the Mako-generated <volk_gnsssdr/volk_gnsssdr.h> and are not buildable.
 */
#define LV_HAVE_GENERIC 1
#include <string.h> /* the resampler headers call memcpy without including it */
#include <volk_gnsssdr_32f_xn_resampler_32f_xn.h>
#include <volk_gnsssdr_32f_xn_high_dynamics_resampler_32f_xn.h>
#include <volk_gnsssdr_s32f_sincos_32fc.h>
#include <volk_gnsssdr_32f_index_max_32u.h>
#include <stdlib.h>

/* out: [taps][n] contiguous */
void ref_resampler_generic(float* out, const float* code, float rem, float step, float* shifts, unsigned int L, int taps, unsigned int n)
{
    float* rows[16];
    for (int t = 0; t < taps && t < 16; t++) rows[t] = out + (size_t)t * n;
    volk_gnsssdr_32f_xn_resampler_32f_xn_generic(rows, code, rem, step, shifts, L, taps, n);
}

void ref_high_dynamics_resampler_generic(float* out, const float* code, float rem, float step, float rate, float* shifts, unsigned int L, int taps, unsigned int n)
{
    float* rows[16];
    for (int t = 0; t < taps && t < 16; t++) rows[t] = out + (size_t)t * n;
    volk_gnsssdr_32f_xn_high_dynamics_resampler_32f_xn_generic(rows, code, rem, step, rate, shifts, L, taps, n);
}

void ref_sincos_generic(float* out, float phase_inc, float* phase, unsigned int n)
{
    volk_gnsssdr_s32f_sincos_32fc_generic((lv_32fc_t*)out, phase_inc, phase, n);
}

unsigned int ref_index_max_generic(const float* src, unsigned int n)
{
    uint32_t t = 0;
    volk_gnsssdr_32f_index_max_32u_generic(&t, src, n);
    return t;
}
