/*
 * oracle/avx_port.c — AVX restatement of the reference's AVX correlator, for the TIMED CPU BASELINE.
 *
 * TEST INFRASTRUCTURE ONLY (as gnss_oracle.c): bench.py's cpu_baseline switches it on with
 * orc_set_simd(1); tests/ check it against the scalar restatement bit for bit.  The product never
 * links it.
 *
 * What volk_gnsssdr runs on an x86 host with AVX (volk_gnsssdr_rank_archs picks u_avx/a_avx):
 *   - volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_u_avx (…rotator_dot_prod_32fc_xn.h:155-316):
 *     16 phasors in four __m256 (4 complex each), advanced by dz = normalise(inc^16) once per
 *     16-sample iteration with _mm256_complexmul_ps, renormalised after iterations m ≡ 0 (mod 64)
 *     with _mm256_complexnormalise_ps (volk_gnsssdr_avx_intrinsics.h:20-29, 56-63), products
 *     accumulated per tap in four __m256 (sample 16m + 4g + j → register g, lane j), summed at the
 *     end as ((r0 + r1) + r2) + r3 then lanes 0..3; the N mod 16 tail serially from normalise(z0);
 *   - volk_gnsssdr_32f_xn_resampler_32f_xn (…resampler_32f_xn.h, u_avx): the chip index
 *     floor(step·n + shift − rem) for 8 samples per __m256, wrapped into [0, L).
 * Every lane operation is the IEEE single op the scalar restatement in gnss_oracle.c performs in the
 * same order, so the results are bit-identical to orc_rotator_dot_prod_avx / orc_resampler_generic
 * (tests/test_oracle_avx_port.py).  Built with per-function target attributes (no -mavx needed);
 * orc_simd_available() reports whether this CPU runs them.
 */
#include <immintrin.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_AVX_TARGET __attribute__((target("avx2")))

int orc_simd_available(void)
{
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") ? 1 : 0;
}

/* _mm256_complexmul_ps: (xr·yr − xi·yi, xi·yr + xr·yi) per complex lane */
ORC_AVX_TARGET static inline __m256 cmul8(__m256 x, __m256 y)
{
    const __m256 yl = _mm256_moveldup_ps(y), yh = _mm256_movehdup_ps(y);
    const __m256 t1 = _mm256_mul_ps(x, yl);
    const __m256 xs = _mm256_shuffle_ps(x, x, 0xB1);
    const __m256 t2 = _mm256_mul_ps(xs, yh);
    return _mm256_addsub_ps(t1, t2);
}

/* _mm256_complexnormalise_ps: z / sqrt(re² + im²) per complex lane */
ORC_AVX_TARGET static inline __m256 cnorm8(__m256 z)
{
    const __m256 sq = _mm256_mul_ps(z, z);
    const __m256 h = _mm256_hadd_ps(sq, sq);
    const __m256 m = _mm256_sqrt_ps(_mm256_shuffle_ps(h, h, 0xD8));
    return _mm256_div_ps(z, m);
}

static inline void cmul1(float a, float b, float c, float d, float* re, float* im)
{
    *re = a * c - b * d;
    *im = a * d + b * c;
}

ORC_AVX_TARGET void orc_rotator_dot_prod_avx_vec(float* result, const float* in_common, float inc_re, float inc_im, float* phase,
    const float* in_a, int num_a_vectors, unsigned int num_points)
{
    const unsigned int sixteenth = num_points / 16;
    float zr[16], zi[16];
    float pr = phase[0], pi = phase[1];
    for (int l = 0; l < 16; l++) {
        zr[l] = pr;
        zi[l] = pi;
        float nr, ni;
        cmul1(pr, pi, inc_re, inc_im, &nr, &ni);
        pr = nr;
        pi = ni;
    }
    float dr = inc_re, di = inc_im;
    for (int k = 0; k < 4; k++) {
        float nr, ni;
        cmul1(dr, di, dr, di, &nr, &ni);
        dr = nr;
        di = ni;
    }
    {
        const float m = sqrtf(dr * dr + di * di);
        dr = dr / m;
        di = di / m;
    }
    __m256 z[4];
    for (int g = 0; g < 4; g++) {
        float tmp[8];
        for (int j = 0; j < 4; j++) {
            tmp[2 * j] = zr[4 * g + j];
            tmp[2 * j + 1] = zi[4 * g + j];
        }
        z[g] = _mm256_loadu_ps(tmp);
    }
    const __m256 dz = _mm256_setr_ps(dr, di, dr, di, dr, di, dr, di);
    __m256 acc[4][8];
    for (int g = 0; g < 4; g++)
        for (int t = 0; t < num_a_vectors; t++) acc[g][t] = _mm256_setzero_ps();
    for (unsigned int m = 0; m < sixteenth; m++) {
        const float* x = in_common + 32 * (size_t)m;
        __m256 p[4];
        for (int g = 0; g < 4; g++) {
            p[g] = cmul8(_mm256_loadu_ps(x + 8 * g), z[g]);
            z[g] = cmul8(z[g], dz);
        }
        for (int t = 0; t < num_a_vectors; t++) {
            const float* c = in_a + (size_t)t * num_points + 16 * (size_t)m;
            const __m256 c01 = _mm256_loadu_ps(c), c23 = _mm256_loadu_ps(c + 8);
            /* (c0,c0,c1,c1,c2,c2,c3,c3) for each group of 4 complex lanes */
            const __m256 lo0 = _mm256_unpacklo_ps(c01, c01), hi0 = _mm256_unpackhi_ps(c01, c01);
            const __m256 lo1 = _mm256_unpacklo_ps(c23, c23), hi1 = _mm256_unpackhi_ps(c23, c23);
            const __m256 e0 = _mm256_permute2f128_ps(lo0, hi0, 0x20), e1 = _mm256_permute2f128_ps(lo0, hi0, 0x31);
            const __m256 e2 = _mm256_permute2f128_ps(lo1, hi1, 0x20), e3 = _mm256_permute2f128_ps(lo1, hi1, 0x31);
            acc[0][t] = _mm256_add_ps(acc[0][t], _mm256_mul_ps(p[0], e0));
            acc[1][t] = _mm256_add_ps(acc[1][t], _mm256_mul_ps(p[1], e1));
            acc[2][t] = _mm256_add_ps(acc[2][t], _mm256_mul_ps(p[2], e2));
            acc[3][t] = _mm256_add_ps(acc[3][t], _mm256_mul_ps(p[3], e3));
        }
        if (m % 64 == 0)
            for (int g = 0; g < 4; g++) z[g] = cnorm8(z[g]);
    }
    float res[16];
    for (int t = 0; t < num_a_vectors; t++) {
        const __m256 v = _mm256_add_ps(_mm256_add_ps(_mm256_add_ps(acc[0][t], acc[1][t]), acc[2][t]), acc[3][t]);
        float e[8];
        _mm256_storeu_ps(e, v);
        float rr = 0.0F, ri = 0.0F;
        for (int j = 0; j < 4; j++) {
            rr += e[2 * j];
            ri += e[2 * j + 1];
        }
        res[2 * t] = rr;
        res[2 * t + 1] = ri;
    }
    {
        float e[8];
        _mm256_storeu_ps(e, z[0]);
        const float mm = sqrtf(e[0] * e[0] + e[1] * e[1]);
        pr = e[0] / mm;
        pi = e[1] / mm;
    }
    for (unsigned int n = sixteenth * 16; n < num_points; n++) {
        float wr, wi;
        cmul1(in_common[2 * n], in_common[2 * n + 1], pr, pi, &wr, &wi);
        float nr, ni;
        cmul1(pr, pi, inc_re, inc_im, &nr, &ni);
        pr = nr;
        pi = ni;
        for (int t = 0; t < num_a_vectors; t++) {
            const float c = in_a[(size_t)t * num_points + n];
            res[2 * t] += wr * c;
            res[2 * t + 1] += wi * c;
        }
    }
    for (int t = 0; t < 2 * num_a_vectors; t++) result[t] = res[t];
    phase[0] = pr;
    phase[1] = pi;
}

static inline int wrap_idx(int idx, unsigned int L)
{
    if (idx < 0) idx += (int)L * (abs(idx) / (int)L + 1);
    return idx % (int)L;
}

ORC_AVX_TARGET void orc_resampler_avx(float* out, const float* local_code, float rem_code_phase_chips, float code_phase_step_chips,
    const float* shifts_chips, unsigned int code_length_chips, int num_out_vectors, unsigned int num_points)
{
    const __m256 step = _mm256_set1_ps(code_phase_step_chips), rem = _mm256_set1_ps(rem_code_phase_chips);
    const __m256i iota = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    const __m256i L = _mm256_set1_epi32((int)code_length_chips), zero = _mm256_setzero_si256();
    const unsigned int n8 = num_points & ~7u;
    for (int t = 0; t < num_out_vectors; t++) {
        float* r = out + (size_t)t * num_points;
        const __m256 sh = _mm256_set1_ps(shifts_chips[t]);
        for (unsigned int n = 0; n < n8; n += 8) {
            const __m256 nf = _mm256_cvtepi32_ps(_mm256_add_epi32(_mm256_set1_epi32((int)n), iota));
            const __m256 v = _mm256_sub_ps(_mm256_add_ps(_mm256_mul_ps(step, nf), sh), rem);
            const __m256i idx = _mm256_cvttps_epi32(_mm256_floor_ps(v));
            const __m256i bad = _mm256_or_si256(_mm256_cmpgt_epi32(zero, idx), _mm256_cmpgt_epi32(idx, _mm256_sub_epi32(L, _mm256_set1_epi32(1))));
            if (_mm256_testz_si256(bad, bad)) {
                _mm256_storeu_ps(r + n, _mm256_i32gather_ps(local_code, idx, 4));
            } else {
                int tmp[8];
                _mm256_storeu_si256((__m256i*)tmp, idx);
                for (int j = 0; j < 8; j++) r[n + j] = local_code[wrap_idx(tmp[j], code_length_chips)];
            }
        }
        for (unsigned int n = n8; n < num_points; n++) {
            const int idx = (int)floor(code_phase_step_chips * (float)n + shifts_chips[t] - rem_code_phase_chips);
            r[n] = local_code[wrap_idx(idx, code_length_chips)];
        }
    }
}
