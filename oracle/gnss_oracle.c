/*
 * oracle/gnss_oracle.c — CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / the timed CPU baseline.  The product
 * (gnss_sim_receiver_amd, libgnsship.so) never links or calls it.
 *
 * Every function restates one reference function (ShingoNishimoto/gnss_sim_receiver, a GNSS-SDR
 * v0.0.19 fork; paths relative to its root) and cites the file:line it follows.  Arithmetic is
 * kept in the reference's types and order: float32 complex products written out as
 * (ac - bd, ad + bc), no FMA contraction (built with -ffp-contract=off, no -march), i.e. the
 * VOLK_GENERIC semantics selected by volk_gnsssdr_rank_archs.c.
 *
 * Pinning: the code generators, the code resampler, the sincos wipeoff
 * recurrence and index_max are checked bit-for-bit against the reference's own sources compiled
 * by oracle/Makefile into oracle/_ref/ (tests/test_oracle_ref.py) and against the committed
 * fixtures under tests/golden/.  The rotator dot-product header includes the Mako-generated
 * <volk_gnsssdr/volk_gnsssdr.h>, which this image cannot generate, so it is restated only.
 */
#include <complex.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAX_TAPS 8

/* ------------------------------------------------------------------------------------------ */
/* Code generators                                                                            */
/* ------------------------------------------------------------------------------------------ */

/* gps_l1_ca_code_gen_int — src/algorithms/libs/gps_sdr_signal_replica.cc:25-110 (G1/G2 LFSR,
 * G2 delays per IS-GPS-200 table at :41-51). */
static const int32_t GPS_G2_DELAYS[210] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470, 471, 472,
    473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862, 863, 950, 947, 948, 950, 67, 103, 91, 19, 679, 225, 625, 946, 638, 161, 1001, 554, 280, 710, 709, 775, 864, 558, 220, 397, 55,
    898, 759, 367, 299, 1018, 729, 695, 780, 801, 788, 732, 34, 320, 327, 389, 407, 525, 405, 221, 761, 260, 326, 955, 653, 699, 422, 188,
    438, 959, 539, 879, 677, 586, 153, 792, 814, 446, 264, 1015, 278, 536, 819, 156, 957, 159, 712, 885, 461, 248, 713, 126, 807, 279, 122,
    197, 693, 632, 771, 467, 647, 203, 145, 175, 52, 21, 237, 235, 886, 657, 634, 762,
    355, 1012, 176, 603, 130, 359, 595, 68, 386, 797, 456, 499, 883, 307, 127, 211, 121, 118, 163, 628, 853, 484, 289, 811, 202,
    1021, 463, 568, 904, 670, 230, 911, 684, 309, 644, 932, 12, 314, 891, 212, 185, 675, 503, 150, 395, 345, 846, 798, 992, 357, 995, 877,
    112, 144, 476, 193, 109, 445, 291, 87, 399, 292, 901, 339, 208, 711, 189, 263, 537, 663, 942, 173, 900, 30, 500, 935, 556, 373, 85,
    652, 310};

int orc_gps_l1_ca_code_gen_int(int32_t* dest, int32_t prn, uint32_t chip_shift)
{
    enum { L = 1023 };
    unsigned char g1[L], g2[L];
    unsigned char r1[10], r2[10];
    const int32_t prn_idx = prn - 1;
    if (prn_idx < 0 || prn_idx > 210) return -1; /* reference returns silently (:66-69) */
    for (int i = 0; i < 10; i++) r1[i] = r2[i] = 1;
    for (int i = 0; i < L; i++) {
        g1[i] = r1[0];
        g2[i] = r2[0];
        const unsigned char f1 = r1[7] ^ r1[0];
        const unsigned char f2 = r2[8] ^ r2[7] ^ r2[4] ^ r2[2] ^ r2[1] ^ r2[0];
        memmove(r1, r1 + 1, 9);
        memmove(r2, r2 + 1, 9);
        r1[9] = f1;
        r2[9] = f2;
    }
    uint32_t delay = (uint32_t)(L - GPS_G2_DELAYS[prn_idx]);
    delay = (delay + chip_shift) % L;
    for (uint32_t i = 0; i < L; i++) {
        dest[i] = (g1[(i + chip_shift) % L] ^ g2[delay]) ? 1 : -1;
        delay = (delay + 1) % L;
    }
    return 0;
}

/* gps_l1_ca_code_gen_float — gps_sdr_signal_replica.cc:113-124 */
int orc_gps_l1_ca_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift)
{
    int32_t tmp[1023];
    if (orc_gps_l1_ca_code_gen_int(tmp, prn, chip_shift)) return -1;
    for (int i = 0; i < 1023; i++) dest[i] = (float)tmp[i];
    return 0;
}

/* Sampled complex replica, code in the IMAGINARY part:
 * gps_l1_ca_code_gen_complex (:127-138) + gps_l1_ca_code_gen_complex_sampled (:145-185).
 * dest: samplesPerCode interleaved (re, im) floats.  Returns samplesPerCode. */
int orc_gps_l1_ca_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t sampling_freq, uint32_t chip_shift)
{
    const int32_t code_freq_basis = 1023000, code_length = 1023;
    const float tc = 1.0F / (float)code_freq_basis;
    const int32_t samples_per_code = (int32_t)((double)sampling_freq / ((double)code_freq_basis / (double)code_length));
    const float ts = 1.0F / (float)sampling_freq;
    int32_t aux_code[1023];
    if (orc_gps_l1_ca_code_gen_int(aux_code, (int32_t)prn, chip_shift)) return -1;
    for (int32_t i = 0; i < samples_per_code; i++) {
        const float aux = (ts * ((float)i + 1)) / tc;
        const int32_t idx = (int32_t)((int64_t)(aux + 1)) - 1; /* AUX_CEIL (:23) */
        const int32_t k = (i == samples_per_code - 1) ? code_length - 1 : idx;
        dest[2 * i] = 0.0F;
        dest[2 * i + 1] = (float)aux_code[k];
    }
    return samples_per_code;
}

/* beidou_b1i_code_gen_int — src/algorithms/libs/beidou_b1i_signal_replica.cc:26-110 */
static const int32_t B1I_PH1[63] = {1, 1, 1, 1, 1, 1, 1, 1, 2, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 6, 6, 6, 6, 8, 8, 8, 9, 9, 10, 2, 3, 3, 3, 3, 3, 4, 4, 5, 5, 5, 5, 6, 8, 9, 9, 3, 5, 7, 4, 4, 5, 5, 5, 5, 6};
static const int32_t B1I_PH2[63] = {3, 4, 5, 6, 8, 9, 10, 11, 7, 4, 5, 6, 8, 9, 10, 11, 5, 6, 8, 9, 10, 11, 6, 8, 9, 10, 11, 8, 9, 10, 11, 9, 10, 11, 10, 11, 11, 7, 4, 6, 8, 10, 11, 5, 9, 6, 8, 10, 11, 9, 9, 10, 11, 7, 7, 9, 5, 9, 6, 8, 10, 11, 9};
static const int32_t B1I_PH3[63] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3};

int orc_beidou_b1i_code_gen_int(int32_t* dest, int32_t prn, uint32_t chip_shift)
{
    enum { L = 2046 };
    unsigned char g1[L], g2[L];
    unsigned char r1[11], r2[11];
    const int32_t prn_idx = prn - 1;
    if (prn_idx < 0 || prn_idx > 62) return -1;
    /* std::bitset<11>(std::string("01010101010")): bit 0 is the LAST character. */
    static const char init[] = "01010101010";
    for (int b = 0; b < 11; b++) r1[b] = r2[b] = (unsigned char)(init[10 - b] == '1');
    for (int i = 0; i < L; i++) {
        g1[i] = r1[0];
        unsigned char v = r2[11 - B1I_PH1[prn_idx]] ^ r2[11 - B1I_PH2[prn_idx]];
        if (B1I_PH3[prn_idx]) v ^= r2[11 - B1I_PH3[prn_idx]];
        g2[i] = v;
        const unsigned char f1 = r1[0] ^ r1[1] ^ r1[2] ^ r1[3] ^ r1[4] ^ r1[10];
        const unsigned char f2 = r2[0] ^ r2[2] ^ r2[3] ^ r2[6] ^ r2[7] ^ r2[8] ^ r2[9] ^ r2[10];
        memmove(r1, r1 + 1, 10);
        memmove(r2, r2 + 1, 10);
        r1[10] = f1;
        r2[10] = f2;
    }
    uint32_t delay = (L + chip_shift) % L;
    for (uint32_t i = 0; i < L; i++) {
        dest[i] = (g1[(i + chip_shift) % L] ^ g2[delay]) ? 1 : -1;
        delay = (delay + 1) % L;
    }
    return 0;
}

/* beidou_b1i_code_gen_float — beidou_b1i_signal_replica.cc:113-124 */
int orc_beidou_b1i_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift)
{
    int32_t tmp[2046];
    if (orc_beidou_b1i_code_gen_int(tmp, prn, chip_shift)) return -1;
    for (int i = 0; i < 2046; i++) dest[i] = (float)tmp[i];
    return 0;
}

/* beidou_b1i_code_gen_complex_sampled — :142-180 (code in the REAL part). */
int orc_beidou_b1i_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t sampling_freq, uint32_t chip_shift)
{
    const int32_t code_freq_basis = 2046000, code_length = 2046;
    const float tc = (float)(1.0 / (double)(float)code_freq_basis); /* double division (:146) */
    const int32_t samples_per_code = (int32_t)((double)sampling_freq / ((double)code_freq_basis / (double)code_length));
    const float ts = 1.0F / (float)sampling_freq;
    int32_t aux_code[2046];
    if (orc_beidou_b1i_code_gen_int(aux_code, (int32_t)prn, chip_shift)) return -1;
    for (int32_t i = 0; i < samples_per_code; i++) {
        const float aux = (ts * ((float)i + 1)) / tc;
        const int32_t idx = (int32_t)((int64_t)(aux + 1)) - 1;
        const int32_t k = (i == samples_per_code - 1) ? code_length - 1 : idx;
        dest[2 * i] = (float)aux_code[k];
        dest[2 * i + 1] = 0.0F;
    }
    return samples_per_code;
}

/* resampler(span<const float>, span<float>, fs_in, fs_out) — src/algorithms/libs/gnss_signal_replica.cc:257-272
 * with AUX_CEIL2(x) = (int32)(int64)(x + 1) (:25). */
void orc_code_resampler(float* dest, uint32_t dest_size, const float* from, uint32_t from_size, float fs_in, float fs_out)
{
    const float t_out = 1.0F / fs_out;
    for (uint32_t i = 0; i + 1 < dest_size; i++) {
        const float aux = (t_out * ((float)i + 1.0F)) * fs_in;
        const uint32_t idx = (uint32_t)((int32_t)(int64_t)(aux + 1) - 1);
        dest[i] = from[idx];
    }
    dest[dest_size - 1] = from[from_size - 1];
}

/* galileo_e1_code_gen_float_sampled without the secondary code — galileo_e1_signal_replica.cc:143-204,
 * from the 4092 primary chips (galileo_e1_code_gen_int output).  kind: 1 = "1B", 2 = "1C".
 * Returns samples per code, or -1 on bad arguments. */
int orc_galileo_e1_code_gen_float_sampled(float* dest, const int32_t* chips, int kind, int cboc, int32_t sampling_freq, uint32_t chip_shift)
{
    const int32_t code_freq_basis = 1023000;
    const int32_t spc = cboc ? 12 : 2;
    const uint32_t code_length = (uint32_t)spc * 4092U;
    uint32_t spcode = (uint32_t)((double)sampling_freq / ((double)code_freq_basis / 4092));
    const uint32_t delay = ((uint32_t)((int32_t)4092 - (int32_t)chip_shift) % (uint32_t)4092) * spcode / 4092U;
    if (spcode < 1) return -1;
    float* sig = (float*)malloc(sizeof(float) * code_length);
    if (!sig) return -1;
    const float alpha = sqrtf(10.0F / 11.0F), beta = sqrtf(1.0F / 11.0F);
    for (uint32_t i = 0; i < 4092U; i++) {
        for (int32_t j = 0; j < spc; j++) {
            const int32_t s11 = (j < spc / 2) ? chips[i] : -chips[i];
            if (cboc) {
                const int32_t s61 = (j % 2 == 0) ? chips[i] : -chips[i];
                sig[i * spc + j] = (kind == 1) ? alpha * (float)s11 + beta * (float)s61 : alpha * (float)s11 - beta * (float)s61;
            } else {
                sig[i * spc + j] = (float)s11;
            }
        }
    }
    float* src = sig;
    float* res = NULL;
    uint32_t n = code_length;
    if (sampling_freq != spc * code_freq_basis) {
        res = (float*)malloc(sizeof(float) * spcode);
        if (!res) {
            free(sig);
            return -1;
        }
        orc_code_resampler(res, spcode, sig, code_length, (float)(spc * code_freq_basis), (float)sampling_freq);
        src = res;
        n = spcode;
    }
    for (uint32_t i = 0; i < spcode && i < n; i++) dest[(i + delay) % spcode] = src[i];
    free(sig);
    free(res);
    return (int)spcode;
}

/* ------------------------------------------------------------------------------------------ */
/* Tracking correlator                                                                        */
/* ------------------------------------------------------------------------------------------ */

/* volk_gnsssdr_32f_xn_resampler_32f_xn_generic —
 * src/algorithms/libs/volk_gnsssdr_module/volk_gnsssdr/kernels/volk_gnsssdr/
 *   volk_gnsssdr_32f_xn_resampler_32f_xn.h:63-80.  out is [num_out_vectors][num_points]. */
void orc_resampler_generic(float* out, const float* local_code, float rem_code_phase_chips, float code_phase_step_chips,
    const float* shifts_chips, unsigned int code_length_chips, int num_out_vectors, unsigned int num_points)
{
    for (int t = 0; t < num_out_vectors; t++) {
        float* r = out + (size_t)t * num_points;
        for (unsigned int n = 0; n < num_points; n++) {
            int idx = (int)floor(code_phase_step_chips * (float)n + shifts_chips[t] - rem_code_phase_chips);
            if (idx < 0) idx += (int)code_length_chips * (abs(idx) / code_length_chips + 1);
            idx = idx % code_length_chips;
            r[n] = local_code[idx];
        }
    }
}

/* volk_gnsssdr_32f_xn_high_dynamics_resampler_32f_xn_generic — …_high_dynamics_resampler_32f_xn.h:67-91.
 * Tap 0 carries the rate term; taps 1.. are circular shifts of tap 0 by round(Δshift/step). */
void orc_high_dynamics_resampler_generic(float* out, const float* local_code, float rem_code_phase_chips, float code_phase_step_chips,
    float code_phase_rate_step_chips, const float* shifts_chips, unsigned int code_length_chips, int num_out_vectors, unsigned int num_points)
{
    for (unsigned int n = 0; n < num_points; n++) {
        int idx = (int)floor(code_phase_step_chips * (float)n + code_phase_rate_step_chips * (float)(n * n) + shifts_chips[0] - rem_code_phase_chips);
        if (idx < 0) idx += (int)code_length_chips * (abs(idx) / code_length_chips + 1);
        idx = idx % code_length_chips;
        out[n] = local_code[idx];
    }
    unsigned int shift_samples = 0;
    for (int t = 1; t < num_out_vectors; t++) {
        shift_samples += (int)round((shifts_chips[t] - shifts_chips[t - 1]) / code_phase_step_chips);
        float* r = out + (size_t)t * num_points;
        memcpy(r, out + shift_samples, (num_points - shift_samples) * sizeof(float));
        memcpy(r + (num_points - shift_samples), out, shift_samples * sizeof(float));
    }
}

/* (a+jb)(c+jd) in float, written out (no FMA: -ffp-contract=off). */
static inline void cmul(float a, float b, float c, float d, float* re, float* im)
{
    *re = a * c - b * d;
    *im = a * d + b * c;
}

/* volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_generic —
 *   volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:66-98.
 * result[2*t..] += (in[n]·phase)·a_t[n]; phase *= phase_inc; |phase| renormalised when n%256 == 0
 * AFTER it was used for sample n.  phase (2 floats) is updated in place, like the reference. */
void orc_rotator_dot_prod_generic(float* result, const float* in_common, float inc_re, float inc_im, float* phase,
    const float* in_a, int num_a_vectors, unsigned int num_points)
{
    float pr = phase[0], pi = phase[1];
    float acc[2 * ORC_MAX_TAPS];
    for (int t = 0; t < 2 * num_a_vectors; t++) acc[t] = 0.0F;
    for (unsigned int n = 0; n < num_points; n++) {
        float tr, ti;
        cmul(in_common[2 * n], in_common[2 * n + 1], pr, pi, &tr, &ti);
        if (n % 256 == 0) {
            const float m = hypotf(pr, pi); /* std::abs(complex<float>) → cabsf → hypotf */
            pr /= m;
            pi /= m;
        }
        float nr, ni;
        cmul(pr, pi, inc_re, inc_im, &nr, &ni);
        pr = nr;
        pi = ni;
        for (int t = 0; t < num_a_vectors; t++) {
            const float c = in_a[(size_t)t * num_points + n];
            acc[2 * t] += tr * c;
            acc[2 * t + 1] += ti * c;
        }
    }
    for (int t = 0; t < 2 * num_a_vectors; t++) result[t] = acc[t];
    phase[0] = pr;
    phase[1] = pi;
}

/* Test-only variant of orc_rotator_dot_prod_generic: the SAME float products (x·phase in float,
 * same phasor recursion and renormalisation), accumulated in double.  Separates the reference's
 * serial-float-sum rounding (≈ √N half-ulps of the accumulator, ~1e-5 relative at N ≥ 1e5) from
 * everything else when judging a parallel reduction at long integrations. */
static void orc_rotator_dot_prod_acc64(float* result, const float* in_common, float inc_re, float inc_im, float* phase,
    const float* in_a, int num_a_vectors, unsigned int num_points)
{
    float pr = phase[0], pi = phase[1];
    double acc[2 * ORC_MAX_TAPS];
    for (int t = 0; t < 2 * num_a_vectors; t++) acc[t] = 0.0;
    for (unsigned int n = 0; n < num_points; n++) {
        float tr, ti;
        cmul(in_common[2 * n], in_common[2 * n + 1], pr, pi, &tr, &ti);
        if (n % 256 == 0) {
            const float m = hypotf(pr, pi);
            pr /= m;
            pi /= m;
        }
        float nr, ni;
        cmul(pr, pi, inc_re, inc_im, &nr, &ni);
        pr = nr;
        pi = ni;
        for (int t = 0; t < num_a_vectors; t++) {
            const float c = in_a[(size_t)t * num_points + n];
            acc[2 * t] += (double)(tr * c);
            acc[2 * t + 1] += (double)(ti * c);
        }
    }
    for (int t = 0; t < 2 * num_a_vectors; t++) result[t] = (float)acc[t];
    phase[0] = pr;
    phase[1] = pi;
}

/* volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_u_avx / _a_avx —
 *   volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:155-316 (a_avx :322-, same arithmetic), with
 *   _mm256_complexmul_ps / _mm256_complexnormalise_ps of volk_gnsssdr_avx_intrinsics.h:20-29,56-63.
 * The variant volk_gnsssdr dispatches on any AVX host (the only non-generic x86 variants of this
 * kernel).  Restated lane by lane in scalar C: every AVX op here is an IEEE single op (mul, add/sub
 * of addsub, hadd = re²+im², sqrt_ps, div_ps), so the scalar form is bit-identical.
 *   - 16 phasors z_l = phase·inc^l (generic chain, :204-208), advanced by dz = normalise(inc^16)
 *     (four complex<float> squarings, :215-225) once per 16-sample iteration;
 *   - the phasors are renormalised after the update of iterations m ≡ 0 (mod 64) (:265-272);
 *   - accumulators: 4 registers × 4 complex lanes per tap (sample 16m + 4g + j → register g, lane
 *     j), summed at the end as ((r0 + r1) + r2) + r3, then lanes 0..3 serially (:276-290);
 *   - the N mod 16 tail continues serially from normalise(z_0) (:292-304).
 * accum_f64: test-only, the same float products summed in double. */
static void orc_rotator_dot_prod_avx_impl(float* result, const float* in_common, float inc_re, float inc_im, float* phase,
    const float* in_a, int num_a_vectors, unsigned int num_points, int accum_f64)
{
    const unsigned int sixteenth = num_points / 16;
    float zr[16], zi[16];
    float pr = phase[0], pi = phase[1];
    for (int l = 0; l < 16; l++) {
        zr[l] = pr;
        zi[l] = pi;
        float nr, ni;
        cmul(pr, pi, inc_re, inc_im, &nr, &ni);
        pr = nr;
        pi = ni;
    }
    float dr = inc_re, di = inc_im;
    for (int k = 0; k < 4; k++) {
        float nr, ni;
        cmul(dr, di, dr, di, &nr, &ni);
        dr = nr;
        di = ni;
    }
    {
        const float m = sqrtf(dr * dr + di * di);
        dr = dr / m;
        di = di / m;
    }
    float acc[4][ORC_MAX_TAPS][8];
    double acc64[2 * ORC_MAX_TAPS];
    memset(acc, 0, sizeof(acc));
    for (int t = 0; t < 2 * num_a_vectors; t++) acc64[t] = 0.0;
    for (unsigned int m = 0; m < sixteenth; m++) {
        float ar[16], ai[16];
        for (int l = 0; l < 16; l++) {
            const unsigned int n = 16 * m + l;
            cmul(in_common[2 * n], in_common[2 * n + 1], zr[l], zi[l], &ar[l], &ai[l]);
            float nr, ni;
            cmul(zr[l], zi[l], dr, di, &nr, &ni);
            zr[l] = nr;
            zi[l] = ni;
        }
        for (int t = 0; t < num_a_vectors; t++)
            for (int l = 0; l < 16; l++) {
                const float c = in_a[(size_t)t * num_points + 16 * m + l];
                if (accum_f64) {
                    acc64[2 * t] += (double)(ar[l] * c);
                    acc64[2 * t + 1] += (double)(ai[l] * c);
                } else {
                    acc[l / 4][t][2 * (l % 4)] += ar[l] * c;
                    acc[l / 4][t][2 * (l % 4) + 1] += ai[l] * c;
                }
            }
        if (m % 64 == 0)
            for (int l = 0; l < 16; l++) {
                const float mm = sqrtf(zr[l] * zr[l] + zi[l] * zi[l]);
                zr[l] = zr[l] / mm;
                zi[l] = zi[l] / mm;
            }
    }
    float res[2 * ORC_MAX_TAPS];
    for (int t = 0; t < num_a_vectors; t++) {
        float v[8];
        for (int e = 0; e < 8; e++) v[e] = ((acc[0][t][e] + acc[1][t][e]) + acc[2][t][e]) + acc[3][t][e];
        float rr = 0.0F, ri = 0.0F;
        for (int j = 0; j < 4; j++) {
            rr += v[2 * j];
            ri += v[2 * j + 1];
        }
        res[2 * t] = rr;
        res[2 * t + 1] = ri;
    }
    {
        const float mm = sqrtf(zr[0] * zr[0] + zi[0] * zi[0]);
        pr = zr[0] / mm;
        pi = zi[0] / mm;
    }
    for (unsigned int n = sixteenth * 16; n < num_points; n++) {
        float wr, wi;
        cmul(in_common[2 * n], in_common[2 * n + 1], pr, pi, &wr, &wi);
        float nr, ni;
        cmul(pr, pi, inc_re, inc_im, &nr, &ni);
        pr = nr;
        pi = ni;
        for (int t = 0; t < num_a_vectors; t++) {
            const float c = in_a[(size_t)t * num_points + n];
            if (accum_f64) {
                acc64[2 * t] += (double)(wr * c);
                acc64[2 * t + 1] += (double)(wi * c);
            } else {
                res[2 * t] += wr * c;
                res[2 * t + 1] += wi * c;
            }
        }
    }
    for (int t = 0; t < 2 * num_a_vectors; t++) result[t] = accum_f64 ? (float)acc64[t] : res[t];
    phase[0] = pr;
    phase[1] = pi;
}

void orc_rotator_dot_prod_avx(float* result, const float* in_common, float inc_re, float inc_im, float* phase,
    const float* in_a, int num_a_vectors, unsigned int num_points)
{
    orc_rotator_dot_prod_avx_impl(result, in_common, inc_re, inc_im, phase, in_a, num_a_vectors, num_points, 0);
}

/* volk_gnsssdr_32fc_32f_high_dynamic_rotator_dot_prod_32fc_xn_generic —
 *   volk_gnsssdr_32fc_32f_high_dynamic_rotator_dot_prod_32fc_xn.h:68-110 (non-Windows branch,
 *   cpowf; note (n*n) is unsigned int and wraps for n >= 65536, as in the reference). */
static void orc_high_dynamic_rotator_dot_prod_impl(float* result, const float* in_common, float inc_re, float inc_im,
    float rate_re, float rate_im, float* phase, const float* in_a, int num_a_vectors, unsigned int num_points, int accum_f64);

void orc_high_dynamic_rotator_dot_prod_generic(float* result, const float* in_common, float inc_re, float inc_im,
    float rate_re, float rate_im, float* phase, const float* in_a, int num_a_vectors, unsigned int num_points)
{
    orc_high_dynamic_rotator_dot_prod_impl(result, in_common, inc_re, inc_im, rate_re, rate_im, phase, in_a, num_a_vectors, num_points, 0);
}

/* accum_f64 = 1: test-only variant, the same float products summed in double (as
 * orc_rotator_dot_prod_acc64). */
static void orc_high_dynamic_rotator_dot_prod_impl(float* result, const float* in_common, float inc_re, float inc_im,
    float rate_re, float rate_im, float* phase, const float* in_a, int num_a_vectors, unsigned int num_points, int accum_f64)
{
    double acc64[2 * ORC_MAX_TAPS];
    for (int t = 0; t < 2 * num_a_vectors; t++) acc64[t] = 0.0;
    float complex ph = phase[0] + phase[1] * I;
    float complex ph_doppler = ph;
    const float complex inc = inc_re + inc_im * I;
    const float complex inc_rate = rate_re + rate_im * I;
    float acc[2 * ORC_MAX_TAPS];
    for (int t = 0; t < 2 * num_a_vectors; t++) acc[t] = 0.0F;
    for (unsigned int n = 0; n < num_points; n++) {
        if (n % 256 == 0) {
            const float m = hypotf(crealf(ph), cimagf(ph));
            ph = crealf(ph) / m + (cimagf(ph) / m) * I;
        }
        float tr, ti;
        cmul(in_common[2 * n], in_common[2 * n + 1], crealf(ph), cimagf(ph), &tr, &ti);
        float dr, di;
        cmul(crealf(ph_doppler), cimagf(ph_doppler), crealf(inc), cimagf(inc), &dr, &di);
        ph_doppler = dr + di * I;
        float complex pdr = cpowf(inc_rate, (float)(n * n) + 0.0F * I);
        const float m2 = hypotf(crealf(pdr), cimagf(pdr));
        pdr = crealf(pdr) / m2 + (cimagf(pdr) / m2) * I;
        float qr, qi;
        cmul(crealf(ph_doppler), cimagf(ph_doppler), crealf(pdr), cimagf(pdr), &qr, &qi);
        ph = qr + qi * I;
        for (int t = 0; t < num_a_vectors; t++) {
            const float c = in_a[(size_t)t * num_points + n];
            if (accum_f64) {
                acc64[2 * t] += (double)(tr * c);
                acc64[2 * t + 1] += (double)(ti * c);
            } else {
                acc[2 * t] += tr * c;
                acc[2 * t + 1] += ti * c;
            }
        }
    }
    for (int t = 0; t < 2 * num_a_vectors; t++) result[t] = accum_f64 ? (float)acc64[t] : acc[t];
    phase[0] = crealf(ph);
    phase[1] = cimagf(ph);
}

/* Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler —
 *   src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.cc:103-126 (+update_local_code :75-100).
 * phase_offset = (cos rem, −sin rem); phase_inc = exp(−j·step) (std::exp of complex<float>, i.e.
 * glibc cexpf → (cosf(−step), sinf(−step))).  scratch: n_taps*signal_length floats or NULL. */
static int orc_multicorrelator_impl(float* corr_out, const float* sig_in, const float* local_code, int code_length_chips,
    const float* shifts_chips, int n_correlators, int flags, float rem_carrier_phase_in_rad, float phase_step_rad,
    float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* scratch, int accum_f64);

/* accum_f64: test-only double accumulation of the same float products. */
int orc_multicorrelator_real_codes_ex(float* corr_out, const float* sig_in, const float* local_code, int code_length_chips,
    const float* shifts_chips, int n_correlators, int flags, float rem_carrier_phase_in_rad, float phase_step_rad,
    float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* scratch, int accum_f64)
{
    return orc_multicorrelator_impl(corr_out, sig_in, local_code, code_length_chips, shifts_chips, n_correlators, flags,
        rem_carrier_phase_in_rad, phase_step_rad, phase_rate_step_rad, rem_code_phase_chips, code_phase_step_chips,
        code_phase_rate_step_chips, signal_length_samples, scratch, accum_f64);
}

/* flags as gnsship_corr_job::flags: bit0 high_dyn, bit1 AVX rotator variant. */
int orc_multicorrelator_real_codes(float* corr_out, const float* sig_in, const float* local_code, int code_length_chips,
    const float* shifts_chips, int n_correlators, int flags, float rem_carrier_phase_in_rad, float phase_step_rad,
    float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* scratch)
{
    return orc_multicorrelator_impl(corr_out, sig_in, local_code, code_length_chips, shifts_chips, n_correlators, flags,
        rem_carrier_phase_in_rad, phase_step_rad, phase_rate_step_rad, rem_code_phase_chips, code_phase_step_chips,
        code_phase_rate_step_chips, signal_length_samples, scratch, 0);
}

/* The AVX restatement (oracle/avx_port.c) for the timed CPU baseline: bit-identical to the scalar
 * restatement, selected by orc_set_simd(1) (off by default; tests pin the two against each other). */
int orc_simd_available(void);
void orc_rotator_dot_prod_avx_vec(float* result, const float* in_common, float inc_re, float inc_im, float* phase,
    const float* in_a, int num_a_vectors, unsigned int num_points);
void orc_resampler_avx(float* out, const float* local_code, float rem_code_phase_chips, float code_phase_step_chips,
    const float* shifts_chips, unsigned int code_length_chips, int num_out_vectors, unsigned int num_points);
static int g_simd = 0;
int orc_set_simd(int on)
{
    g_simd = (on && orc_simd_available()) ? 1 : 0;
    return g_simd;
}

/* flags: bit0 high-dynamics resampler/rotator, bit1 the AVX rotator variant (the job flags of
 * gnsship_corr_job; high_dyn has only generic variants, so bit1 is ignored with bit0). */
static int orc_multicorrelator_impl(float* corr_out, const float* sig_in, const float* local_code, int code_length_chips,
    const float* shifts_chips, int n_correlators, int flags, float rem_carrier_phase_in_rad, float phase_step_rad,
    float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* scratch, int accum_f64)
{
    const int high_dyn = flags & 1;
    if (n_correlators < 1 || n_correlators > ORC_MAX_TAPS || signal_length_samples < 0) return -1;
    if (high_dyn) { /* the reference's memcpy lengths go negative outside [0, N]: refused, not run */
        unsigned int s = 0;
        for (int t = 1; t < n_correlators; t++) {
            s += (int)round((shifts_chips[t] - shifts_chips[t - 1]) / code_phase_step_chips);
            if (s > (unsigned int)signal_length_samples) return -1;
        }
    }
    float* codes = scratch;
    int own = 0;
    if (!codes) {
        codes = (float*)malloc((size_t)n_correlators * (size_t)(signal_length_samples > 0 ? signal_length_samples : 1) * sizeof(float));
        if (!codes) return -2;
        own = 1;
    }
    if (high_dyn)
        orc_high_dynamics_resampler_generic(codes, local_code, rem_code_phase_chips, code_phase_step_chips, code_phase_rate_step_chips,
            shifts_chips, (unsigned)code_length_chips, n_correlators, (unsigned)signal_length_samples);
    else if (g_simd && (flags & 2))
        orc_resampler_avx(codes, local_code, rem_code_phase_chips, code_phase_step_chips, shifts_chips, (unsigned)code_length_chips,
            n_correlators, (unsigned)signal_length_samples);
    else
        orc_resampler_generic(codes, local_code, rem_code_phase_chips, code_phase_step_chips, shifts_chips, (unsigned)code_length_chips,
            n_correlators, (unsigned)signal_length_samples);
    float phase[2] = {cosf(rem_carrier_phase_in_rad), -sinf(rem_carrier_phase_in_rad)};
    float inc_re = cosf(-phase_step_rad), inc_im = sinf(-phase_step_rad);
    if (high_dyn) {
        const float rr = cosf(-phase_rate_step_rad), ri = sinf(-phase_rate_step_rad);
        orc_high_dynamic_rotator_dot_prod_impl(corr_out, sig_in, inc_re, inc_im, rr, ri, phase, codes, n_correlators,
            (unsigned)signal_length_samples, accum_f64);
    } else if ((flags & 2) && g_simd && !accum_f64) {
        orc_rotator_dot_prod_avx_vec(corr_out, sig_in, inc_re, inc_im, phase, codes, n_correlators, (unsigned)signal_length_samples);
    } else if (flags & 2) {
        orc_rotator_dot_prod_avx_impl(corr_out, sig_in, inc_re, inc_im, phase, codes, n_correlators, (unsigned)signal_length_samples,
            accum_f64);
    } else if (accum_f64) {
        orc_rotator_dot_prod_acc64(corr_out, sig_in, inc_re, inc_im, phase, codes, n_correlators, (unsigned)signal_length_samples);
    } else {
        orc_rotator_dot_prod_generic(corr_out, sig_in, inc_re, inc_im, phase, codes, n_correlators, (unsigned)signal_length_samples);
    }
    if (own) free(codes);
    return 0;
}

/* ---- Batched jobs (same 80-byte layout as gnsship_corr_job in include/gnsship.h) ---------- */
typedef struct orc_job {
    int64_t sample_offset;
    int32_t n_samples;
    int32_t code_id;
    int32_t n_taps;
    int32_t flags;
    float rem_carrier_phase_rad, phase_step_rad, phase_rate_step_rad;
    float rem_code_phase_chips, code_phase_step_chips, code_phase_rate_step_chips;
    float shifts_chips[ORC_MAX_TAPS];
} orc_job;

typedef struct {
    const float* samples;
    const orc_job* jobs;
    const float* const* codes;
    const int* code_lengths;
    float* out;
    int j0, j1;
    int max_n;
    int accum_f64;
} orc_batch_arg;

static void* orc_batch_worker(void* p)
{
    orc_batch_arg* a = (orc_batch_arg*)p;
    float* scratch = (float*)malloc((size_t)ORC_MAX_TAPS * (size_t)(a->max_n > 0 ? a->max_n : 1) * sizeof(float));
    for (int j = a->j0; j < a->j1; j++) {
        const orc_job* jb = &a->jobs[j];
        orc_multicorrelator_impl(a->out + (size_t)j * 2 * ORC_MAX_TAPS, a->samples + 2 * jb->sample_offset, a->codes[jb->code_id],
            a->code_lengths[jb->code_id], jb->shifts_chips, jb->n_taps, jb->flags & 7, jb->rem_carrier_phase_rad, jb->phase_step_rad,
            jb->phase_rate_step_rad, jb->rem_code_phase_chips, jb->code_phase_step_chips, jb->code_phase_rate_step_chips, jb->n_samples,
            scratch, a->accum_f64);
    }
    free(scratch);
    return NULL;
}

/* Run n_jobs correlations over host CF32 samples with n_threads pthreads (GNU Radio runs one
 * thread per channel block; here jobs are split in contiguous ranges).  out: n_jobs × 8 taps. */
int orc_corr_batch_ex(const float* samples, const orc_job* jobs, int n_jobs, const float* const* codes, const int* code_lengths,
    float* out, int n_threads, int accum_f64);

int orc_corr_batch(const float* samples, const orc_job* jobs, int n_jobs, const float* const* codes, const int* code_lengths,
    float* out, int n_threads)
{
    return orc_corr_batch_ex(samples, jobs, n_jobs, codes, code_lengths, out, n_threads, 0);
}

/* accum_f64 = 1: the test-only double-accumulation variant (orc_rotator_dot_prod_acc64). */
int orc_corr_batch_ex(const float* samples, const orc_job* jobs, int n_jobs, const float* const* codes, const int* code_lengths,
    float* out, int n_threads, int accum_f64)
{
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    int max_n = 1;
    for (int j = 0; j < n_jobs; j++)
        if (jobs[j].n_samples > max_n) max_n = jobs[j].n_samples;
    memset(out, 0, (size_t)n_jobs * 2 * ORC_MAX_TAPS * sizeof(float));
    pthread_t th[256];
    orc_batch_arg args[256];
    int started = 0;
    for (int t = 0; t < n_threads; t++) {
        args[t].samples = samples;
        args[t].jobs = jobs;
        args[t].codes = codes;
        args[t].code_lengths = code_lengths;
        args[t].out = out;
        args[t].j0 = (int)((int64_t)n_jobs * t / n_threads);
        args[t].j1 = (int)((int64_t)n_jobs * (t + 1) / n_threads);
        args[t].max_n = max_n;
        args[t].accum_f64 = accum_f64;
        if (n_threads == 1) {
            orc_batch_worker(&args[t]);
        } else if (pthread_create(&th[t], NULL, orc_batch_worker, &args[t]) == 0) {
            started++;
        } else {
            orc_batch_worker(&args[t]);
            th[t] = 0;
        }
    }
    if (n_threads > 1)
        for (int t = 0; t < n_threads; t++)
            if (th[t]) pthread_join(th[t], NULL);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Acquisition helpers                                                                        */
/* ------------------------------------------------------------------------------------------ */

/* volk_gnsssdr_s32f_sincos_32fc_generic — volk_gnsssdr_s32f_sincos_32fc.h:390-400:
 * out[i] = (cosf(phi), sinf(phi)), phi += phase_inc accumulated in float. */
void orc_sincos_generic(float* out, float phase_inc, float* phase, unsigned int num_points)
{
    float ph = *phase;
    for (unsigned int i = 0; i < num_points; i++) {
        out[2 * i] = cosf(ph);
        out[2 * i + 1] = sinf(ph);
        ph += phase_inc;
    }
    *phase = ph;
}

/* Phase sequence only (the float recurrence above without the trig), for device tables. */
void orc_sincos_phases(float* out_phase, float phase_inc, float phase0, unsigned int num_points)
{
    float ph = phase0;
    for (unsigned int i = 0; i < num_points; i++) {
        out_phase[i] = ph;
        ph += phase_inc;
    }
}

/* pcps_acquisition::update_local_carrier + update_grid_doppler_wipeoffs —
 *   pcps_acquisition.cc:232-245, :295-302.  table: n_bins × fft_size complex. */
void orc_doppler_wipeoff_grid(float* table, int n_bins, int fft_size, int doppler_max, int doppler_step, int doppler_center,
    int doppler_bias, int64_t fs)
{
    const float two_pi = (float)(2.0 * 3.141592653589793238462643383279502884197169399375105820974944592);
    for (int i = 0; i < n_bins; i++) {
        const int32_t doppler = -(int32_t)doppler_max + doppler_center + doppler_step * i;
        const float freq = (float)(doppler_bias + doppler);
        const float step = two_pi * freq / (float)fs;
        float ph = 0.0F;
        orc_sincos_generic(table + (size_t)2 * i * fft_size, -step, &ph, (unsigned)fft_size);
    }
}

/* volk_gnsssdr_32f_index_max_32u_generic — volk_gnsssdr_32f_index_max_32u.h:446-465
 * (first index of the strict maximum). */
uint32_t orc_index_max_generic(const float* src0, uint32_t num_points)
{
    uint32_t index = 0;
    if (num_points > 0) {
        float m = src0[0];
        for (uint32_t i = 1; i < num_points; ++i)
            if (src0[i] > m) {
                index = i;
                m = src0[i];
            }
    }
    return index;
}

/* std::accumulate(float*, float*, 0.0F) — serial float sum (pcps_acquisition.cc:518). */
float orc_sum_serial_f32(const float* x, uint32_t n)
{
    float s = 0.0F;
    for (uint32_t i = 0; i < n; i++) s += x[i];
    return s;
}

typedef struct orc_acq_stat {
    uint32_t doppler_index;
    uint32_t code_index;
    int32_t doppler_hz;
    float peak;
    float input_power; /* CFAR: input power; first_vs_second: the second peak */
    float test_statistic;
    double acq_delay_samples;
} orc_acq_stat;

/* max_to_input_power_statistic — pcps_acquisition.cc:496-528 (step one only), plus the
 * Gnss_Synchro fields written at :693-695.  grid: n_bins × n (magnitude grid rows). */
void orc_max_to_input_power_statistic(const float* grid, uint32_t n_bins, uint32_t n, int32_t doppler_max, int32_t doppler_step,
    int32_t doppler_center, uint32_t dwells, float samples_per_code, orc_acq_stat* st)
{
    float grid_maximum = 0.0F;
    uint32_t index_doppler = 0, index_time = 0;
    for (uint32_t i = 0; i < n_bins; i++) {
        const float* row = grid + (size_t)i * n;
        const uint32_t t = orc_index_max_generic(row, n);
        if (row[t] > grid_maximum) {
            grid_maximum = row[t];
            index_doppler = i;
            index_time = t;
        }
    }
    const uint32_t index_opp = (index_doppler + n_bins / 2) % n_bins;
    const float s = orc_sum_serial_f32(grid + (size_t)index_opp * n, n);
    const float input_power = (float)((double)(s / (float)(int32_t)n) / 2.0 / (double)dwells);
    st->doppler_index = index_doppler;
    st->code_index = index_time;
    st->doppler_hz = -(int32_t)doppler_max + doppler_center + doppler_step * (int32_t)index_doppler;
    st->peak = grid_maximum;
    st->input_power = input_power;
    st->test_statistic = grid_maximum / input_power;
    st->acq_delay_samples = (double)fmodf((float)index_time, samples_per_code);
}

/* first_vs_second_peak_statistic — pcps_acquisition.cc:531-597. */
void orc_first_vs_second_peak_statistic(const float* grid, uint32_t n_bins, uint32_t n, int32_t doppler_max, int32_t doppler_step,
    int32_t doppler_center, uint32_t samples_per_chip, float samples_per_code, orc_acq_stat* st)
{
    float first = 0.0F;
    uint32_t index_doppler = 0, index_time = 0;
    for (uint32_t i = 0; i < n_bins; i++) {
        const float* row = grid + (size_t)i * n;
        const uint32_t t = orc_index_max_generic(row, n);
        if (row[t] > first) {
            first = row[t];
            index_doppler = i;
            index_time = t;
        }
    }
    int32_t e1 = (int32_t)index_time - (int32_t)samples_per_chip;
    int32_t e2 = (int32_t)index_time + (int32_t)samples_per_chip;
    if (e1 < 0)
        e1 = (int32_t)n + e1;
    else if (e2 >= (int32_t)n)
        e2 = e2 - (int32_t)n;
    float* tmp = (float*)malloc((size_t)n * sizeof(float));
    memcpy(tmp, grid + (size_t)index_doppler * n, (size_t)n * sizeof(float));
    int32_t idx = e1;
    do {
        tmp[idx] = 0.0F;
        idx++;
        if (idx == (int32_t)n) idx = 0;
    } while (idx != e2);
    const uint32_t t2 = orc_index_max_generic(tmp, n);
    const float second = tmp[t2];
    free(tmp);
    st->doppler_index = index_doppler;
    st->code_index = index_time;
    st->doppler_hz = -(int32_t)doppler_max + doppler_center + doppler_step * (int32_t)index_doppler;
    st->peak = first;
    st->input_power = second;
    st->test_statistic = first / second;
    st->acq_delay_samples = (double)fmodf((float)index_time, samples_per_code);
}

/* complex<float> × complex<float> elementwise (volk_32fc_x2_multiply_32fc generic) and
 * |x|² (volk_32fc_magnitude_squared_32f generic); conj (volk_32fc_conjugate_32fc). */
void orc_cf32_multiply(float* out, const float* a, const float* b, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) cmul(a[2 * i], a[2 * i + 1], b[2 * i], b[2 * i + 1], &out[2 * i], &out[2 * i + 1]);
}

void orc_cf32_magnitude_squared(float* out, const float* a, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) out[i] = a[2 * i] * a[2 * i] + a[2 * i + 1] * a[2 * i + 1];
}

int orc_abi_version(void) { return 1; }

/* ---- acquisition resampler (gnss_flowgraph.cc:1070-1113) ------------------------------------
 * GNU Radio (absent here, version unpinned) restated from its published algorithm:
 * gr::filter::firdes::low_pass(gain, fs, cutoff, transition) with the default Hamming window —
 * compute_ntaps: (int)(53 · fs / (22 · transition)), forced odd; window w[n] = 0.54 − 0.46·cosf(2πn/M)
 * (fft::window::coswindow, M = ntaps − 1, float); windowed sinc h[n+M'] = sin(n·ω)/(nπ)·w (ω = 2π·
 * cutoff/fs, centre ω/π·w); DC gain normalised in double.  Returns ntaps (taps == NULL: count). */
int orc_firdes_low_pass(double gain, double fs, double cutoff, double transition, float* taps)
{
    int ntaps = (int)(53.0 * fs / (22.0 * transition));
    if (!(ntaps & 1)) ntaps += 1;
    if (!taps) return ntaps;
    const int half = (ntaps - 1) / 2;
    const float Mw = (float)(ntaps - 1);
    const double omega = 2.0 * M_PI * cutoff / fs;
    for (int i = 0; i < ntaps; i++) {
        const float w = 0.54F - 0.46F * cosf((float)((2.0 * M_PI * (double)i) / (double)Mw));
        const int n = i - half;
        taps[i] = (n == 0) ? (float)(omega / M_PI * (double)w) : (float)(sin((double)n * omega) / ((double)n * M_PI) * (double)w);
    }
    double dc = (double)taps[half];
    for (int n = 1; n <= half; n++) dc += (double)(2.0F * taps[half + n]);
    const double g = gain / dc;
    for (int i = 0; i < ntaps; i++) taps[i] = (float)((double)taps[i] * g);
    return ntaps;
}

/* gr::filter::fir_filter_ccf(decimation, taps) over CF32 input with ntaps − 1 history samples
 * (hist[0..ntaps−2], oldest first; updated in place): out[k] = volk_32fc_32f_dot_prod_32fc_generic
 * of x_ext[k·D .. k·D + ntaps − 1] with the reversed taps (serial float sums).  n_in % D == 0. */
void orc_fir_decimate(const float* in, int64_t n_in, float* hist, const float* taps, int ntaps, int decim, float* out)
{
    const int nh = ntaps - 1;
    const int64_t n_out = n_in / decim;
    for (int64_t k = 0; k < n_out; k++) {
        float re = 0.0F, im = 0.0F;
        for (int t = 0; t < ntaps; t++) {
            const int64_t g = k * decim + t - nh;
            const float* x = g < 0 ? &hist[2 * (nh + g)] : &in[2 * g];
            const float h = taps[ntaps - 1 - t];
            re += x[0] * h;
            im += x[1] * h;
        }
        out[2 * k] = re;
        out[2 * k + 1] = im;
    }
    /* history: the last nh samples of (hist ‖ in) */
    if (nh > 0) {
        float* tmp = (float*)malloc(sizeof(float) * 2 * (size_t)nh);
        for (int i = 0; i < nh; i++) {
            const int64_t g = n_in - nh + i;
            const float* x = g < 0 ? &hist[2 * (nh + g)] : &in[2 * g];
            tmp[2 * i] = x[0];
            tmp[2 * i + 1] = x[1];
        }
        memcpy(hist, tmp, sizeof(float) * 2 * (size_t)nh);
        free(tmp);
    }
}
