/* trk_oracle.c — CPU restatement of the DLL/PLL tracking loop.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the device-resident loop in
 * gnss_sim_receiver_amd/csrc/trk_kernel.hip.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  Pinned by the reference's own known-answer tests
 * (tracking_loop_filter_test.cc, discriminator_test.cc) in tests/test_oracle_trk.py.
 *
 * Follows, function by function (types as in the reference: float where it stores float):
 *   Tracking_loop_filter            src/algorithms/tracking/libs/tracking_loop_filter.cc:58-200
 *   Tracking_FLL_PLL_filter         tracking_FLL_PLL_filter.cc:23-110
 *   discriminators                  tracking_discriminators.cc:30-160
 *   cn0_m2m4_estimator / carrier_lock_detector   lock_detectors.cc:90-147
 *   Exponential_Smoother            exponential_smoother.cc:29-105
 *   dll_pll_veml_tracking           gnuradio_blocks/dll_pll_veml_tracking.cc:
 *       start_tracking :643-883, state 1 pull-in :1757-1788, state 2 :1789-1932, state 4 :1971-2028,
 *       cn0_and_tracking_lock_status :972-1029, do_correlation_step :1037-1062,
 *       run_dll_pll :1065-1152, save_correlation_results :1262-1350, update_tracking_vars :1189-1260,
 *       acquire_secondary :925-970.
 * Also restated: extended coherent integration (state 3, extend_correlation_symbols > 1), the FLL
 * branches of run_dll_pll (:1080-1097) and the high_dyn NCO rate smoothing (:1205-1255) with the
 * high-dynamics multicorrelator.  The Doppler-correction experiment is not (default off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TRK_MAX_SEC 256

/* ---- Tracking_loop_filter ----------------------------------------------------------------- */
typedef struct {
    float noise_bandwidth, update_interval;
    int order, include_last_integrator;
    float in_coef[4], out_coef[3];
    int n_in, n_out;
    float inputs[4], outputs[4];
    int idx;
} orc_loop_filter;

void orc_lf_update_coefficients(orc_loop_filter* f)
{
    const float T = f->update_interval;
    const float zeta = 1.0F / sqrtf(2.0F);
    float g1, g2, g3, wn;
    switch (f->order) {
    case 1:
        wn = f->noise_bandwidth * 4.0F;
        g1 = wn;
        if (f->include_last_integrator) {
            f->n_in = 2;
            f->in_coef[0] = (float)(g1 * T / 2.0);
            f->in_coef[1] = (float)(g1 * T / 2.0);
            f->n_out = 1;
            f->out_coef[0] = 1.0F;
        } else {
            f->n_in = 1;
            f->in_coef[0] = g1;
            f->n_out = 0;
        }
        break;
    case 2:
        wn = f->noise_bandwidth * (8.0F * zeta) / (4.0F * zeta * zeta + 1.0F);
        g1 = wn * wn;
        g2 = wn * 2.0F * zeta;
        if (f->include_last_integrator) {
            f->n_in = 3;
            f->in_coef[0] = (float)(T / 2.0 * (g1 * T / 2.0 + g2));
            f->in_coef[1] = (float)(T * T / 2.0 * g1);
            f->in_coef[2] = (float)(T / 2.0 * (g1 * T / 2.0 - g2));
            f->n_out = 2;
            f->out_coef[0] = 2.0F;
            f->out_coef[1] = -1.0F;
        } else {
            f->n_in = 2;
            f->in_coef[0] = (float)(g1 * T / 2.0 + g2);
            f->in_coef[1] = (float)(g1 * T / 2.0 - g2);
            f->n_out = 1;
            f->out_coef[0] = 1.0F;
        }
        break;
    default: { /* 3 */
        wn = f->noise_bandwidth / 0.7845F;
        const float a3 = 1.1F;
        const float b3 = 2.4F;
        g1 = wn * wn * wn;
        g2 = a3 * wn * wn;
        g3 = b3 * wn;
        if (f->include_last_integrator) {
            f->n_in = 4;
            f->in_coef[0] = (float)(T / 2.0 * (g3 + T / 2.0 * (g2 + T / 2.0 * g1)));
            f->in_coef[1] = (float)(T / 2.0 * (-g3 + T / 2.0 * (g2 + 3.0 * T / 2.0 * g1)));
            f->in_coef[2] = (float)(T / 2.0 * (-g3 - T / 2.0 * (g2 - 3.0 * T / 2.0 * g1)));
            f->in_coef[3] = (float)(T / 2.0 * (g3 - T / 2.0 * (g2 - T / 2.0 * g1)));
            f->n_out = 3;
            f->out_coef[0] = 3.0F;
            f->out_coef[1] = -3.0F;
            f->out_coef[2] = 1.0F;
        } else {
            f->n_in = 3;
            f->in_coef[0] = (float)(g3 + T / 2.0 * (g2 + T / 2.0 * g1));
            f->in_coef[1] = (float)(g1 * T * T / 2.0 - 2.0 * g3);
            f->in_coef[2] = (float)(g3 + T / 2.0 * (-g2 + T / 2.0 * g1));
            f->n_out = 2;
            f->out_coef[0] = 2.0F;
            f->out_coef[1] = -1.0F;
        }
    } break;
    }
}

void orc_lf_init(orc_loop_filter* f, float update_interval, float noise_bandwidth, int order, int include_last_integrator)
{
    memset(f, 0, sizeof(*f));
    f->update_interval = update_interval;
    f->noise_bandwidth = noise_bandwidth;
    f->order = order;
    f->include_last_integrator = include_last_integrator;
    f->idx = 0;
    orc_lf_update_coefficients(f);
}

void orc_lf_initialize(orc_loop_filter* f, float initial_output)
{
    for (int i = 0; i < 4; i++) {
        f->inputs[i] = 0.0F;
        f->outputs[i] = initial_output;
    }
    f->idx = 3;
}

float orc_lf_apply(orc_loop_filter* f, float current_input)
{
    float result = 0.0F;
    for (int ii = 0; ii < f->n_out; ii++) result += f->out_coef[ii] * f->outputs[(f->idx + ii) % 4];
    f->idx--;
    if (f->idx < 0) f->idx += 4;
    f->inputs[f->idx] = current_input;
    for (int ii = 0; ii < f->n_in; ii++) result += f->in_coef[ii] * f->inputs[(f->idx + ii) % 4];
    f->outputs[f->idx] = result;
    return result;
}

/* ---- Tracking_FLL_PLL_filter -------------------------------------------------------------- */
typedef struct {
    float w, x, w0p3, w0f2, a2, w0f, a3, w0p2, b3, w0p;
    int order;
} orc_fll_pll;

void orc_fp_set_params(orc_fll_pll* f, float fll_bw_hz, float pll_bw_hz, int order)
{
    f->order = order;
    if (order == 3) {
        f->b3 = 2.400F;
        f->a3 = 1.100F;
        f->a2 = 1.414F;
        f->w0p = pll_bw_hz / 0.7845F;
        f->w0p2 = f->w0p * f->w0p;
        f->w0p3 = f->w0p2 * f->w0p;
        f->w0f = fll_bw_hz / 0.53F;
        f->w0f2 = f->w0f * f->w0f;
    } else {
        f->a2 = 1.414F;
        f->w0p = pll_bw_hz / 0.53F;
        f->w0p2 = f->w0p * f->w0p;
        f->w0f = fll_bw_hz / 0.25F;
    }
}

void orc_fp_initialize(orc_fll_pll* f, float acq_doppler_hz)
{
    if (f->order == 3) {
        f->x = 2.0F * acq_doppler_hz;
        f->w = 0.0F;
    } else {
        f->w = acq_doppler_hz;
        f->x = 0.0F;
    }
}

float orc_fp_get_carrier_error(orc_fll_pll* f, float fll_disc, float pll_disc, float T)
{
    float e;
    if (f->order == 3) {
        f->w = f->w + T * (f->w0p3 * pll_disc + f->w0f2 * fll_disc);
        f->x = f->x + T * (0.5F * f->w + f->a2 * f->w0f * fll_disc + f->a3 * f->w0p2 * pll_disc);
        e = 0.5F * f->x + f->b3 * f->w0p * pll_disc;
    } else {
        const float w_new = f->w + pll_disc * f->w0p2 * T + fll_disc * f->w0f * T;
        e = 0.5F * (w_new + f->w) + f->a2 * f->w0p * pll_disc;
        f->w = w_new;
    }
    return e;
}

/* ---- discriminators (complex values as float pairs) ----------------------------------------- */
double orc_pll_cloop_two_quadrant_atan(float i, float q)
{
    if (i != 0.0F) return (double)atanf(q / i);
    return 0.0;
}

/* gr::fast_atan2f is a table-based approximation (GNU Radio, absent here): restated as atan2f;
 * the difference (< 1e-6 rad per GNU Radio's docs) only enters after secondary-code lock. */
double orc_pll_four_quadrant_atan(float i, float q) { return (double)atan2f(q, i); }

double orc_dll_nc_e_minus_l_normalized(float er, float ei, float lr, float li, float spc, float slope, float y_intercept)
{
    const double p_early = (double)hypotf(er, ei);
    const double p_late = (double)hypotf(lr, li);
    const double e_plus_l = p_early + p_late;
    if (e_plus_l == 0.0) return 0.0;
    return (double)((y_intercept - slope * spc) / slope) * (p_early - p_late) / e_plus_l;
}

double orc_dll_nc_vemlp_normalized(const float* ve, const float* e, const float* l, const float* vl)
{
    const double early = (double)sqrtf(ve[0] * ve[0] + ve[1] * ve[1] + e[0] * e[0] + e[1] * e[1]);
    const double late = (double)sqrtf(l[0] * l[0] + l[1] * l[1] + vl[0] * vl[0] + vl[1] * vl[1]);
    const double e_plus_l = early + late;
    if (e_plus_l == 0.0) return 0.0;
    return (early - late) / e_plus_l;
}

/* ---- lock detectors ------------------------------------------------------------------------ */
float orc_cn0_m2m4_estimator(const float* prompt, int length, float coh_integration_time_s)
{
    float snr_aux, psig = 0.0F, m_2 = 0.0F, m_4 = 0.0F, aux;
    const float n = (float)length;
    for (int i = 0; i < length; i++) {
        psig += fabsf(prompt[2 * i]);
        aux = prompt[2 * i + 1] * prompt[2 * i + 1] + prompt[2 * i] * prompt[2 * i];
        m_2 += aux;
        m_4 += aux * aux;
    }
    psig /= n;
    psig = psig * psig;
    m_2 /= n;
    m_4 /= n;
    aux = sqrtf(2.0F * m_2 * m_2 - m_4);
    if (isnan(aux))
        snr_aux = psig / (m_2 - psig);
    else
        snr_aux = aux / (m_2 - aux);
    return 10.0F * log10f(snr_aux) - 10.0F * log10f(coh_integration_time_s);
}

float orc_carrier_lock_detector(const float* prompt, int length)
{
    float si = 0.0F, sq = 0.0F;
    for (int i = 0; i < length; i++) {
        si += prompt[2 * i];
        sq += prompt[2 * i + 1];
    }
    const float nbp = si * si + sq * sq;
    const float nbd = si * si - sq * sq;
    return nbd / nbp;
}

/* ---- Exponential_Smoother (float overload) ------------------------------------------------- */
typedef struct {
    float alpha, one_minus_alpha, min_value, offset, old_value, init_sum;
    int samples_for_init, initializing, counter;
} orc_smoother;

void orc_sm_init(orc_smoother* s, float alpha, float min_value, float offset, int samples_for_init)
{
    memset(s, 0, sizeof(*s));
    s->alpha = alpha < 0.0F ? 0.0F : (alpha > 1.0F ? 1.0F : alpha);
    s->one_minus_alpha = 1.0F - s->alpha;
    s->min_value = min_value;
    s->offset = offset;
    s->samples_for_init = samples_for_init <= 0 ? 1 : samples_for_init;
    s->initializing = 1;
}

void orc_sm_reset(orc_smoother* s)
{
    s->initializing = 1;
    s->counter = 0;
    s->init_sum = 0.0F;
}

float orc_sm_smooth(orc_smoother* s, float raw)
{
    float v;
    if (s->initializing) {
        s->counter++;
        v = raw;
        s->init_sum += v; /* std::accumulate(init_buffer, 0.0F): same left-to-right float sum */
        if (s->counter == s->samples_for_init) {
            s->old_value = s->init_sum / (float)s->counter;
            if (s->old_value < (s->min_value + s->offset)) {
                s->counter = 0;
                s->init_sum = 0.0F;
            } else {
                s->initializing = 0;
            }
        }
    } else {
        v = s->alpha * raw + s->one_minus_alpha * s->old_value;
        s->old_value = v;
    }
    return v;
}

/* MATH_CONSTANTS.h:47-49: the GNSS value of pi (not M_PI) */
#define TRK_GNSS_PI 3.1415926535898
#define TRK_HALF_PI (TRK_GNSS_PI / 2.0)
#define TRK_TWO_PI (2.0 * TRK_GNSS_PI)

/* phase_unwrap / fll_diff_atan (tracking_discriminators.cc:27-41, 68-76): std::atan of the float
 * quotients (float overload), difference as float, NaN → 0, unwrapped by ±pi. */
static double orc_phase_unwrap(double phase_rad)
{
    if (phase_rad >= TRK_HALF_PI) return phase_rad - TRK_GNSS_PI;
    if (phase_rad <= -TRK_HALF_PI) return phase_rad + TRK_GNSS_PI;
    return phase_rad;
}

double orc_fll_diff_atan(const float* s1, const float* s2, double t1, double t2)
{
    double diff_atan = (double)(atanf(s2[1] / s2[0]) - atanf(s1[1] / s1[0]));
    if (isnan(diff_atan)) diff_atan = 0;
    return orc_phase_unwrap(diff_atan) / (t2 - t1);
}

/* ---- channel ---------------------------------------------------------------------------- */
typedef struct {
    /* Dll_Pll_Conf subset + signal constants (set by the caller, as the adapters do) */
    double fs_in, carrier_lock_th, code_chip_rate, signal_carrier_freq, code_period;
    float pll_bw_hz, dll_bw_hz, fll_bw_hz, early_late_space_chips, very_early_late_space_chips, slope, spc, y_intercept;
    float cn0_smoother_alpha, carrier_lock_test_smoother_alpha;
    uint32_t pull_in_time_s, bit_synchronization_time_limit_s, vector_length;
    int32_t pll_filter_order, dll_filter_order, cn0_samples, cn0_smoother_samples, carrier_lock_test_smoother_samples, cn0_min;
    int32_t max_code_lock_fail, max_carrier_lock_fail, carrier_aiding, track_pilot, veml;
    int32_t code_length_chips, code_samples_per_chip, symbols_per_bit, secondary, secondary_code_length, data_secondary_code_length;
    char secondary_code[TRK_MAX_SEC + 1];
    char data_secondary_code[TRK_MAX_SEC + 1];
    /* extended coherent integration (dll_pll_conf.h:48-53,66): enabled when extend > 1 (:515-523) */
    int32_t extend_correlation_symbols;
    float pll_bw_narrow_hz, dll_bw_narrow_hz, early_late_space_narrow_chips, very_early_late_space_narrow_chips;
    int32_t enable_fll_pull_in, enable_fll_steady_state; /* dll_pll_conf.h:75-76 */
    int32_t high_dyn;         /* dll_pll_conf.h:80: high-dynamics correlator + NCO rate smoothing */
    uint32_t smoother_length; /* dll_pll_conf.h:62 (dll_pll_conf.cc:118-123 raises 0 to 1) */
    int32_t rotator_avx;      /* 1: the rotator dot-product is volk's u_avx/a_avx variant (what volk_gnsssdr
                                 dispatches on an AVX host, volk_gnsssdr_rank_archs.c), 0: generic */
    int32_t accum_f64;        /* test-only: the same float products summed in double (long epochs, see
                                 orc_rotator_dot_prod_acc64) */
    int32_t pad_trig;         /* unused (layout) */
    int32_t pad_if;
    /* Carrier IF of the signal in the buffer [Hz], whole Hz (with a whole-Hz fs_in).  The reference removes
     * it ahead of the channels (InputFilter.IF, freq_xlating_fir_filter; conf/gnss-sdr_BDS_B3I_GPS_L1_CA_
     * ibyte.conf:45-92) so its tracking sees the IF-free signal; this restatement (like the engine, see
     * include/gnsship.h if_hz) folds it into the correlation arguments instead: carr_step + 2π·if/fs, and
     * rem_carr + 2π·frac(if·n/fs) at the epoch's first absolute sample n.  The loop itself is unchanged. */
    double if_hz;
} orc_trk_conf;

#define TRK_MAX_SMOOTHER 64

typedef struct {
    int state, cloop, pull_in, veml, n_taps, pll_180;
    uint64_t acq_sample_stamp;
    uint64_t nitems_read; /* absolute index of the next input sample */
    double acq_code_phase_samples, acq_carrier_doppler_hz;
    double carrier_doppler_hz, carrier_phase_step_rad, code_freq_chips, code_phase_step_chips, rem_code_phase_chips, rem_code_phase_samples;
    double acc_carrier_phase_rad, carr_phase_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips, current_correlation_time_s;
    double T_chip_seconds, T_prn_seconds, T_prn_samples, K_blk_samples;
    float rem_carr_phase_rad;
    int32_t current_prn_length_samples;
    float shifts[5];
    float spc;
    float ve[2], e[2], p[2], l[2], vl[2], p_data[2], p_old[2];
    int cn0_counter, carrier_fail, code_fail, current_symbol, current_data_symbol, acc_carrier_phase_initialized;
    float prompt_buf[2 * 64];
    float cn0_db_hz, carrier_lock_test;
    char prompt_sign[TRK_MAX_SEC]; /* d_Prompt_circular_buffer as real < 0 flags, oldest first */
    int prompt_count;
    orc_loop_filter code_filter;
    orc_fll_pll carrier_filter;
    orc_smoother cn0_sm, lock_sm;
    int extend_count; /* d_extend_correlation_symbols_count */
    /* high_dyn: d_carr_ph_history / d_code_ph_history (boost::circular_buffer of capacity
     * 2·smoother_length, :557-566) — pushed together with the same sample count, so one ring */
    double carrier_phase_rate_step_rad, code_phase_rate_step_chips;
    double hist_carr[2 * TRK_MAX_SMOOTHER], hist_code[2 * TRK_MAX_SMOOTHER], hist_samples[2 * TRK_MAX_SMOOTHER];
    int hist_head, hist_count;
    uint32_t prn; /* Gnss_Synchro::PRN (dump records) */
    int64_t if_num; /* IF phase at nitems_read = if_num / fs cycles, exactly */
} orc_trk_channel;

/* (if·n) mod fs for whole-Hz if and fs, exact (if reduced into [0, fs) first). */
static int64_t orc_if_num(const orc_trk_conf* k, uint64_t n)
{
    const int64_t fs = (int64_t)k->fs_in;
    const int64_t ifm = (((int64_t)k->if_hz % fs) + fs) % fs;
    return (int64_t)(((unsigned __int128)(uint64_t)ifm * (n % (uint64_t)fs)) % (uint64_t)fs);
}

/* The tracking dump record log_data writes field by field (dll_pll_veml_tracking.cc:1376-1466;
 * read back by tracking_dump_reader.cc:26-47): 96 bytes, no padding. */
#pragma pack(push, 4)
typedef struct {
    float abs_VE, abs_E, abs_P, abs_L, abs_VL, prompt_I, prompt_Q;
    uint64_t PRN_start_sample_count;
    float acc_carrier_phase_rad, carrier_doppler_hz, carrier_doppler_rate_hz, code_freq_chips, code_freq_rate_chips;
    float carr_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips, CN0_SNV_dB_Hz, carrier_lock_test;
    float aux1;
    double aux2;
    uint32_t PRN;
} orc_trk_dump;
#pragma pack(pop)

typedef struct { /* Gnss_Synchro subset emitted per epoch (dll_pll_veml_tracking.cc:1996-2091) */
    uint64_t sample_counter;
    double prompt_i, prompt_q, code_phase_samples, carrier_phase_rads, carrier_doppler_hz, cn0_db_hz;
    float carrier_lock_test;
    int32_t state, flags; /* flags: 1 valid symbol, 2 loss of lock, 4 PLL 180°, 16 log_data record written */
    double code_freq_chips, rem_code_phase_chips;
    float rem_carr_phase_rad;
    int32_t prn_length_samples;
} orc_trk_epoch;

static void clear_tracking_vars(orc_trk_channel* c)
{
    memset(c->p_data, 0, sizeof(c->p_data));
    memset(c->p_old, 0, sizeof(c->p_old));
    c->carr_phase_error_hz = 0.0;
    c->carr_error_filt_hz = 0.0;
    c->code_error_chips = 0.0;
    c->code_error_filt_chips = 0.0;
    c->current_symbol = 0;
    c->current_data_symbol = 0;
    c->prompt_count = 0;
    c->carrier_phase_rate_step_rad = 0.0; /* :1182-1185 */
    c->code_phase_rate_step_chips = 0.0;
    c->hist_head = 0;
    c->hist_count = 0;
}

/* start_tracking (:643-883) then the state-1 pull-in alignment (:1757-1788) evaluated when the
 * block first sees sample index `first_sample`. */
void orc_trk_start(const orc_trk_conf* k, orc_trk_channel* c, double acq_delay_samples, double acq_doppler_hz, uint64_t acq_samplestamp,
    uint64_t first_sample)
{
    memset(c, 0, sizeof(*c));
    c->acq_code_phase_samples = acq_delay_samples;
    c->acq_carrier_doppler_hz = acq_doppler_hz;
    c->acq_sample_stamp = acq_samplestamp;
    c->carrier_doppler_hz = acq_doppler_hz;
    c->carrier_phase_step_rad = TRK_TWO_PI * c->carrier_doppler_hz / k->fs_in;
    c->veml = k->veml;
    c->n_taps = k->veml ? 5 : 3;
    const float spcf = (float)k->code_samples_per_chip;
    if (k->veml) {
        c->shifts[0] = -k->very_early_late_space_chips * spcf;
        c->shifts[1] = -k->early_late_space_chips * spcf;
        c->shifts[2] = 0.0F;
        c->shifts[3] = k->early_late_space_chips * spcf;
        c->shifts[4] = k->very_early_late_space_chips * spcf;
    } else {
        c->shifts[0] = -k->early_late_space_chips * spcf;
        c->shifts[1] = 0.0F;
        c->shifts[2] = k->early_late_space_chips * spcf;
    }
    c->carrier_lock_test = 1.0F;
    c->cn0_db_hz = 0.0F;
    c->current_correlation_time_s = k->code_period;
    c->spc = k->spc;
    orc_fp_set_params(&c->carrier_filter, k->fll_bw_hz, k->pll_bw_hz, k->pll_filter_order);
    orc_lf_init(&c->code_filter, (float)k->code_period, k->dll_bw_hz, k->dll_filter_order, 0);
    orc_fp_initialize(&c->carrier_filter, (float)acq_doppler_hz);
    orc_lf_initialize(&c->code_filter, 0.0F);
    int ns = k->cn0_smoother_samples / (int)(k->code_period * 1000.0);
    orc_sm_init(&c->cn0_sm, k->cn0_smoother_alpha, 25.0F, 12.0F, ns);
    orc_sm_init(&c->lock_sm, k->carrier_lock_test_smoother_alpha, -1.0F, 0.0F, k->carrier_lock_test_smoother_samples);
    clear_tracking_vars(c);
    c->cloop = 1;
    c->pull_in = 1;
    /* state 1 */
    const int64_t acq_trk_diff_samples = (int64_t)first_sample - (int64_t)c->acq_sample_stamp;
    const double delta = (double)acq_trk_diff_samples - c->acq_code_phase_samples;
    c->code_freq_chips = k->code_chip_rate;
    c->code_phase_step_chips = c->code_freq_chips / k->fs_in;
    const double T_chip_mod_seconds = 1.0 / c->code_freq_chips;
    const double T_prn_mod_seconds = T_chip_mod_seconds * (double)k->code_length_chips;
    const double T_prn_mod_samples = T_prn_mod_seconds * k->fs_in;
    c->acq_code_phase_samples = T_prn_mod_samples - fmod(delta, T_prn_mod_samples);
    c->current_prn_length_samples = (int32_t)round(T_prn_mod_samples);
    const int32_t samples_offset = (int32_t)round(c->acq_code_phase_samples);
    c->acc_carrier_phase_rad -= c->carrier_phase_step_rad * (double)samples_offset;
    c->state = 2;
    orc_sm_reset(&c->cn0_sm);
    orc_sm_reset(&c->lock_sm);
    c->nitems_read = first_sample + (uint64_t)samples_offset;
    c->if_num = k->if_hz != 0.0 ? orc_if_num(k, c->nitems_read) : 0;
}

/* do_correlation_step arguments (:1037-1062) for the next epoch: the float values passed to
 * Carrier_wipeoff_multicorrelator_resampler.  out[6] = rem_carr, carr_step, carr_rate,
 * rem_code·spc, code_step·spc, code_rate·spc. */
void orc_trk_correlation_args(const orc_trk_conf* k, const orc_trk_channel* c, float* out)
{
    const float spcf = (float)k->code_samples_per_chip;
    out[0] = c->rem_carr_phase_rad;
    out[1] = (float)c->carrier_phase_step_rad;
    if (k->if_hz != 0.0) { /* the IF folded into the carrier arguments (orc_trk_conf::if_hz) */
        const double fs = (double)(int64_t)k->fs_in;
        out[0] = (float)fmod((double)c->rem_carr_phase_rad + TRK_TWO_PI * ((double)c->if_num / fs), TRK_TWO_PI);
        out[1] = (float)(c->carrier_phase_step_rad + TRK_TWO_PI * k->if_hz / k->fs_in);
    }
    out[2] = (float)c->carrier_phase_rate_step_rad;
    out[3] = (float)c->rem_code_phase_chips * spcf;
    out[4] = (float)c->code_phase_step_chips * spcf;
    out[5] = (float)c->code_phase_rate_step_chips * spcf; /* do_correlation_step :1043-1048 */
}

static int cn0_and_tracking_lock_status(const orc_trk_conf* k, orc_trk_channel* c, double coh_integration_time_s)
{
    if (c->cn0_counter < k->cn0_samples) {
        c->prompt_buf[2 * c->cn0_counter] = c->p[0];
        c->prompt_buf[2 * c->cn0_counter + 1] = c->p[1];
        c->cn0_counter++;
        return 1;
    }
    const int slot = c->cn0_counter % k->cn0_samples;
    c->prompt_buf[2 * slot] = c->p[0];
    c->prompt_buf[2 * slot + 1] = c->p[1];
    c->cn0_counter++;
    const float raw = orc_cn0_m2m4_estimator(c->prompt_buf, k->cn0_samples, (float)coh_integration_time_s);
    c->cn0_db_hz = orc_sm_smooth(&c->cn0_sm, raw);
    c->carrier_lock_test = orc_sm_smooth(&c->lock_sm, orc_carrier_lock_detector(c->prompt_buf, 1));
    if (!c->pull_in) {
        if ((double)c->carrier_lock_test < k->carrier_lock_th)
            c->carrier_fail++;
        else if (c->carrier_fail > 0)
            c->carrier_fail--;
        if (c->cn0_db_hz < (float)k->cn0_min)
            c->code_fail++;
        else if (c->code_fail > 0)
            c->code_fail--;
    }
    if (c->carrier_fail > k->max_carrier_lock_fail || c->code_fail > k->max_code_lock_fail) {
        c->carrier_fail = 0;
        c->code_fail = 0;
        return 0;
    }
    return 1;
}

static void run_dll_pll(const orc_trk_conf* k, orc_trk_channel* c)
{
    if (c->cloop)
        c->carr_phase_error_hz = orc_pll_cloop_two_quadrant_atan(c->p[0], c->p[1]) / TRK_TWO_PI;
    else
        c->carr_phase_error_hz = orc_pll_four_quadrant_atan(c->p[0], c->p[1]) / TRK_TWO_PI;
    if ((c->pull_in && k->enable_fll_pull_in) || k->enable_fll_steady_state) { /* :1080-1097 */
        const double fe = orc_fll_diff_atan(c->p_old, c->p, 0.0, c->current_correlation_time_s) / TRK_TWO_PI;
        c->p_old[0] = c->p[0];
        c->p_old[1] = c->p[1];
        if (c->pull_in && k->enable_fll_pull_in)
            c->carr_error_filt_hz = orc_fp_get_carrier_error(&c->carrier_filter, (float)fe, 0.0F, (float)c->current_correlation_time_s);
        else
            c->carr_error_filt_hz = orc_fp_get_carrier_error(&c->carrier_filter, (float)fe, (float)c->carr_phase_error_hz, (float)c->current_correlation_time_s);
    } else {
        c->carr_error_filt_hz = orc_fp_get_carrier_error(&c->carrier_filter, 0.0F, (float)c->carr_phase_error_hz, (float)c->current_correlation_time_s);
    }
    c->carrier_doppler_hz = c->carr_error_filt_hz;
    if (c->veml)
        c->code_error_chips = orc_dll_nc_vemlp_normalized(c->ve, c->e, c->l, c->vl);
    else
        c->code_error_chips = orc_dll_nc_e_minus_l_normalized(c->e[0], c->e[1], c->l[0], c->l[1], c->spc, k->slope, k->y_intercept);
    c->code_error_filt_chips = orc_lf_apply(&c->code_filter, (float)c->code_error_chips);
    c->code_freq_chips = k->code_chip_rate - c->code_error_filt_chips;
    if (k->carrier_aiding) c->code_freq_chips += c->carrier_doppler_hz * k->code_chip_rate / k->signal_carrier_freq;
}

/* The high_dyn rate estimate (:1205-1222, :1238-1255): mean phase step of the newest
 * smoother_length entries minus the mean of the oldest, over the newest entries' sample count.
 * Both sums run in the reference's index order. */
static double smoothed_rate(const orc_trk_channel* c, const double* first, int L)
{
    const int cap = 2 * L;
    double cp1 = 0.0, cp2 = 0.0, samples = 0.0;
    for (int i = 0; i < L; i++) {
        const int a = (c->hist_head + i) % cap, b = (c->hist_head + cap - i - 1) % cap;
        cp1 += first[a];
        cp2 += first[b];
        samples += c->hist_samples[b];
    }
    cp1 /= (double)L;
    cp2 /= (double)L;
    return (cp2 - cp1) / samples;
}

static void update_tracking_vars(const orc_trk_conf* k, orc_trk_channel* c)
{
    c->T_chip_seconds = 1.0 / c->code_freq_chips;
    c->T_prn_seconds = c->T_chip_seconds * (double)k->code_length_chips;
    c->T_prn_samples = c->T_prn_seconds * k->fs_in;
    c->K_blk_samples = c->T_prn_samples + c->rem_code_phase_samples;
    c->current_prn_length_samples = (int32_t)floor(c->K_blk_samples);
    c->carrier_phase_step_rad = TRK_TWO_PI * c->carrier_doppler_hz / k->fs_in;
    const double n = (double)c->current_prn_length_samples;
    c->code_phase_step_chips = c->code_freq_chips / k->fs_in;
    if (k->high_dyn) {
        /* push_back on the ring (a full circular_buffer drops its oldest entry) */
        const int L = (int)(k->smoother_length < 1 ? 1 : k->smoother_length), cap = 2 * L;
        int slot;
        if (c->hist_count < cap) {
            slot = (c->hist_head + c->hist_count) % cap;
            c->hist_count++;
        } else {
            slot = c->hist_head;
            c->hist_head = (c->hist_head + 1) % cap;
        }
        c->hist_carr[slot] = c->carrier_phase_step_rad;
        c->hist_code[slot] = c->code_phase_step_chips;
        c->hist_samples[slot] = n;
        if (c->hist_count == cap) {
            c->carrier_phase_rate_step_rad = smoothed_rate(c, c->hist_carr, L);
            c->code_phase_rate_step_chips = smoothed_rate(c, c->hist_code, L);
        }
    }
    const double adv = c->carrier_phase_step_rad * n + 0.5 * c->carrier_phase_rate_step_rad * n * n;
    c->rem_carr_phase_rad += (float)adv;
    c->rem_carr_phase_rad = (float)fmod((double)c->rem_carr_phase_rad, TRK_TWO_PI);
    c->acc_carrier_phase_rad -= adv;
    c->rem_code_phase_samples = c->K_blk_samples - n;
    c->rem_code_phase_chips = c->code_freq_chips * c->rem_code_phase_samples / k->fs_in;
}

static void cadd(float* acc, const float* v, float sgn)
{
    acc[0] += sgn * v[0];
    acc[1] += sgn * v[1];
}

static void save_correlation_results(const orc_trk_conf* k, orc_trk_channel* c, const float* taps, const float* pdata)
{
    const float* VE = taps;
    const float* E = c->veml ? taps + 2 : taps;
    const float* P = c->veml ? taps + 4 : taps + 2;
    const float* L = c->veml ? taps + 6 : taps + 4;
    const float* VL = taps + 8;
    float sgn = 1.0F;
    if (k->secondary) {
        sgn = (k->secondary_code[c->current_symbol] == '0') ? 1.0F : -1.0F;
        c->current_symbol = (c->current_symbol + 1) % k->secondary_code_length;
    }
    if (c->veml) {
        cadd(c->ve, VE, sgn);
        cadd(c->vl, VL, sgn);
    }
    cadd(c->e, E, sgn);
    cadd(c->p, P, sgn);
    cadd(c->l, L, sgn);
    const float* src = k->track_pilot ? pdata : P;
    if (k->symbols_per_bit > 1) {
        if (k->data_secondary_code_length > 0) {
            cadd(c->p_data, src, k->data_secondary_code[c->current_data_symbol] == '0' ? 1.0F : -1.0F);
            c->current_data_symbol = (c->current_data_symbol + 1) % k->data_secondary_code_length;
        } else {
            cadd(c->p_data, src, 1.0F);
            c->current_data_symbol = (c->current_data_symbol + 1) % k->symbols_per_bit;
        }
    } else {
        c->p_data[0] = src[0];
        c->p_data[1] = src[1];
    }
    c->cloop = k->track_pilot ? 0 : 1;
}

static int acquire_secondary(const orc_trk_conf* k, orc_trk_channel* c)
{
    int corr = 0;
    for (int i = 0; i < k->secondary_code_length; i++) {
        const int neg = c->prompt_sign[i];
        if (neg)
            corr += (k->secondary_code[i] == '0') ? 1 : -1;
        else
            corr += (k->secondary_code[i] == '0') ? -1 : 1;
    }
    if (abs(corr) == k->secondary_code_length) {
        c->pll_180 = corr < 0;
        return 1;
    }
    return 0;
}

static void push_prompt_sign(const orc_trk_conf* k, orc_trk_channel* c, float prompt_re)
{
    const int cap = k->secondary_code_length;
    if (c->prompt_count == cap) {
        memmove(c->prompt_sign, c->prompt_sign + 1, (size_t)cap - 1);
        c->prompt_sign[cap - 1] = prompt_re < 0.0F;
    } else {
        c->prompt_sign[c->prompt_count++] = prompt_re < 0.0F;
    }
}

static int extend_symbols(const orc_trk_conf* k) { return k->extend_correlation_symbols > 1 ? k->extend_correlation_symbols : 1; }

/* State 2 → extended integration (dll_pll_veml_tracking.cc:1890-1926): integration time
 * extend × code period, narrow DLL/PLL bandwidths (the filters keep their state), narrow taps. */
static void enter_extended_integration(const orc_trk_conf* k, orc_trk_channel* c)
{
    c->extend_count = 0;
    c->current_correlation_time_s = (float)extend_symbols(k) * (float)k->code_period;
    c->code_filter.update_interval = (float)c->current_correlation_time_s; /* set_update_interval */
    orc_lf_update_coefficients(&c->code_filter);
    c->code_filter.noise_bandwidth = k->dll_bw_narrow_hz; /* set_noise_bandwidth */
    orc_lf_update_coefficients(&c->code_filter);
    orc_fp_set_params(&c->carrier_filter, k->fll_bw_hz, k->pll_bw_narrow_hz, k->pll_filter_order);
    const float spcf = (float)k->code_samples_per_chip;
    if (c->veml) {
        c->shifts[0] = -k->very_early_late_space_narrow_chips * spcf;
        c->shifts[1] = -k->early_late_space_narrow_chips * spcf;
        c->shifts[3] = k->early_late_space_narrow_chips * spcf;
        c->shifts[4] = k->very_early_late_space_narrow_chips * spcf;
    } else {
        c->shifts[0] = -k->early_late_space_narrow_chips * spcf;
        c->shifts[2] = k->early_late_space_narrow_chips * spcf;
    }
    c->spc = k->early_late_space_narrow_chips;
    c->state = 3;
}

/* One general_work call in state 2, 3 or 4 for the epoch starting at c->nitems_read, given the
 * correlator outputs of that epoch (taps: n_taps complex, pdata: data-prompt complex).
 * Advances nitems_read by the new current_prn_length_samples.  Returns 0 when the channel is
 * (or becomes) idle. */
/* log_data (:1376-1466) at epoch start `nir`, after update_tracking_vars. */
static void log_data(const orc_trk_conf* k, const orc_trk_channel* c, const float* taps, const float* pdata, uint64_t nir, orc_trk_dump* d)
{
    if (!d) return;
    const int eo = c->veml ? 2 : 0;
    const float* prompt = k->track_pilot ? pdata : taps + eo + 2;
    d->prompt_I = prompt[0];
    d->prompt_Q = prompt[1];
    d->abs_VE = c->veml ? hypotf(c->ve[0], c->ve[1]) : 0.0F;
    d->abs_VL = c->veml ? hypotf(c->vl[0], c->vl[1]) : 0.0F;
    d->abs_E = hypotf(c->e[0], c->e[1]);
    d->abs_P = hypotf(c->p[0], c->p[1]);
    d->abs_L = hypotf(c->l[0], c->l[1]);
    d->PRN_start_sample_count = nir + (uint64_t)c->current_prn_length_samples;
    d->acc_carrier_phase_rad = (float)c->acc_carrier_phase_rad;
    d->carrier_doppler_hz = (float)c->carrier_doppler_hz;
    d->carrier_doppler_rate_hz = (float)(c->carrier_phase_rate_step_rad * k->fs_in * k->fs_in / TRK_TWO_PI);
    d->code_freq_chips = (float)c->code_freq_chips;
    d->code_freq_rate_chips = (float)(c->code_phase_rate_step_chips * k->fs_in * k->fs_in);
    d->carr_error_hz = (float)c->carr_phase_error_hz;
    d->carr_error_filt_hz = (float)c->carr_error_filt_hz;
    d->code_error_chips = (float)c->code_error_chips;
    d->code_error_filt_chips = (float)c->code_error_filt_chips;
    d->CN0_SNV_dB_Hz = c->cn0_db_hz;
    d->carrier_lock_test = c->carrier_lock_test;
    d->aux1 = (float)c->rem_code_phase_samples;
    d->aux2 = (double)(nir + (uint64_t)c->current_prn_length_samples);
    d->PRN = c->prn;
}

int orc_trk_epoch_update(const orc_trk_conf* k, orc_trk_channel* c, const float* taps, const float* pdata, orc_trk_epoch* rec, orc_trk_dump* dump)
{
    if (dump) memset(dump, 0, sizeof(*dump));
    memset(rec, 0, sizeof(*rec));
    if (c->state != 2 && c->state != 3 && c->state != 4) return 0;
    const uint64_t nir = c->nitems_read;
    rec->sample_counter = nir;
    if (c->pull_in) {
        if ((uint64_t)k->pull_in_time_s < (nir - c->acq_sample_stamp) / (uint64_t)(int)k->fs_in) {
            c->pull_in = 0;
            c->carrier_fail = 0;
            c->code_fail = 0;
        }
    }
    int loss = 0;
    const int st = c->state;
    if (st == 2) {
        const float* VE = taps;
        if (c->veml) {
            c->ve[0] = VE[0];
            c->ve[1] = VE[1];
            c->vl[0] = taps[8];
            c->vl[1] = taps[9];
        }
        const int eo = c->veml ? 2 : 0;
        c->e[0] = taps[eo];
        c->e[1] = taps[eo + 1];
        c->p[0] = taps[eo + 2];
        c->p[1] = taps[eo + 3];
        c->l[0] = taps[eo + 4];
        c->l[1] = taps[eo + 5];
        c->spc = k->early_late_space_chips;
        rec->prompt_i = (double)c->p[0]; /* diagnostic: the epoch's prompt (no symbol flag in state 2) */
        rec->prompt_q = (double)c->p[1];
        if ((uint64_t)k->bit_synchronization_time_limit_s < (nir - c->acq_sample_stamp) / (uint64_t)(int)k->fs_in) c->carrier_fail = 300000;
        if (!cn0_and_tracking_lock_status(k, c, k->code_period)) {
            clear_tracking_vars(c);
            c->state = 0;
            loss = 1;
        } else {
            int next_state = 0;
            run_dll_pll(k, c);
            update_tracking_vars(k, c);
            log_data(k, c, taps, pdata, nir, dump);
            rec->flags |= 16;
            if (!c->pull_in) {
                if (k->secondary || k->symbols_per_bit > 1) {
                    push_prompt_sign(k, c, taps[eo + 2]);
                    if (c->prompt_count == k->secondary_code_length) next_state = acquire_secondary(k, c);
                } else {
                    next_state = 1;
                }
            }
            if (next_state) {
                memset(c->ve, 0, sizeof(c->ve));
                memset(c->e, 0, sizeof(c->e));
                memset(c->p, 0, sizeof(c->p));
                memset(c->p_data, 0, sizeof(c->p_data));
                memset(c->l, 0, sizeof(c->l));
                memset(c->vl, 0, sizeof(c->vl));
                c->prompt_count = 0;
                c->current_symbol = 0;
                c->current_data_symbol = 0;
                if (extend_symbols(k) > 1)
                    enter_extended_integration(k, c);
                else
                    c->state = 4;
            }
        }
    } else if (st == 3) { /* coherent integration (:1933-1970): accumulate, no loop update */
        save_correlation_results(k, c, taps, pdata);
        update_tracking_vars(k, c);
        if (c->current_data_symbol == 0) {
            log_data(k, c, taps, pdata, nir, dump);
            rec->flags |= 16;
            rec->prompt_i = (double)c->p_data[0];
            rec->prompt_q = (double)c->p_data[1];
            rec->flags |= 1;
            c->p_data[0] = c->p_data[1] = 0.0F;
        }
        c->extend_count++;
        if (c->extend_count == extend_symbols(k) - 1) {
            c->extend_count = 0;
            c->state = 4;
        }
    } else {
        save_correlation_results(k, c, taps, pdata);
        if (!cn0_and_tracking_lock_status(k, c, k->code_period * (double)extend_symbols(k))) {
            clear_tracking_vars(c);
            c->state = 0;
            loss = 1;
        } else {
            run_dll_pll(k, c);
            update_tracking_vars(k, c);
            if (!c->acc_carrier_phase_initialized) { /* check_carrier_phase_coherent_initialization */
                c->acc_carrier_phase_rad = -(double)c->rem_carr_phase_rad;
                c->acc_carrier_phase_initialized = 1;
            }
            if (c->current_data_symbol == 0) {
                log_data(k, c, taps, pdata, nir, dump);
                rec->flags |= 16;
                rec->prompt_i = (double)c->p_data[0];
                rec->prompt_q = (double)c->p_data[1];
                rec->flags |= 1;
                c->p_data[0] = c->p_data[1] = 0.0F;
            }
            memset(c->ve, 0, sizeof(c->ve));
            memset(c->e, 0, sizeof(c->e));
            memset(c->p, 0, sizeof(c->p));
            memset(c->l, 0, sizeof(c->l));
            memset(c->vl, 0, sizeof(c->vl));
            if (extend_symbols(k) > 1) c->state = 3; /* next coherent integration cycle */
        }
    }
    rec->state = st;
    if (loss) rec->flags |= 2;
    if (c->pll_180) rec->flags |= 4;
    rec->code_phase_samples = c->rem_code_phase_samples;
    rec->carrier_phase_rads = c->acc_carrier_phase_rad;
    rec->carrier_doppler_hz = c->carrier_doppler_hz;
    rec->cn0_db_hz = (double)c->cn0_db_hz;
    rec->carrier_lock_test = c->carrier_lock_test;
    rec->code_freq_chips = c->code_freq_chips;
    rec->rem_code_phase_chips = c->rem_code_phase_chips;
    rec->rem_carr_phase_rad = c->rem_carr_phase_rad;
    rec->prn_length_samples = c->current_prn_length_samples;
    if (loss) return 0;
    c->nitems_read += (uint64_t)c->current_prn_length_samples; /* consume_each (:2061) */
    if (k->if_hz != 0.0) {
        const int64_t fs = (int64_t)k->fs_in;
        c->if_num = (c->if_num + ((((int64_t)k->if_hz % fs) + fs) % fs) * (int64_t)c->current_prn_length_samples) % fs;
    }
    return 1;
}

int orc_trk_sizeof_channel(void) { return (int)sizeof(orc_trk_channel); }
int orc_trk_sizeof_conf(void) { return (int)sizeof(orc_trk_conf); }
int orc_trk_sizeof_epoch(void) { return (int)sizeof(orc_trk_epoch); }
int orc_trk_sizeof_dump(void) { return (int)sizeof(orc_trk_dump); }
void orc_trk_set_prn(orc_trk_channel* c, uint32_t prn) { c->prn = prn; }
uint64_t orc_trk_nitems_read(const orc_trk_channel* c) { return c->nitems_read; }
int orc_trk_state(const orc_trk_channel* c) { return c->state; }
/* msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:617-640): telemetry event 1 forces the
 * loss-of-lock condition at the next lock check. */
void orc_trk_telemetry_fault(orc_trk_channel* c) { c->carrier_fail = 200000; }

int orc_multicorrelator_real_codes_ex(float* corr_out, const float* sig_in, const float* local_code, int code_length_chips,
    const float* shifts_chips, int n_correlators, int flags, float rem_carrier_phase_in_rad, float phase_step_rad,
    float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* scratch, int accum_f64);

/* Closed loop over host CF32 samples (samples[i] = absolute sample buffer_first + i) for one channel: for each epoch, correlate
 * vector_length samples at nitems_read with the oracle multicorrelator (the tracking code and,
 * when track_pilot, the data code with one prompt tap), then update.  Stops after max_epochs,
 * when the channel goes idle, or when the next window leaves the buffer.  Returns epochs run. */
int orc_trk_run(const orc_trk_conf* k, orc_trk_channel* c, const float* samples, uint64_t buffer_first, int64_t n_samples, const float* code,
    int code_len, const float* data_code, int max_epochs, orc_trk_epoch* out, orc_trk_dump* dump)
{
    const int vl = (int)k->vector_length;
    float* scratch = (float*)malloc((size_t)5 * (size_t)vl * sizeof(float));
    const int cflags = (k->high_dyn ? 1 : 0) | (k->rotator_avx ? 2 : 0); /* gnsship_corr_job flags */
    int e = 0;
    for (; e < max_epochs; e++) {
        if (c->state != 2 && c->state != 3 && c->state != 4) break;
        if (c->nitems_read < buffer_first || (int64_t)(c->nitems_read - buffer_first) + vl > n_samples) break;
        float args[6];
        orc_trk_correlation_args(k, c, args);
        float taps[10] = {0}, pdata[2] = {0};
        const float* x = samples + 2 * (c->nitems_read - buffer_first);
        orc_multicorrelator_real_codes_ex(taps, x, code, code_len, c->shifts, c->n_taps, cflags, args[0], args[1], args[2], args[3], args[4], args[5], vl,
            scratch, k->accum_f64);
        if (k->track_pilot && data_code) {
            const float zero = 0.0F;
            orc_multicorrelator_real_codes_ex(pdata, x, data_code, code_len, &zero, 1, cflags, args[0], args[1], args[2], args[3], args[4], args[5], vl,
                scratch, k->accum_f64);
        }
        if (!orc_trk_epoch_update(k, c, taps, pdata, &out[e], dump ? &dump[e] : NULL)) {
            e++;
            break;
        }
    }
    free(scratch);
    return e;
}

int orc_trk_sizeof_loop_filter(void) { return (int)sizeof(orc_loop_filter); }
int orc_trk_sizeof_fll_pll(void) { return (int)sizeof(orc_fll_pll); }
int orc_trk_sizeof_smoother(void) { return (int)sizeof(orc_smoother); }
