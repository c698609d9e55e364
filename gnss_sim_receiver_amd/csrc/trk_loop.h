// trk_loop.h — the per-epoch DLL/PLL loop of dll_pll_veml_tracking as device functions, shared by
// the round-based step kernel (trk_kernel.hip: one lane per channel between correlator launches) and
// the persistent per-channel kernel (trk_persist.hip: one workgroup per channel for a whole run).
//
// Reference functions restated here (types as in the reference):
//   Tracking_loop_filter::apply           tracking_loop_filter.cc:58-84
//   Tracking_FLL_PLL_filter::get_carrier_error   tracking_FLL_PLL_filter.cc:72-110
//   pll_cloop_two_quadrant_atan / pll_four_quadrant_atan / dll_nc_e_minus_l_normalized /
//   dll_nc_vemlp_normalized               tracking_discriminators.cc:99-160
//   cn0_m2m4_estimator / carrier_lock_detector   lock_detectors.cc:90-147
//   Exponential_Smoother::smooth(float)   exponential_smoother.cc:76-105
//   cn0_and_tracking_lock_status :972-1029, run_dll_pll :1065-1152, update_tracking_vars
//   :1189-1260, save_correlation_results :1262-1350, acquire_secondary :925-970,
//   general_work states 2 (:1789-1932), 3 (:1933-1970) and 4 (:1971-2028).
#pragma once
// GNSSHIP_LOOP_INLINE: the loop functions' inlining attribute — trk_fast.hip forces them inline (its
// epoch loops are large enough for the inliner to give up, and an out-of-line call there caps the
// whole kernel's registers); the other engines leave the choice to the compiler.
#ifndef GNSSHIP_LOOP_INLINE
#define GNSSHIP_LOOP_INLINE
#endif
#include <cmath>
#include <type_traits>

#include "exact_div.h"
#include "trk_engine.h"

// Phase hook for the profiling build of the persistent kernel (trk_persist.hip); empty otherwise.
#ifndef GNSSHIP_TRK_LOOP_STAMP
#define GNSSHIP_TRK_LOOP_STAMP(k) ((void)0)
#endif

namespace gnsship {
namespace {


// MATH_CONSTANTS.h:47-49: the reference's pi is the GNSS value 3.1415926535898
constexpr double kGnssPi = 3.1415926535898;
constexpr double kTwoPi = 2.0 * kGnssPi;
constexpr double kInvTwoPi = 1.0 / kTwoPi;
// x / TWO_PI, fmod(x, TWO_PI), x / fs_in and x / carrier_freq, each the IEEE result (exact_div.h)
__device__ __forceinline__ double div_2pi(double x) { return div_by(x, kTwoPi, kInvTwoPi); }
__device__ __forceinline__ double fmod_2pi(double x) { return fmod_by(x, kTwoPi, kInvTwoPi); }
template <class K>
__device__ __forceinline__ double div_fs(const K& k, double x) { return div_by(x, k.conf.fs_in, k.inv_fs); }
template <class K>
__device__ __forceinline__ double div_carrier(const K& k, double x) { return div_by(x, k.carrier_freq, k.inv_carrier_freq); }
constexpr double kHalfPi = kGnssPi / 2.0;

// fll_diff_atan + phase_unwrap (tracking_discriminators.cc:27-41, 68-76)
__device__ GNSSHIP_LOOP_INLINE double fll_diff_atan(const float* s1, const float* s2, double t1, double t2)
{
    double d = static_cast<double>(__fsub_rn(glibc_atanf(__fdiv_rn(s2[1], s2[0])), glibc_atanf(__fdiv_rn(s1[1], s1[0]))));
    if (isnan(d)) d = 0.0;
    if (d >= kHalfPi)
        d -= kGnssPi;
    else if (d <= -kHalfPi)
        d += kGnssPi;
    return d / (t2 - t1);
}

__device__ GNSSHIP_LOOP_INLINE float smooth(Smoother& s, float raw, float alpha, float one_minus_alpha, float min_value, float offset, int init_samples)
{
    float v;
    if (s.initializing) {
        s.counter++;
        v = raw;
        s.init_sum = __fadd_rn(s.init_sum, v);
        if (s.counter == init_samples) {
            s.old_value = __fdiv_rn(s.init_sum, static_cast<float>(s.counter));
            if (s.old_value < __fadd_rn(min_value, offset)) {
                s.counter = 0;
                s.init_sum = 0.0f;
            } else {
                s.initializing = 0;
            }
        }
    } else {
        v = __fadd_rn(__fmul_rn(alpha, raw), __fmul_rn(one_minus_alpha, s.old_value));
        s.old_value = v;
    }
    return v;
}

// The three running sums over the prompt buffer in index order.  N > 0: the length as a constant
// (the buffer read in one batch of LDS loads instead of a load round trip per entry).
template <int N>
__device__ __forceinline__ void m2m4_sums(const float* prompt, int length, float& psig, float& m_2, float& m_4)
{
    float aux;
    const int n = N > 0 ? N : length;
#pragma unroll
    for (int i = 0; i < (N > 0 ? N : n); i++) {
        psig = __fadd_rn(psig, fabsf(prompt[2 * i]));
        aux = __fadd_rn(__fmul_rn(prompt[2 * i + 1], prompt[2 * i + 1]), __fmul_rn(prompt[2 * i], prompt[2 * i]));
        m_2 = __fadd_rn(m_2, aux);
        m_4 = __fadd_rn(m_4, __fmul_rn(aux, aux));
    }
}

__device__ GNSSHIP_LOOP_INLINE float cn0_m2m4(const float* prompt, int length, float coh_integration_time_s)
{
    float psig = 0.0f, m_2 = 0.0f, m_4 = 0.0f, aux;
    const float n = static_cast<float>(length);
    if (length == 20)  // every system's default (cn0_samples)
        m2m4_sums<20>(prompt, length, psig, m_2, m_4);
    else
        m2m4_sums<0>(prompt, length, psig, m_2, m_4);
    psig = __fdiv_rn(psig, n);
    psig = __fmul_rn(psig, psig);
    m_2 = __fdiv_rn(m_2, n);
    m_4 = __fdiv_rn(m_4, n);
    aux = sqrt_rn_f32(__fsub_rn(__fmul_rn(__fmul_rn(2.0f, m_2), m_2), m_4));
    const float snr = isnan(aux) ? __fdiv_rn(psig, __fsub_rn(m_2, psig)) : __fdiv_rn(aux, __fsub_rn(m_2, aux));
    // glibc's log10f (glibc_logf.h): the CN0 the reference computes, to the bit
    return __fsub_rn(__fmul_rn(10.0f, glibc_log10f(snr)), __fmul_rn(10.0f, glibc_log10f(coh_integration_time_s)));
}

__device__ GNSSHIP_LOOP_INLINE float carrier_lock_detector(const float* prompt)  // called with length 1 (:989)
{
    const float si = prompt[0], sq = prompt[1];
    const float nbp = __fadd_rn(__fmul_rn(si, si), __fmul_rn(sq, sq));
    const float nbd = __fsub_rn(__fmul_rn(si, si), __fmul_rn(sq, sq));
    return __fdiv_rn(nbd, nbp);
}

__device__ GNSSHIP_LOOP_INLINE bool lock_status(const TrkParams& k, TrkChannel& c, double coh_integration_time_s)
{
    const int ns = k.conf.cn0_samples;
    if (c.cn0_counter < ns) {
        c.prompt_buf[2 * c.cn0_counter] = c.p[0];
        c.prompt_buf[2 * c.cn0_counter + 1] = c.p[1];
        c.cn0_counter++;
        return true;
    }
    const int slot = ns == 20 ? c.cn0_counter % 20 : c.cn0_counter % ns;  // the default as a constant divisor
    c.prompt_buf[2 * slot] = c.p[0];
    c.prompt_buf[2 * slot + 1] = c.p[1];
    c.cn0_counter++;
    const float raw = cn0_m2m4(c.prompt_buf, ns, static_cast<float>(coh_integration_time_s));
    c.cn0_db_hz = smooth(c.cn0_sm, raw, k.cn0_alpha, k.cn0_one_minus_alpha, k.cn0_min_value, k.cn0_offset, k.cn0_init_samples);
    c.carrier_lock_test = smooth(c.lock_sm, carrier_lock_detector(c.prompt_buf), k.lock_alpha, k.lock_one_minus_alpha, k.lock_min_value,
        k.lock_offset, k.lock_init_samples);
    if (!c.pull_in) {
        if (static_cast<double>(c.carrier_lock_test) < k.conf.carrier_lock_th)
            c.carrier_fail++;
        else if (c.carrier_fail > 0)
            c.carrier_fail--;
        if (c.cn0_db_hz < static_cast<float>(k.conf.cn0_min))
            c.code_fail++;
        else if (c.code_fail > 0)
            c.code_fail--;
    }
    if (c.carrier_fail > k.conf.max_carrier_lock_fail || c.code_fail > k.conf.max_code_lock_fail) {
        c.carrier_fail = 0;
        c.code_fail = 0;
        return false;
    }
    return true;
}

// The loop filters and NCO update of one epoch (run_dll_pll, update_tracking_vars) on a register
// copy of the members they use: the persistent kernel loads it in one batch, computes without a
// memory round trip per member, and stores it back only if the lock test beside it passes.  The
// Tracking_loop_filter rings are kept in logical order (index 0 = newest).
struct LoopRegs {
    int32_t cloop, narrow, geo, pull_in;
    float p[2], e[2], l[2], ve[2], vl[2], spc;
    double carrier_phase_rate_step_rad;
    float p_old[2], fp_w, fp_x, rem_carr_phase_rad;
    float lfi[4], lfo[4];
    int32_t lf_idx, current_prn_length_samples;
    double carr_phase_error_hz, carr_error_filt_hz, carrier_doppler_hz, code_error_chips, code_error_filt_chips, code_freq_chips;
    double K_blk_samples, carrier_phase_step_rad, code_phase_step_chips, acc_carrier_phase_rad, rem_code_phase_samples, rem_code_phase_chips;
    LoopSet q;
};

// A channel held in registers for a whole run (the fast persistent kernel, trk_fast.hip): every
// scalar member of TrkChannel the loop touches, the Tracking_loop_filter rings in logical order (as
// LoopRegs), and a pointer to the channel's memory copy (LDS) for what stays there — the sign
// history, and the lock-detector members (prompt buffer, CN0 / lock-test smoothers and fail
// counters), which another wave updates beside the loop update (lock_status).
struct RChan {
    int32_t state, geo, narrow, ext_count, cloop, pull_in, pll_180, acc_phase_init, sign_count;
    uint32_t prn;
    uint64_t acq_sample_stamp, nitems_read, epoch_start;
    double carrier_doppler_hz, carrier_phase_step_rad, code_freq_chips, code_phase_step_chips;
    double rem_code_phase_chips, rem_code_phase_samples, acc_carrier_phase_rad;
    double carr_phase_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips, K_blk_samples;
    double carrier_phase_rate_step_rad, code_phase_rate_step_chips;
    float rem_carr_phase_rad;
    int32_t current_prn_length_samples;
    float spc;
    float ve[2], e[2], p[2], l[2], vl[2], p_data[2], p_old[2];
    int32_t current_symbol, current_data_symbol;
    float lfi[4], lfo[4];
    int32_t lf_idx;
    float fp_w, fp_x;
    int32_t hist_head, hist_count;  // high_dyn rings are not on this path (kept for the shared templates)
    int64_t if_num;
    double if_cyc;
    TrkChannel* m;  // the memory copy: sign_bits and the lock-detector members
};

__device__ __forceinline__ const LoopSet& loopset(const TrkParams& k, const TrkChannel& c) { return k.ls[c.narrow ? 1 + c.geo : 0]; }
__device__ __forceinline__ const LoopSet& loopset(const TrkParams&, const LoopRegs& c) { return c.q; }
// RChan lives in a whole wave's registers with the same value in every lane: indices into the
// parameter block go through readfirstlane so that the compiler reads it with scalar loads instead
// of one vector load per lane on the critical path.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ const LoopSet& loopset(const TrkParams& k, const RChan& c) { return k.ls[uni(c.narrow ? 1 + c.geo : 0)]; }
__device__ __forceinline__ const SymSync& syncset(const TrkParams& k, const TrkChannel& c) { return k.sync[c.geo]; }
__device__ __forceinline__ const SymSync& syncset(const TrkParams& k, const RChan& c) { return k.sync[uni(c.geo)]; }
__device__ __forceinline__ const SymSync& syncset(const TrkParams& k, const LoopRegs& c) { return k.sync[c.geo]; }

// The parameters one channel's loop reads, as register values for a whole run (the fast kernel's
// control wave): inside the epoch loop every TrkParams member is otherwise a dependent scalar load on
// the epoch's critical chain.  The member names are TrkParams's, so the loop templates read either;
// the channel's symbol-sync profile and its wide / narrow loop sets are selected once (a channel's
// geo profile is fixed from start_tracking on), the secondary-code bit tables stay in memory.
struct KFastConf {
    double fs_in;
    uint32_t pull_in_time_s, bit_synchronization_time_limit_s, smoother_length;
    int32_t enable_fll_pull_in, enable_fll_steady_state, carrier_aiding;
    float slope, y_intercept, early_late_space_chips;
};
struct SyncView {
    int32_t symbols_per_bit, secondary, secondary_len, data_secondary_len, extend;
    float T_ext;
    const uint32_t* secondary_bits;
    const uint32_t* data_secondary_bits;
};
struct KFast {
    KFastConf conf;
    double code_chip_rate, carrier_freq, code_period, if_step_rad;
    int64_t if_mod, fs_int;
    double inv_fs, inv_carrier_freq;
    int32_t code_length_chips, veml, track_pilot, fp_order, has_if;
    float spc_n;
    LoopSet ls_w, ls_n;  // the wide set and this channel's narrow set (k.ls[0], k.ls[1 + geo])
    SyncView sv;         // k.sync[geo]
};
__device__ __forceinline__ KFast make_kfast(const TrkParams& k, int geo)
{
    KFast f;
    f.conf.fs_in = k.conf.fs_in;
    f.conf.pull_in_time_s = k.conf.pull_in_time_s;
    f.conf.bit_synchronization_time_limit_s = k.conf.bit_synchronization_time_limit_s;
    f.conf.smoother_length = k.conf.smoother_length;
    f.conf.enable_fll_pull_in = k.conf.enable_fll_pull_in;
    f.conf.enable_fll_steady_state = k.conf.enable_fll_steady_state;
    f.conf.carrier_aiding = k.conf.carrier_aiding;
    f.conf.slope = k.conf.slope;
    f.conf.y_intercept = k.conf.y_intercept;
    f.conf.early_late_space_chips = k.conf.early_late_space_chips;
    f.code_chip_rate = k.code_chip_rate;
    f.carrier_freq = k.carrier_freq;
    f.code_period = k.code_period;
    f.if_step_rad = k.if_step_rad;
    f.if_mod = k.if_mod;
    f.fs_int = k.fs_int;
    f.inv_fs = k.inv_fs;
    f.inv_carrier_freq = k.inv_carrier_freq;
    f.code_length_chips = k.code_length_chips;
    f.veml = k.veml;
    f.track_pilot = k.track_pilot;
    f.fp_order = k.fp_order;
    f.has_if = k.has_if;
    f.spc_n = k.spc_n;
    const int g = uni(geo);
    f.ls_w = k.ls[0];
    f.ls_n = k.ls[1 + g];
    const SymSync& s = k.sync[g];
    f.sv = SyncView{s.symbols_per_bit, s.secondary, s.secondary_len, s.data_secondary_len, s.extend, s.T_ext, s.secondary_bits, s.data_secondary_bits};
    return f;
}
__device__ __forceinline__ LoopSet loopset(const KFast& k, const RChan& c) { return uni(c.narrow) ? k.ls_n : k.ls_w; }
__device__ __forceinline__ const SyncView& syncset(const KFast& k, const RChan&) { return k.sv; }

// The members cn0_and_tracking_lock_status owns (prompt buffer, smoothers, fail counters, CN0 and
// lock test) and the sign history live in memory for both channel forms.
__device__ __forceinline__ TrkChannel& mem(TrkChannel& c) { return c; }
__device__ __forceinline__ const TrkChannel& mem(const TrkChannel& c) { return c; }
__device__ __forceinline__ TrkChannel& mem(RChan& c) { return *c.m; }
__device__ __forceinline__ const TrkChannel& mem(const RChan& c) { return *c.m; }

__device__ __forceinline__ void rchan_load(const TrkChannel& c, TrkChannel* mcopy, RChan& r)
{
    r.state = c.state;
    r.geo = c.geo;
    r.narrow = c.narrow;
    r.ext_count = c.ext_count;
    r.cloop = c.cloop;
    r.pull_in = c.pull_in;
    r.pll_180 = c.pll_180;
    r.acc_phase_init = c.acc_phase_init;
    r.sign_count = c.sign_count;
    r.prn = c.prn;
    r.acq_sample_stamp = c.acq_sample_stamp;
    r.nitems_read = c.nitems_read;
    r.epoch_start = c.epoch_start;
    r.carrier_doppler_hz = c.carrier_doppler_hz;
    r.carrier_phase_step_rad = c.carrier_phase_step_rad;
    r.code_freq_chips = c.code_freq_chips;
    r.code_phase_step_chips = c.code_phase_step_chips;
    r.rem_code_phase_chips = c.rem_code_phase_chips;
    r.rem_code_phase_samples = c.rem_code_phase_samples;
    r.acc_carrier_phase_rad = c.acc_carrier_phase_rad;
    r.carr_phase_error_hz = c.carr_phase_error_hz;
    r.carr_error_filt_hz = c.carr_error_filt_hz;
    r.code_error_chips = c.code_error_chips;
    r.code_error_filt_chips = c.code_error_filt_chips;
    r.K_blk_samples = c.K_blk_samples;
    r.carrier_phase_rate_step_rad = c.carrier_phase_rate_step_rad;
    r.code_phase_rate_step_chips = c.code_phase_rate_step_chips;
    r.rem_carr_phase_rad = c.rem_carr_phase_rad;
    r.current_prn_length_samples = c.current_prn_length_samples;
    r.spc = c.spc;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        r.ve[i] = c.ve[i];
        r.e[i] = c.e[i];
        r.p[i] = c.p[i];
        r.l[i] = c.l[i];
        r.vl[i] = c.vl[i];
        r.p_data[i] = c.p_data[i];
        r.p_old[i] = c.p_old[i];
    }
    r.current_symbol = c.current_symbol;
    r.current_data_symbol = c.current_data_symbol;
    r.lf_idx = c.lf_idx;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        r.lfi[i] = c.lf_inputs[(c.lf_idx + i) & 3];
        r.lfo[i] = c.lf_outputs[(c.lf_idx + i) & 3];
    }
    r.fp_w = c.fp_w;
    r.fp_x = c.fp_x;
    r.hist_head = c.hist_head;
    r.hist_count = c.hist_count;
    r.if_num = c.if_num;
    r.if_cyc = c.if_cyc;
    r.m = mcopy;
}

// The register members back into the memory copy (the lock-detector members and sign bits are
// there already).
__device__ __forceinline__ void rchan_store(const RChan& r, TrkChannel& c)
{
    c.state = r.state;
    c.geo = r.geo;
    c.narrow = r.narrow;
    c.ext_count = r.ext_count;
    c.cloop = r.cloop;
    c.pull_in = r.pull_in;
    c.pll_180 = r.pll_180;
    c.acc_phase_init = r.acc_phase_init;
    c.sign_count = r.sign_count;
    c.prn = r.prn;
    c.acq_sample_stamp = r.acq_sample_stamp;
    c.nitems_read = r.nitems_read;
    c.epoch_start = r.epoch_start;
    c.carrier_doppler_hz = r.carrier_doppler_hz;
    c.carrier_phase_step_rad = r.carrier_phase_step_rad;
    c.code_freq_chips = r.code_freq_chips;
    c.code_phase_step_chips = r.code_phase_step_chips;
    c.rem_code_phase_chips = r.rem_code_phase_chips;
    c.rem_code_phase_samples = r.rem_code_phase_samples;
    c.acc_carrier_phase_rad = r.acc_carrier_phase_rad;
    c.carr_phase_error_hz = r.carr_phase_error_hz;
    c.carr_error_filt_hz = r.carr_error_filt_hz;
    c.code_error_chips = r.code_error_chips;
    c.code_error_filt_chips = r.code_error_filt_chips;
    c.K_blk_samples = r.K_blk_samples;
    c.carrier_phase_rate_step_rad = r.carrier_phase_rate_step_rad;
    c.code_phase_rate_step_chips = r.code_phase_rate_step_chips;
    c.rem_carr_phase_rad = r.rem_carr_phase_rad;
    c.current_prn_length_samples = r.current_prn_length_samples;
    c.spc = r.spc;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        c.ve[i] = r.ve[i];
        c.e[i] = r.e[i];
        c.p[i] = r.p[i];
        c.l[i] = r.l[i];
        c.vl[i] = r.vl[i];
        c.p_data[i] = r.p_data[i];
        c.p_old[i] = r.p_old[i];
    }
    c.current_symbol = r.current_symbol;
    c.current_data_symbol = r.current_data_symbol;
    c.lf_idx = r.lf_idx;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        c.lf_inputs[(r.lf_idx + i) & 3] = r.lfi[i];
        c.lf_outputs[(r.lf_idx + i) & 3] = r.lfo[i];
    }
    c.fp_w = r.fp_w;
    c.fp_x = r.fp_x;
    c.hist_head = r.hist_head;
    c.hist_count = r.hist_count;
    c.if_num = r.if_num;
    c.if_cyc = r.if_cyc;
}

__device__ __forceinline__ void load_regs(const TrkParams& k, const TrkChannel& c, LoopRegs& r)
{
    r.cloop = c.cloop;
    r.narrow = c.narrow;
    r.geo = c.geo;
    r.pull_in = c.pull_in;
    for (int i = 0; i < 2; i++) {
        r.p[i] = c.p[i];
        r.e[i] = c.e[i];
        r.l[i] = c.l[i];
        r.ve[i] = c.ve[i];
        r.vl[i] = c.vl[i];
        r.p_old[i] = c.p_old[i];
    }
    r.spc = c.spc;
    r.carrier_phase_rate_step_rad = c.carrier_phase_rate_step_rad;
    r.fp_w = c.fp_w;
    r.fp_x = c.fp_x;
    r.rem_carr_phase_rad = c.rem_carr_phase_rad;
    r.lf_idx = c.lf_idx;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        r.lfi[i] = c.lf_inputs[(c.lf_idx + i) & 3];
        r.lfo[i] = c.lf_outputs[(c.lf_idx + i) & 3];
    }
    r.current_prn_length_samples = c.current_prn_length_samples;
    r.carr_phase_error_hz = c.carr_phase_error_hz;
    r.carr_error_filt_hz = c.carr_error_filt_hz;
    r.carrier_doppler_hz = c.carrier_doppler_hz;
    r.code_error_chips = c.code_error_chips;
    r.code_error_filt_chips = c.code_error_filt_chips;
    r.code_freq_chips = c.code_freq_chips;
    r.K_blk_samples = c.K_blk_samples;
    r.carrier_phase_step_rad = c.carrier_phase_step_rad;
    r.code_phase_step_chips = c.code_phase_step_chips;
    r.acc_carrier_phase_rad = c.acc_carrier_phase_rad;
    r.rem_code_phase_samples = c.rem_code_phase_samples;
    r.rem_code_phase_chips = c.rem_code_phase_chips;
    r.q = loopset(k, c);
}

// The members run_dll_pll / update_tracking_vars write.
__device__ __forceinline__ void store_regs(const LoopRegs& r, TrkChannel& c)
{
    c.p_old[0] = r.p_old[0];
    c.p_old[1] = r.p_old[1];
    c.fp_w = r.fp_w;
    c.fp_x = r.fp_x;
    c.rem_carr_phase_rad = r.rem_carr_phase_rad;
    c.lf_idx = r.lf_idx;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        c.lf_inputs[(r.lf_idx + i) & 3] = r.lfi[i];
        c.lf_outputs[(r.lf_idx + i) & 3] = r.lfo[i];
    }
    c.current_prn_length_samples = r.current_prn_length_samples;
    c.carr_phase_error_hz = r.carr_phase_error_hz;
    c.carr_error_filt_hz = r.carr_error_filt_hz;
    c.carrier_doppler_hz = r.carrier_doppler_hz;
    c.code_error_chips = r.code_error_chips;
    c.code_error_filt_chips = r.code_error_filt_chips;
    c.code_freq_chips = r.code_freq_chips;
    c.K_blk_samples = r.K_blk_samples;
    c.carrier_phase_step_rad = r.carrier_phase_step_rad;
    c.code_phase_step_chips = r.code_phase_step_chips;
    c.acc_carrier_phase_rad = r.acc_carrier_phase_rad;
    c.rem_code_phase_samples = r.rem_code_phase_samples;
    c.rem_code_phase_chips = r.rem_code_phase_chips;
}

__device__ GNSSHIP_LOOP_INLINE float loop_filter_apply(const TrkParams& k, TrkChannel& c, float x)
{
    const LoopSet& q = loopset(k, c);
    float result = 0.0f;
    for (int ii = 0; ii < q.lf_n_out; ii++) result = __fadd_rn(result, __fmul_rn(q.lf_out[ii], c.lf_outputs[(c.lf_idx + ii) % 4]));
    c.lf_idx--;
    if (c.lf_idx < 0) c.lf_idx += 4;
    c.lf_inputs[c.lf_idx] = x;
    for (int ii = 0; ii < q.lf_n_in; ii++) result = __fadd_rn(result, __fmul_rn(q.lf_in[ii], c.lf_inputs[(c.lf_idx + ii) % 4]));
    c.lf_outputs[c.lf_idx] = result;
    return result;
}

// Tracking_loop_filter::apply (tracking_loop_filter.cc:58-84) on the logical-order rings: the same
// products in the same order (outputs[(idx+ii)%4] ≡ lfo[ii] before the insert, inputs[(idx'+ii)%4] ≡
// lfi[ii] after it).
template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE float loop_filter_apply(const K& k, C& c, float x)
{
    const LoopSet& q = loopset(k, c);
    float result = 0.0f;
#pragma unroll
    for (int ii = 0; ii < 3; ii++)
        if (ii < q.lf_n_out) result = __fadd_rn(result, __fmul_rn(q.lf_out[ii], c.lfo[ii]));
    c.lf_idx = (c.lf_idx + 3) & 3;
#pragma unroll
    for (int ii = 3; ii > 0; ii--) c.lfi[ii] = c.lfi[ii - 1];
    c.lfi[0] = x;
#pragma unroll
    for (int ii = 0; ii < 4; ii++)
        if (ii < q.lf_n_in) result = __fadd_rn(result, __fmul_rn(q.lf_in[ii], c.lfi[ii]));
#pragma unroll
    for (int ii = 3; ii > 0; ii--) c.lfo[ii] = c.lfo[ii - 1];
    c.lfo[0] = result;
    return result;
}

template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE float carrier_filter(const K& k, C& c, float fll, float pll, float T)
{
    const LoopSet& q = loopset(k, c);
    if (k.fp_order == 3) {
        c.fp_w = __fadd_rn(c.fp_w, __fmul_rn(T, __fadd_rn(__fmul_rn(q.fp_w0p3, pll), __fmul_rn(q.fp_w0f2, fll))));
        const float inner = __fadd_rn(__fadd_rn(__fmul_rn(0.5f, c.fp_w), __fmul_rn(__fmul_rn(q.fp_a2, q.fp_w0f), fll)),
            __fmul_rn(__fmul_rn(q.fp_a3, q.fp_w0p2), pll));
        c.fp_x = __fadd_rn(c.fp_x, __fmul_rn(T, inner));
        return __fadd_rn(__fmul_rn(0.5f, c.fp_x), __fmul_rn(__fmul_rn(q.fp_b3, q.fp_w0p), pll));
    }
    const float w_new = __fadd_rn(__fadd_rn(c.fp_w, __fmul_rn(__fmul_rn(pll, q.fp_w0p2), T)), __fmul_rn(__fmul_rn(fll, q.fp_w0f), T));
    const float e = __fadd_rn(__fmul_rn(0.5f, __fadd_rn(w_new, c.fp_w)), __fmul_rn(__fmul_rn(q.fp_a2, q.fp_w0p), pll));
    c.fp_w = w_new;
    return e;
}

// run_dll_pll's hook after the carrier filter set the Doppler (the fast kernel hands the next epoch's
// carrier step to its derive wave there); the default does nothing
struct NoDopplerHook {
    __device__ void operator()(double) const {}
};

// The PLL discriminator in Hz (:1065-1078): pll_cloop_two_quadrant_atan, or pll_four_quadrant_atan
// once the pilot is tracked (gr::fast_atan2f restated as atan2f, glibc_atanf.h), over 2π.
__device__ __forceinline__ double pll_error_hz(int cloop, float p0, float p1)
{
    double disc;
    if (cloop)
        disc = (p0 != 0.0f) ? static_cast<double>(glibc_atanf(__fdiv_rn(p1, p0))) : 0.0;
    else
        disc = static_cast<double>(glibc_atan2f(p1, p0));
    return div_2pi(disc);
}

// The DLL discriminator in chips (:1100-1110): dll_nc_vemlp_normalized or dll_nc_e_minus_l_normalized.
template <class K>
__device__ __forceinline__ double dll_error_chips(const K& k, const float* ve, const float* e, const float* l, const float* vl, float spc)
{
    if (k.veml) {
        const double early = static_cast<double>(sqrt_rn_f32(__fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(ve[0], ve[0]), __fmul_rn(ve[1], ve[1])),
                                                                          __fmul_rn(e[0], e[0])),
            __fmul_rn(e[1], e[1]))));
        const double late = static_cast<double>(sqrt_rn_f32(__fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(l[0], l[0]), __fmul_rn(l[1], l[1])),
                                                                         __fmul_rn(vl[0], vl[0])),
            __fmul_rn(vl[1], vl[1]))));
        const double s = early + late;
        return (s == 0.0) ? 0.0 : (early - late) / s;
    }
    const double pe = static_cast<double>(hypotf_glibc(e[0], e[1]));
    const double pl = static_cast<double>(hypotf_glibc(l[0], l[1]));
    const double s = pe + pl;
    const float slope = k.conf.slope;
    const float norm = __fdiv_rn(__fsub_rn(k.conf.y_intercept, __fmul_rn(slope, spc)), slope);
    return (s == 0.0) ? 0.0 : static_cast<double>(norm) * (pe - pl) / s;
}

// Both discriminators of an epoch evaluated ahead by other waves (the fast kernel's accumulator waves,
// from the same taps with the same operations); ok bit 0: pll, bit 1: dll.
struct PreDisc {
    double pll, dll;
    int ok;
};

template <class K, class C, class H = NoDopplerHook>
__device__ GNSSHIP_LOOP_INLINE void run_dll_pll(const K& k, C& c, const H& on_doppler = H{}, const PreDisc* pre = nullptr)
{
    c.carr_phase_error_hz = (pre && (pre->ok & 1)) ? pre->pll : pll_error_hz(c.cloop, c.p[0], c.p[1]);
    GNSSHIP_TRK_LOOP_STAMP(37);
    // d_current_correlation_time_s: the code period, or extend × code period once extended
    const float T = c.narrow ? syncset(k, c).T_ext : static_cast<float>(k.code_period);
    if ((c.pull_in && k.conf.enable_fll_pull_in) || k.conf.enable_fll_steady_state) {  // :1080-1097
        // d_current_correlation_time_s is a double: the code period, or (float)extend·(float)period
        const double Td = c.narrow ? static_cast<double>(syncset(k, c).T_ext) : k.code_period;
        const double fe = div_2pi(fll_diff_atan(c.p_old, c.p, 0.0, Td));
        c.p_old[0] = c.p[0];
        c.p_old[1] = c.p[1];
        const float pll = (c.pull_in && k.conf.enable_fll_pull_in) ? 0.0f : static_cast<float>(c.carr_phase_error_hz);
        c.carr_error_filt_hz = carrier_filter(k, c, static_cast<float>(fe), pll, T);
    } else {
        c.carr_error_filt_hz = carrier_filter(k, c, 0.0f, static_cast<float>(c.carr_phase_error_hz), T);
    }
    c.carrier_doppler_hz = c.carr_error_filt_hz;
    on_doppler(c.carrier_doppler_hz);
    GNSSHIP_TRK_LOOP_STAMP(38);
    c.code_error_chips = (pre && (pre->ok & 2)) ? pre->dll : dll_error_chips(k, c.ve, c.e, c.l, c.vl, c.spc);
    GNSSHIP_TRK_LOOP_STAMP(39);
    c.code_error_filt_chips = loop_filter_apply(k, c, static_cast<float>(c.code_error_chips));
    GNSSHIP_TRK_LOOP_STAMP(40);
    c.code_freq_chips = k.code_chip_rate - c.code_error_filt_chips;
    if (k.conf.carrier_aiding) c.code_freq_chips += div_carrier(k, c.carrier_doppler_hz * k.code_chip_rate);
}

// high_dyn rate estimate (:1208-1221, :1241-1254): mean step of the newest smoother_length entries
// minus the mean of the oldest, over the newest entries' samples; sums in the reference's order.
__device__ GNSSHIP_LOOP_INLINE double smoothed_rate(const TrkChannel& c, const TrkHist& h, const double* first, int L)
{
    const int cap = 2 * L;
    double cp1 = 0.0, cp2 = 0.0, samples = 0.0;
    for (int i = 0; i < L; i++) {
        int a = c.hist_head + i;
        if (a >= cap) a -= cap;
        int b = c.hist_head + cap - i - 1;
        if (b >= cap) b -= cap;
        cp1 += first[a];
        cp2 += first[b];
        samples += static_cast<double>(h.samples[b]);
    }
    cp1 /= static_cast<double>(L);
    cp2 /= static_cast<double>(L);
    return (cp2 - cp1) / samples;
}

// update_tracking_vars' carrier advance over the epoch's n samples and the new remainder phase
// (:1235-1245); the fast kernel's derive wave evaluates the same functions ahead of the loop.
__device__ __forceinline__ double carr_advance(double step, double rate, double n) { return step * n + 0.5 * rate * n * n; }
__device__ __forceinline__ float carr_rem_next(float rem, double adv)
{
    return static_cast<float>(fmod_2pi(static_cast<double>(__fadd_rn(rem, static_cast<float>(adv)))));
}

template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE void update_tracking_vars(const K& k, C& c, TrkHist* h)
{
    const double fs = k.conf.fs_in;
    const double T_chip = 1.0 / c.code_freq_chips;
    const double T_prn = T_chip * static_cast<double>(k.code_length_chips);
    const double T_prn_samples = T_prn * fs;
    c.K_blk_samples = T_prn_samples + c.rem_code_phase_samples;
    c.current_prn_length_samples = static_cast<int32_t>(floor(c.K_blk_samples));
    c.carrier_phase_step_rad = div_fs(k, kTwoPi * c.carrier_doppler_hz);
    const double n = static_cast<double>(c.current_prn_length_samples);
    c.code_phase_step_chips = div_fs(k, c.code_freq_chips);
    if constexpr (std::is_same<C, TrkChannel>::value) if (h) {  // high_dyn: push_back on the ring (full: drop the oldest), rates once it is full
        const int L = static_cast<int>(k.conf.smoother_length), cap = 2 * L;
        int slot;
        if (c.hist_count < cap) {
            slot = c.hist_head + c.hist_count;
            if (slot >= cap) slot -= cap;
            c.hist_count++;
        } else {
            slot = c.hist_head;
            c.hist_head = c.hist_head + 1 == cap ? 0 : c.hist_head + 1;
        }
        h->carr[slot] = c.carrier_phase_step_rad;
        h->code[slot] = c.code_phase_step_chips;
        h->samples[slot] = c.current_prn_length_samples;
        if (c.hist_count == cap) {
            c.carrier_phase_rate_step_rad = smoothed_rate(c, *h, h->carr, L);
            c.code_phase_rate_step_chips = smoothed_rate(c, *h, h->code, L);
        }
    }
    const double adv = carr_advance(c.carrier_phase_step_rad, c.carrier_phase_rate_step_rad, n);
    c.rem_carr_phase_rad = carr_rem_next(c.rem_carr_phase_rad, adv);
    c.acc_carrier_phase_rad -= adv;
    c.rem_code_phase_samples = c.K_blk_samples - n;
    c.rem_code_phase_chips = div_fs(k, c.code_freq_chips * c.rem_code_phase_samples);
}

__device__ __forceinline__ int bit_at(const uint32_t* bits, int i) { return (bits[i >> 5] >> (i & 31)) & 1; }

template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE void push_sign(const K& k, C& c, float prompt_re)
{
    const int cap = syncset(k, c).secondary_len;
    const uint32_t neg = prompt_re < 0.0f ? 1u : 0u;
    uint32_t* bits = mem(c).sign_bits;
    if (c.sign_count == cap) {  // boost::circular_buffer::push_back on a full buffer drops the oldest
        for (int w = 0; w < kTrkMaxSecondary / 32; w++) {
            const uint32_t carry = (w + 1 < kTrkMaxSecondary / 32) ? (bits[w + 1] & 1u) : 0u;
            bits[w] = (bits[w] >> 1) | (carry << 31);
        }
        const int i = cap - 1;
        bits[i >> 5] = (bits[i >> 5] & ~(1u << (i & 31))) | (neg << (i & 31));
    } else {
        const int i = c.sign_count++;
        bits[i >> 5] = (bits[i >> 5] & ~(1u << (i & 31))) | (neg << (i & 31));
    }
}

template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE bool acquire_secondary(const K& k, C& c)
{
    int corr = 0;
    const uint32_t* bits = mem(c).sign_bits;
    for (int i = 0; i < syncset(k, c).secondary_len; i++) {
        const int neg = bit_at(bits, i);
        const int one = bit_at(syncset(k, c).secondary_bits, i);
        corr += (neg ^ one) ? 1 : -1;  // +1 for (real < 0, '0') and (real ≥ 0, '1')
    }
    if (abs(corr) == syncset(k, c).secondary_len) {
        c.pll_180 = corr < 0 ? 1 : 0;
        return true;
    }
    return false;
}

template <class C>
__device__ GNSSHIP_LOOP_INLINE void clear_tracking_vars(C& c)
{
    c.p_data[0] = c.p_data[1] = 0.0f;
    c.p_old[0] = c.p_old[1] = 0.0f;
    c.carr_phase_error_hz = 0.0;
    c.carr_error_filt_hz = 0.0;
    c.code_error_chips = 0.0;
    c.code_error_filt_chips = 0.0;
    c.current_symbol = 0;
    c.current_data_symbol = 0;
    c.sign_count = 0;
    c.carrier_phase_rate_step_rad = 0.0;  // :1182-1185
    c.code_phase_rate_step_chips = 0.0;
    c.hist_head = 0;
    c.hist_count = 0;
}

__device__ __forceinline__ void cadd(float* acc, const float* v, float sgn)
{
    acc[0] = __fadd_rn(acc[0], __fmul_rn(sgn, v[0]));
    acc[1] = __fadd_rn(acc[1], __fmul_rn(sgn, v[1]));
}

template <class C>
__device__ GNSSHIP_LOOP_INLINE void zero_accu(C& c)
{
    c.ve[0] = c.ve[1] = c.e[0] = c.e[1] = c.p[0] = c.p[1] = 0.0f;
    c.l[0] = c.l[1] = c.vl[0] = c.vl[1] = 0.0f;
}

// log_data (:1376-1466) at epoch start nir, after update_tracking_vars.
template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE void log_data(const K& k, const C& c, const float* taps, const float* pdata, uint64_t nir, gnsship_trk_dump_record* d)
{
    if (!d) return;
    const int eo = k.veml ? 2 : 0;
    const float* prompt = k.track_pilot ? pdata : taps + eo + 2;
    const double fs = k.conf.fs_in;
    d->abs_VE = k.veml ? hypotf_glibc(c.ve[0], c.ve[1]) : 0.0f;
    d->abs_E = hypotf_glibc(c.e[0], c.e[1]);
    d->abs_P = hypotf_glibc(c.p[0], c.p[1]);
    d->abs_L = hypotf_glibc(c.l[0], c.l[1]);
    d->abs_VL = k.veml ? hypotf_glibc(c.vl[0], c.vl[1]) : 0.0f;
    d->prompt_I = prompt[0];
    d->prompt_Q = prompt[1];
    d->PRN_start_sample_count = nir + static_cast<uint64_t>(c.current_prn_length_samples);
    d->acc_carrier_phase_rad = static_cast<float>(c.acc_carrier_phase_rad);
    d->carrier_doppler_hz = static_cast<float>(c.carrier_doppler_hz);
    d->carrier_doppler_rate_hz = static_cast<float>(c.carrier_phase_rate_step_rad * fs * fs / kTwoPi);
    d->code_freq_chips = static_cast<float>(c.code_freq_chips);
    d->code_freq_rate_chips = static_cast<float>(c.code_phase_rate_step_chips * fs * fs);
    d->carr_error_hz = static_cast<float>(c.carr_phase_error_hz);
    d->carr_error_filt_hz = static_cast<float>(c.carr_error_filt_hz);
    d->code_error_chips = static_cast<float>(c.code_error_chips);
    d->code_error_filt_chips = static_cast<float>(c.code_error_filt_chips);
    d->CN0_SNV_dB_Hz = mem(c).cn0_db_hz;
    d->carrier_lock_test = mem(c).carrier_lock_test;
    d->aux1 = static_cast<float>(c.rem_code_phase_samples);
    d->aux2 = static_cast<double>(nir + static_cast<uint64_t>(c.current_prn_length_samples));
    d->PRN = c.prn;
}

// One general_work call is split in phases so that the persistent kernel can run the lock
// detectors beside the loop filters (the two share no state):
//   epoch_pre    — pull-in timer, the epoch's correlations into the accumulators (state 2: copy,
//                  states 3/4: save_correlation_results) and all of state 3 (no lock test there);
//                  returns the coherent integration time lock_status is called with, or 0;
//   lock_status  — cn0_and_tracking_lock_status (:972-1029);
//   epoch_loop   — run_dll_pll + update_tracking_vars (:1065-1260), which the reference runs only
//                  when the lock test passes (the persistent kernel runs it speculatively beside
//                  the lock test on a LoopRegs copy and keeps it only on a pass);
//   epoch_post   — the rest of the state's branch given the lock outcome;
//   epoch_finish — the epoch record's loop outputs and consume_each.
// The pull-in and bit-synchronisation timers compare whole seconds of samples:
// `limit < (nir − stamp) / fs` ⟺ `nir − stamp ≥ (limit + 1)·fs` (unsigned, exact), no 64-bit division.
__device__ __forceinline__ bool seconds_exceed(uint64_t elapsed, uint32_t limit_s, uint64_t fs_int)
{
    return elapsed >= (static_cast<uint64_t>(limit_s) + 1u) * fs_int;
}

// (i + 1) % n for a counter kept in [0, n) — the reference's modulo without an integer division
// (any other value still takes the division, so the result is (i + 1) % n for every i ≥ 0)
__device__ __forceinline__ int next_mod(int i, int n)
{
    const int v = i + 1;
    return v < n ? v : (v == n ? 0 : v % n);
}

template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE double epoch_pre(const K& k, C& c, const float* taps, const float* pdata, gnsship_trk_epoch& rec, TrkHist* h,
    gnsship_trk_dump_record* dump)
{
    const uint64_t nir = c.epoch_start;
    const uint64_t fs_int = static_cast<uint64_t>(static_cast<int>(k.conf.fs_in));
    rec.sample_counter = nir;
    if (c.pull_in && seconds_exceed(nir - c.acq_sample_stamp, k.conf.pull_in_time_s, fs_int)) {
        c.pull_in = 0;
        mem(c).carrier_fail = 0;
        mem(c).code_fail = 0;
    }
    const int eo = k.veml ? 2 : 0;
    const int st = c.state;
    rec.state = st;
    if (st == 2) {
        if (k.veml) {
            c.ve[0] = taps[0];
            c.ve[1] = taps[1];
            c.vl[0] = taps[8];
            c.vl[1] = taps[9];
        }
        c.e[0] = taps[eo];
        c.e[1] = taps[eo + 1];
        c.p[0] = taps[eo + 2];
        c.p[1] = taps[eo + 3];
        c.l[0] = taps[eo + 4];
        c.l[1] = taps[eo + 5];
        c.spc = k.conf.early_late_space_chips;
        rec.prompt_i = static_cast<double>(c.p[0]);  // diagnostic: the epoch's prompt (no symbol flag in state 2)
        rec.prompt_q = static_cast<double>(c.p[1]);
        if (seconds_exceed(nir - c.acq_sample_stamp, k.conf.bit_synchronization_time_limit_s, fs_int)) mem(c).carrier_fail = 300000;
        return k.code_period;
    }
    // save_correlation_results
    float sgn = 1.0f;
    if (syncset(k, c).secondary) {
        sgn = bit_at(syncset(k, c).secondary_bits, c.current_symbol) ? -1.0f : 1.0f;
        c.current_symbol = next_mod(c.current_symbol, syncset(k, c).secondary_len);
    }
    if (k.veml) {
        cadd(c.ve, taps, sgn);
        cadd(c.vl, taps + 8, sgn);
    }
    cadd(c.e, taps + eo, sgn);
    cadd(c.p, taps + eo + 2, sgn);
    cadd(c.l, taps + eo + 4, sgn);
    const float* src = k.track_pilot ? pdata : taps + eo + 2;
    if (syncset(k, c).symbols_per_bit > 1) {
        if (syncset(k, c).data_secondary_len > 0) {
            cadd(c.p_data, src, bit_at(syncset(k, c).data_secondary_bits, c.current_data_symbol) ? -1.0f : 1.0f);
            c.current_data_symbol = next_mod(c.current_data_symbol, syncset(k, c).data_secondary_len);
        } else {
            cadd(c.p_data, src, 1.0f);
            c.current_data_symbol = next_mod(c.current_data_symbol, syncset(k, c).symbols_per_bit);
        }
    } else {
        c.p_data[0] = src[0];
        c.p_data[1] = src[1];
    }
    c.cloop = k.track_pilot ? 0 : 1;
    if (st == 3) {  // coherent integration (:1933-1970): accumulate, NCO advance only
        update_tracking_vars(k, c, h);
        if (c.current_data_symbol == 0) {
            log_data(k, c, taps, pdata, nir, dump);
            rec.flags |= 16;
            rec.prompt_i = static_cast<double>(c.p_data[0]);
            rec.prompt_q = static_cast<double>(c.p_data[1]);
            rec.flags |= 1;
            c.p_data[0] = c.p_data[1] = 0.0f;
        }
        c.ext_count++;
        if (c.ext_count == syncset(k, c).extend - 1) {
            c.ext_count = 0;
            c.state = 4;
        }
        return 0.0;
    }
    return k.code_period * static_cast<double>(syncset(k, c).extend);
}

template <class K, class C, class H = NoDopplerHook>
__device__ __forceinline__ void epoch_loop(const K& k, C& c, TrkHist* h, const H& on_doppler = H{}, const PreDisc* pre = nullptr)
{
    GNSSHIP_TRK_LOOP_STAMP(9);
    run_dll_pll(k, c, on_doppler, pre);
    GNSSHIP_TRK_LOOP_STAMP(10);
    update_tracking_vars(k, c, h);
    GNSSHIP_TRK_LOOP_STAMP(11);
}

// After epoch_pre returned a coherent time: the rest of state 2 / 4 given the lock outcome (epoch_loop
// has run iff locked).
template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE void epoch_post(const K& k, C& c, const float* taps, const float* pdata, gnsship_trk_epoch& rec, bool locked,
    gnsship_trk_dump_record* dump)
{
    const uint64_t nir = c.epoch_start;
    const int eo = k.veml ? 2 : 0;
    if (!locked) {
        clear_tracking_vars(c);
        c.state = 0;
        rec.flags |= 2;
        return;
    }
    if (c.state == 2) {
        bool next_state = false;
        log_data(k, c, taps, pdata, nir, dump);
        GNSSHIP_TRK_LOOP_STAMP(12);
        rec.flags |= 16;
        if (!c.pull_in) {
            if (syncset(k, c).secondary || syncset(k, c).symbols_per_bit > 1) {
                push_sign(k, c, taps[eo + 2]);
                if (c.sign_count == syncset(k, c).secondary_len) next_state = acquire_secondary(k, c);
            } else {
                next_state = true;
            }
        }
        if (next_state) {
            zero_accu(c);
            c.p_data[0] = c.p_data[1] = 0.0f;
            c.sign_count = 0;
            c.current_symbol = 0;
            c.current_data_symbol = 0;
            if (syncset(k, c).extend > 1) {  // extended integration (:1890-1926): narrow loops and taps, state 3
                c.ext_count = 0;
                c.narrow = 1;
                c.spc = k.spc_n;
                c.state = 3;
            } else {
                c.state = 4;
            }
        }
        return;
    }
    // state 4 (:1971-2028)
    if (!c.acc_phase_init) {
        c.acc_carrier_phase_rad = -static_cast<double>(c.rem_carr_phase_rad);
        c.acc_phase_init = 1;
    }
    if (c.current_data_symbol == 0) {
        log_data(k, c, taps, pdata, nir, dump);
        rec.flags |= 16;
        rec.prompt_i = static_cast<double>(c.p_data[0]);
        rec.prompt_q = static_cast<double>(c.p_data[1]);
        rec.flags |= 1;
        c.p_data[0] = c.p_data[1] = 0.0f;
    }
    zero_accu(c);
    if (syncset(k, c).extend > 1) c.state = 3;  // next coherent integration cycle
}

template <class K, class C>
__device__ __forceinline__ void advance_if(const K& k, C& c, int32_t consumed);

// consume_each (:2061) and the IF phase of the consumed samples.
template <class K, class C>
__device__ __forceinline__ void epoch_consume(const K& k, C& c)
{
    c.nitems_read = c.epoch_start + static_cast<uint64_t>(c.current_prn_length_samples);
    advance_if(k, c, c.current_prn_length_samples);
}

// The record's loop outputs and consume_each (:2061); false when the channel stopped (loss of lock).
// consume = false: the caller has already run epoch_consume (the fast kernel's early seed).
template <class K, class C>
__device__ GNSSHIP_LOOP_INLINE bool epoch_finish(const K& k, C& c, gnsship_trk_epoch& rec, bool consume = true)
{
    if (c.pll_180) rec.flags |= 4;
    rec.code_phase_samples = c.rem_code_phase_samples;
    rec.carrier_phase_rads = c.acc_carrier_phase_rad;
    rec.carrier_doppler_hz = c.carrier_doppler_hz;
    rec.cn0_db_hz = static_cast<double>(mem(c).cn0_db_hz);
    rec.carrier_lock_test = mem(c).carrier_lock_test;
    rec.code_freq_chips = c.code_freq_chips;
    rec.rem_code_phase_chips = c.rem_code_phase_chips;
    rec.rem_carr_phase_rad = c.rem_carr_phase_rad;
    rec.prn_length_samples = c.current_prn_length_samples;
    if (rec.flags & 2) return false;
    if (consume) epoch_consume(k, c);
    return true;
}

// The IF phase follows the consumed samples (gnsship_trk_conf::if_hz): if_num += if_mod·len (mod fs).
template <class K, class C>
__device__ __forceinline__ void advance_if(const K& k, C& c, int32_t consumed)
{
    if (!k.has_if) return;
    c.if_num = (c.if_num + k.if_mod * static_cast<int64_t>(consumed)) % k.fs_int;
    c.if_cyc = static_cast<double>(c.if_num) / static_cast<double>(k.fs_int);
}

// do_correlation_step's carrier arguments with the IF fused in (include/gnsship.h if_hz): the
// correlator wipes off IF + Doppler, the loop keeps the IF-free quantities.
template <class K, class C>
__device__ __forceinline__ float corr_rem_carr(const K& k, const C& c)
{
    if (!k.has_if) return c.rem_carr_phase_rad;
    return static_cast<float>(fmod_2pi(static_cast<double>(c.rem_carr_phase_rad) + kTwoPi * c.if_cyc));
}
template <class K, class C>
__device__ __forceinline__ float corr_phase_step(const K& k, const C& c)
{
    return static_cast<float>(c.carrier_phase_step_rad + k.if_step_rad);  // + 0.0 without IF: exact
}

// The phases in the reference's order on one lane (the round-based step kernel).
__device__ GNSSHIP_LOOP_INLINE bool epoch_update(const TrkParams& k, TrkChannel& c, const float* taps, const float* pdata, gnsship_trk_epoch& rec, TrkHist* h,
    gnsship_trk_dump_record* dump)
{
    const double coh = epoch_pre(k, c, taps, pdata, rec, h, dump);
    if (coh > 0.0) {
        GNSSHIP_TRK_LOOP_STAMP(8);
        const bool locked = lock_status(k, c, coh);
        if (locked) epoch_loop(k, c, h);
        epoch_post(k, c, taps, pdata, rec, locked, dump);
    }
    return epoch_finish(k, c, rec);
}

}  // namespace
}  // namespace gnsship
