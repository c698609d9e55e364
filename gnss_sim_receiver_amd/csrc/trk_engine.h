// trk_engine.h — internal types of the device-resident tracking loop (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "engine.h"
#include "gnsship.h"

namespace gnsship {

constexpr int kTrkMaxSecondary = 256;  // longest sign pattern searched (GPS preamble: 160 symbols)
constexpr int kTrkMaxCn0Samples = 64;  // prompt buffer of the CN0 / carrier-lock estimators
constexpr int kTrkMaxSmoother = 64;    // high_dyn: smoother_length bound (ring of 2·smoother_length)

// Signal constants the reference selects per system/signal (dll_pll_veml_tracking.cc:142-330,
// start_tracking :662-826) plus the loop-filter coefficients derived from Dll_Pll_Conf once.
struct LoopSet {
    float lf_in[4], lf_out[3];
    int32_t lf_n_in, lf_n_out;
    float fp_w0p3, fp_w0f2, fp_a2, fp_w0f, fp_a3, fp_w0p2, fp_b3, fp_w0p;
};

// Symbol synchronisation of one satellite class: the members start_tracking sets per PRN
// (:762-797).  Profile 0 is the system's; profile 1 the BeiDou B1I GEO one (PRN 1-5, 59+: D2
// navigation at 2 symbols per bit, 22-symbol preamble search, no NH code, extend capped at 2).
struct SymSync {
    int32_t symbols_per_bit, secondary, secondary_len, data_secondary_len;
    int32_t extend;   // d_extend_correlation_symbols (> 1: extended integration enabled)
    float T_ext;      // (float)extend · (float)code_period
    uint32_t secondary_bits[kTrkMaxSecondary / 32];       // bit i = character i == '1'
    uint32_t data_secondary_bits[kTrkMaxSecondary / 32];
};

struct TrkParams {
    gnsship_trk_conf conf;
    double code_chip_rate, carrier_freq, code_period;
    int32_t code_length_chips, code_samples_per_chip, veml, track_pilot, n_taps;
    SymSync sync[2];
    float shifts[5];                                        // d_local_code_shift_chips (× samples per chip)
    // Tracking_loop_filter (code) coefficients and Tracking_FLL_PLL_filter constants; set 1 + geo is
    // the narrow configuration of extended integration (:1902-1904) for sync profile geo
    LoopSet ls[3];
    int32_t fp_order;
    float shifts_n[5];   // narrow taps
    float spc_n;
    // Exponential_Smoother settings
    float cn0_alpha, cn0_one_minus_alpha, cn0_min_value, cn0_offset;
    int32_t cn0_init_samples;
    float lock_alpha, lock_one_minus_alpha, lock_min_value, lock_offset;
    int32_t lock_init_samples;
    // job layout
    int32_t jobs_per_channel;  // 1, or 2 with the E1 data prompt
    int32_t chunks_per_job;
    // carrier IF fused into the correlator NCO (gnsship_trk_conf::if_hz): 2π·if_hz/fs, and the IF phase
    // per sample as the exact fraction if_mod / fs_int of a cycle (0 ≤ if_mod < fs_int)
    int32_t has_if;
    int32_t pad_if;
    double if_step_rad;
    int64_t if_mod, fs_int;
    // RN(1/fs_in) and RN(1/carrier_freq): the loop's quotients by them as exact FMA sequences (exact_div.h)
    double inv_fs, inv_carrier_freq;
};

struct Smoother {
    float old_value, init_sum;
    int32_t initializing, counter;
};

// One channel: the dll_pll_veml_tracking members the per-epoch path reads or writes.
struct TrkChannel {
    int32_t state;  // 0 idle / lost, 2 wide tracking, 3 coherent integration, 4 narrow tracking
    int32_t geo;    // symbol-sync profile (TrkParams::sync): 1 for a BeiDou B1I GEO satellite
    uint32_t prn;   // Gnss_Synchro::PRN (dump records)
    int32_t narrow;     // loop set / taps in use (1 after entering extended integration)
    int32_t ext_count;  // d_extend_correlation_symbols_count
    int32_t cloop, pull_in, pll_180, ran, acc_phase_init;
    int32_t code_id, data_code_id;
    uint64_t acq_sample_stamp;
    uint64_t nitems_read;      // absolute index of the next input sample
    uint64_t epoch_start;      // nitems_read of the epoch whose correlation is in flight
    double carrier_doppler_hz, carrier_phase_step_rad, code_freq_chips, code_phase_step_chips;
    double rem_code_phase_chips, rem_code_phase_samples, acc_carrier_phase_rad;
    double carr_phase_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips, K_blk_samples;
    float rem_carr_phase_rad;
    int32_t current_prn_length_samples;
    float spc;
    float ve[2], e[2], p[2], l[2], vl[2], p_data[2];
    float p_old[2];  // d_P_accu_old (FLL discriminator)
    int32_t cn0_counter, carrier_fail, code_fail, current_symbol, current_data_symbol;
    float cn0_db_hz, carrier_lock_test;
    float prompt_buf[2 * kTrkMaxCn0Samples];
    uint32_t sign_bits[kTrkMaxSecondary / 32];  // d_Prompt_circular_buffer (real < 0), oldest first
    int32_t sign_count;
    // Tracking_loop_filter state
    float lf_inputs[4], lf_outputs[4];
    int32_t lf_idx;
    // Tracking_FLL_PLL_filter state
    float fp_w, fp_x;
    Smoother cn0_sm, lock_sm;
    // high_dyn (:1205-1255): the smoothed NCO rates and the ring state of TrkHist
    double carrier_phase_rate_step_rad, code_phase_rate_step_chips;
    int32_t hist_head, hist_count;
    // IF phase at nitems_read: if_num / fs_int cycles exactly (if_cyc = that quotient in double)
    int64_t if_num;
    double if_cyc;
};

// high_dyn: d_carr_ph_history and d_code_ph_history of one channel (boost::circular_buffer of
// capacity 2·smoother_length, :557-566).  Both are pushed together with the same sample count, so
// they share one ring; kept out of TrkChannel (which the step kernel holds in registers).
struct TrkHist {
    double carr[2 * kTrkMaxSmoother];
    double code[2 * kTrkMaxSmoother];
    int32_t samples[2 * kTrkMaxSmoother];
};

// One round: consume the previous epoch's correlations (when `consume`), then lay down the next
// epoch's jobs / chunk lengths for every channel whose window is in the buffer (when `emit`) and
// replay their rotator anchors into `anchors` (standard path; the correlation launch then runs
// only its CORRELATE stage).
// With high_dyn the epoch's correlations are high-dynamics jobs (hd_jobs / hd_chunks, the fixed
// HdPlan of the engine) and `hist` holds the channels' rate-smoother rings; otherwise all three are
// null and the jobs go to the standard correlator (jobs / chunks).
hipError_t launch_trk_step(const TrkParams* params, TrkChannel* chans, int n_chans, DevJob* jobs, ChunkDesc* chunks, const float* corr_out,
    uint64_t buf_first, int64_t buf_len, int consume, int emit, gnsship_trk_epoch* rec, gnsship_trk_dump_record* dump, int* ran_count,
    TrkHist* hist, HdJob* hd_jobs, HdChunk* hd_chunks, Anchor* anchors, hipStream_t stream);

// Persistent closed loop (trk_persist.hip): one workgroup per channel runs all of its epochs in the
// buffer within one launch (standard correlator only; not high_dyn).  code_cap_floats: LDS floats per
// code replica (padded_code_quads(max code length) · 4).  LDS bytes of the dynamic region:
size_t trk_persist_lds_bytes(const TrkParams& p, int code_cap_floats, bool avx);
// Tap layouts the persistent kernel is instantiated for (3 or 5 taps, the E1 data prompt with 5);
// others run the round-based loop (generic rotator only).
inline bool trk_persist_supports(const TrkParams& p)
{
    const bool data = p.jobs_per_channel > 1;
    return (p.n_taps == 3 && !data) || (p.n_taps == 5 && !data) || (p.n_taps == 5 && data);
}
constexpr size_t kTrkPersistMaxLds = 150 * 1024;  // of the 160 KiB per CU, beside the static state
hipError_t launch_trk_persist(const TrkParams* params_dev, const TrkParams& params, TrkChannel* chans, int n_chans, const CodeDesc* codes,
    int n_codes, int code_cap_floats, const void* samples, int fmt, uint64_t buf_first, int64_t buf_len, int max_rounds, gnsship_trk_epoch* rec,
    gnsship_trk_dump_record* dump, gnsship_trk_corr_trace* trace, int* ran_count, bool avx, hipStream_t stream);
// The latency-optimised persistent loop for the AVX rotator (trk_fast.hip): register-resident loop
// state, flagless phasor slots, lock detectors beside the loop update.
bool trk_fast_supported(const TrkParams& p, int code_cap_floats, int n_chans);
bool trk_fast_thru(int n_chans);  // the throughput form (more channels than CUs)
int trk_device_cus();             // compute units of the current device
// The throughput form with one 16-lane row per channel (trk_lane.hip): every code ±1 (codes_binary),
// the buffer addressable with 32-bit byte offsets; used above one channel per CU (GNSSHIP_TRK_LANE=0/1
// forces it off / on).
bool trk_lane_supported(const TrkParams& p, int code_cap_floats, int n_chans, int fmt, int64_t buf_len, bool codes_binary);
hipError_t launch_trk_lane(const TrkParams* params_dev, const TrkParams& params, TrkChannel* chans, int n_chans, const CodeDesc* codes, int n_codes,
    int code_cap_floats, const void* samples, int fmt, uint64_t buf_first, int64_t buf_len, int max_rounds, gnsship_trk_epoch* rec,
    gnsship_trk_dump_record* dump, gnsship_trk_corr_trace* trace, int* ran_count, hipStream_t stream);
hipError_t launch_trk_fast(const TrkParams* params_dev, const TrkParams& params, TrkChannel* chans, int n_chans, const CodeDesc* codes, int n_codes,
    int code_cap_floats, const void* samples, int fmt, uint64_t buf_first, int64_t buf_len, int max_rounds, gnsship_trk_epoch* rec,
    gnsship_trk_dump_record* dump, gnsship_trk_corr_trace* trace, int* ran_count, hipStream_t stream);

}  // namespace gnsship
