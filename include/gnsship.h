/*
 * gnsship.h — C ABI of the MI355X-native GNSS acquisition + tracking correlator engine.
 *
 * This is the drop-in boundary.  Everything behind it is HIP code for gfx950;
 * everything in front of it is plain C: opaque handles, plain pointers and sizes, int status
 * codes.  No exceptions, no exit(), no torch / STL types cross this boundary.
 *
 * What each group of entry points replaces in the reference (ShingoNishimoto/gnss_sim_receiver,
 * a GNSS-SDR v0.0.19 fork; paths relative to its root):
 *
 *  gnsship_corr_*       Cpu_Multicorrelator_Real_Codes
 *                         (src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.h:37-61,
 *                          .cc:36-167), i.e. volk_gnsssdr_32f_xn_resampler_32f_xn +
 *                          volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn, as called from
 *                          dll_pll_veml_tracking::do_correlation_step (dll_pll_veml_tracking.cc:1037-1062).
 *  gnsship_batch_*      The same correlation for many (channel, epoch) jobs in one launch: what
 *                         GNU Radio's thread-per-channel scheduling does across all channels.
 *  gnsship_acq_*        pcps_acquisition::set_local_code (pcps_acquisition.cc:175-208),
 *                         update_grid_doppler_wipeoffs (:295-302), acquisition_core (:600-871),
 *                         max_to_input_power_statistic / first_vs_second_peak_statistic (:496-597).
 *  gnsship_trk_*        dll_pll_veml_tracking::{start_tracking, general_work} (dll_pll_veml_tracking.cc:
 *                         643-883, 1728-2094) for many channels, the loop on the device.
 *  gnsship_comm_*       The flowgraph's fan-out of one signal-conditioner output to every channel
 *                         (gnss_flowgraph.cc:1127-1136) across GPUs: one RCCL communicator over
 *                         xGMI, the IF block broadcast from the reading rank, per-PRN acquisition
 *                         results all-gathered.
 *
 * Threading: handles are not re-entrant; distinct handles may be used from distinct threads
 * (each context owns one HIP stream).  All *_run calls are synchronous unless named *_launch.
 */
#ifndef GNSSHIP_H
#define GNSSHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: gnsship_trk_conf gained `rotator` and `if_hz` (a caller built against version 1 passes a shorter
 * struct — bindings compare gnsship_abi_version() with the header they were built from at load time). */
#define GNSSHIP_ABI_VERSION 2

/* ---- status codes (reference: bool-always-true + LOG/throw; here explicit) ---- */
#define GNSSHIP_OK 0
#define GNSSHIP_E_INVAL (-1)   /* bad argument / shape */
#define GNSSHIP_E_NOMEM (-2)   /* device or host allocation failed */
#define GNSSHIP_E_DEVICE (-3)  /* HIP runtime error (message in gnsship_last_error) */
#define GNSSHIP_E_STATE (-4)   /* call order violated (e.g. run before set_local_code) */
#define GNSSHIP_E_RCCL (-5)    /* RCCL (collective) error (message in gnsship_last_error)   */

/* ---- IF sample formats (reference item types: gr_complex, cshort, ibyte/cbyte) ---- */
#define GNSSHIP_FMT_CF32 0 /* interleaved float32 I,Q  (gr_complex)            */
#define GNSSHIP_FMT_CI16 1 /* interleaved int16  I,Q  (lv_16sc_t / cshort)      */
#define GNSSHIP_FMT_CI8 2  /* interleaved int8   I,Q  (ibyte/cbyte), no scaling  */

#define GNSSHIP_MAX_TAPS 8

/* ---- rotator dot-product variant (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn) ----
 * The reference's correlations depend on which volk_gnsssdr variant its dispatcher picks
 * (volk_gnsssdr_rank_archs.c): the generic C kernel (:66-98; VOLK_GENERIC set, or no AVX) or the
 * u_avx/a_avx kernel (:155-316; any AVX host without a volk_gnsssdr_config override): 16 phasors
 * advanced by normalise(inc^16), renormalised every 64 iterations.  The two differ by up to 1e-2
 * relative at 50 Msps with a 7 MHz IF, so the engine reproduces either one, selected per job / per
 * tracking engine.  Generic: the phasor chain and the serial float sum per tap component are
 * replayed in the reference's order (bit-identical taps; GNSSHIP_JOB_ROTATOR_TREE selects the faster
 * anchored tree sums for batch jobs).  AVX: all 16 phasor lanes are replayed and continued with the
 * reference's float products, in u_avx's accumulation order in the tracking engines (bit-identical taps).
 * Default in every binding (Python TrkConf.defaults, the C++ mirror's Dll_Pll_Conf, tools/gnsship_rx):
 * GNSSHIP_ROTATOR_AUTO, i.e. what the reference itself would run on this host. */
#define GNSSHIP_ROTATOR_GENERIC 0
#define GNSSHIP_ROTATOR_AVX 1
#define GNSSHIP_ROTATOR_AUTO (-1) /* what volk_gnsssdr dispatches on this host (gnsship_rotator_dispatch) */
/* gnsship_corr_job::flags bits */
#define GNSSHIP_JOB_HIGH_DYN 1     /* high-dynamics resampler + rotator (set_high_dynamics_resampler) */
#define GNSSHIP_JOB_ROTATOR_AVX 2  /* the AVX rotator variant (ignored with GNSSHIP_JOB_HIGH_DYN) */
/* Generic rotator with the anchored parallel sums (the phasor bit-identical at every renormalisation
 * point, the taps summed as a tree: within 1e-5 of the exact sum of the reference's float products,
 * not in its serial order).  Without this flag (and without _AVX / _HIGH_DYN) a job runs the
 * generic rotator in the reference's own order — one phasor chain and one serial float sum per tap
 * component, bit-identical taps (one workgroup per job, latency ≈ the N-step chain). */
#define GNSSHIP_JOB_ROTATOR_TREE 4
/* The variant volk_gnsssdr's dispatcher would select for the rotator dot-product on this host:
 * VOLK_GENERIC set in the environment -> generic; an entry for the kernel in the volk_gnsssdr
 * preferences file ($VOLK_CONFIGPATH or $HOME/.volk_gnsssdr/volk_gnsssdr_config) -> that entry
 * (its aligned and unaligned names are taken as the same variant: a_avx / u_avx and generic are
 * reproduced; any other entry, e.g. generic_reload, returns GNSSHIP_E_INVAL naming it in
 * gnsship_rotator_dispatch_detail); otherwise the AVX variant when the CPU has AVX.
 * *variant = GNSSHIP_ROTATOR_GENERIC / _AVX. */
int gnsship_rotator_dispatch(int* variant);
/* What the last gnsship_rotator_dispatch call on this thread matched (the environment, the
 * preferences file and its entry, or the CPU), as text. */
int gnsship_rotator_dispatch_detail(char* buf, int cap);

typedef struct gnsship_ctx gnsship_ctx;
typedef struct gnsship_corr gnsship_corr;
typedef struct gnsship_batch gnsship_batch;
typedef struct gnsship_acq gnsship_acq;

/* ------------------------------------------------------------------------------------------ */
/* Context: one HIP device + one stream + a code bank.                                        */
/* ------------------------------------------------------------------------------------------ */
int gnsship_abi_version(void);
int gnsship_device_count(int* n_devices);
int gnsship_ctx_create(int device, gnsship_ctx** out);
int gnsship_ctx_destroy(gnsship_ctx* ctx);
const char* gnsship_last_error(const gnsship_ctx* ctx);
int gnsship_ctx_sync(gnsship_ctx* ctx);
/* hipStream_t of the context, as void*, so a caller can order its own work against ours. */
int gnsship_ctx_stream(gnsship_ctx* ctx, void** stream);
/* HIP events recorded on the context stream (slots 0..15), for in-stream kernel timing. */
int gnsship_ctx_event_record(gnsship_ctx* ctx, int slot);
int gnsship_ctx_event_elapsed_ms(gnsship_ctx* ctx, int slot_begin, int slot_end, float* ms);

/* Device buffers (HBM).  The IF sample stream lives in one of these. */
int gnsship_dev_alloc(gnsship_ctx* ctx, size_t bytes, void** dev_ptr);
int gnsship_dev_free(gnsship_ctx* ctx, void* dev_ptr);
int gnsship_dev_upload(gnsship_ctx* ctx, void* dev_dst, const void* host_src, size_t bytes);
int gnsship_dev_download(gnsship_ctx* ctx, void* host_dst, const void* dev_src, size_t bytes);

/* Code bank: local code replicas (float, one value per code sample, e.g. 1023 for GPS C/A,
 * 8184 for Galileo E1 sinBOC(1,1) at 2 samples/chip).  Jobs refer to a code by its id.
 * Replaces the borrowed pointer of set_local_code_and_taps (cpu_multicorrelator_real_codes.cc:53-63):
 * the code is COPIED to the device. */
int gnsship_code_set(gnsship_ctx* ctx, int code_id, const float* code, int code_length);
int gnsship_code_count(gnsship_ctx* ctx, int* n_codes);

/* Local code replica generators (product side; reference src/algorithms/libs/ *_signal_replica.cc). */
/* gps_l1_ca_code_gen_float (gps_sdr_signal_replica.cc:113): dest[1023] = ±1 */
int gnsship_gps_l1_ca_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift);
/* gps_l1_ca_code_gen_complex_sampled (:145): dest = n complex (code in imag); returns n or <0 */
int gnsship_gps_l1_ca_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t sampling_freq, uint32_t chip_shift);
/* beidou_b1i_code_gen_float (beidou_b1i_signal_replica.cc:113): dest[2046] = ±1 */
int gnsship_beidou_b1i_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift);
/* beidou_b1i_code_gen_complex_sampled (:142): dest = n complex (code in real); returns n or <0 */
int gnsship_beidou_b1i_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t sampling_freq, uint32_t chip_shift);
/* samples per code period: (int)(fs / (chip_rate / code_len)) as the generators compute it */
int gnsship_code_samples_per_code(int32_t chip_rate, int32_t code_len, int32_t fs);

/* ------------------------------------------------------------------------------------------ */
/* Per-channel correlator: mirror of Cpu_Multicorrelator_Real_Codes.                          */
/* ------------------------------------------------------------------------------------------ */
/* init(max_signal_length_samples, n_correlators)  (cpu_multicorrelator_real_codes.cc:36-50) */
int gnsship_corr_create(gnsship_ctx* ctx, int max_signal_length_samples, int n_correlators, gnsship_corr** out);
/* set_local_code_and_taps(code_length_chips, local_code_in, shifts_chips)  (:53-63) */
int gnsship_corr_set_local_code_and_taps(gnsship_corr* c, int code_length_chips, const float* local_code_in, const float* shifts_chips);
/* set_high_dynamics_resampler (:163-167).  Default false, as Dll_Pll_Conf::high_dyn (dll_pll_conf.h:80). */
int gnsship_corr_set_high_dynamics_resampler(gnsship_corr* c, int enable);
/* Which volk_gnsssdr rotator variant the volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn call inside
 * Carrier_wipeoff_multicorrelator_resampler (:123-124) runs as: GNSSHIP_ROTATOR_GENERIC (the handle's
 * default; serial order, bit-identical taps), _AVX (u_avx: 16 phasor lanes) or _AUTO (what the
 * dispatcher would pick on this host, gnsship_rotator_dispatch; E_INVAL if it names a variant the
 * engine does not reproduce).  The C++ / Python mirrors default to _AUTO. */
int gnsship_corr_set_rotator(gnsship_corr* c, int variant);
/* Carrier_wipeoff_multicorrelator_resampler(...)  (:103-126).  `sig` is `fmt` samples; if
 * sig_on_device != 0 it is a device pointer (e.g. into a gnsship_dev_alloc ring), else host.
 * corr_out receives n_correlators complex<float> (2 floats each).  Synchronous. */
int gnsship_corr_run(gnsship_corr* c, const void* sig, int fmt, int sig_on_device,
    float rem_carrier_phase_in_rad, float phase_step_rad, float phase_rate_step_rad,
    float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* corr_out);
/* free()  (:147-160) */
int gnsship_corr_destroy(gnsship_corr* c);

/* ------------------------------------------------------------------------------------------ */
/* Batched correlation: many (channel, epoch) jobs per launch.                                */
/* ------------------------------------------------------------------------------------------ */
/* One job = one call of Carrier_wipeoff_multicorrelator_resampler for one channel-epoch.
 * NCO arguments carry the same meaning and float type as the reference call
 * (dll_pll_veml_tracking.cc:1041-1048): code phases are in code SAMPLES (chips × samples/chip). */
typedef struct gnsship_corr_job {
    int64_t sample_offset;   /* first IF sample of this epoch in the device sample buffer      */
    int32_t n_samples;       /* correlation length (vector_length)                            */
    int32_t code_id;         /* code bank id                                                   */
    int32_t n_taps;          /* 1..GNSSHIP_MAX_TAPS                                            */
    int32_t flags;           /* GNSSHIP_JOB_HIGH_DYN | GNSSHIP_JOB_ROTATOR_AVX | _TREE           */
    float rem_carrier_phase_rad;
    float phase_step_rad;
    float phase_rate_step_rad;
    float rem_code_phase_chips;
    float code_phase_step_chips;
    float code_phase_rate_step_chips;
    float shifts_chips[GNSSHIP_MAX_TAPS];
} gnsship_corr_job; /* 80 bytes */

int gnsship_batch_create(gnsship_ctx* ctx, int max_jobs, gnsship_batch** out);
/* Copy job descriptors host→device (validated on the host: shapes, code ids, bounds). */
int gnsship_batch_set_jobs(gnsship_batch* b, const gnsship_corr_job* jobs, int n_jobs, int64_t n_buffer_samples);
/* Enqueue the correlation of all jobs on the context stream; results stay on the device.
 * dev_samples: device IF buffer in `fmt`; n_buffer_samples bounds every job. Asynchronous. */
int gnsship_batch_launch(gnsship_batch* b, const void* dev_samples, int fmt);
/* Profiling split of gnsship_batch_launch: stages bit0 = rotator-anchor replay (NCO arguments
 * only), bit1 = correlation (+ chunk reduction).  3 == gnsship_batch_launch. */
#define GNSSHIP_STAGE_ANCHORS 1
#define GNSSHIP_STAGE_CORRELATE 2
int gnsship_batch_launch_stages(gnsship_batch* b, const void* dev_samples, int fmt, int stages);
/* Wait for the last launch and copy results: out[j*2*GNSSHIP_MAX_TAPS + 2*t + {0,1}] = tap t of job j. */
/* Correlate b and, inside the same launch, replay the rotator anchors of `next` (another batch of the
 * same context; NULL for none) — the double-buffered form of batch_launch for a pair of batches
 * alternated on the context stream, with no cross-stream event per launch.  b's own anchors come
 * from the previous launch that named it as `next` (or are computed first).  Do not mix with
 * gnsship_batch_launch_stages on the same batches. */
int gnsship_batch_launch_pipelined(gnsship_batch* b, const void* dev_samples, int fmt, gnsship_batch* next);
/* Three-batch ring form (A, B, C, A, ...): correlate b, finish the anchor replay of `next` and run
 * the first half of `next2`'s (each job's replay chain split at its middle renormalisation block),
 * so every launch carries half a replay chain per batch instead of a whole one.  next / next2 may
 * be NULL; next2 == NULL is gnsship_batch_launch_pipelined. */
int gnsship_batch_launch_pipelined2(gnsship_batch* b, const void* dev_samples, int fmt, gnsship_batch* next, gnsship_batch* next2);
int gnsship_batch_results(gnsship_batch* b, float* out);
/* Device pointer of the result array (n_jobs × GNSSHIP_MAX_TAPS complex<float>). */
int gnsship_batch_results_device(gnsship_batch* b, void** dev_out);
int gnsship_batch_destroy(gnsship_batch* b);

/* ------------------------------------------------------------------------------------------ */
/* PCPS acquisition.                                                                          */
/* ------------------------------------------------------------------------------------------ */
/* Mirror of the Acq_Conf fields the core reads (acq_conf.h:33-81). */
typedef struct gnsship_acq_conf {
    int64_t fs_in;              /* sampling rate [Sps] (resampled_fs when no resampler)    */
    int32_t fft_size;           /* d_fft_size = consumed samples (sampled_ms == ms_per_code) */
    int32_t doppler_max;        /* [Hz]                                                       */
    int32_t doppler_step;       /* [Hz]                                                       */
    int32_t doppler_center;     /* [Hz]                                                       */
    int32_t max_dwells;         /* non-coherent dwells accumulated into the grid              */
    int32_t use_cfar;           /* 1: max_to_input_power_statistic, 0: first_vs_second_peak   */
    int32_t samples_per_chip;   /* ceil(fs / chip_rate)                                       */
    float samples_per_code;     /* samples_per_ms * ms_per_code                               */
    int32_t max_prns;           /* number of local-code slots (PRNs searched per call)        */
    int32_t consumed_samples;   /* d_consumed_samples (:71): input samples per dwell, the rest of
                                   the fft_size buffer zero-padded (sampled_ms != ms_per_code:
                                   fft_size = 2 x consumed, :84-91); 0 = fft_size              */
    int32_t bit_transition_flag; /* code in the second half after N/2 zeros, grid rows = the
                                   second half of |IFFT|^2 (:187-192, :663-664)                 */
    float resampler_ratio;       /* acquisition resampler decimation (Acq_Conf::resampler_ratio,
                                   acq_conf.cc:91-107); 0 or 1 = no resampler. Acq_delay_samples
                                   is scaled by it and reduced by the latency (:686-687)        */
    uint32_t resampler_latency_samples; /* (taps - 1) / 2 of the resampler FIR (gnss_flowgraph.cc:1113) */
} gnsship_acq_conf;

/* What acquisition_core leaves in Gnss_Synchro + block members (pcps_acquisition.cc:683-696). */
typedef struct gnsship_acq_result {
    uint32_t doppler_index;      /* winning Doppler bin                                       */
    uint32_t code_index;         /* indext: winning FFT sample index                          */
    int32_t doppler_hz;          /* Acq_doppler_hz                                            */
    float peak;                  /* grid maximum (or first peak)                             */
    float input_power;           /* d_input_power (CFAR) / second peak (first_vs_second)     */
    float test_statistic;        /* d_test_statistics                                         */
    double acq_delay_samples;    /* fmod(indext, samples_per_code)·resampler_ratio − latency   */
} gnsship_acq_result;

int gnsship_acq_create(gnsship_ctx* ctx, const gnsship_acq_conf* conf, gnsship_acq** out);
/* Rebuild the Doppler wipeoff table (update_grid_doppler_wipeoffs): row i is exp(j*phi_n),
 * phi accumulated in float32 exactly as volk_gnsssdr_s32f_sincos_32fc_generic. */
int gnsship_acq_set_grid(gnsship_acq* a, int doppler_max, int doppler_step, int doppler_center);
/* set_local_code (:175-208): `code` is the sampled code, complex<float>: fft_size/2 values with
 * bit_transition_flag, else consumed_samples values (zero-padded in front to fft_size); FFT + conj on device. */
int gnsship_acq_set_local_code(gnsship_acq* a, int prn_slot, const float* code);
/* update_grid_doppler_wipeoffs_step2 (:305-312), make_2_steps: nb2 bins around the step-one Doppler.
 * Results then carry the step-two Doppler (:553-556); with CFAR the statistic divides by
 * step_one_input_power, as the reference leaves d_input_power at its step-one value (:516-525).
 * gnsship_acq_set_grid returns to step one. */
int gnsship_acq_set_grid_step2(gnsship_acq* a, float doppler_center_step_two, float doppler_step2, int num_doppler_bins_step2,
    float step_one_input_power);
/* acquisition_core over prn slots [0, n_prns): one dwell of fft_size samples, all bins.
 * results[n_prns]; grid (optional, host, n_prns*n_bins*fft_size floats) receives |IFFT|^2. */
int gnsship_acq_run(gnsship_acq* a, const void* sig, int fmt, int sig_on_device, int n_prns,
    gnsship_acq_result* results, float* grid);
int gnsship_acq_num_bins(gnsship_acq* a, int* n_bins);
/* Restart the non-coherent dwell accumulation (d_num_noncoherent_integrations_counter = 0 after a
 * decision, pcps_acquisition.cc:783,835,860-864): the next gnsship_acq_run is dwell 1. */
int gnsship_acq_reset_dwells(gnsship_acq* a);
int gnsship_acq_destroy(gnsship_acq* a);

/* Acquisition resampler (GNSS-SDR.use_acquisition_resampler; gnss_flowgraph.cc:1028-1113): the
 * decimating low-pass FIR in front of a channel's acquisition, and the Acq_Conf side
 * (ConfigureAutomaticResampler, acq_conf.cc:91-107).  Taps are GNU Radio's
 * firdes::low_pass(gain, fs, cutoff, transition) with the default Hamming window (GNU Radio is not
 * in the reference tree; restated from its published algorithm). */
typedef struct gnsship_acq_resampler gnsship_acq_resampler;
/* taps == NULL: only *n_taps.  E_INVAL for the arguments firdes rejects (sanity_check_1f). */
int gnsship_firdes_low_pass(double gain, double sampling_freq, double cutoff_freq, double transition_width, float* taps, int taps_cap,
    int* n_taps);
/* The flowgraph's design for a signal whose optimum acquisition rate is opt_acq_fs (e.g.
 * GPS_L1_CA_OPT_ACQ_FS_SPS = 2e6): decimation = floor(fs/opt) lowered until it divides fs, taps =
 * firdes::low_pass(1, fs, fs_dec/2.1, fs_dec/2).  *decimation = 1 and *n_taps = 0 when no resampler
 * is used (opt >= fs or decimation 1).  resampler_latency_samples = (n_taps - 1) / 2. */
int gnsship_acq_resampler_design(int64_t fs_in, double opt_acq_fs, int* decimation, float* taps, int taps_cap, int* n_taps);
/* fir_filter_ccf(decimation, taps) over a sample stream: ntaps - 1 samples of history carried
 * between runs (zeros after create / reset). */
int gnsship_acq_resampler_create(gnsship_ctx* ctx, const float* taps, int n_taps, int decimation, int64_t max_in_samples,
    gnsship_acq_resampler** out);
/* Filter n_in samples (a multiple of the decimation) in `fmt` (converted in the loads, no scaling):
 * n_in / decimation CF32 outputs, left in device memory (*dev_out, valid until the next run) and,
 * when host_out != NULL, copied there before returning.  Asynchronous otherwise (context stream). */
int gnsship_acq_resampler_run(gnsship_acq_resampler* r, const void* in, int fmt, int in_on_device, int64_t n_in, float* host_out,
    void** dev_out, int64_t* n_out);
int gnsship_acq_resampler_reset(gnsship_acq_resampler* r);
int gnsship_acq_resampler_destroy(gnsship_acq_resampler* r);

/* ---------------------------------------------------------------------------------------------
 * Closed-loop tracking engine: the per-epoch DLL/PLL of dll_pll_veml_tracking
 * resident on the device.  Replaces, for N channels at once, the general_work loop of
 * src/algorithms/tracking/gnuradio_blocks/dll_pll_veml_tracking.cc:1728-2094 around
 * do_correlation_step (:1037-1062): cn0_and_tracking_lock_status (:972-1029), run_dll_pll
 * (:1065-1152), update_tracking_vars (:1189-1260), save_correlation_results and the bit /
 * secondary-code synchronisation of states 2 and 4.  start_tracking (:643-883) and the state-1
 * pull-in (:1757-1788) run on the host in gnsship_trk_start.  States 2, 3 (extended coherent
 * integration, extend_correlation_symbols > 1) and 4, with the FLL branches (enable_fll_*) and
 * high_dyn (high-dynamics correlator fed by the smoothed NCO rates); BeiDou B1I GEO satellites by
 * the start arguments' PRN.
 * ------------------------------------------------------------------------------------------- */
#define GNSSHIP_SYS_GPS_L1CA 0 /* GPS L1 C/A: 3 taps, bit sync on the 160-symbol preamble */
#define GNSSHIP_SYS_GAL_E1 1   /* Galileo E1 B/C: VEML 5 taps on the pilot + data prompt, CS25 secondary */
#define GNSSHIP_SYS_BDS_B1I 2  /* BeiDou B1I MEO/IGSO (PRN 6-58): 3 taps, 20-chip NH secondary code */

typedef struct gnsship_trk_conf { /* Dll_Pll_Conf (dll_pll_conf.h:33-80), same names and units */
    double fs_in;
    double carrier_lock_th;
    float pll_bw_hz;
    float dll_bw_hz;
    float fll_bw_hz;
    float early_late_space_chips;
    float very_early_late_space_chips;
    float slope;
    float spc;
    float y_intercept;
    float cn0_smoother_alpha;
    float carrier_lock_test_smoother_alpha;
    uint32_t pull_in_time_s;
    uint32_t bit_synchronization_time_limit_s;
    uint32_t vector_length;
    int32_t pll_filter_order;
    int32_t dll_filter_order;
    int32_t cn0_samples;
    int32_t cn0_smoother_samples;
    int32_t carrier_lock_test_smoother_samples;
    int32_t cn0_min;
    int32_t max_code_lock_fail;
    int32_t max_carrier_lock_fail;
    int32_t carrier_aiding;
    int32_t track_pilot;
    int32_t system; /* GNSSHIP_SYS_*: the signal constants the adapter selects */
    int32_t extend_correlation_symbols; /* > 1: extended coherent integration, state 3 (:515-523) */
    float pll_bw_narrow_hz;
    float dll_bw_narrow_hz;
    float early_late_space_narrow_chips;
    float very_early_late_space_narrow_chips;
    int32_t enable_fll_pull_in;      /* FLL-assisted carrier loop during the pull-in (:1080-1097) */
    int32_t enable_fll_steady_state; /* ... and after it */
    int32_t high_dyn;                /* high-dynamics correlator + NCO rate smoothing (:1205-1255) */
    uint32_t smoother_length;        /* rate smoother length, 1..64 (0 is raised to 1, dll_pll_conf.cc:118-123) */
    int32_t rotator;                 /* GNSSHIP_ROTATOR_*: which volk_gnsssdr rotator variant the correlations
                                        reproduce (0 = generic; high_dyn has only the generic variant) */
    int32_t reserved0;               /* 0 */
    /* ABI 2.  Carrier IF of this engine's signal in the IF buffer [Hz] (e.g. +7.161e6 for GPS L1 / Galileo
     * E1 and −7.161e6 for BeiDou B1I in a 1568.259 MHz-centred front end).  The reference removes it
     * ahead of the channels (InputFilter.IF → freq_xlating_fir_filter, conf/gnss-sdr_BDS_B3I_GPS_L1_CA_
     * ibyte.conf:45-92; GNSSFlowgraph connects the filtered output to every channel); here it is fused
     * into the correlator's carrier NCO: phase_step = (float)(carrier_phase_step_rad + 2π·if_hz/fs) and
     * rem_carrier_phase = (float)fmod(rem_carr_phase_rad + 2π·frac(if_hz·n/fs), 2π) at the epoch's first
     * absolute sample n (frac(if_hz·n/fs) carried per channel in double, exact for integer if_hz and
     * fs).  The loop, its Doppler, carrier phase and all outputs stay IF-free, as in the reference.
     * 0 = the buffer is at baseband. */
    double if_hz;
} gnsship_trk_conf;

typedef struct gnsship_trk_start_args { /* Gnss_Synchro fields start_tracking reads (:647-649) */
    int32_t code_id;      /* code-bank entry of the tracking replica (pilot for E1) */
    int32_t data_code_id; /* E1 with track_pilot: data replica; otherwise ignored */
    double acq_delay_samples;
    double acq_doppler_hz;
    uint64_t acq_samplestamp_samples;
    uint64_t first_sample; /* nitems_read when the block first runs after start (state-1 pull-in) */
    int32_t prn;           /* Gnss_Synchro::PRN: BeiDou B1I PRN 1-5 and 59+ are GEO satellites (:765-781) */
    int32_t reserved;      /* 0 */
} gnsship_trk_start_args;

typedef struct gnsship_trk_epoch { /* one general_work call of one channel (Gnss_Synchro subset) */
    uint64_t sample_counter;       /* nitems_read at the epoch start */
    double prompt_i, prompt_q;     /* valid when flags & 1 (state 4 symbol output) */
    double code_phase_samples;     /* d_rem_code_phase_samples */
    double carrier_phase_rads;     /* d_acc_carrier_phase_rad */
    double carrier_doppler_hz;
    double cn0_db_hz;
    float carrier_lock_test;
    int32_t state;                 /* state the epoch ran in (2, 3 or 4) */
    int32_t flags;                 /* 1 valid symbol, 2 loss of lock, 4 PLL 180°, 8 epoch ran,
                                      16 log_data record written (gnsship_trk_run_dump) */
    int32_t pad;
    double code_freq_chips;
    double rem_code_phase_chips;
    float rem_carr_phase_rad;
    int32_t prn_length_samples;    /* d_current_prn_length_samples after the update */
} gnsship_trk_epoch; /* 96 bytes */

typedef struct gnsship_trk gnsship_trk;
int gnsship_trk_create(gnsship_ctx* ctx, const gnsship_trk_conf* conf, int max_channels, gnsship_trk** out);
int gnsship_trk_start(gnsship_trk* t, int channel, const gnsship_trk_start_args* args);
/* n gnsship_trk_start calls in one transaction (a mass hand-off from acquisition): channels[i]
 * starts from args[i]; every channel is validated before any device state changes (on an error
 * nothing is started); one upload, one scatter launch, one synchronisation.  Distinct channels. */
int gnsship_trk_start_many(gnsship_trk* t, int n, const int32_t* channels, const gnsship_trk_start_args* args);
int gnsship_trk_stop(gnsship_trk* t, int channel);
/* msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:617-640): a telemetry fault (tlm_event 1)
 * from the channel's telemetry decoder sets the carrier lock-fail counter to 200000, so the next
 * lock check of the loop declares loss of lock.  Other event values are ignored, as there. */
int gnsship_trk_telemetry_event(gnsship_trk* t, int channel, int tlm_event);
/* Runs up to max_rounds epochs of every tracking channel over the IF buffer holding absolute
 * samples [buffer_first_sample, +n_buffer_samples) (device pointer when sig_on_device, else host
 * memory staged to the device).  Per round each channel whose next vector_length window lies in
 * the buffer runs one epoch; no host round trip between rounds.  out (optional): max_rounds ×
 * max_channels records, flags & 8 marking the epochs that ran.  *rounds_done: rounds in which at
 * least one channel ran. */
int gnsship_trk_run(gnsship_trk* t, const void* sig, int fmt, int sig_on_device, uint64_t buffer_first_sample, int64_t n_buffer_samples,
    int max_rounds, gnsship_trk_epoch* out, int* rounds_done);
/* The tracking dump record dll_pll_veml_tracking::log_data writes per valid loop update when
 * `dump` is on (:1376-1466; read back by tracking_dump_reader.cc:26-47): 96 bytes, packed exactly
 * as the file — a per-channel .dat dump is the concatenation of the records whose epoch has
 * flags & 16, in round order. */
#pragma pack(push, 4)
typedef struct gnsship_trk_dump_record {
    float abs_VE, abs_E, abs_P, abs_L, abs_VL; /* |accumulators| (VE/VL 0 without VEML)            */
    float prompt_I, prompt_Q;                 /* this epoch's prompt (data prompt with track_pilot) */
    uint64_t PRN_start_sample_count;          /* nitems_read + d_current_prn_length_samples     */
    float acc_carrier_phase_rad;
    float carrier_doppler_hz;
    float carrier_doppler_rate_hz;            /* carrier_phase_rate_step_rad·fs²/2π (high_dyn)   */
    float code_freq_chips;
    float code_freq_rate_chips;               /* code_phase_rate_step_chips·fs²                  */
    float carr_error_hz, carr_error_filt_hz;
    float code_error_chips, code_error_filt_chips;
    float CN0_SNV_dB_Hz, carrier_lock_test;
    float aux1;                               /* d_rem_code_phase_samples                        */
    double aux2;                              /* (double)(nitems_read + prn length)              */
    uint32_t PRN;
} gnsship_trk_dump_record;
#pragma pack(pop)
/* gnsship_trk_run that also fills dump[max_rounds × max_channels] (optional) with the log_data
 * records of the epochs flagged 16. */
int gnsship_trk_run_dump(gnsship_trk* t, const void* sig, int fmt, int sig_on_device, uint64_t buffer_first_sample, int64_t n_buffer_samples,
    int max_rounds, gnsship_trk_epoch* out, gnsship_trk_dump_record* dump, int* rounds_done);
/* Asynchronous form: enqueue the run on the context stream and return (dev_sig: a device buffer that
 * stays valid until gnsship_trk_collect); records / dump records are kept on the device when
 * requested.  Engines on different contexts of one device then run concurrently from one host
 * thread (e.g. a hybrid receiver's GPS, Galileo and BeiDou engines over one IF block).  Every launch
 * is followed by exactly one gnsship_trk_collect, which waits for it and copies the records
 * (out / dump as in gnsship_trk_run_dump, NULL to skip; a non-NULL out / dump that the launch did not
 * keep — want_records / want_dump 0 — is GNSSHIP_E_INVAL, the buffer untouched, the launch finished). */
int gnsship_trk_launch(gnsship_trk* t, const void* dev_sig, int fmt, uint64_t buffer_first_sample, int64_t n_buffer_samples, int max_rounds,
    int want_records, int want_dump);
int gnsship_trk_collect(gnsship_trk* t, gnsship_trk_epoch* out, gnsship_trk_dump_record* dump, int* rounds_done);
int gnsship_trk_channel_state(gnsship_trk* t, int channel, int* state, uint64_t* next_sample);
/* Correlation trace: each channel-epoch's do_correlation_step call (dll_pll_veml_tracking.cc:1037-1062)
 * as the engine ran it — the float arguments of Carrier_wipeoff_multicorrelator_resampler
 * (cpu_multicorrelator_real_codes.cc:103-126, the carrier ones with the IF folded in) and the
 * correlator outputs — so that a caller can re-run exactly those correlations on the reference's
 * CPU correlator and compare them tap by tap.  Off by default (a debugging aid: 104 bytes per
 * channel-epoch written to HBM). */
typedef struct gnsship_trk_corr_trace {
    uint64_t sample_counter;               /* absolute first sample of the epoch (nitems_read) */
    int32_t n_samples;                     /* vector_length */
    int32_t n_taps;
    float rem_carrier_phase_rad, phase_step_rad;
    float rem_code_phase_samples, code_phase_step_samples;  /* rem_code_phase_chips·spc, code_phase_step_chips·spc */
    float shifts[5];                       /* local code shifts in code samples (narrow taps once narrowed) */
    float taps[10];                        /* complex output per tap */
    float data_prompt[2];                  /* the data correlator's prompt (track_pilot), else 0 */
    int32_t pad;
} gnsship_trk_corr_trace; /* 104 bytes */
int gnsship_trk_set_trace(gnsship_trk* t, int enable);
/* The last run's trace: max_rounds × max_channels records (the run's max_rounds), zero where no epoch ran. */
int gnsship_trk_trace_records(gnsship_trk* t, gnsship_trk_corr_trace* out, int max_records);
/* Which kernel the last gnsship_trk_run / _launch ran (GNSSHIP_TRK_ENGINE_*; NONE before any run):
 * the AVX rotator runs trk_fast's latency form while the channels fit one per compute unit and
 * trk_lane beyond (one 16-lane row per channel; trk_fast's throughput form when a code is not ±1),
 * the generic rotator trk_persist, high_dyn and epochs too long for LDS the round-based loop. */
#define GNSSHIP_TRK_ENGINE_NONE 0
#define GNSSHIP_TRK_ENGINE_FAST_LATENCY 1
#define GNSSHIP_TRK_ENGINE_FAST_THROUGHPUT 2
#define GNSSHIP_TRK_ENGINE_PERSIST 3
#define GNSSHIP_TRK_ENGINE_ROUNDS 4
#define GNSSHIP_TRK_ENGINE_LANES 5
int gnsship_trk_last_engine(gnsship_trk* t, int* engine);
int gnsship_trk_destroy(gnsship_trk* t);

/* ------------------------------------------------------------------------------------------ */
/* Multi-GPU fan-out: one process per GPU, one RCCL communicator per context.  */
/* The reference connects one conditioner output to every channel block (gnss_flowgraph.cc:    */
/* 1127-1136); across GPUs that connection is a broadcast of the raw IF block from the rank     */
/* that reads the front end, after which every rank tracks / acquires its own channel or PRN    */
/* shard with no further data-path collective.  Collectives are enqueued on the context stream  */
/* (ordered before any later launch of that context; gnsship_ctx_sync waits for them).          */
/* ------------------------------------------------------------------------------------------ */
typedef struct gnsship_comm gnsship_comm;
#define GNSSHIP_COMM_ID_BYTES 128
/* Rank 0 creates the id and hands it to the other ranks out of band (e.g. the launcher's store). */
int gnsship_comm_unique_id(void* id);
int gnsship_comm_create(gnsship_ctx* ctx, int n_ranks, int rank, const void* id, gnsship_comm** out);
int gnsship_comm_rank(gnsship_comm* c, int* rank, int* n_ranks);
/* In-place broadcast of `bytes` of a device buffer from `root` (raw IF samples in any format). */
int gnsship_comm_broadcast(gnsship_comm* c, void* dev_buf, size_t bytes, int root);
/* dev_recv[r·bytes_per_rank ...] = rank r's dev_send (per-PRN acquisition results, records). */
int gnsship_comm_allgather(gnsship_comm* c, const void* dev_send, void* dev_recv, size_t bytes_per_rank);
/* In-place max over ranks of `count` doubles (timing: the slowest rank's wall time). */
int gnsship_comm_allreduce_max_f64(gnsship_comm* c, double* dev_buf, size_t count);
int gnsship_comm_destroy(gnsship_comm* c);

#ifdef __cplusplus
}
#endif
#endif /* GNSSHIP_H */
