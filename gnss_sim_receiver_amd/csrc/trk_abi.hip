// trk_abi.hip — C-ABI of the device-resident tracking loop (include/gnsship.h, gnsship_trk_*).
//
// Host side of dll_pll_veml_tracking: the constructor's per-signal constants (:142-330), the
// loop-filter / smoother set-up (:462-466, :540-553, Tracking_loop_filter::update_coefficients
// tracking_loop_filter.cc:100-200, Tracking_FLL_PLL_filter::set_params :23-55), and
// start_tracking + the state-1 pull-in (:643-883, :1757-1788).  The per-epoch loop runs on the
// device (trk_kernel.hip) between fixed-plan correlator launches.
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "engine.h"
#include "trk_engine.h"

namespace gnsship {
int fail(gnsship_ctx* ctx, int code, const char* what);
int hip_fail(gnsship_ctx* ctx, hipError_t e, const char* where);
int set_device(gnsship_ctx* ctx);
int sync_code_table(gnsship_ctx* ctx);
size_t fmt_bytes(int fmt);
int chunks_per_item_setting();
}  // namespace gnsship

using namespace gnsship;
static_assert(sizeof(gnsship_trk_epoch) == 96, "gnsship_trk_epoch layout");
static_assert(sizeof(gnsship_trk_corr_trace) == 104, "gnsship_trk_corr_trace layout");
static_assert(sizeof(gnsship_trk_dump_record) == 96 && offsetof(gnsship_trk_dump_record, PRN_start_sample_count) == 28 &&
                  offsetof(gnsship_trk_dump_record, aux2) == 84 && offsetof(gnsship_trk_dump_record, PRN) == 92,
    "gnsship_trk_dump_record = the log_data file record");

#define HIP_TRY(ctx, expr)                                       \
    do {                                                         \
        hipError_t _e = (expr);                                  \
        if (_e != hipSuccess) return hip_fail((ctx), _e, #expr); \
    } while (0)

struct gnsship_trk {
    gnsship_ctx* ctx = nullptr;
    TrkParams params{};
    int max_channels = 0;
    int n_jobs = 0, n_chunks = 0;
    bool any_multi = false;
    ChunkClass classes[kChunkClasses]{};
    std::vector<TrkChannel> host_chans;
    std::vector<ChunkDesc> chunks_host;   // plan (lengths are rewritten on the device each round)
    std::vector<int32_t> jobs_first_chunk;
    std::vector<int32_t> job_code;        // code-bank id per job (−1: channel never started)
    uint64_t attached_version = 0;        // ctx->codes_version the chunk code pointers reflect
    TrkParams* params_dev = nullptr;
    TrkChannel* chans_dev = nullptr;
    DevJob* jobs_dev = nullptr;
    ChunkDesc* chunks_dev = nullptr;
    WorkItem* items_dev = nullptr;
    int n_items = 0;
    Anchor* anchors_dev = nullptr;
    float* partials_dev = nullptr;
    float* out_dev = nullptr;
    gnsship_trk_epoch* rec_dev = nullptr;
    size_t rec_cap = 0;
    gnsship_trk_dump_record* dump_dev = nullptr;
    size_t dump_cap = 0;
    int* ran_dev = nullptr;
    size_t ran_cap = 0;
    void* stage_dev = nullptr;
    size_t stage_cap = 0;
    void* start_stage_dev = nullptr;  // gnsship_trk_start_many's staged channel states + indices
    size_t start_stage_cap = 0;
    // high_dyn: the high-dynamics correlator's fixed plan (one HdJob per job, out_index = job) and
    // the channels' rate-smoother rings
    bool high_dyn = false;
    HdPlan hd;
    TrkHist* hist_dev = nullptr;
    bool force_rounds = false;  // GNSSHIP_TRK_ROUNDS=1: the round-based loop even where the persistent one applies
    // gnsship_trk_launch → gnsship_trk_collect: the enqueued run's rounds (−1: none pending)
    int pending_rounds = -1;
    bool pending_out = false, pending_dump = false;
    // gnsship_trk_set_trace: per channel-epoch correlation trace of the last run
    bool trace_on = false;
    int last_engine = GNSSHIP_TRK_ENGINE_NONE;  // the engine the last run / launch used
    gnsship_trk_corr_trace* trace_dev = nullptr;
    size_t trace_cap = 0;
    size_t trace_n = 0;  // records of the last run (max_rounds × max_channels)
};

namespace {

void set_bits(uint32_t* bits, const char* s)
{
    for (int i = 0; s[i]; i++)
        if (s[i] == '1') bits[i >> 5] |= 1u << (i & 31);
}

// GPS L1 C/A preamble 10001011 at 20 symbols per bit (GPS_L1_CA.h:73, IS-GPS-200 TLM word)
void gps_preamble_symbols(char* out)
{
    const char bits[] = "10001011";
    int n = 0;
    for (int b = 0; b < 8; b++)
        for (int r = 0; r < 20; r++) out[n++] = bits[b];
    out[n] = '\0';
}

// Tracking_loop_filter::update_coefficients (tracking_loop_filter.cc:100-200), no last integrator
// (the tracking block constructs it with include_last_integrator = false, :465).
void loop_filter_coefficients(float T, float bw, int order, LoopSet& p)
{
    const float zeta = 1.0F / std::sqrt(2.0F);
    float g1, g2, g3, wn;
    switch (order) {
    case 1:
        wn = bw * 4.0F;
        g1 = wn;
        p.lf_n_in = 1;
        p.lf_in[0] = g1;
        p.lf_n_out = 0;
        break;
    case 2:
        wn = bw * (8.0F * zeta) / (4.0F * zeta * zeta + 1.0F);
        g1 = wn * wn;
        g2 = wn * 2.0F * zeta;
        p.lf_n_in = 2;
        p.lf_in[0] = static_cast<float>(g1 * T / 2.0 + g2);
        p.lf_in[1] = static_cast<float>(g1 * T / 2.0 - g2);
        p.lf_n_out = 1;
        p.lf_out[0] = 1.0F;
        break;
    default: {
        wn = bw / 0.7845F;
        const float a3 = 1.1F, b3 = 2.4F;
        g1 = wn * wn * wn;
        g2 = a3 * wn * wn;
        g3 = b3 * wn;
        p.lf_n_in = 3;
        p.lf_in[0] = static_cast<float>(g3 + T / 2.0 * (g2 + T / 2.0 * g1));
        p.lf_in[1] = static_cast<float>(g1 * T * T / 2.0 - 2.0 * g3);
        p.lf_in[2] = static_cast<float>(g3 + T / 2.0 * (-g2 + T / 2.0 * g1));
        p.lf_n_out = 2;
        p.lf_out[0] = 2.0F;
        p.lf_out[1] = -1.0F;
    } break;
    }
}

bool build_params(const gnsship_trk_conf& c, TrkParams& p)
{
    std::memset(&p, 0, sizeof(p));
    p.conf = c;
    if (p.conf.smoother_length < 1) p.conf.smoother_length = 1;  // dll_pll_conf.cc:119-123
    char sec[kTrkMaxSecondary + 1] = {0};
    SymSync& g = p.sync[0];
    switch (c.system) {
    case GNSSHIP_SYS_GPS_L1CA:  // :142-200 (1C), start_tracking :662-668 forces track_pilot = false
        p.code_chip_rate = 1.023e6;
        p.carrier_freq = 1575.42e6;
        p.code_period = 0.001;
        p.code_length_chips = 1023;
        p.code_samples_per_chip = 1;
        g.symbols_per_bit = 20;
        p.veml = 0;
        p.track_pilot = 0;
        g.secondary = 0;
        gps_preamble_symbols(sec);
        g.secondary_len = 160;
        set_bits(g.secondary_bits, sec);
        break;
    case GNSSHIP_SYS_GAL_E1:  // :262-291 (1B); Galileo_E1.h:35-52
        p.code_chip_rate = 1.023e6;
        p.carrier_freq = 1575.42e6;
        p.code_period = 0.004;
        p.code_length_chips = 4092;
        p.code_samples_per_chip = 2;
        g.symbols_per_bit = 1;
        p.veml = 1;
        p.track_pilot = c.track_pilot ? 1 : 0;
        if (p.track_pilot) {
            g.secondary = 1;
            g.secondary_len = 25;
            set_bits(g.secondary_bits, "0011100000001010110110010");  // CS25 (GALILEO_E1_C_SECONDARY_CODE)
        }
        break;
    case GNSSHIP_SYS_BDS_B1I:  // :762-797 (MEO/IGSO branch); Beidou_B1I.h:35-48
        p.code_chip_rate = 2.046e6;
        p.carrier_freq = 1561.098e6;
        p.code_period = 0.001;
        p.code_length_chips = 2046;
        p.code_samples_per_chip = 1;
        g.symbols_per_bit = 20;
        p.veml = 0;
        p.track_pilot = 0;
        g.secondary = 1;
        g.secondary_len = 20;
        set_bits(g.secondary_bits, "00000100110101001110");  // NH code (BEIDOU_B1I_SECONDARY_CODE_STR)
        g.data_secondary_len = 20;
        set_bits(g.data_secondary_bits, "00000100110101001110");
        break;
    default: return false;
    }
    p.n_taps = p.veml ? 5 : 3;
    const float spcf = static_cast<float>(p.code_samples_per_chip);
    if (p.veml) {
        p.shifts[0] = -c.very_early_late_space_chips * spcf;
        p.shifts[1] = -c.early_late_space_chips * spcf;
        p.shifts[2] = 0.0F;
        p.shifts[3] = c.early_late_space_chips * spcf;
        p.shifts[4] = c.very_early_late_space_chips * spcf;
    } else {
        p.shifts[0] = -c.early_late_space_chips * spcf;
        p.shifts[1] = 0.0F;
        p.shifts[2] = c.early_late_space_chips * spcf;
    }
    // extended integration (:515-523): enabled when extend_correlation_symbols > 1
    g.extend = c.extend_correlation_symbols > 1 ? c.extend_correlation_symbols : 1;
    g.T_ext = static_cast<float>(g.extend) * static_cast<float>(p.code_period);
    // BeiDou B1I GEO satellites (start_tracking :765-781; Beidou_B1I.h:41-49): D2 navigation at 2
    // symbols per bit, no NH code, bit synchronisation on the 22-symbol preamble, extend ≤ 2
    p.sync[1] = g;
    if (c.system == GNSSHIP_SYS_BDS_B1I) {
        SymSync& geo = p.sync[1];
        std::memset(geo.secondary_bits, 0, sizeof(geo.secondary_bits));
        std::memset(geo.data_secondary_bits, 0, sizeof(geo.data_secondary_bits));
        geo.symbols_per_bit = 2;
        geo.secondary = 0;
        geo.secondary_len = 22;
        set_bits(geo.secondary_bits, "1111110000001100001100");  // BEIDOU_B1I_GEO_PREAMBLE_SYMBOLS_STR
        geo.data_secondary_len = 0;
        if (geo.extend > 2) geo.extend = 2;
        geo.T_ext = static_cast<float>(geo.extend) * static_cast<float>(p.code_period);
    }
    if (p.veml) {
        p.shifts_n[0] = -c.very_early_late_space_narrow_chips * spcf;
        p.shifts_n[1] = -c.early_late_space_narrow_chips * spcf;
        p.shifts_n[2] = 0.0F;
        p.shifts_n[3] = c.early_late_space_narrow_chips * spcf;
        p.shifts_n[4] = c.very_early_late_space_narrow_chips * spcf;
    } else {
        p.shifts_n[0] = -c.early_late_space_narrow_chips * spcf;
        p.shifts_n[1] = 0.0F;
        p.shifts_n[2] = c.early_late_space_narrow_chips * spcf;
    }
    p.spc_n = c.early_late_space_narrow_chips;
    // wide: (code period, dll_bw); narrow: set_update_interval(T_ext) + set_noise_bandwidth(dll_bw_narrow)
    loop_filter_coefficients(static_cast<float>(p.code_period), c.dll_bw_hz, c.dll_filter_order, p.ls[0]);
    loop_filter_coefficients(p.sync[0].T_ext, c.dll_bw_narrow_hz, c.dll_filter_order, p.ls[1]);
    loop_filter_coefficients(p.sync[1].T_ext, c.dll_bw_narrow_hz, c.dll_filter_order, p.ls[2]);
    // Tracking_FLL_PLL_filter::set_params (tracking_FLL_PLL_filter.cc:23-55): wide, then narrow (:1904)
    p.fp_order = c.pll_filter_order;
    for (int s = 0; s < 3; s++) {
        LoopSet& q = p.ls[s];
        const float pll_bw = s ? c.pll_bw_narrow_hz : c.pll_bw_hz;
        if (p.fp_order == 3) {
            q.fp_b3 = 2.400F;
            q.fp_a3 = 1.100F;
            q.fp_a2 = 1.414F;
            q.fp_w0p = pll_bw / 0.7845F;
            q.fp_w0p2 = q.fp_w0p * q.fp_w0p;
            q.fp_w0p3 = q.fp_w0p2 * q.fp_w0p;
            q.fp_w0f = c.fll_bw_hz / 0.53F;
            q.fp_w0f2 = q.fp_w0f * q.fp_w0f;
        } else {
            q.fp_a2 = 1.414F;
            q.fp_w0p = pll_bw / 0.53F;
            q.fp_w0p2 = q.fp_w0p * q.fp_w0p;
            q.fp_w0f = c.fll_bw_hz / 0.25F;
        }
    }
    // Exponential_Smoother settings (:540-553, exponential_smoother.cc:29-73)
    auto clamp01 = [](float a) { return a < 0.0F ? 0.0F : (a > 1.0F ? 1.0F : a); };
    p.cn0_alpha = clamp01(c.cn0_smoother_alpha);
    p.cn0_one_minus_alpha = 1.0F - p.cn0_alpha;
    p.cn0_min_value = 25.0F;
    p.cn0_offset = 12.0F;
    int ns = c.cn0_smoother_samples / static_cast<int>(p.code_period * 1000.0);
    p.cn0_init_samples = ns <= 0 ? 1 : ns;
    p.lock_alpha = clamp01(c.carrier_lock_test_smoother_alpha);
    p.lock_one_minus_alpha = 1.0F - p.lock_alpha;
    p.lock_min_value = -1.0F;
    p.lock_offset = 0.0F;
    p.lock_init_samples = c.carrier_lock_test_smoother_samples <= 0 ? 1 : c.carrier_lock_test_smoother_samples;
    p.jobs_per_channel = p.track_pilot ? 2 : 1;
    p.chunks_per_job = (static_cast<int>(c.vector_length) + kCorrChunk - 1) / kCorrChunk;
    // carrier IF fused into the correlator NCO (include/gnsship.h if_hz; gnsship_trk_create checked
    // that if_hz and fs_in are whole Hz)
    p.has_if = c.if_hz != 0.0 ? 1 : 0;
    p.if_step_rad = p.has_if ? 6.2831853071796 * c.if_hz / c.fs_in : 0.0;
    p.fs_int = static_cast<int64_t>(c.fs_in);
    const int64_t ifi = static_cast<int64_t>(c.if_hz);
    p.if_mod = p.fs_int > 0 ? ((ifi % p.fs_int) + p.fs_int) % p.fs_int : 0;
    p.inv_fs = 1.0 / c.fs_in;
    p.inv_carrier_freq = 1.0 / p.carrier_freq;
    return true;
}

// high_dyn: bind a job's code replica in its HdJob (the step kernel keeps these fields).
hipError_t upload_hd_code(gnsship_trk* t, int job, const CodeDesc& cd)
{
    static_assert(offsetof(HdJob, code_len) == offsetof(HdJob, code) + sizeof(const float*), "HdJob code fields");
    HdJob& j = t->hd.jobs[job];
    j.code = cd.ptr;
    j.code_len = cd.ptr ? cd.len : 0;
    return hipMemcpyAsync(reinterpret_cast<char*>(t->hd.jobs_dev + job) + offsetof(HdJob, code), &j.code, sizeof(const float*) + sizeof(int32_t),
        hipMemcpyHostToDevice, t->ctx->stream);
}

void release(gnsship_trk* t)
{
    void* ptrs[] = {t->params_dev, t->chans_dev, t->jobs_dev, t->chunks_dev, t->items_dev, t->anchors_dev, t->partials_dev, t->out_dev, t->rec_dev,
        t->ran_dev, t->stage_dev, t->hist_dev, t->dump_dev, t->trace_dev, t->start_stage_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    hd_plan_free(t->hd);
}

}  // namespace

extern "C" int gnsship_trk_last_engine(gnsship_trk* t, int* engine)
{
    if (!t || !engine) return GNSSHIP_E_INVAL;
    *engine = t->last_engine;
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_destroy(gnsship_trk* t)
{
    if (!t) return GNSSHIP_E_INVAL;
    (void)hipSetDevice(t->ctx->device);
    (void)hipStreamSynchronize(t->ctx->stream);
    release(t);
    delete t;
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_create(gnsship_ctx* ctx, const gnsship_trk_conf* conf, int max_channels, gnsship_trk** out)
{
    if (!ctx || !conf || !out) return GNSSHIP_E_INVAL;
    *out = nullptr;
    if (max_channels < 1 || conf->fs_in <= 0.0 || conf->vector_length < 1 || conf->cn0_samples < 1 || conf->cn0_samples > kTrkMaxCn0Samples ||
        conf->pll_filter_order < 2 || conf->pll_filter_order > 3 || conf->dll_filter_order < 1 || conf->dll_filter_order > 3 ||
        (conf->high_dyn && conf->smoother_length > static_cast<uint32_t>(kTrkMaxSmoother)) || conf->rotator < GNSSHIP_ROTATOR_AUTO ||
        conf->rotator > GNSSHIP_ROTATOR_AVX || conf->reserved0 != 0)
        return fail(ctx, GNSSHIP_E_INVAL,
            "gnsship_trk_create: bad configuration (cn0_samples 1..64, pll order 2..3, dll order 1..3, smoother_length <= 64)");
    if (conf->if_hz != 0.0 && (!std::isfinite(conf->if_hz) || conf->if_hz != std::floor(conf->if_hz) || conf->fs_in != std::floor(conf->fs_in) ||
                                  std::fabs(conf->if_hz) >= conf->fs_in || conf->fs_in > 4.0e9))
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_create: if_hz must be a whole number of Hz below fs_in, with fs_in whole Hz");
    gnsship_trk* t = new (std::nothrow) gnsship_trk();
    if (!t) return GNSSHIP_E_NOMEM;
    t->ctx = ctx;
    if (!build_params(*conf, t->params)) {
        delete t;
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_create: unknown system");
    }
    if (t->params.conf.rotator == GNSSHIP_ROTATOR_AUTO) {
        // a preference entry the engine does not reproduce (generic_reload, another variant name) is
        // an error, not a silent fall-back to the nearest variant
        if (gnsship_rotator_dispatch(&t->params.conf.rotator) != GNSSHIP_OK) {
            char detail[256] = {0}, msg[320];
            gnsship_rotator_dispatch_detail(detail, sizeof(detail));
            std::snprintf(msg, sizeof(msg), "gnsship_trk_create: rotator dispatch: %s", detail);
            delete t;
            return fail(ctx, GNSSHIP_E_INVAL, msg);
        }
    }
    if (t->params.conf.high_dyn) t->params.conf.rotator = GNSSHIP_ROTATOR_GENERIC;  // only generic high-dynamics variants exist
    if (t->params.conf.rotator == GNSSHIP_ROTATOR_AVX && !trk_persist_supports(t->params)) {
        delete t;
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_create: the AVX rotator runs in the persistent loop, which has no kernel for this tap layout");
    }
    {
        const char* env = std::getenv("GNSSHIP_TRK_ROUNDS");  // A/B: force the round-based loop
        t->force_rounds = env && env[0] == '1';
    }
    if (int rc = set_device(ctx)) {
        delete t;
        return rc;
    }
    t->max_channels = max_channels;
    const TrkParams& p = t->params;
    t->n_jobs = max_channels * p.jobs_per_channel;
    std::vector<DevJob> jobs(t->n_jobs);
    for (int i = 0; i < t->n_jobs; i++) {
        std::memset(&jobs[i], 0, sizeof(DevJob));
        jobs[i].n_samples = static_cast<int32_t>(conf->vector_length);
        jobs[i].n_taps = (p.jobs_per_channel == 2 && (i % 2) == 1) ? 1 : p.n_taps;
        jobs[i].in_margin = 0;
    }
    std::vector<ChunkDesc> chunks;
    std::vector<WorkItem> items;
    int64_t n_anchors = 0;
    // codes are bound when channels start: items only group the chunks of one job
    t->n_chunks = plan_chunks(jobs, chunks, items, t->any_multi, &n_anchors, t->classes, chunks_per_item_setting(), false);
    t->n_items = static_cast<int>(items.size());
    for (auto& j : jobs) j.n_samples = 0;  // idle until a channel starts
    for (auto& c : chunks) c.len = 0;      // (code pointers are attached when a channel starts)
    t->chunks_host = chunks;
    t->jobs_first_chunk.resize(t->n_jobs);
    for (int i = 0; i < t->n_jobs; i++) t->jobs_first_chunk[i] = jobs[i].first_chunk;
    t->job_code.assign(t->n_jobs, -1);
    t->attached_version = ctx->codes_version;
    t->host_chans.assign(max_channels, TrkChannel{});
    for (auto& c : t->host_chans) std::memset(&c, 0, sizeof(TrkChannel));
    hipError_t e = hipMalloc(&t->params_dev, sizeof(TrkParams));
    if (e == hipSuccess) e = hipMemcpy(t->params_dev, &t->params, sizeof(TrkParams), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&t->chans_dev, sizeof(TrkChannel) * max_channels);
    if (e == hipSuccess) e = hipMemcpy(t->chans_dev, t->host_chans.data(), sizeof(TrkChannel) * max_channels, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&t->jobs_dev, sizeof(DevJob) * t->n_jobs);
    if (e == hipSuccess) e = hipMemcpy(t->jobs_dev, jobs.data(), sizeof(DevJob) * t->n_jobs, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&t->chunks_dev, sizeof(ChunkDesc) * t->n_chunks);
    if (e == hipSuccess) e = hipMemcpy(t->chunks_dev, chunks.data(), sizeof(ChunkDesc) * t->n_chunks, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&t->items_dev, sizeof(WorkItem) * t->n_items);
    if (e == hipSuccess) e = hipMemcpy(t->items_dev, items.data(), sizeof(WorkItem) * t->n_items, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&t->anchors_dev, sizeof(Anchor) * static_cast<size_t>(n_anchors + kAnchorPad));
    if (e == hipSuccess) e = hipMemset(t->anchors_dev, 0, sizeof(Anchor) * static_cast<size_t>(n_anchors + kAnchorPad));
    if (e == hipSuccess) e = hipMalloc(&t->partials_dev, sizeof(float) * 2 * kMaxTaps * static_cast<size_t>(t->n_chunks));
    if (e == hipSuccess) e = hipMalloc(&t->out_dev, sizeof(float) * 2 * kMaxTaps * static_cast<size_t>(t->n_jobs));
    t->high_dyn = conf->high_dyn != 0;
    if (e == hipSuccess && t->high_dyn) {
        t->hd.jobs.assign(t->n_jobs, HdJob{});
        for (int i = 0; i < t->n_jobs; i++) {
            HdJob& j = t->hd.jobs[i];
            j.n_samples = static_cast<int32_t>(conf->vector_length);
            j.n_taps = (p.jobs_per_channel == 2 && (i % 2) == 1) ? 1 : p.n_taps;
            j.out_index = i;
        }
        e = hd_plan_upload(t->hd, ctx->stream);  // chunk layout and anchor offsets for vector_length
        if (e == hipSuccess) {  // idle until a channel starts (the step kernel rewrites both every round)
            for (auto& j : t->hd.jobs) j.n_samples = 0;
            for (auto& c : t->hd.chunks) c.len = 0;
            e = hipMemcpy(t->hd.jobs_dev, t->hd.jobs.data(), sizeof(HdJob) * t->hd.jobs.size(), hipMemcpyHostToDevice);
        }
        if (e == hipSuccess) e = hipMemcpy(t->hd.chunks_dev, t->hd.chunks.data(), sizeof(HdChunk) * t->hd.chunks.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc(&t->hist_dev, sizeof(TrkHist) * static_cast<size_t>(max_channels));
    }
    if (e != hipSuccess) {
        release(t);
        delete t;
        return hip_fail(ctx, e, "gnsship_trk_create");
    }
    *out = t;
    return GNSSHIP_OK;
}

// start_tracking (:643-883) and the state-1 pull-in (:1757-1788) at nitems_read = first_sample: the
// channel's state on the host (validated), and the channel's jobs' code ids in the host tables.
static int trk_start_state(gnsship_trk* t, int channel, const gnsship_trk_start_args* a, TrkChannel& c)
{
    gnsship_ctx* ctx = t->ctx;
    if (!a || channel < 0 || channel >= t->max_channels) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_start: bad channel / arguments");
    if (a->code_id < 0 || a->code_id >= static_cast<int>(ctx->codes_host.size()) || !ctx->codes_host[a->code_id].ptr)
        return fail(ctx, GNSSHIP_E_STATE, "gnsship_trk_start: tracking code not in the code bank");
    const TrkParams& p = t->params;
    if (p.track_pilot && (a->data_code_id < 0 || a->data_code_id >= static_cast<int>(ctx->codes_host.size()) || !ctx->codes_host[a->data_code_id].ptr))
        return fail(ctx, GNSSHIP_E_STATE, "gnsship_trk_start: data code not in the code bank");
    if (a->first_sample < a->acq_samplestamp_samples) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_start: first_sample before the acquisition stamp");
    std::memset(&c, 0, sizeof(c));
    const gnsship_trk_conf& k = p.conf;
    c.code_id = a->code_id;
    c.prn = a->prn > 0 ? static_cast<uint32_t>(a->prn) : 0u;
    // GEO satellites use the D2 symbol-sync profile (start_tracking :765-781)
    c.geo = (p.conf.system == GNSSHIP_SYS_BDS_B1I && ((a->prn > 0 && a->prn < 6) || a->prn > 58)) ? 1 : 0;
    c.data_code_id = p.track_pilot ? a->data_code_id : a->code_id;
    c.acq_sample_stamp = a->acq_samplestamp_samples;
    c.carrier_doppler_hz = a->acq_doppler_hz;
    c.carrier_phase_step_rad = 6.2831853071796 * c.carrier_doppler_hz / k.fs_in;  // TWO_PI = 2·GNSS_PI (MATH_CONSTANTS.h:47-49)
    c.carrier_lock_test = 1.0F;
    c.cn0_db_hz = 0.0F;
    c.spc = k.spc;
    // carrier filter initialize(acq doppler); code filter initialize(0) (tracking_loop_filter.cc:50-56)
    if (p.fp_order == 3) {
        c.fp_x = 2.0F * static_cast<float>(a->acq_doppler_hz);
        c.fp_w = 0.0F;
    } else {
        c.fp_w = static_cast<float>(a->acq_doppler_hz);
        c.fp_x = 0.0F;
    }
    c.lf_idx = 3;
    c.cn0_sm.initializing = 1;
    c.lock_sm.initializing = 1;
    c.cloop = 1;
    c.pull_in = 1;
    // state 1
    const int64_t diff = static_cast<int64_t>(a->first_sample) - static_cast<int64_t>(c.acq_sample_stamp);
    const double delta = static_cast<double>(diff) - a->acq_delay_samples;
    c.code_freq_chips = p.code_chip_rate;
    c.code_phase_step_chips = c.code_freq_chips / k.fs_in;
    const double T_chip = 1.0 / c.code_freq_chips;
    const double T_prn = T_chip * static_cast<double>(p.code_length_chips);
    const double T_prn_samples = T_prn * k.fs_in;
    const double acq_code_phase_samples = T_prn_samples - std::fmod(delta, T_prn_samples);
    c.current_prn_length_samples = static_cast<int32_t>(std::round(T_prn_samples));
    const int32_t samples_offset = static_cast<int32_t>(std::round(acq_code_phase_samples));
    c.acc_carrier_phase_rad -= c.carrier_phase_step_rad * static_cast<double>(samples_offset);
    c.state = 2;
    c.nitems_read = a->first_sample + static_cast<uint64_t>(samples_offset);
    if (p.has_if) {  // IF phase at nitems_read: (if_mod · n) mod fs exactly (both factors < fs ≤ 4e9 → split n)
        const uint64_t fsu = static_cast<uint64_t>(p.fs_int);
        const unsigned __int128 prod = static_cast<unsigned __int128>(static_cast<uint64_t>(p.if_mod)) * (c.nitems_read % fsu);
        c.if_num = static_cast<int64_t>(prod % fsu);
        c.if_cyc = static_cast<double>(c.if_num) / static_cast<double>(p.fs_int);
    }
    // the channel's chunks carry its code replica(s) (host tables; the caller uploads them)
    for (int q = 0; q < p.jobs_per_channel; q++) {
        const int job = channel * p.jobs_per_channel + q;
        t->job_code[job] = q == 0 ? c.code_id : c.data_code_id;
        const CodeDesc& cd = ctx->codes_host[t->job_code[job]];
        for (int m = 0; m < p.chunks_per_job; m++) {
            ChunkDesc& d = t->chunks_host[t->jobs_first_chunk[job] + m];
            d.code = cd.ptr;
            d.code_len = cd.len;
        }
    }
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_start(gnsship_trk* t, int channel, const gnsship_trk_start_args* a)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    TrkChannel c;
    if (int rc = trk_start_state(t, channel, a, c)) return rc;
    if (int rc = set_device(ctx)) return rc;
    const TrkParams& p = t->params;
    // only the chunks' code fields are rewritten (the device owns the lengths)
    for (int q = 0; q < p.jobs_per_channel; q++) {
        const int job = channel * p.jobs_per_channel + q;
        for (int m = 0; m < p.chunks_per_job; m++) {
            const int ci = t->jobs_first_chunk[job] + m;
            const ChunkDesc& d = t->chunks_host[ci];
            HIP_TRY(ctx, hipMemcpyAsync(reinterpret_cast<char*>(t->chunks_dev + ci) + offsetof(ChunkDesc, code_len), &d.code_len,
                             sizeof(ChunkDesc) - offsetof(ChunkDesc, code_len), hipMemcpyHostToDevice, ctx->stream));
        }
        if (t->high_dyn) HIP_TRY(ctx, upload_hd_code(t, job, ctx->codes_host[t->job_code[job]]));
    }
    HIP_TRY(ctx, hipMemcpyAsync(t->chans_dev + channel, &c, sizeof(TrkChannel), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

// Scatter of staged channel states: block b copies channel record b to its slot idx[b].
__global__ void trk_scatter_kernel(TrkChannel* __restrict__ chans, const TrkChannel* __restrict__ staged, const int32_t* __restrict__ idx, int n)
{
    const int b = blockIdx.x;
    if (b >= n) return;
    constexpr int kWords = sizeof(TrkChannel) / 4;
    const int* src = reinterpret_cast<const int*>(staged + b);
    int* dst = reinterpret_cast<int*>(chans + idx[b]);
    for (int i = threadIdx.x; i < kWords; i += blockDim.x) dst[i] = src[i];
}

// n start_tracking calls at once: the channel states built on the host, one upload of states +
// channel indices, one scatter launch, one upload of the chunk table's code fields, one sync.
extern "C" int gnsship_trk_start_many(gnsship_trk* t, int n, const int32_t* channels, const gnsship_trk_start_args* args)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (n < 0 || (n > 0 && (!channels || !args))) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_start_many: bad arguments");
    if (n == 0) return GNSSHIP_OK;
    std::vector<int32_t> seen(t->max_channels, 0);
    for (int i = 0; i < n; i++) {
        if (channels[i] < 0 || channels[i] >= t->max_channels) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_start_many: bad channel");
        if (seen[channels[i]]++) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_start_many: a channel appears twice");
    }
    // staging: n TrkChannel records, then the n channel indices
    const size_t st_bytes = sizeof(TrkChannel) * static_cast<size_t>(n), idx_off = (st_bytes + 15) & ~size_t{15};
    std::vector<char> host(idx_off + sizeof(int32_t) * static_cast<size_t>(n));
    // validate and build every channel before anything reaches the device (a failure leaves the
    // device state untouched; the host code tables of the channels built so far are restored)
    const std::vector<int32_t> job_code_before = t->job_code;
    const std::vector<ChunkDesc> chunks_before = t->chunks_host;
    for (int i = 0; i < n; i++) {
        if (int rc = trk_start_state(t, channels[i], args + i, reinterpret_cast<TrkChannel*>(host.data())[i])) {
            t->job_code = job_code_before;
            t->chunks_host = chunks_before;
            return rc;
        }
    }
    std::memcpy(host.data() + idx_off, channels, sizeof(int32_t) * static_cast<size_t>(n));
    if (int rc = set_device(ctx)) return rc;
    if (t->start_stage_cap < host.size()) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (t->start_stage_dev) HIP_TRY(ctx, hipFree(t->start_stage_dev));
        t->start_stage_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&t->start_stage_dev, host.size()));
        t->start_stage_cap = host.size();
    }
    char* stage = static_cast<char*>(t->start_stage_dev);
    HIP_TRY(ctx, hipMemcpyAsync(stage, host.data(), host.size(), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(trk_scatter_kernel, dim3(n), dim3(256), 0, ctx->stream, t->chans_dev, reinterpret_cast<const TrkChannel*>(stage),
        reinterpret_cast<const int32_t*>(stage + idx_off), n);
    HIP_TRY(ctx, hipGetLastError());
    // the chunk table (the round-based loop's code pointers; its lengths are rewritten by the step
    // kernel before any correlation of a run)
    HIP_TRY(ctx, hipMemcpyAsync(t->chunks_dev, t->chunks_host.data(), sizeof(ChunkDesc) * t->n_chunks, hipMemcpyHostToDevice, ctx->stream));
    if (t->high_dyn)
        for (int i = 0; i < n; i++)
            for (int q = 0; q < t->params.jobs_per_channel; q++) {
                const int job = channels[i] * t->params.jobs_per_channel + q;
                HIP_TRY(ctx, upload_hd_code(t, job, ctx->codes_host[t->job_code[job]]));
            }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_stop(gnsship_trk* t, int channel)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (channel < 0 || channel >= t->max_channels) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_stop: bad channel");
    if (int rc = set_device(ctx)) return rc;
    const int32_t zero = 0;
    HIP_TRY(ctx, hipMemcpyAsync(reinterpret_cast<char*>(t->chans_dev + channel) + offsetof(TrkChannel, state), &zero, sizeof(zero),
                     hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_telemetry_event(gnsship_trk* t, int channel, int tlm_event)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (channel < 0 || channel >= t->max_channels) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_telemetry_event: bad channel");
    if (tlm_event != 1) return GNSSHIP_OK;  // only the telemetry fault is acted on (:623-629)
    if (int rc = set_device(ctx)) return rc;
    const int32_t forced = 200000;  // d_carrier_lock_fail_counter: force the loss-of-lock condition
    HIP_TRY(ctx, hipMemcpyAsync(reinterpret_cast<char*>(t->chans_dev + channel) + offsetof(TrkChannel, carrier_fail), &forced, sizeof(forced),
                     hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_channel_state(gnsship_trk* t, int channel, int* state, uint64_t* next_sample)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (channel < 0 || channel >= t->max_channels) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_channel_state: bad channel");
    if (int rc = set_device(ctx)) return rc;
    TrkChannel c;
    HIP_TRY(ctx, hipMemcpyAsync(&c, t->chans_dev + channel, sizeof(TrkChannel), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (state) *state = c.state;
    if (next_sample) *next_sample = c.nitems_read;
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_run(gnsship_trk* t, const void* sig, int fmt, int sig_on_device, uint64_t buffer_first_sample, int64_t n_buffer_samples,
    int max_rounds, gnsship_trk_epoch* out, int* rounds_done)
{
    return gnsship_trk_run_dump(t, sig, fmt, sig_on_device, buffer_first_sample, n_buffer_samples, max_rounds, out, nullptr, rounds_done);
}

// Enqueue a run on the context stream (the body of gnsship_trk_run_dump up to the record copies).
static int trk_enqueue(gnsship_trk* t, const void* src, int fmt, uint64_t buffer_first_sample, int64_t n_buffer_samples, int max_rounds, bool out,
    bool dump)
{
    gnsship_ctx* ctx = t->ctx;
    int max_len = 1;
    for (const auto& cd : ctx->codes_host)
        if (cd.ptr && cd.len > max_len) max_len = cd.len;
    if (t->attached_version != ctx->codes_version) {  // code bank changed: refresh every chunk's code pointer
        for (int job = 0; job < t->n_jobs; job++) {
            const int id = t->job_code[job];
            const bool ok = id >= 0 && id < static_cast<int>(ctx->codes_host.size());
            for (int m = 0; m < t->params.chunks_per_job; m++) {
                ChunkDesc& d = t->chunks_host[t->jobs_first_chunk[job] + m];
                d.code = ok ? ctx->codes_host[id].ptr : nullptr;
                d.code_len = ok ? ctx->codes_host[id].len : 0;
                d.len = 0;  // rewritten by the first step kernel of this run before any correlation
            }
            if (t->high_dyn) HIP_TRY(ctx, upload_hd_code(t, job, ok ? ctx->codes_host[id] : CodeDesc{nullptr, 0, 0}));
        }
        HIP_TRY(ctx, hipMemcpyAsync(t->chunks_dev, t->chunks_host.data(), sizeof(ChunkDesc) * t->n_chunks, hipMemcpyHostToDevice, ctx->stream));
        t->attached_version = ctx->codes_version;
    }
    const size_t nrec = static_cast<size_t>(max_rounds) * t->max_channels;
    if (dump && t->dump_cap < nrec) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (t->dump_dev) HIP_TRY(ctx, hipFree(t->dump_dev));
        t->dump_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&t->dump_dev, sizeof(gnsship_trk_dump_record) * nrec));
        t->dump_cap = nrec;
    }
    if (out && t->rec_cap < nrec) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (t->rec_dev) HIP_TRY(ctx, hipFree(t->rec_dev));
        t->rec_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&t->rec_dev, sizeof(gnsship_trk_epoch) * nrec));
        t->rec_cap = nrec;
    }
    if (t->ran_cap < static_cast<size_t>(max_rounds) + 1) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (t->ran_dev) HIP_TRY(ctx, hipFree(t->ran_dev));
        t->ran_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&t->ran_dev, sizeof(int) * (max_rounds + 1)));
        t->ran_cap = static_cast<size_t>(max_rounds) + 1;
    }
    HIP_TRY(ctx, hipMemsetAsync(t->ran_dev, 0, sizeof(int) * (max_rounds + 1), ctx->stream));
    const int nc = t->max_channels;
    const bool avx = t->params.conf.rotator == GNSSHIP_ROTATOR_AVX;
    const int code_cap = padded_code_quads(max_len) * 4;
    const bool persist = !t->high_dyn && trk_persist_supports(t->params) && trk_persist_lds_bytes(t->params, code_cap, avx) <= kTrkPersistMaxLds &&
                         !(t->force_rounds && !avx);
    if (avx && !persist) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_run: the AVX rotator needs the persistent loop (epoch too long for LDS)");
    gnsship_trk_corr_trace* trace = nullptr;
    t->trace_n = 0;
    if (t->trace_on && persist) {
        if (t->trace_cap < nrec) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if (t->trace_dev) HIP_TRY(ctx, hipFree(t->trace_dev));
            t->trace_dev = nullptr;
            HIP_TRY(ctx, hipMalloc(&t->trace_dev, sizeof(gnsship_trk_corr_trace) * nrec));
            t->trace_cap = nrec;
        }
        HIP_TRY(ctx, hipMemsetAsync(t->trace_dev, 0, sizeof(gnsship_trk_corr_trace) * nrec, ctx->stream));
        trace = t->trace_dev;
        t->trace_n = nrec;
    }
    if (persist) {
        // records of epochs a channel did not run stay zero (flags 0), as in the round-based loop
        if (out) HIP_TRY(ctx, hipMemsetAsync(t->rec_dev, 0, sizeof(gnsship_trk_epoch) * nrec, ctx->stream));
        if (dump) HIP_TRY(ctx, hipMemsetAsync(t->dump_dev, 0, sizeof(gnsship_trk_dump_record) * nrec, ctx->stream));
        const int n_codes = static_cast<int>(ctx->codes_host.size());
        hipError_t e;
        // the sign-bit replicas need every chip ±1 — of the codes this tracker's channels use
        bool binary = true;
        for (int id : t->job_code)
            if (id >= 0 && id < n_codes && ctx->codes_host[id].ptr && !ctx->codes_host[id].binary) binary = false;
        // GNSSHIP_TRK_FAST=0 (A/B runs against trk_persist.hip) turns both exact AVX forms off
        const char* fast_env = std::getenv("GNSSHIP_TRK_FAST");
        const bool no_fast = fast_env && fast_env[0] == '0';
        const bool lanes = avx && !no_fast && trk_lane_supported(t->params, code_cap, nc, fmt, n_buffer_samples, binary);
        const bool fast = avx && !lanes && trk_fast_supported(t->params, code_cap, nc);
        t->last_engine = GNSSHIP_TRK_ENGINE_NONE;
        if (lanes)
            e = launch_trk_lane(t->params_dev, t->params, t->chans_dev, nc, ctx->codes_dev, n_codes, code_cap, src, fmt, buffer_first_sample,
                n_buffer_samples, max_rounds, out ? t->rec_dev : nullptr, dump ? t->dump_dev : nullptr, trace, t->ran_dev, ctx->stream);
        else if (fast)
            e = launch_trk_fast(t->params_dev, t->params, t->chans_dev, nc, ctx->codes_dev, n_codes, code_cap, src, fmt, buffer_first_sample,
                n_buffer_samples, max_rounds, out ? t->rec_dev : nullptr, dump ? t->dump_dev : nullptr, trace, t->ran_dev, ctx->stream);
        else
            e = launch_trk_persist(t->params_dev, t->params, t->chans_dev, nc, ctx->codes_dev, n_codes, code_cap, src, fmt, buffer_first_sample,
                n_buffer_samples, max_rounds, out ? t->rec_dev : nullptr, dump ? t->dump_dev : nullptr, trace, t->ran_dev, avx, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, lanes ? "launch_trk_lane" : fast ? "launch_trk_fast" : "launch_trk_persist");
        t->last_engine = lanes  ? GNSSHIP_TRK_ENGINE_LANES
                         : fast ? (trk_fast_thru(nc) ? GNSSHIP_TRK_ENGINE_FAST_THROUGHPUT : GNSSHIP_TRK_ENGINE_FAST_LATENCY)
                                : GNSSHIP_TRK_ENGINE_PERSIST;
    }
    if (!persist) t->last_engine = GNSSHIP_TRK_ENGINE_ROUNDS;
    for (int r = 0; r <= max_rounds && !persist; r++) {
        const int consume = r > 0 ? 1 : 0, emit = r < max_rounds ? 1 : 0;
        gnsship_trk_epoch* rec = (out && r > 0) ? t->rec_dev + static_cast<size_t>(r - 1) * nc : nullptr;
        gnsship_trk_dump_record* drec = (dump && r > 0) ? t->dump_dev + static_cast<size_t>(r - 1) * nc : nullptr;
        hipError_t e = launch_trk_step(t->params_dev, t->chans_dev, nc, t->jobs_dev, t->chunks_dev, t->out_dev, buffer_first_sample, n_buffer_samples,
            consume, emit, rec, drec, t->ran_dev + r, t->hist_dev, t->high_dyn ? t->hd.jobs_dev : nullptr, t->high_dyn ? t->hd.chunks_dev : nullptr,
            t->high_dyn ? nullptr : t->anchors_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_trk_step");
        if (!emit) break;
        if (t->high_dyn) {
            t->hd.max_code_len = max_len;
            e = launch_corr_hd(src, fmt, t->hd, t->out_dev, ctx->stream);
            if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_hd(tracking)");
            continue;
        }
        e = launch_corr_batch(src, fmt, t->jobs_dev, t->n_jobs, t->chunks_dev, t->items_dev, t->n_items, t->classes, max_len, t->any_multi,
            t->anchors_dev, t->partials_dev, t->out_dev, ctx->stream, GNSSHIP_STAGE_CORRELATE);  // anchors: replayed by the step kernel
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_batch(tracking)");
    }
    t->pending_rounds = max_rounds;
    t->pending_out = out;
    t->pending_dump = dump;
    return GNSSHIP_OK;
}

// Wait for the enqueued run and copy its records (the tail of gnsship_trk_run_dump).
static int trk_finish(gnsship_trk* t, gnsship_trk_epoch* out, gnsship_trk_dump_record* dump, int* rounds_done)
{
    gnsship_ctx* ctx = t->ctx;
    const int max_rounds = t->pending_rounds;
    const size_t nrec = static_cast<size_t>(max_rounds) * t->max_channels;
    std::vector<int> ran(max_rounds + 1);
    HIP_TRY(ctx, hipMemcpyAsync(ran.data(), t->ran_dev, sizeof(int) * (max_rounds + 1), hipMemcpyDeviceToHost, ctx->stream));
    if ((out && !t->pending_out) || (dump && !t->pending_dump)) {  // the launch did not keep them: nothing to copy
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        t->pending_rounds = -1;
        if (rounds_done) {  // the launch ran and advanced the channels: report the epochs it consumed
            int n = 0;
            for (int r = 0; r < max_rounds; r++)
                if (ran[r] > 0) n = r + 1;
            *rounds_done = n;
        }
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_collect: records / dump requested that the launch did not keep (want_records / want_dump)");
    }
    if (out) HIP_TRY(ctx, hipMemcpyAsync(out, t->rec_dev, sizeof(gnsship_trk_epoch) * nrec, hipMemcpyDeviceToHost, ctx->stream));
    if (dump) HIP_TRY(ctx, hipMemcpyAsync(dump, t->dump_dev, sizeof(gnsship_trk_dump_record) * nrec, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    t->pending_rounds = -1;
    if (rounds_done) {
        int n = 0;
        for (int r = 0; r < max_rounds; r++)
            if (ran[r] > 0) n = r + 1;
        *rounds_done = n;
    }
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_run_dump(gnsship_trk* t, const void* sig, int fmt, int sig_on_device, uint64_t buffer_first_sample,
    int64_t n_buffer_samples, int max_rounds, gnsship_trk_epoch* out, gnsship_trk_dump_record* dump, int* rounds_done)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (!sig || n_buffer_samples < 0 || max_rounds < 0 || fmt_bytes(fmt) == 0) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_run: bad arguments");
    if (t->pending_rounds >= 0) return fail(ctx, GNSSHIP_E_STATE, "gnsship_trk_run: a gnsship_trk_launch is still pending (gnsship_trk_collect first)");
    if (rounds_done) *rounds_done = 0;
    if (max_rounds == 0) return GNSSHIP_OK;
    if (int rc = set_device(ctx)) return rc;
    if (int rc = sync_code_table(ctx)) return rc;
    const void* src = sig;
    if (!sig_on_device) {
        const size_t bytes = fmt_bytes(fmt) * static_cast<size_t>(n_buffer_samples);
        if (t->stage_cap < bytes) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if (t->stage_dev) HIP_TRY(ctx, hipFree(t->stage_dev));
            t->stage_dev = nullptr;
            HIP_TRY(ctx, hipMalloc(&t->stage_dev, bytes));
            t->stage_cap = bytes;
        }
        HIP_TRY(ctx, hipMemcpyAsync(t->stage_dev, sig, bytes, hipMemcpyHostToDevice, ctx->stream));
        src = t->stage_dev;
    }
    if (int rc = trk_enqueue(t, src, fmt, buffer_first_sample, n_buffer_samples, max_rounds, out != nullptr, dump != nullptr)) {
        t->pending_rounds = -1;
        return rc;
    }
    return trk_finish(t, out, dump, rounds_done);
}

extern "C" int gnsship_trk_launch(gnsship_trk* t, const void* dev_sig, int fmt, uint64_t buffer_first_sample, int64_t n_buffer_samples,
    int max_rounds, int want_records, int want_dump)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (!dev_sig || n_buffer_samples < 0 || max_rounds < 1 || fmt_bytes(fmt) == 0)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_launch: bad arguments (device buffer, max_rounds >= 1)");
    if (t->pending_rounds >= 0) return fail(ctx, GNSSHIP_E_STATE, "gnsship_trk_launch: the previous launch was not collected");
    if (int rc = set_device(ctx)) return rc;
    if (int rc = sync_code_table(ctx)) return rc;
    if (int rc = trk_enqueue(t, dev_sig, fmt, buffer_first_sample, n_buffer_samples, max_rounds, want_records != 0, want_dump != 0)) {
        t->pending_rounds = -1;
        return rc;
    }
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_collect(gnsship_trk* t, gnsship_trk_epoch* out, gnsship_trk_dump_record* dump, int* rounds_done)
{
    if (!t) return GNSSHIP_E_INVAL;
    if (t->pending_rounds < 0) return fail(t->ctx, GNSSHIP_E_STATE, "gnsship_trk_collect: nothing launched");
    if (int rc = set_device(t->ctx)) return rc;
    return trk_finish(t, out, dump, rounds_done);
}

extern "C" int gnsship_trk_set_trace(gnsship_trk* t, int enable)
{
    if (!t) return GNSSHIP_E_INVAL;
    t->trace_on = enable != 0;
    return GNSSHIP_OK;
}

extern "C" int gnsship_trk_trace_records(gnsship_trk* t, gnsship_trk_corr_trace* out, int max_records)
{
    if (!t) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = t->ctx;
    if (!out || max_records < 0) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_trace_records: bad arguments");
    if (t->trace_n == 0) return fail(ctx, GNSSHIP_E_STATE, "gnsship_trk_trace_records: no traced run (gnsship_trk_set_trace, persistent loop)");
    if (static_cast<size_t>(max_records) < t->trace_n) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_trk_trace_records: buffer smaller than the run");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(out, t->trace_dev, sizeof(gnsship_trk_corr_trace) * t->trace_n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}
