// acq_abi.hip — C-ABI of the PCPS acquisition engine (include/gnsship.h, gnsship_acq_*).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <vector>

#include "acq_engine.h"
#include "engine.h"

namespace gnsship {
int fail(gnsship_ctx* ctx, int code, const char* what);
int hip_fail(gnsship_ctx* ctx, hipError_t e, const char* where);
size_t fmt_bytes(int fmt);

bool make_fft_plan(int n, FftPlan& plan)
{
    if (n < 2 || n > kMaxAcqN) return false;
    plan.n = n;
    plan.n_passes = 0;
    int m = n;
    const int radices[] = {8, 5, 4, 3, 2};
    for (int r : radices) {
        while (m % r == 0) {
            if (plan.n_passes >= kMaxPasses) return false;
            plan.radix[plan.n_passes++] = r;
            m /= r;
        }
    }
    return m == 1;
}

// Transform layout for size n: the single-pass LDS transform when it fits, else the four-step
// N = P·M (smallest supported P with M = N/P ≤ 1024 and M {2,3,5}-smooth).  force_big selects the
// four-step at sizes the LDS transform also covers (test knob GNSSHIP_ACQ_FORCE_BIG=1).
// Beyond that (or when no such P exists) the huge layout: N = P·M with P ∈ {4,…,32} register
// points and M ≤ 16384 LDS rows, as separate kernels (smallest P first: the longest LDS rows).
// force: 1 = four-step, 2 = huge, at sizes a smaller layout also covers (test knobs
// GNSSHIP_ACQ_FORCE_BIG=1 / GNSSHIP_ACQ_FORCE_HUGE=1).
bool choose_acq_layout(int n, int force, FftPlan& plan, int& P, bool& huge)
{
    P = 0;
    huge = false;
    // The four-step with a compile-time plan in small workgroups beats the single-workgroup LDS
    // transform at the C1 size (1 ms of GPS at 4 Msps: 4000 = 16 × 250).
    if (force == 0 && n == 4000 && make_fft_plan(250, plan)) {
        P = 16;
        return true;
    }
    if (force == 0 && make_fft_plan(n, plan)) return true;
    if (force != 2 && n >= 2 && n <= kMaxAcqBigN) {
        for (int p = 16; p <= 32; p++) {
            if (!big_p_supported(p) || n % p != 0) continue;
            const int m = n / p;
            if (m > kAcqThreads || m < 2) continue;
            if (make_fft_plan(m, plan)) {
                P = p;
                return true;
            }
        }
    }
    if (n < 8 || n > kMaxAcqHugeN) return false;
    // Prefer rows with a compile-time plan: 10000 = 10⁴ (four radix-10 passes, one butterfly per
    // thread) before 12500 (five passes, two or three butterflies per thread); GNSSHIP_ACQ_HUGE_P
    // picks P for measurement.
    int p_env = 0;
    if (const char* env = std::getenv("GNSSHIP_ACQ_HUGE_P")) p_env = std::atoi(env);
    for (const int mc : {10000, 12500}) {
        const int p = n / mc;
        if (n % mc != 0 || !huge_p_supported(p) || (p_env && p != p_env) || !make_fft_plan(mc, plan)) continue;
        P = p;
        huge = true;
        return true;
    }
    for (int p = 4; p <= 32; p++) {
        if (p_env && p != p_env) continue;
        if (!huge_p_supported(p) || n % p != 0) continue;
        if (make_fft_plan(n / p, plan)) {
            P = p;
            huge = true;
            return true;
        }
    }
    return false;
}
}  // namespace gnsship

using namespace gnsship;

#define HIP_TRY(ctx, expr)                                      \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return hip_fail((ctx), _e, #expr); \
    } while (0)

struct gnsship_acq {
    gnsship_ctx* ctx = nullptr;
    gnsship_acq_conf conf{};
    FftPlan plan{};              // whole transform (P == 0) or the M-point row transform (P > 0)
    int P = 0;                   // four-step / huge register points; spectra are then stored transposed
    bool huge = false;           // huge layout (separate column and row kernels)
    float2* twM = nullptr;       // huge: M twiddles exp(-2πi t/M) of the row transform
    float2* twC = nullptr;       // huge: the column twiddles in column layout, twC[kq·M + m] = exp(-2πi m·kq/N)
    float2* T = nullptr;         // huge: forward column-stage scratch, n_bins × N
    float2* U = nullptr;         // huge: inverse row-stage scratch, prn_batch × n_bins × N
    float* grid_scratch = nullptr; // unused: the huge search keeps no |y|² rows without a kept grid
    TileStat* tiles = nullptr;   // huge: lanes × prn_batch × n_bins × huge_tiles(M)
    int prn_batch = 0;
    int first_share = 50;        // huge, two lanes: percent of the PRNs in the first batch
    int lanes = 1;               // huge: PRN batches in flight together (U and tiles per lane)
    hipStream_t lane_stream = nullptr;  // huge, lanes = 2: the second batch lane
    hipEvent_t ev_fwd = nullptr, ev_lane = nullptr;
    int n_bins = 0;
    int dwell_count = 0;
    float2* tw = nullptr;        // N twiddles exp(-2πi t/N)
    float2* wipe = nullptr;      // n_bins × N Doppler wipeoffs
    float2* codes_fft = nullptr; // max_prns × N  conj(FFT(code))
    float2* X = nullptr;         // n_bins × N  FFT(in ⊙ w_b)
    RowStat* rowstat = nullptr;  // max_prns × n_bins
    // The decision kernel writes the results straight into mapped pinned host memory (res_dev is its
    // device address): no device-to-host copy after the sweep, only the host memcpy to the caller.
    gnsship_acq_result* res_host = nullptr;
    gnsship_acq_result* res_dev = nullptr;
    void* sig_dev = nullptr;     // staging for host input (N CF32)
    float* grid_dev = nullptr;   // optional |Y|² grid (max_prns × n_bins × N)
    size_t grid_bytes = 0;
    std::vector<char> code_set;
    int consumed = 0;            // d_consumed_samples: input samples used, the rest zero-padded
    Step2Spec step2{};           // make_2_steps: step-two grid active
    // The huge layout's sweep (forward transform, two batch lanes of row / column / finalize launches
    // with their events, decision) as one hipGraph, re-captured when any launch argument changes:
    // launched one by one it is 5 % slower (E1 0.760 → 0.797 ms).  The four launches of the other
    // layouts go straight to the stream: the graph's launch latency (≈ 12 µs to the first kernel)
    // outweighed the gaps it saved (C3 0.164 → 0.153 ms, C1 shape 0.069 → 0.058 ms without it).
    // GNSSHIP_ACQ_GRAPH=0 / 1: plain launches / a graph for every layout.
    hipGraphExec_t graph = nullptr;
    struct GraphKey {
        const void* src;
        int fmt, n_prns, accumulate, keep_grid, dwell;
        const float* grid;
        Step2Spec step2;
    } graph_key{};
    bool graph_broken = false;   // a capture failed once: plain launches from then on
    RowSpec rows() const
    {
        const int N = conf.fft_size;
        const bool bt = conf.bit_transition_flag != 0;
        return RowSpec{conf.samples_per_chip, bt ? N / 2 : 0, bt ? N / 2 : N, N};
    }
};

static void acq_graph_reset(gnsship_acq* a)
{
    if (a->graph) (void)hipGraphExecDestroy(a->graph);
    a->graph = nullptr;
}

static void acq_free_grid_buffers(gnsship_acq* a)
{
    acq_graph_reset(a);
    void* hp[] = {a->T, a->U, a->grid_scratch, a->tiles};
    for (void* p : hp)
        if (p) (void)hipFree(p);
    a->T = nullptr;
    a->U = nullptr;
    a->grid_scratch = nullptr;
    a->tiles = nullptr;
    a->prn_batch = 0;
    if (a->wipe) (void)hipFree(a->wipe);
    if (a->X) (void)hipFree(a->X);
    if (a->rowstat) (void)hipFree(a->rowstat);
    if (a->grid_dev) (void)hipFree(a->grid_dev);
    a->wipe = nullptr;
    a->X = nullptr;
    a->rowstat = nullptr;
    a->grid_dev = nullptr;
    a->grid_bytes = 0;
}

extern "C" int gnsship_acq_destroy(gnsship_acq* a)
{
    if (!a) return GNSSHIP_E_INVAL;
    (void)hipSetDevice(a->ctx->device);
    (void)hipStreamSynchronize(a->ctx->stream);
    acq_free_grid_buffers(a);
    acq_graph_reset(a);
    void* ptrs[] = {a->tw, a->twM, a->twC, a->codes_fft, a->sig_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (a->res_host) (void)hipHostFree(a->res_host);
    if (a->lane_stream) (void)hipStreamDestroy(a->lane_stream);
    if (a->ev_fwd) (void)hipEventDestroy(a->ev_fwd);
    if (a->ev_lane) (void)hipEventDestroy(a->ev_lane);
    delete a;
    return GNSSHIP_OK;
}

// Doppler wipeoff rows: row i = volk_gnsssdr_s32f_sincos_32fc_generic(−2π·f_i/fs) (update_local_carrier,
// pcps_acquisition.cc:232-245) — cosf/sinf of a float-accumulated phase, computed here on the host
// with the same libm so the table is bit-identical.
static int acq_upload_wipeoffs(gnsship_acq* a, int nb, const std::vector<float>& freqs)
{
    gnsship_ctx* ctx = a->ctx;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const int N = a->conf.fft_size;
    if (nb != a->n_bins || !a->wipe) {
        acq_free_grid_buffers(a);
        HIP_TRY(ctx, hipMalloc(&a->wipe, sizeof(float2) * static_cast<size_t>(nb) * N));
        HIP_TRY(ctx, hipMalloc(&a->X, sizeof(float2) * static_cast<size_t>(nb) * N));
        HIP_TRY(ctx, hipMalloc(&a->rowstat, sizeof(RowStat) * static_cast<size_t>(nb) * a->conf.max_prns));
        a->n_bins = nb;
        if (a->huge) {
            // PRNs searched per round: the PRNs split over the two batch lanes, one round each (E1 at 25
            // Msps: 2 × 16 PRNs, 1.05 GB of inverse row-stage scratch U), so that batch 0's column stage
            // and finalize overlap batch 1's row stage with the fewest persistent-row launches and
            // drains (GNSSHIP_ACQ_U_MIB caps U instead, for measurement: 0.84 ms at 2 × 16 against 0.89
            // at 11 + 11 + 10 and 0.94 at 16 rounds of 2; GNSSHIP_ACQ_SPLIT sets the first batch's
            // percentage: 18 + 14, 20 + 12 and 23 + 9 measured the same as 16 + 16).  Two batch lanes
            // (GNSSHIP_ACQ_LANES=1: one): batch i runs on lane i mod 2 with its own U and tiles.
            const size_t cell = static_cast<size_t>(nb) * N * sizeof(float2);
            a->lanes = 2;
            if (const char* env = std::getenv("GNSSHIP_ACQ_LANES")) a->lanes = std::atoi(env) == 1 ? 1 : 2;
            if (const char* env = std::getenv("GNSSHIP_ACQ_SPLIT")) a->first_share = std::min(95, std::max(5, std::atoi(env)));
            int pb = a->lanes == 2 ? (a->conf.max_prns * a->first_share + 99) / 100 : a->conf.max_prns;
            size_t u_cap = size_t(4) << 30;  // U above 4 GiB: more, smaller rounds
            if (const char* env = std::getenv("GNSSHIP_ACQ_U_MIB")) u_cap = static_cast<size_t>(std::max(1, std::atoi(env))) << 20;
            if (cell * pb * a->lanes > u_cap) pb = static_cast<int>(u_cap / (cell * a->lanes));
            a->prn_batch = pb < 1 ? 1 : (pb > a->conf.max_prns ? a->conf.max_prns : pb);
            const size_t tiles = static_cast<size_t>(a->prn_batch) * nb * huge_tiles(a->plan.n);
            HIP_TRY(ctx, hipMalloc(&a->T, sizeof(float2) * static_cast<size_t>(nb) * N));
            HIP_TRY(ctx, hipMalloc(&a->U, cell * a->prn_batch * a->lanes));
            HIP_TRY(ctx, hipMalloc(&a->tiles, sizeof(TileStat) * tiles * a->lanes));
            if (a->lanes == 2 && !a->lane_stream) {
                HIP_TRY(ctx, hipStreamCreateWithFlags(&a->lane_stream, hipStreamNonBlocking));
                HIP_TRY(ctx, hipEventCreateWithFlags(&a->ev_fwd, hipEventDisableTiming));
                HIP_TRY(ctx, hipEventCreateWithFlags(&a->ev_lane, hipEventDisableTiming));
            }
        }
    }
    std::vector<float2> host(static_cast<size_t>(nb) * N);
    const float two_pi = static_cast<float>(2.0 * M_PI);
    for (int i = 0; i < nb; i++) {
        const float step = -(two_pi * freqs[i] / static_cast<float>(a->conf.fs_in));
        float ph = 0.0F;
        float2* row = host.data() + static_cast<size_t>(i) * N;
        for (int n = 0; n < N; n++) {
            row[n] = make_float2(std::cos(ph), std::sin(ph));
            ph += step;
        }
    }
    HIP_TRY(ctx, hipMemcpy(a->wipe, host.data(), sizeof(float2) * host.size(), hipMemcpyHostToDevice));
    a->dwell_count = 0;
    return GNSSHIP_OK;
}

// update_grid_doppler_wipeoffs (pcps_acquisition.cc:295-302): f_i = −dmax + center + step·i (+ GLONASS
// bias, 0 for CDMA signals), nb = ceil(2·dmax/step) (:261).  Leaves step two.
extern "C" int gnsship_acq_set_grid(gnsship_acq* a, int doppler_max, int doppler_step, int doppler_center)
{
    if (!a) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = a->ctx;
    if (doppler_max < 0 || doppler_step <= 0) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_set_grid: doppler_max >= 0, doppler_step > 0");
    const int nb = static_cast<int>(std::ceil(static_cast<double>(2 * doppler_max) / static_cast<double>(doppler_step)));  // :261
    if (nb < 1) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_set_grid: empty Doppler grid");
    std::vector<float> f(nb);
    for (int i = 0; i < nb; i++) f[i] = static_cast<float>(-doppler_max + doppler_center + doppler_step * i);
    if (int rc = acq_upload_wipeoffs(a, nb, f)) return rc;
    a->conf.doppler_max = doppler_max;
    a->conf.doppler_step = doppler_step;
    a->conf.doppler_center = doppler_center;
    a->step2 = Step2Spec{};
    acq_graph_reset(a);
    return GNSSHIP_OK;
}

// update_grid_doppler_wipeoffs_step2 (pcps_acquisition.cc:305-312): the narrow grid of make_2_steps,
// f_i = center + (i − floor(nb2/2))·step2 in float.  Until the next gnsship_acq_set_grid, results
// report the step-two Doppler (:553-556) and, with the CFAR statistic, divide by the step-one input
// power passed here (d_input_power is not recomputed in step two, :516-525).
extern "C" int gnsship_acq_set_grid_step2(gnsship_acq* a, float doppler_center_step_two, float doppler_step2, int num_doppler_bins_step2,
    float step_one_input_power)
{
    if (!a) return GNSSHIP_E_INVAL;
    if (num_doppler_bins_step2 < 1 || !(doppler_step2 > 0.0f))
        return fail(a->ctx, GNSSHIP_E_INVAL, "gnsship_acq_set_grid_step2: num_doppler_bins_step2 >= 1, doppler_step2 > 0");
    std::vector<float> f(num_doppler_bins_step2);
    for (int i = 0; i < num_doppler_bins_step2; i++) {
        const float doppler = (static_cast<float>(i) - static_cast<float>(std::floor(num_doppler_bins_step2 / 2.0))) * doppler_step2;
        f[i] = doppler_center_step_two + doppler;
    }
    if (int rc = acq_upload_wipeoffs(a, num_doppler_bins_step2, f)) return rc;
    a->step2 = Step2Spec{1, doppler_center_step_two, doppler_step2, step_one_input_power};
    acq_graph_reset(a);
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_create(gnsship_ctx* ctx, const gnsship_acq_conf* conf, gnsship_acq** out)
{
    if (!ctx || !conf || !out) return GNSSHIP_E_INVAL;
    *out = nullptr;
    FftPlan plan;
    int P = 0;
    bool huge = false;
    const char* fb = std::getenv("GNSSHIP_ACQ_FORCE_BIG");
    const char* fh = std::getenv("GNSSHIP_ACQ_FORCE_HUGE");
    const int force = (fh && fh[0] == '1') ? 2 : ((fb && fb[0] == '1') ? 1 : 0);
    if (!choose_acq_layout(conf->fft_size, force, plan, P, huge))
        return fail(ctx, GNSSHIP_E_INVAL,
            "gnsship_acq_create: fft_size must be 2^a 3^b 5^c: <= 16384, or P*M (P in {16..32}, M <= 1024), or P*M (P in {4..32}, M <= 16384), max 524288");
    if (conf->fs_in <= 0 || conf->max_prns < 1 || conf->max_dwells < 1 || conf->samples_per_chip < 0 || conf->samples_per_code <= 0.0f)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_create: bad configuration");
    if (conf->consumed_samples < 0 || conf->consumed_samples > conf->fft_size || (conf->bit_transition_flag && (conf->fft_size & 1)))
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_create: consumed_samples in [0, fft_size]; bit_transition_flag needs an even fft_size");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    gnsship_acq* a = new (std::nothrow) gnsship_acq();
    if (!a) return GNSSHIP_E_NOMEM;
    a->ctx = ctx;
    a->conf = *conf;
    a->plan = plan;
    a->P = P;
    a->huge = huge;
    a->code_set.assign(conf->max_prns, 0);
    a->consumed = conf->consumed_samples > 0 ? conf->consumed_samples : conf->fft_size;
    const int N = conf->fft_size;
    std::vector<float2> tw(N);
    for (int t = 0; t < N; t++) {
        const double ang = -2.0 * M_PI * static_cast<double>(t) / static_cast<double>(N);
        tw[t] = make_float2(static_cast<float>(std::cos(ang)), static_cast<float>(std::sin(ang)));
    }
    hipError_t e = hipMalloc(&a->tw, sizeof(float2) * N);
    if (e == hipSuccess) e = hipMemcpy(a->tw, tw.data(), sizeof(float2) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&a->codes_fft, sizeof(float2) * static_cast<size_t>(N) * conf->max_prns);
    if (e == hipSuccess && huge && plan.n == 10000) e = ensure_lane_perm10();
    if (e == hipSuccess && huge) {
        const int M = plan.n;
        std::vector<float2> twm(M);
        for (int t = 0; t < M; t++) {
            const double ang = -2.0 * M_PI * static_cast<double>(t) / static_cast<double>(M);
            twm[t] = make_float2(static_cast<float>(std::cos(ang)), static_cast<float>(std::sin(ang)));
        }
        e = hipMalloc(&a->twM, sizeof(float2) * M);
        if (e == hipSuccess) e = hipMemcpy(a->twM, twm.data(), sizeof(float2) * M, hipMemcpyHostToDevice);
        // the N-table re-laid out for the column stages: thread m reads twC[kq·M + m] (consecutive
        // threads, consecutive entries) instead of tw[m·kq] (stride kq); the same values
        std::vector<float2> twc(static_cast<size_t>(N));
        for (int kq = 0; kq < P; kq++)
            for (int m = 0; m < M; m++) twc[static_cast<size_t>(kq) * M + m] = tw[static_cast<size_t>(m) * kq];
        if (e == hipSuccess) e = hipMalloc(&a->twC, sizeof(float2) * N);
        if (e == hipSuccess) e = hipMemcpy(a->twC, twc.data(), sizeof(float2) * N, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&a->res_host), sizeof(gnsship_acq_result) * conf->max_prns, hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&a->res_dev), a->res_host, 0);
    if (e == hipSuccess) e = hipMalloc(&a->sig_dev, sizeof(float2) * static_cast<size_t>(N));
    if (e != hipSuccess) {
        gnsship_acq_destroy(a);
        return hip_fail(ctx, e, "gnsship_acq_create");
    }
    if (int rc = gnsship_acq_set_grid(a, conf->doppler_max, conf->doppler_step, conf->doppler_center)) {
        gnsship_acq_destroy(a);
        return rc;
    }
    *out = a;
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_reset_dwells(gnsship_acq* a)
{
    if (!a) return GNSSHIP_E_INVAL;
    a->dwell_count = 0;
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_num_bins(gnsship_acq* a, int* n_bins)
{
    if (!a || !n_bins) return GNSSHIP_E_INVAL;
    *n_bins = a->n_bins;
    return GNSSHIP_OK;
}

// pcps_acquisition::set_local_code (:175-208), sampled_ms == ms_per_code, no bit-transition padding:
// FFT of the code, then volk_32fc_conjugate_32fc.
extern "C" int gnsship_acq_set_local_code(gnsship_acq* a, int prn_slot, const float* code)
{
    if (!a) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = a->ctx;
    if (!code || prn_slot < 0 || prn_slot >= a->conf.max_prns) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_set_local_code: bad slot / code");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const int N = a->conf.fft_size;
    // the FFT input buffer as set_local_code fills it (pcps_acquisition.cc:186-203): with
    // bit_transition_flag [N/2 zeros | code[0, N/2)]; with sampled_ms != ms_per_code
    // [N − consumed zeros | code[0, consumed)]; else code[0, N)
    const int n_code = a->conf.bit_transition_flag ? N / 2 : a->consumed;
    std::vector<float2> buf(static_cast<size_t>(N), make_float2(0.0f, 0.0f));
    std::memcpy(buf.data() + (N - n_code), code, sizeof(float2) * n_code);
    HIP_TRY(ctx, hipMemcpyAsync(a->sig_dev, buf.data(), sizeof(float2) * N, hipMemcpyHostToDevice, ctx->stream));
    float2* dst = a->codes_fft + static_cast<size_t>(prn_slot) * N;
    if (a->huge)
        HIP_TRY(ctx, launch_acq_fft_huge(a->sig_dev, GNSSHIP_FMT_CF32, nullptr, 1, a->P, a->plan, a->twC, a->twM, a->T, dst, 1, N, ctx->stream));
    else if (a->P)
        HIP_TRY(ctx, launch_acq_fft_big(a->sig_dev, GNSSHIP_FMT_CF32, nullptr, 1, a->P, a->plan, a->tw, dst, 1, N, ctx->stream));
    else
        HIP_TRY(ctx, launch_acq_fft_rows(a->sig_dev, GNSSHIP_FMT_CF32, nullptr, 1, a->plan, a->tw, dst, 1, N, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    a->code_set[prn_slot] = 1;
    return GNSSHIP_OK;
}

// acquisition_core (:600-871), step one, one dwell per call (dwells accumulate into the grid when
// max_dwells > 1 and a grid is kept on the device; the statistic divides by the dwell count).
extern "C" int gnsship_acq_run(gnsship_acq* a, const void* sig, int fmt, int sig_on_device, int n_prns, gnsship_acq_result* results,
    float* grid)
{
    if (!a) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = a->ctx;
    if (!sig || !results || n_prns < 1 || n_prns > a->conf.max_prns || fmt_bytes(fmt) == 0)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_run: bad arguments");
    for (int p = 0; p < n_prns; p++)
        if (!a->code_set[p]) return fail(ctx, GNSSHIP_E_STATE, "gnsship_acq_run: set_local_code missing for a prn slot");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const void* src = sig;
    if (!sig_on_device) {
        HIP_TRY(ctx, hipMemcpyAsync(a->sig_dev, sig, fmt_bytes(fmt) * a->consumed, hipMemcpyHostToDevice, ctx->stream));
        src = a->sig_dev;
    }
    const bool keep_grid = (grid != nullptr) || a->conf.max_dwells > 1;
    const RowSpec rs = a->rows();
    const size_t gbytes = sizeof(float) * static_cast<size_t>(a->conf.max_prns) * a->n_bins * rs.row_len;
    if (keep_grid && a->grid_bytes < gbytes) {
        if (a->grid_dev) HIP_TRY(ctx, hipFree(a->grid_dev));
        a->grid_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&a->grid_dev, gbytes));
        a->grid_bytes = gbytes;
    }
    // non-coherent dwells (:657-665): restart the accumulation after max_dwells
    if (a->dwell_count >= a->conf.max_dwells) a->dwell_count = 0;
    const int accumulate = (a->conf.max_dwells > 1 && a->dwell_count > 0) ? 1 : 0;
    a->dwell_count++;
    auto enqueue = [&]() -> int {
        if (a->huge) {
            HIP_TRY(ctx, launch_acq_fft_huge(src, fmt, a->wipe, a->n_bins, a->P, a->plan, a->twC, a->twM, a->T, a->X, 0, a->consumed, ctx->stream));
            const bool two = a->lanes == 2 && n_prns > a->prn_batch;
            if (two) {
                HIP_TRY(ctx, hipEventRecord(a->ev_fwd, ctx->stream));
                HIP_TRY(ctx, hipStreamWaitEvent(a->lane_stream, a->ev_fwd, 0));  // lane 1 reads the forward spectra
            }
            const size_t u_lane = static_cast<size_t>(a->prn_batch) * a->n_bins * a->conf.fft_size;
            const size_t t_lane = static_cast<size_t>(a->prn_batch) * a->n_bins * huge_tiles(a->plan.n);
            for (int p0 = 0, i = 0, np = 0; p0 < n_prns; p0 += np, i++) {
                np = std::min(a->prn_batch, n_prns - p0);
                if (two && i == 0) np = std::min(np, std::max(1, (n_prns * a->first_share + 99) / 100));
                const int lane = two ? (i & 1) : 0;  // batches i and i + 2 share a lane's U and tiles, in stream order
                // without a kept grid the |y|² rows never reach HBM (tile statistics + finalize's recomputation)
                float* g = keep_grid ? a->grid_dev + static_cast<size_t>(p0) * a->n_bins * rs.row_len : nullptr;
                HIP_TRY(ctx, launch_acq_search_huge(a->X, a->codes_fft, p0, np, a->n_bins, a->P, a->plan, a->twC, a->twM, a->U + lane * u_lane, g,
                                 keep_grid ? accumulate : 0, a->tiles + lane * t_lane, rs, a->rowstat, lane ? a->lane_stream : ctx->stream));
            }
            if (two) {  // the decision reads every batch's row statistics
                HIP_TRY(ctx, hipEventRecord(a->ev_lane, a->lane_stream));
                HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, a->ev_lane, 0));
            }
        } else if (a->P) {
            HIP_TRY(ctx, launch_acq_fft_big(src, fmt, a->wipe, a->n_bins, a->P, a->plan, a->tw, a->X, 0, a->consumed, ctx->stream));
            HIP_TRY(ctx, launch_acq_search_big(a->X, a->codes_fft, n_prns, a->n_bins, a->P, a->plan, a->tw, rs, accumulate,
                             a->rowstat, keep_grid ? a->grid_dev : nullptr, ctx->stream));
        } else {
            HIP_TRY(ctx, launch_acq_fft_rows(src, fmt, a->wipe, a->n_bins, a->plan, a->tw, a->X, 0, a->consumed, ctx->stream));
            HIP_TRY(ctx, launch_acq_search(a->X, a->codes_fft, n_prns, a->n_bins, a->plan, a->tw, rs, accumulate,
                             a->rowstat, keep_grid ? a->grid_dev : nullptr, ctx->stream));
        }
        HIP_TRY(ctx, launch_acq_decide(a->rowstat, n_prns, a->n_bins, rs.row_len, a->conf.doppler_max, a->conf.doppler_step, a->conf.doppler_center,
                         a->dwell_count, a->conf.use_cfar, a->conf.samples_per_code, a->conf.resampler_ratio > 0.0f ? a->conf.resampler_ratio : 1.0f,
                         a->conf.resampler_latency_samples, a->step2, a->res_dev, ctx->stream));
        return GNSSHIP_OK;
    };
    static const int graph_env = [] {
        const char* env = std::getenv("GNSSHIP_ACQ_GRAPH");
        return env ? (env[0] == '0' ? 0 : 1) : -1;
    }();
    const bool graphs_on = graph_env < 0 ? a->huge : graph_env == 1;
    if (graphs_on && !a->graph_broken) {
        const gnsship_acq::GraphKey key{src, fmt, n_prns, accumulate, keep_grid ? 1 : 0, a->dwell_count, keep_grid ? a->grid_dev : nullptr, a->step2};
        const bool same = a->graph && std::memcmp(&key, &a->graph_key, sizeof(key)) == 0;
        if (!same) {
            acq_graph_reset(a);
            hipGraph_t g = nullptr;
            int rc = GNSSHIP_OK;
            if (hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal) == hipSuccess) {
                rc = enqueue();
                const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
                if (rc == GNSSHIP_OK && e == hipSuccess && g && hipGraphInstantiate(&a->graph, g, nullptr, nullptr, 0) == hipSuccess)
                    a->graph_key = key;
                else
                    a->graph = nullptr;
                if (g) (void)hipGraphDestroy(g);
            }
            (void)hipGetLastError();
            if (!a->graph) {  // capture unavailable: launch directly, now and from now on
                a->graph_broken = true;
                if (int rc2 = enqueue()) return rc2;
            }
        }
        if (a->graph) HIP_TRY(ctx, hipGraphLaunch(a->graph, ctx->stream));
    } else if (int rc = enqueue()) {
        return rc;
    }
    if (grid)
        HIP_TRY(ctx, hipMemcpyAsync(grid, a->grid_dev, sizeof(float) * static_cast<size_t>(n_prns) * a->n_bins * rs.row_len, hipMemcpyDeviceToHost,
                         ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(results, a->res_host, sizeof(gnsship_acq_result) * n_prns);
    return GNSSHIP_OK;
}
static_assert(sizeof(gnsship_acq_conf) == 64, "gnsship_acq_conf layout (abi.AcqConf)");
