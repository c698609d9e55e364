// acq_resampler.hip — the acquisition resampler (GNSS-SDR.use_acquisition_resampler) for gfx950.
//
// Replaces the decimating FIR the flowgraph inserts in front of a channel's acquisition when the
// input rate exceeds the signal's optimum acquisition rate (gnss_flowgraph.cc:1028-1113):
//   decimation = floor(fs / acq_fs), decremented until it divides fs               (:1074-1079)
//   taps = gr::filter::firdes::low_pass(1.0, fs, acq_fs_dec / 2.1, acq_fs_dec / 2)  (:1085-1088)
//   gr::filter::fir_filter_ccf::make(decimation, taps)                              (:1090)
//   acquisition()->set_resampler_latency((taps.size() − 1) / 2)                     (:1113)
// and the adapters' Acq_Conf::ConfigureAutomaticResampler (acq_conf.cc:91-107), which picks the
// same decimation and runs the acquisition at resampled_fs.
//
// GNU Radio is not in the reference tree (version unpinned); its published algorithm is
// restated: firdes::low_pass with the default Hamming window (max attenuation 53: ntaps =
// (int)(53·fs / (22·transition)), made odd; windowed sinc; DC gain normalised to `gain`), and
// fir_filter_ccf with decimation D over a stream with ntaps − 1 samples of history (zeros before
// the first call): y[k] = Σ_{t<ntaps} x[k·D + t − (ntaps − 1)]·h[ntaps − 1 − t], each output a
// serial float dot product in t order as volk_32fc_32f_dot_prod_32fc_generic forms it.
//
// Device form: one 256-lane workgroup per tile of up to 256 outputs; the tile's input span
// ((outputs − 1)·D + ntaps samples, converted from the IF format in the load) and the reversed
// taps are staged in LDS once, then lane j forms output j serially.  HBM traffic is one read of
// the input plus the decimated output (2 or 8 B in, 8/D B out per input sample) — a streaming
// kernel far below the HBM roofline at receiver rates; it runs once per acquisition dwell.
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "engine.h"

#pragma clang fp contract(off)

namespace gnsship {
int fail(gnsship_ctx* ctx, int code, const char* what);
int hip_fail(gnsship_ctx* ctx, hipError_t e, const char* where);
int set_device(gnsship_ctx* ctx);
size_t fmt_bytes(int fmt);
}  // namespace gnsship

using namespace gnsship;

namespace {

constexpr int kFirThreads = 256;
constexpr int kFirMaxTaps = 4096;
constexpr int kFirSpanMax = 8192;  // float2 samples of input span staged per workgroup (64 KiB)

template <int FMT>
__device__ __forceinline__ float2 fir_load(const void* in, int64_t i)
{
    if constexpr (FMT == GNSSHIP_FMT_CF32) {
        return reinterpret_cast<const float2*>(in)[i];
    } else if constexpr (FMT == GNSSHIP_FMT_CI16) {
        const short2 v = reinterpret_cast<const short2*>(in)[i];
        return make_float2(static_cast<float>(v.x), static_cast<float>(v.y));
    } else {
        const char2 v = reinterpret_cast<const char2*>(in)[i];
        return make_float2(static_cast<float>(v.x), static_cast<float>(v.y));
    }
}

// Outputs [tile·opb, tile·opb + opb) ∩ [0, n_out).  hist: the previous call's last ntaps − 1 input
// samples (oldest first) standing in for x[−(ntaps − 1) .. −1].
template <int FMT>
__global__ __launch_bounds__(kFirThreads) void fir_decim_kernel(const void* __restrict__ in, const float2* __restrict__ hist,
    const float* __restrict__ taps_rev, int ntaps, int decim, int opb, int64_t n_out, float2* __restrict__ out)
{
    extern __shared__ float2 fir_lds[];
    float* h = reinterpret_cast<float*>(fir_lds);                // ntaps floats (padded to float2)
    float2* span = fir_lds + (ntaps + 1) / 2;
    const int64_t k0 = static_cast<int64_t>(blockIdx.x) * opb;
    const int64_t nk = (n_out - k0) < opb ? (n_out - k0) : opb;
    const int64_t base = k0 * decim - (ntaps - 1);
    const int len = static_cast<int>((nk - 1) * decim) + ntaps;
    for (int t = threadIdx.x; t < ntaps; t += kFirThreads) h[t] = taps_rev[t];
    for (int i = threadIdx.x; i < len; i += kFirThreads) {
        const int64_t g = base + i;
        span[i] = g < 0 ? hist[(ntaps - 1) + g] : fir_load<FMT>(in, g);
    }
    __syncthreads();
    const int j = threadIdx.x;
    if (j >= nk) return;
    const float2* x = span + static_cast<int64_t>(j) * decim;
    float re = 0.0f, im = 0.0f;
    for (int t = 0; t < ntaps; t++) {
        re = __fadd_rn(re, __fmul_rn(x[t].x, h[t]));
        im = __fadd_rn(im, __fmul_rn(x[t].y, h[t]));
    }
    out[k0 + j] = make_float2(re, im);
}

// History after a call of n_in samples: the last ntaps − 1 samples of (old history ‖ input).
template <int FMT>
__global__ void fir_history_kernel(const void* __restrict__ in, int64_t n_in, const float2* __restrict__ old_hist, int n_hist,
    float2* __restrict__ new_hist)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_hist) return;
    const int64_t g = n_in - n_hist + i;  // index into the input; < 0 reads the old history
    new_hist[i] = g < 0 ? old_hist[n_hist + g] : fir_load<FMT>(in, g);
}

// fft::window::coswindow(ntaps, 0.54, 0.46, 0) — the Hamming window of GNU Radio's firdes.
std::vector<float> hamming_window(int ntaps)
{
    std::vector<float> w(ntaps);
    const float M = static_cast<float>(ntaps - 1);
    for (int n = 0; n < ntaps; n++) {
        const double arg = (2.0 * M_PI * n) / static_cast<double>(M);
        w[n] = 0.54F - 0.46F * std::cos(static_cast<float>(arg));
    }
    return w;
}

}  // namespace

struct gnsship_acq_resampler {
    gnsship_ctx* ctx = nullptr;
    int ntaps = 0, decim = 1, opb = 0;
    int64_t max_in = 0;
    float* taps_rev_dev = nullptr;
    float2* hist_dev[2] = {nullptr, nullptr};
    int hist_cur = 0;
    void* stage_dev = nullptr;
    size_t stage_cap = 0;
    float2* out_dev = nullptr;
};

// gr::filter::firdes::low_pass(gain, fs, cutoff, transition) with the default Hamming window.
extern "C" int gnsship_firdes_low_pass(double gain, double sampling_freq, double cutoff_freq, double transition_width, float* taps, int taps_cap,
    int* n_taps)
{
    if (!n_taps || sampling_freq <= 0.0 || cutoff_freq <= 0.0 || cutoff_freq > sampling_freq / 2.0 || transition_width <= 0.0)
        return GNSSHIP_E_INVAL;  // firdes::sanity_check_1f
    int nt = static_cast<int>(53.0 * sampling_freq / (22.0 * transition_width));  // compute_ntaps, max_attenuation(HAMMING) = 53
    if ((nt & 1) == 0) nt++;
    *n_taps = nt;
    if (!taps) return GNSSHIP_OK;  // size query
    if (taps_cap < nt) return GNSSHIP_E_INVAL;
    const std::vector<float> w = hamming_window(nt);
    const int M = (nt - 1) / 2;
    const double fwT0 = 2.0 * M_PI * cutoff_freq / sampling_freq;
    for (int n = -M; n <= M; n++) {
        if (n == 0)
            taps[n + M] = static_cast<float>(fwT0 / M_PI * w[n + M]);
        else
            taps[n + M] = static_cast<float>(std::sin(n * fwT0) / (n * M_PI) * w[n + M]);
    }
    double fmax = taps[M];
    for (int n = 1; n <= M; n++) fmax += 2 * taps[n + M];
    gain /= fmax;
    for (int i = 0; i < nt; i++) taps[i] = static_cast<float>(taps[i] * gain);
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_resampler_design(int64_t fs_in, double opt_acq_fs, int* decimation, float* taps, int taps_cap, int* n_taps)
{
    if (!decimation || !n_taps || fs_in <= 0 || opt_acq_fs <= 0.0) return GNSSHIP_E_INVAL;
    *decimation = 1;
    *n_taps = 0;
    if (opt_acq_fs >= static_cast<double>(fs_in)) return GNSSHIP_OK;  // "input sampling frequency is too low"
    int d = static_cast<int>(std::floor(static_cast<double>(fs_in) / opt_acq_fs));
    while (d > 1 && fs_in % d > 0) d--;
    if (d <= 1) return GNSSHIP_OK;
    const double acq_fs_dec = static_cast<double>(fs_in) / static_cast<double>(d);
    *decimation = d;
    return gnsship_firdes_low_pass(1.0, static_cast<double>(fs_in), acq_fs_dec / 2.1, acq_fs_dec / 2.0, taps, taps_cap, n_taps);
}

extern "C" int gnsship_acq_resampler_destroy(gnsship_acq_resampler* r)
{
    if (!r) return GNSSHIP_E_INVAL;
    (void)hipSetDevice(r->ctx->device);
    (void)hipStreamSynchronize(r->ctx->stream);
    void* ptrs[] = {r->taps_rev_dev, r->hist_dev[0], r->hist_dev[1], r->stage_dev, r->out_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete r;
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_resampler_create(gnsship_ctx* ctx, const float* taps, int n_taps, int decimation, int64_t max_in_samples,
    gnsship_acq_resampler** out)
{
    if (!ctx || !out) return GNSSHIP_E_INVAL;
    *out = nullptr;
    if (!taps || n_taps < 1 || n_taps > kFirMaxTaps || decimation < 1 || max_in_samples < decimation)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_resampler_create: 1 <= n_taps <= 4096, decimation >= 1, max_in_samples >= decimation");
    const int opb = static_cast<int>(std::min<int64_t>(kFirThreads, (kFirSpanMax - n_taps) / decimation + 1));
    if (opb < 1) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_resampler_create: decimation x taps exceed the LDS span");
    if (int rc = set_device(ctx)) return rc;
    gnsship_acq_resampler* r = new (std::nothrow) gnsship_acq_resampler();
    if (!r) return GNSSHIP_E_NOMEM;
    r->ctx = ctx;
    r->ntaps = n_taps;
    r->decim = decimation;
    r->opb = opb;
    r->max_in = max_in_samples;
    std::vector<float> rev(n_taps);
    for (int t = 0; t < n_taps; t++) rev[t] = taps[n_taps - 1 - t];  // fir_filter's d_taps (reversed)
    const size_t hist_bytes = sizeof(float2) * static_cast<size_t>(n_taps > 1 ? n_taps - 1 : 1);
    hipError_t e = hipMalloc(&r->taps_rev_dev, sizeof(float) * n_taps);
    if (e == hipSuccess) e = hipMemcpy(r->taps_rev_dev, rev.data(), sizeof(float) * n_taps, hipMemcpyHostToDevice);
    for (int b = 0; b < 2 && e == hipSuccess; b++) {
        e = hipMalloc(&r->hist_dev[b], hist_bytes);
        if (e == hipSuccess) e = hipMemset(r->hist_dev[b], 0, hist_bytes);
    }
    if (e == hipSuccess) e = hipMalloc(&r->out_dev, sizeof(float2) * static_cast<size_t>(max_in_samples / decimation));
    if (e != hipSuccess) {
        gnsship_acq_resampler_destroy(r);
        return hip_fail(ctx, e, "gnsship_acq_resampler_create");
    }
    *out = r;
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_resampler_reset(gnsship_acq_resampler* r)
{
    if (!r) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = r->ctx;
    if (int rc = set_device(ctx)) return rc;
    const size_t hist_bytes = sizeof(float2) * static_cast<size_t>(r->ntaps > 1 ? r->ntaps - 1 : 1);
    for (int b = 0; b < 2; b++) {
        hipError_t e = hipMemsetAsync(r->hist_dev[b], 0, hist_bytes, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "gnsship_acq_resampler_reset");
    }
    return GNSSHIP_OK;
}

extern "C" int gnsship_acq_resampler_run(gnsship_acq_resampler* r, const void* in, int fmt, int in_on_device, int64_t n_in, float* host_out,
    void** dev_out, int64_t* n_out)
{
    if (!r) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = r->ctx;
    if (!in || fmt_bytes(fmt) == 0 || n_in < r->decim || n_in > r->max_in || n_in % r->decim != 0)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_acq_resampler_run: n_in must be a multiple of the decimation, <= max_in_samples");
    if (int rc = set_device(ctx)) return rc;
    const void* src = in;
    if (!in_on_device) {
        const size_t bytes = fmt_bytes(fmt) * static_cast<size_t>(n_in);
        if (r->stage_cap < bytes) {
            if (r->stage_dev) (void)hipFree(r->stage_dev);
            r->stage_dev = nullptr;
            r->stage_cap = 0;
            hipError_t e = hipMalloc(&r->stage_dev, bytes);
            if (e != hipSuccess) return hip_fail(ctx, e, "gnsship_acq_resampler_run(stage)");
            r->stage_cap = bytes;
        }
        hipError_t e = hipMemcpyAsync(r->stage_dev, in, bytes, hipMemcpyHostToDevice, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "gnsship_acq_resampler_run(upload)");
        src = r->stage_dev;
    }
    const int64_t nk = n_in / r->decim;
    const int64_t blocks = (nk + r->opb - 1) / r->opb;
    const int span_max = (r->opb - 1) * r->decim + r->ntaps;
    const size_t lds = sizeof(float2) * static_cast<size_t>((r->ntaps + 1) / 2 + span_max);
    const float2* hist = r->hist_dev[r->hist_cur];
    float2* hist_next = r->hist_dev[r->hist_cur ^ 1];
    const int n_hist = r->ntaps - 1;
    const int hb = (n_hist + 255) / 256;
    switch (fmt) {
    case GNSSHIP_FMT_CF32:
        hipLaunchKernelGGL(fir_decim_kernel<GNSSHIP_FMT_CF32>, dim3(static_cast<unsigned>(blocks)), dim3(kFirThreads), lds, ctx->stream, src, hist,
            r->taps_rev_dev, r->ntaps, r->decim, r->opb, nk, r->out_dev);
        if (n_hist > 0)
            hipLaunchKernelGGL(fir_history_kernel<GNSSHIP_FMT_CF32>, dim3(hb), dim3(256), 0, ctx->stream, src, n_in, hist, n_hist, hist_next);
        break;
    case GNSSHIP_FMT_CI16:
        hipLaunchKernelGGL(fir_decim_kernel<GNSSHIP_FMT_CI16>, dim3(static_cast<unsigned>(blocks)), dim3(kFirThreads), lds, ctx->stream, src, hist,
            r->taps_rev_dev, r->ntaps, r->decim, r->opb, nk, r->out_dev);
        if (n_hist > 0)
            hipLaunchKernelGGL(fir_history_kernel<GNSSHIP_FMT_CI16>, dim3(hb), dim3(256), 0, ctx->stream, src, n_in, hist, n_hist, hist_next);
        break;
    default:
        hipLaunchKernelGGL(fir_decim_kernel<GNSSHIP_FMT_CI8>, dim3(static_cast<unsigned>(blocks)), dim3(kFirThreads), lds, ctx->stream, src, hist,
            r->taps_rev_dev, r->ntaps, r->decim, r->opb, nk, r->out_dev);
        if (n_hist > 0)
            hipLaunchKernelGGL(fir_history_kernel<GNSSHIP_FMT_CI8>, dim3(hb), dim3(256), 0, ctx->stream, src, n_in, hist, n_hist, hist_next);
        break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "gnsship_acq_resampler_run(launch)");
    if (n_hist > 0) r->hist_cur ^= 1;
    if (host_out) {
        e = hipMemcpyAsync(host_out, r->out_dev, sizeof(float2) * static_cast<size_t>(nk), hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "gnsship_acq_resampler_run(download)");
    }
    if (dev_out) *dev_out = r->out_dev;
    if (n_out) *n_out = nk;
    return GNSSHIP_OK;
}
