// gnsship_abi.hip — C-ABI implementation (include/gnsship.h): contexts, device buffers, the code
// bank, the per-channel correlator handle and the batched correlator.  The acquisition entry
// points live in acq_abi.hip.  No exception or exit() crosses the ABI: every entry point maps
// failures to an int status and keeps the message in ctx->last_error.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>

#include "engine.h"

using namespace gnsship;

namespace gnsship {

int fail(gnsship_ctx* ctx, int code, const char* what)
{
    if (ctx) ctx->last_error = what;
    return code;
}

int hip_fail(gnsship_ctx* ctx, hipError_t e, const char* where)
{
    if (ctx) {
        char buf[256];
        std::snprintf(buf, sizeof(buf), "%s: %s", where, hipGetErrorString(e));
        ctx->last_error = buf;
    }
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? GNSSHIP_E_NOMEM : GNSSHIP_E_DEVICE;
}

#define HIP_TRY(ctx, expr)                                      \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return hip_fail((ctx), _e, #expr); \
    } while (0)

int set_device(gnsship_ctx* ctx)
{
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return GNSSHIP_OK;
}

// Upload the code bank table when codes changed (synchronous w.r.t. the ctx stream).
int sync_code_table(gnsship_ctx* ctx)
{
    if (!ctx->codes_dirty) return GNSSHIP_OK;
    const int n = static_cast<int>(ctx->codes_host.size());
    if (n > ctx->codes_dev_cap) {
        if (ctx->codes_dev) HIP_TRY(ctx, hipFree(ctx->codes_dev));
        ctx->codes_dev = nullptr;
        const int cap = n < 64 ? 64 : 2 * n;
        HIP_TRY(ctx, hipMalloc(&ctx->codes_dev, sizeof(CodeDesc) * cap));
        ctx->codes_dev_cap = cap;
    }
    HIP_TRY(ctx, hipMemcpyAsync(ctx->codes_dev, ctx->codes_host.data(), sizeof(CodeDesc) * n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->codes_dirty = false;
    return GNSSHIP_OK;
}

// Host-side derivation of the device job from one reference-style call (see engine.h DevJob).
// The phasors are formed with the reference's float operations:
//   phase_offset_as_complex = (cos(rem), -sin(rem))             cpu_multicorrelator_real_codes.cc:115
//   phase_inc = std::exp(complex<float>(0, -phase_step_rad))     :123  (glibc cexpf → cosf/sinf)
bool derive_job(const gnsship_corr_job& in, int code_len, DevJob& out)
{
    // ≤ 2^24 samples per call: (float)n then steps exactly by 1 in the correlator's lanes
    if (in.n_samples < 0 || in.n_samples > (1 << 24) || in.n_taps < 1 || in.n_taps > kMaxTaps || in.sample_offset < 0) return false;
    if (in.flags & 1) return false;  // high-dynamics variants: not on the device path yet
    const float p0r = std::cos(in.rem_carrier_phase_rad), p0i = -std::sin(in.rem_carrier_phase_rad);
    const float incr = std::cos(-in.phase_step_rad), inci = std::sin(-in.phase_step_rad);
    out.sample_offset = in.sample_offset;
    out.n_samples = in.n_samples;
    out.code_id = in.code_id;
    out.n_taps = in.n_taps;
    out.p0_re = p0r;
    out.p0_im = p0i;
    out.inc_re = incr;
    out.inc_im = inci;
    out.dtheta = std::atan2(static_cast<double>(inci), static_cast<double>(incr));
    out.log_mag_inc = static_cast<float>(std::log(std::hypot(static_cast<double>(incr), static_cast<double>(inci))));
    // AVX variant: dz = inc^16 by four written-out float squarings (dz *= dz, :221-225), then
    // _mm256_complexnormalise_ps (IEEE sqrt and division); host and device form it identically
    // (-ffp-contract=off), the replay and the correlation both read this value
    out.rot_avx = (in.flags & GNSSHIP_JOB_ROTATOR_AVX) ? 1 : 0;
    out.dz_re = 1.0f;
    out.dz_im = 0.0f;
    if (out.rot_avx) {
        float dr = incr, di = inci;
        for (int q = 0; q < 4; q++) {
            const float a = dr * dr, b = di * di, c = dr * di, d = di * dr;
            dr = a - b;
            di = c + d;
        }
        const float m = std::sqrt(dr * dr + di * di);
        out.dz_re = dr / m;
        out.dz_im = di / m;
    }
    out.rem_code = in.rem_code_phase_chips;
    out.code_step = in.code_phase_step_chips;
    for (int t = 0; t < kMaxTaps; t++) out.shifts[t] = (t < in.n_taps) ? in.shifts_chips[t] : 0.0f;
    // Range of floor(step·n + shift − rem) over the job, bounded in double with 2 chips of slack
    // (each float rounding moves a value < 2^15 by far less than one chip): inside the padded
    // LDS replica the kernel skips the modulo.
    double smin = in.shifts_chips[0], smax = in.shifts_chips[0];
    for (int t = 1; t < in.n_taps; t++) {
        smin = std::min(smin, static_cast<double>(in.shifts_chips[t]));
        smax = std::max(smax, static_cast<double>(in.shifts_chips[t]));
    }
    const double span = static_cast<double>(in.code_phase_step_chips) * static_cast<double>(in.n_samples > 0 ? in.n_samples - 1 : 0);
    const double lo = std::min(0.0, span) + smin - in.rem_code_phase_chips - 2.0;
    const double hi = std::max(0.0, span) + smax - in.rem_code_phase_chips + 2.0;
    out.in_margin = (std::isfinite(lo) && std::isfinite(hi) && lo >= -kCodeMargin && hi < static_cast<double>(code_len + kCodeMargin)) ? 1 : 0;
    return true;
}

// Split jobs into ≤kCorrChunk-sample chunks, lay out their rotator anchors and group the chunks of
// each class into work items (see engine.h).  Returns the number of chunks.
int plan_chunks(std::vector<DevJob>& jobs, std::vector<ChunkDesc>& chunks, std::vector<WorkItem>& items, bool& any_multi, int64_t* n_anchors,
    ChunkClass* classes, int chunks_per_item, bool pair_by_code)
{
    chunks.clear();
    items.clear();
    any_multi = false;
    chunks_per_item = chunks_per_item < 1 ? 1 : (chunks_per_item > kMaxChunksPerItem ? kMaxChunksPerItem : chunks_per_item);
    int64_t anchors = 0;
    for (size_t j = 0; j < jobs.size(); j++) {
        const int n = jobs[j].n_samples;
        jobs[j].anchor_offset = static_cast<int32_t>(anchors);
        anchors += anchor_entries(n > 0 ? n : 0, jobs[j].rot_avx != 0);
        jobs[j].n_chunks = n <= 0 ? 1 : (n + kCorrChunk - 1) / kCorrChunk;
        if (jobs[j].n_chunks > 1) any_multi = true;
    }
    auto job_chunk = [&](int j, int k) {
        ChunkDesc d;
        d.job = j;
        d.start = k * kCorrChunk;
        const int rem = jobs[j].n_samples - d.start;
        d.len = rem < kCorrChunk ? (rem > 0 ? rem : 0) : kCorrChunk;
        d.code_len = 0;
        d.code = nullptr;
        return d;
    };
    // chunks grouped by class (one launch each), job order kept inside a class
    for (int c = 0; c < kChunkClasses; c++) {
        classes[c].start = static_cast<int32_t>(items.size());
        std::map<int, std::vector<int>> open;  // code id → pending single-chunk jobs
        auto emit_jobs = [&](std::vector<int>& js) {
            WorkItem it{static_cast<int32_t>(chunks.size()), static_cast<int32_t>(js.size())};
            for (int j : js) {
                jobs[j].first_chunk = static_cast<int32_t>(chunks.size());
                chunks.push_back(job_chunk(j, 0));
            }
            items.push_back(it);
            js.clear();
        };
        for (size_t j = 0; j < jobs.size(); j++) {
            if (chunk_class(jobs[j].n_taps, jobs[j].in_margin, jobs[j].rot_avx) != c) continue;
            const int nch = jobs[j].n_chunks;
            if (nch == 1 && pair_by_code && chunks_per_item > 1) {
                std::vector<int>& pend = open[jobs[j].code_id];
                pend.push_back(static_cast<int>(j));
                if (static_cast<int>(pend.size()) == chunks_per_item) emit_jobs(pend);
                continue;
            }
            // a long job: its chunks contiguous and in order, cut into items
            jobs[j].first_chunk = static_cast<int32_t>(chunks.size());
            for (int k = 0; k < nch; k += chunks_per_item) {
                const int cnt = std::min(chunks_per_item, nch - k);
                items.push_back(WorkItem{static_cast<int32_t>(chunks.size()), cnt});
                for (int m = 0; m < cnt; m++) chunks.push_back(job_chunk(static_cast<int>(j), k + m));
            }
        }
        for (auto& kv : open)
            if (!kv.second.empty()) emit_jobs(kv.second);
        classes[c].count = static_cast<int32_t>(items.size()) - classes[c].start;
    }
    *n_anchors = anchors > 0 ? anchors : 1;
    return static_cast<int>(chunks.size());
}

hipError_t upload_padded_code(const float* code, int len, float** chip0)
{
    std::vector<float> pad(static_cast<size_t>(padded_code_quads(len)) * 4, 0.0f);
    for (int i = -kCodeMargin; i < len + kCodeMargin; i++) pad[i + kCodeMargin] = code[((i % len) + len) % len];
    float* base = nullptr;
    hipError_t e = hipMalloc(&base, sizeof(float) * pad.size());
    if (e != hipSuccess) return e;
    e = hipMemcpy(base, pad.data(), sizeof(float) * pad.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(base);
        return e;
    }
    *chip0 = base + kCodeMargin;
    return hipSuccess;
}

hipError_t free_padded_code(const float* chip0)
{
    return chip0 ? hipFree(const_cast<float*>(chip0 - kCodeMargin)) : hipSuccess;
}

int chunks_per_item_setting()
{
    const char* e = std::getenv("GNSSHIP_CHUNKS_PER_ITEM");  // tuning knob
    const int v = e ? std::atoi(e) : kChunksPerItemDefault;
    return v < 1 ? 1 : (v > kMaxChunksPerItem ? kMaxChunksPerItem : v);
}

void attach_codes(std::vector<ChunkDesc>& chunks, const std::vector<DevJob>& jobs, const std::vector<CodeDesc>& table)
{
    for (auto& c : chunks) {
        const int id = jobs[c.job].code_id;
        const bool ok = id >= 0 && id < static_cast<int>(table.size());
        c.code = ok ? table[id].ptr : nullptr;
        c.code_len = ok ? table[id].len : 0;
    }
}

size_t fmt_bytes(int fmt)
{
    switch (fmt) {
    case GNSSHIP_FMT_CF32: return 8;
    case GNSSHIP_FMT_CI16: return 4;
    case GNSSHIP_FMT_CI8: return 2;
    default: return 0;
    }
}

}  // namespace gnsship

// ============================================================================ context / buffers
extern "C" int gnsship_abi_version(void) { return GNSSHIP_ABI_VERSION; }


extern "C" int gnsship_device_count(int* n)
{
    if (!n) return GNSSHIP_E_INVAL;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        return GNSSHIP_E_DEVICE;
    }
    *n = c;
    return GNSSHIP_OK;
}

extern "C" int gnsship_ctx_create(int device, gnsship_ctx** out)
{
    if (!out) return GNSSHIP_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GNSSHIP_E_DEVICE;
    if (device < 0 || device >= n) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = new (std::nothrow) gnsship_ctx();
    if (!ctx) return GNSSHIP_E_NOMEM;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return GNSSHIP_E_DEVICE;
    }
    for (auto& ev : ctx->events) {
        if (hipEventCreate(&ev) != hipSuccess) {
            delete ctx;
            return GNSSHIP_E_DEVICE;
        }
    }
    *out = ctx;
    return GNSSHIP_OK;
}

extern "C" int gnsship_ctx_destroy(gnsship_ctx* ctx)
{
    if (!ctx) return GNSSHIP_E_INVAL;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& c : ctx->codes_host)
        if (c.ptr) (void)free_padded_code(c.ptr);
    if (ctx->codes_dev) (void)hipFree(ctx->codes_dev);
    for (auto& ev : ctx->events)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return GNSSHIP_OK;
}

extern "C" const char* gnsship_last_error(const gnsship_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

extern "C" int gnsship_ctx_sync(gnsship_ctx* ctx)
{
    if (!ctx) return GNSSHIP_E_INVAL;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_ctx_stream(gnsship_ctx* ctx, void** stream)
{
    if (!ctx || !stream) return GNSSHIP_E_INVAL;
    *stream = reinterpret_cast<void*>(ctx->stream);
    return GNSSHIP_OK;
}

extern "C" int gnsship_ctx_event_record(gnsship_ctx* ctx, int slot)
{
    if (!ctx || slot < 0 || slot >= 16) return GNSSHIP_E_INVAL;
    HIP_TRY(ctx, hipEventRecord(ctx->events[slot], ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_ctx_event_elapsed_ms(gnsship_ctx* ctx, int a, int b, float* ms)
{
    if (!ctx || !ms || a < 0 || a >= 16 || b < 0 || b >= 16) return GNSSHIP_E_INVAL;
    HIP_TRY(ctx, hipEventSynchronize(ctx->events[b]));
    HIP_TRY(ctx, hipEventElapsedTime(ms, ctx->events[a], ctx->events[b]));
    return GNSSHIP_OK;
}

extern "C" int gnsship_dev_alloc(gnsship_ctx* ctx, size_t bytes, void** p)
{
    if (!ctx || !p) return GNSSHIP_E_INVAL;
    *p = nullptr;
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(ctx, hipMalloc(p, bytes ? bytes : 16));
    return GNSSHIP_OK;
}

extern "C" int gnsship_dev_free(gnsship_ctx* ctx, void* p)
{
    if (!ctx) return GNSSHIP_E_INVAL;
    if (!p) return GNSSHIP_OK;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(p));
    return GNSSHIP_OK;
}

extern "C" int gnsship_dev_upload(gnsship_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (!ctx || (!dst && bytes) || (!src && bytes)) return GNSSHIP_E_INVAL;
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_dev_download(gnsship_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (!ctx || (!dst && bytes) || (!src && bytes)) return GNSSHIP_E_INVAL;
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_code_set(gnsship_ctx* ctx, int code_id, const float* code, int len)
{
    if (!ctx || !code || code_id < 0 || code_id >= (1 << 20) || len < 1 || len > kMaxCodeLen)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_code_set: bad code id / length (1..16384)");
    if (int rc = set_device(ctx)) return rc;
    if (static_cast<int>(ctx->codes_host.size()) <= code_id) ctx->codes_host.resize(code_id + 1, CodeDesc{nullptr, 0, 0});
    CodeDesc& d = ctx->codes_host[code_id];
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (d.ptr) {
        HIP_TRY(ctx, free_padded_code(d.ptr));
        d.ptr = nullptr;
        d.len = 0;
    }
    float* p = nullptr;
    HIP_TRY(ctx, upload_padded_code(code, len, &p));
    d.ptr = p;
    d.len = len;
    d.binary = 1;
    for (int i = 0; i < len; i++)
        if (code[i] != 1.0f && code[i] != -1.0f) d.binary = 0;
    ctx->codes_dirty = true;
    ctx->codes_version++;
    return GNSSHIP_OK;
}

extern "C" int gnsship_code_count(gnsship_ctx* ctx, int* n)
{
    if (!ctx || !n) return GNSSHIP_E_INVAL;
    *n = static_cast<int>(ctx->codes_host.size());
    return GNSSHIP_OK;
}

// ============================================================================ batched correlator
struct gnsship_batch {
    gnsship_ctx* ctx = nullptr;
    int max_jobs = 0;
    int n_jobs = 0;
    int n_chunks = 0;
    int max_code_len = 1;
    bool any_multi = false;
    ChunkClass classes[kChunkClasses] = {};
    int chunk_cap = 0;
    int n_items = 0;
    int item_cap = 0;
    DevJob* jobs_dev = nullptr;
    ChunkDesc* chunks_dev = nullptr;
    WorkItem* items_dev = nullptr;
    float* partials_dev = nullptr;
    float* out_dev = nullptr;
    Anchor* anchors_dev = nullptr;
    int64_t anchor_cap = 0;
    std::vector<DevJob> jobs_host;
    std::vector<ChunkDesc> chunks_host;
    std::vector<WorkItem> items_host;
    // The anchor replay (NCO arguments only, latency-bound, few waves) runs on the batch's own
    // stream; the correlation on the context stream waits for it.  With two batches in flight the
    // replay of one overlaps the correlation of the other.
    hipStream_t aux = nullptr;
    hipEvent_t anchors_ready = nullptr;  // aux → ctx: anchors written
    hipEvent_t corr_done = nullptr;      // ctx → aux: correlation finished reading the anchors
    // gnsship_batch_launch_pipelined(2): replay segments of the current job set already written on
    // the context stream by launches that carried this batch as `next` / `next2` (0..kAnchorSegments);
    // cleared by set_jobs.
    int anchor_segs = 0;
    int replay_lanes = 1;  // kAvxLanes when any job uses the AVX rotator variant
    // high-dynamics jobs (flags bit 0): correlated by corr_hd_kernel.hip after the main classes; their
    // slots in the main plan are empty jobs
    HdPlan hd;
    // generic-rotator jobs in the reference's serial order (no AVX / TREE / HIGH_DYN flag):
    // corr_serial.hip after the main classes, likewise empty slots in the main plan
    std::vector<SerialJob> serial;
    SerialJob* serial_dev = nullptr;
    int serial_cap = 0;
};

static void batch_release(gnsship_batch* b)
{
    hd_plan_free(b->hd);
    void* ptrs[] = {b->jobs_dev, b->chunks_dev, b->items_dev, b->partials_dev, b->out_dev, b->anchors_dev, b->serial_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (b->anchors_ready) (void)hipEventDestroy(b->anchors_ready);
    if (b->corr_done) (void)hipEventDestroy(b->corr_done);
    if (b->aux) (void)hipStreamDestroy(b->aux);
    delete b;
}

extern "C" int gnsship_batch_create(gnsship_ctx* ctx, int max_jobs, gnsship_batch** out)
{
    if (!ctx || !out || max_jobs < 1) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_create: bad arguments");
    *out = nullptr;
    if (int rc = set_device(ctx)) return rc;
    gnsship_batch* b = new (std::nothrow) gnsship_batch();
    if (!b) return GNSSHIP_E_NOMEM;
    b->ctx = ctx;
    b->max_jobs = max_jobs;
    hipError_t e = hipMalloc(&b->jobs_dev, sizeof(DevJob) * max_jobs);
    if (e == hipSuccess) e = hipMalloc(&b->out_dev, sizeof(float) * 2 * kMaxTaps * max_jobs);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->aux, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b->anchors_ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b->corr_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(b->corr_done, ctx->stream);
    if (e != hipSuccess) {
        batch_release(b);
        return hip_fail(ctx, e, "gnsship_batch_create");
    }
    *out = b;
    return GNSSHIP_OK;
}

extern "C" int gnsship_batch_set_jobs(gnsship_batch* b, const gnsship_corr_job* jobs, int n_jobs, int64_t n_buffer_samples)
{
    if (!b) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = b->ctx;
    if ((!jobs && n_jobs) || n_jobs < 0 || n_jobs > b->max_jobs) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: n_jobs out of range");
    if (int rc = set_device(ctx)) return rc;
    b->anchor_segs = 0;
    if (int rc = sync_code_table(ctx)) return rc;
    b->jobs_host.resize(n_jobs);
    b->hd.jobs.clear();
    b->serial.clear();
    int max_len = 1;
    for (int j = 0; j < n_jobs; j++) {
        const gnsship_corr_job& in = jobs[j];
        if (in.code_id < 0 || in.code_id >= static_cast<int>(ctx->codes_host.size()) || !ctx->codes_host[in.code_id].ptr)
            return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: job refers to an unset code id");
        if (in.flags & ~(GNSSHIP_JOB_HIGH_DYN | GNSSHIP_JOB_ROTATOR_AVX | GNSSHIP_JOB_ROTATOR_TREE))
            return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: unknown job flags");
        if ((in.flags & GNSSHIP_JOB_ROTATOR_AVX) && (in.flags & GNSSHIP_JOB_ROTATOR_TREE))
            return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: GNSSHIP_JOB_ROTATOR_AVX and _TREE are exclusive");
        if (in.flags & 1) {  // high-dynamics resampler/rotator: its own plan, an empty slot here
            HdJob h;
            if (!derive_hd_job(in, ctx->codes_host[in.code_id].ptr, ctx->codes_host[in.code_id].len, j, h))
                return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: invalid high-dynamics job (taps, length, offset or tap shifts)");
            b->hd.jobs.push_back(h);
            gnsship_corr_job empty = in;
            empty.flags = 0;
            empty.n_samples = 0;
            derive_job(empty, ctx->codes_host[in.code_id].len, b->jobs_host[j]);
            if (in.sample_offset + in.n_samples > n_buffer_samples) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: job reads past the sample buffer");
            continue;
        }
        if (!derive_job(in, ctx->codes_host[in.code_id].len, b->jobs_host[j]))
            return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: invalid job (taps, length, offset or flags)");
        if (in.sample_offset + in.n_samples > n_buffer_samples) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_set_jobs: job reads past the sample buffer");
        if (!(in.flags & (GNSSHIP_JOB_ROTATOR_AVX | GNSSHIP_JOB_ROTATOR_TREE))) {  // generic, serial order: its own kernel
            const CodeDesc& cd = ctx->codes_host[in.code_id];
            b->serial.push_back(SerialJob{b->jobs_host[j], cd.ptr, cd.len, j});
            gnsship_corr_job empty = in;
            empty.n_samples = 0;
            derive_job(empty, cd.len, b->jobs_host[j]);
            continue;
        }
        if (ctx->codes_host[in.code_id].len > max_len) max_len = ctx->codes_host[in.code_id].len;
    }
    b->max_code_len = max_len;
    b->replay_lanes = 1;
    for (const auto& dj : b->jobs_host)
        if (dj.rot_avx) b->replay_lanes = kAvxLanes;
    int64_t n_anchors = 0;
    b->n_chunks = plan_chunks(b->jobs_host, b->chunks_host, b->items_host, b->any_multi, &n_anchors, b->classes, chunks_per_item_setting(), true);
    b->n_items = static_cast<int>(b->items_host.size());
    attach_codes(b->chunks_host, b->jobs_host, ctx->codes_host);
    if (b->n_items > b->item_cap) {
        if (b->items_dev) HIP_TRY(ctx, hipFree(b->items_dev));
        b->items_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&b->items_dev, sizeof(WorkItem) * b->n_items));
        b->item_cap = b->n_items;
    }
    if (b->n_items) HIP_TRY(ctx, hipMemcpy(b->items_dev, b->items_host.data(), sizeof(WorkItem) * b->n_items, hipMemcpyHostToDevice));
    if (n_anchors > b->anchor_cap) {
        if (b->anchors_dev) HIP_TRY(ctx, hipFree(b->anchors_dev));
        b->anchors_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&b->anchors_dev, sizeof(Anchor) * (n_anchors + kAnchorPad)));
        HIP_TRY(ctx, hipMemset(b->anchors_dev, 0, sizeof(Anchor) * (n_anchors + kAnchorPad)));
        b->anchor_cap = n_anchors;
    }
    if (b->n_chunks > b->chunk_cap) {
        if (b->chunks_dev) HIP_TRY(ctx, hipFree(b->chunks_dev));
        if (b->partials_dev) HIP_TRY(ctx, hipFree(b->partials_dev));
        b->chunks_dev = nullptr;
        b->partials_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&b->chunks_dev, sizeof(ChunkDesc) * b->n_chunks));
        HIP_TRY(ctx, hipMalloc(&b->partials_dev, sizeof(float) * 2 * kMaxTaps * b->n_chunks));
        b->chunk_cap = b->n_chunks;
    }
    b->n_jobs = n_jobs;
    HIP_TRY(ctx, hd_plan_upload(b->hd, ctx->stream));
    if (static_cast<int>(b->serial.size()) > b->serial_cap) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (b->serial_dev) HIP_TRY(ctx, hipFree(b->serial_dev));
        b->serial_dev = nullptr;
        HIP_TRY(ctx, hipMalloc(&b->serial_dev, sizeof(SerialJob) * b->serial.size()));
        b->serial_cap = static_cast<int>(b->serial.size());
    }
    if (!b->serial.empty())
        HIP_TRY(ctx, hipMemcpyAsync(b->serial_dev, b->serial.data(), sizeof(SerialJob) * b->serial.size(), hipMemcpyHostToDevice, ctx->stream));
    if (n_jobs) {
        HIP_TRY(ctx, hipMemcpyAsync(b->jobs_dev, b->jobs_host.data(), sizeof(DevJob) * n_jobs, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(b->chunks_dev, b->chunks_host.data(), sizeof(ChunkDesc) * b->n_chunks, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    return GNSSHIP_OK;
}

extern "C" int gnsship_batch_launch(gnsship_batch* b, const void* dev_samples, int fmt)
{
    return gnsship_batch_launch_stages(b, dev_samples, fmt, GNSSHIP_STAGE_ANCHORS | GNSSHIP_STAGE_CORRELATE);
}

extern "C" int gnsship_batch_launch_stages(gnsship_batch* b, const void* dev_samples, int fmt, int stages)
{
    if (!b || stages < 1 || stages > 3) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = b->ctx;
    if (fmt_bytes(fmt) == 0) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_launch: unknown sample format");
    if (!dev_samples && b->n_jobs) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_launch: null sample buffer");
    if (b->n_jobs == 0) return GNSSHIP_OK;
    if (ctx->codes_dirty) return fail(ctx, GNSSHIP_E_STATE, "gnsship_batch_launch: code bank changed after set_jobs");
    if (stages & GNSSHIP_STAGE_ANCHORS) {
        // WAR: the previous correlation of this batch must have consumed the anchors
        HIP_TRY(ctx, hipStreamWaitEvent(b->aux, b->corr_done, 0));
        hipError_t e = launch_corr_batch(dev_samples, fmt, b->jobs_dev, b->n_jobs, b->chunks_dev, b->items_dev, b->n_items, b->classes,
            b->max_code_len, b->any_multi, b->anchors_dev, b->partials_dev, b->out_dev, b->aux, GNSSHIP_STAGE_ANCHORS, nullptr, b->replay_lanes);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_batch(anchors)");
        HIP_TRY(ctx, hipEventRecord(b->anchors_ready, b->aux));
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, b->anchors_ready, 0));  // RAW: correlation (or caller) after replay
    }
    if (stages & GNSSHIP_STAGE_CORRELATE) {
        hipError_t e = launch_corr_batch(dev_samples, fmt, b->jobs_dev, b->n_jobs, b->chunks_dev, b->items_dev, b->n_items, b->classes,
            b->max_code_len, b->any_multi, b->anchors_dev, b->partials_dev, b->out_dev, ctx->stream, GNSSHIP_STAGE_CORRELATE);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_batch(correlate)");
        e = launch_corr_hd(dev_samples, fmt, b->hd, b->out_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_hd");
        e = launch_corr_serial(dev_samples, fmt, b->serial_dev, static_cast<int>(b->serial.size()), b->out_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_serial");
        HIP_TRY(ctx, hipEventRecord(b->corr_done, ctx->stream));
    }
    return GNSSHIP_OK;
}

// Correlate `b` and, in the same launch, replay rotator anchors of the batches that follow it
// (leading workgroups of the correlation grid; see corr_batch_kernel): all remaining segments of
// `next`, so that it is complete for the next launch, and the first segment of `next2`.
// Everything on the context stream, so a ring of batches A, B, C, A, ... (or a pair A, B, A, ...
// without next2) needs no cross-stream event: each launch finds its anchors written by earlier
// ones, and same-stream order keeps a replay from overwriting anchors a correlation still reads.
// The replay work is always done for the named batches (a batch named as `next` is replayed even
// when its anchors are still complete).  `b`'s anchors are computed first when no earlier launch
// completed them (first call, or after set_jobs).
extern "C" int gnsship_batch_launch_pipelined2(gnsship_batch* b, const void* dev_samples, int fmt, gnsship_batch* next, gnsship_batch* next2)
{
    if (!b) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = b->ctx;
    if (fmt_bytes(fmt) == 0) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_launch_pipelined: unknown sample format");
    if (next == b || next2 == b || (next2 && next2 == next) || (next && next->ctx != ctx) || (next2 && next2->ctx != ctx))
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_launch_pipelined: next / next2 must be distinct other batches of the same context");
    if (!dev_samples && b->n_jobs) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_batch_launch_pipelined: null sample buffer");
    if (ctx->codes_dirty) return fail(ctx, GNSSHIP_E_STATE, "gnsship_batch_launch_pipelined: code bank changed after set_jobs");
    if (int rc = set_device(ctx)) return rc;
    AnchorPrefetch pf{};
    const bool p1 = next && next->n_jobs > 0, p2 = next2 && next2->n_jobs > 0;
    if (p1)
        pf.task[0] = ReplayTask{next->jobs_dev, next->anchors_dev, next->n_jobs, next->anchor_segs == 1 ? 1 : 0, kAnchorSegments, kAnchorSegments, 0,
            next->replay_lanes};
    if (p2) pf.task[1] = ReplayTask{next2->jobs_dev, next2->anchors_dev, next2->n_jobs, 0, 1, kAnchorSegments, 0, next2->replay_lanes};
    if (b->n_jobs > 0 && b->anchor_segs < kAnchorSegments) {
        hipError_t e = launch_corr_batch(dev_samples, fmt, b->jobs_dev, b->n_jobs, b->chunks_dev, b->items_dev, b->n_items, b->classes,
            b->max_code_len, b->any_multi, b->anchors_dev, b->partials_dev, b->out_dev, ctx->stream, GNSSHIP_STAGE_ANCHORS, nullptr, b->replay_lanes);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_batch(anchors)");
    }
    if (b->n_jobs > 0 || p1 || p2) {
        hipError_t e = launch_corr_batch(dev_samples, fmt, b->jobs_dev, b->n_jobs, b->chunks_dev, b->items_dev, b->n_jobs > 0 ? b->n_items : 0,
            b->classes, b->max_code_len, b->any_multi, b->anchors_dev, b->partials_dev, b->out_dev, ctx->stream, GNSSHIP_STAGE_CORRELATE,
            (p1 || p2) ? &pf : nullptr);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_batch(pipelined)");
    }
    if (b->n_jobs > 0) {
        hipError_t e = launch_corr_hd(dev_samples, fmt, b->hd, b->out_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_hd");
        e = launch_corr_serial(dev_samples, fmt, b->serial_dev, static_cast<int>(b->serial.size()), b->out_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_serial");
    }
    b->anchor_segs = b->n_jobs > 0 ? kAnchorSegments : 0;
    if (p1) next->anchor_segs = kAnchorSegments;
    if (p2) next2->anchor_segs = 1;
    return GNSSHIP_OK;
}

extern "C" int gnsship_batch_launch_pipelined(gnsship_batch* b, const void* dev_samples, int fmt, gnsship_batch* next)
{
    return gnsship_batch_launch_pipelined2(b, dev_samples, fmt, next, nullptr);
}

extern "C" int gnsship_batch_results(gnsship_batch* b, float* out)
{
    if (!b || (!out && b->n_jobs)) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = b->ctx;
    if (b->n_jobs == 0) return GNSSHIP_OK;
    HIP_TRY(ctx, hipMemcpyAsync(out, b->out_dev, sizeof(float) * 2 * kMaxTaps * b->n_jobs, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_batch_results_device(gnsship_batch* b, void** dev_out)
{
    if (!b || !dev_out) return GNSSHIP_E_INVAL;
    *dev_out = b->out_dev;
    return GNSSHIP_OK;
}

extern "C" int gnsship_batch_destroy(gnsship_batch* b)
{
    if (!b) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = b->ctx;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (b->aux) (void)hipStreamSynchronize(b->aux);
    batch_release(b);
    return GNSSHIP_OK;
}

// ============================================================================ per-channel correlator
// Mirror of Cpu_Multicorrelator_Real_Codes: one handle = one channel's correlator bank.
struct gnsship_corr {
    gnsship_ctx* ctx = nullptr;
    int max_samples = 0;
    int n_taps = 0;
    bool high_dyn = false;
    bool code_set = false;
    int code_len = 0;
    float shifts[kMaxTaps] = {};
    float* code_dev = nullptr;
    CodeDesc* code_table_dev = nullptr;
    void* sig_dev = nullptr;  // staging for host input (max_samples CF32)
    DevJob* job_dev = nullptr;
    ChunkDesc* chunks_dev = nullptr;
    WorkItem* items_dev = nullptr;
    float* partials_dev = nullptr;
    float* out_dev = nullptr;
    Anchor* anchors_dev = nullptr;
    int chunk_cap = 0;
    HdPlan hd;  // set_high_dynamics_resampler(true): the high-dynamics kernels
    int rotator = GNSSHIP_ROTATOR_GENERIC;  // gnsship_corr_set_rotator (resolved: GENERIC or AVX)
    SerialJob* serial_dev = nullptr;        // the generic rotator's job (corr_serial.hip)
};

extern "C" int gnsship_corr_create(gnsship_ctx* ctx, int max_signal_length_samples, int n_correlators, gnsship_corr** out)
{
    if (!ctx || !out || max_signal_length_samples < 1 || n_correlators < 1 || n_correlators > kMaxTaps)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_corr_create: bad arguments (1..8 correlators)");
    *out = nullptr;
    if (int rc = set_device(ctx)) return rc;
    gnsship_corr* c = new (std::nothrow) gnsship_corr();
    if (!c) return GNSSHIP_E_NOMEM;
    c->ctx = ctx;
    c->max_samples = max_signal_length_samples;
    c->n_taps = n_correlators;
    c->chunk_cap = (max_signal_length_samples + kCorrChunk - 1) / kCorrChunk;
    hipError_t e = hipMalloc(&c->code_table_dev, sizeof(CodeDesc));
    if (e == hipSuccess) e = hipMalloc(&c->sig_dev, 8 * static_cast<size_t>(max_signal_length_samples));
    if (e == hipSuccess) e = hipMalloc(&c->job_dev, sizeof(DevJob));
    if (e == hipSuccess) e = hipMalloc(&c->chunks_dev, sizeof(ChunkDesc) * c->chunk_cap);
    if (e == hipSuccess) e = hipMalloc(&c->items_dev, sizeof(WorkItem) * c->chunk_cap);
    if (e == hipSuccess) e = hipMalloc(&c->partials_dev, sizeof(float) * 2 * kMaxTaps * c->chunk_cap);
    if (e == hipSuccess) e = hipMalloc(&c->out_dev, sizeof(float) * 2 * kMaxTaps);
    const size_t n_anc = static_cast<size_t>(anchor_entries(max_signal_length_samples, true)) + 1 + kAnchorPad;  // either variant
    if (e == hipSuccess) e = hipMalloc(&c->anchors_dev, sizeof(Anchor) * n_anc);
    if (e == hipSuccess) e = hipMemset(c->anchors_dev, 0, sizeof(Anchor) * n_anc);
    if (e != hipSuccess) {
        gnsship_corr_destroy(c);
        return hip_fail(ctx, e, "gnsship_corr_create");
    }
    *out = c;
    return GNSSHIP_OK;
}

extern "C" int gnsship_corr_set_local_code_and_taps(gnsship_corr* c, int code_length_chips, const float* code, const float* shifts)
{
    if (!c) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = c->ctx;
    if (!code || !shifts || code_length_chips < 1 || code_length_chips > kMaxCodeLen)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_corr_set_local_code_and_taps: bad code / shifts");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (c->code_dev) {
        HIP_TRY(ctx, free_padded_code(c->code_dev));
        c->code_dev = nullptr;
        c->code_set = false;
    }
    HIP_TRY(ctx, upload_padded_code(code, code_length_chips, &c->code_dev));
    c->code_len = code_length_chips;
    CodeDesc d{c->code_dev, code_length_chips, 0};
    HIP_TRY(ctx, hipMemcpy(c->code_table_dev, &d, sizeof(d), hipMemcpyHostToDevice));
    for (int t = 0; t < c->n_taps; t++) c->shifts[t] = shifts[t];
    c->code_set = true;
    return GNSSHIP_OK;
}

extern "C" int gnsship_corr_set_high_dynamics_resampler(gnsship_corr* c, int enable)
{
    if (!c) return GNSSHIP_E_INVAL;
    c->high_dyn = enable != 0;
    return GNSSHIP_OK;
}

extern "C" int gnsship_corr_set_rotator(gnsship_corr* c, int variant)
{
    if (!c) return GNSSHIP_E_INVAL;
    if (variant == GNSSHIP_ROTATOR_AUTO) {
        if (gnsship_rotator_dispatch(&variant) != GNSSHIP_OK)
            return fail(c->ctx, GNSSHIP_E_INVAL, "gnsship_corr_set_rotator: the host's volk_gnsssdr preference names a rotator variant the engine does not reproduce");
    }
    if (variant != GNSSHIP_ROTATOR_GENERIC && variant != GNSSHIP_ROTATOR_AVX) return fail(c->ctx, GNSSHIP_E_INVAL, "gnsship_corr_set_rotator: unknown variant");
    c->rotator = variant;
    return GNSSHIP_OK;
}

extern "C" int gnsship_corr_run(gnsship_corr* c, const void* sig, int fmt, int sig_on_device, float rem_carr, float phase_step,
    float phase_rate_step, float rem_code, float code_step, float code_rate_step, int n, float* corr_out)
{
    if (!c) return GNSSHIP_E_INVAL;
    gnsship_ctx* ctx = c->ctx;
    if (!c->code_set) return fail(ctx, GNSSHIP_E_STATE, "gnsship_corr_run: set_local_code_and_taps not called");
    if (!sig || !corr_out || n < 0 || n > c->max_samples || fmt_bytes(fmt) == 0)
        return fail(ctx, GNSSHIP_E_INVAL, "gnsship_corr_run: bad arguments (length > max_signal_length_samples?)");
    if (int rc = set_device(ctx)) return rc;
    gnsship_corr_job in{};
    in.sample_offset = 0;
    in.n_samples = n;
    in.code_id = 0;
    in.n_taps = c->n_taps;
    in.flags = c->rotator == GNSSHIP_ROTATOR_AVX ? GNSSHIP_JOB_ROTATOR_AVX : 0;
    in.rem_carrier_phase_rad = rem_carr;
    in.phase_step_rad = phase_step;
    in.phase_rate_step_rad = phase_rate_step;
    in.rem_code_phase_chips = rem_code;
    in.code_phase_step_chips = code_step;
    in.code_phase_rate_step_chips = code_rate_step;
    for (int t = 0; t < kMaxTaps; t++) in.shifts_chips[t] = t < c->n_taps ? c->shifts[t] : 0.0f;
    const void* src = sig;
    if (!sig_on_device) {
        HIP_TRY(ctx, hipMemcpyAsync(c->sig_dev, sig, fmt_bytes(fmt) * static_cast<size_t>(n), hipMemcpyHostToDevice, ctx->stream));
        src = c->sig_dev;
    }
    if (c->high_dyn) {  // cpu_multicorrelator_real_codes.cc:80-90,116-119
        c->hd.jobs.resize(1);
        if (!derive_hd_job(in, c->code_dev, c->code_len, 0, c->hd.jobs[0]))
            return fail(ctx, GNSSHIP_E_INVAL, "gnsship_corr_run: invalid high-dynamics job (tap shifts beyond the signal length?)");
        HIP_TRY(ctx, hd_plan_upload(c->hd, ctx->stream));
        hipError_t e = launch_corr_hd(src, fmt, c->hd, c->out_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_hd");
        float tmp[2 * kMaxTaps];
        HIP_TRY(ctx, hipMemcpyAsync(tmp, c->out_dev, sizeof(tmp), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        std::memcpy(corr_out, tmp, sizeof(float) * 2 * c->n_taps);
        return GNSSHIP_OK;
    }
    std::vector<DevJob> jobs(1);
    if (!derive_job(in, c->code_len, jobs[0])) return fail(ctx, GNSSHIP_E_INVAL, "gnsship_corr_run: invalid job");
    if (c->rotator == GNSSHIP_ROTATOR_GENERIC) {  // the generic rotator in the reference's order (corr_serial.hip)
        if (!c->serial_dev) HIP_TRY(ctx, hipMalloc(&c->serial_dev, sizeof(SerialJob)));
        const SerialJob sj{jobs[0], c->code_dev, c->code_len, 0};
        HIP_TRY(ctx, hipMemcpyAsync(c->serial_dev, &sj, sizeof(sj), hipMemcpyHostToDevice, ctx->stream));
        hipError_t e = launch_corr_serial(src, fmt, c->serial_dev, 1, c->out_dev, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_serial");
        float tmp[2 * kMaxTaps];
        HIP_TRY(ctx, hipMemcpyAsync(tmp, c->out_dev, sizeof(tmp), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        std::memcpy(corr_out, tmp, sizeof(float) * 2 * c->n_taps);
        return GNSSHIP_OK;
    }
    std::vector<ChunkDesc> chunks;
    std::vector<WorkItem> items;
    bool multi = false;
    int64_t n_anchors = 0;
    ChunkClass classes[kChunkClasses];
    const int nch = plan_chunks(jobs, chunks, items, multi, &n_anchors, classes, chunks_per_item_setting(), false);
    attach_codes(chunks, jobs, std::vector<CodeDesc>{CodeDesc{c->code_dev, c->code_len, 0}});
    HIP_TRY(ctx, hipMemcpyAsync(c->job_dev, jobs.data(), sizeof(DevJob), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(c->chunks_dev, chunks.data(), sizeof(ChunkDesc) * nch, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(c->items_dev, items.data(), sizeof(WorkItem) * items.size(), hipMemcpyHostToDevice, ctx->stream));
    hipError_t e = launch_corr_batch(src, fmt, c->job_dev, 1, c->chunks_dev, c->items_dev, static_cast<int>(items.size()), classes, c->code_len, multi,
        c->anchors_dev, c->partials_dev, c->out_dev, ctx->stream, GNSSHIP_STAGE_ANCHORS | GNSSHIP_STAGE_CORRELATE, nullptr, kAvxLanes);  // the AVX variant
    if (e != hipSuccess) return hip_fail(ctx, e, "launch_corr_batch");
    float tmp[2 * kMaxTaps];
    HIP_TRY(ctx, hipMemcpyAsync(tmp, c->out_dev, sizeof(tmp), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(corr_out, tmp, sizeof(float) * 2 * c->n_taps);
    return GNSSHIP_OK;
}

extern "C" int gnsship_corr_destroy(gnsship_corr* c)
{
    if (!c) return GNSSHIP_E_INVAL;
    (void)hipSetDevice(c->ctx->device);
    (void)hipStreamSynchronize(c->ctx->stream);
    (void)free_padded_code(c->code_dev);
    hd_plan_free(c->hd);
    void* ptrs[] = {c->code_table_dev, c->sig_dev, c->job_dev, c->chunks_dev, c->items_dev, c->partials_dev, c->out_dev, c->anchors_dev, c->serial_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete c;
    return GNSSHIP_OK;
}
