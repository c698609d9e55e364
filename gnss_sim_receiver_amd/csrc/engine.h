// engine.h — internal (non-ABI) types shared by the HIP kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "gnsship.h"

namespace gnsship {

constexpr int kMaxTaps = GNSSHIP_MAX_TAPS;
constexpr int kCorrThreads = 256;        // one workgroup = 4 wave64
constexpr int kCorrSamplesPerThread = 16;
constexpr int kCorrChunk = kCorrThreads * kCorrSamplesPerThread;  // 4096 samples per workgroup
constexpr int kCorrWavesPerSimd = 4;     // ≥4 resident workgroups per CU (≤128 VGPRs)
constexpr int kMaxCodeLen = 16384;       // LDS budget for the local code replica (64 KiB + margins)

// A local code replica resident in HBM.
struct CodeDesc {
    const float* ptr;
    int32_t len;
    int32_t pad;
};

constexpr int kRenorm = 256;             // the generic rotator renormalises |phase| every 256 samples

// Device-side job, derived on the host from gnsship_corr_job.  The two phasors the reference
// forms per call are evaluated on the host with the reference's own float operations
// (cpu_multicorrelator_real_codes.cc:115,123: (cos rem, −sin rem) and std::exp(complex<float>(0,−step))
// = glibc cexpf → (cosf(−step), sinf(−step))); the device then reproduces the rotator recursion.
struct DevJob {
    int64_t sample_offset;
    int32_t n_samples;
    int32_t code_id;
    int32_t n_taps;
    int32_t n_chunks;       // workgroups covering this job
    int32_t first_chunk;    // index of its first chunk (partials row)
    int32_t anchor_offset;  // first of ceil(n/256) anchors of this job
    float p0_re, p0_im;     // phase_offset_as_complex
    float inc_re, inc_im;   // phase_inc
    double dtheta;          // arg(phase_inc) in double (exact angle of the float phasor)
    float log_mag_inc;      // log|phase_inc| (magnitude growth between renormalisations)
    float rem_code;         // rem_code_phase_chips  (float, as passed by the reference)
    float code_step;        // code_phase_step_chips
    int32_t in_margin;      // 1: every chip index of the job lies in [−kCodeMargin, L + kCodeMargin)
    float shifts[kMaxTaps];
};

// The LDS copy of a code replica is padded with kCodeMargin wrapped chips on both sides, so chip
// indices a few chips outside [0, L) — the usual case at epoch edges with early/late taps — need
// no modulo.  Jobs that can leave the margin (checked on the host) take the general wrap path.
constexpr int kCodeMargin = 32;

// Rotator anchor of one 256-sample block k of a job: `a` = the phasor the reference multiplies
// sample 256k by (before renormalising), `q` = a/|a| (the renormalised phasor it then rotates).
struct Anchor {
    float a_re, a_im, q_re, q_im;
};

struct ChunkDesc {
    int32_t job;
    int32_t start;  // first sample (relative to the job)
    int32_t len;
    int32_t pad;
};

// Launch the batched correlator: partials[chunk][2*kMaxTaps] then per-job reduction into out.
// Chunks are grouped by class = 2·tap_class + in_margin, tap_class: 0 → 1 tap, 1 → ≤3, 2 → ≤5, 3 → ≤8;
// each class is one kernel launch over chunks[start, start + count).
constexpr int kChunkClasses = 8;
struct ChunkClass {
    int32_t start;
    int32_t count;
};
inline int chunk_class(int n_taps, int in_margin)
{
    const int tc = n_taps <= 1 ? 0 : n_taps <= 3 ? 1 : n_taps <= 5 ? 2 : 3;
    return 2 * tc + (in_margin ? 1 : 0);
}

// Anchor replay of another job set carried by a correlation launch (leading workgroups).
struct AnchorPrefetch {
    const DevJob* jobs;
    int32_t n_jobs;
    Anchor* anchors;
    int32_t n_blocks;  // set by launch_corr_batch
};

// anchors: scratch of Σ ceil(n_j/256) Anchor entries, recomputed by every launch.  prefetch
// (optional, with the CORRELATE stage): replay `prefetch->jobs`' anchors in the same launch.
hipError_t launch_corr_batch(const void* samples, int fmt, const DevJob* jobs, int n_jobs, const ChunkDesc* chunks, int n_chunks,
    const ChunkClass* classes, const CodeDesc* codes, int max_code_len, bool any_multi_chunk, Anchor* anchors, float* partials, float* out,
    hipStream_t stream, int stages = GNSSHIP_STAGE_ANCHORS | GNSSHIP_STAGE_CORRELATE, const AnchorPrefetch* prefetch = nullptr);

}  // namespace gnsship

struct gnsship_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t events[16] = {};
    std::string last_error;
    // code bank
    std::vector<gnsship::CodeDesc> codes_host;  // ptr = device pointer
    gnsship::CodeDesc* codes_dev = nullptr;
    int codes_dev_cap = 0;
    bool codes_dirty = false;
};
