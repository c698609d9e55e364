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
constexpr int kCorrSamplesPerThread = 16;  // 4096-sample chunk = 64 lanes × 64 samples (one wave per chunk)
constexpr int kCorrChunk = kCorrThreads * kCorrSamplesPerThread;  // 4096 samples per workgroup
constexpr int kCorrWavesPerSimd = 4;     // ≥4 resident workgroups per CU (≤128 VGPRs)
constexpr int kMaxCodeLen = 16384;       // LDS budget for the local code replica (64 KiB + margins)

// A local code replica resident in HBM.
struct CodeDesc {
    const float* ptr;
    int32_t len;
    int32_t binary;  // every chip is exactly +1 or -1 (gnsship_code_set)
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
    float dz_re, dz_im;     // rot_avx: dz = normalise(phase_inc^16) exactly as the AVX recursion forms it
    float log_mag_inc;      // log|phase_inc| (magnitude growth between renormalisations)
    float rem_code;         // rem_code_phase_chips  (float, as passed by the reference)
    float code_step;        // code_phase_step_chips
    int32_t in_margin;      // 1: every chip index of the job lies in [−kCodeMargin, L + kCodeMargin)
    int32_t rot_avx;        // 1: anchors from the AVX rotator recursion (GNSSHIP_JOB_ROTATOR_AVX), 0: generic
    float shifts[kMaxTaps];
};

// The LDS copy of a code replica is padded with kCodeMargin wrapped chips on both sides, so chip
// indices a few chips outside [0, L) — the usual case at epoch edges with early/late taps — need
// no modulo.  Jobs that can leave the margin (checked on the host) take the general wrap path.
constexpr int kCodeMargin = 32;
// Device code replicas are stored pre-wrapped in HBM, [code[L−M..L−1] | code[0..L−1] | code[0..M−1]]
// (M = kCodeMargin) rounded up to whole 16-byte quads; the pointer handed around (CodeDesc::ptr,
// ChunkDesc::code) is chip 0.  The correlator copies the padded span into LDS with aligned 16-byte
// loads and no index arithmetic.
constexpr int padded_code_quads(int len) { return (len + 2 * kCodeMargin + 3) / 4; }
hipError_t upload_padded_code(const float* code, int len, float** chip0);  // allocates; *chip0 = chip 0
hipError_t free_padded_code(const float* chip0);

// AVX-variant jobs (rot_avx) keep their own anchor layout in the same buffer, in f2 (8-byte) units
// from anchor_offset·4: Z[16t + l] = the phasor AVX lane l uses at iteration 16t (before its update;
// task t = iterations [16t, 16t + 16) ∩ [0, N/16)), for every task, then the ≤ 15 phasors of the
// serial N mod 16 tail at Z[16·T + j] (T tasks).  Every phasor is then continued bit-exactly by the
// correlating lanes (corr_kernel.hip), so nothing is approximated.
constexpr int kAvxLanes = 16;       // phasors of the u_avx rotator (…rotator_dot_prod_32fc_xn.h:199-213)
constexpr int kAvxTaskIters = 16;   // iterations per anchored task
__host__ __device__ constexpr int avx_tasks_of(int n_samples) { return (n_samples / kAvxLanes + kAvxTaskIters - 1) / kAvxTaskIters; }
// Anchor entries (32 B each) of a job's layout: generic ceil(n/256), AVX 4·(tasks + 1).
__host__ __device__ constexpr int anchor_entries(int n_samples, bool avx)
{
    return avx ? 4 * (avx_tasks_of(n_samples) + 1) : (n_samples + 255) / 256;
}

// Rotator anchor of one 256-sample block k of a job: the phasors the reference rotates samples
// 256k + s by, s = 0..3 — p[0..1] = the renormalised q = a/|a| (the reference multiplies sample 256k
// by a = |a|·q; see corr_kernel.hip), p[2s..2s+1] = q·inc^s in the reference's float recursion.
// A lane covering samples 256k + 4t + s rotates them by p_s · E_{4t}.
struct Anchor {
    float p[8];
};
// Anchor buffers carry kAnchorPad entries past the last job: a wave reads the anchor of the block
// after its current one unconditionally (scalar prefetch).
constexpr int kBlocksPerChunk = kCorrChunk / 256;  // renormalisation blocks per chunk (16)
constexpr int kAnchorPad = kBlocksPerChunk;

struct ChunkDesc {
    int32_t job;
    int32_t start;     // first sample (relative to the job)
    int32_t len;
    int32_t code_len;  // the job's code replica, carried here so that a workgroup fetches it
    const float* code; // without waiting for the job descriptor (attach_codes)
};

// A workgroup's work: chunks [first, first + count) of the (reordered) chunk array, all sharing
// one code replica (corr_batch_kernel stages it in LDS once per item).
constexpr int kMaxChunksPerItem = 4;
constexpr int kChunksPerItemDefault = 4;
struct WorkItem {
    int32_t first;
    int32_t count;
};

// Launch the batched correlator: partials[chunk][2*kMaxTaps] then per-job reduction into out.
// Chunks are grouped by class = 8·avx + 2·tap_class + in_margin, tap_class: 0 → 1 tap, 1 → ≤3, 2 → ≤5,
// 3 → ≤8; each class is one kernel launch over work items [start, start + count).
constexpr int kChunkClasses = 16;
struct ChunkClass {
    int32_t start;
    int32_t count;
};
inline int chunk_class(int n_taps, int in_margin, int avx)
{
    const int tc = n_taps <= 1 ? 0 : n_taps <= 3 ? 1 : n_taps <= 5 ? 2 : 3;
    return 8 * (avx ? 1 : 0) + 2 * tc + (in_margin ? 1 : 0);
}

// Anchor replay of another job set carried by a correlation launch (leading workgroups).
// Anchor replay carried by the leading workgroups of a correlation launch (see corr_batch_kernel).
// A job's replay chain is split at its middle renormalisation block into kAnchorSegments
// segments; segment s > 0 resumes from the anchor segment s − 1 stored (gnsship_batch_launch_pipelined2
// spreads one batch's replay over two consecutive launches).
constexpr int kAnchorSegments = 2;     // the pair / three-batch ring (gnsship_batch_launch_pipelined2)
constexpr int kAnchorRingMax = 4;      // gnsship_batch_launch_ring: up to 4 following batches, 4 segments
struct ReplayTask {
    const DevJob* jobs;
    Anchor* anchors;
    int32_t n_jobs;
    int32_t seg_lo, seg_hi;  // segments [seg_lo, seg_hi) of n_segs equal block ranges
    int32_t n_segs;
    int32_t n_blocks;        // workgroups (set by launch_corr_batch)
    int32_t lanes;           // threads per job: 1, or kAvxLanes when any job uses the AVX variant
};
struct AnchorPrefetch {
    ReplayTask task[kAnchorRingMax];
    int32_t n_blocks;        // all leading workgroups, a multiple of 8 (set by launch_corr_batch)
};

// Fill ChunkDesc::code / code_len from a code table indexed by the chunks' jobs' code ids.
void attach_codes(std::vector<ChunkDesc>& chunks, const std::vector<struct DevJob>& jobs, const std::vector<CodeDesc>& table);

// anchors: scratch of Σ ceil(n_j/256) Anchor entries, recomputed by every launch.  prefetch
// (optional, with the CORRELATE stage): replay `prefetch->jobs`' anchors in the same launch.
// replay_lanes: threads per job of the anchor stage (1, or kAvxLanes when any job is rot_avx).
hipError_t launch_corr_batch(const void* samples, int fmt, const DevJob* jobs, int n_jobs, const ChunkDesc* chunks, const WorkItem* items,
    int n_items, const ChunkClass* classes, int max_code_len, bool any_multi_chunk, Anchor* anchors, float* partials, float* out,
    hipStream_t stream, int stages = GNSSHIP_STAGE_ANCHORS | GNSSHIP_STAGE_CORRELATE, const AnchorPrefetch* prefetch = nullptr,
    int replay_lanes = 1);

// Plan chunks (≤ kCorrChunk samples), rotator anchors and work items for a job list: chunks of one
// job stay contiguous and in order; single-chunk jobs with equal code id (pair_by_code) share items
// of up to chunks_per_item chunks in job order.  Returns the chunk count.
int plan_chunks(std::vector<DevJob>& jobs, std::vector<ChunkDesc>& chunks, std::vector<WorkItem>& items, bool& any_multi, int64_t* n_anchors,
    ChunkClass* classes, int chunks_per_item, bool pair_by_code);

// ---- Generic-rotator jobs in the reference's serial order (corr_serial.hip) ---------------------
// One workgroup per job: the job's own DevJob (its slot in the chunk plan is an empty job), its
// padded code replica (chip 0) and the output row.
struct SerialJob {
    DevJob job;
    const float* code;
    int32_t code_len;
    int32_t out_index;
};
hipError_t launch_corr_serial(const void* samples, int fmt, const SerialJob* jobs, int n_jobs, float* out, hipStream_t stream);

// ---- High-dynamics correlator (Dll_Pll_Conf::high_dyn; corr_hd_kernel.hip) -------------------
// Replaces volk_gnsssdr_32f_xn_high_dynamics_resampler_32f_xn_generic + volk_gnsssdr_32fc_32f_
// high_dynamic_rotator_dot_prod_32fc_xn_generic, the pair Cpu_Multicorrelator_Real_Codes runs when
// set_high_dynamics_resampler(true) (cpu_multicorrelator_real_codes.cc:75-100,116-119).
struct HdJob {
    int64_t sample_offset;
    int32_t n_samples;
    int32_t n_taps;
    int32_t out_index;      // row of the output array
    int32_t anchor_offset;  // ceil(n/256) Doppler-chain anchors
    int32_t first_chunk, n_chunks;
    float p0_re, p0_im;     // phase_offset_as_complex: the unnormalised start of the Doppler chain
    float inc_re, inc_im;   // phase_inc
    double dtheta;          // arg(phase_inc) in double
    float log_mag_inc;      // log|phase_inc|
    float rate_arg;         // Im clogf(phase_inc_rate) = atan2f(im, re): glibc cpowf's angle per n²
    float rem_code, code_step, code_rate, shift0;
    uint32_t shift_samples[kMaxTaps];  // tap t = tap 0 circularly shifted by this many samples
    const float* code;
    int32_t code_len;
    int32_t pad;
};
struct HdAnchor {  // the Doppler chain at sample 256k (unnormalised)
    float q_re, q_im;
};
struct HdChunk {
    int32_t job, start, len, pad;
};
// Host-side plan of the high-dynamics jobs of a batch (or of one gnsship_corr_run).
struct HdPlan {
    std::vector<HdJob> jobs;
    std::vector<HdChunk> chunks;
    int64_t n_anchors = 0;
    int max_code_len = 1;
    HdJob* jobs_dev = nullptr;
    HdChunk* chunks_dev = nullptr;
    HdAnchor* anchors_dev = nullptr;
    float* partials_dev = nullptr;
    int job_cap = 0, chunk_cap = 0;
    int64_t anchor_cap = 0;
};
// Derive one HdJob from a reference-style call; false when the arguments are outside what the
// reference itself can run (taps, shifts that would make its memcpy lengths negative).
bool derive_hd_job(const gnsship_corr_job& in, const float* code_dev, int code_len, int out_index, HdJob& out);
// Chunks + anchor layout for plan.jobs; (re)allocates and uploads the device copies.
hipError_t hd_plan_upload(HdPlan& plan, hipStream_t stream);
void hd_plan_free(HdPlan& plan);
// Doppler-chain anchors, per-chunk correlation, per-job reduction into out[out_index].
hipError_t launch_corr_hd(const void* samples, int fmt, const HdPlan& plan, float* out, hipStream_t stream);

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
    uint64_t codes_version = 0;  // bumped by every gnsship_code_set (holders of code pointers re-attach)
};
