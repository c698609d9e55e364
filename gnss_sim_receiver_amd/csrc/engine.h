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
constexpr int kMaxCodeLen = 16384;       // LDS budget for the local code replica (64 KiB)

// A local code replica resident in HBM.
struct CodeDesc {
    const float* ptr;
    int32_t len;
    int32_t pad;
};

// Device-side job, derived on the host from gnsship_corr_job: every float argument that the
// reference turns into a phasor is pre-evaluated ONCE per job on the host with the reference's
// own float operations (cosf/sinf of float, as std::cos / std::exp(complex<float>) do in
// cpu_multicorrelator_real_codes.cc:115,123), then its exact angle / magnitude taken in double.
struct DevJob {
    int64_t sample_offset;
    int32_t n_samples;
    int32_t code_id;
    int32_t n_taps;
    int32_t n_chunks;       // workgroups covering this job
    int32_t first_chunk;    // index of its first chunk (partials row)
    int32_t pad0;
    double theta0;          // arg(phase_offset_as_complex)
    double dtheta;          // arg(phase_inc) = arg(exp(-j*phase_step_rad)) in float, exactly
    float mag0;             // |phase_offset_as_complex|
    float log_mag_inc;      // log|phase_inc| (per-sample magnitude growth between renormalisations)
    float rem_code;         // rem_code_phase_chips  (float, as passed by the reference)
    float code_step;        // code_phase_step_chips
    float shifts[kMaxTaps];
};

struct ChunkDesc {
    int32_t job;
    int32_t start;  // first sample (relative to the job)
    int32_t len;
    int32_t pad;
};

// Launch the batched correlator: partials[chunk][2*kMaxTaps] then per-job reduction into out.
hipError_t launch_corr_batch(const void* samples, int fmt, const DevJob* jobs, int n_jobs, const ChunkDesc* chunks, int n_chunks,
    const CodeDesc* codes, int max_code_len, bool any_multi_chunk, float* partials, float* out, hipStream_t stream);

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
