// acq_engine.h — internal types of the PCPS acquisition engine (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "gnsship.h"

namespace gnsship {

constexpr int kAcqThreads = 1024;   // one workgroup per transform: 16 wave64
constexpr int kMaxAcqN = 16384;     // LDS-resident transform: 16384 complex64 = 128 KiB
constexpr int kMaxPasses = 16;
constexpr int kMaxAcqBigN = 32768;  // four-step limit: 32 register points × 1024 LDS rows

struct FftPlan {
    int32_t n;
    int32_t n_passes;
    int32_t radix[kMaxPasses];
};

// Which part of |IFFT|² forms a grid row: [row_off, row_off + row_len) — the second half with
// bit_transition_flag (pcps_acquisition.cc:663-664) — and the modulus of the second-peak exclusion
// window (d_fft_size, :573-580); spc = samples_per_chip.
struct RowSpec {
    int32_t spc, row_off, row_len, win_mod;
};
// make_2_steps step two (pcps_acquisition.cc:305-312, 516-525, 553-556).
struct Step2Spec {
    int32_t active;
    float center, step, input_power;
};

// Per (prn, bin) row statistics of the |IFFT|² grid.
struct RowStat {
    float max;     // first-index maximum value
    int32_t argmax;
    float sum;     // row sum (CFAR input power numerator)
    float second;  // max outside the ±samples_per_chip window around argmax
};

// Factor n into radices {8,5,4,3,2} (largest first); false if n has another prime factor.
bool make_fft_plan(int n, FftPlan& plan);

hipError_t launch_acq_fft_rows(const void* sig, int fmt, const float2* mult, int n_rows, const FftPlan& plan, const float2* tw, float2* rows,
    int conj_out, int n_valid, hipStream_t stream);
hipError_t launch_acq_search(const float2* X, const float2* codes_fft, int n_prns, int n_bins, const FftPlan& plan, const float2* tw,
    RowSpec rs, int accumulate, RowStat* rowstat, float* grid, hipStream_t stream);
// Large transforms (N > kMaxAcqN): N = P·M, P ∈ {16,18,20,24,25,27,30,32} in registers, M ≤ 1024 in LDS.
bool big_p_supported(int P);
hipError_t launch_acq_fft_big(const void* sig, int fmt, const float2* mult, int n_rows, int P, const FftPlan& row_plan, const float2* tw,
    float2* rowsT, int conj_out, int n_valid, hipStream_t stream);
hipError_t launch_acq_search_big(const float2* XT, const float2* codesT, int n_prns, int n_bins, int P, const FftPlan& row_plan,
    const float2* tw, RowSpec rs, int accumulate, RowStat* rowstat, float* grid, hipStream_t stream);
// Huge transforms (N > kMaxAcqBigN): N = P·M, P ∈ {4,5,8,10,16,20,25,32} register points per
// column, M ≤ kMaxAcqN LDS rows, column and row stages as separate kernels through HBM.
constexpr int kMaxAcqHugeN = 32 * kMaxAcqN;
struct TileStat {  // one column tile of one |IFFT|² row
    float max;
    int32_t argmax;
    float sum;
    int32_t pad;
};
bool huge_p_supported(int P);
bool huge_ct_rows(int M);
hipError_t ensure_lane_perm10();  // the 10000-point rows' butterfly table on the current device (outside any capture)  // M-point rows with a compile-time plan and the pipelined search rows
constexpr int huge_tiles(int M) { return (M + 255) / 256; }
// rowsT[b] = transposed FFT(sig ⊙ mult[b]) for b < n_rows; scratch: n_rows × N complex.
hipError_t launch_acq_fft_huge(const void* sig, int fmt, const float2* mult, int n_rows, int P, const FftPlan& row_plan, const float2* twN,
    const float2* twM, float2* scratch, float2* rowsT, int conj_out, int n_valid, hipStream_t stream);
// PRN slots [prn_offset, prn_offset + n_prns): U scratch n_prns × n_bins × N complex, grid rows
// (n_prns × n_bins × N floats, relative to prn_offset), tiles n_prns × n_bins × huge_tiles(M).
hipError_t launch_acq_search_huge(const float2* XT, const float2* codesT, int prn_offset, int n_prns, int n_bins, int P, const FftPlan& row_plan,
    const float2* twN, const float2* twM, float2* U, float* grid, int accumulate, TileStat* tiles, RowSpec rs, RowStat* rowstat,
    hipStream_t stream);
hipError_t launch_acq_decide(const RowStat* rowstat, int n_prns, int n_bins, int N, int doppler_max, int doppler_step, int doppler_center,
    int dwells, int use_cfar, float samples_per_code, float resampler_ratio, uint32_t resampler_latency, Step2Spec step2, gnsship_acq_result* out,
    hipStream_t stream);

}  // namespace gnsship
