// corr_serial.hip — the batched correlator's generic-rotator jobs in the reference's serial order.
//
// A generic job (gnsship_corr_job without GNSSHIP_JOB_ROTATOR_AVX / _TREE / _HIGH_DYN) is one call of
// Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler
// (cpu_multicorrelator_real_codes.cc:103-126) with the generic rotator
// (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:66-98).  One 256-thread workgroup per job runs the
// serial pipeline of serial_rotator.h (phasor lane → two producer waves → accumulator wave), so every
// tap equals the reference's bit for bit: the same phasor chain, the same rounded products, one
// serial float sum per tap component.  The code replica is read from its padded HBM copy (the
// producers are off the critical path; the copy stays in L1/L2).
#include "serial_rotator.h"

#pragma clang fp contract(off)

namespace gnsship {
namespace {

constexpr int kSerThreads = 256;

template <int FMT>
__global__ __launch_bounds__(kSerThreads) void corr_serial_kernel(const void* __restrict__ samples, const SerialJob* __restrict__ jobs, int rc,
    float* __restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ SerialSync sy;
    const SerialJob& sj = jobs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid == 0) sy = SerialSync{};
    __syncthreads();
    const DevJob& job = sj.job;
    const int N = job.n_samples, nt = job.n_taps;
    f2* Zr = reinterpret_cast<f2*>(lds);
    float* P = lds + 2 * kSChunk * rc;
    if (wave == 0) {
        if (lane == 0) serial_replay(sy, Zr, rc, N, f2{job.p0_re, job.p0_im}, f2{job.inc_re, job.inc_im});
    } else if (wave < 3) {
        const i4v span = sample_span<FMT>(samples, job.sample_offset, N);
        const float* code[kMaxTaps];
        float shift[kMaxTaps];
#pragma unroll
        for (int t = 0; t < kMaxTaps; t++) {
            code[t] = sj.code;
            shift[t] = job.shifts[t];
        }
        if (job.in_margin)
            serial_produce<FMT, kMaxTaps, true>(sy, Zr, P, rc, span, N, nt, code, shift, sj.code_len, job.code_step, job.rem_code, lane, wave - 1);
        else
            serial_produce<FMT, kMaxTaps, false>(sy, Zr, P, rc, span, N, nt, code, shift, sj.code_len, job.code_step, job.rem_code, lane, wave - 1);
    } else {
        const float acc = serial_accumulate(sy, P, rc, N, nt, lane);
        if (lane < 2 * kMaxTaps) out[static_cast<size_t>(sj.out_index) * 2 * kMaxTaps + lane] = lane < 2 * nt ? acc : 0.0f;
    }
}

}  // namespace

// Ring chunks per workgroup: 8 (4.9 KB per chunk at 8 taps: ≈ 39 KB, four workgroups per CU).
constexpr int kSerRing = 8;

hipError_t launch_corr_serial(const void* samples, int fmt, const SerialJob* jobs, int n_jobs, float* out, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    const size_t lds = serial_ring_bytes(kSerRing, 2 * kMaxTaps);
    dim3 grid(n_jobs), block(kSerThreads);
    switch (fmt) {
    case GNSSHIP_FMT_CF32: hipLaunchKernelGGL(corr_serial_kernel<GNSSHIP_FMT_CF32>, grid, block, lds, stream, samples, jobs, kSerRing, out); break;
    case GNSSHIP_FMT_CI16: hipLaunchKernelGGL(corr_serial_kernel<GNSSHIP_FMT_CI16>, grid, block, lds, stream, samples, jobs, kSerRing, out); break;
    case GNSSHIP_FMT_CI8: hipLaunchKernelGGL(corr_serial_kernel<GNSSHIP_FMT_CI8>, grid, block, lds, stream, samples, jobs, kSerRing, out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gnsship
