// corr_kernel.hip — batched carrier-wipeoff + code-resampler multicorrelator for gfx950.
//
// Replaces, per (channel, epoch) job, the pair
//   volk_gnsssdr_32f_xn_resampler_32f_xn_generic       (volk_gnsssdr_32f_xn_resampler_32f_xn.h:63-80)
//   volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_generic (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:66-98)
// as driven by Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler
// (cpu_multicorrelator_real_codes.cc:103-126), without materialising the taps×N resampled code
// (the reference writes and re-reads it; here the chip index is computed in registers and the code
// replica is read from LDS).
//
// Work decomposition: one 256-thread workgroup (4 wave64) per chunk of ≤4096 samples of one job.
// Each lane owns samples {start + tid + 256k}: every load instruction of a wave is 64 consecutive
// samples (512 B for CF32), coalesced.  Per-tap complex sums live in registers, are reduced with
// wave64 xor-shuffles, then across the 4 waves in LDS.  Jobs longer than one chunk write per-chunk
// partials that a second tiny kernel sums in chunk order (deterministic, no atomics).
//
// Numerics (parity contract: |Δ|/|ref| ≤ 1e-5 per tap vs the generic reference):
//  * chip index: floor(step·(float)n + shift − rem) evaluated with __fmul_rn/__fadd_rn/__fsub_rn in
//    the reference's association order — bit-identical to the generic resampler;
//  * carrier phasor: the reference rotates a float phasor recursively (phase *= phase_inc,
//    renormalised every 256 samples).  Its angle is exactly θ0 + n·Δ up to rounding noise, where
//    Δ = arg(float phase_inc) and θ0 = arg(float phase_offset); its magnitude grows as |phase_inc|^m
//    between renormalisations (m = ((n−1) mod 256)+1).  Both systematic terms are evaluated here
//    directly per sample (θ in double, range-reduced, accurate sincosf), which removes the
//    recursion's serial dependency while tracking the reference's deterministic drift.
#include "engine.h"

namespace gnsship {

template <int FMT>
__device__ __forceinline__ float2 load_sample(const void* __restrict__ base, int64_t i)
{
    if constexpr (FMT == GNSSHIP_FMT_CF32) {
        return reinterpret_cast<const float2*>(base)[i];
    } else if constexpr (FMT == GNSSHIP_FMT_CI16) {
        const short2 s = reinterpret_cast<const short2*>(base)[i];
        return make_float2(static_cast<float>(s.x), static_cast<float>(s.y));
    } else {
        const char2 s = reinterpret_cast<const char2*>(base)[i];
        return make_float2(static_cast<float>(s.x), static_cast<float>(s.y));
    }
}

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int FMT, int NT>
__device__ __forceinline__ void corr_chunk(const void* __restrict__ samples, const DevJob& job, const ChunkDesc& ch,
    const float* __restrict__ lds_code, int L, float* __restrict__ dst)
{
    __shared__ float red[kCorrThreads / 64][2 * kMaxTaps];
    constexpr double kTwoPi = 6.283185307179586476925286766559;
    constexpr double kInvTwoPi = 0.15915494309189533576888376337251;

    float acc[2 * NT];
#pragma unroll
    for (int v = 0; v < 2 * NT; v++) acc[v] = 0.0f;

    float shifts[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) shifts[t] = (t < job.n_taps) ? job.shifts[t] : 0.0f;

    const int tid = threadIdx.x;
    const int64_t base = job.sample_offset;
#pragma unroll 4
    for (int k = 0; k < kCorrSamplesPerThread; k++) {
        const int r = tid + k * kCorrThreads;
        if (r >= ch.len) break;
        const int n = ch.start + r;  // sample index relative to the job (the reference's loop counter)
        const float2 x = load_sample<FMT>(samples, base + n);

        // carrier phasor model (see header)
        double th = fma(static_cast<double>(n), job.dtheta, job.theta0);
        th = fma(-kTwoPi, rint(th * kInvTwoPi), th);
        float s, c;
        sincosf(static_cast<float>(th), &s, &c);
        const int m = (n == 0) ? 0 : (((n - 1) & 255) + 1);
        const float mag = (n == 0) ? job.mag0 : __fmaf_rn(static_cast<float>(m), job.log_mag_inc, 1.0f);
        const float pr = mag * c, pi = mag * s;
        const float tr = __fsub_rn(__fmul_rn(x.x, pr), __fmul_rn(x.y, pi));
        const float ti = __fadd_rn(__fmul_rn(x.x, pi), __fmul_rn(x.y, pr));

        // code resampler, generic association order: ((step*n) + shift) - rem
        const float sn = __fmul_rn(job.code_step, static_cast<float>(n));
#pragma unroll
        for (int t = 0; t < NT; t++) {
            int idx = static_cast<int>(floorf(__fsub_rn(__fadd_rn(sn, shifts[t]), job.rem_code)));
            if (static_cast<unsigned>(idx) >= static_cast<unsigned>(L)) {
                idx %= L;
                if (idx < 0) idx += L;
            }
            const float cv = lds_code[idx];
            acc[2 * t] = __fmaf_rn(tr, cv, acc[2 * t]);
            acc[2 * t + 1] = __fmaf_rn(ti, cv, acc[2 * t + 1]);
        }
    }

    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int v = 0; v < 2 * NT; v++) {
        const float w = wave_sum(acc[v]);
        if (lane == 0) red[wave][v] = w;
    }
    __syncthreads();
    if (tid < 2 * kMaxTaps) {
        float s = 0.0f;
        if (tid < 2 * NT && tid < 2 * job.n_taps) {
#pragma unroll
            for (int w = 0; w < kCorrThreads / 64; w++) s += red[w][tid];
        }
        dst[tid] = s;
    }
}

template <int FMT>
__global__ __launch_bounds__(kCorrThreads) void corr_batch_kernel(const void* __restrict__ samples, const DevJob* __restrict__ jobs,
    const ChunkDesc* __restrict__ chunks, int n_chunks, const CodeDesc* __restrict__ codes, float* __restrict__ partials,
    float* __restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) float lds_code[];
    const int ci = blockIdx.x;
    if (ci >= n_chunks) return;
    const ChunkDesc ch = chunks[ci];
    const DevJob job = jobs[ch.job];
    const CodeDesc cd = codes[job.code_id];
    const int L = cd.len;
    for (int i = threadIdx.x; i < L; i += kCorrThreads) lds_code[i] = cd.ptr[i];
    __syncthreads();
    float* dst = (job.n_chunks == 1) ? out + static_cast<int64_t>(ch.job) * 2 * kMaxTaps
                                     : partials + static_cast<int64_t>(ci) * 2 * kMaxTaps;
    switch (job.n_taps) {
    case 1: corr_chunk<FMT, 1>(samples, job, ch, lds_code, L, dst); break;
    case 3: corr_chunk<FMT, 3>(samples, job, ch, lds_code, L, dst); break;
    case 5: corr_chunk<FMT, 5>(samples, job, ch, lds_code, L, dst); break;
    default: corr_chunk<FMT, kMaxTaps>(samples, job, ch, lds_code, L, dst); break;
    }
}

// Sum the chunk partials of multi-chunk jobs, in chunk order.
__global__ void corr_reduce_kernel(const DevJob* __restrict__ jobs, int n_jobs, const float* __restrict__ partials, float* __restrict__ out)
{
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = gid / (2 * kMaxTaps), v = gid % (2 * kMaxTaps);
    if (j >= n_jobs) return;
    const DevJob& job = jobs[j];
    if (job.n_chunks == 1) return;
    float s = 0.0f;
    for (int c = 0; c < job.n_chunks; c++) s += partials[static_cast<int64_t>(job.first_chunk + c) * 2 * kMaxTaps + v];
    out[static_cast<int64_t>(j) * 2 * kMaxTaps + v] = s;
}

hipError_t launch_corr_batch(const void* samples, int fmt, const DevJob* jobs, int n_jobs, const ChunkDesc* chunks, int n_chunks,
    const CodeDesc* codes, int max_code_len, bool any_multi_chunk, float* partials, float* out, hipStream_t stream)
{
    if (n_chunks <= 0) return hipSuccess;
    if (max_code_len < 1 || max_code_len > kMaxCodeLen) return hipErrorInvalidValue;
    const size_t lds = (static_cast<size_t>(max_code_len) * sizeof(float) + 15) & ~static_cast<size_t>(15);
    dim3 grid(n_chunks), block(kCorrThreads);
    switch (fmt) {
    case GNSSHIP_FMT_CF32:
        hipLaunchKernelGGL(corr_batch_kernel<GNSSHIP_FMT_CF32>, grid, block, lds, stream, samples, jobs, chunks, n_chunks, codes, partials, out);
        break;
    case GNSSHIP_FMT_CI16:
        hipLaunchKernelGGL(corr_batch_kernel<GNSSHIP_FMT_CI16>, grid, block, lds, stream, samples, jobs, chunks, n_chunks, codes, partials, out);
        break;
    case GNSSHIP_FMT_CI8:
        hipLaunchKernelGGL(corr_batch_kernel<GNSSHIP_FMT_CI8>, grid, block, lds, stream, samples, jobs, chunks, n_chunks, codes, partials, out);
        break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !any_multi_chunk) return e;
    const int total = n_jobs * 2 * kMaxTaps;
    hipLaunchKernelGGL(corr_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, jobs, n_jobs, partials, out);
    return hipGetLastError();
}

}  // namespace gnsship
