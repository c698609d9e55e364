// corr_kernel.hip — batched carrier-wipeoff + code-resampler multicorrelator for gfx950.
//
// Replaces, per (channel, epoch) job, the pair
//   volk_gnsssdr_32f_xn_resampler_32f_xn_generic          (volk_gnsssdr_32f_xn_resampler_32f_xn.h:63-80)
//   volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_generic (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:66-98)
// as driven by Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler
// (cpu_multicorrelator_real_codes.cc:103-126), without materialising the taps×N resampled code
// (the reference writes and re-reads it; here the chip index is computed in registers and the code
// replica is read from LDS).
//
// Two kernels per launch:
//  1. corr_anchor_kernel — one lane per job replays the reference's phasor recursion
//     (phase = phase·phase_inc in float, |phase| renormalised with hypotf every 256 samples) and
//     stores, for every 256-sample block k, the phasor used at sample 256k and its renormalised
//     value.  Only arithmetic on NCO arguments: no IF samples are read.  The recursion is serial
//     by definition; one lane per job keeps every job's chain in flight at once.
//  2. corr_batch_kernel — one 256-thread workgroup (4 wave64) per chunk of ≤4096 samples.  Lane t
//     owns samples {start + t + 256m}, so every wave-load is 64 consecutive samples (coalesced) and
//     lane t is always at offset j = t inside its 256-sample block: the rotation from the block's
//     renormalised anchor to sample j, E_j = |phase_inc|^j·e^{i·j·Δ}, is computed ONCE per lane
//     (double-precision sincos) and reused for all its samples; per sample the phasor is one complex
//     product q_k·E_j.  Per-tap sums live in registers, are reduced with wave64 xor-shuffles and then
//     across the 4 waves in LDS.  Jobs longer than one chunk write per-chunk partials that a third
//     tiny kernel sums in chunk order (deterministic, no atomics).
//
// Numerics (parity contract |Δ|/|ref| ≤ 1e-5 per tap vs the generic reference):
//  * chip index: floor(step·(float)n + shift − rem) with __fmul_rn/__fadd_rn/__fsub_rn in the
//    reference's association order — bit-identical to the generic resampler;
//  * phasor: exact at every renormalisation point (anchor replay); inside a block the only
//    deviation from the reference is its own ≤255-step rounding walk (≈1e-6 rad).
#include "engine.h"

namespace gnsship {

__device__ __forceinline__ float2 cmul_rn(float ar, float ai, float br, float bi)
{
    return make_float2(__fsub_rn(__fmul_rn(ar, br), __fmul_rn(ai, bi)), __fadd_rn(__fmul_rn(ar, bi), __fmul_rn(ai, br)));
}

// std::abs(std::complex<float>) → glibc hypotf, which evaluates sqrt(x²+y²) in double and rounds once.
__device__ __forceinline__ float hypotf_glibc(float x, float y)
{
    const double dx = x, dy = y;
    return static_cast<float>(__dsqrt_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy))));
}

__global__ void corr_anchor_kernel(const DevJob* __restrict__ jobs, int n_jobs, Anchor* __restrict__ anchors)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_jobs) return;
    const DevJob job = jobs[j];
    const int nblk = (job.n_samples + kRenorm - 1) / kRenorm;
    Anchor* out = anchors + job.anchor_offset;
    float pr = job.p0_re, pi = job.p0_im;
    const float ir = job.inc_re, ii = job.inc_im;
    for (int k = 0; k < nblk; k++) {
        // sample 256k uses `a = phase`; then phase /= |phase|; then 256 rotations reach 256(k+1)
        const float m = hypotf_glibc(pr, pi);
        const float qr = __fdiv_rn(pr, m), qi = __fdiv_rn(pi, m);
        out[k] = Anchor{pr, pi, qr, qi};
        pr = qr;
        pi = qi;
        const int steps = (k == nblk - 1) ? 0 : kRenorm;
        for (int s = 0; s < steps; s++) {
            const float2 p = cmul_rn(pr, pi, ir, ii);
            pr = p.x;
            pi = p.y;
        }
    }
}

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
    const Anchor* __restrict__ anchors, const float* __restrict__ lds_code, int L, float* __restrict__ dst)
{
    __shared__ float red[kCorrThreads / 64][2 * kMaxTaps];

    float acc[2 * NT];
#pragma unroll
    for (int v = 0; v < 2 * NT; v++) acc[v] = 0.0f;

    float shifts[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) shifts[t] = (t < job.n_taps) ? job.shifts[t] : 0.0f;

    const int tid = threadIdx.x;  // == offset j inside every 256-sample block this lane visits
    // E_j = |inc|^j · e^{i j Δ}: rotation from the renormalised anchor to sample 256k + j
    float er, ei;
    {
        double s, c;
        sincos(static_cast<double>(tid) * job.dtheta, &s, &c);
        const double mag = 1.0 + static_cast<double>(tid) * static_cast<double>(job.log_mag_inc);
        er = static_cast<float>(mag * c);
        ei = static_cast<float>(mag * s);
    }
    const int64_t base = job.sample_offset;
    const Anchor* anc = anchors + job.anchor_offset + (ch.start >> 8);
#pragma unroll 4
    for (int m = 0; m < kCorrSamplesPerThread; m++) {
        const int r = tid + m * kCorrThreads;
        if (r >= ch.len) break;
        const int n = ch.start + r;  // sample index relative to the job (the reference's loop counter)
        const float2 x = load_sample<FMT>(samples, base + n);
        const Anchor a = anc[m];  // wave-uniform address
        const float2 p = (tid == 0) ? make_float2(a.a_re, a.a_im) : cmul_rn(a.q_re, a.q_im, er, ei);
        const float2 tt = cmul_rn(x.x, x.y, p.x, p.y);  // in_common[n] * phase

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
            acc[2 * t] = __fmaf_rn(tt.x, cv, acc[2 * t]);
            acc[2 * t + 1] = __fmaf_rn(tt.y, cv, acc[2 * t + 1]);
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
    const ChunkDesc* __restrict__ chunks, int n_chunks, const CodeDesc* __restrict__ codes, const Anchor* __restrict__ anchors,
    float* __restrict__ partials, float* __restrict__ out)
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
    case 1: corr_chunk<FMT, 1>(samples, job, ch, anchors, lds_code, L, dst); break;
    case 3: corr_chunk<FMT, 3>(samples, job, ch, anchors, lds_code, L, dst); break;
    case 5: corr_chunk<FMT, 5>(samples, job, ch, anchors, lds_code, L, dst); break;
    default: corr_chunk<FMT, kMaxTaps>(samples, job, ch, anchors, lds_code, L, dst); break;
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
    const CodeDesc* codes, int max_code_len, bool any_multi_chunk, Anchor* anchors, float* partials, float* out, hipStream_t stream,
    int stages)
{
    if (n_chunks <= 0) return hipSuccess;
    if (max_code_len < 1 || max_code_len > kMaxCodeLen) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    if (stages & GNSSHIP_STAGE_ANCHORS) {
        hipLaunchKernelGGL(corr_anchor_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, stream, jobs, n_jobs, anchors);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (!(stages & GNSSHIP_STAGE_CORRELATE)) return hipSuccess;
    const size_t lds = (static_cast<size_t>(max_code_len) * sizeof(float) + 15) & ~static_cast<size_t>(15);
    dim3 grid(n_chunks), block(kCorrThreads);
    switch (fmt) {
    case GNSSHIP_FMT_CF32:
        hipLaunchKernelGGL(corr_batch_kernel<GNSSHIP_FMT_CF32>, grid, block, lds, stream, samples, jobs, chunks, n_chunks, codes, anchors, partials, out);
        break;
    case GNSSHIP_FMT_CI16:
        hipLaunchKernelGGL(corr_batch_kernel<GNSSHIP_FMT_CI16>, grid, block, lds, stream, samples, jobs, chunks, n_chunks, codes, anchors, partials, out);
        break;
    case GNSSHIP_FMT_CI8:
        hipLaunchKernelGGL(corr_batch_kernel<GNSSHIP_FMT_CI8>, grid, block, lds, stream, samples, jobs, chunks, n_chunks, codes, anchors, partials, out);
        break;
    default: return hipErrorInvalidValue;
    }
    e = hipGetLastError();
    if (e != hipSuccess || !any_multi_chunk) return e;
    const int total = n_jobs * 2 * kMaxTaps;
    hipLaunchKernelGGL(corr_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, jobs, n_jobs, partials, out);
    return hipGetLastError();
}

}  // namespace gnsship
