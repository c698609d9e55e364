// corr_hd_kernel.hip — the high-dynamics multicorrelator (Dll_Pll_Conf::high_dyn) for gfx950.
//
// Replaces, per job, the pair Cpu_Multicorrelator_Real_Codes runs after
// set_high_dynamics_resampler(true) (cpu_multicorrelator_real_codes.cc:75-100, 116-119):
//   volk_gnsssdr_32f_xn_high_dynamics_resampler_32f_xn_generic
//       (volk_gnsssdr_32f_xn_high_dynamics_resampler_32f_xn.h:67-91)
//   volk_gnsssdr_32fc_32f_high_dynamic_rotator_dot_prod_32fc_xn_generic
//       (volk_gnsssdr_32fc_32f_high_dynamic_rotator_dot_prod_32fc_xn.h:68-110; only generic
//        variants exist, so this is always what the reference dispatches).
//
// Reference semantics restated (n = 0 .. N−1, N = signal_length_samples):
//  * tap 0 chip index  floor(((step·(float)n + rate·(float)(n·n)) + shift0) − rem), n·n in
//    32-bit unsigned (wraps for n ≥ 65536), negative indices wrapped to [0, L);
//  * tap t ≥ 1 is tap 0 circularly shifted by S_t = Σ_{u≤t} (int)round((shift_u − shift_{u−1})/step)
//    samples over the N-sample buffer: code_t[n] = code_0[(n + S_t) mod N];
//  * Doppler chain pd_0 = phase_offset (NOT normalised), pd_{n+1} = pd_n·phase_inc in float;
//  * phasor of sample 0: phase_offset/|phase_offset|; of sample n ≥ 1: pd_n·r_{n−1} with
//    r_k = cpowf(phase_inc_rate, (float)(k·k)) / |·|, renormalised when n % 256 == 0;
//  * result_t = Σ (x[n]·phasor_n)·code_t[n].
// Device form: the Doppler chain is replayed exactly (float products, one lane per job) and
// stored every 256 samples (hd_anchor_kernel); a workgroup of 256 lanes covers a 4096-sample
// chunk, lane t at offset j = t of every 256-sample block, pd_{256k+j} = D_k·E_j with
// E_j = |inc|^j e^{ijΔ} (as corr_kernel.hip).  glibc cpowf(z, v) = cexpf(v·clogf(z)): its angle
// is fl(v · atan2f(z)) — formed bit-exactly here — and its magnitude e^{v·log|z|} is divided out
// by the reference's own normalisation, so r_k = (cos θ_k, sin θ_k) with an accurate sincosf.
// (Where e^{v·log|z|} overflows float — |v·log|z|| ≳ 88, i.e. only for N ≳ 5·10⁴ — the
// reference's r_k is inf/NaN and its correlation NaN; the device keeps the normalised phasor.)
#include <algorithm>
#include <cmath>

#include "engine.h"
#include "nco_math.h"

#pragma clang fp contract(off)

namespace gnsship {

namespace {

constexpr int kHdThreads = 256;
constexpr int kHdChunk = 4096;
constexpr int kHdPerThread = kHdChunk / kHdThreads;

template <int FMT>
__device__ __forceinline__ float2 load_if(const void* samples, int64_t i)
{
    if constexpr (FMT == GNSSHIP_FMT_CF32) {
        return reinterpret_cast<const float2*>(samples)[i];
    } else if constexpr (FMT == GNSSHIP_FMT_CI16) {
        const short2 v = reinterpret_cast<const short2*>(samples)[i];
        return make_float2(static_cast<float>(v.x), static_cast<float>(v.y));
    } else {
        const char2 v = reinterpret_cast<const char2*>(samples)[i];
        return make_float2(static_cast<float>(v.x), static_cast<float>(v.y));
    }
}

// Positive modulo of the reference's wrap (…_high_dynamics_resampler_32f_xn.h:77-79).
__device__ __forceinline__ int wrap_chip(int idx, int L)
{
    int r = idx % L;
    return r < 0 ? r + L : r;
}

// Tap-0 chip index at buffer position m, in the reference's association order.
__device__ __forceinline__ int hd_chip_index(const HdJob& job, uint32_t m)
{
    const float fm = __uint2float_rn(m);
    const float fmm = __uint2float_rn(m * m);  // unsigned int product, wraps like the reference
    const float v = __fsub_rn(__fadd_rn(__fadd_rn(__fmul_rn(job.code_step, fm), __fmul_rn(job.code_rate, fmm)), job.shift0), job.rem_code);
    return wrap_chip(static_cast<int>(floorf(v)), job.code_len);
}

}  // namespace

__global__ void hd_anchor_kernel(const HdJob* __restrict__ jobs, int n_jobs, HdAnchor* __restrict__ anchors)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_jobs) return;
    const HdJob job = jobs[j];
    const int nblk = (job.n_samples + kRenorm - 1) / kRenorm;
    HdAnchor* out = anchors + job.anchor_offset;
    float pr = job.p0_re, pi = job.p0_im;
    for (int k = 0; k < nblk; k++) {
        out[k] = HdAnchor{pr, pi};
        if (k == nblk - 1) break;
        for (int s = 0; s < kRenorm; s++) {
            const float2 p = cmul_rn(pr, pi, job.inc_re, job.inc_im);
            pr = p.x;
            pi = p.y;
        }
    }
}

template <int FMT>
__global__ __launch_bounds__(kHdThreads) void hd_corr_kernel(const void* __restrict__ samples, const HdJob* __restrict__ jobs,
    const HdChunk* __restrict__ chunks, const HdAnchor* __restrict__ anchors, float* __restrict__ partials)
{
    extern __shared__ float code_lds[];
    __shared__ float red[kHdThreads / 64][2 * kMaxTaps];
    const HdChunk ch = chunks[blockIdx.x];
    const HdJob job = jobs[ch.job];
    const int tid = threadIdx.x;
    for (int i = tid; i < job.code_len; i += kHdThreads) code_lds[i] = job.code[i];
    // E_j for j = tid (chunk starts are multiples of 256)
    constexpr double kTwoPi = 6.283185307179586476925286766559;
    double th = static_cast<double>(tid) * job.dtheta;
    th = fma(-kTwoPi, rint(th / kTwoPi), th);
    float es, ec;
    sincosf(static_cast<float>(th), &es, &ec);
    const float emag = expf(static_cast<float>(tid) * job.log_mag_inc);
    const float er = emag * ec, ei = emag * es;
    __syncthreads();
    float acc[2 * kMaxTaps];
#pragma unroll
    for (int v = 0; v < 2 * kMaxTaps; v++) acc[v] = 0.0f;
    const uint32_t N = static_cast<uint32_t>(job.n_samples);
    for (int u = 0; u < kHdPerThread; u++) {
        const int r = tid + u * kHdThreads;
        if (r >= ch.len) break;
        const uint32_t n = static_cast<uint32_t>(ch.start + r);
        const float2 x = load_if<FMT>(samples, job.sample_offset + n);
        float pr, pi;
        if (n == 0) {
            const float m = hypotf_glibc(job.p0_re, job.p0_im);
            pr = __fdiv_rn(job.p0_re, m);
            pi = __fdiv_rn(job.p0_im, m);
        } else {
            const HdAnchor a = anchors[job.anchor_offset + (n >> 8)];
            const float dr = a.q_re * er - a.q_im * ei, di = a.q_re * ei + a.q_im * er;  // pd_n
            const uint32_t k = n - 1u;
            const float theta = __fmul_rn(__uint2float_rn(k * k), job.rate_arg);
            float rs, rc;
            sincosf(theta, &rs, &rc);
            const float2 p = cmul_rn(dr, di, rc, rs);
            pr = p.x;
            pi = p.y;
            if ((n & (kRenorm - 1)) == 0) {
                const float m = hypotf_glibc(pr, pi);
                pr = __fdiv_rn(pr, m);
                pi = __fdiv_rn(pi, m);
            }
        }
        const float2 t = cmul_rn(x.x, x.y, pr, pi);
#pragma unroll
        for (int tap = 0; tap < kMaxTaps; tap++) {
            if (tap < job.n_taps) {
                uint32_t m = n + job.shift_samples[tap];
                if (m >= N) m -= N;
                const float c = code_lds[hd_chip_index(job, m)];
                acc[2 * tap] = __fadd_rn(acc[2 * tap], __fmul_rn(t.x, c));
                acc[2 * tap + 1] = __fadd_rn(acc[2 * tap + 1], __fmul_rn(t.y, c));
            }
        }
    }
    // wave64 butterfly, then the four waves in LDS (fixed order: deterministic)
#pragma unroll
    for (int v = 0; v < 2 * kMaxTaps; v++) {
        float s = acc[v];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((tid & 63) == 0) red[tid >> 6][v] = s;
    }
    __syncthreads();
    if (tid < 2 * kMaxTaps) {
        float s = 0.0f;
        for (int w = 0; w < kHdThreads / 64; w++) s += red[w][tid];
        partials[static_cast<int64_t>(blockIdx.x) * 2 * kMaxTaps + tid] = (tid < 2 * job.n_taps) ? s : 0.0f;
    }
}

__global__ void hd_reduce_kernel(const HdJob* __restrict__ jobs, int n_jobs, const float* __restrict__ partials, float* __restrict__ out)
{
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = gid / (2 * kMaxTaps), v = gid % (2 * kMaxTaps);
    if (j >= n_jobs) return;
    const HdJob& job = jobs[j];
    float s = 0.0f;
    for (int c = 0; c < job.n_chunks; c++) s += partials[static_cast<int64_t>(job.first_chunk + c) * 2 * kMaxTaps + v];
    out[static_cast<int64_t>(job.out_index) * 2 * kMaxTaps + v] = s;
}

hipError_t launch_corr_hd(const void* samples, int fmt, const HdPlan& plan, float* out, hipStream_t stream)
{
    const int n_jobs = static_cast<int>(plan.jobs.size());
    const int n_chunks = static_cast<int>(plan.chunks.size());
    if (n_jobs == 0) return hipSuccess;
    if (plan.max_code_len < 1 || plan.max_code_len > kMaxCodeLen) return hipErrorInvalidValue;
    hipLaunchKernelGGL(hd_anchor_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, stream, plan.jobs_dev, n_jobs, plan.anchors_dev);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n_chunks > 0) {
        const size_t lds = sizeof(float) * static_cast<size_t>(plan.max_code_len);
        switch (fmt) {
        case GNSSHIP_FMT_CF32:
            hipLaunchKernelGGL(hd_corr_kernel<GNSSHIP_FMT_CF32>, dim3(n_chunks), dim3(kHdThreads), lds, stream, samples, plan.jobs_dev, plan.chunks_dev,
                plan.anchors_dev, plan.partials_dev);
            break;
        case GNSSHIP_FMT_CI16:
            hipLaunchKernelGGL(hd_corr_kernel<GNSSHIP_FMT_CI16>, dim3(n_chunks), dim3(kHdThreads), lds, stream, samples, plan.jobs_dev, plan.chunks_dev,
                plan.anchors_dev, plan.partials_dev);
            break;
        case GNSSHIP_FMT_CI8:
            hipLaunchKernelGGL(hd_corr_kernel<GNSSHIP_FMT_CI8>, dim3(n_chunks), dim3(kHdThreads), lds, stream, samples, plan.jobs_dev, plan.chunks_dev,
                plan.anchors_dev, plan.partials_dev);
            break;
        default: return hipErrorInvalidValue;
        }
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const int total = n_jobs * 2 * kMaxTaps;
    hipLaunchKernelGGL(hd_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, plan.jobs_dev, n_jobs, plan.partials_dev, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------- host-side planning
bool derive_hd_job(const gnsship_corr_job& in, const float* code_dev, int code_len, int out_index, HdJob& out)
{
    if (in.n_samples < 0 || in.n_taps < 1 || in.n_taps > kMaxTaps || in.sample_offset < 0 || code_len < 1 || !code_dev) return false;
    out = HdJob{};
    out.sample_offset = in.sample_offset;
    out.n_samples = in.n_samples;
    out.n_taps = in.n_taps;
    out.out_index = out_index;
    // the reference's float phasors (cpu_multicorrelator_real_codes.cc:115-117): glibc cosf/sinf/cexpf
    out.p0_re = std::cos(in.rem_carrier_phase_rad);
    out.p0_im = -std::sin(in.rem_carrier_phase_rad);
    out.inc_re = std::cos(-in.phase_step_rad);
    out.inc_im = std::sin(-in.phase_step_rad);
    out.dtheta = std::atan2(static_cast<double>(out.inc_im), static_cast<double>(out.inc_re));
    out.log_mag_inc = static_cast<float>(std::log(std::hypot(static_cast<double>(out.inc_re), static_cast<double>(out.inc_im))));
    const float rr = std::cos(-in.phase_rate_step_rad), ri = std::sin(-in.phase_rate_step_rad);
    out.rate_arg = std::atan2(ri, rr);  // glibc clogf imaginary part = atan2f(im, re)
    out.rem_code = in.rem_code_phase_chips;
    out.code_step = in.code_phase_step_chips;
    out.code_rate = in.code_phase_rate_step_chips;
    out.shift0 = in.shifts_chips[0];
    out.code = code_dev;
    out.code_len = code_len;
    // cumulative circular shifts (…_high_dynamics_resampler_32f_xn.h:83-90): unsigned int sum of
    // (int)round(float quotient); outside [0, N] the reference's memcpy lengths go negative
    uint32_t s = 0;
    out.shift_samples[0] = 0;
    for (int t = 1; t < in.n_taps; t++) {
        const float q = (in.shifts_chips[t] - in.shifts_chips[t - 1]) / in.code_phase_step_chips;
        const double rq = std::round(static_cast<double>(q));
        if (!std::isfinite(rq)) return false;
        s += static_cast<uint32_t>(static_cast<int>(rq));
        if (s > static_cast<uint32_t>(in.n_samples)) return false;
        out.shift_samples[t] = s;
    }
    return true;
}

void hd_plan_free(HdPlan& plan)
{
    void* ptrs[] = {plan.jobs_dev, plan.chunks_dev, plan.anchors_dev, plan.partials_dev};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    plan.jobs_dev = nullptr;
    plan.chunks_dev = nullptr;
    plan.anchors_dev = nullptr;
    plan.partials_dev = nullptr;
    plan.job_cap = plan.chunk_cap = 0;
    plan.anchor_cap = 0;
}

hipError_t hd_plan_upload(HdPlan& plan, hipStream_t stream)
{
    plan.chunks.clear();
    int64_t anchors = 0;
    int max_len = 1;
    for (size_t j = 0; j < plan.jobs.size(); j++) {
        HdJob& job = plan.jobs[j];
        job.anchor_offset = static_cast<int32_t>(anchors);
        anchors += (job.n_samples + kRenorm - 1) / kRenorm;
        job.first_chunk = static_cast<int32_t>(plan.chunks.size());
        job.n_chunks = (job.n_samples + kHdChunk - 1) / kHdChunk;
        for (int k = 0; k < job.n_chunks; k++) {
            const int start = k * kHdChunk;
            plan.chunks.push_back(HdChunk{static_cast<int32_t>(j), start, std::min(kHdChunk, job.n_samples - start), 0});
        }
        max_len = std::max(max_len, job.code_len);
    }
    plan.n_anchors = anchors > 0 ? anchors : 1;
    plan.max_code_len = max_len;
    const int nj = static_cast<int>(plan.jobs.size()), nc = static_cast<int>(plan.chunks.size());
    hipError_t e = hipSuccess;
    if (nj > plan.job_cap) {
        if (plan.jobs_dev) (void)hipFree(plan.jobs_dev);
        plan.jobs_dev = nullptr;
        if ((e = hipMalloc(&plan.jobs_dev, sizeof(HdJob) * nj)) != hipSuccess) return e;
        plan.job_cap = nj;
    }
    if (nc > plan.chunk_cap) {
        if (plan.chunks_dev) (void)hipFree(plan.chunks_dev);
        if (plan.partials_dev) (void)hipFree(plan.partials_dev);
        plan.chunks_dev = nullptr;
        plan.partials_dev = nullptr;
        if ((e = hipMalloc(&plan.chunks_dev, sizeof(HdChunk) * nc)) != hipSuccess) return e;
        if ((e = hipMalloc(&plan.partials_dev, sizeof(float) * 2 * kMaxTaps * nc)) != hipSuccess) return e;
        plan.chunk_cap = nc;
    }
    if (plan.n_anchors > plan.anchor_cap) {
        if (plan.anchors_dev) (void)hipFree(plan.anchors_dev);
        plan.anchors_dev = nullptr;
        if ((e = hipMalloc(&plan.anchors_dev, sizeof(HdAnchor) * plan.n_anchors)) != hipSuccess) return e;
        plan.anchor_cap = plan.n_anchors;
    }
    if (nj && (e = hipMemcpyAsync(plan.jobs_dev, plan.jobs.data(), sizeof(HdJob) * nj, hipMemcpyHostToDevice, stream)) != hipSuccess) return e;
    if (nc && (e = hipMemcpyAsync(plan.chunks_dev, plan.chunks.data(), sizeof(HdChunk) * nc, hipMemcpyHostToDevice, stream)) != hipSuccess) return e;
    return hipStreamSynchronize(stream);
}

}  // namespace gnsship
