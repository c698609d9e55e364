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

// Every product/sum on the parity path is rounded on its own, like the reference's generic C;
// the few fused multiply-adds wanted are written explicitly (__fmaf_rn).
#pragma clang fp contract(off)

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

// The reference rotator recursion of one job, stored at every renormalisation point.
__device__ __forceinline__ void replay_anchors(const DevJob& job, Anchor* __restrict__ anchors)
{
    const int nblk = (job.n_samples + kRenorm - 1) / kRenorm;
    Anchor* out = anchors + job.anchor_offset;
    typedef float f2v __attribute__((ext_vector_type(2)));
    float pr = job.p0_re, pi = job.p0_im;
    // phase·inc = (pr·ir − pi·ii, pr·ii + pi·ir) as two packed products + one packed add, each
    // rounded separately like the reference's written-out complex product (no FMA).  The sign
    // sits in the constant: fl(pi·(−ii)) = −fl(pi·ii) and x + (−y) ≡ x − y, bit for bit.
    const f2v inc_a = {job.inc_re, job.inc_im};   // × pr
    const f2v inc_b = {-job.inc_im, job.inc_re};  // × pi
    for (int k = 0; k < nblk; k++) {
        // sample 256k uses `a = phase`; then phase /= |phase|; then 256 rotations reach 256(k+1)
        const float m = hypotf_glibc(pr, pi);
        const float qr = __fdiv_rn(pr, m), qi = __fdiv_rn(pi, m);
        out[k] = Anchor{pr, pi, qr, qi};
        f2v p = {qr, qi};
        if (k != nblk - 1) {
#pragma unroll 16
            for (int s = 0; s < kRenorm; s++) {
                const f2v m1 = f2v{p.x, p.x} * inc_a;
                const f2v m2 = f2v{p.y, p.y} * inc_b;
                p = m1 + m2;
            }
        }
        pr = p.x;
        pi = p.y;
    }
}

__global__ void corr_anchor_kernel(const DevJob* __restrict__ jobs, int n_jobs, Anchor* __restrict__ anchors)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_jobs) return;
    const DevJob job = jobs[j];
    replay_anchors(job, anchors);
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

typedef float f2 __attribute__((ext_vector_type(2)));

// (a·b) for phasor products off the parity-critical path (contraction allowed: one packed
// multiply + one packed FMA).  bsw = (−b.im, b.re).
__device__ __forceinline__ f2 cmul_pk(f2 a, f2 b, f2 bsw)
{
    return __builtin_elementwise_fma(f2{a.y, a.y}, bsw, f2{a.x, a.x} * b);
}

// (int)floor(x) in one instruction (V_CVT_FLR_I32_F32), as the resampler's (int)floor(...) for
// in-range values.
__device__ __forceinline__ int cvt_floor_i32(float x)
{
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// Positive modulo of the reference's wrap (volk_gnsssdr_32f_xn_resampler_32f_xn.h:75-77).
__device__ __forceinline__ int wrap_index(int idx, int L)
{
    idx = idx < 0 ? idx + L : idx;
    idx = idx >= L ? idx - L : idx;
    if (static_cast<unsigned>(idx) >= static_cast<unsigned>(L)) {  // more than one period away
        idx %= L;
        if (idx < 0) idx += L;
    }
    return idx;
}

// One chunk of one job.  `code` points at chip 0 of the padded LDS replica (valid indices
// [−kCodeMargin, L + kCodeMargin)).  IN_MARGIN: the host proved every index of the job lies in the
// padded range, so the chip index is used directly (no modulo).
template <int FMT, int NT, bool IN_MARGIN>
__device__ __forceinline__ void corr_chunk(const void* __restrict__ samples, const DevJob& job, const ChunkDesc& ch,
    const Anchor* __restrict__ anchors, const float* __restrict__ code, int L, float* __restrict__ dst)
{
    __shared__ float red[kCorrThreads / 64][2 * kMaxTaps];
    if (ch.len <= 0) {  // zero-length job (workgroup-uniform): nothing to read, outputs are zero
        if (threadIdx.x < 2 * kMaxTaps) dst[threadIdx.x] = 0.0f;
        return;
    }

    f2 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = f2{0.0f, 0.0f};
    float shifts[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) shifts[t] = (t < job.n_taps) ? job.shifts[t] : 0.0f;

    const int tid = threadIdx.x;  // == offset j inside every 256-sample block this lane visits
    const int64_t base = job.sample_offset + ch.start;
    // E_j = |inc|^j · e^{i j Δ}: rotation from the renormalised anchor to sample 256k + j
    // (angle formed and range-reduced in double, then an accurate float sincos)
    f2 e, esw;
    {
        constexpr double kTwoPi = 6.283185307179586476925286766559;
        constexpr double kInvTwoPi = 0.15915494309189533576888376337251;
        double th = static_cast<double>(tid) * job.dtheta;
        th = fma(-kTwoPi, rint(th * kInvTwoPi), th);
        float s, c;
        sincosf(static_cast<float>(th), &s, &c);
        const float mag = __fmaf_rn(static_cast<float>(tid), job.log_mag_inc, 1.0f);
        e = f2{mag * c, mag * s};
        esw = f2{-e.y, e.x};
    }
    const Anchor* anc = anchors + job.anchor_offset + (ch.start >> 8);
    const int last_blk = (ch.len - 1) >> 8;  // last 256-sample block of the chunk (chunk-uniform)
    const bool lane_j0 = (tid == 0);

    // Software pipeline over groups of kGroup samples per lane, ping-pong register buffers: the
    // loads of group g+1 are in flight while group g is correlated.  Whole groups inside the chunk
    // run without any tail test; in the (at most one) partial group, lanes past the chunk end read
    // the chunk's last sample and contribute zero.
    constexpr int kGroup = 4;
    constexpr int kGroups = kCorrSamplesPerThread / kGroup;
    constexpr int kGroupSpan = kGroup * kCorrThreads;
    static_assert(kGroups % 2 == 0, "ping-pong over pairs of groups");
    auto load_group = [&](int g, f2 (&dstx)[kGroup]) {
        if ((g + 1) * kGroupSpan <= ch.len) {
#pragma unroll
            for (int u = 0; u < kGroup; u++) {
                const float2 v = load_sample<FMT>(samples, base + tid + (g * kGroup + u) * kCorrThreads);
                dstx[u] = f2{v.x, v.y};
            }
        } else {
#pragma unroll
            for (int u = 0; u < kGroup; u++) {
                const int r = tid + (g * kGroup + u) * kCorrThreads;
                const float2 v = load_sample<FMT>(samples, base + (r < ch.len ? r : ch.len - 1));
                dstx[u] = (r < ch.len) ? f2{v.x, v.y} : f2{0.0f, 0.0f};
            }
        }
    };
    auto correlate_group = [&](int g, const f2 (&xg)[kGroup]) {
        // anchors of this group's 256-sample blocks: chunk-uniform addresses → scalar loads
        Anchor ag[kGroup];
#pragma unroll
        for (int u = 0; u < kGroup; u++) {
            const int m = g * kGroup + u;
            ag[u] = anc[m < last_blk ? m : last_blk];
        }
        const bool full = (g + 1) * kGroupSpan <= ch.len;  // group-uniform
#pragma unroll
        for (int u = 0; u < kGroup; u++) {
            const int r = tid + (g * kGroup + u) * kCorrThreads;
            const int n = ch.start + (full ? r : (r < ch.len ? r : ch.len - 1));  // reference loop counter
            // phasor at sample n: the anchor itself at j = 0, else q_k · E_j (select, no branch)
            const f2 pq = cmul_pk(f2{ag[u].q_re, ag[u].q_im}, e, esw);
            const f2 p = lane_j0 ? f2{ag[u].a_re, ag[u].a_im} : pq;
            const f2 tt = cmul_pk(xg[u], p, f2{-p.y, p.x});  // in_common[n] * phase
            // code resampler, generic association order: ((step*n) + shift) - rem, each rounded
            // on its own (the file is built with -ffp-contract=off)
            const float sn = job.code_step * static_cast<float>(n);
#pragma unroll
            for (int t = 0; t < NT; t++) {
                int idx = cvt_floor_i32((sn + shifts[t]) - job.rem_code);
                if constexpr (!IN_MARGIN) idx = wrap_index(idx, L);
                const float cv = code[idx];
                acc[t] = __builtin_elementwise_fma(tt, f2{cv, cv}, acc[t]);
            }
        }
    };
    f2 xa[kGroup], xb[kGroup];
    load_group(0, xa);
#pragma unroll
    for (int g = 0; g < kGroups; g += 2) {
        if (g * kGroupSpan >= ch.len) break;  // chunk-uniform
        if ((g + 1) * kGroupSpan < ch.len) load_group(g + 1, xb);
        correlate_group(g, xa);
        if ((g + 1) * kGroupSpan >= ch.len) break;
        if (g + 2 < kGroups && (g + 2) * kGroupSpan < ch.len) load_group(g + 2, xa);
        correlate_group(g + 1, xb);
    }

    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const float wr = wave_sum(acc[t].x), wi = wave_sum(acc[t].y);
        if (lane == 0) {
            red[wave][2 * t] = wr;
            red[wave][2 * t + 1] = wi;
        }
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

// One launch per chunk class (tap-count template × in-margin flag), so each kernel is compiled
// for exactly its path and the register allocation is not the worst case over all variants.
template <int FMT, int NT, bool IN_MARGIN>
__global__ __launch_bounds__(kCorrThreads, kCorrWavesPerSimd) void corr_batch_kernel(const void* __restrict__ samples, const DevJob* __restrict__ jobs,
    const ChunkDesc* __restrict__ chunks, int n_chunks, int chunk_base, const CodeDesc* __restrict__ codes,
    const Anchor* __restrict__ anchors, float* __restrict__ partials, float* __restrict__ out, AnchorPrefetch pf)
{
    extern __shared__ __attribute__((aligned(16))) float lds_code[];
    // Leading workgroups replay the rotator anchors of ANOTHER batch (the next one of a
    // double-buffered pair): one lane per job, latency-bound chains that run beside the
    // correlation instead of in a separate stream behind a cross-queue event.
    if (static_cast<int>(blockIdx.x) < pf.n_blocks) {
        const int j = blockIdx.x * kCorrThreads + threadIdx.x;
        if (j < pf.n_jobs) {
            const DevJob pj = pf.jobs[j];
            replay_anchors(pj, pf.anchors);
        }
        return;
    }
    // XCD-aware chunk order: workgroups are dealt round-robin over the 8 XCDs (b and b+8 share
    // one), so give each XCD a CONTIGUOUS range of chunks.  Jobs arrive epoch-major, so the
    // channels that read the same IF samples then share one XCD's L2 (bijective for any grid).
    // pf.n_blocks is a multiple of 8, so b keeps the hardware's b mod 8 placement.
    const int nb = static_cast<int>(gridDim.x) - pf.n_blocks;
    const int b = blockIdx.x - pf.n_blocks;
    const int q = nb >> 3, rmd = nb & 7, x = b & 7;
    const int ci = x * q + (x < rmd ? x : rmd) + (b >> 3);
    if (ci >= n_chunks) return;
    const ChunkDesc ch = chunks[ci];
    const DevJob job = jobs[ch.job];
    float* dst = (job.n_chunks == 1) ? out + static_cast<int64_t>(ch.job) * 2 * kMaxTaps
                                     : partials + static_cast<int64_t>(chunk_base + ci) * 2 * kMaxTaps;
    // Idle chunk (tracking channels without a window this round, zero-length jobs): touch neither
    // the code bank (the job's code slot may be empty) nor the samples.  Workgroup-uniform.
    if (ch.len <= 0) {
        if (threadIdx.x < 2 * kMaxTaps) dst[threadIdx.x] = 0.0f;
        return;
    }
    const CodeDesc cd = codes[job.code_id];
    const int L = cd.len;
    if (L <= 0 || cd.ptr == nullptr) {
        if (threadIdx.x < 2 * kMaxTaps) dst[threadIdx.x] = 0.0f;
        return;
    }
    // padded replica in LDS: lds[kCodeMargin + i] = code[i mod L] for i in [−kCodeMargin, L + kCodeMargin)
    const int total = L + 2 * kCodeMargin;
    for (int i = threadIdx.x; i < total; i += kCorrThreads) {
        int src = i - kCodeMargin;
        src = src < 0 ? src + L * ((-src + L - 1) / L) : src;
        src = src % L;
        lds_code[i] = cd.ptr[src];
    }
    __syncthreads();
    const float* code = lds_code + kCodeMargin;
    corr_chunk<FMT, NT, IN_MARGIN>(samples, job, ch, anchors, code, L, dst);
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
    const ChunkClass* classes, const CodeDesc* codes, int max_code_len, bool any_multi_chunk, Anchor* anchors, float* partials, float* out,
    hipStream_t stream, int stages, const AnchorPrefetch* prefetch)
{
    AnchorPrefetch pf{nullptr, 0, nullptr, 0};
    if (prefetch && prefetch->n_jobs > 0 && (stages & GNSSHIP_STAGE_CORRELATE)) {
        pf = *prefetch;
        pf.n_blocks = ((pf.n_jobs + kCorrThreads - 1) / kCorrThreads + 7) & ~7;
    }
    if (n_chunks <= 0) {
        if (pf.n_jobs > 0) {
            hipLaunchKernelGGL(corr_anchor_kernel, dim3((pf.n_jobs + 63) / 64), dim3(64), 0, stream, pf.jobs, pf.n_jobs, pf.anchors);
            return hipGetLastError();
        }
        return hipSuccess;
    }
    if (max_code_len < 1 || max_code_len > kMaxCodeLen) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    if (stages & GNSSHIP_STAGE_ANCHORS) {
        hipLaunchKernelGGL(corr_anchor_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, stream, jobs, n_jobs, anchors);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (!(stages & GNSSHIP_STAGE_CORRELATE)) return hipSuccess;
    const size_t lds = (static_cast<size_t>(max_code_len + 2 * kCodeMargin) * sizeof(float) + 15) & ~static_cast<size_t>(15);
    for (int c = 0; c < kChunkClasses; c++) {
        const int cnt = classes[c].count;
        if (cnt <= 0) continue;
        const ChunkDesc* cc = chunks + classes[c].start;
        const int cb = classes[c].start;
        dim3 grid(cnt + pf.n_blocks), block(kCorrThreads);
#define GNSSHIP_LAUNCH_CORR(F, NTV, MV) \
    hipLaunchKernelGGL((corr_batch_kernel<F, NTV, MV>), grid, block, lds, stream, samples, jobs, cc, cnt, cb, codes, anchors, partials, out, pf)
#define GNSSHIP_LAUNCH_NT(F)                                                     \
    switch (c) {                                                                 \
    case 0: GNSSHIP_LAUNCH_CORR(F, 1, false); break;                             \
    case 1: GNSSHIP_LAUNCH_CORR(F, 1, true); break;                              \
    case 2: GNSSHIP_LAUNCH_CORR(F, 3, false); break;                             \
    case 3: GNSSHIP_LAUNCH_CORR(F, 3, true); break;                              \
    case 4: GNSSHIP_LAUNCH_CORR(F, 5, false); break;                             \
    case 5: GNSSHIP_LAUNCH_CORR(F, 5, true); break;                              \
    case 6: GNSSHIP_LAUNCH_CORR(F, kMaxTaps, false); break;                      \
    default: GNSSHIP_LAUNCH_CORR(F, kMaxTaps, true); break;                      \
    }
        switch (fmt) {
        case GNSSHIP_FMT_CF32: GNSSHIP_LAUNCH_NT(GNSSHIP_FMT_CF32); break;
        case GNSSHIP_FMT_CI16: GNSSHIP_LAUNCH_NT(GNSSHIP_FMT_CI16); break;
        case GNSSHIP_FMT_CI8: GNSSHIP_LAUNCH_NT(GNSSHIP_FMT_CI8); break;
        default: return hipErrorInvalidValue;
        }
#undef GNSSHIP_LAUNCH_NT
#undef GNSSHIP_LAUNCH_CORR
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        pf = AnchorPrefetch{nullptr, 0, nullptr, 0};  // only the first class launch carries the prefetch
    }
    e = hipGetLastError();
    if (e != hipSuccess || !any_multi_chunk) return e;
    const int total = n_jobs * 2 * kMaxTaps;
    hipLaunchKernelGGL(corr_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, jobs, n_jobs, partials, out);
    return hipGetLastError();
}

}  // namespace gnsship
