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
//  2. corr_batch_kernel — one 256-thread workgroup (4 wave64) per work item of up to four
//     ≤4096-sample chunks sharing one code replica (staged once in LDS); wave w correlates chunk w.
//     Lane t owns samples {256k + 4t + s : s < 4} of every 256-sample block k, so a wave-load is
//     2 KiB of consecutive samples and lane t always sits at offsets 4t..4t+3 of its blocks: the
//     block's four phasors q_k·inc^s are uniform (scalar loads of the anchor), the lane factor
//     E_{4t} = |phase_inc|^{4t}·e^{i·4t·Δ} is applied once per chunk to the tap sums.  Per sample:
//     chip indices + LDS code reads, one complex product with a scalar operand, one packed FMA per
//     tap.  Sums are reduced within the wave (DPP + lane shuffles).  Jobs longer than one chunk
//     write per-chunk partials that a third tiny kernel sums in chunk order (no atomics).
//
// Numerics (parity contract |Δ|/|ref| ≤ 1e-5 per tap vs the generic reference):
//  * chip index: floor(step·(float)n + shift − rem) with __fmul_rn/__fadd_rn/__fsub_rn in the
//    reference's association order — bit-identical to the generic resampler;
//  * phasor: exact at every renormalisation point (anchor replay); inside a block the only
//    deviation from the reference is its own ≤255-step rounding walk (≈1e-6 rad).
#include "anchor_replay.h"
#include "corr_device.h"
#include "engine.h"
#include "nco_math.h"

// Every product/sum on the parity path is rounded on its own, like the reference's generic C;
// the few fused multiply-adds wanted are written explicitly (__fmaf_rn).
#pragma clang fp contract(off)

namespace gnsship {

// Workgroup phase timestamps for the profiling build only (make prof → libgnsship_prof.so,
// scripts/corr_wg_profile.py): slot [8·blockIdx + k] = wall_clock64() at phase k, thread 0.
#ifdef GNSSHIP_CORR_PROFILE
__device__ unsigned long long* g_corr_prof = nullptr;
#define GNSSHIP_PROF_STAMP(k)                                                                                                        \
    do {                                                                                                                             \
        if (threadIdx.x == 0 && g_corr_prof) g_corr_prof[static_cast<size_t>(blockIdx.x) * 8 + (k)] = wall_clock64();               \
    } while (0)
#else
#define GNSSHIP_PROF_STAMP(k) \
    do {                      \
    } while (0)
#endif

// lanes: threads per job (1, or kAvxLanes when the job set has AVX-variant jobs).
__global__ void corr_anchor_kernel(const DevJob* __restrict__ jobs, int n_jobs, Anchor* __restrict__ anchors, int seg_lo, int seg_hi, int n_segs,
    int lanes)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = lanes == 1 ? g : g / kAvxLanes, l = lanes == 1 ? 0 : g % kAvxLanes;
    if (j >= n_jobs) return;
    const DevJob job = jobs[j];
    replay_anchors(job, anchors, seg_lo, seg_hi, n_segs, l);
}

// Waves per SIMD the register allocation must allow: the 1- and 3-tap in-margin classes (GPS/B1I
// E-P-L, E1 data prompt) are held to 8 waves (≤ 64 VGPRs; measured +2% over 7); wider tap classes keep the
// general bound.
#ifndef GNSSHIP_CORR_WAVES_EPL
#define GNSSHIP_CORR_WAVES_EPL 8
#endif
template <int NT, bool IN_MARGIN, bool AVX>
constexpr int corr_waves_per_simd()
{
    return (NT <= 3 && IN_MARGIN && !AVX) ? GNSSHIP_CORR_WAVES_EPL : kCorrWavesPerSimd;
}

// AVX-variant chunk (engine.h AVX layout): the chunk's iterations [m0, m0 + 256) ∩ [0, M) are tasks of
// 16; a wave takes groups of four tasks, lane = 16·(task in group) + phasor lane l, and continues
// lane l's phasor from the task's anchor through the task's iterations with the reference's own
// float products (z ← z·dz, normalised after the update of iterations ≡ 0 mod 64) — every phasor
// bit-identical to u_avx's — correlating sample 16m + l at iteration m.  The N mod 16 tail (serial
// from normalise(z_0), anchors after the tasks) goes to the lanes < tail of the chunk's first wave.
// Sums stay in the sample frame (no lane factor).
template <int FMT, int NT, bool IN_MARGIN>
__device__ __forceinline__ void correlate_chunk_avx(const DevJob& job, const ChunkDesc& ch, i4v span, const f2* __restrict__ Z, const float (&shifts)[NT],
    const float* __restrict__ code, int L, int lane, int part, int wpc, f2 (&acc)[NT])
{
    constexpr int SB = sample_bytes<FMT>();
    const int M = job.n_samples / kAvxLanes, T = avx_tasks_of(job.n_samples);
    const int m0 = ch.start / kAvxLanes;
    const int it_end = min(m0 + kCorrChunk / kAvxLanes, M);
    const int n_tasks = it_end > m0 ? (it_end - m0 + kAvxTaskIters - 1) / kAvxTaskIters : 0;
    const int n_groups = (n_tasks + 3) / 4;
    const int per = (n_groups + wpc - 1) / wpc;
    const int g0 = min(part * per, n_groups), g1 = min(g0 + per, n_groups);
    const f2 dz = f2{job.dz_re, job.dz_im};
    const float step = job.code_step, rem = job.rem_code;
    const int tl = lane >> 4, l = lane & (kAvxLanes - 1);
    for (int g = g0; g < g1; g++) {
        const int tc = 4 * g + tl;  // task within the chunk
        const bool active = tc < n_tasks;
        const int t = m0 / kAvxTaskIters + (active ? tc : 0);
        const int m_lo = t * kAvxTaskIters;
        const int cnt = active ? min(kAvxTaskIters, M - m_lo) : 0;
        const int n0 = kAvxLanes * m_lo + l;  // job-relative sample of iteration m_lo
        f2 x[kAvxTaskIters];
#pragma unroll
        for (int i = 0; i < kAvxTaskIters; i++) x[i] = load_sample<FMT>(span, (n0 - ch.start + kAvxLanes * i) * SB, 0);
        f2 z = Z[t * kAvxLanes + l];
        float fn = static_cast<float>(n0);  // (float)n, exact steps of 16 (n < 2^24)
#pragma unroll
        for (int i = 0; i < kAvxTaskIters; i++) {
            const bool on = i < cnt;
            const f2 r = on ? cmul_pk2(x[i], z) : f2{0.0f, 0.0f};
            f2 zn = cmul_exact(z, dz);
            if (i == 0 && (t & 3) == 0) zn = normalise_avx(zn);  // after iteration m_lo ≡ 0 (mod 64)
            z = zn;
            const float sn = __fmul_rn(step, on ? fn : static_cast<float>(n0));
#pragma unroll
            for (int q = 0; q < NT; q++) {
                const float c = code_at<IN_MARGIN>(code, L, sn, shifts[q], rem);
                acc[q] = __builtin_elementwise_fma(r, f2{c, c}, acc[q]);
            }
            fn += static_cast<float>(kAvxLanes);
        }
    }
    const int tail = job.n_samples - kAvxLanes * M;
    const int n_t = kAvxLanes * M;  // first tail sample
    if (part == 0 && tail > 0 && n_t >= ch.start && n_t < ch.start + ch.len && lane < tail) {
        const int n = n_t + lane;
        const f2 xv = load_sample<FMT>(span, (n - ch.start) * SB, 0);
        const f2 r = cmul_pk2(xv, Z[T * kAvxLanes + lane]);
        const float sn = __fmul_rn(step, static_cast<float>(n));
#pragma unroll
        for (int q = 0; q < NT; q++) {
            const float c = code_at<IN_MARGIN>(code, L, sn, shifts[q], rem);
            acc[q] = __builtin_elementwise_fma(r, f2{c, c}, acc[q]);
        }
    }
}

// One launch per chunk class (tap-count template × in-margin flag), so each kernel is compiled
// for exactly its path and the register allocation is not the worst case over all variants.
// One workgroup per WORK ITEM: up to kMaxChunksPerItem (4) chunks sharing one code replica
// (consecutive chunks of one long job, or same-code jobs such as consecutive epochs of one
// channel).  The replica is staged in LDS once per workgroup; then wave w correlates chunk w of the
// item on its own — 64 samples per lane, a block of four per step with the next block's samples in
// flight — and reduces it within the wave (no further barrier).
template <int FMT, int NT, bool IN_MARGIN, bool AVX>
__global__ __launch_bounds__(kCorrThreads, (corr_waves_per_simd<NT, IN_MARGIN, AVX>())) void corr_batch_kernel(const void* __restrict__ samples,
    const DevJob* __restrict__ jobs, const ChunkDesc* __restrict__ chunks, const WorkItem* __restrict__ items, int n_items,
    const Anchor* __restrict__ anchors, float* __restrict__ partials, float* __restrict__ out, AnchorPrefetch pf)
{
    extern __shared__ __attribute__((aligned(16))) float lds_code[];
    GNSSHIP_PROF_STAMP(0);
    // Leading workgroups replay the rotator anchors of OTHER batches (the next ones of a
    // pipelined ring): one lane per job, latency-bound chains that run beside the correlation
    // instead of in a separate stream behind a cross-queue event.
    if (static_cast<int>(blockIdx.x) < pf.n_blocks) {
#ifndef GNSSHIP_NO_REPLAY_PRIO
        __builtin_amdgcn_s_setprio(3);  // a latency-bound serial chain: first pick of its SIMD's issue slots
#endif
        int ti = 0, base = 0;
        while (ti + 1 < kAnchorRingMax && static_cast<int>(blockIdx.x) >= base + pf.task[ti].n_blocks) base += pf.task[ti++].n_blocks;
        const ReplayTask& t = pf.task[ti];
        const int gi = (blockIdx.x - base) * kCorrThreads + threadIdx.x;
        const int j = t.lanes == 1 ? gi : gi / kAvxLanes;
        if (j < t.n_jobs) {
            const DevJob pj = t.jobs[j];
            replay_anchors(pj, t.anchors, t.seg_lo, t.seg_hi, t.n_segs, t.lanes == 1 ? 0 : gi % kAvxLanes);
        }
        GNSSHIP_PROF_STAMP(5);
        return;
    }
    // XCD-aware item order: workgroups are dealt round-robin over the 8 XCDs (b and b+8 share one),
    // so give each XCD a CONTIGUOUS range of items.  Jobs arrive epoch-major, so the channels that
    // read the same IF samples then share one XCD's L2 (bijective for any grid).  pf.n_blocks is a
    // multiple of 8, so b keeps the hardware's b mod 8 placement.
    const int nb = static_cast<int>(gridDim.x) - pf.n_blocks;
    const int b = blockIdx.x - pf.n_blocks;
    const int q = nb >> 3, rmd = nb & 7, xcd = b & 7;
    const int ii = xcd * q + (xcd < rmd ? xcd : rmd) + (b >> 3);
    if (ii >= n_items) return;
    const WorkItem it = items[ii];
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6), lane = static_cast<int>(threadIdx.x) & (kWave - 1);
    const ChunkDesc c0 = chunks[it.first];
    const int L = c0.code_len;  // one replica for the whole item
    if (L <= 0 || c0.code == nullptr) {  // no code (never happens for a valid plan): outputs zero
        if (wave < it.count) {
            const ChunkDesc cz = chunks[it.first + wave];
            const DevJob& jz = jobs[cz.job];
            float* dz = (jz.n_chunks == 1) ? out + static_cast<int64_t>(cz.job) * 2 * kMaxTaps : partials + static_cast<int64_t>(it.first + wave) * 2 * kMaxTaps;
            if (lane < 2 * kMaxTaps) dz[lane] = 0.0f;
        }
        return;
    }
    // The code replica straight into LDS (global_load_lds_dwordx4: no VGPRs), pre-wrapped in HBM
    // (engine.h padded_code_quads): lds[kCodeMargin + i] = code[i mod L], i in [−kCodeMargin, L + kCodeMargin).
    {
        typedef __attribute__((address_space(1))) const void* gptr;
        typedef __attribute__((address_space(3))) void* lptr;
        const int nq = padded_code_quads(L);
        const float4* src4 = reinterpret_cast<const float4*>(c0.code - kCodeMargin);
        float4* lds4 = reinterpret_cast<float4*>(lds_code);
        const int wave_base = threadIdx.x & ~63;
        for (int q0 = 0; q0 < nq; q0 += kCorrThreads) {  // GPS 2 passes, B1I 3, E1 9
            if (q0 + static_cast<int>(threadIdx.x) < nq)
                __builtin_amdgcn_global_load_lds((gptr)(src4 + q0 + threadIdx.x), (lptr)(lds4 + q0 + wave_base), 16, 0, 0);
        }
    }
    // this wave's chunk: an item of 1 or 2 chunks spreads each chunk over 4 or 2 waves (block ranges,
    // combined in LDS below), so a lone chunk — a closed-loop epoch, the tail of a long job — still
    // runs on the whole workgroup; the first sample block is in flight while the barrier waits for
    // the replica
    const int wpc = it.count >= 3 ? 1 : (it.count == 2 ? 2 : 4);  // waves per chunk (workgroup-uniform)
    const int cidx = wave / wpc, part = wave - cidx * wpc;
    const bool active = cidx < it.count;
    const ChunkDesc ch = chunks[it.first + (active ? cidx : 0)];
    const DevJob job = jobs[ch.job];
    const i4v span = sample_span<FMT>(samples, job.sample_offset + ch.start, active ? ch.len : 0);
    const int nblk_all = active ? (ch.len + kRenorm - 1) / kRenorm : 0;  // blocks of this chunk (0..16)
    const int per = (nblk_all + wpc - 1) / wpc;
    const int kb0 = part * per < nblk_all ? part * per : nblk_all;
    const int kb1 = kb0 + per < nblk_all ? kb0 + per : nblk_all;  // this wave's blocks [kb0, kb1)
    f2 xa[kLaneSamples], xb[kLaneSamples];
    if (!AVX && kb0 < kb1) load_any<FMT>(span, lane, kb0, ch.len, xa);
    __builtin_amdgcn_s_waitcnt(0);  // the replica's LDS-DMA (and the first block) landed
    __syncthreads();
    if (!active) return;  // only when wpc == 1: no barrier follows
    GNSSHIP_PROF_STAMP(1);
    const float* code = lds_code + kCodeMargin;
    float shifts[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) shifts[t] = (t < job.n_taps) ? job.shifts[t] : 0.0f;
    // the block's four uniform phasors (scalar loads; the next block's issued one step ahead —
    // anchor buffers are padded past the last job)
    // read through the constant address space: scalar loads (this launch never writes the
    // anchors it correlates with — its replay workgroups write other batches' — but the compiler
    // cannot prove that and would otherwise load them per lane)
    typedef __attribute__((address_space(4))) const float* cfloat_ptr;
    const cfloat_ptr anc_c = (cfloat_ptr)(anchors + job.anchor_offset + (ch.start >> 8));
    auto anc = [&](int k) {
        Anchor a;
#pragma unroll
        for (int i = 0; i < 8; i++) a.p[i] = anc_c[8 * k + i];
        return a;
    };
    f2 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = f2{0.0f, 0.0f};
    if constexpr (AVX) {
        correlate_chunk_avx<FMT, NT, IN_MARGIN>(job, ch, span, reinterpret_cast<const f2*>(anchors + job.anchor_offset), shifts, code, L, lane, part, wpc,
            acc);
        float val = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const float sr = wave_sum(acc[t].x), si = wave_sum(acc[t].y);
            val = (lane == 2 * t) ? sr : val;
            val = (lane == 2 * t + 1) ? si : val;
        }
        if (wpc > 1) {  // the chunk's waves combine in LDS, in part order (deterministic)
            __shared__ float red_avx[kCorrThreads / kWave][2 * kMaxTaps];
            if (lane < 2 * kMaxTaps) red_avx[wave][lane] = val;
            __syncthreads();
            if (part != 0) return;
            float sum = 0.0f;
            for (int w = 0; w < wpc; w++) sum += (lane < 2 * kMaxTaps) ? red_avx[wave + w][lane] : 0.0f;
            val = sum;
        }
        float* dst = (job.n_chunks == 1) ? out + static_cast<int64_t>(ch.job) * 2 * kMaxTaps : partials + static_cast<int64_t>(it.first + cidx) * 2 * kMaxTaps;
        if (lane < 2 * kMaxTaps) dst[lane] = (lane < 2 * job.n_taps && ch.len > 0) ? val : 0.0f;
        return;
    }
    Anchor A = anc(kb0);
    // ping-pong over blocks: block kb0 + 2i in xa, kb0 + 2i + 1 in xb
    for (int kb = kb0; kb < kb1; kb += 2) {
        const Anchor An = anc(kb + 1);
        if (kb + 1 < kb1) load_any<FMT>(span, lane, kb + 1, ch.len, xb);
        if ((kb + 1) * kRenorm <= ch.len)
            correlate_block<NT, IN_MARGIN, true>(job, ch, A, shifts, code, L, lane, kb, xa, acc);
        else
            correlate_block<NT, IN_MARGIN, false>(job, ch, A, shifts, code, L, lane, kb, xa, acc);
        if (kb + 1 >= kb1) break;
        A = anc(kb + 2);
        if (kb + 2 < kb1) load_any<FMT>(span, lane, kb + 2, ch.len, xa);
        if ((kb + 2) * kRenorm <= ch.len)
            correlate_block<NT, IN_MARGIN, true>(job, ch, An, shifts, code, L, lane, kb + 1, xb, acc);
        else
            correlate_block<NT, IN_MARGIN, false>(job, ch, An, shifts, code, L, lane, kb + 1, xb, acc);
    }
    GNSSHIP_PROF_STAMP(3);
    // anchor frame → sample frame (× E_{4·lane}), then the wave's sums (lane v holds value v)
    const f2 e = lane_rotation(job, kLaneSamples * lane);
    const f2 esw = f2{-e.y, e.x};
    float val = 0.0f;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const f2 r = cmul_pk(acc[t], e, esw);
        const float sr = wave_sum(r.x), si = wave_sum(r.y);
        val = (lane == 2 * t) ? sr : val;
        val = (lane == 2 * t + 1) ? si : val;
    }
    if (wpc > 1) {  // the chunk's waves combine in LDS, in block order (deterministic)
        __shared__ float red[kCorrThreads / kWave][2 * kMaxTaps];
        if (lane < 2 * kMaxTaps) red[wave][lane] = val;
        __syncthreads();
        if (part != 0) return;
        float sum = 0.0f;
        for (int w = 0; w < wpc; w++) sum += (lane < 2 * kMaxTaps) ? red[wave + w][lane] : 0.0f;
        val = sum;
    }
    float* dst = (job.n_chunks == 1) ? out + static_cast<int64_t>(ch.job) * 2 * kMaxTaps : partials + static_cast<int64_t>(it.first + cidx) * 2 * kMaxTaps;
    if (lane < 2 * kMaxTaps) dst[lane] = (lane < 2 * job.n_taps && ch.len > 0) ? val : 0.0f;
    GNSSHIP_PROF_STAMP(4);
}

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

#ifdef GNSSHIP_CORR_PROFILE
}  // namespace gnsship
extern "C" int gnsship_debug_corr_profile(void* dev_buf)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(gnsship::g_corr_prof), &dev_buf, sizeof(void*)) == hipSuccess ? 0 : -3;
}
namespace gnsship {
#endif

hipError_t launch_corr_batch(const void* samples, int fmt, const DevJob* jobs, int n_jobs, const ChunkDesc* chunks, const WorkItem* items,
    int n_items, const ChunkClass* classes, int max_code_len, bool any_multi_chunk, Anchor* anchors, float* partials, float* out,
    hipStream_t stream, int stages, const AnchorPrefetch* prefetch, int replay_lanes)
{
    if (replay_lanes < 1) replay_lanes = 1;
    const int n_chunks = n_items;  // work items to launch (0: nothing to correlate)
    AnchorPrefetch pf{};
    if (prefetch && (stages & GNSSHIP_STAGE_CORRELATE)) {
        pf = *prefetch;
        int nb = 0;
        for (auto& t : pf.task) {
            if (t.lanes < 1) t.lanes = 1;
            t.n_blocks = (t.n_jobs > 0 && t.seg_lo < t.seg_hi) ? (t.n_jobs * t.lanes + kCorrThreads - 1) / kCorrThreads : 0;
            nb += t.n_blocks;
        }
        pf.n_blocks = (nb + 7) & ~7;
    }
    if (n_chunks <= 0) {
        for (const auto& t : pf.task) {
            if (t.n_blocks == 0) continue;
            hipLaunchKernelGGL(corr_anchor_kernel, dim3((t.n_jobs * t.lanes + 63) / 64), dim3(64), 0, stream, t.jobs, t.n_jobs, t.anchors, t.seg_lo,
                t.seg_hi, t.n_segs, t.lanes);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (max_code_len < 1 || max_code_len > kMaxCodeLen) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    if (stages & GNSSHIP_STAGE_ANCHORS) {
        const int threads = n_jobs * replay_lanes;
        hipLaunchKernelGGL(corr_anchor_kernel, dim3((threads + 63) / 64), dim3(64), 0, stream, jobs, n_jobs, anchors, 0, kAnchorSegments,
            kAnchorSegments, replay_lanes);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (!(stages & GNSSHIP_STAGE_CORRELATE)) return hipSuccess;
    const size_t lds = (static_cast<size_t>(max_code_len + 2 * kCodeMargin) * sizeof(float) + 15) & ~static_cast<size_t>(15);
    for (int c = 0; c < kChunkClasses; c++) {
        const int cnt = classes[c].count;
        if (cnt <= 0) continue;
        const WorkItem* ic = items + classes[c].start;
        dim3 grid(cnt + pf.n_blocks), block(kCorrThreads);
#define GNSSHIP_LAUNCH_CORR(F, NTV, MV, AV) \
    hipLaunchKernelGGL((corr_batch_kernel<F, NTV, MV, AV>), grid, block, lds, stream, samples, jobs, chunks, ic, cnt, anchors, partials, out, pf)
#define GNSSHIP_LAUNCH_NT(F)                                                     \
    switch (c) {                                                                 \
    case 0: GNSSHIP_LAUNCH_CORR(F, 1, false, false); break;                      \
    case 1: GNSSHIP_LAUNCH_CORR(F, 1, true, false); break;                       \
    case 2: GNSSHIP_LAUNCH_CORR(F, 3, false, false); break;                      \
    case 3: GNSSHIP_LAUNCH_CORR(F, 3, true, false); break;                       \
    case 4: GNSSHIP_LAUNCH_CORR(F, 5, false, false); break;                      \
    case 5: GNSSHIP_LAUNCH_CORR(F, 5, true, false); break;                       \
    case 6: GNSSHIP_LAUNCH_CORR(F, kMaxTaps, false, false); break;               \
    case 7: GNSSHIP_LAUNCH_CORR(F, kMaxTaps, true, false); break;                \
    case 8: GNSSHIP_LAUNCH_CORR(F, 1, false, true); break;                       \
    case 9: GNSSHIP_LAUNCH_CORR(F, 1, true, true); break;                        \
    case 10: GNSSHIP_LAUNCH_CORR(F, 3, false, true); break;                      \
    case 11: GNSSHIP_LAUNCH_CORR(F, 3, true, true); break;                       \
    case 12: GNSSHIP_LAUNCH_CORR(F, 5, false, true); break;                      \
    case 13: GNSSHIP_LAUNCH_CORR(F, 5, true, true); break;                       \
    case 14: GNSSHIP_LAUNCH_CORR(F, kMaxTaps, false, true); break;               \
    default: GNSSHIP_LAUNCH_CORR(F, kMaxTaps, true, true); break;                \
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
        pf = AnchorPrefetch{};  // only the first class launch carries the prefetch
    }
    e = hipGetLastError();
    if (e != hipSuccess || !any_multi_chunk) return e;
    const int total = n_jobs * 2 * kMaxTaps;
    hipLaunchKernelGGL(corr_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, jobs, n_jobs, partials, out);
    return hipGetLastError();
}

}  // namespace gnsship
