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

// First renormalisation block of replay segment seg of a job with nblk blocks (segments split at
// the middle block; kAnchorSegments == 2).
__device__ __forceinline__ int segment_block(int seg, int nblk)
{
    return seg <= 0 ? 0 : (seg >= kAnchorSegments ? nblk : (nblk + 1) / 2);
}

// The reference rotator recursion of one job, stored at every renormalisation point — blocks of
// segments [seg_lo, seg_hi).  A later segment resumes from the stored anchor of the block before
// it: the chain after a renormalisation depends only on the renormalised phasor q.
__device__ __forceinline__ void replay_anchors(const DevJob& job, Anchor* __restrict__ anchors, int seg_lo, int seg_hi)
{
    const int nblk = (job.n_samples + kRenorm - 1) / kRenorm;
    const int kb = segment_block(seg_lo, nblk), ke = segment_block(seg_hi, nblk);
    if (kb >= ke) return;
    Anchor* out = anchors + job.anchor_offset;
    typedef float f2v __attribute__((ext_vector_type(2)));
    // phase·inc = (pr·ir − pi·ii, pr·ii + pi·ir) as two packed products + one packed add, each
    // rounded separately like the reference's written-out complex product (no FMA).  The sign
    // sits in the constant: fl(pi·(−ii)) = −fl(pi·ii) and x + (−y) ≡ x − y, bit for bit.
    const f2v inc_a = {job.inc_re, job.inc_im};   // × pr
    const f2v inc_b = {-job.inc_im, job.inc_re};  // × pi
    f2v p;
    if (kb == 0) {
        p = f2v{job.p0_re, job.p0_im};
    } else {
        p = f2v{out[kb - 1].q_re, out[kb - 1].q_im};
#pragma unroll 16
        for (int s = 0; s < kRenorm; s++) p = f2v{p.x, p.x} * inc_a + f2v{p.y, p.y} * inc_b;
    }
    for (int k = kb; k < ke; k++) {
        // sample 256k uses `a = phase`; then phase /= |phase|; then 256 rotations reach 256(k+1)
        const float m = hypotf_glibc(p.x, p.y);
        const float qr = __fdiv_rn(p.x, m), qi = __fdiv_rn(p.y, m);
        out[k] = Anchor{qr, qi};
        p = f2v{qr, qi};
        if (k != ke - 1) {
#pragma unroll 16
            for (int s = 0; s < kRenorm; s++) {
                const f2v m1 = f2v{p.x, p.x} * inc_a;
                const f2v m2 = f2v{p.y, p.y} * inc_b;
                p = m1 + m2;
            }
        }
    }
}

__global__ void corr_anchor_kernel(const DevJob* __restrict__ jobs, int n_jobs, Anchor* __restrict__ anchors, int seg_lo, int seg_hi)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_jobs) return;
    const DevJob job = jobs[j];
    replay_anchors(job, anchors, seg_lo, seg_hi);
}

typedef float f2v_t __attribute__((ext_vector_type(2)));

// IF samples are read through raw buffer loads: a chunk's samples get their own buffer resource
// (base = its first sample, num_records = its length in bytes), so lanes past the chunk end read
// zeros from the hardware range check — no clamps, selects or exec masks on the tail — and the
// per-load offsets are SGPR constants (soffset) over one per-lane VGPR offset.
typedef int i4v __attribute__((ext_vector_type(4)));
extern "C" __device__ f2v_t gnsship_raw_buffer_load_f32x2(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2f32");
extern "C" __device__ int gnsship_raw_buffer_load_i32(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
extern "C" __device__ short gnsship_raw_buffer_load_i16(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i16");

template <int FMT>
constexpr int sample_bytes() { return FMT == GNSSHIP_FMT_CF32 ? 8 : (FMT == GNSSHIP_FMT_CI16 ? 4 : 2); }

// Buffer resource over samples [first, first + len) (gfx9 raw buffer: stride 0, dword3 0x00020000).
template <int FMT>
__device__ __forceinline__ i4v sample_span(const void* samples, int64_t first, int len)
{
    const uint64_t p = reinterpret_cast<uint64_t>(samples) + static_cast<uint64_t>(first) * sample_bytes<FMT>();
    return i4v{static_cast<int>(p & 0xffffffffu), static_cast<int>((p >> 32) & 0xffffu), (len > 0 ? len : 0) * sample_bytes<FMT>(), 0x00020000};
}

template <int FMT>
__device__ __forceinline__ f2v_t load_sample(i4v span, int voffset, int soffset)
{
    if constexpr (FMT == GNSSHIP_FMT_CF32) {
        return gnsship_raw_buffer_load_f32x2(span, voffset, soffset, 0);
    } else if constexpr (FMT == GNSSHIP_FMT_CI16) {
        const int v = gnsship_raw_buffer_load_i32(span, voffset, soffset, 0);
        return f2v_t{static_cast<float>(static_cast<short>(v & 0xffff)), static_cast<float>(static_cast<short>(v >> 16))};
    } else {
        const int v = gnsship_raw_buffer_load_i16(span, voffset, soffset, 0);
        return f2v_t{static_cast<float>(static_cast<signed char>(v & 0xff)), static_cast<float>(static_cast<signed char>((v >> 8) & 0xff))};
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sum over each 16-lane row of the wave, valid in every lane of the row: a DPP butterfly (no LDS
// round trip) — xor 1, xor 2 (quad_perm), then the 8- and 16-lane mirrors, each pairing two
// already-summed halves.  The four row sums of a wave are combined with the other waves' in LDS.
__device__ __forceinline__ float row_sum(float v)
{
    v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);  // row_half_mirror
    v += dpp_mov<0x140>(v);  // row_mirror
    return v;
}

typedef float f2 __attribute__((ext_vector_type(2)));

// (a·b) for phasor products off the parity-critical path (contraction allowed: one packed
// multiply + one packed FMA).  bsw = (−b.im, b.re).
__device__ __forceinline__ f2 cmul_pk(f2 a, f2 b, f2 bsw)
{
    return __builtin_elementwise_fma(f2{a.y, a.y}, bsw, f2{a.x, a.x} * b);
}

// x·p for packed complex values in two VOP3P instructions, the operand swizzles in op_sel /
// neg modifiers (no moves):  t = (x.re·p.re, x.re·p.im);  x·p = (x.im·(−p.im) + t.re, x.im·p.re + t.im)
__device__ __forceinline__ f2 cmul_pk2(f2 x, f2 p)
{
    f2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(x), "v"(p));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(x), "v"(p), "v"(t));
    return r;
}

// x·q with q wave-uniform (an anchor from the chunk's scalar block): q stays in its SGPR pair.
__device__ __forceinline__ f2 cmul_pk2_s(f2 x, f2 q)
{
    f2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(x), "s"(q));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(x), "s"(q), "v"(t));
    return r;
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

#ifndef GNSSHIP_CORR_GROUP
#define GNSSHIP_CORR_GROUP 4
#endif
constexpr int kGroup = GNSSHIP_CORR_GROUP;  // samples per lane per pipeline stage
constexpr int kGroups = kCorrSamplesPerThread / kGroup;
constexpr int kGroupSpan = kGroup * kCorrThreads;
static_assert(kGroups % 2 == 0, "ping-pong over pairs of groups");

// Samples of pipeline group g of a chunk for this lane (zeros past the chunk end).
template <int FMT>
__device__ __forceinline__ void load_group(i4v span, int g, f2 (&dstx)[kGroup])
{
    const int voff = static_cast<int>(threadIdx.x) * sample_bytes<FMT>();
#pragma unroll
    for (int u = 0; u < kGroup; u++) dstx[u] = load_sample<FMT>(span, voff, (g * kGroup + u) * kCorrThreads * sample_bytes<FMT>());
}

// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8]) that
// wait on the vector-memory counter only.
constexpr int waitcnt_vm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }
constexpr int kWaitVmcntGroup = waitcnt_vm(kGroup);

// E_j = |inc|^j · e^{i j Δ}: rotation from a renormalised anchor to sample 256k + j, for this
// lane's j = threadIdx.x (angle formed and range-reduced in double, then an accurate float sincos).
__device__ __forceinline__ f2 anchor_to_lane_rotation(const DevJob& job)
{
    constexpr double kTwoPi = 6.283185307179586476925286766559;
    constexpr double kInvTwoPi = 0.15915494309189533576888376337251;
    const int tid = threadIdx.x;
#ifndef GNSSHIP_EJ_LIBM
    // angle in revolutions, range-reduced in double; the hardware sin/cos (V_SIN/V_COS_F32) take
    // revolutions — E_j to a few 1e-7, against the 1e-5 correlation tolerance (the libm sincosf
    // form, GNSSHIP_EJ_LIBM, costs ~50 more VALU per chunk)
    const double rev = static_cast<double>(tid) * (job.dtheta * kInvTwoPi);
    const float rf = static_cast<float>(rev - rint(rev));
    const float s = __builtin_amdgcn_sinf(rf), c = __builtin_amdgcn_cosf(rf);
    (void)kTwoPi;
#else
    double th = static_cast<double>(tid) * job.dtheta;
    th = fma(-kTwoPi, rint(th * kInvTwoPi), th);
    float s, c;
    sincosf(static_cast<float>(th), &s, &c);
#endif
    const float mag = __fmaf_rn(static_cast<float>(tid), job.log_mag_inc, 1.0f);
    return f2{mag * c, mag * s};
}

// Correlation of one pipeline group (kGroup samples per lane) of one chunk into acc.
// `code` points at chip 0 of the padded LDS replica (valid indices [−kCodeMargin, L + kCodeMargin)).
// IN_MARGIN: the host proved every chip index of the job lies in the padded range (no modulo).
// FULL: the whole group lies inside the chunk (group-uniform; only a chunk's last group can be
// partial) — no tail clamps in the fast path.
template <int NT, bool IN_MARGIN, bool FULL>
__device__ __forceinline__ void correlate_group(const DevJob& job, const ChunkDesc& ch, const Anchor (&qk)[kBlocksPerChunk], f2 e,
    f2 esw, const float (&shifts)[NT], const float* __restrict__ code, int L, int g, const f2 (&xg)[kGroup], f2 (&acc)[NT])
{
    const int tid = threadIdx.x;  // == offset j inside every 256-sample block this lane visits
    // phase 1: every chip index of the group and its LDS read, all in flight together (the code
    // resampler, generic association order ((step*n) + shift) - rem, each rounded on its own; the
    // file is built with -ffp-contract=off)
    float cv[kGroup][NT];
    // (float)n for the group's first sample; the later ones are exact float increments of 256
    // (n + 256u is representable whenever (float)n's ulp divides 256, i.e. for every int32 n)
    const float fn0 = static_cast<float>(ch.start + tid + g * kGroupSpan);
#pragma unroll
    for (int u = 0; u < kGroup; u++) {
        const int r = tid + (g * kGroup + u) * kCorrThreads;
        const float fn = FULL ? fn0 + static_cast<float>(u * kCorrThreads) : static_cast<float>(ch.start + (r < ch.len ? r : ch.len - 1));
        const float sn = job.code_step * fn;  // reference loop counter n, as float
#ifndef GNSSHIP_CORR_SCALAR_INDEX
        // two taps per packed add: (sn + shift) then + (−rem) — x + (−r) ≡ x − r bit for bit
#pragma unroll
        for (int t = 0; t < NT; t += 2) {
            if (t + 1 < NT) {
                const f2 v = (f2{sn, sn} + f2{shifts[t], shifts[t + 1]}) + f2{-job.rem_code, -job.rem_code};
                int i0 = cvt_floor_i32(v.x), i1 = cvt_floor_i32(v.y);
                if constexpr (!IN_MARGIN) {
                    i0 = wrap_index(i0, L);
                    i1 = wrap_index(i1, L);
                }
                cv[u][t] = code[i0];
                cv[u][t + 1] = code[i1];
            } else {
                int idx = cvt_floor_i32((sn + shifts[t]) - job.rem_code);
                if constexpr (!IN_MARGIN) idx = wrap_index(idx, L);
                cv[u][t] = code[idx];
            }
        }
#else
#pragma unroll
        for (int t = 0; t < NT; t++) {
            int idx = cvt_floor_i32((sn + shifts[t]) - job.rem_code);
            if constexpr (!IN_MARGIN) idx = wrap_index(idx, L);
            cv[u][t] = code[idx];
        }
#endif
    }
    // phase 2: phasor at sample n = 256k + j: q_k · E_j, with E_0 = 1 — lane 0 uses the
    // renormalised anchor q_k where the reference uses a_k = |a_k|·q_k (|a_k| − 1 ≲ 1.5e-5 on one
    // sample in 256: ≲ 6e-8 of a tap sum); then in_common[n]·phase and the tap sums
#pragma unroll
    for (int u = 0; u < kGroup; u++) {
        const Anchor& a = qk[g * kGroup + u];  // block of sample u: chunk-uniform (SGPRs)
        const f2 x = xg[u];  // zero past the chunk end (buffer range check)
#ifndef GNSSHIP_CORR_NO_EFACTOR
        // E_j is the same for every sample of this lane (j = tid in every block): the sums are
        // kept in the anchor frame, Σ (x·q_k)·c, and rotated by E_j once per chunk (rotate_sums)
        (void)e;
        (void)esw;
        const f2 tt = cmul_pk2_s(x, f2{a.q_re, a.q_im});
#else
        const f2 p = cmul_pk(f2{a.q_re, a.q_im}, e, esw);
        const f2 tt = cmul_pk2(x, p);
#endif
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = __builtin_elementwise_fma(tt, f2{cv[u][t], cv[u][t]}, acc[t]);
    }
}

// Waves per SIMD the register allocation must allow: the 1- and 3-tap in-margin classes (GPS/B1I
// E-P-L, E1 data prompt) are held to 7 waves (≤ 72 VGPRs, spill-free): residency hides the sample
// and LDS latency of a kernel whose issue is otherwise VALU-bound; wider tap classes keep the
// general bound.  (Measured: 6 → 7 waves +1%, 8 slower.)
#ifndef GNSSHIP_CORR_WAVES_EPL
#define GNSSHIP_CORR_WAVES_EPL 7
#endif
template <int NT, bool IN_MARGIN>
constexpr int corr_waves_per_simd()
{
    return (NT <= 3 && IN_MARGIN) ? GNSSHIP_CORR_WAVES_EPL : kCorrWavesPerSimd;
}

// One launch per chunk class (tap-count template × in-margin flag), so each kernel is compiled
// for exactly its path and the register allocation is not the worst case over all variants.
// One workgroup per WORK ITEM: up to kMaxChunksPerItem chunks sharing one code replica
// (consecutive chunks of one long job, or same-code jobs such as consecutive epochs of one
// channel).  Per workgroup the replica is staged in LDS once, the sample pipeline runs on across
// chunk boundaries (the next chunk's first group loads while this chunk's last group is
// correlated), per-chunk wave sums park in LDS, and one barrier closes the item.
template <int FMT, int NT, bool IN_MARGIN>
__global__ __launch_bounds__(kCorrThreads, (corr_waves_per_simd<NT, IN_MARGIN>())) void corr_batch_kernel(const void* __restrict__ samples,
    const DevJob* __restrict__ jobs, const ChunkDesc* __restrict__ chunks, const WorkItem* __restrict__ items, int n_items,
    const Anchor* __restrict__ anchors, float* __restrict__ partials, float* __restrict__ out, AnchorPrefetch pf)
{
    extern __shared__ __attribute__((aligned(16))) float lds_code[];
    __shared__ float red[kMaxChunksPerItem][kCorrThreads / 16][2 * NT];  // per chunk: 16 row sums per value
    GNSSHIP_PROF_STAMP(0);
    // Leading workgroups replay the rotator anchors of ANOTHER batch (the next one of a
    // double-buffered pair): one lane per job, latency-bound chains that run beside the
    // correlation instead of in a separate stream behind a cross-queue event.
    if (static_cast<int>(blockIdx.x) < pf.n_blocks) {
#ifndef GNSSHIP_NO_REPLAY_PRIO
        __builtin_amdgcn_s_setprio(3);  // a latency-bound serial chain: first pick of its SIMD's issue slots
#endif
        const bool t1 = static_cast<int>(blockIdx.x) >= pf.task[0].n_blocks;
        const ReplayTask& t = pf.task[t1 ? 1 : 0];
        const int j = (blockIdx.x - (t1 ? pf.task[0].n_blocks : 0)) * kCorrThreads + threadIdx.x;
        if (j < t.n_jobs) {
            const DevJob pj = t.jobs[j];
            replay_anchors(pj, t.anchors, t.seg_lo, t.seg_hi);
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
    const int q = nb >> 3, rmd = nb & 7, x = b & 7;
    const int ii = x * q + (x < rmd ? x : rmd) + (b >> 3);
    if (ii >= n_items) return;
    const WorkItem it = items[ii];
    const ChunkDesc c0 = chunks[it.first];
    const int L = c0.code_len;  // one replica for the whole item
    if (L <= 0 || c0.code == nullptr) {  // no code (never happens for a valid plan): outputs zero
        for (int c = 0; c < it.count; c++) {
            const ChunkDesc cz = chunks[it.first + c];
            const DevJob& jz = jobs[cz.job];
            float* dz = (jz.n_chunks == 1) ? out + static_cast<int64_t>(cz.job) * 2 * kMaxTaps : partials + static_cast<int64_t>(it.first + c) * 2 * kMaxTaps;
            if (threadIdx.x < 2 * kMaxTaps) dz[threadIdx.x] = 0.0f;
        }
        return;
    }
    // Latency order: the code replica first, loaded straight into LDS (global_load_lds_dwordx4: no
    // VGPRs, nothing to spill, in flight across the sample prefetch), then this lane's first sample
    // group, then E_j while both are in flight.  The replica is pre-wrapped in HBM (engine.h:
    // padded_code_quads): lds[kCodeMargin + i] = code[i mod L], i in [−kCodeMargin, L + kCodeMargin).
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
    f2 xa[kGroup], xb[kGroup];
    f2 e;
    {
        const DevJob& j0 = jobs[c0.job];
        load_group<FMT>(sample_span<FMT>(samples, j0.sample_offset + c0.start, c0.len), 0, xa);
        e = anchor_to_lane_rotation(j0);  // ALU work while the loads are in flight
        // the replica's loads were issued before the kGroup sample loads (vmcnt retires in order)
        __builtin_amdgcn_s_waitcnt(kWaitVmcntGroup);
    }
    __syncthreads();
    GNSSHIP_PROF_STAMP(1);
    const float* code = lds_code + kCodeMargin;
    int prev_job = c0.job;

    for (int c = 0; c < it.count; c++) {
        const ChunkDesc ch = chunks[it.first + c];
        const DevJob job = jobs[ch.job];
        if (c > 0 && ch.job != prev_job) e = anchor_to_lane_rotation(job);  // same job: same E_j
        prev_job = ch.job;
        // only what the next chunk's first sample group needs is carried across the chunk
        const bool has_next = c + 1 < it.count;
        i4v next_span = i4v{0, 0, 0, 0x00020000};
        if (has_next) {
            const ChunkDesc chn = chunks[it.first + c + 1];
            next_span = sample_span<FMT>(samples, jobs[chn.job].sample_offset + chn.start, chn.len);
        }
        const f2 esw = f2{-e.y, e.x};
        float shifts[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) shifts[t] = (t < job.n_taps) ? job.shifts[t] : 0.0f;
        // the chunk's 16 anchors as one contiguous uniform block (scalar loads, one wait before the
        // loop: in the loop only in-order LDS reads use lgkmcnt).  Blocks past the chunk end (the
        // job's tail, padded buffer end) are finite values multiplied by zero samples.
        const Anchor* anc = anchors + job.anchor_offset + (ch.start >> 8);
        Anchor qk[kBlocksPerChunk];
#pragma unroll
        for (int m = 0; m < kBlocksPerChunk; m++) qk[m] = anc[m];
        const i4v span = sample_span<FMT>(samples, job.sample_offset + ch.start, ch.len);
        const int ng = (ch.len + kGroupSpan - 1) / kGroupSpan;  // groups in this chunk (0..kGroups)
        GNSSHIP_PROF_STAMP(c == 0 ? 2 : 6);
        f2 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = f2{0.0f, 0.0f};
        // ping-pong over groups: group g in xa (g even) / xb (g odd); the load issued with group g
        // is group g+1 of this chunk, or — after the last group — group 0 of the next chunk.
#pragma unroll
        for (int g = 0; g < kGroups; g++) {
            if (g < ng) {  // chunk-uniform
                f2(&cur)[kGroup] = (g & 1) ? xb : xa;
                f2(&nxt)[kGroup] = (g & 1) ? xa : xb;
                if (g + 1 < ng)
                    load_group<FMT>(span, g + 1, nxt);
                else if (has_next)
                    load_group<FMT>(next_span, 0, nxt);
                if ((g + 1) * kGroupSpan <= ch.len)
                    correlate_group<NT, IN_MARGIN, true>(job, ch, qk, e, esw, shifts, code, L, g, cur, acc);
                else
                    correlate_group<NT, IN_MARGIN, false>(job, ch, qk, e, esw, shifts, code, L, g, cur, acc);
            }
        }
        // next chunk's group 0 sits in buffer ng & 1 → move it to xa (an empty chunk issued none)
        if (ng == 0 && has_next) load_group<FMT>(next_span, 0, xa);
        if (ng & 1) {
#pragma unroll
            for (int u = 0; u < kGroup; u++) xa[u] = xb[u];
        }
        GNSSHIP_PROF_STAMP(c == 0 ? 3 : 7);
#ifndef GNSSHIP_CORR_NO_EFACTOR
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = cmul_pk(acc[t], e, esw);  // anchor frame → sample frame (× E_j)
#endif
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const float wr = row_sum(acc[t].x), wi = row_sum(acc[t].y);
            if ((threadIdx.x & 15) == 0) {
                red[c][threadIdx.x >> 4][2 * t] = wr;
                red[c][threadIdx.x >> 4][2 * t + 1] = wi;
            }
        }
    }
    __syncthreads();
    // per-chunk outputs: thread (c, v) sums the 16 row partials of value v of chunk c, in lane order
    for (int k = threadIdx.x; k < it.count * 2 * kMaxTaps; k += kCorrThreads) {
        const int c = k / (2 * kMaxTaps), v = k % (2 * kMaxTaps);
        const ChunkDesc cc = chunks[it.first + c];
        const DevJob& jc = jobs[cc.job];
        float* dst = (jc.n_chunks == 1) ? out + static_cast<int64_t>(cc.job) * 2 * kMaxTaps : partials + static_cast<int64_t>(it.first + c) * 2 * kMaxTaps;
        float s = 0.0f;
        if (v < 2 * NT && v < 2 * jc.n_taps && cc.len > 0) {
#pragma unroll
            for (int w = 0; w < kCorrThreads / 16; w++) s += red[c][w][v];
        }
        dst[v] = s;
    }
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
    hipStream_t stream, int stages, const AnchorPrefetch* prefetch)
{
    const int n_chunks = n_items;  // work items to launch (0: nothing to correlate)
    AnchorPrefetch pf{};
    if (prefetch && (stages & GNSSHIP_STAGE_CORRELATE)) {
        pf = *prefetch;
        int nb = 0;
        for (auto& t : pf.task) {
            t.n_blocks = (t.n_jobs > 0 && t.seg_lo < t.seg_hi) ? (t.n_jobs + kCorrThreads - 1) / kCorrThreads : 0;
            nb += t.n_blocks;
        }
        pf.n_blocks = (nb + 7) & ~7;
    }
    if (n_chunks <= 0) {
        for (const auto& t : pf.task) {
            if (t.n_blocks == 0) continue;
            hipLaunchKernelGGL(corr_anchor_kernel, dim3((t.n_jobs + 63) / 64), dim3(64), 0, stream, t.jobs, t.n_jobs, t.anchors, t.seg_lo, t.seg_hi);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (max_code_len < 1 || max_code_len > kMaxCodeLen) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    if (stages & GNSSHIP_STAGE_ANCHORS) {
        hipLaunchKernelGGL(corr_anchor_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, stream, jobs, n_jobs, anchors, 0, kAnchorSegments);
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
#define GNSSHIP_LAUNCH_CORR(F, NTV, MV) \
    hipLaunchKernelGGL((corr_batch_kernel<F, NTV, MV>), grid, block, lds, stream, samples, jobs, chunks, ic, cnt, anchors, partials, out, pf)
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
        pf = AnchorPrefetch{};  // only the first class launch carries the prefetch
    }
    e = hipGetLastError();
    if (e != hipSuccess || !any_multi_chunk) return e;
    const int total = n_jobs * 2 * kMaxTaps;
    hipLaunchKernelGGL(corr_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, jobs, n_jobs, partials, out);
    return hipGetLastError();
}

}  // namespace gnsship
