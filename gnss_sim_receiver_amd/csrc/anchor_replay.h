// anchor_replay.h — the reference rotator recursion replayed on the device (shared by the batched
// correlator's anchor stage, corr_kernel.hip, and the tracking step kernel, trk_kernel.hip, which
// replays its channels' next-epoch anchors right after deriving their NCO).  Generic jobs: one
// thread per job; AVX jobs: one thread per (job, phasor lane).
#pragma once
#include "engine.h"
#include "nco_math.h"

#pragma clang fp contract(off)

namespace gnsship {

// First renormalisation block of replay segment seg of a job with nblk blocks (segments split at
// the middle block; kAnchorSegments == 2).
__device__ __forceinline__ int segment_block(int seg, int nblk, int n_segs = kAnchorSegments)
{
    // n_segs near-equal block ranges; for 2 segments the split is at (nblk + 1) / 2
    return seg <= 0 ? 0 : (seg >= n_segs ? nblk : (nblk * seg + n_segs - 1) / n_segs);
}

// The reference rotator recursion of one job, stored at every renormalisation point — blocks of
// segments [seg_lo, seg_hi).  Block k stores the renormalised q_k and the chain's next three phasors
// q_k·inc, q_k·inc², q_k·inc³ (engine.h Anchor).  A later segment resumes from the stored q of the
// block before it: the chain after a renormalisation depends only on q.
typedef float f2v __attribute__((ext_vector_type(2)));

// The reference's complex<float> product a·b written out (re = ar·br − ai·bi, im = ar·bi + ai·br),
// each product rounded separately (no FMA).
__device__ __forceinline__ f2v avx_cmul(f2v a, f2v b) { return f2v{a.x, a.x} * b + f2v{a.y, a.y} * f2v{-b.y, b.x}; }

// _mm256_complexnormalise_ps (volk_gnsssdr_avx_intrinsics.h:56-63): z / sqrt(re² + im²).
__device__ __forceinline__ f2v avx_normalise(f2v z)
{
    const float m = sqrt_rn_f32(__fadd_rn(__fmul_rn(z.x, z.x), __fmul_rn(z.y, z.y)));
    return f2v{__fdiv_rn(z.x, m), __fdiv_rn(z.y, m)};
}

// Anchors of the AVX rotator variant (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_u_avx,
// volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:155-316), one thread per phasor lane l (engine.h
// AVX layout): 16 phasors z_l = phase·inc^l (the generic chain, :204-208); iteration m (samples
// 16m..16m+15) uses z_l and then advances z_l ← z_l·dz, normalising after the update of iterations
// m ≡ 0 (mod 64) (:240-272).  Z[16t + l] = z_l at iteration 16t; segment s of n_segs covers tasks
// [segment_block(s), segment_block(s + 1)) and a later segment resumes from the task before it.  The
// last segment's lane 0 writes the serial tail: normalise(z_0) after the loop, then ·inc per sample
// (:286-304).  Every product is the reference's float product (avx_cmul), bit for bit.
__device__ __forceinline__ void replay_anchors_avx(const DevJob& job, f2v* __restrict__ Z, int lane, int seg_lo, int seg_hi, int n_segs)
{
    const int N = job.n_samples, M = N / kAvxLanes, T = avx_tasks_of(N);
    const int kb = segment_block(seg_lo, T, n_segs), ke = segment_block(seg_hi, T, n_segs);
    const f2v inc = f2v{job.inc_re, job.inc_im};
    const f2v dz = f2v{job.dz_re, job.dz_im};
    auto step = [&](f2v z, int m) {
        z = avx_cmul(z, dz);
        return (m & 63) == 0 ? avx_normalise(z) : z;
    };
    f2v z;
    if (kb == 0) {
        z = f2v{job.p0_re, job.p0_im};
        for (int i = 0; i < kAvxLanes - 1; i++)
            if (i < lane) z = avx_cmul(z, inc);
    } else {
        z = Z[(kb - 1) * kAvxLanes + lane];
        const int m0 = (kb - 1) * kAvxTaskIters;
        for (int i = 0; i < kAvxTaskIters && m0 + i < M; i++) z = step(z, m0 + i);
    }
    for (int t = kb; t < ke; t++) {
        Z[t * kAvxLanes + lane] = z;
        if (t + 1 == ke && ke < T) break;  // the next segment resumes from here
        const int m0 = t * kAvxTaskIters;
        if (m0 + kAvxTaskIters <= M) {
            z = step(z, m0);  // m0 ≡ 0 (mod 16): only the first update can normalise
#pragma unroll
            for (int i = 1; i < kAvxTaskIters; i++) z = avx_cmul(z, dz);
        } else {
            for (int i = 0; m0 + i < M; i++) z = step(z, m0 + i);
        }
    }
    if (ke == T && lane == 0) {  // the tail, from normalise(z_0) after the loop
        f2v p = avx_normalise(z);
        for (int j = 0; j < N - kAvxLanes * M; j++) {
            Z[T * kAvxLanes + j] = p;
            p = avx_cmul(p, inc);
        }
    }
}

// lane: this thread's phasor lane for AVX jobs (0..15, replay launched with kAvxLanes threads per
// job); generic jobs run on lane 0 only.
__device__ __forceinline__ void replay_anchors(const DevJob& job, Anchor* __restrict__ anchors, int seg_lo, int seg_hi,
    int n_segs = kAnchorSegments, int lane = 0)
{
    if (job.rot_avx) {
        replay_anchors_avx(job, reinterpret_cast<f2v*>(anchors + job.anchor_offset), lane, seg_lo, seg_hi, n_segs);
        return;
    }
    if (lane != 0) return;
    const int nblk = (job.n_samples + kRenorm - 1) / kRenorm;
    const int kb = segment_block(seg_lo, nblk, n_segs), ke = segment_block(seg_hi, nblk, n_segs);
    if (kb >= ke) return;
    Anchor* out = anchors + job.anchor_offset;
    // phase·inc = (pr·ir − pi·ii, pr·ii + pi·ir) as two packed products + one packed add, each
    // rounded separately like the reference's written-out complex product (no FMA).  The sign
    // sits in the constant: fl(pi·(−ii)) = −fl(pi·ii) and x + (−y) ≡ x − y, bit for bit.
    const f2v inc_a = {job.inc_re, job.inc_im};   // × pr
    const f2v inc_b = {-job.inc_im, job.inc_re};  // × pi
    f2v p;
    if (kb == 0) {
        p = f2v{job.p0_re, job.p0_im};
    } else {
        p = f2v{out[kb - 1].p[0], out[kb - 1].p[1]};
#pragma unroll 16
        for (int s = 0; s < kRenorm; s++) p = f2v{p.x, p.x} * inc_a + f2v{p.y, p.y} * inc_b;
    }
    for (int k = kb; k < ke; k++) {
        // sample 256k uses `a = phase`; then phase /= |phase|; then 256 rotations reach 256(k+1)
        const float m = hypotf_glibc(p.x, p.y);
        const float qr = __fdiv_rn(p.x, m), qi = __fdiv_rn(p.y, m);
        Anchor A;
        A.p[0] = qr;
        A.p[1] = qi;
        p = f2v{qr, qi};
        // the first 16 rotations peeled: q·inc^1..3 are stored on the way (the chain keeps the
        // shape of a 16-step unrolled loop — 15 more such steps reach 256(k+1))
#pragma unroll
        for (int s = 1; s <= 16; s++) {
            p = f2v{p.x, p.x} * inc_a + f2v{p.y, p.y} * inc_b;
            if (s < 4) {
                A.p[2 * s] = p.x;
                A.p[2 * s + 1] = p.y;
            }
        }
        out[k] = A;
        if (k != ke - 1) {
            for (int s0 = 16; s0 < kRenorm; s0 += 16) {
#pragma unroll
                for (int s = 0; s < 16; s++) {
                    const f2v m1 = f2v{p.x, p.x} * inc_a;
                    const f2v m2 = f2v{p.y, p.y} * inc_b;
                    p = m1 + m2;
                }
            }
        }
    }
}

}  // namespace gnsship
