// serial_rotator.h — the generic rotator dot product in the reference's own order, on the device.
//
// volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_generic (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:
// 66-98) is, per call:
//     result[t] = 0;
//     for n in 0..N−1:  tmp = in[n]·phase;  if n % 256 == 0: phase /= |phase|;  phase *= phase_inc;
//                       result[t] += tmp·a_t[n]   (every tap t)
// i.e. one phasor chain of N dependent complex products and, per tap component, ONE serial float sum
// of N terms.  Neither chain can be split without changing the rounding, so the device runs them as
// a three-stage pipeline inside one workgroup, through LDS rings of kSChunk-sample chunks:
//   * the phasor lane (one lane of one wave) replays the chain and stores the phase of every sample;
//   * two producer waves (alternate chunks, one lane per sample) form tmp = x·phase (ac − bd,
//     ad + bc, every product rounded) and tmp·a_t[n] for every tap (complex × float: two rounded
//     products), the chips from the resampler's index (code_at);
//   * the accumulator wave's lane j adds component j's products in sample order.
// The chain is the critical path (≈ 6 dependent VALU per sample); the other stages keep pace.
// Used by the persistent tracking loop (trk_persist.hip) and by the batched correlator's generic jobs
// (corr_serial.hip).
#pragma once
#include "corr_device.h"

#pragma clang fp contract(off)

namespace gnsship {

constexpr int kSChunk = 64;         // samples per ring chunk (one producer lane each)
constexpr int kSRow = kSChunk + 4;  // product row stride: lane j's 16-byte reads start on bank 4j

// Ring progress counters (LDS), reset before each call.
struct SerialSync {
    int32_t zpub;     // chunks whose phases are in the ring
    int32_t ppub[2];  // chunks producer p (chunks ≡ p mod 2) has multiplied
    int32_t adone;    // chunks the accumulator has added
};

// LDS bytes of the rings for RC chunks and NA product components.
__host__ __device__ constexpr size_t serial_ring_bytes(int rc, int na)
{
    return static_cast<size_t>(rc) * (kSChunk * 2 * sizeof(float) + static_cast<size_t>(na) * kSRow * sizeof(float));
}

// The publishing wave's LDS operations complete in program order, so a counter stored after the
// data it announces lands after it (and after the reads issued before it): a relaxed store behind
// a wavefront-scope fence (which keeps the compiler from reordering) suffices, and a reader that
// acquires the counter then sees the data.
__device__ __forceinline__ void sr_publish(int32_t* p, int v)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void sr_wait(int32_t* p, int need)
{
    while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) __builtin_amdgcn_s_sleep(1);
}

// Phasor lane: Zr[(c mod RC)·64 + i] = the phase sample 64c + i is multiplied by (:77), then the
// renormalisation when n % 256 == 0 (:80-89: glibc hypotf, IEEE division) and phase *= phase_inc (:91).
__device__ __forceinline__ void serial_replay(SerialSync& s, f2* Zr, int RC, int N, f2 p, f2 inc)
{
    const int nch = (N + kSChunk - 1) / kSChunk;
    for (int c = 0; c < nch; c++) {
        if (c >= RC) sr_wait(&s.ppub[(c - RC) & 1], ((c - RC) >> 1) + 1);  // the slot's phases were read
        f2* zs = Zr + (c & (RC - 1)) * kSChunk;
        zs[0] = p;
        if ((c & 3) == 0) {  // n = 64c ≡ 0 mod 256
            const float m = hypotf_glibc(p.x, p.y);
            p = f2{__fdiv_rn(p.x, m), __fdiv_rn(p.y, m)};
        }
        p = cmul_exact_s(p, inc);
#pragma unroll 9
        for (int i = 1; i < kSChunk; i++) {
            zs[i] = p;
            p = cmul_exact_s(p, inc);
        }
        sr_publish(&s.zpub, c + 1);
    }
}

// Producer pw ∈ {0, 1} (chunks c ≡ pw mod 2), lane = sample.  Tap t < nt reads code[t] (chip 0 of a
// padded replica, LDS or global) at shift[t]; products go to component rows 2t (re) and 2t + 1 (im).
// Samples past the call hold −0 (x + (−0) = x for every x, −0 included), so the accumulator adds
// whole chunks.  The chips are looked up before the phases are awaited.
template <int FMT, int TMAX, bool IN_MARGIN>
__device__ __forceinline__ void serial_produce(SerialSync& s, const f2* Zr, float* P, int RC, i4v span, int N, int nt,
    const float* const (&code)[TMAX], const float (&shift)[TMAX], int L, float step, float rem, int lane, int pw)
{
    constexpr int SB = sample_bytes<FMT>();
    const int na = 2 * nt;
    const int nch = (N + kSChunk - 1) / kSChunk;
    f2 xn = load_sample<FMT>(span, (kSChunk * pw + lane) * SB, 0);  // past the call: 0 (buffer range check)
    for (int c = pw, i = 0; c < nch; c += 2, i++) {
        const f2 x = xn;
        if (c + 2 < nch) xn = load_sample<FMT>(span, (kSChunk * (c + 2) + lane) * SB, 0);
        const int n = kSChunk * c + lane;
        const bool on = n < N;
        const float sn = __fmul_rn(step, static_cast<float>(on ? n : N - 1));
        float cv[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; t++) cv[t] = t < nt ? code_at<IN_MARGIN>(code[t], L, sn, shift[t], rem) : 0.0f;
        if (c >= RC) sr_wait(&s.adone, c - RC + 1);  // the slot's products were added
        sr_wait(&s.zpub, c + 1);
        const int slot = c & (RC - 1);
        const f2 tmp = cmul_exact_sc(x, Zr[slot * kSChunk + lane]);
        float* dst = P + slot * na * kSRow + lane;
#pragma unroll
        for (int t = 0; t < TMAX; t++) {
            if (t < nt) {
                dst[(2 * t) * kSRow] = on ? __fmul_rn(tmp.x, cv[t]) : -0.0f;
                dst[(2 * t + 1) * kSRow] = on ? __fmul_rn(tmp.y, cv[t]) : -0.0f;
            }
        }
        sr_publish(&s.ppub[pw], i + 1);
    }
}

// Accumulator: lane j < 2·nt adds component j's products chunk after chunk, in sample order, from 0
// (result[n_vec] = 0, :71-74).  Returns the lane's sum (lanes ≥ 2·nt: a copy of component 0's).
__device__ __forceinline__ float serial_accumulate(SerialSync& s, const float* P, int RC, int N, int nt, int lane)
{
    const int na = 2 * nt;
    const int nch = (N + kSChunk - 1) / kSChunk;
    const int j = lane < na ? lane : 0;
    float acc = 0.0f;
    for (int c = 0; c < nch; c++) {
        sr_wait(&s.ppub[c & 1], (c >> 1) + 1);
        const f4v_t* src = reinterpret_cast<const f4v_t*>(P + ((c & (RC - 1)) * na + j) * kSRow);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            f4v_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = src[8 * h + u];
            if (h == 1) sr_publish(&s.adone, c + 1);  // every read of the slot is issued (LDS keeps the wave's order)
#pragma unroll
            for (int u = 0; u < 8; u++) {
                acc = __fadd_rn(acc, v[u].x);
                acc = __fadd_rn(acc, v[u].y);
                acc = __fadd_rn(acc, v[u].z);
                acc = __fadd_rn(acc, v[u].w);
            }
        }
    }
    return acc;
}

}  // namespace gnsship
