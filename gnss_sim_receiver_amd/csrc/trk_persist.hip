// trk_persist.hip — the closed DLL/PLL loop with one workgroup per channel for a whole run.
//
// dll_pll_veml_tracking::general_work (dll_pll_veml_tracking.cc:1728-2094) runs one epoch per call:
// do_correlation_step (:1037-1062) → Cpu_Multicorrelator_Real_Codes (cpu_multicorrelator_real_codes.cc:
// 103-126) → the loop update (trk_loop.h).  Epoch k+1's NCO depends on epoch k's correlations, so a
// channel is a strictly serial chain of epochs, while channels are independent.  This kernel gives
// every channel its own 256-thread workgroup that runs ALL of the channel's epochs in the IF buffer
// inside one launch: no kernel boundary, no host round trip and no grid-wide synchronisation
// between epochs.  Per epoch:
//   1. thread 0 derives the correlator arguments from the channel state (do_correlation_step);
//   2. wave 0 replays the reference's rotator recursion and publishes its anchors to LDS block by
//      block, while waves 1-3 correlate every block whose anchor is published, in a static order
//      (wave w takes work items w − 1 mod 3): the replay — the serial floor of the epoch — overlaps
//      the correlation, and every sum is formed in the same order on every run (the results are
//      bit-reproducible, independent of wave scheduling and of the other channels in the launch);
//   3. the tap sums are reduced in LDS and thread 0 runs the loop update on the channel state,
//      which lives in LDS for the whole run, and writes the epoch's record.
//
// Rotator variants (include/gnsship.h GNSSHIP_ROTATOR_*):
//  * generic (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:66-98): one phasor, N dependent
//    products per epoch, renormalised every 256 samples, and ONE serial float sum per tap component
//    (result[t] += (x·phase)·a_t[n], n = 0..N−1).  Reproduced bit for bit as a three-stage pipeline
//    through LDS rings of 64-sample chunks: wave 0's lane 0 replays the phasor chain and stores the
//    phase of every sample; waves 1-2 (alternate chunks, one lane per sample) form x·phase and its
//    products with every tap's chip; wave 3's lane j < 2·taps (+2 for the data prompt) adds tap
//    component j's products serially in sample order — the reference's own float sum.
//  * AVX (…:155-316, what volk_gnsssdr dispatches on AVX hosts): 16 phasors z_l advanced by
//    dz = normalise(inc^16), renormalised every 64 iterations.  The replay is 16 lanes × N/16 steps
//    (16× shorter than the generic chain); it publishes z_l at every renormalisation, and the
//    correlating lane of (segment, l) continues that lane's chain itself — the same float products
//    in the same order, so every phasor is bit-identical to the reference's (the sums are trees;
//    the exact AVX engines are trk_fast.hip and trk_lane.hip).
//
// High-dynamics tracking and epochs too long for LDS stay on the round-based path (trk_kernel.hip).
#include <cstdlib>

#include "corr_device.h"
#include "serial_rotator.h"
#include "trk_engine.h"

// Epoch phase timestamps for the profiling build only (make prof → scripts/libgnsship_prof.so,
// scripts/trk_wg_profile.py): slot [(channel·kProfEpochs + epoch)·16 + k] = wall_clock64() at phase
// k (0-6 and 16-21 in the kernel, 8-12 inside the loop update — trk_loop.h GNSSHIP_TRK_LOOP_STAMP —
// 13-15 inside the AVX replay; slot 7 holds the replay's shader cycles).
#ifdef GNSSHIP_CORR_PROFILE
namespace gnsship {
constexpr int kProfEpochs = 64;
constexpr int kProfSlots = 32;
__device__ unsigned long long* g_trk_prof = nullptr;
__shared__ int g_prof_epoch;
__device__ __forceinline__ void trk_prof_stamp(int e, int k)
{
    if (g_trk_prof && e < kProfEpochs) g_trk_prof[(static_cast<size_t>(blockIdx.x) * kProfEpochs + e) * kProfSlots + k] = wall_clock64();
}
}  // namespace gnsship
#define GNSSHIP_TRK_STAMP(e, k) gnsship::trk_prof_stamp((e), (k))
#define GNSSHIP_TRK_LOOP_STAMP(k) gnsship::trk_prof_stamp(gnsship::g_prof_epoch, (k))
#else
#define GNSSHIP_TRK_STAMP(e, k) \
    do {                        \
    } while (0)
#endif

#include "trk_loop.h"

#pragma clang fp contract(off)

namespace gnsship {
namespace {

constexpr int kPThreads = 256;
constexpr int kPWaves = kPThreads / kWave;
constexpr int kAvxSeg = 64;    // its renormalisation period in 16-sample iterations (:265-272)

// The epoch being correlated (LDS): the reference's call arguments as a DevJob plus the AVX step.
struct PEpoch {
    DevJob job;
    float dz_re, dz_im;  // normalise(inc^16) (AVX)
    int32_t runnable;
    int32_t in_margin;   // every chip index of the epoch lies in the padded LDS replica
    int32_t published;   // AVX: segments whose anchors are ready (S + 1 = all, tail included)
    SerialSync sync;     // generic: the serial pipeline's ring counters
    int32_t locked;      // lock_status outcome (wave 1) for the loop update (wave 0)
    double coh;          // epoch_pre's coherent integration time (0: no lock test this epoch)
    float trace_rem_carr, trace_step;  // the carrier arguments as passed (IF folded in)
    float red[kPWaves][2 * (kMaxTaps + 1)];
    float taps[2 * kMaxTaps + 2];  // the epoch's tap sums (+ the data prompt), as epoch_update reads them
    gnsship_trk_epoch rec;
    gnsship_trk_dump_record dump;
};

// The publishing wave's LDS operations complete in program order, so a counter stored after the
// data it announces lands after it: a relaxed store behind a wavefront-scope fence (which only
// keeps the compiler from reordering) needs no wait for the data store, and a reader that acquires
// the counter then sees the data.
__device__ __forceinline__ void publish(int32_t* p, int v)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void wait_published(int32_t* p, int need)
{
    while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) __builtin_amdgcn_s_sleep(1);
}

// AVX geometry of an N-sample epoch: M = N/16 iterations, cut into tasks of G iterations (G = 16,
// 32 or 64, a divisor of the renormalisation period, chosen by the LDS budget): task 0 = iteration 0,
// task t ≥ 1 = iterations [G(t−1)+1, Gt] ∩ [0, M).  Renormalisations (after iterations ≡ 0 mod 64)
// then only ever fall after a task's last iteration.  The N mod 16 tail runs serially after them.
__host__ __device__ __forceinline__ int avx_tasks(int M, int G) { return M <= 1 ? 1 : 1 + (M - 1 + G - 1) / G; }

// ---- the generic rotator: serial pipeline (serial_rotator.h) ---------------------------------------
// Ring of RC chunks in the dynamic LDS after the codes: phases, then 2·(taps + data prompt) product
// rows per chunk.  The accumulator's lane j stores component j where the loop update reads it.
template <int FMT, int NT, bool DATA>
__device__ void serial_epoch(PEpoch& ep, float* anc, int RC, i4v span, int N, const float* c0, const float* c1, int L, int lane, int wave)
{
    constexpr int TM = NT + (DATA ? 1 : 0);
    SerialSync& sy = ep.sync;
    f2* Zr = reinterpret_cast<f2*>(anc);
    float* P = anc + 2 * kSChunk * RC;
    if (wave == 0) {
        if (lane == 0) serial_replay(sy, Zr, RC, N, f2{ep.job.p0_re, ep.job.p0_im}, f2{ep.job.inc_re, ep.job.inc_im});
    } else if (wave < kPWaves - 1) {
        const float* code[TM];
        float shift[TM];
#pragma unroll
        for (int t = 0; t < TM; t++) {
            code[t] = t < NT ? c0 : c1;
            shift[t] = t < NT ? ep.job.shifts[t] : 0.0f;
        }
        if (ep.in_margin)
            serial_produce<FMT, TM, true>(sy, Zr, P, RC, span, N, TM, code, shift, L, ep.job.code_step, ep.job.rem_code, lane, wave - 1);
        else
            serial_produce<FMT, TM, false>(sy, Zr, P, RC, span, N, TM, code, shift, L, ep.job.code_step, ep.job.rem_code, lane, wave - 1);
    } else {
        const float acc = serial_accumulate(sy, P, RC, N, TM, lane);
        // the taps' components, then the data prompt at 2·kMaxTaps (the other entries were zeroed)
        if (lane < 2 * TM) ep.taps[lane < 2 * NT ? lane : 2 * kMaxTaps + lane - 2 * NT] = acc;
    }
}

// AVX (lanes 0..15 = phasor l): Z[t·16 + l] = the phasor lane l starts task t with; T[j] = the
// tail phasor of sample 16M + j.  The initial phasors are the generic chain phase·inc^l (:204-208);
// dz = normalise(inc^16) (:215-225); after iteration m's update, renormalise when m ≡ 0 mod 64.
// Whole renormalisation periods (iterations 64s+1 … 64(s+1), tasks 1 + P·s … P·(s+1) for P = 64/G)
// run as one unrolled block each — G steps, store and publish the next task's start, per task; the
// renormalisation after the block — with no per-task bookkeeping on the chain; the < 64 iterations
// after the last whole period hold no renormalisation.
template <int G>
__device__ void replay_avx(const PEpoch& ep, f2* Z, f2* T, int N, int lane, int32_t* published)
{
    constexpr int kPer = kAvxSeg / G;
    const int M = N / kAvxLanes, S = avx_tasks(M, G);
    const f2 inc = f2{ep.job.inc_re, ep.job.inc_im};
    const f2 dz = f2{ep.dz_re, ep.dz_im};
    f2 z = f2{ep.job.p0_re, ep.job.p0_im};
    for (int i = 0; i < kAvxLanes - 1; i++)
        if (i < lane) z = cmul_exact(z, inc);
    Z[lane] = z;
    if (lane == 0) publish(published, 1);
    if (M > 0) {  // iteration 0 (task 0), renormalised after its update
        z = normalise_avx(cmul_exact(z, dz));
        if (S > 1) {
            Z[kAvxLanes + lane] = z;
            if (lane == 0) publish(published, 2);
        }
    }
    if (lane == 0) GNSSHIP_TRK_LOOP_STAMP(13);
#ifdef GNSSHIP_CORR_PROFILE
    const long long c13 = clock64();  // shader cycles of the task loop → slot 7 (not a timestamp)
#endif
    const int n_per = M > 0 ? (M - 1) / kAvxSeg : 0;
    for (int sg = 0; sg < n_per; sg++) {
#pragma unroll
        for (int u = 0; u < kPer; u++) {
#pragma unroll
            for (int i = 0; i < G; i++) z = cmul_exact(z, dz);
            if (u == kPer - 1) z = normalise_avx(z);
            const int t = 1 + kPer * sg + u;  // the task just run
            if (t + 1 < S) {
                Z[(t + 1) * kAvxLanes + lane] = z;
                if (lane == 0) publish(published, t + 2);
            }
        }
    }
    for (int t = 1 + kPer * n_per; t < S; t++) {
        const int cnt = min(G * t, M - 1) - G * (t - 1);
        if (cnt == G) {
#pragma unroll
            for (int i = 0; i < G; i++) z = cmul_exact(z, dz);
        } else {
            for (int i = 0; i < cnt; i++) z = cmul_exact(z, dz);
        }
        if (t + 1 < S) {
            Z[(t + 1) * kAvxLanes + lane] = z;
            if (lane == 0) publish(published, t + 2);
        }
    }
    if (lane == 0) {  // z0 = normalise(z0) after the loop, then the serial tail (:286-304)
        GNSSHIP_TRK_LOOP_STAMP(14);
#ifdef GNSSHIP_CORR_PROFILE
        if (g_trk_prof && g_prof_epoch < kProfEpochs)
            g_trk_prof[(static_cast<size_t>(blockIdx.x) * kProfEpochs + g_prof_epoch) * kProfSlots + 7] = static_cast<unsigned long long>(clock64() - c13);
#endif
        f2 t = normalise_avx(z);
        for (int j = 0; j < N - kAvxLanes * M; j++) {
            T[j] = t;
            t = cmul_exact(t, inc);
        }
        publish(published, S + 1);
        GNSSHIP_TRK_LOOP_STAMP(15);
    }
}

// ---- correlation (AVX) ---------------------------------------------------------------------------
// AVX: wave step g = tasks 4g..4g+3 × the 16 phasors (64 lanes: lane = 16·(t − 4g) + l), each lane
// continuing its phasor's chain over the task's ≤ G iterations (sample 16m + l at iteration m), 16
// iterations per step with the next 16 samples in flight (the first 16 are loaded before the
// task's anchors are awaited); the step after the last correlates the N mod 16 tail samples.
template <int FMT, int NT, bool DATA, bool IN_MARGIN, int kB>
__device__ void consume_avx(PEpoch& ep, const f2* Z, const f2* T, i4v span, int N, int G, const float* code0, const float* code1, int L,
    int lane, int wave, f2 (&acc)[NT + 1])
{
    const DevJob& job = ep.job;
    const int M = N / kAvxLanes, S = avx_tasks(M, G);
    const int n_groups = (S + 3) / 4, tail = N - kAvxLanes * M;
    const int n_steps = n_groups + (tail > 0 ? 1 : 0);
    const f2 dz = f2{ep.dz_re, ep.dz_im};
    const float step = job.code_step, rem = job.rem_code;
    float shifts[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) shifts[t] = job.shifts[t];
    constexpr int SB = sample_bytes<FMT>();
    if (wave == 0) return;  // the replay wave
    for (int g = wave - 1; g < n_steps; g += kPWaves - 1) {  // static: wave w ≥ 1 takes steps w − 1 (mod 3)
        if (g == n_groups) {  // the serial tail (:292-304)
            wait_published(&ep.published, S + 1);
            if (lane < tail) {
                const int n = kAvxLanes * M + lane;
                const f2 x = load_sample<FMT>(span, n * SB, 0);
                const f2 r = cmul_pk2(x, T[lane]);
                const float sn = __fmul_rn(step, static_cast<float>(n));
#pragma unroll
                for (int t = 0; t < NT; t++) {
                    const float c = code_at<IN_MARGIN>(code0, L, sn, shifts[t], rem);
                    acc[t] = __builtin_elementwise_fma(r, f2{c, c}, acc[t]);
                }
                if constexpr (DATA) {
                    const float c = code_at<IN_MARGIN>(code1, L, sn, 0.0f, rem);
                    acc[NT] = __builtin_elementwise_fma(r, f2{c, c}, acc[NT]);
                }
            }
            continue;
        }
        const int t = 4 * g + (lane >> 4), l = lane & (kAvxLanes - 1);
        const bool active = t < S;
        const int m_lo = t == 0 ? 0 : G * (t - 1) + 1;
        int cnt = 0;
        if (active) cnt = t == 0 ? (M > 0 ? 1 : 0) : min(G * t, M - 1) - m_lo + 1;
        int cmax = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, __shfl_xor(cmax, o, kWave));
        cmax = __builtin_amdgcn_readfirstlane(cmax);
        // sample n = 16m + l: the lane's voffset advances by 16 samples per iteration
        const int v0 = (kAvxLanes * m_lo + l) * SB;
        f2 xa[kB], xb[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) xa[u] = load_sample<FMT>(span, v0 + u * kAvxLanes * SB, 0);
        wait_published(&ep.published, (4 * g + 4 < S ? 4 * g + 4 : S));
        f2 z = active ? Z[(active ? t : 0) * kAvxLanes + l] : f2{0.0f, 0.0f};
        for (int i0 = 0; i0 < cmax; i0 += kB) {
            if (i0 + kB < cmax) {
#pragma unroll
                for (int u = 0; u < kB; u++) xb[u] = load_sample<FMT>(span, v0 + (i0 + kB + u) * kAvxLanes * SB, 0);
            }
#pragma unroll
            for (int u = 0; u < kB; u++) {
                const int i = i0 + u;
                // past the task: weight 0, and the chip index of a sample inside the epoch (the
                // padded replica covers [0, N) only; a product 0·code[far] could meet a NaN)
                const bool on = i < cnt;
                const f2 r = on ? cmul_pk2(xa[u], z) : f2{0.0f, 0.0f};
                z = cmul_exact(z, dz);
                const int n = on ? kAvxLanes * (m_lo + i) + l : 0;
                const float sn = __fmul_rn(step, static_cast<float>(n));
#pragma unroll
                for (int q = 0; q < NT; q++) {
                    const float c = code_at<IN_MARGIN>(code0, L, sn, shifts[q], rem);
                    acc[q] = __builtin_elementwise_fma(r, f2{c, c}, acc[q]);
                }
                if constexpr (DATA) {
                    const float c = code_at<IN_MARGIN>(code1, L, sn, 0.0f, rem);
                    acc[NT] = __builtin_elementwise_fma(r, f2{c, c}, acc[NT]);
                }
            }
#pragma unroll
            for (int u = 0; u < kB; u++) xa[u] = xb[u];
        }
    }
}

// do_correlation_step's arguments for the epoch at c.nitems_read (derive_job on the device; the
// generic lane factor needs arg/|inc| in double, the AVX path needs dz instead).
// p0 / inc: (cos rem, −sin rem) and (cos −step, sin −step), evaluated by two lanes of wave 0 at once.
template <bool AVX>
__device__ void derive_epoch(PEpoch& ep, const TrkParams& k, const TrkChannel& c, int64_t off, int L, f2 p0, f2 inc)
{
    const int NT = k.n_taps;
    const float* sh = c.narrow ? k.shifts_n : k.shifts;
    DevJob& j = ep.job;
    const float spcf = static_cast<float>(k.code_samples_per_chip);
    j.sample_offset = off;
    j.n_samples = static_cast<int32_t>(k.conf.vector_length);
    j.code_id = c.code_id;
    j.n_taps = NT;
    j.rot_avx = 0;  // (the batch path's flag: this kernel has its own replays)
    j.p0_re = p0.x;
    j.p0_im = p0.y;
    j.inc_re = inc.x;
    j.inc_im = inc.y;
    j.rem_code = __fmul_rn(static_cast<float>(c.rem_code_phase_chips), spcf);
    j.code_step = __fmul_rn(static_cast<float>(c.code_phase_step_chips), spcf);
    for (int t = 0; t < kMaxTaps; t++) j.shifts[t] = t < NT ? sh[t] : 0.0f;
    if constexpr (AVX) {
        f2 d = f2{j.inc_re, j.inc_im};
        for (int q = 0; q < 4; q++) d = cmul_exact(d, d);  // dz *= dz four times (:221-225)
        d = normalise_avx(d);
        ep.dz_re = d.x;
        ep.dz_im = d.y;
    }
    // chip-index range (monotone in n): inside the padded replica the modulo is skipped (the data
    // prompt's shift 0 lies inside the taps' range)
    float smin = 0.0f, smax = 0.0f;
    for (int t = 0; t < NT; t++) {
        smin = fminf(smin, j.shifts[t]);
        smax = fmaxf(smax, j.shifts[t]);
    }
    const double span = static_cast<double>(j.code_step) * static_cast<double>(j.n_samples > 0 ? j.n_samples - 1 : 0);
    const double lo = fmin(0.0, span) + smin - j.rem_code - 2.0;
    const double hi = fmax(0.0, span) + smax - j.rem_code + 2.0;
    ep.in_margin = (isfinite(lo) && isfinite(hi) && lo >= -kCodeMargin && hi < static_cast<double>(L + kCodeMargin)) ? 1 : 0;
}

// Stage a padded code replica (engine.h padded_code_quads) in LDS.
__device__ void stage_code(float* dst, const CodeDesc& cd)
{
    const int nq = padded_code_quads(cd.len);
    const float4* src = reinterpret_cast<const float4*>(cd.ptr - kCodeMargin);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int q = threadIdx.x; q < nq; q += kPThreads) d4[q] = src[q];
}

// THRU: the throughput variant for more channels than CUs — ≤ 128 VGPRs (4 workgroups per CU) and
// a 4-deep sample prefetch; otherwise one workgroup per CU may use every register for a 16-deep one.
template <bool THRU>
constexpr int persist_waves_per_simd() { return THRU ? 4 : 1; }

template <int FMT, int NT, bool DATA, bool AVX, bool THRU>
__global__ __launch_bounds__(kPThreads, persist_waves_per_simd<THRU>()) void trk_persist_kernel(const TrkParams* __restrict__ pk, TrkChannel* __restrict__ chans,
    const CodeDesc* __restrict__ codes, int n_codes, const void* __restrict__ samples, uint64_t buf_first, int64_t buf_len, int max_rounds,
    int n_chans, int code_cap_floats, int avx_g, gnsship_trk_epoch* __restrict__ rec, gnsship_trk_dump_record* __restrict__ dump,
    gnsship_trk_corr_trace* __restrict__ trace, int* __restrict__ ran_count)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ TrkChannel sc;
    __shared__ PEpoch ep;
    __shared__ int32_t skip;
    const int ch = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const TrkParams& k = *pk;
    {
        const int* src = reinterpret_cast<const int*>(chans + ch);
        int* dst = reinterpret_cast<int*>(&sc);
        for (int i = tid; i < static_cast<int>(sizeof(TrkChannel) / 4); i += kPThreads) dst[i] = src[i];
    }
    __syncthreads();
    if (tid == 0) {
        const bool tracking = sc.state == 2 || sc.state == 3 || sc.state == 4;
        const bool codes_ok = sc.code_id >= 0 && sc.code_id < n_codes && codes[sc.code_id].ptr && codes[sc.code_id].len > 0 &&
                              padded_code_quads(codes[sc.code_id].len) * 4 <= code_cap_floats &&
                              (!DATA || (sc.data_code_id >= 0 && sc.data_code_id < n_codes && codes[sc.data_code_id].ptr &&
                                            codes[sc.data_code_id].len == codes[sc.code_id].len));
        skip = (tracking && codes_ok) ? 0 : 1;
    }
    __syncthreads();
    if (skip) return;  // idle channel: its state is untouched
    float* code0 = lds;
    float* code1 = lds + code_cap_floats;
    float* anc = lds + (DATA ? 2 : 1) * code_cap_floats;
    stage_code(code0, codes[sc.code_id]);
    if constexpr (DATA) stage_code(code1, codes[sc.data_code_id]);
    const int L = codes[sc.code_id].len;
    const float* c0 = code0 + kCodeMargin;
    const float* c1 = code1 + kCodeMargin;
    const int N = static_cast<int>(k.conf.vector_length);
    f2* Z = reinterpret_cast<f2*>(anc);
    f2* T = AVX ? Z + (avx_tasks(N / kAvxLanes, avx_g) + 1) * kAvxLanes : nullptr;
    for (int e = 0; e < max_rounds; e++) {
        if (wave == 0) {
            if (lane == 0) GNSSHIP_TRK_STAMP(e, 0);
#ifdef GNSSHIP_CORR_PROFILE
            if (lane == 0) g_prof_epoch = e;
#endif
            // the epoch's two phasors (cpu_multicorrelator_real_codes.cc:115,123), lane 0: rem_carr,
            // lane 1: −step, each glibc's cosf / sinf (glibc_sincosf.h)
            const float a = lane == 0 ? corr_rem_carr(k, sc) : -corr_phase_step(k, sc);
            if (lane == 0) {
                ep.trace_rem_carr = corr_rem_carr(k, sc);
                ep.trace_step = corr_phase_step(k, sc);
            }
            float sf, cf;
            glibc_sincosf(a, &sf, &cf);
            const f2 p0 = f2{__shfl(cf, 0, kWave), -__shfl(sf, 0, kWave)};
            const f2 inc = f2{__shfl(cf, 1, kWave), __shfl(sf, 1, kWave)};
            if (lane == 0) {
                const uint64_t vl = k.conf.vector_length;
                const bool runnable = (sc.state == 2 || sc.state == 3 || sc.state == 4) && sc.nitems_read >= buf_first &&
                                      sc.nitems_read + vl <= buf_first + static_cast<uint64_t>(buf_len);
                ep.runnable = runnable ? 1 : 0;
                if (runnable) {
                    derive_epoch<AVX>(ep, k, sc, static_cast<int64_t>(sc.nitems_read - buf_first), L, p0, inc);
                    sc.epoch_start = sc.nitems_read;
                }
                ep.published = 0;
                ep.sync = SerialSync{};
                if constexpr (!AVX)
                    for (int i = 0; i < 2 * kMaxTaps + 2; i++) ep.taps[i] = 0.0f;
                GNSSHIP_TRK_STAMP(e, 1);
            }
        }
        __syncthreads();  // also: the code replicas are staged (first epoch)
        if (!ep.runnable) break;
        // the epoch's first sample as a wave-uniform value: read from LDS it is per-lane, and a per-lane
        // buffer resource turns every sample load into a waterfall loop
        const uint64_t off64 = static_cast<uint64_t>(ep.job.sample_offset);
        const int64_t off_u = static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(off64 >> 32)))) << 32) |
                                                   static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(off64 & 0xffffffffu))));
        const i4v span = sample_span<FMT>(samples, off_u, N);
        f2 acc[NT + 1];
#pragma unroll
        for (int t = 0; t <= NT; t++) acc[t] = f2{0.0f, 0.0f};
        if constexpr (AVX) {
            if (wave == 0 && lane < kAvxLanes) {
                if (avx_g == 16) replay_avx<16>(ep, Z, T, N, lane, &ep.published);
                else if (avx_g == 32) replay_avx<32>(ep, Z, T, N, lane, &ep.published);
                else replay_avx<64>(ep, Z, T, N, lane, &ep.published);
            }
            if (tid == 0) GNSSHIP_TRK_STAMP(e, 2);
            if (ep.in_margin)
                consume_avx<FMT, NT, DATA, true, THRU ? 4 : 16>(ep, Z, T, span, N, avx_g, c0, c1, L, lane, wave, acc);
            else
                consume_avx<FMT, NT, DATA, false, THRU ? 4 : 16>(ep, Z, T, span, N, avx_g, c0, c1, L, lane, wave, acc);
        } else {
            serial_epoch<FMT, NT, DATA>(ep, anc, avx_g, span, N, c0, c1, L, lane, wave);  // avx_g = the ring's chunks
            if (tid == 0) GNSSHIP_TRK_STAMP(e, 2);
        }
        if (lane == 0) GNSSHIP_TRK_STAMP(e, wave <= 1 ? 3 + wave : 14 + wave);  // waves 2, 3: slots 16, 17
        if constexpr (AVX) {
            constexpr int kOut = NT + (DATA ? 1 : 0);
#pragma unroll
            for (int t = 0; t < kOut; t++) {
                const float sr = wave_sum(acc[t].x), si = wave_sum(acc[t].y);
                if (lane == 0) {
                    ep.red[wave][2 * t] = sr;
                    ep.red[wave][2 * t + 1] = si;
                }
            }
            if (lane == 0) GNSSHIP_TRK_STAMP(e, 18 + wave);  // wave sums stored: slots 18-21
            __syncthreads();
            // tap sums over the waves (each in the serial order w = 0..3), the data prompt at 2·kMaxTaps
            if (tid < 2 * kMaxTaps + 2) {
                const int v = tid < 2 * kMaxTaps ? tid : 2 * NT + (tid - 2 * kMaxTaps);
                float s = 0.0f;
                if (tid < 2 * NT || (DATA && tid >= 2 * kMaxTaps))
                    for (int w = 0; w < kPWaves; w++) s += ep.red[w][v];
                ep.taps[tid] = s;
            }
        }
        __syncthreads();
        const float* taps = ep.taps;
        const float* pdata = DATA ? ep.taps + 2 * kMaxTaps : ep.taps;
        gnsship_trk_dump_record* dr = dump ? &ep.dump : nullptr;
        if (tid == 0) {
            GNSSHIP_TRK_STAMP(e, 5);
            ep.rec = gnsship_trk_epoch{};
            ep.rec.flags = 8;
            ep.coh = epoch_pre(k, sc, taps, pdata, ep.rec, nullptr, dr);
        }
        __syncthreads();
        // the lock detectors (wave 1) beside the loop filters and NCO update (wave 0), which run
        // speculatively on a register copy of their members, stored only when the lock test passes
        // (trk_loop.h epoch phases)
        const double coh = ep.coh;
        LoopRegs lr;
        if (coh > 0.0) {
            if (tid == kWave) {
                GNSSHIP_TRK_LOOP_STAMP(8);
                ep.locked = lock_status(k, sc, coh) ? 1 : 0;
            } else if (tid == 0) {
                load_regs(k, sc, lr);
                epoch_loop(k, lr, nullptr);
            }
            __syncthreads();
        }
        if (tid == 0) {
            if (coh > 0.0) {
                const bool locked = ep.locked != 0;
                if (locked) store_regs(lr, sc);
                epoch_post(k, sc, taps, pdata, ep.rec, locked, dr);
            }
            epoch_finish(k, sc, ep.rec);
            const size_t slot = static_cast<size_t>(e) * n_chans + ch;
            if (rec) rec[slot] = ep.rec;
            if (dump && (ep.rec.flags & 16)) dump[slot] = ep.dump;
            if (trace) {
                gnsship_trk_corr_trace tr{};
                tr.sample_counter = sc.epoch_start;
                tr.n_samples = N;
                tr.n_taps = NT;
                tr.rem_carrier_phase_rad = ep.trace_rem_carr;
                tr.phase_step_rad = ep.trace_step;
                tr.rem_code_phase_samples = ep.job.rem_code;
                tr.code_phase_step_samples = ep.job.code_step;
                for (int t = 0; t < 5; t++) tr.shifts[t] = ep.job.shifts[t];
                for (int t = 0; t < 10; t++) tr.taps[t] = t < 2 * NT ? taps[t] : 0.0f;
                tr.data_prompt[0] = DATA ? pdata[0] : 0.0f;
                tr.data_prompt[1] = DATA ? pdata[1] : 0.0f;
                trace[slot] = tr;
            }
            atomicAdd(ran_count + e, 1);
            GNSSHIP_TRK_STAMP(e, 6);
        }
        __syncthreads();
    }
    if (tid == 0) sc.ran = 0;
    __syncthreads();
    {
        const int* src = reinterpret_cast<const int*>(&sc);
        int* dst = reinterpret_cast<int*>(chans + ch);
        for (int i = tid; i < static_cast<int>(sizeof(TrkChannel) / 4); i += kPThreads) dst[i] = src[i];
    }
}

}  // namespace

#ifdef GNSSHIP_CORR_PROFILE
}  // namespace gnsship
extern "C" int gnsship_debug_trk_profile(void* dev_buf)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(gnsship::g_trk_prof), &dev_buf, sizeof(void*)) == hipSuccess ? 0 : -3;
}
namespace gnsship {
#endif

// LDS bytes of the persistent kernel's dynamic region (codes + rings) and, for the AVX rotator, the
// task granularity G (16 iterations where the anchors fit, else 32 or 64), for the generic rotator the
// serial pipeline's ring chunks.
static size_t persist_lds(const TrkParams& p, int code_cap_floats, bool avx, int* g_out)
{
    const int N = static_cast<int>(p.conf.vector_length);
    const size_t codes = static_cast<size_t>(p.jobs_per_channel > 1 ? 2 : 1) * code_cap_floats * sizeof(float);
    if (!avx) {  // the serial pipeline's rings: 16 chunks where they fit, else 8 or 4 (g_out = RC)
        const int na = 2 * (p.n_taps + (p.jobs_per_channel > 1 ? 1 : 0));
        size_t bytes = 0;
        for (int rc = 16; rc >= 4; rc /= 2) {
            bytes = codes + serial_ring_bytes(rc, na);
            if (g_out) *g_out = rc;
            if (bytes <= kTrkPersistMaxLds) break;
        }
        return bytes;
    }
    size_t bytes = 0;
    for (int G = 16; G <= kAvxSeg; G *= 2) {
        bytes = codes + static_cast<size_t>(avx_tasks(N / kAvxLanes, G) + 2) * kAvxLanes * sizeof(f2);
        if (g_out) *g_out = G;
        if (bytes <= kTrkPersistMaxLds) break;
    }
    return bytes;
}

size_t trk_persist_lds_bytes(const TrkParams& p, int code_cap_floats, bool avx) { return persist_lds(p, code_cap_floats, avx, nullptr); }

hipError_t launch_trk_persist(const TrkParams* params_dev, const TrkParams& params, TrkChannel* chans, int n_chans, const CodeDesc* codes,
    int n_codes, int code_cap_floats, const void* samples, int fmt, uint64_t buf_first, int64_t buf_len, int max_rounds, gnsship_trk_epoch* rec,
    gnsship_trk_dump_record* dump, gnsship_trk_corr_trace* trace, int* ran_count, bool avx, hipStream_t stream)
{
    int avx_g = 0;
    const size_t lds = persist_lds(params, code_cap_floats, avx, &avx_g);
    const bool data = params.jobs_per_channel > 1;
    // more channels than CUs: the throughput variant (GNSSHIP_TRK_THRU=0/1 overrides, for A/B runs)
    bool thru = n_chans > 256;
    if (const char* env = std::getenv("GNSSHIP_TRK_THRU")) thru = env[0] == '1';
    const int nt = params.n_taps;
    dim3 grid(n_chans), block(kPThreads);
#define GNSSHIP_PERSIST(F, NTV, DV, AV)                                                                                                        \
    do {                                                                                                                                       \
        auto kfn = thru ? trk_persist_kernel<F, NTV, DV, AV, true> : trk_persist_kernel<F, NTV, DV, AV, false>;                                                                                         \
        hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)); \
        if (e0 != hipSuccess) return e0;                                                                                                       \
        hipLaunchKernelGGL(kfn, grid, block, lds, stream, params_dev, chans, codes, n_codes, samples, buf_first, buf_len, max_rounds, n_chans,  \
            code_cap_floats, avx_g, rec, dump, trace, ran_count);                                                                                     \
    } while (0)
#define GNSSHIP_PERSIST_F(F)                                                      \
    do {                                                                          \
        if (nt == 3 && !data) {                                                   \
            if (avx) GNSSHIP_PERSIST(F, 3, false, true);                          \
            else GNSSHIP_PERSIST(F, 3, false, false);                             \
        } else if (nt == 5 && !data) {                                            \
            if (avx) GNSSHIP_PERSIST(F, 5, false, true);                          \
            else GNSSHIP_PERSIST(F, 5, false, false);                             \
        } else if (nt == 5 && data) {                                             \
            if (avx) GNSSHIP_PERSIST(F, 5, true, true);                           \
            else GNSSHIP_PERSIST(F, 5, true, false);                              \
        } else {                                                                  \
            return hipErrorInvalidValue;                                          \
        }                                                                         \
    } while (0)
    switch (fmt) {
    case GNSSHIP_FMT_CF32: GNSSHIP_PERSIST_F(GNSSHIP_FMT_CF32); break;
    case GNSSHIP_FMT_CI16: GNSSHIP_PERSIST_F(GNSSHIP_FMT_CI16); break;
    case GNSSHIP_FMT_CI8: GNSSHIP_PERSIST_F(GNSSHIP_FMT_CI8); break;
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_PERSIST_F
#undef GNSSHIP_PERSIST
    return hipGetLastError();
}

}  // namespace gnsship
