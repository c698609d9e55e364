// trk_fast.hip — the closed DLL/PLL loop with the AVX rotator variant (the one volk_gnsssdr
// dispatches on AVX hosts), one workgroup per channel for a whole run, organised around the epoch's
// serial critical path and bit-exact to the reference's correlator.
//
// dll_pll_veml_tracking::general_work (dll_pll_veml_tracking.cc:1728-2094) is a strictly serial
// chain per channel: epoch k's correlations (do_correlation_step :1037-1062 →
// Cpu_Multicorrelator_Real_Codes, volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn u_avx :155-316)
// feed its loop update (cn0_and_tracking_lock_status :972-1029, run_dll_pll :1065-1152,
// update_tracking_vars :1189-1260), which sets epoch k+1's NCO.  The rate at which one channel
// advances is 1 / (epoch latency), so this kernel shortens the chain itself:
//
//  * the phasor wave: from the seed (or, in state 4, speculatively from the loop's early values,
//    confirmed by the seed) it derives glibc's cos/sin of the NCO phase and step (glibc_sincosf.h),
//    dz = normalise(inc^16) and the 16 AVX lane starts, then replays the 16 phasor chains (z ← z·dz,
//    the reference's float products, two lanes per chain with a DPP partner product; one asm block
//    per 64-iteration block) and stores each chain's phasor at every task start (G = 8 iterations)
//    with a plain LDS store — no fence, no flag: the slot itself is the signal (all-ones NaN = not
//    yet written); then the N mod 16 tail's products;
//  * the producer waves: groups of four tasks, lane (task, chain) polls its slot and continues chain l
//    over the task's iterations with the same float products — every phasor bit-identical to
//    u_avx's — forming at iteration m the sample product a = x[16m + l]·z_l(m) (_mm256_complexmul_ps
//    rounding) and per tap a·code[tap] (_mm256_mul_ps); four iterations of one product slot (2·tap +
//    component) go to the product ring as one 16-byte store, slot-major (ProdLayout); a group's flag
//    is set once its products have landed.  Producer 0 also runs the lock detectors (lock_status)
//    beside the control wave's speculative loop update, kept only when the lock test passes;
//  * the accumulator waves (one per four product slots): lane (slot row, chain l) keeps u_avx's
//    accumulator of chain l for ONE slot and adds its products in iteration order (dotProdVal +=
//    c, :257-260), four per 16-byte load, as the groups land (the group's flag and loads in one
//    batch); then combines the 16 chains exactly as u_avx does — ((d_k + d_{k+4}) + d_{k+8}) +
//    d_{k+12}, then the four lanes serially from 0 (:279-291) — and adds the serial N mod 16 tail
//    (:298-308): every tap bit-identical to the reference's;
//  * the control wave: the channel's loop state in its registers for the whole run (RChan,
//    trk_loop.h); epoch_pre → run_dll_pll (publishing the next carrier step for the phasor wave
//    right after the carrier filter) → update_tracking_vars; in state 4 it publishes the next epoch's
//    correlator arguments (the seed) before the lock test's outcome — which a failed test cancels (the
//    channel stops) — and only then finishes this epoch and writes its records.
// Roles go by SIMD (the phasor wave with accumulator 0, the control wave with accumulator 1, the
// producers in pairs, numbered round-robin over their SIMDs); the throughput form (more channels than
// CUs) runs the same roles with fewer producers, two workgroups per CU.
//
// Epochs too long for the LDS rings, the generic rotator and high_dyn stay on trk_persist.hip / the
// round-based loop.
#include <algorithm>
#include <cstdlib>

#include "corr_device.h"
#include "trk_engine.h"

#ifdef GNSSHIP_CORR_PROFILE
namespace gnsship {
namespace {
constexpr int kFProfEpochs = 16;  // profiled epochs kFProfFirst .. kFProfFirst + 15, stamped into LDS
constexpr int kFProfFirst = 8;
constexpr int kFProfSlots = 88;
__device__ unsigned long long* g_trkf_prof = nullptr;
__shared__ int g_fprof_epoch;
// stamps go to LDS and out to g_trkf_prof when the kernel ends: a global store per stamp would put
// its write acknowledgement (≈ 0.8 µs) into the next vmcnt wait of the stamping wave
__shared__ unsigned long long g_fprof_lds[kFProfEpochs * kFProfSlots];
#ifndef GNSSHIP_PROF_MASK  // the stamps compiled in (bit k: slot k; bit 63: slots 63 and up)
#define GNSSHIP_PROF_MASK 0xffffffffffffffffull
#endif
__device__ __forceinline__ constexpr bool prof_on(int k) { return ((GNSSHIP_PROF_MASK) >> (k < 63 ? k : 63)) & 1ull; }
__device__ __forceinline__ void trkf_prof_stamp(int e, int k)
{
    if (!prof_on(k)) return;
    const int r = e - kFProfFirst;
    if (g_trkf_prof && r >= 0 && r < kFProfEpochs && (threadIdx.x & 63) == 0) g_fprof_lds[r * kFProfSlots + k] = wall_clock64();
}
}  // namespace
}  // namespace gnsship
namespace gnsship {
__device__ __forceinline__ void trkf_prof_clock(int e, int k)
{
    if (!prof_on(k)) return;
    const int r = e - kFProfFirst;
    if (g_trkf_prof && r >= 0 && r < kFProfEpochs && (threadIdx.x & 63) == 0) g_fprof_lds[r * kFProfSlots + k] = clock64();
}
}  // namespace gnsship
namespace gnsship {
// a duration (shader cycles) into slot k of epoch e (per-role wait accounting)
__device__ __forceinline__ void trkf_prof_val(int e, int k, unsigned long long v)
{
    const int r = e - kFProfFirst;
    if (g_trkf_prof && r >= 0 && r < kFProfEpochs && (threadIdx.x & 63) == 0) g_fprof_lds[r * kFProfSlots + k] = v;
}
__device__ __forceinline__ void trkf_prof_hwid(int k)  // HW_ID (wave slot, SIMD, CU, SE) of the stamping wave (row 0)
{
    if (g_trkf_prof && (threadIdx.x & 63) == 0) g_fprof_lds[k] = static_cast<uint32_t>(__builtin_amdgcn_s_getreg(4 | (31 << 11)));
}
}  // namespace gnsship
#define GNSSHIP_FSTAMP(e, k) gnsship::trkf_prof_stamp((e), (k))
#define GNSSHIP_FCLK(e, k) gnsship::trkf_prof_clock((e), (k))
#define GNSSHIP_FHWID(k) gnsship::trkf_prof_hwid((k))
#define GNSSHIP_FVAL(e, k, v) gnsship::trkf_prof_val((e), (k), (v))
#define GNSSHIP_FCLOCK() clock64()
#define GNSSHIP_TRK_LOOP_STAMP(k) gnsship::trkf_prof_stamp(gnsship::g_fprof_epoch, (k))
#else
#define GNSSHIP_FSTAMP(e, k) \
    do {                     \
    } while (0)
#define GNSSHIP_FCLK(e, k) \
    do {                   \
    } while (0)
#define GNSSHIP_FHWID(k) \
    do {                 \
    } while (0)
#define GNSSHIP_FVAL(e, k, v) \
    do {                      \
    } while (0)
#define GNSSHIP_FCLOCK() 0ull
#endif

#define GNSSHIP_LOOP_INLINE __attribute__((always_inline))
#include "trk_loop.h"

#pragma clang fp contract(off)

namespace gnsship {
namespace {

#ifndef GNSSHIP_FAST_WAVES
#define GNSSHIP_FAST_WAVES 8
#endif
#ifndef GNSSHIP_THRU_WAVES  // more channels than CUs: two workgroups per CU, fewer waves each
#define GNSSHIP_THRU_WAVES 6
#endif
#ifndef GNSSHIP_FAST_WAVES_LONG  // long epochs (N ≥ kLongEpoch): production throughput counts, more producers
#define GNSSHIP_FAST_WAVES_LONG 8
#endif
constexpr int kFWaves = GNSSHIP_FAST_WAVES;
constexpr int kFWavesLong = GNSSHIP_FAST_WAVES_LONG;
constexpr int kLongEpoch = 10000;  // samples per epoch from which the long-epoch wave count applies
// The accumulation's waves: one per four product slots (2·taps, the data prompt included: GPS and
// B1I 6 slots → 2 waves, the E1 engine's 12 → 3), so that each lane adds ONE slot per iteration —
// a single serial chain per lane (fast_accumulate).
#ifndef GNSSHIP_PRE_DISC  // the accumulator waves evaluate the discriminators ahead of the loop (0: the control wave does)
#define GNSSHIP_PRE_DISC 1
#endif
#ifndef GNSSHIP_ROLE_PLAN_LONG
#define GNSSHIP_ROLE_PLAN_LONG 3
#endif
#ifndef GNSSHIP_ROLE_PLAN  // wave roles by SIMD: 0 phasor + accumulator 0 share a SIMD; 1 one primary role per SIMD
#define GNSSHIP_ROLE_PLAN 0
#endif
template <int NTT>
constexpr int acc_waves() { return (2 * NTT + 3) / 4; }
// every wave but the phasor, control and accumulator waves forms products
template <int NTT, int W>
constexpr int n_producers() { return W - 2 - acc_waves<NTT>(); }
constexpr int kMaxAccWaves = 4;  // 2·(kMaxTaps + 1) slots / 4 rows
static_assert(kFWaves - 4 >= 1 && GNSSHIP_THRU_WAVES - 4 >= 1, "trk_fast needs at least one producer wave");
// Wave roles (fast_roles): the control wave and the phasor wave each get a SIMD of their own — the
// phasor chain is the epoch's critical path and the control wave's loop update is the next — and the
// producers share the other SIMDs (two producer waves on a SIMD interleave their issue).
constexpr int kRoleControl = 0, kRoleReplay = 1, kRoleProducer = 2, kRoleAccum = 3;
// Polling waves back off this many s_sleep units (≈ 64 cycles each) between LDS polls.
// Critical-path probes (A/B builds only): n × s_sleep 4 (≈ 256 cycles each; s_sleep takes 3 bits)
#define GNSSHIP_PROBE(NAME)                                                  \
    do {                                                                     \
        _Pragma("unroll") for (int pr_ = 0; pr_ < (NAME); pr_++) __builtin_amdgcn_s_sleep(4); \
    } while (0)
#ifndef GNSSHIP_DELAY_ACC
#define GNSSHIP_DELAY_ACC 0
#endif
#ifndef GNSSHIP_DELAY_PROD
#define GNSSHIP_DELAY_PROD 0
#endif
#ifndef GNSSHIP_DELAY_REPLAY
#define GNSSHIP_DELAY_REPLAY 0
#endif
#ifndef GNSSHIP_DELAY_LOOP
#define GNSSHIP_DELAY_LOOP 0
#endif
#ifndef GNSSHIP_POLL_SLEEP
#define GNSSHIP_POLL_SLEEP 0
#endif
constexpr uint64_t kSlotEmpty = ~0ull;  // an unwritten phasor slot (NaN, NaN)

// The epoch's correlation as the producers need it (LDS: the seed from wave 0, dz from wave 1).
struct FJob {
    int64_t off;  // first sample of the epoch in the IF buffer
    float rem_code, code_step;  // do_correlation_step's rem_code_phase_chips·spc, code_phase_step_chips·spc
    float shifts[5];
    float dz_re, dz_im;  // normalise(inc^16)
    float rem_carr, step;  // the carrier arguments (IF folded in), for the trace
    int32_t runnable, in_margin, M, S, tail, pad;
};

// What the loop hands the derive wave once its carrier filter ran (state 4): the next epoch's
// carrier step, and the inputs of its remainder phase if the epoch length stays n_pred samples.
struct SpecArgs {
    double step_d, rate;
    int64_t if_num;
    float rem_prev;
    int32_t n_pred;
};

struct SpecPred {
    float rem, step, dz_re, dz_im;
};

struct FShared {
    FJob job;
    float taps[2][2 * kMaxTaps + 2];  // epoch e's tap sums in [e & 1] (+ the data prompt at 2·kMaxTaps), as epoch_pre reads them
    int32_t taps_seq[kMaxAccWaves];    // [a]: e + 1 once accumulator wave a stored its taps of epoch e
    gnsship_trk_dump_record drec;  // log_data's record of the epoch
    double coh;       // the coherent time lock_status is called with (0: no lock test this epoch)
    int32_t seed_seq; // e + 1 once wave 0 published epoch e's NCO arguments (sh.job without dz)
    int32_t job_seq;  // e + 1 once wave 1 completed epoch e's job (dz) — the producers start
    int32_t pre_seq;  // e + 1 once wave 0 published this epoch's prompt / pull-in / coh
    int32_t lock_seq; // e + 1 once wave 2 published the lock outcome
    int32_t locked;
    int32_t tail_seq;   // e + 1 once wave 1 stored epoch e's N mod 16 tail products
    int32_t acc_groups[kMaxAccWaves]; // [a]: product groups accumulator wave a has consumed (counted over the run)
    int32_t step_seq;   // e + 1 once wave 0 published epoch e's early loop values (state 4, SpecArgs)
    SpecArgs spec;      // those values
    SpecPred pred;      // wave 1's phasor prediction for epoch e (published as pred_seq = e + 1)
    int32_t pred_seq;
    int32_t verdict;    // 4·(e + 1) + 1: wave 0 confirmed epoch e's prediction and published the job; + 2: refuted; + 3: not seen
    f2 tailp[kAvxLanes][kMaxTaps + 1];  // the tail's products (sample 16M + j, tap), wave 1 → wave 0
    double pre_pll[2], pre_dll[2];  // epoch e's discriminators in [e & 1], from accumulator waves 0 / 1 (PreDisc)
    int32_t pll_seq, dll_seq;       // e + 1 once they are stored
};

// The job as wave-uniform values (scalar registers): read from LDS it would otherwise be per-lane,
// and a per-lane buffer resource turns every sample load into a waterfall loop.
__device__ __forceinline__ float unif(float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v))); }
__device__ __forceinline__ FJob uniform_job(const FJob& s)
{
    FJob j;
    const uint64_t off = static_cast<uint64_t>(s.off);
    j.off = static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(off >> 32)))) << 32) |
                                 static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(off & 0xffffffffu))));
    j.rem_code = unif(s.rem_code);
    j.code_step = unif(s.code_step);
    for (int t = 0; t < 5; t++) j.shifts[t] = unif(s.shifts[t]);
    j.dz_re = unif(s.dz_re);
    j.dz_im = unif(s.dz_im);
    j.rem_carr = unif(s.rem_carr);
    j.step = unif(s.step);
    j.runnable = __builtin_amdgcn_readfirstlane(s.runnable);
    j.in_margin = __builtin_amdgcn_readfirstlane(s.in_margin);
    j.M = __builtin_amdgcn_readfirstlane(s.M);
    j.S = __builtin_amdgcn_readfirstlane(s.S);
    j.tail = __builtin_amdgcn_readfirstlane(s.tail);
    j.pad = 0;
    return j;
}

__device__ __forceinline__ void store_slot(uint64_t* p, f2 z) { __hip_atomic_store(p, __builtin_bit_cast(uint64_t, z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ uint64_t load_slot(const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

__device__ __forceinline__ void publish_seq(int32_t* p, int v)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wait_seq(int32_t* p, int need)
{
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Product-ring flags: a producer's stores are complete (lgkmcnt) before its flag store; a reader
// that saw the flag issues its loads after it (the loads follow the polling loop in program order,
// and one wave's LDS operations are performed in order).
__device__ __forceinline__ void lds_release_store(int32_t* p, int v)
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_eq(const int32_t* p, int v)
{
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != v) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_wait_ge(const int32_t* p, int v)
{
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
    asm volatile("" ::: "memory");
}

// ---- wave 1: the AVX phasor replay ---------------------------------------------------------------
// Chain l (< 16) starts at z_l = phase·inc^l at iteration 0 (:204-208).  Task t = iterations
// [G·t, G·t + G) ∩ [0, M); its slot gets z_l at iteration G·t.  After iteration m's update the chains
// normalise when m ≡ 0 (mod 64) (:265-272) — for G | 64 only a task's first iteration can be one.
// The last task is continued by its consumer lanes; the replay goes on only for the N mod 16 tail.
//
// Two lanes per chain (lane 2l holds re, 2l + 1 im): one product z·dz is a plain multiply by dz.re,
// a DPP multiply of the partner lane's component by ∓dz.im and one add — re' = fl(fl(re·c) +
// fl(im·(−d))) ≡ fl(ac − bd), im' = fl(fl(im·c) + fl(re·d)) ≡ fl(ad + bc): the reference's
// products bit for bit, in three single-rate VALU ops instead of six (measured 15.7 vs 30 shader
// cycles per iteration on one wave, scripts/replay_bench.hip).  A DPP read needs two wait states
// after the VALU write of its source: the step's plain multiply and one s_nop.  Each lane stores its
// 32-bit half of the slot (the consumer polls until both halves are written).
#define GNSSHIP_PSTEP(X, Y)                                                                   \
    "v_mul_f32 %[t], %[c], " X "\n\t"                                                      \
    "s_nop 0\n\t"                                                                           \
    "v_mul_f32_dpp %[u], " X ", %[k2] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t" \
    "v_add_f32 " Y ", %[t], %[u]\n\t"

// N iterations (1-4) in one asm block (the hazard recognizer pads each block boundary with one
// s_nop); STORE: the block's input (the task start) goes to its slot half at `lds_off` (a byte offset
// in LDS), after the first product has read it and long before it is overwritten.
#define GNSSHIP_PSTEP_ASM(BODY)                                                                              \
    do {                                                                                                   \
        if constexpr (STORE)                                                                               \
            asm volatile(BODY : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [v] "=&v"(v)        \
                         : [c] "s"(c), [k2] "v"(k2), [p] "v"(lds_off)                                       \
                         : "memory");                                                                      \
        else                                                                                               \
            asm volatile(BODY : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [v] "=&v"(v)        \
                         : [c] "s"(c), [k2] "v"(k2), [p] "v"(lds_off));                                     \
    } while (0)
#define GNSSHIP_ST "ds_write_b32 %[p], %[x]\n\t"
template <int N, bool STORE>
__device__ __forceinline__ float pstep(float x, float c, float k2, uint32_t lds_off)
{
    static_assert(N >= 1 && N <= 4, "1-4 iterations per block");
    float t, u, w, v;
    if constexpr (N == 1) {
        if constexpr (STORE)
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_ST "v_mov_b32 %[x], %[w]\n\t");
        else
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[x]"));
    } else if constexpr (N == 2) {
        if constexpr (STORE)
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_ST GNSSHIP_PSTEP("%[w]", "%[x]"));
        else
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_PSTEP("%[w]", "%[x]"));
    } else if constexpr (N == 3) {
        if constexpr (STORE)
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_ST GNSSHIP_PSTEP("%[w]", "%[v]") GNSSHIP_PSTEP("%[v]", "%[x]"));
        else
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_PSTEP("%[w]", "%[v]") GNSSHIP_PSTEP("%[v]", "%[x]"));
    } else {
        if constexpr (STORE)
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_ST GNSSHIP_PSTEP("%[w]", "%[v]") GNSSHIP_PSTEP("%[v]", "%[w]")
                    GNSSHIP_PSTEP("%[w]", "%[x]"));
        else
            GNSSHIP_PSTEP_ASM(GNSSHIP_PSTEP("%[x]", "%[w]") GNSSHIP_PSTEP("%[w]", "%[v]") GNSSHIP_PSTEP("%[v]", "%[w]") GNSSHIP_PSTEP("%[w]", "%[x]"));
    }
    return x;
}
#undef GNSSHIP_ST
#undef GNSSHIP_PSTEP_ASM

// One whole 64-iteration block of 8-iteration tasks after its normalisation (the block's first
// iteration and its task-0 store are done): the 7 remaining iterations of task 0, then tasks 1-7 —
// each stores its start value (ds_write_b32 at its slot row, an immediate offset) and runs 8 steps —
// as ONE asm block.  The hazard recognizer pads every inline-asm boundary with an s_nop and the
// slot address would be re-derived per task otherwise; here one address serves the block.
#define GNSSHIP_PS(A, B) GNSSHIP_PSTEP("%[" #A "]", "%[" #B "]")
#define GNSSHIP_TST(A, OFF) "ds_write_b32 %[p], %[" #A "] offset:" #OFF "\n\t"
#define GNSSHIP_TASK8(A, B, OFF)                                                                                            \
    GNSSHIP_PS(A, B) GNSSHIP_TST(A, OFF) GNSSHIP_PS(B, A) GNSSHIP_PS(A, B) GNSSHIP_PS(B, A) GNSSHIP_PS(A, B) GNSSHIP_PS(B, A) \
        GNSSHIP_PS(A, B) GNSSHIP_PS(B, A)
__device__ __forceinline__ float pblock64_g8(float x, float c, float k2, uint32_t lds_off)
{
    float t, u, w;
    asm volatile(GNSSHIP_PS(x, w) GNSSHIP_PS(w, x) GNSSHIP_PS(x, w) GNSSHIP_PS(w, x) GNSSHIP_PS(x, w) GNSSHIP_PS(w, x)
                     GNSSHIP_PS(x, w) GNSSHIP_TASK8(w, x, 128) GNSSHIP_TASK8(w, x, 256) GNSSHIP_TASK8(w, x, 384) GNSSHIP_TASK8(w, x, 512)
                         GNSSHIP_TASK8(w, x, 640) GNSSHIP_TASK8(w, x, 768) GNSSHIP_TASK8(w, x, 896) "v_mov_b32 %[x], %[w]\n\t"
                 : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w)
                 : [c] "s"(c), [k2] "v"(k2), [p] "v"(lds_off)
                 : "memory");
    return x;
}
#undef GNSSHIP_TST
#undef GNSSHIP_TASK8
#undef GNSSHIP_PS
// x·dz^N: N ≥ 0 iterations
template <int N>
__device__ __forceinline__ float ppow(float x, float c, float k2)
{
    if constexpr (N >= 4) return ppow<N - 4>(pstep<4, false>(x, c, k2, 0), c, k2);
    else if constexpr (N > 0) return pstep<N, false>(x, c, k2, 0);
    else return x;
}
#undef GNSSHIP_PSTEP

// _mm256_complexnormalise_ps on the lane pair: both lanes form fl(re² + im²) (the partner's square
// by DPP), then x / sqrt(·) — normalise_avx's operations.
__device__ __forceinline__ float pnormalise(float x)
{
    const float s = __fmul_rn(x, x);
    const float o = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s), 0xB1, 0xF, 0xF, false));
    return __fdiv_rn(x, sqrt_rn_f32(__fadd_rn(s, o)));
}

// Lanes 0-31.  `x` = this lane's component of z_l, k2 = (lane odd ? dz.im : −dz.im), c = dz.re
// (uniform).  Returns the component of z_l after the last task's start (or at M with a tail).
// The slots form a ring of `rs` tasks (rs = S: one slot per task of the epoch, no ring).  In the
// ring (SRING) a slot still holds task t − rs until its producer re-armed it; the replay reads the
// state of the slot it writes next one task ahead and waits only if that slot is still taken.
template <int G, bool SRING>
__device__ __forceinline__ float fast_replay(float x, float c, float k2, int M, int S, int tail, uint64_t* __restrict__ Zs, int rs, int lane)
{
    static_assert(G % 4 == 0 && G >= 4 && G <= 64, "task length");
    constexpr int kTB = 64 / G;  // tasks per 64-iteration block
    if (S <= 0) return x;
    c = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, c)));  // dz.re in an SGPR (uniform)
    // the flat address of an LDS location carries its LDS offset in the low 32 bits
    const uint32_t base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(Zs)) + 4u * static_cast<uint32_t>(lane);
    uint32_t off = base;
    constexpr uint32_t kSlotRow = kAvxLanes * sizeof(uint64_t);
    uint32_t* const half0 = reinterpret_cast<uint32_t*>(Zs) + lane;
    int ts = 0;  // ring slot of the task
    if constexpr (!SRING) {
        const int full = (S - 1) / kTB;  // whole blocks before the last task
#pragma unroll 1
        for (int b = 0; b < full; b++) {
            if constexpr (G == 8 && kSlotRow == 128) {
                // the block's first iteration normalises; the other 63 run in one asm block
                x = pblock64_g8(pnormalise(pstep<1, true>(x, c, k2, off)), c, k2, off);
                off += kTB * kSlotRow;
            } else {
#pragma unroll
                for (int q = 0; q < kTB; q++) {
                    if (q == 0)  // the block's first iteration normalises
                        x = ppow<G - 1>(pnormalise(pstep<1, true>(x, c, k2, off)), c, k2);
                    else
                        x = ppow<G - 4>(pstep<4, true>(x, c, k2, off), c, k2);
                    off += kSlotRow;
                }
            }
        }
        if (full * kTB < S - 1) {  // a partial block: its first task normalises, the rest do not
            x = ppow<G - 1>(pnormalise(pstep<1, true>(x, c, k2, off)), c, k2);
            off += kSlotRow;
#pragma unroll 1
            for (int t = full * kTB + 1; t < S - 1; t++) {
                x = ppow<G - 4>(pstep<4, true>(x, c, k2, off), c, k2);
                off += kSlotRow;
            }
        }
        ts = S - 1;
    } else {
        // The slot ring (rs tasks, a multiple of kTB): a task's slot is rewritten once its producer
        // re-armed it (its previous lap consumed).  Whole 64-iteration blocks check their kTB slots
        // once, before the block, and run as one asm block; the rest go task by task.  (A slot read
        // per task in front of the asm blocks cost a full LDS round trip per task.)
        int t = 0;
        if constexpr (G == 8 && kSlotRow == 128) {
            if (rs % kTB == 0) {
                const int full = (S - 1) / kTB;
#pragma unroll 1
                for (int b = 0; b < full; b++, t += kTB) {
                    const int ts0 = t % rs;
                    if (t >= rs) {
                        bool busy = true;
                        while (busy) {
                            uint32_t v[kTB];
#pragma unroll
                            for (int q = 0; q < kTB; q++) v[q] = __hip_atomic_load(half0 + 2 * kAvxLanes * (ts0 + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            busy = false;
#pragma unroll
                            for (int q = 0; q < kTB; q++) busy = busy || v[q] != ~0u;
                            if (busy) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
                        }
                    }
                    off = base + static_cast<uint32_t>(ts0) * kSlotRow;
                    x = pblock64_g8(pnormalise(pstep<1, true>(x, c, k2, off)), c, k2, off);
                }
            }
        }
        ts = t % rs;
        off = base + static_cast<uint32_t>(ts) * kSlotRow;
#pragma unroll 1
        for (; t < S - 1; t++) {
            if (t >= rs)
                while (__hip_atomic_load(half0 + 2 * kAvxLanes * ts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != ~0u) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
            if (t % kTB == 0)
                x = ppow<G - 1>(pnormalise(pstep<1, true>(x, c, k2, off)), c, k2);
            else
                x = ppow<G - 4>(pstep<4, true>(x, c, k2, off), c, k2);
            ts = ts + 1 == rs ? 0 : ts + 1;
            off = base + static_cast<uint32_t>(ts) * kSlotRow;
        }
        if (S - 1 >= rs)
            while (__hip_atomic_load(half0 + 2 * kAvxLanes * ts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != ~0u) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
    }
    // the last task: its producers continue it
    __hip_atomic_store(half0 + 2 * kAvxLanes * ts, __builtin_bit_cast(uint32_t, x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (tail > 0) {  // z_l(M) for the tail (chain 0's is what the reference keeps)
        for (int m = G * (S - 1); m < M; m++) {
            x = pstep<1, false>(x, c, k2, 0);
            if ((m & 63) == 0) x = pnormalise(x);
        }
    }
    return x;
}

// Producer phase A, before the group's phasor slots are ready: the code value of every tap at
// every sample of this lane's task (the resampler, volk_gnsssdr_32f_xn_resampler_32f_xn.h:63-80), in
// registers — it depends only on the code NCO, so it runs ahead of the replay.
template <int NT, bool DATA, bool IN_MARGIN, int G, bool FULL>
__device__ __forceinline__ void group_codes(const float* __restrict__ code0, const float* __restrict__ code1, int L, int n0, int cnt, float step,
    float rem, const float (&shifts)[NT], float (&cv)[G][NT + (DATA ? 1 : 0)])
{
    float fn = static_cast<float>(n0);  // (float)n, exact steps of 16 (n < 2^24)
    const float fn0 = fn;
#pragma unroll
    for (int i = 0; i < G; i++) {
        const bool on = FULL || i < cnt;
        const float sn = __fmul_rn(step, on ? fn : fn0);
#pragma unroll
        for (int q = 0; q < NT; q++) cv[i][q] = code_at<IN_MARGIN>(code0, L, sn, shifts[q], rem);
        if constexpr (DATA) cv[i][NT] = code_at<IN_MARGIN>(code1, L, sn, 0.0f, rem);
        fn += static_cast<float>(kAvxLanes);
    }
}

typedef float f4 __attribute__((ext_vector_type(4)));

// The product ring's layout (floats): group r, product slot s (2·tap + component), chain l, iteration
// j of the group's 4G at  r·kGroup + s·kSlot + l·kRow + j.  A producer lane (task t, chain l) stores
// four iterations of one slot at once (16 bytes at j = G·t + 4h), an accumulator lane (slot row,
// chain l) loads four at once; rows padded to kRow = 4G + 4 floats make both conflict-free (the
// eight lanes of a ds_write_b128 group start 4 banks apart, the sixteen of a ds_read_b128 group too).
template <int NTT, int G>
struct ProdLayout {
    static constexpr int kJ = 4 * G;
    static constexpr int kRow = kJ + 4;
    static constexpr int kSlot = kAvxLanes * kRow;
    static constexpr int kGroup = 2 * NTT * kSlot;
};

// The products of four consecutive iterations of every product slot (2·tap + component) from the
// iterations' sample products a = x·z_l and code values: c = _mm256_mul_ps(a, code) (:252-258), one
// 16-byte store per slot.  An iteration past the epoch's last holds −0, which the accumulator adds
// unconditionally: x + (−0) = x for every x, so its sums are the reference's.
template <int NTT, int G, bool FULL, class PL>
__device__ __forceinline__ void store_products4(float* __restrict__ pdst, int i0, int cnt, const f2 (&a)[4], const float (&cv)[G][NTT])
{
    f4 q[2 * NTT];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const bool on = FULL || i0 + u < cnt;
#pragma unroll
        for (int t = 0; t < NTT; t++) {
            q[2 * t][u] = on ? __fmul_rn(a[u].x, cv[i0 + u][t]) : -0.0f;
            q[2 * t + 1][u] = on ? __fmul_rn(a[u].y, cv[i0 + u][t]) : -0.0f;
        }
    }
#pragma unroll
    for (int sl = 0; sl < 2 * NTT; sl++) *reinterpret_cast<f4*>(pdst + sl * PL::kSlot + i0) = q[sl];
}

// Producer phase B, once the slot holds z_l at the task start: per iteration the sample product
// a = x·z_l (_mm256_complexmul_ps rounding) and its products with the taps' code values, and the
// chain's own update z·dz (renormalised after the task's first iteration when that is ≡ 0 mod 64,
// :265-272).  FULL: every lane's task has all G iterations, so nothing is masked.
template <int FMT, int NTT, int G, bool FULL, class PL>
__device__ __forceinline__ void group_phasors(i4v span, f2 z, f2 dz, bool renorm, int n0, int cnt, float* __restrict__ pdst, const float (&cv)[G][NTT],
    f2 (&xa)[G < 8 ? G : 8], f2 (&xb)[G < 8 ? G : 8])
{
    constexpr int SB = sample_bytes<FMT>();
    constexpr int kB = G < 8 ? G : 8;
    static_assert(kB % 4 == 0, "16-byte product stores");
#pragma unroll 1
    for (int i0 = 0; i0 < G; i0 += kB) {
        if (i0 + kB < G) {
#pragma unroll
            for (int u = 0; u < kB; u++) xb[u] = load_sample<FMT>(span, (n0 + kAvxLanes * (i0 + kB + u)) * SB, 0);
        }
#pragma unroll
        for (int h = 0; h < kB; h += 4) {
            f2 a[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + h + u;
                a[u] = cmul_exact_pk(xa[h + u], z);
                f2 zn = cmul_exact_s(z, dz);
                if (i == 0 && renorm) zn = normalise_avx(zn);
                z = zn;
            }
            store_products4<NTT, G, FULL, PL>(pdst, i0 + h, cnt, a, cv);
        }
        if (i0 + kB < G) {
#pragma unroll
            for (int u = 0; u < kB; u++) xa[u] = xb[u];
        }
    }
}

// ---- producer waves -------------------------------------------------------------------------------
// Ring group r (of rg) holds one group of 4 tasks = 4G iterations: the products of every iteration of
// the group, chain, tap and component (ProdLayout).  Group tags count over the run (gbase = epoch ·
// n_groups): no flag is re-armed.  A ring group is reused once every accumulator wave consumed it.
// One producer per group; producer pw takes groups pw, pw + NP, ...
template <int FMT, int NT, bool DATA, bool IN_MARGIN, int G, int W>
__device__ __forceinline__ void fast_produce(const FJob& job, i4v span, const float* __restrict__ code0, const float* __restrict__ code1, int L,
    uint64_t* __restrict__ Zs, int rs, float* __restrict__ Pp, int rg, int32_t* ready, const int32_t* acc_groups, int gbase, int lane, int pw, int pe,
    f2 (&xa)[G < 8 ? G : 8], float (&cv)[G][NT + (DATA ? 1 : 0)])
{
    constexpr int SB = sample_bytes<FMT>();
    constexpr int NTT = NT + (DATA ? 1 : 0);
    constexpr int NP = n_producers<NTT, W>();
    constexpr int NA = acc_waves<NTT>();
    using PL = ProdLayout<NTT, G>;
    constexpr int kB = G < 8 ? G : 8;  // iterations whose samples are in flight together
    const int M = job.M, S = job.S;
    const int n_groups = (S + 3) / 4;
    const f2 dz = f2{job.dz_re, job.dz_im};
    const float step = job.code_step, rem = job.rem_code;
    float shifts[NT];
#pragma unroll
    for (int q = 0; q < NT; q++) shifts[q] = job.shifts[q];
    const int tl = lane >> 4, l = lane & (kAvxLanes - 1);
    f2 xb[kB];
    int rslot = pw % rg;
    const int rstep = NP % rg;
    unsigned long long w_ring = 0, w_slot = 0, w_codes = 0, w_prod = 0;  // profiling: ring / slot waits, phase A / B
    [[maybe_unused]] const unsigned long long t_run = GNSSHIP_FCLOCK();
    for (int g = pw; g < n_groups; g += NP) {
        const int t = 4 * g + tl;
        const bool active = t < S;
        const int m_lo = G * (active ? t : 0);
        const int cnt = active ? min(G, M - m_lo) : 0;
        const int n0 = kAvxLanes * m_lo + l;
        const bool full = 4 * g + 4 <= S && G * (4 * g + 4) <= M;  // every task of the group whole
        const unsigned long long tA = GNSSHIP_FCLOCK();
#pragma unroll
        for (int u = 0; u < kB; u++) xa[u] = load_sample<FMT>(span, (n0 + kAvxLanes * u) * SB, 0);  // in flight during phase A and the slot poll
        if (full)
            group_codes<NT, DATA, IN_MARGIN, G, true>(code0, code1, L, n0, G, step, rem, shifts, cv);
        else
            group_codes<NT, DATA, IN_MARGIN, G, false>(code0, code1, L, n0, cnt, step, rem, shifts, cv);
#ifdef GNSSHIP_CORR_PROFILE
        for (int i = 0; i < G; i++)  // phase A's code loads landed (profiling only)
            for (int q = 0; q < NTT; q++) asm volatile("" ::"v"(cv[i][q]));
#endif
        w_codes += GNSSHIP_FCLOCK() - tA;
        // the ring group is free once every accumulator wave consumed its previous occupant — and in
        // the slot ring (rg ≤ 16 groups of its 64 tasks) that also means the slot this lane polls next
        // was consumed on its previous lap (whichever producer took it)
        const unsigned long long t0 = GNSSHIP_FCLOCK();
        if (g >= rg) {
#pragma unroll
            for (int a = 0; a < NA; a++) lds_wait_ge(acc_groups + a, gbase + g - rg + 1);
        }
        const unsigned long long t1 = GNSSHIP_FCLOCK();
        w_ring += t1 - t0;
        uint64_t* slot = Zs + (active ? t % rs : 0) * kAvxLanes + l;
        uint64_t v = kSlotEmpty;
        if (active) {
            // written when neither 32-bit half is the sentinel any more (two replay lanes write it)
            while (static_cast<uint32_t>(v = load_slot(slot)) == ~0u || static_cast<uint32_t>(v >> 32) == ~0u) __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
            store_slot(slot, __builtin_bit_cast(f2, kSlotEmpty));  // re-armed for the next lap / epoch
        }
        w_slot += GNSSHIP_FCLOCK() - t1;
        if (g == pw && pw == 0) GNSSHIP_FSTAMP(pe, 30);
        if (g + NP >= n_groups && pw == 1) GNSSHIP_FSTAMP(pe, 31);
        const f2 z = active ? __builtin_bit_cast(f2, v) : f2{0.0f, 0.0f};
        const bool renorm = ((G * t) & 63) == 0;
        float* pdst = Pp + static_cast<size_t>(rslot) * PL::kGroup + l * PL::kRow + G * tl;
        const unsigned long long tB = GNSSHIP_FCLOCK();
        if (full)
            group_phasors<FMT, NTT, G, true, PL>(span, z, dz, renorm, n0, G, pdst, cv, xa, xb);
        else
            group_phasors<FMT, NTT, G, false, PL>(span, z, dz, renorm, n0, cnt, pdst, cv, xa, xb);
        GNSSHIP_PROBE(GNSSHIP_DELAY_PROD);
        if (lane == 0) lds_release_store(ready + 2 * rslot, gbase + g + 1);
        w_prod += GNSSHIP_FCLOCK() - tB;
        if (g < 8) GNSSHIP_FSTAMP(pe, 48 + g);
        rslot += rstep;
        if (rslot >= rg) rslot -= rg;
    }
    if (pw == 0) {  // slots 41-43, 79, 80: producer 0's ring waits, slot waits, whole production, phase A, phase B
        GNSSHIP_FVAL(pe, 41, w_ring);
        GNSSHIP_FVAL(pe, 42, w_slot);
        GNSSHIP_FVAL(pe, 43, GNSSHIP_FCLOCK() - t_run);
        GNSSHIP_FVAL(pe, 79, w_codes);
        GNSSHIP_FVAL(pe, 80, w_prod);
    }
}

// ---- accumulator waves: the accumulation in u_avx's order ---------------------------------------
// Accumulator wave a (of NA) lane (r, l): chain l's accumulators of the product slots
// s_k = 4·(a + NA·k) + r (slot s = 2·tap + component) — each c = _mm256_mul_ps(a, code) the producers
// formed is added in iteration order, dotProdVal_{l/4}[tap] += c (:252-260), one v_add_f32 per slot
// and iteration, four iterations of a slot per 16-byte load.  A slot index past the last reads the
// last slot (its sums are discarded).
template <int NTT>
constexpr int acc_slots() { return (2 * NTT + 4 * acc_waves<NTT>() - 1) / (4 * acc_waves<NTT>()); }
template <int NTT>
__device__ __forceinline__ int acc_slot(int a, int r, int k) { return 4 * (a + acc_waves<NTT>() * k) + r; }

template <int NTT, int G>
__device__ __forceinline__ void fast_accumulate(const float* __restrict__ Pp, int rg, const int32_t* ready, int32_t* acc_done, int gbase, int S,
    int lane, int a, float (&acc)[acc_slots<NTT>()], int pe)
{
    using PL = ProdLayout<NTT, G>;
    constexpr int NS = acc_slots<NTT>();
    constexpr int kQ = PL::kJ / 4;  // four-iteration loads per slot and group
    const int l = lane & (kAvxLanes - 1), r = lane >> 4;
    const int n_groups = (S + 3) / 4;
    int off[NS];
#pragma unroll
    for (int k = 0; k < NS; k++) {
        acc[k] = 0.0f;
        off[k] = min(acc_slot<NTT>(a, r, k), 2 * NTT - 1) * PL::kSlot + l * PL::kRow;
    }
    unsigned long long w_flag = 0;  // profiling: cycles spent waiting for the groups' flags
    [[maybe_unused]] const unsigned long long t_run = GNSSHIP_FCLOCK();
    int rslot = 0;
    // per group: its flag, then all its loads in one batch, then the adds in iteration order (every
    // group is added whole: a partial group's iterations past the epoch's end hold −0)
    for (int g = 0; g < n_groups; g++) {
        const unsigned long long t0 = GNSSHIP_FCLOCK();
        lds_wait_eq(ready + 2 * rslot, gbase + g + 1);  // the group's loads follow the flag
        const float* src = Pp + static_cast<size_t>(rslot) * PL::kGroup;
        f4 v[kQ][NS];
#pragma unroll
        for (int q = 0; q < kQ; q++)
#pragma unroll
            for (int k = 0; k < NS; k++) v[q][k] = *reinterpret_cast<const f4*>(src + off[k] + 4 * q);
        w_flag += GNSSHIP_FCLOCK() - t0;
#pragma unroll
        for (int q = 0; q < kQ; q++)
#pragma unroll
            for (int k = 0; k < NS; k++)
#pragma unroll
                for (int u = 0; u < 4; u++) acc[k] = __fadd_rn(acc[k], v[q][k][u]);
        if (g == 0) GNSSHIP_FSTAMP(pe, 28);
        if (g == n_groups - 1) GNSSHIP_FSTAMP(pe, 29);
        // released after its adds: they consumed every load of the group, so the ring slot may be rewritten
#pragma unroll
        for (int k = 0; k < NS; k++) asm volatile("" ::"v"(acc[k]) : "memory");
        GNSSHIP_PROBE(GNSSHIP_DELAY_ACC);
        if (lane == 0) __hip_atomic_store(acc_done, gbase + g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        rslot = rslot + 1 == rg ? 0 : rslot + 1;
    }
    if (a < 2) {  // slots 44/45 (accumulator 0), 46/47 (accumulator 1): flag waits, whole accumulation
        GNSSHIP_FVAL(pe, 44 + 2 * a, w_flag);
        GNSSHIP_FVAL(pe, 45 + 2 * a, GNSSHIP_FCLOCK() - t_run);
    }
}

// u_avx's final combination of the 16 chains (:279-291), valid at lane 0 of each 16-lane row:
// ((d_k + d_{k+4}) + d_{k+8}) + d_{k+12} for k = 0..3, then (((0 + s_0) + s_1) + s_2) + s_3.
__device__ __forceinline__ float avx_chain_sum(float d)
{
    float s = d + dpp_mov<0x12C>(d);  // row_ror:12 — lane k reads lane k + 4
    s = s + dpp_mov<0x128>(d);        // row_ror:8  — lane k + 8
    s = s + dpp_mov<0x124>(d);        // row_ror:4  — lane k + 12
    float r = 0.0f + s;
    r = r + dpp_mov<0x101>(s);  // row_shl:1 — lane 0 reads lane 1
    r = r + dpp_mov<0x102>(s);  // row_shl:2
    r = r + dpp_mov<0x103>(s);  // row_shl:3
    return r;
}

// The N mod 16 tail (:298-308) on wave 1: lane j < tail forms sample 16M + j's products with the
// serial phasor T[j] (the accumulator adds them in order after the chain combination).
template <int FMT, int NT, bool DATA, bool IN_MARGIN>
__device__ __forceinline__ void fast_tail_products(const FJob& job, i4v span, const float* __restrict__ code0, const float* __restrict__ code1, int L,
    const f2* T, int lane, f2 (*tp)[kMaxTaps + 1])
{
    constexpr int SB = sample_bytes<FMT>();
    if (lane >= job.tail) return;
    const int n = kAvxLanes * job.M + lane;
    const f2 x = load_sample<FMT>(span, n * SB, 0);
    const f2 wo = cmul_exact(x, T[lane]);  // wo = in_common[n] · _phase
    const float sn = __fmul_rn(job.code_step, static_cast<float>(n));
#pragma unroll
    for (int q = 0; q < NT; q++) {
        const float c = code_at<IN_MARGIN>(code0, L, sn, job.shifts[q], job.rem_code);
        tp[lane][q] = wo * f2{c, c};
    }
    if constexpr (DATA) {
        const float c = code_at<IN_MARGIN>(code1, L, sn, 0.0f, job.rem_code);
        tp[lane][NT] = wo * f2{c, c};
    }
}

__device__ __forceinline__ void stage_code_f(float* dst, const CodeDesc& cd, int nthreads)
{
    const int nq = padded_code_quads(cd.len);
    const float4* src = reinterpret_cast<const float4*>(cd.ptr - kCodeMargin);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int q = threadIdx.x; q < nq; q += nthreads) d4[q] = src[q];
}

// THRU (more channels than CUs): two workgroups per CU; otherwise one.  Two waves on a SIMD each keep
// their own issue cadence.
template <bool THRU, int W>
constexpr int fast_waves_per_simd() { return ((THRU ? 2 : 1) * W + 3) / 4; }

template <bool THRU>
__device__ __forceinline__ const auto& loop_params(const TrkParams& k, const KFast& kf)
{
    if constexpr (THRU)
        return k;
    else
        return kf;
}

// The carrier step's phasor inc = (cos −step, sin −step) (cpu_multicorrelator_real_codes.cc:123, glibc
// cosf / sinf) and the AVX rotator's dz = normalise(inc^16) by four squarings (:215-225).
__device__ __forceinline__ void derive_step(float step, f2& inc, f2& dz)
{
    float s, c;
    glibc_sincosf(-step, &s, &c);
    inc = f2{c, s};
    f2 d = inc;
#pragma unroll
    for (int i = 0; i < 4; i++) d = cmul_exact_sc(d, d);
    dz = normalise_avx(d);
}

// derive_step and derive_chains at once: both phasors, then the 15-step z chain with dz's four
// squarings interleaved (independent chains, one instruction stream)
__device__ __forceinline__ void derive_all(float step, float rem, int lane, f2& inc, f2& dz, f2& zinit)
{
    float ss, cs, sr, cr;
    glibc_sincosf(-step, &ss, &cs);
    glibc_sincosf(rem, &sr, &cr);
    inc = f2{cs, ss};
    const f2 p0 = f2{cr, -sr};
    f2 w = p0, z = p0, d = inc;
#pragma unroll
    for (int i = 0; i < kAvxLanes - 1; i++) {
        w = cmul_exact_sc(w, inc);
        if (i < 4) d = cmul_exact_sc(d, d);
        z = i + 1 == (lane >> 1) ? w : z;
    }
    dz = normalise_avx(d);
    zinit = z;
}

// a wave-uniform 64-bit value as scalar registers
__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v)), hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// z_l = phase·inc^l, the generic chain (:204-208) from phase = (cos rem, −sin rem) (glibc cosf / sinf,
// cpu_multicorrelator_real_codes.cc:115), for the replay's lane pairs (lanes 2l, 2l + 1: chain l).
__device__ __forceinline__ f2 derive_chains(float rem, f2 inc, int lane)
{
    float sfn, cfn;
    glibc_sincosf(rem, &sfn, &cfn);
    const f2 p0 = f2{cfn, -sfn};
    f2 w = p0, z = p0;
#pragma unroll
    for (int i = 0; i < kAvxLanes - 1; i++) {
        w = cmul_exact_sc(w, inc);
        z = i + 1 == (lane >> 1) ? w : z;
    }
    return z;
}

template <int FMT, int NT, bool DATA, int G, bool THRU, bool SRING, int W>
__global__ __launch_bounds__(W * kWave, (fast_waves_per_simd<THRU, W>())) void trk_fast_kernel(const TrkParams* __restrict__ pk, TrkChannel* __restrict__ chans,
    const CodeDesc* __restrict__ codes, int n_codes, const void* __restrict__ samples, uint64_t buf_first, int64_t buf_len, int max_rounds,
    int n_chans, int code_cap_floats, int rs, int rg, gnsship_trk_epoch* __restrict__ rec, gnsship_trk_dump_record* __restrict__ dump,
    gnsship_trk_corr_trace* __restrict__ trace, int* __restrict__ ran_count)
{
    constexpr int NTT = NT + (DATA ? 1 : 0);
    constexpr int kFWaves = W;  // this instance's waves
    constexpr int kFThreads = kFWaves * kWave;
    static_assert(acc_waves<NTT>() <= kMaxAccWaves && n_producers<NTT, kFWaves>() >= 1, "trk_fast wave roles");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ TrkChannel sc;
    __shared__ FShared sh;
    __shared__ int32_t skip;
    __shared__ f2 tailz[kAvxLanes];
    const int ch = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // (an LDS copy of the parameters measured slower: 8.20 vs 8.00 us per C2 epoch, profiling build)
    const TrkParams& k = *pk;
    {
        const int* src = reinterpret_cast<const int*>(chans + ch);
        int* dst = reinterpret_cast<int*>(&sc);
        for (int i = tid; i < static_cast<int>(sizeof(TrkChannel) / 4); i += kFThreads) dst[i] = src[i];
    }
    // dynamic LDS: phasor slots (rs tasks) | code replica(s) | ring: sample products (rg groups) |
    // ring: code values | ring flags
    uint64_t* Zs = reinterpret_cast<uint64_t*>(lds);  // first: the replay's slot stores address it through M0[15:0]
    float* code0 = reinterpret_cast<float*>(Zs + static_cast<size_t>(rs) * kAvxLanes);
    float* code1 = code0 + code_cap_floats;
    float* Pp = code0 + (DATA ? 2 : 1) * code_cap_floats;
    int32_t* ready = reinterpret_cast<int32_t*>(Pp + static_cast<size_t>(rg) * ProdLayout<NTT, G>::kGroup);
    for (int i = tid; i < rs * kAvxLanes; i += kFThreads) Zs[i] = kSlotEmpty;
    for (int i = tid; i < 2 * rg; i += kFThreads) ready[i] = 0;
    __shared__ int32_t simd_of[kFWaves];
    if (lane == 0) simd_of[wave] = static_cast<int32_t>((__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3);  // HW_ID.SIMD_ID
#ifdef GNSSHIP_CORR_PROFILE
    for (int i = tid; i < kFProfEpochs * kFProfSlots; i += kFThreads) g_fprof_lds[i] = 0;
#endif
    __syncthreads();
    // The role of each wave, by SIMD: the phasor wave (the epoch's critical chain) takes the SIMD with
    // the fewest waves and shares it with accumulator wave 0 (whose adds trail the replay); the control
    // wave and accumulator wave 1 go next, the producers fill the rest.  pw: the index within the role.
    constexpr int NA = acc_waves<NTT>();
    int role = kRoleProducer, pw = 0;
    {
        auto count = [&](int sd) {
            int c = 0;
            for (int w = 0; w < kFWaves; w++) c += (simd_of[w] & 3) == sd ? 1 : 0;
            return c;
        };
        // plan 1: one primary role per SIMD — the phasor wave, the accumulators, the control wave —
        // each beside producers only; plan 0: the phasor wave shares its SIMD with accumulator 0.
        // A plan that leaves a role unassigned (an unusual wave placement) falls back to plan 0.
        auto assign = [&](int plan) __attribute__((always_inline)) {
            int nacc = 0, nprod = 0, nsimd = 0;
            bool ctl = false, rep = false;
            // SIMDs in order of their wave count (no arrays: a dynamically indexed one would live in scratch)
            for (int cc = 1; cc <= kFWaves; cc++)
                for (int sd = 0; sd < 4; sd++) {
                    if (count(sd) != cc) continue;
                    bool first = true;
                    for (int w = 0; w < kFWaves; w++) {
                        if ((simd_of[w] & 3) != sd) continue;
                        int rl, idx = 0;
                        if (plan == 3) {
                            // the phasor wave beside a producer, the accumulators together, the
                            // control wave beside a producer
                            if (nsimd == 0 && !rep) {
                                rl = kRoleReplay;
                                rep = true;
                            } else if (nsimd == 1 && nacc < NA) {
                                rl = kRoleAccum;
                                idx = nacc++;
                            } else if (nsimd == 2 && !ctl) {
                                rl = kRoleControl;
                                ctl = true;
                            } else if (nsimd >= 2 && nacc < NA) {
                                rl = kRoleAccum;
                                idx = nacc++;
                            } else if (nsimd >= 3 && !ctl) {
                                rl = kRoleControl;
                                ctl = true;
                            } else {
                                rl = kRoleProducer;
                                idx = nprod++;
                            }
                        } else if (plan == 2) {
                            // the phasor wave beside the control wave (whose loop work mostly falls
                            // between replays), the accumulators together, the producers together
                            if (nsimd == 0 && !rep) {
                                rl = kRoleReplay;
                                rep = true;
                            } else if (nsimd == 0 && !ctl) {
                                rl = kRoleControl;
                                ctl = true;
                            } else if (nsimd >= 1 && nacc < NA) {
                                rl = kRoleAccum;
                                idx = nacc++;
                            } else if (!ctl) {
                                rl = kRoleControl;
                                ctl = true;
                            } else {
                                rl = kRoleProducer;
                                idx = nprod++;
                            }
                        } else if (!rep) {
                            rl = kRoleReplay;
                            rep = true;
                        } else if (plan == 1 ? (first && nacc < NA) : nacc == 0) {
                            rl = kRoleAccum;
                            idx = nacc++;
                        } else if (plan == 1 ? (first && !ctl) : !ctl) {
                            rl = kRoleControl;
                            ctl = true;
                        } else if (plan == 0 && nacc < NA) {
                            rl = kRoleAccum;
                            idx = nacc++;
                        } else {
                            rl = kRoleProducer;
                            idx = nprod++;
                        }
                        first = false;
                        if (w == wave) {
                            role = rl;
                            pw = idx;
                        }
                    }
                    nsimd++;
                }
            return rep && ctl && nacc == NA && nprod >= 1;
        };
        // long epochs (N ≥ kLongEpoch) run plan GNSSHIP_ROLE_PLAN_LONG: the phasor wave beside a producer
        // only, the accumulators together (measured: GPS 25 Msps 42.1× vs 39.8× real time, E1 C4 share
        // 26.9× vs 26.4×, C5 share 8.7× vs 8.1×; at 4 Msps that plan costs the headline 3-9 %)
        const int plan = static_cast<int>(k.conf.vector_length) >= kLongEpoch ? GNSSHIP_ROLE_PLAN_LONG : GNSSHIP_ROLE_PLAN;
        if (!assign(plan)) assign(0);
        role = __builtin_amdgcn_readfirstlane(role);
        pw = __builtin_amdgcn_readfirstlane(pw);
    }
    __shared__ int32_t role_of[kFWaves];
    if (lane == 0) role_of[wave] = role;
    if (tid == 0) {
        const bool tracking = sc.state == 2 || sc.state == 3 || sc.state == 4;
        const bool codes_ok = sc.code_id >= 0 && sc.code_id < n_codes && codes[sc.code_id].ptr && codes[sc.code_id].len > 0 &&
                              padded_code_quads(codes[sc.code_id].len) * 4 <= code_cap_floats &&
                              (!DATA || (sc.data_code_id >= 0 && sc.data_code_id < n_codes && codes[sc.data_code_id].ptr &&
                                            codes[sc.data_code_id].len == codes[sc.code_id].len));
        skip = (tracking && codes_ok) ? 0 : 1;
        sh.seed_seq = 0;
        sh.job_seq = 0;
        sh.pre_seq = 0;
        sh.lock_seq = 0;
        sh.tail_seq = 0;
        for (int a = 0; a < kMaxAccWaves; a++) sh.taps_seq[a] = sh.acc_groups[a] = 0;
        sh.step_seq = 0;
        sh.pred_seq = 0;
        sh.verdict = 0;
        sh.pll_seq = sh.dll_seq = 0;
    }
    __syncthreads();
    if (skip) return;  // idle channel: its state is untouched
    if (role == kRoleProducer) {
        // producers numbered round-robin over their SIMDs (rank within the SIMD first), so that the
        // producers of consecutive groups — the epoch's last two above all — sit on different SIMDs
        auto rank_in_simd = [&](int w) {
            int r = 0;
            for (int v = 0; v < w; v++) r += (role_of[v] == kRoleProducer && (simd_of[v] & 3) == (simd_of[w] & 3)) ? 1 : 0;
            return r;
        };
        const int rk = rank_in_simd(wave), sd = simd_of[wave] & 3;
        int idx = 0;
        for (int v = 0; v < kFWaves; v++) {
            if (v == wave || role_of[v] != kRoleProducer) continue;
            const int rv = rank_in_simd(v), sv = simd_of[v] & 3;
            idx += (rv < rk || (rv == rk && sv < sd)) ? 1 : 0;
        }
        pw = __builtin_amdgcn_readfirstlane(idx);
    }
    if (wave < 4) GNSSHIP_FHWID(20 + wave);  // epoch 0's slots 20-23 (the epoch loop stamps 0-15)
#ifdef GNSSHIP_CORR_PROFILE
    if (g_trkf_prof && lane == 0)  // row 0's slots 72-77: HW_ID | role << 32 of every wave
        g_fprof_lds[72 + wave] = static_cast<uint32_t>(__builtin_amdgcn_s_getreg(4 | (31 << 11))) | (static_cast<unsigned long long>(role) << 32);
#endif
    stage_code_f(code0, codes[sc.code_id], kFThreads);
    if constexpr (DATA) stage_code_f(code1, codes[sc.data_code_id], kFThreads);
    __syncthreads();  // the code replicas are staged before any wave correlates
    const int L = codes[sc.code_id].len;
    const float* c0 = code0 + kCodeMargin;
    const float* c1 = code1 + kCodeMargin;
    const int N = static_cast<int>(k.conf.vector_length);
    const int M = N / kAvxLanes;
    const int S = (M + G - 1) / G;
    const int tail = N - kAvxLanes * M;
    const int n_groups = (S + 3) / 4;
    RChan rc;
    if (role == kRoleControl) rchan_load(sc, &sc, rc);
    // wave 0's loop parameters in registers for the run (two workgroups per CU have no registers to
    // spare: they keep reading TrkParams)
    KFast kf = make_kfast(k, sc.geo);
    // the sign patterns epoch_pre reads every epoch (bit_at), in LDS: a global load there is a
    // dependent memory round trip on the loop's chain
    __shared__ uint32_t sec_bits[kTrkMaxSecondary / 32], dsec_bits[kTrkMaxSecondary / 32];
    if constexpr (!THRU) {
        if (tid < kTrkMaxSecondary / 32) {
            sec_bits[tid] = kf.sv.secondary_bits[tid];
            dsec_bits[tid] = kf.sv.data_secondary_bits[tid];
        }
        kf.sv.secondary_bits = sec_bits;
        kf.sv.data_secondary_bits = dsec_bits;
        __syncthreads();
    }
    const auto& kp = loop_params<THRU>(k, kf);
    // Discriminators ahead of the loop: where every state-4 epoch's E / P / L are its own taps (no
    // secondary code to strip, no extended integration), the accumulator waves evaluate the PLL and
    // DLL discriminators right after storing the taps — the same operations on the same floats as
    // epoch_pre + run_dll_pll — while the control wave runs epoch_pre; it then takes both values.
    const bool pre_disc = __builtin_amdgcn_readfirstlane(GNSSHIP_PRE_DISC && !k.sync[sc.geo].secondary && k.sync[sc.geo].extend == 1 ? 1 : 0) != 0;
    // Wave roles (one channel per workgroup, its epochs a serial chain): see the file header.  The
    // control wave hands the next epoch's NCO arguments (the seed) to the phasor wave as soon as they
    // are settled, so the derive and the first tasks of epoch e + 1 overlap epoch e's record writes.
    uint64_t seed_start = 0;              // wave 0: the epoch start the seed was made for
    // wave 0: the seed's per-run constants, read once (inside the epoch loop each TrkParams member is a
    // dependent scalar load on the chain)
    const uint64_t vl = k.conf.vector_length;
    const float spcf = static_cast<float>(k.code_samples_per_chip);
    const int32_t has_if = k.has_if;
    const double if_step = k.if_step_rad;
    float shv_w[5], shv_n[5];
    float smin_w = 0.0f, smax_w = 0.0f, smin_n = 0.0f, smax_n = 0.0f;
#pragma unroll
    for (int t = 0; t < 5; t++) {
        shv_w[t] = t < NT ? k.shifts[t] : 0.0f;
        shv_n[t] = t < NT ? k.shifts_n[t] : 0.0f;
        smin_w = fminf(smin_w, shv_w[t]);
        smax_w = fmaxf(smax_w, shv_w[t]);
        smin_n = fminf(smin_n, shv_n[t]);
        smax_n = fmaxf(smax_n, shv_n[t]);
    }
    // wave 0: the job's code and sample arguments for an epoch starting at absolute sample nir
    auto code_fields = [&](FJob& j, uint64_t nir) __attribute__((always_inline)) {
        const bool nw = uni(rc.narrow) != 0;
        j.off = static_cast<int64_t>(nir - buf_first);
        j.rem_code = __fmul_rn(static_cast<float>(rc.rem_code_phase_chips), spcf);
        j.code_step = __fmul_rn(static_cast<float>(rc.code_phase_step_chips), spcf);
#pragma unroll
        for (int t = 0; t < 5; t++) j.shifts[t] = nw ? shv_n[t] : shv_w[t];
        const float smin = nw ? smin_n : smin_w, smax = nw ? smax_n : smax_w;
        const double span = static_cast<double>(j.code_step) * static_cast<double>(N > 0 ? N - 1 : 0);
        const double lo = fmin(0.0, span) + smin - j.rem_code - 2.0;
        const double hi = fmax(0.0, span) + smax - j.rem_code + 2.0;
        j.in_margin = (isfinite(lo) && isfinite(hi) && lo >= -kCodeMargin && hi < static_cast<double>(L + kCodeMargin)) ? 1 : 0;
        j.M = M;
        j.S = S;
        j.tail = tail;
    };
    // wave 0: do_correlation_step's arguments for the epoch at nitems_read (all but the phasors)
    auto make_seed = [&](int e) {
        const bool runnable = e < max_rounds && (rc.state == 2 || rc.state == 3 || rc.state == 4) && rc.nitems_read >= buf_first &&
                              rc.nitems_read + vl <= buf_first + static_cast<uint64_t>(buf_len);
        // corr_rem_carr / corr_phase_step (trk_loop.h) on the hoisted IF constants
        const float rem_carr = has_if ? static_cast<float>(fmod_2pi(static_cast<double>(rc.rem_carr_phase_rad) + kTwoPi * rc.if_cyc))
                                      : rc.rem_carr_phase_rad;
        const float stepf = static_cast<float>(rc.carrier_phase_step_rad + if_step);
        if (runnable) rc.epoch_start = rc.nitems_read;
        seed_start = rc.epoch_start;
        if (lane == 0) {
            FJob& j = sh.job;
            j.runnable = runnable ? 1 : 0;
            if (runnable) {
                code_fields(j, rc.nitems_read);
                j.rem_carr = rem_carr;
                j.step = stepf;
            }
            // wave 1's speculative replay of this epoch (whole-epoch slots): confirmed here when its
            // remainder phase and step are the seed's floats, and the job goes out with the seed
            int code = 3;
            if (!SRING && __hip_atomic_load(&sh.pred_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= e + 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // sh.pred is read after its sequence number
                code = 2;
                if (runnable && __builtin_bit_cast(uint32_t, sh.pred.rem) == __builtin_bit_cast(uint32_t, rem_carr) &&
                    __builtin_bit_cast(uint32_t, sh.pred.step) == __builtin_bit_cast(uint32_t, stepf)) {
                    j.dz_re = sh.pred.dz_re;
                    j.dz_im = sh.pred.dz_im;
                    code = 1;
                }
            }
            sh.verdict = 4 * (e + 1) + code;
            publish_seq(&sh.seed_seq, e + 1);
            if (code == 1) publish_seq(&sh.job_seq, e + 1);
        }
    };
    if (role == kRoleControl) make_seed(0);
    int e_done = 0;
    bool cancel = false;  // wave 0: the current epoch was seeded before a lock test that failed
    // One epoch loop per role: the roles never share a control-flow path, so the waits the compiler
    // places for one role's memory operations are not charged to another (a merged loop made the
    // control wave wait for the producers' sample loads it never issued).
    if (role == kRoleReplay) {
        for (int e = 0;; e++) {
            FJob job;
                // ---- derive: the phasors of the seeded epoch ----
                // In state 4 the loop publishes its early values (SpecArgs) once the carrier filter ran,
                // before the DLL, update_tracking_vars and the seed.  With whole-epoch slots the next
                // epoch's phasors are then derived from them — the step exactly, the remainder phase for
                // an unchanged epoch length — and replayed speculatively; the seed, when it comes, confirms
                // both floats (the job is published mid-replay) or the slots are cleared and the epoch is
                // derived again from the seed.  With the slot ring only the step's part is done early.
                bool spec = false;
                SpecArgs sp{};
                while (__hip_atomic_load(&sh.seed_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < e + 1) {
                    if (__hip_atomic_load(&sh.step_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= e + 1) {
                        sp.step_d = __builtin_bit_cast(double, uni64(__builtin_bit_cast(uint64_t, sh.spec.step_d)));
                        sp.rate = __builtin_bit_cast(double, uni64(__builtin_bit_cast(uint64_t, sh.spec.rate)));
                        sp.if_num = static_cast<int64_t>(uni64(static_cast<uint64_t>(sh.spec.if_num)));
                        sp.rem_prev = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sh.spec.rem_prev)));
                        sp.n_pred = __builtin_amdgcn_readfirstlane(sh.spec.n_pred);
                        spec = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(GNSSHIP_POLL_SLEEP);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                GNSSHIP_FSTAMP(e, 0);
    #ifdef GNSSHIP_CORR_PROFILE
                if (lane == 0) g_fprof_epoch = e;
    #endif
                f2 zinit = f2{0.0f, 0.0f}, inc = f2{1.0f, 0.0f}, dz = f2{1.0f, 0.0f};
                float step_pre = 0.0f;
                bool published = false;
                float xl = 0.0f;
                if (spec) step_pre = static_cast<float>(sp.step_d + if_step);  // make_seed's j.step
                if (SRING && spec) derive_step(step_pre, inc, dz);
                if (!SRING && spec) {
                    // make_seed's j.rem_carr after update_tracking_vars and epoch_consume, for n = n_pred
                    float rem_pred = carr_rem_next(sp.rem_prev, carr_advance(sp.step_d, sp.rate, static_cast<double>(sp.n_pred)));
                    if (has_if) {
                        const int64_t ifn = (sp.if_num + kp.if_mod * static_cast<int64_t>(sp.n_pred)) % kp.fs_int;
                        const double ifc = static_cast<double>(ifn) / static_cast<double>(kp.fs_int);
                        rem_pred = static_cast<float>(fmod_2pi(static_cast<double>(rem_pred) + kTwoPi * ifc));
                    }
                    derive_all(step_pre, rem_pred, lane, inc, dz, zinit);
                    GNSSHIP_FSTAMP(e, 35);
                    GNSSHIP_PROBE(GNSSHIP_DELAY_REPLAY);
                    // the prediction goes to wave 0, which confirms it when it makes the seed (and then
                    // publishes the job itself); the replay runs without looking at the seed
                    if (lane == 0) {
                        sh.pred.rem = rem_pred;
                        sh.pred.step = step_pre;
                        sh.pred.dz_re = dz.x;
                        sh.pred.dz_im = dz.y;
                        publish_seq(&sh.pred_seq, e + 1);
                    }
                    xl = (lane & 1) ? zinit.y : zinit.x;
                    if (lane < 2 * kAvxLanes) xl = fast_replay<G, false>(xl, dz.x, (lane & 1) ? dz.y : -dz.y, M, S, tail, Zs, rs, lane);
                    GNSSHIP_FSTAMP(e, 34);
                    wait_seq(&sh.seed_seq, e + 1);
                    const int v = __builtin_amdgcn_readfirstlane(sh.verdict);
                    int status = (v >> 2) == e + 1 ? (v & 3) : 3;
                    if (status == 3) {  // the seed was made before the prediction was published: compare here
                        const FJob sd = uniform_job(sh.job);
                        status = 2;
                        if (sd.runnable && __builtin_bit_cast(uint32_t, sd.step) == __builtin_bit_cast(uint32_t, step_pre) &&
                            __builtin_bit_cast(uint32_t, sd.rem_carr) == __builtin_bit_cast(uint32_t, rem_pred)) {
                            if (lane == 0) {
                                sh.job.dz_re = dz.x;
                                sh.job.dz_im = dz.y;
                                publish_seq(&sh.job_seq, e + 1);
                            }
                            status = 1;
                        }
                    }
                    GNSSHIP_FVAL(e, 78, static_cast<unsigned long long>(status));  // profiling: 1 confirmed, 2 refuted
                    if (status == 1) {
                        published = true;
                    } else {  // mispredicted (or the end of the run): the slots are cleared before the job goes out
                        for (int i = lane; i < S * kAvxLanes; i += kWave) Zs[i] = kSlotEmpty;
                    }
                    GNSSHIP_FSTAMP(e, 36);
                }
                if (!published) {
                    wait_seq(&sh.seed_seq, e + 1);
                    const FJob sd = uniform_job(sh.job);
                    if (sd.runnable) {
                        // (cos rem, −sin rem) and (cos −step, sin −step) (cpu_multicorrelator_real_codes.cc:115,123),
                        // each glibc's cosf / sinf (glibc_sincosf.h)
                        if (!(spec && __builtin_bit_cast(uint32_t, sd.step) == __builtin_bit_cast(uint32_t, step_pre))) derive_step(sd.step, inc, dz);
                        zinit = derive_chains(sd.rem_carr, inc, lane);
                        if (lane == 0) {
                            sh.job.dz_re = dz.x;
                            sh.job.dz_im = dz.y;
                        }
                    }
                    if (lane == 0) publish_seq(&sh.job_seq, e + 1);
                    if (!sd.runnable) break;
                }
                GNSSHIP_FSTAMP(e, 1);
                GNSSHIP_FCLK(e, 12);
                job = uniform_job(sh.job);
                if (!published) {
                    xl = (lane & 1) ? zinit.y : zinit.x;
                    if (lane < 2 * kAvxLanes) xl = fast_replay<G, SRING>(xl, job.dz_re, (lane & 1) ? job.dz_im : -job.dz_im, M, S, tail, Zs, rs, lane);
                }
                if (tail > 0) {  // the serial tail from normalise(z_0) after the loop (:294-308)
                    const i4v span = sample_span<FMT>(samples, job.off, N);
                    const f2 zl = f2{__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xl), 0)),
                        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xl), 1))};
                    if (lane == 0) {
                        f2 p = normalise_avx(zl);
                        for (int j = 0; j < tail; j++) {
                            tailz[j] = p;
                            p = cmul_exact(p, inc);
                        }
                    }
                    if (job.in_margin)
                        fast_tail_products<FMT, NT, DATA, true>(job, span, c0, c1, L, tailz, lane, sh.tailp);
                    else
                        fast_tail_products<FMT, NT, DATA, false>(job, span, c0, c1, L, tailz, lane, sh.tailp);
                    if (lane == 0) publish_seq(&sh.tail_seq, e + 1);
                }
                GNSSHIP_FSTAMP(e, 2);
                GNSSHIP_FCLK(e, 13);
        }
    } else if (role == kRoleProducer) {
        f2 xa[G < 8 ? G : 8];
        float cv[G][NTT];
        for (int e = 0;; e++) {
            const int gbase = e * n_groups;  // the epoch's first product-group tag - 1
            wait_seq(&sh.job_seq, e + 1);
            const FJob job = uniform_job(sh.job);
            if (!job.runnable) break;
            const i4v span = sample_span<FMT>(samples, job.off, N);
            if (job.in_margin)
                fast_produce<FMT, NT, DATA, true, G, kFWaves>(job, span, c0, c1, L, Zs, rs, Pp, rg, ready, sh.acc_groups, gbase, lane, pw, e, xa, cv);
            else
                fast_produce<FMT, NT, DATA, false, G, kFWaves>(job, span, c0, c1, L, Zs, rs, Pp, rg, ready, sh.acc_groups, gbase, lane, pw, e, xa, cv);
            if (pw < 2) GNSSHIP_FSTAMP(e, 3 + pw);  // 3, 4: producers 0 and 1 done
            if (pw == 0) {
                // cn0_and_tracking_lock_status (:972-1029) on the LDS copy of its members, beside the loop update
                wait_seq(&sh.pre_seq, e + 1);
                const double coh = sh.coh;
                if (lane == 0) {
                    GNSSHIP_TRK_LOOP_STAMP(8);
                    sh.locked = (coh > 0.0 && !lock_status(k, sc, coh)) ? 0 : 1;
                    GNSSHIP_TRK_LOOP_STAMP(26);
                    publish_seq(&sh.lock_seq, e + 1);
                }
            }
        }
    } else if (role == kRoleAccum) {
        for (int e = 0;; e++) {
            const int gbase = e * n_groups;  // the epoch's first product-group tag - 1
            wait_seq(&sh.job_seq, e + 1);
            const FJob job = uniform_job(sh.job);
            if (!job.runnable) break;
            // ---- the epoch's taps in u_avx's order ----
            {
                constexpr int NS = acc_slots<NTT>();
                float acc[NS];
                GNSSHIP_FSTAMP(e, 27);
                fast_accumulate<NTT, G>(Pp, rg, ready, &sh.acc_groups[pw], gbase, S, lane, pw, acc, e);
                GNSSHIP_FSTAMP(e, 5);
                const int r = lane >> 4;
    #pragma unroll
                for (int kk = 0; kk < NS; kk++) acc[kk] = avx_chain_sum(acc[kk]);
                if (job.tail > 0) {  // the serial tail, sample by sample (:298-308)
                    wait_seq(&sh.tail_seq, e + 1);
                    for (int j = 0; j < job.tail; j++) {
    #pragma unroll
                        for (int kk = 0; kk < NS; kk++) {
                            const int sl = min(acc_slot<NTT>(pw, r, kk), 2 * NTT - 1);
                            const f2 tv = sh.tailp[j][sl >> 1];
                            acc[kk] = acc[kk] + ((sl & 1) ? tv.y : tv.x);
                        }
                    }
                }
                if ((lane & 15) == 0) {
    #pragma unroll
                    for (int kk = 0; kk < NS; kk++) {
                        const int sl = acc_slot<NTT>(pw, r, kk);  // slot 2·tap + component
                        if (sl < 2 * NTT) {
                            const int tap = sl >> 1;
                            const int o = (DATA && tap == NT) ? 2 * kMaxTaps : 2 * tap;
                            sh.taps[e & 1][o + (sl & 1)] = acc[kk];
                        }
                    }
                }
                if (lane == 0) lds_release_store(&sh.taps_seq[pw], e + 1);
                if (pre_disc && pw < 2) {
                    // the discriminators of this epoch from its taps, as epoch_pre's save_correlation_results
                    // (0 + 1·tap) and run_dll_pll form them (used by the control wave in state 4 only)
#pragma unroll
                    for (int a = 0; a < NA; a++) wait_seq(&sh.taps_seq[a], e + 1);
                    const float* tp = sh.taps[e & 1];
                    const int eo = k.veml ? 2 : 0;
                    auto own = [&](int i) { return __fadd_rn(0.0f, __fmul_rn(1.0f, tp[i])); };
                    if (pw == 0 || NA == 1) {
                        const double v = pll_error_hz(k.track_pilot ? 0 : 1, own(eo + 2), own(eo + 3));
                        if (lane == 0) {
                            sh.pre_pll[e & 1] = v;
                            publish_seq(&sh.pll_seq, e + 1);
                        }
                    }
                    if (pw == 1 || NA == 1) {
                        const float ve[2] = {k.veml ? own(0) : 0.0f, k.veml ? own(1) : 0.0f};
                        const float ee[2] = {own(eo), own(eo + 1)};
                        const float ll[2] = {own(eo + 4), own(eo + 5)};
                        const float vl[2] = {k.veml ? own(8) : 0.0f, k.veml ? own(9) : 0.0f};
                        const double v = dll_error_chips(k, ve, ee, ll, vl, k.conf.early_late_space_chips);
                        if (lane == 0) {
                            sh.pre_dll[e & 1] = v;
                            publish_seq(&sh.dll_seq, e + 1);
                        }
                    }
                }
            }
            GNSSHIP_FSTAMP(e, 6);
        }
    } else {
        for (int e = 0;; e++) {
            const int gbase = e * n_groups;  // the epoch's first product-group tag - 1
            wait_seq(&sh.job_seq, e + 1);
            const FJob job = uniform_job(sh.job);
            if (!job.runnable) break;
#pragma unroll
            for (int a = 0; a < NA; a++) wait_seq(&sh.taps_seq[a], e + 1);  // the accumulator waves' taps of this epoch
            GNSSHIP_FCLK(e, 14);
            if (cancel) {
                // the epoch seeded speculatively before the last lock test failed: the channel stopped
                // there (state 0), so nothing of this epoch is kept — no lock test, no record — and
                // the seed for the next one says "not runnable", which ends every wave's loop
                cancel = false;
                if (lane == 0) {
                    sh.coh = 0.0;
                    publish_seq(&sh.pre_seq, e + 1);
                }
                make_seed(e + 1);
                continue;
            }
            {
                const float* taps = sh.taps[e & 1];
                GNSSHIP_FSTAMP(e, 16);
                GNSSHIP_PROBE(GNSSHIP_DELAY_LOOP);
                const float* pdata = DATA ? taps + 2 * kMaxTaps : taps;
                gnsship_trk_epoch r{};
                r.flags = 8;
                gnsship_trk_dump_record* dr = dump ? &sh.drec : nullptr;
                const uint64_t es = rc.epoch_start;  // this epoch's first sample
                const double coh = epoch_pre(kp, rc, taps, pdata, r, nullptr, dr);
                GNSSHIP_FSTAMP(e, 17);
                // hand the prompt to the lock detectors (producer 0; coh 0: no lock test this epoch)
                if (lane == 0) {
                    sc.p[0] = rc.p[0];
                    sc.p[1] = rc.p[1];
                    sc.pull_in = rc.pull_in;
                    sh.coh = coh;
                    publish_seq(&sh.pre_seq, e + 1);
                }
                GNSSHIP_FSTAMP(e, 18);
                bool seeded = false;
                if (coh > 0.0) {  // the loop runs speculatively beside the lock test
                    // what the record shows if the test fails (the channel then stops: nothing else of the
                    // loop's output is ever read)
                    const double k_rcs = rc.rem_code_phase_samples, k_acc = rc.acc_carrier_phase_rad, k_dop = rc.carrier_doppler_hz;
                    const double k_cf = rc.code_freq_chips, k_rcc = rc.rem_code_phase_chips;
                    const float k_rem = rc.rem_carr_phase_rad;
                    const int32_t k_len = rc.current_prn_length_samples;
                    // state 4: the next epoch's carrier step to wave 1 once the carrier filter ran (the seed
                    // repeats it; wave 1 checks they agree)
                    auto early_step = [&](double dop) {
                        if (rc.state == 4 && lane == 0) {
                            sh.spec.step_d = div_fs(kp, kTwoPi * dop);  // update_tracking_vars' carrier_phase_step_rad
                            sh.spec.rate = rc.carrier_phase_rate_step_rad;
                            sh.spec.if_num = rc.if_num;
                            sh.spec.rem_prev = rc.rem_carr_phase_rad;
                            sh.spec.n_pred = rc.current_prn_length_samples;
                            publish_seq(&sh.step_seq, e + 2);
                        }
                        GNSSHIP_FSTAMP(e, 32);
                    };
                    // the accumulator waves' discriminators (state 4 with the run's spacing; epoch_pre
                    // left E / P / L equal to 0 + the taps, as they formed them)
                    PreDisc pd{0.0, 0.0, 0};
                    if (pre_disc && r.state == 4 && __builtin_bit_cast(uint32_t, unif(rc.spc)) == __builtin_bit_cast(uint32_t, k.conf.early_late_space_chips)) {
                        wait_seq(&sh.pll_seq, e + 1);
                        wait_seq(&sh.dll_seq, e + 1);
                        pd.pll = sh.pre_pll[e & 1];
                        pd.dll = sh.pre_dll[e & 1];
                        pd.ok = 3;
                    }
                    epoch_loop(kp, rc, nullptr, early_step, &pd);
                    // State 4: epoch_post cannot change what the next epoch's correlation needs (the
                    // channel stays runnable — 4, or 3 for extended integration — on the same taps), so
                    // the next epoch is seeded now, before the lock test's outcome, and wave 1 derives
                    // it while this epoch finishes.  A failed test (the channel stops) cancels it.
                    const uint64_t k_nir = rc.nitems_read;
                    const int64_t k_ifn = rc.if_num;
                    const double k_ifc = rc.if_cyc;
                    if (rc.state == 4) {
                        epoch_consume(kp, rc);
                        make_seed(e + 1);
                        GNSSHIP_FSTAMP(e, 33);
                        rc.epoch_start = es;  // epoch_post and the record still describe this epoch
                        seeded = true;
                    }
                    wait_seq(&sh.lock_seq, e + 1);
                    GNSSHIP_FSTAMP(e, 19);
                    const bool locked = sh.locked != 0;
                    if (!locked) {  // the reference runs the loop only on a passed lock test
                        rc.rem_code_phase_samples = k_rcs;
                        rc.acc_carrier_phase_rad = k_acc;
                        rc.carrier_doppler_hz = k_dop;
                        rc.code_freq_chips = k_cf;
                        rc.rem_code_phase_chips = k_rcc;
                        rc.rem_carr_phase_rad = k_rem;
                        rc.current_prn_length_samples = k_len;
                        rc.nitems_read = k_nir;
                        rc.if_num = k_ifn;
                        rc.if_cyc = k_ifc;
                        cancel = seeded;
                    }
                    epoch_post(kp, rc, taps, pdata, r, locked, dr);
                }
                GNSSHIP_FSTAMP(e, 24);
                epoch_finish(kp, rc, r, !seeded);  // (a stopped channel consumes nothing either way)
                if (!seeded)
                    make_seed(e + 1);  // wave 1 derives the next epoch while the records go out
                else if (!cancel)
                    rc.epoch_start = seed_start;  // the next epoch, as make_seed left it
                GNSSHIP_FSTAMP(e, 25);
                if (lane == 0) {
                    const size_t slot = static_cast<size_t>(e) * n_chans + ch;
                    if (rec) rec[slot] = r;
                    if (dump && (r.flags & 16)) dump[slot] = sh.drec;
                    if (trace) {
                        gnsship_trk_corr_trace tr{};
                        tr.sample_counter = es;
                        tr.n_samples = N;
                        tr.n_taps = NT;
                        tr.rem_carrier_phase_rad = job.rem_carr;
                        tr.phase_step_rad = job.step;
                        tr.rem_code_phase_samples = job.rem_code;
                        tr.code_phase_step_samples = job.code_step;
                        for (int t = 0; t < 5; t++) tr.shifts[t] = job.shifts[t];
                        for (int t = 0; t < 10; t++) tr.taps[t] = t < 2 * NT ? taps[t] : 0.0f;
                        tr.data_prompt[0] = DATA ? pdata[0] : 0.0f;
                        tr.data_prompt[1] = DATA ? pdata[1] : 0.0f;
                        trace[slot] = tr;
                    }
                }
                e_done = e + 1;
                GNSSHIP_FSTAMP(e, 7);
                GNSSHIP_FCLK(e, 15);
            }
        }
    }
    if (role == kRoleControl && lane == 0) {
        rchan_store(rc, sc);
        sc.ran = 0;
        if (e_done > 0) atomicAdd(ran_count + e_done - 1, 1);  // rounds_done = the longest channel's epochs
    }
    __syncthreads();
#ifdef GNSSHIP_CORR_PROFILE
    if (g_trkf_prof)
        for (int i = tid; i < kFProfEpochs * kFProfSlots; i += kFThreads) g_trkf_prof[static_cast<size_t>(blockIdx.x) * kFProfEpochs * kFProfSlots + i] = g_fprof_lds[i];
#endif
    {
        const int* src = reinterpret_cast<const int*>(&sc);
        int* dst = reinterpret_cast<int*>(chans + ch);
        for (int i = tid; i < static_cast<int>(sizeof(TrkChannel) / 4); i += kFThreads) dst[i] = src[i];
    }
}

}  // namespace

#ifdef GNSSHIP_CORR_PROFILE
}  // namespace gnsship
extern "C" int gnsship_debug_trk_fast_profile(void* dev_buf)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(gnsship::g_trkf_prof), &dev_buf, sizeof(void*)) == hipSuccess ? 0 : -3;
}
namespace gnsship {
#endif

// The LDS plan of a run: task length G (iterations per phasor slot), the phasor-slot ring (rs tasks;
// rs = S: one slot per task of the epoch) and the product ring (rg groups of 4 tasks; rg = n_groups:
// the whole epoch).  G = 8 (half the slot stores and asm-block boundaries of G = 4 on the replay
// chain, C2 profiling build: 8.24 -> 8.00 us per epoch); the whole epoch's slots and products when
// they fit, otherwise a product ring of as many groups as fit (at least 2), with the slots in a ring
// of 16 groups when the whole epoch's slots leave too little room.  `bytes` 0: no plan fits.
// Compute units of the current device (the "more channels than CUs" switch), queried once per device.
static int device_cus()
{
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int n = 0;
        cache[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) ? n : 256;
    }
    return cache[dev];
}

// More channels than CUs: the throughput form (fast_waves<true>, two workgroups per CU, each with
// half the LDS budget).  GNSSHIP_TRK_THRU=0/1 forces either form (A/B, tests).
static bool fast_thru(int n_chans)
{
    if (const char* env = std::getenv("GNSSHIP_TRK_THRU")) return env[0] == '1';
    return n_chans > device_cus();
}

struct FastPlan {
    size_t bytes = 0;
    int G = 8, rs = 0, rg = 0;
};
#ifndef GNSSHIP_FAST_G
#define GNSSHIP_FAST_G 8
#endif
constexpr int kFastG = GNSSHIP_FAST_G;
constexpr int kFastSlotRingGroups = 16;
constexpr int kFastMinRingGroups = 4;
constexpr size_t kFastMaxSlotBytes = 48 * 1024;
static FastPlan fast_plan(const TrkParams& p, int code_cap_floats, int n_chans)
{
    FastPlan f;
    const int N = static_cast<int>(p.conf.vector_length);
    const int M = N / kAvxLanes;
    const int G = kFastG;
    const int S = std::max(1, (M + G - 1) / G);
    const int n_groups = (S + 3) / 4;
    const int ntt = p.n_taps + (p.jobs_per_channel > 1 ? 1 : 0);
    const size_t codes = static_cast<size_t>(p.jobs_per_channel > 1 ? 2 : 1) * code_cap_floats * sizeof(float);
    const size_t slot_b = kAvxLanes * sizeof(uint64_t);
    // a group's products (ProdLayout: 4 tasks of G iterations × 2·ntt slots × 16 chains, each task
    // padded by 16 floats) and its flag
    const size_t group_b = static_cast<size_t>(2 * ntt) * kAvxLanes * (4 * G + 4) * sizeof(float) + 2 * sizeof(int32_t);  // ProdLayout + flags
    // more channels than CUs: two workgroups per CU share its LDS
    size_t budget = fast_thru(n_chans) ? 72 * 1024 : kTrkPersistMaxLds;
    if (const char* env = std::getenv("GNSSHIP_TRK_FAST_LDS"))  // tests: a smaller budget forces the rings
        budget = std::min(budget, static_cast<size_t>(std::atol(env)) * 1024);
    auto fit = [&](int rs) -> int {  // product groups that fit beside `rs` slots (0: fewer than 2)
        const size_t used = codes + static_cast<size_t>(rs) * slot_b;
        if (used >= budget) return 0;
        const int rg = static_cast<int>(std::min<size_t>((budget - used) / group_b, static_cast<size_t>(n_groups)));
        return rg >= std::min(2, n_groups) ? rg : 0;
    };
    // whole-epoch slots only while they stay within the first 48 KiB of LDS (the replay's slot stores
    // address them through M0[15:0], beside the static LDS)
    int rs = S, rg = static_cast<size_t>(S) * slot_b <= kFastMaxSlotBytes ? fit(S) : 0;
    // the slot ring must hold at least 4 tasks per product group (a producer passed the ring's
    // back-pressure before it polls a slot, so the slot's previous lap is consumed).  It is used only
    // when the whole epoch's slots leave fewer than kFastMinRingGroups product groups: with every
    // slot in LDS the replay never waits and may run speculatively (ahead of the seed).
    if (rg < std::min(n_groups, kFastMinRingGroups) && S > 4 * kFastSlotRingGroups) {
        const int rg2 = std::min(fit(4 * kFastSlotRingGroups), kFastSlotRingGroups);
        if (rg2 > rg) {
            rs = 4 * kFastSlotRingGroups;
            rg = rg2;
        }
    }
    if (rg == 0) return f;
    f.G = G;
    f.rs = rs;
    f.rg = rg;
    f.bytes = codes + static_cast<size_t>(rs) * slot_b + static_cast<size_t>(rg) * group_b;
    return f;
}

bool trk_fast_thru(int n_chans) { return fast_thru(n_chans); }
int trk_device_cus() { return device_cus(); }

bool trk_fast_supported(const TrkParams& p, int code_cap_floats, int n_chans)
{
    if (!trk_persist_supports(p) || p.conf.rotator != GNSSHIP_ROTATOR_AVX || p.conf.high_dyn) return false;
    if (p.n_taps + (p.jobs_per_channel > 1 ? 1 : 0) > 2 * 4) return false;  // the accumulator's two taps per lane row
    if (const char* env = std::getenv("GNSSHIP_TRK_FAST")) {  // A/B against trk_persist.hip
        if (env[0] == '0') return false;
        if (env[0] == '1') return fast_plan(p, code_cap_floats, n_chans).bytes > 0;
    }
    // every channel count: with more channels than CUs the throughput form (fast_thru), which keeps
    // u_avx's accumulation order as the latency form does (trk_persist.hip's tree sums do not)
    return fast_plan(p, code_cap_floats, n_chans).bytes > 0;
}

hipError_t launch_trk_fast(const TrkParams* params_dev, const TrkParams& params, TrkChannel* chans, int n_chans, const CodeDesc* codes, int n_codes,
    int code_cap_floats, const void* samples, int fmt, uint64_t buf_first, int64_t buf_len, int max_rounds, gnsship_trk_epoch* rec,
    gnsship_trk_dump_record* dump, gnsship_trk_corr_trace* trace, int* ran_count, hipStream_t stream)
{
    const FastPlan f = fast_plan(params, code_cap_floats, n_chans);
    if (f.bytes == 0) return hipErrorInvalidValue;
    const int N = static_cast<int>(params.conf.vector_length);
    const int S = std::max(1, (N / kAvxLanes + f.G - 1) / f.G);
    const bool sring = f.rs < S;
    const bool data = params.jobs_per_channel > 1;
    const bool thru = fast_thru(n_chans);
    const int nt = params.n_taps;
    // the form: throughput (more channels than CUs), long epochs (more producer waves), latency
    const int form = thru ? 1 : (N >= kLongEpoch ? 2 : 0);
    const int waves = form == 1 ? GNSSHIP_THRU_WAVES : form == 2 ? kFWavesLong : kFWaves;
    dim3 grid(n_chans), block(waves * kWave);
#define GNSSHIP_FAST(F, NTV, DV, SR)                                                                                                               \
    do {                                                                                                                                         \
        auto kfn = form == 1 ? trk_fast_kernel<F, NTV, DV, kFastG, true, SR, GNSSHIP_THRU_WAVES>                                                  \
                             : form == 2 ? trk_fast_kernel<F, NTV, DV, kFastG, false, SR, kFWavesLong> : trk_fast_kernel<F, NTV, DV, kFastG, false, SR, kFWaves>; \
        hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(f.bytes)); \
        if (e0 != hipSuccess) return e0;                                                                                                         \
        hipLaunchKernelGGL(kfn, grid, block, f.bytes, stream, params_dev, chans, codes, n_codes, samples, buf_first, buf_len, max_rounds, n_chans, \
            code_cap_floats, f.rs, f.rg, rec, dump, trace, ran_count);                                                                           \
    } while (0)
#define GNSSHIP_FAST_R(F, NTV, DV)                        \
    do {                                                  \
        if (sring) GNSSHIP_FAST(F, NTV, DV, true);        \
        else GNSSHIP_FAST(F, NTV, DV, false);             \
    } while (0)
#define GNSSHIP_FAST_F(F)                                    \
    do {                                                     \
        if (nt == 3 && !data) GNSSHIP_FAST_R(F, 3, false);   \
        else if (nt == 5 && !data) GNSSHIP_FAST_R(F, 5, false); \
        else if (nt == 5 && data) GNSSHIP_FAST_R(F, 5, true); \
        else return hipErrorInvalidValue;                    \
    } while (0)
    switch (fmt) {
    case GNSSHIP_FMT_CF32: GNSSHIP_FAST_F(GNSSHIP_FMT_CF32); break;
    case GNSSHIP_FMT_CI16: GNSSHIP_FAST_F(GNSSHIP_FMT_CI16); break;
    case GNSSHIP_FMT_CI8: GNSSHIP_FAST_F(GNSSHIP_FMT_CI8); break;
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_FAST_F
#undef GNSSHIP_FAST_R
#undef GNSSHIP_FAST
    return hipGetLastError();
}

}  // namespace gnsship
