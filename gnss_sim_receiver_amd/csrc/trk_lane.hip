// trk_lane.hip — the AVX closed loop's throughput form: one 16-lane row of a wave per channel.
//
// volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_u_avx (…rotator_dot_prod_32fc_xn.h:155-316) keeps
// sixteen phasor chains z_l (four __m256 of four complex lanes) and, per tap, sixteen accumulators:
// chain l takes the samples 16m + l, and each accumulator is a serial float sum over m.  A wave holds
// four such AVX register files: lane 16·r + l runs chain l of the wave's channel r exactly as the
// reference's AVX lane does — the sample times z_l (_mm256_complexmul_ps rounding), z_l·dz
// (renormalised after iteration m ≡ 0 mod 64), the taps' code products and the serial adds — so every
// tap is the reference's own float sum with no cross-lane traffic inside the epoch.  The chain
// combination (:279-291) is a DPP reduction inside the row, the N mod 16 tail (:294-308) runs on the
// row's lane 0, and then the row's lane 0 runs the loop update (trk_loop.h: epoch_pre, lock_status,
// epoch_loop, epoch_post, epoch_finish) on the channel's LDS-resident state, in the reference's order
// (the lock test, then the loop filters only when it passed, dll_pll_veml_tracking.cc:1971-2028).
//
// An epoch takes M = N/16 dependent iterations per chain — the reference's own single-core latency —
// so this form is for many channels at once: workgroups of GNSSHIP_LANE_WAVES waves (4 channels per
// wave), several waves per SIMD, channels beyond the resident workgroups in successive generations.
// The code replicas are held as sign bits in LDS (every chip ±1, checked when the code is set —
// gnsship_code_set): the product a·c of the sample product with a ±1 chip is a sign flip, exact, so the
// taps are bit-identical to the float replica's.  The latency form for few channels is trk_fast.hip.
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <type_traits>

#include "corr_device.h"
#include "trk_engine.h"
#include "trk_loop.h"

#pragma clang fp contract(off)

namespace gnsship {
namespace {

#ifndef GNSSHIP_LANE_WAVES
#define GNSSHIP_LANE_WAVES 4
#endif
#ifndef GNSSHIP_LANE_OCC
#define GNSSHIP_LANE_OCC 4  // waves per SIMD the register budget is sized for (512 / OCC VGPRs each)
#endif
#ifndef GNSSHIP_LANE_BLOCK
#define GNSSHIP_LANE_BLOCK 4  // iterations per block with three taps (4: no spills in the loop update at 128 VGPRs)
#endif
constexpr int kLRows = kWave / kAvxLanes;  // channels per wave
constexpr int kLWaves = GNSSHIP_LANE_WAVES;
constexpr int kLChans = kLWaves * kLRows;  // channels per workgroup
constexpr int kLThreads = kLWaves * kWave;
// iterations per block: their samples are in flight and their chips looked up together (kB divides 64)
template <int NTT>
constexpr int lane_block() { return NTT > 3 ? 4 : GNSSHIP_LANE_BLOCK; }

// Sign-bit replica of a padded code (engine.h padded_code_quads): bit p of the table is chip
// p − kCodeMargin < 0 (p over the replica and its wrapped margins).
__host__ __device__ constexpr int lane_code_words(int code_cap_floats) { return (code_cap_floats + 31) / 32; }

// The chip (±1.0f) the resampler picks for tap shift `sh` at sample n (sn = step·(float)n): the chip
// index as code_at (corr_device.h) forms it, looked up in the sign-bit replica.
static_assert(kCodeMargin == 32, "chip i sits at bit i & 31 of word (i >> 5) + 1");
template <bool IN_MARGIN>
__device__ __forceinline__ float code_chip(const uint32_t* bits, int L, float sn, float sh, float rem)
{
    int i = cvt_floor_i32(__fsub_rn(__fadd_rn(sn, sh), rem));
    if constexpr (!IN_MARGIN) i = wrap_index(i, L);
    const uint32_t w = bits[(i >> 5) + 1];
    return __builtin_bit_cast(float, ((w >> (i & 31)) << 31) | 0x3f800000u);
}

// acc + a·c for a chip c = ±1: a·c is exact (a or −a), so the fused form rounds exactly as the
// reference's product-then-add (_mm256_mul_ps, _mm256_add_ps, :252-260)
__device__ __forceinline__ f2 add_chip(f2 acc, f2 a, float c) { return __builtin_elementwise_fma(a, f2{c, c}, acc); }

// Build the sign-bit replica of code `cd` at dst (the whole wave, one 64-chip ballot per step).
__device__ void stage_code_bits(uint32_t* dst, const CodeDesc& cd, int words, int lane)
{
    const int P = cd.len + 2 * kCodeMargin;
    for (int base = 0; base < 32 * words; base += kWave) {
        const int i = base + lane;
        const float v = i < P ? cd.ptr[i - kCodeMargin] : 1.0f;
        const unsigned long long m = __ballot(v < 0.0f);
        if (lane == 0) {
            dst[base >> 5] = static_cast<uint32_t>(m);
            if ((base >> 5) + 1 < words) dst[(base >> 5) + 1] = static_cast<uint32_t>(m >> 32);
        }
    }
}

// The epoch's correlator arguments for the lane's channel (do_correlation_step, :1037-1062, and
// Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler, cpu_multicorrelator_real_
// codes.cc:103-126), evaluated by every lane of the row.
struct LJob {
    int off;  // the epoch's first sample, relative to the buffer
    int in_margin;
    float rem_code, code_step, shifts[kMaxTaps];
    float rem_carr, step;  // as passed (trace)
    f2 inc, dz, z;         // phase_inc, dz = normalise(inc^16), this lane's chain start phase·inc^l
};

template <int NT>
__device__ __forceinline__ LJob lane_job(const TrkParams& k, const TrkChannel& c, uint64_t buf_first, int L, int l)
{
    LJob j;
    const float spcf = static_cast<float>(k.code_samples_per_chip);
    j.off = static_cast<int>(c.nitems_read - buf_first);
    j.rem_code = __fmul_rn(static_cast<float>(c.rem_code_phase_chips), spcf);
    j.code_step = __fmul_rn(static_cast<float>(c.code_phase_step_chips), spcf);
    const float* sh = c.narrow ? k.shifts_n : k.shifts;
    float smin = 0.0f, smax = 0.0f;
#pragma unroll
    for (int t = 0; t < kMaxTaps; t++) {
        j.shifts[t] = t < NT ? sh[t] : 0.0f;
        smin = fminf(smin, j.shifts[t]);
        smax = fmaxf(smax, j.shifts[t]);
    }
    const int N = static_cast<int>(k.conf.vector_length);
    const double span = static_cast<double>(j.code_step) * static_cast<double>(N > 0 ? N - 1 : 0);
    const double lo = fmin(0.0, span) + smin - j.rem_code - 2.0;
    const double hi = fmax(0.0, span) + smax - j.rem_code + 2.0;
    j.in_margin = (isfinite(lo) && isfinite(hi) && lo >= -kCodeMargin && hi < static_cast<double>(L + kCodeMargin)) ? 1 : 0;
    // phase = (cos rem, −sin rem) (:115), phase_inc = (cos −step, sin −step) (:123), glibc's sincosf
    j.rem_carr = corr_rem_carr(k, c);
    j.step = corr_phase_step(k, c);
    float sr, cr, ss, cs;
    glibc_sincosf(j.rem_carr, &sr, &cr);
    glibc_sincosf(-j.step, &ss, &cs);
    j.inc = f2{cs, ss};
    // phase_vec[l] = phase·inc^l (:195-199); dz = inc^16 by four squarings, normalised (:206-218)
    f2 w = f2{cr, -sr}, z = w, d = j.inc;
#pragma unroll
    for (int i = 0; i < kAvxLanes - 1; i++) {
        w = cmul_exact_sc(w, j.inc);
        if (i < 4) d = cmul_exact_sc(d, d);
        z = i + 1 == l ? w : z;
    }
    j.dz = normalise_avx(d);
    j.z = z;
    return j;
}

// The u_avx main loop (:220-275) on this lane's chain: M iterations, sample 16m + l at iteration m.
template <int FMT, int NT, bool DATA, bool IN_MARGIN>
__device__ __forceinline__ void lane_correlate(i4v span, const LJob& j, int M, int l, const uint32_t* b0, const uint32_t* b1, int L, f2& z,
    f2 (&acc)[NT + (DATA ? 1 : 0)])
{
    constexpr int SB = sample_bytes<FMT>();
    constexpr int NTT = NT + (DATA ? 1 : 0);
    constexpr int kB = lane_block<NTT>();
    const int v0 = (j.off + l) * SB;
    constexpr int kStride = kAvxLanes * SB;
    f2 xa[kB], xb[kB];
#pragma unroll
    for (int u = 0; u < kB; u++) xa[u] = load_sample<FMT>(span, v0 + u * kStride, 0);
    float fn = static_cast<float>(l);  // (float)n for n = 16m + l, exact (n < 2^24)
    // the chips of a block's iterations, looked up before its arithmetic (the LDS reads overlap)
    float cv[kB][NTT];
    auto block_chips = [&](int cnt) __attribute__((always_inline)) {
        float f = fn;
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const float sn = __fmul_rn(j.code_step, u < cnt ? f : fn);
#pragma unroll
            for (int t = 0; t < NT; t++) cv[u][t] = code_chip<IN_MARGIN>(b0, L, sn, j.shifts[t], j.rem_code);
            if constexpr (DATA) cv[u][NT] = code_chip<IN_MARGIN>(b1, L, sn, 0.0f, j.rem_code);
            f += static_cast<float>(kAvxLanes);
        }
        fn = f;
    };
    // one iteration; RENORM: "Force the rotators back onto the unit circle" after it (m ≡ 0 mod 64, :266-272)
    auto iteration = [&](f2 x, const float (&c)[NTT], auto renorm) __attribute__((always_inline)) {
        const f2 a = cmul_exact_pk(x, z);  // a = x·z_l
        z = cmul_exact_pk(z, j.dz);
        if constexpr (decltype(renorm)::value) z = normalise_avx(z);
#pragma unroll
        for (int t = 0; t < NTT; t++) acc[t] = add_chip(acc[t], a, c[t]);
    };
    using Renorm = std::true_type;
    using Plain = std::false_type;
    int m0 = 0;
    for (; m0 + kB <= M; m0 += kB) {
        if (m0 + 2 * kB <= M) {
#pragma unroll
            for (int u = 0; u < kB; u++) xb[u] = load_sample<FMT>(span, v0 + (m0 + kB + u) * kStride, 0);
        } else {
#pragma unroll
            for (int u = 0; u < kB; u++) xb[u] = m0 + kB + u < M ? load_sample<FMT>(span, v0 + (m0 + kB + u) * kStride, 0) : f2{0.0f, 0.0f};
        }
        block_chips(kB);
        // kB divides 64: only a block's first iteration can be followed by a renormalisation
        if ((m0 & 63) == 0) iteration(xa[0], cv[0], Renorm{});
        else iteration(xa[0], cv[0], Plain{});
#pragma unroll
        for (int u = 1; u < kB; u++) iteration(xa[u], cv[u], Plain{});
#pragma unroll
        for (int u = 0; u < kB; u++) xa[u] = xb[u];
    }
    if (m0 < M) {  // fewer than kB iterations left (the lookups past them repeat the last sample's index)
        block_chips(M - m0);
        if ((m0 & 63) == 0) iteration(xa[0], cv[0], Renorm{});
        else iteration(xa[0], cv[0], Plain{});
#pragma unroll
        for (int u = 1; u < kB; u++)
            if (m0 + u < M) iteration(xa[u], cv[u], Plain{});
    }
}

// u_avx's final combination of the 16 chains (:279-291), valid at lane 0 of each 16-lane row:
// ((d_k + d_{k+4}) + d_{k+8}) + d_{k+12} for k = 0..3, then (((0 + s_0) + s_1) + s_2) + s_3.
__device__ __forceinline__ float avx_chain_sum_row(float d)
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

template <int FMT, int NT, bool DATA>
__global__ __launch_bounds__(kLThreads, GNSSHIP_LANE_OCC) void trk_lane_kernel(const TrkParams* __restrict__ pk, TrkChannel* __restrict__ chans,
    const CodeDesc* __restrict__ codes, int n_codes, const void* __restrict__ samples, uint64_t buf_first, int64_t buf_len, int max_rounds,
    int n_chans, int code_cap_floats, gnsship_trk_epoch* __restrict__ rec, gnsship_trk_dump_record* __restrict__ dump,
    gnsship_trk_corr_trace* __restrict__ trace, int* __restrict__ ran_count)
{
    constexpr int NTT = NT + (DATA ? 1 : 0);
    constexpr int SB = sample_bytes<FMT>();
    extern __shared__ uint32_t lbits[];
    __shared__ TrkChannel sc[kLChans];
    __shared__ float staps[kLChans][2 * kMaxTaps + 2];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int row = lane >> 4, l = lane & (kAvxLanes - 1);
    const int nthreads = blockDim.x, wg_chans = (nthreads / kWave) * kLRows;  // ≤ kLChans
    const int cs = wave * kLRows + row;  // the lane's channel slot in the workgroup
    const int ch0 = blockIdx.x * wg_chans;
    const int ch = ch0 + cs;
    const TrkParams& k = *pk;
    const int CW = lane_code_words(code_cap_floats);
    {
        const int n_here = min(wg_chans, n_chans - ch0);
        constexpr int kWords = sizeof(TrkChannel) / 4;
        const int* src = reinterpret_cast<const int*>(chans + ch0);
        int* dst = reinterpret_cast<int*>(sc);
        for (int i = tid; i < n_here * kWords; i += nthreads) dst[i] = src[i];
    }
    __syncthreads();  // the waves are independent from here on
    TrkChannel& c = sc[cs];
    // a channel that is not tracking, or whose codes are missing, is skipped: its state is untouched
    bool valid = false;
    if (ch < n_chans) {
        const bool tracking = c.state == 2 || c.state == 3 || c.state == 4;
        const bool codes_ok = c.code_id >= 0 && c.code_id < n_codes && codes[c.code_id].ptr && codes[c.code_id].len > 0 &&
                              padded_code_quads(codes[c.code_id].len) * 4 <= code_cap_floats &&
                              (!DATA || (c.data_code_id >= 0 && c.data_code_id < n_codes && codes[c.data_code_id].ptr &&
                                            codes[c.data_code_id].len == codes[c.code_id].len));
        valid = tracking && codes_ok;
    }
    uint32_t* b0 = lbits + cs * (DATA ? 2 : 1) * CW;
    uint32_t* b1 = DATA ? b0 + CW : b0;
    const unsigned long long valid_rows = __ballot(valid && l == 0);
    for (int r = 0; r < kLRows; r++) {
        if (!((valid_rows >> (16 * r)) & 1ull)) continue;
        const TrkChannel& cr = sc[wave * kLRows + r];
        uint32_t* d0 = lbits + (wave * kLRows + r) * (DATA ? 2 : 1) * CW;
        stage_code_bits(d0, codes[cr.code_id], CW, lane);
        if constexpr (DATA) stage_code_bits(d0 + CW, codes[cr.data_code_id], CW, lane);
    }
    // lane 0 wrote the replicas (and, below, each row's lane 0 updates its channel in LDS) that the
    // row's other lanes read next: order those LDS accesses within the wave
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int L = valid ? codes[c.code_id].len : 1;
    const int N = static_cast<int>(k.conf.vector_length);
    const int M = N / kAvxLanes, tail = N - kAvxLanes * M;
    const uint64_t vl = k.conf.vector_length;
    const i4v span = sample_span<FMT>(samples, 0, static_cast<int>(buf_len));  // the host keeps buf_len·SB < 2^31
    bool live = valid;
    for (int e = 0; e < max_rounds; e++) {
        // every lane of the row derives the epoch from its channel's state
        bool run = false;
        if (live)
            run = (c.state == 2 || c.state == 3 || c.state == 4) && c.nitems_read >= buf_first &&
                  c.nitems_read + vl <= buf_first + static_cast<uint64_t>(buf_len);
        live = run;  // a channel that cannot run stays so (its state does not change, nitems_read only grows)
        const unsigned long long run_rows = __ballot(run && l == 0);
        if (run_rows == 0) break;
        if (run) {
            const LJob j = lane_job<NT>(k, c, buf_first, L, l);
            f2 acc[NTT];
#pragma unroll
            for (int t = 0; t < NTT; t++) acc[t] = f2{0.0f, 0.0f};
            f2 z = j.z;
            // the in-margin form when every running row's chip indices lie in the padded replica
            const bool all_in = __ballot(run && l == 0 && !j.in_margin) == 0;
            if (all_in)
                lane_correlate<FMT, NT, DATA, true>(span, j, M, l, b0, b1, L, z, acc);
            else
                lane_correlate<FMT, NT, DATA, false>(span, j, M, l, b0, b1, L, z, acc);
            // the sixteen chains combined (:279-291), at lane 0 of the row
#pragma unroll
            for (int t = 0; t < NTT; t++) acc[t] = f2{avx_chain_sum_row(acc[t].x), avx_chain_sum_row(acc[t].y)};
            if (l == 0) {
                // the serial tail (:294-308): _phase = normalise(z_0), then sample by sample
                f2 ph = normalise_avx(z);
                for (int q = 0; q < tail; q++) {
                    const int n = kAvxLanes * M + q;
                    const f2 x = load_sample<FMT>(span, (j.off + n) * SB, 0);
                    const f2 wo = cmul_exact(x, ph);  // wo = in_common[n]·_phase
                    ph = cmul_exact(ph, j.inc);
                    const float sn = __fmul_rn(j.code_step, static_cast<float>(n));
#pragma unroll
                    for (int t = 0; t < NT; t++) acc[t] = add_chip(acc[t], wo, code_chip<false>(b0, L, sn, j.shifts[t], j.rem_code));
                    if constexpr (DATA) acc[NT] = add_chip(acc[NT], wo, code_chip<false>(b1, L, sn, 0.0f, j.rem_code));
                }
                float* taps = staps[cs];
#pragma unroll
                for (int t = 0; t < NTT; t++) {
                    const int o = (DATA && t == NT) ? 2 * kMaxTaps : 2 * t;
                    taps[o] = acc[t].x;
                    taps[o + 1] = acc[t].y;
                }
                // the loop update on the channel's state
                c.epoch_start = c.nitems_read;
                const float* pdata = DATA ? taps + 2 * kMaxTaps : taps;
                const size_t slot = static_cast<size_t>(e) * n_chans + ch;
                gnsship_trk_dump_record* dr = dump ? dump + slot : nullptr;
                gnsship_trk_epoch r{};
                r.flags = 8;
                const double coh = epoch_pre(k, c, taps, pdata, r, nullptr, dr);
                if (coh > 0.0) {
                    const bool locked = lock_status(k, c, coh);
                    if (locked) {
                        LoopRegs lr;
                        load_regs(k, c, lr);
                        epoch_loop(k, lr, nullptr);
                        store_regs(lr, c);
                    }
                    epoch_post(k, c, taps, pdata, r, locked, dr);
                }
                epoch_finish(k, c, r);
                if (rec) rec[slot] = r;
                if (trace) {
                    gnsship_trk_corr_trace tr{};
                    tr.sample_counter = c.epoch_start;
                    tr.n_samples = N;
                    tr.n_taps = NT;
                    tr.rem_carrier_phase_rad = j.rem_carr;
                    tr.phase_step_rad = j.step;
                    tr.rem_code_phase_samples = j.rem_code;
                    tr.code_phase_step_samples = j.code_step;
                    for (int t = 0; t < 5; t++) tr.shifts[t] = j.shifts[t];
                    for (int t = 0; t < 10; t++) tr.taps[t] = t < 2 * NT ? taps[t] : 0.0f;
                    tr.data_prompt[0] = DATA ? pdata[0] : 0.0f;
                    tr.data_prompt[1] = DATA ? pdata[1] : 0.0f;
                    trace[slot] = tr;
                }
            }
        }
        if (lane == 0) atomicAdd(ran_count + e, __popcll(run_rows));
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the loop update's state, before the next epoch's reads
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // before the write-back reads the updated state
    if (valid) {
        if (l == 0) c.ran = 0;
        // the channel's state back to HBM, all but the prompt buffer's unused capacity (entries past
        // cn0_samples are never written: 352 of the 928 bytes at the default 20 samples)
        constexpr int kWords = sizeof(TrkChannel) / 4;
        constexpr int kPb = static_cast<int>(offsetof(TrkChannel, prompt_buf) / 4), kPbEnd = kPb + 2 * kTrkMaxCn0Samples;
        const int pb_used = kPb + 2 * static_cast<int>(k.conf.cn0_samples);
        const int* src = reinterpret_cast<const int*>(&c);
        int* dst = reinterpret_cast<int*>(chans + ch);
        for (int i = l; i < kWords; i += kAvxLanes)
            if (i < pb_used || i >= kPbEnd) dst[i] = src[i];
    }
}

}  // namespace

bool trk_lane_supported(const TrkParams& p, int code_cap_floats, int n_chans, int fmt, int64_t buf_len, bool codes_binary)
{
    if (p.conf.rotator != GNSSHIP_ROTATOR_AVX || p.conf.high_dyn || !trk_persist_supports(p) || !codes_binary) return false;
    const int sb = fmt == GNSSHIP_FMT_CF32 ? 8 : (fmt == GNSSHIP_FMT_CI16 ? 4 : 2);
    if (buf_len < 0 || buf_len * sb >= (int64_t{1} << 31)) return false;  // one 32-bit buffer offset space
    const size_t lds = static_cast<size_t>(kLChans) * (p.jobs_per_channel > 1 ? 2 : 1) * lane_code_words(code_cap_floats) * sizeof(uint32_t);
    if (lds + kLChans * (sizeof(TrkChannel) + (2 * kMaxTaps + 2) * sizeof(float)) > 64 * 1024) return false;
    if (const char* env = std::getenv("GNSSHIP_TRK_LANE")) return env[0] == '1';
    return trk_fast_thru(n_chans);
}

hipError_t launch_trk_lane(const TrkParams* params_dev, const TrkParams& params, TrkChannel* chans, int n_chans, const CodeDesc* codes, int n_codes,
    int code_cap_floats, const void* samples, int fmt, uint64_t buf_first, int64_t buf_len, int max_rounds, gnsship_trk_epoch* rec,
    gnsship_trk_dump_record* dump, gnsship_trk_corr_trace* trace, int* ran_count, hipStream_t stream)
{
    const bool data = params.jobs_per_channel > 1;
    const int nt = params.n_taps;
    // waves per workgroup: up to kLWaves, fewer while that leaves compute units idle
    const int cus = trk_device_cus();
    const int nw = std::max(1, std::min(kLWaves, (n_chans + kLRows * cus - 1) / (kLRows * cus)));
    const int wg_chans = nw * kLRows;
    const size_t lds = static_cast<size_t>(wg_chans) * (data ? 2 : 1) * lane_code_words(code_cap_floats) * sizeof(uint32_t);
    dim3 grid((n_chans + wg_chans - 1) / wg_chans), block(nw * kWave);
#define GNSSHIP_LANE(F, NTV, DV)                                                                                                                         \
    do {                                                                                                                                                 \
        auto kfn = trk_lane_kernel<F, NTV, DV>;                                                                                                          \
        hipError_t e0 = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));     \
        if (e0 != hipSuccess) return e0;                                                                                                                 \
        hipLaunchKernelGGL(kfn, grid, block, lds, stream, params_dev, chans, codes, n_codes, samples, buf_first, buf_len, max_rounds, n_chans,          \
            code_cap_floats, rec, dump, trace, ran_count);                                                                                               \
    } while (0)
#define GNSSHIP_LANE_F(F)                                   \
    do {                                                    \
        if (nt == 3 && !data) GNSSHIP_LANE(F, 3, false);    \
        else if (nt == 5 && !data) GNSSHIP_LANE(F, 5, false); \
        else if (nt == 5 && data) GNSSHIP_LANE(F, 5, true); \
        else return hipErrorInvalidValue;                   \
    } while (0)
    switch (fmt) {
    case GNSSHIP_FMT_CF32: GNSSHIP_LANE_F(GNSSHIP_FMT_CF32); break;
    case GNSSHIP_FMT_CI16: GNSSHIP_LANE_F(GNSSHIP_FMT_CI16); break;
    case GNSSHIP_FMT_CI8: GNSSHIP_LANE_F(GNSSHIP_FMT_CI8); break;
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_LANE_F
#undef GNSSHIP_LANE
    return hipGetLastError();
}

}  // namespace gnsship
