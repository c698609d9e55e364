// corr_device.h — device helpers shared by the correlator kernels (corr_kernel.hip) and the
// persistent tracking kernel (trk_persist.hip): raw buffer loads of the IF samples (CF32 / CI16 /
// CI8 converted in the load), DPP/shuffle wave reductions, packed complex products, the code
// resampler's bit-exact chip index, and the anchored block correlation of the generic rotator.
#pragma once
#include "engine.h"
#include "nco_math.h"

#pragma clang fp contract(off)

namespace gnsship {

typedef float f2v_t __attribute__((ext_vector_type(2)));

// IF samples are read through raw buffer loads: a chunk's samples get their own buffer resource
// (base = its first sample, num_records = its length in bytes), so lanes past the chunk end read
// zeros from the hardware range check — no clamps, selects or exec masks on the tail — and the
// per-load offsets are SGPR constants (soffset) over one per-lane VGPR offset.
typedef int i4v __attribute__((ext_vector_type(4)));
extern "C" __device__ f2v_t gnsship_raw_buffer_load_f32x2(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2f32");
extern "C" __device__ int gnsship_raw_buffer_load_i32(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
extern "C" __device__ short gnsship_raw_buffer_load_i16(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i16");
typedef float f4v_t __attribute__((ext_vector_type(4)));
typedef int i2v_t __attribute__((ext_vector_type(2)));
extern "C" __device__ f4v_t gnsship_raw_buffer_load_f32x4(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
extern "C" __device__ i4v gnsship_raw_buffer_load_i32x4(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
extern "C" __device__ i2v_t gnsship_raw_buffer_load_i32x2(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");

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

// x·z rounded exactly as _mm256_complexmul_ps / the written-out (ac − bd, ad + bc): every product
// rounded, then one add and one subtract — three packed ops, the swizzles in op_sel / neg modifiers:
//   t = (xr·zr, xr·zi);  u = (xi·zi, xi·zr);  x·z = (t.lo − u.lo, t.hi + u.hi)
__device__ __forceinline__ f2 cmul_exact_pk(f2 x, f2 z)
{
    f2 t, u, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(x), "v"(z));
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(u) : "v"(x), "v"(z));
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(t), "v"(u));
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
#ifndef GNSSHIP_FLOOR_TWO_OPS
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
#else
    return static_cast<int>(__builtin_floorf(x));  // v_floor_f32 + v_cvt_i32_f32
#endif
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

// Lane layout: one wave per chunk; lane t covers samples 256k + 4t + s (s = 0..3) of every
// 256-sample block k of the chunk — four consecutive samples per lane per block, one 2 KiB
// contiguous span per wave-load (CF32: two dwordx4 per lane).
constexpr int kLaneSamples = 4;
constexpr int kWave = 64;

// The four samples of this lane in block kb of a chunk (full block: wide loads).
template <int FMT>
__device__ __forceinline__ void load_block(i4v span, int lane, int kb, f2 (&x)[kLaneSamples])
{
    const int off = (kb * kRenorm + kLaneSamples * lane) * sample_bytes<FMT>();
    if constexpr (FMT == GNSSHIP_FMT_CF32) {
        const f4v_t a = gnsship_raw_buffer_load_f32x4(span, off, 0, 0);
        const f4v_t b = gnsship_raw_buffer_load_f32x4(span, off + 16, 0, 0);
        x[0] = f2{a.x, a.y};
        x[1] = f2{a.z, a.w};
        x[2] = f2{b.x, b.y};
        x[3] = f2{b.z, b.w};
    } else if constexpr (FMT == GNSSHIP_FMT_CI16) {
        const i4v v = gnsship_raw_buffer_load_i32x4(span, off, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; u++)
            x[u] = f2{static_cast<float>(static_cast<short>(v[u] & 0xffff)), static_cast<float>(static_cast<short>(v[u] >> 16))};
    } else {
        const i2v_t v = gnsship_raw_buffer_load_i32x2(span, off, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int w = v[u >> 1] >> (16 * (u & 1));
            x[u] = f2{static_cast<float>(static_cast<signed char>(w & 0xff)), static_cast<float>(static_cast<signed char>((w >> 8) & 0xff))};
        }
    }
}

// The same samples one load each (the chunk's partial last block: the buffer range check zeroes
// every sample past the chunk end on its own).
template <int FMT>
__device__ __forceinline__ void load_block_tail(i4v span, int lane, int kb, f2 (&x)[kLaneSamples])
{
    const int off = (kb * kRenorm + kLaneSamples * lane) * sample_bytes<FMT>();
#pragma unroll
    for (int u = 0; u < kLaneSamples; u++) x[u] = load_sample<FMT>(span, off + u * sample_bytes<FMT>(), 0);
}

template <int FMT>
__device__ __forceinline__ void load_any(i4v span, int lane, int kb, int len, f2 (&x)[kLaneSamples])
{
    if ((kb + 1) * kRenorm <= len)  // wave-uniform
        load_block<FMT>(span, lane, kb, x);
    else
        load_block_tail<FMT>(span, lane, kb, x);
}

// E_j = |inc|^j · e^{i j Δ} for this lane's j = 4·lane (angle formed and range-reduced in double,
// hardware sin/cos in revolutions — E_j to a few 1e-7, against the 1e-5 tolerance).  Generic
// variant only (AVX-variant jobs continue every phasor exactly, corr_kernel.hip correlate_chunk_avx).
__device__ __forceinline__ f2 lane_rotation(const DevJob& job, int j)
{
    constexpr double kInvTwoPi = 0.15915494309189533576888376337251;
    const double ang = static_cast<double>(j) * job.dtheta;
#ifndef GNSSHIP_EJ_LIBM
    const double rev = ang * kInvTwoPi;
    const float rf = static_cast<float>(rev - rint(rev));
    const float s = __builtin_amdgcn_sinf(rf), c = __builtin_amdgcn_cosf(rf);
#else
    constexpr double kTwoPi = 6.283185307179586476925286766559;
    double th = ang;
    th = fma(-kTwoPi, rint(th * kInvTwoPi), th);
    float s, c;
    sincosf(static_cast<float>(th), &s, &c);
#endif
    const float mag = __fmaf_rn(static_cast<float>(j), job.log_mag_inc, 1.0f);
    return f2{mag * c, mag * s};
}

// Correlation of one block (four samples per lane) into acc, kept in the lane's anchor frame:
// Σ (x·P_s)·c with P_s = the block's uniform phasor of offset s (Anchor), the lane factor E_{4t}
// applied once per chunk.  `code` = chip 0 of the padded LDS replica.
// IN_MARGIN: the host proved every chip index of the job lies in the padded range (no modulo).
// FULL: the whole block lies inside the chunk (wave-uniform; only the last block can be partial).
template <int NT, bool IN_MARGIN, bool FULL>
__device__ __forceinline__ void correlate_block(const DevJob& job, const ChunkDesc& ch, const Anchor& A, const float (&shifts)[NT],
    const float* __restrict__ code, int L, int lane, int kb, const f2 (&x)[kLaneSamples], f2 (&acc)[NT])
{
    // phase 1: every chip index of the block and its LDS read (the code resampler, generic
    // association order ((step*n) + shift) - rem, each rounded on its own; built with
    // -ffp-contract=off).  (float)n of the lane's first sample; the next three are exact float
    // increments (jobs are at most 2^24 samples, derive_job).
    float cv[kLaneSamples][NT];
    const int r0 = kb * kRenorm + kLaneSamples * lane;
    const float fn0 = static_cast<float>(ch.start + r0);
    // (float)n and step·(float)n of the four samples, two per packed operation
    f2 sn2[kLaneSamples / 2];
#pragma unroll
    for (int h = 0; h < kLaneSamples / 2; h++) {
        f2 fn;
        if constexpr (FULL) {
            fn = f2{fn0, fn0} + f2{static_cast<float>(2 * h), static_cast<float>(2 * h + 1)};
        } else {
            const int ra = r0 + 2 * h, rb = ra + 1;
            fn = f2{static_cast<float>(ch.start + (ra < ch.len ? ra : ch.len - 1)), static_cast<float>(ch.start + (rb < ch.len ? rb : ch.len - 1))};
        }
        sn2[h] = f2{job.code_step, job.code_step} * fn;  // reference loop counter n, as float
    }
    const f2 nrem = f2{-job.rem_code, -job.rem_code};  // x + (−rem) ≡ x − rem, bit for bit
#pragma unroll
    for (int u = 0; u < kLaneSamples; u++) {
        const float sn = (u & 1) ? sn2[u >> 1].y : sn2[u >> 1].x;
#pragma unroll
        for (int t = 0; t + 1 < NT; t += 2) {  // two taps of one sample per packed add
            const f2 v = (f2{sn, sn} + f2{shifts[t], shifts[t + 1]}) + nrem;
            int i0 = cvt_floor_i32(v.x), i1 = cvt_floor_i32(v.y);
            if constexpr (!IN_MARGIN) {
                i0 = wrap_index(i0, L);
                i1 = wrap_index(i1, L);
            }
            cv[u][t] = code[i0];
            cv[u][t + 1] = code[i1];
        }
    }
    if constexpr (NT & 1) {  // the odd tap of two samples per packed add
#pragma unroll
        for (int h = 0; h < kLaneSamples / 2; h++) {
            const f2 v = (sn2[h] + f2{shifts[NT - 1], shifts[NT - 1]}) + nrem;
            int i0 = cvt_floor_i32(v.x), i1 = cvt_floor_i32(v.y);
            if constexpr (!IN_MARGIN) {
                i0 = wrap_index(i0, L);
                i1 = wrap_index(i1, L);
            }
            cv[2 * h][NT - 1] = code[i0];
            cv[2 * h + 1][NT - 1] = code[i1];
        }
    }
    // phase 2: in_common[n]·phase (anchor frame) and the tap sums
#pragma unroll
    for (int u = 0; u < kLaneSamples; u++) {
        const f2 tt = cmul_pk2_s(x[u], f2{A.p[2 * u], A.p[2 * u + 1]});
#pragma unroll
        for (int t = 0; t < NT; t++) acc[t] = __builtin_elementwise_fma(tt, f2{cv[u][t], cv[u][t]}, acc[t]);
    }
}

// Complex product rounded exactly as the reference's written-out (ac − bd, ad + bc) (the AVX
// rotator's _mm256_complexmul_ps and std::complex<float>): two packed products and one packed add,
// no contraction (fl(x + fl(−y)) ≡ fl(x − y)).
__device__ __forceinline__ f2 cmul_exact(f2 a, f2 b)
{
    const f2 t = f2{a.x, a.x} * b;
    const f2 u = f2{a.y, a.y} * f2{-b.y, b.x};
    return t + u;
}

// The same product in single-rate scalar ops (6 VALU, two deep): for short dependent chains, where a
// dependent packed op issues several times slower on gfx950.
__device__ __forceinline__ f2 cmul_exact_sc(f2 a, f2 b)
{
    const float re = __fsub_rn(__fmul_rn(a.x, b.x), __fmul_rn(a.y, b.y));
    const float im = __fadd_rn(__fmul_rn(a.x, b.y), __fmul_rn(a.y, b.x));
    return f2{re, im};
}

// The same product on a serial chain with q wave-uniform (q in an SGPR pair): six single-rate VALU
// ops (4 cycles each for a lone wave) instead of three packed ones, whose dependent issue costs
// several times more on gfx950 — the AVX phasor replay is a chain of these.
// One asm block per STEPS products: the hazard recognizer pads every inline-asm boundary with an
// s_nop, so a chain written one product per statement would pay one per product.  Within a step
// the products read re, re, im, im and the sums come last (re − bd, ad + bc: the reference's order).
#define GNSSHIP_CMUL_STEP                  \
    "v_mul_f32 %2, %6, %0\n\t"             \
    "v_mul_f32 %4, %7, %0\n\t"             \
    "v_mul_f32 %3, %7, %1\n\t"             \
    "v_mul_f32 %5, %6, %1\n\t"             \
    "v_sub_f32 %0, %2, %3\n\t"             \
    "v_add_f32 %1, %4, %5\n\t"
template <int STEPS>
__device__ __forceinline__ f2 cmul_chain_s(f2 a, f2 q)
{
    static_assert(STEPS >= 1 && STEPS <= 4, "cmul_chain_s: 1-4 steps per block");
    float re = a.x, im = a.y, ac, bd, ad, bc;
    if constexpr (STEPS == 1)
        asm(GNSSHIP_CMUL_STEP : "+v"(re), "+v"(im), "=&v"(ac), "=&v"(bd), "=&v"(ad), "=&v"(bc) : "s"(q.x), "s"(q.y));
    else if constexpr (STEPS == 2)
        asm(GNSSHIP_CMUL_STEP GNSSHIP_CMUL_STEP : "+v"(re), "+v"(im), "=&v"(ac), "=&v"(bd), "=&v"(ad), "=&v"(bc) : "s"(q.x), "s"(q.y));
    else if constexpr (STEPS == 3)
        asm(GNSSHIP_CMUL_STEP GNSSHIP_CMUL_STEP GNSSHIP_CMUL_STEP
            : "+v"(re), "+v"(im), "=&v"(ac), "=&v"(bd), "=&v"(ad), "=&v"(bc)
            : "s"(q.x), "s"(q.y));
    else
        asm(GNSSHIP_CMUL_STEP GNSSHIP_CMUL_STEP GNSSHIP_CMUL_STEP GNSSHIP_CMUL_STEP
            : "+v"(re), "+v"(im), "=&v"(ac), "=&v"(bd), "=&v"(ad), "=&v"(bc)
            : "s"(q.x), "s"(q.y));
    return f2{re, im};
}
#undef GNSSHIP_CMUL_STEP
__device__ __forceinline__ f2 cmul_exact_s(f2 a, f2 q) { return cmul_chain_s<1>(a, q); }
// z·q^n for n ≥ 0 as n successive exact products.
template <int N>
__device__ __forceinline__ f2 cmul_pow_s(f2 z, f2 q)
{
    if constexpr (N >= 4) return cmul_pow_s<N - 4>(cmul_chain_s<4>(z, q), q);
    else if constexpr (N > 0) return cmul_chain_s<N>(z, q);
    else return z;
}

// _mm256_complexnormalise_ps (volk_gnsssdr_avx_intrinsics.h:56-63): z / sqrt(re² + im²), IEEE sqrt
// and division.
__device__ __forceinline__ f2 normalise_avx(f2 z)
{
    const float m = sqrt_rn_f32(__fadd_rn(__fmul_rn(z.x, z.x), __fmul_rn(z.y, z.y)));
    return f2{__fdiv_rn(z.x, m), __fdiv_rn(z.y, m)};
}

// Chip index of tap shift `sh` at sample n: floor(step·(float)n + shift − rem), each operation
// rounded in the reference's order (volk_gnsssdr_32f_xn_resampler_32f_xn.h:63-80); sn = step·(float)n.
template <bool IN_MARGIN>
__device__ __forceinline__ float code_at(const float* code, int L, float sn, float sh, float rem)
{
    int i = cvt_floor_i32(__fsub_rn(__fadd_rn(sn, sh), rem));
    if constexpr (!IN_MARGIN) i = wrap_index(i, L);
    return code[i];
}

// Sum over the 64 lanes of the wave (every lane gets it): DPP row sums, then the four rows.
__device__ __forceinline__ float wave_sum(float v)
{
    v = row_sum(v);
    v += __shfl_xor(v, 16, kWave);
    v += __shfl_xor(v, 32, kWave);
    return v;
}

}  // namespace gnsship
