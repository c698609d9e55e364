// acq_kernel.hip — PCPS (parallel code phase search) acquisition for gfx950.
//
// Reference: pcps_acquisition::acquisition_core (pcps_acquisition.cc:600-871), whose Doppler loop
// (:640-672) does, per bin i:   wipe = in ⊙ w_i;  X = FFT(wipe);  Y = IFFT(X ⊙ conj(FFT(code)));
// grid_i = |Y|².  Then max_to_input_power_statistic / first_vs_second_peak_statistic (:496-597).
//
// MI355X structure (all FFTs are LDS-resident, one workgroup per transform):
//   acq_fft_rows_kernel   X_b = FFT(sig ⊙ w_b) for every bin b — computed ONCE per bin and shared by
//                         every PRN searched in the same call (the reference recomputes it per
//                         channel); also used for the code FFT (conj) in set_local_code.
//   acq_search_kernel     per (prn, bin): Y = IFFT(X_b ⊙ C_p) in LDS, |Y|² fused, then the row
//                         statistics the reference derives from the grid — first-index maximum,
//                         row sum (CFAR input power) and the second peak outside ±samples_per_chip —
//                         reduced in-block; the |Y|² grid row is written only when requested.
//   acq_decide_kernel     per prn: the reference's bin-ordered strict-greater search over the row
//                         maxima + opposite-row input power → gnsship_acq_result.
// FFT: Stockham autosort, mixed radix {2,3,4,5,8}, natural order in and out, twiddles from an
// N-entry table rounded from double.  Unnormalised like FFTW (forward e^{-j}, backward e^{+j}).
#include <vector>

#include "acq_engine.h"

namespace gnsship {

// Phase timestamps of acq_search_big_kernel for the profiling build only (make prof,
// scripts/acq_wg_profile.py): slot [workgroup·16 + k] = wall_clock64() at phase k, thread 0.
#ifdef GNSSHIP_CORR_PROFILE
__device__ unsigned long long* g_acq_prof = nullptr;
#define GNSSHIP_ACQ_STAMP(k) \
    do { \
        if (g_acq_prof && threadIdx.x == 0) g_acq_prof[(static_cast<size_t>(blockIdx.y) * gridDim.x + blockIdx.x) * 16 + (k)] = wall_clock64(); \
    } while (0)
#define GNSSHIP_ACQ_STAMP_LANE(k, tid) \
    do { \
        if (g_acq_prof && threadIdx.x == (tid)) g_acq_prof[(static_cast<size_t>(blockIdx.y) * gridDim.x + blockIdx.x) * 16 + (k)] = wall_clock64(); \
    } while (0)
#else
#define GNSSHIP_ACQ_STAMP(k) \
    do { \
    } while (0)
#define GNSSHIP_ACQ_STAMP_LANE(k, tid) \
    do { \
    } while (0)
#endif

// The FFT arithmetic (complex products, butterflies) contracts to FMAs: the reference's transform
// (FFTW through gr::fft) is matched to float accuracy, not bit for bit, and a contracted complex
// product is 2 multiplies + 2 FMAs instead of 4 + 2 (the C3 search is VALU-bound).  The
// bit-specified steps keep explicit roundings: |y|² as volk_32fc_magnitude_squared_32f, the grid
// accumulation, the decision's arithmetic.
__device__ __forceinline__ float2 cmulf(float2 a, float2 b)
{
#pragma clang fp contract(fast)
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <int FMT>
__device__ __forceinline__ float2 load_if(const void* __restrict__ base, int64_t i)
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

// Small DFTs on registers.  SIGN = -1 forward, +1 backward.
template <int R, int SIGN>
__device__ __forceinline__ void dft_small(float2* v)
{
#pragma clang fp contract(fast)
    if constexpr (R == 2) {
        const float2 a = v[0], b = v[1];
        v[0] = make_float2(a.x + b.x, a.y + b.y);
        v[1] = make_float2(a.x - b.x, a.y - b.y);
    } else if constexpr (R == 3) {
        constexpr float c1 = -0.5f, s1 = SIGN * 0.86602540378443864676f;
        const float2 a = v[0], b = v[1], c = v[2];
        const float2 t = make_float2(b.x + c.x, b.y + c.y), d = make_float2(b.x - c.x, b.y - c.y);
        v[0] = make_float2(a.x + t.x, a.y + t.y);
        const float2 m = make_float2(a.x + c1 * t.x, a.y + c1 * t.y);
        v[1] = make_float2(m.x - s1 * d.y, m.y + s1 * d.x);
        v[2] = make_float2(m.x + s1 * d.y, m.y - s1 * d.x);
    } else if constexpr (R == 4) {
        const float2 a = v[0], b = v[1], c = v[2], d = v[3];
        const float2 s0 = make_float2(a.x + c.x, a.y + c.y), d0 = make_float2(a.x - c.x, a.y - c.y);
        const float2 s1 = make_float2(b.x + d.x, b.y + d.y), d1 = make_float2(b.x - d.x, b.y - d.y);
        // multiply d1 by SIGN*j
        const float2 jd1 = make_float2(-SIGN * d1.y, SIGN * d1.x);
        v[0] = make_float2(s0.x + s1.x, s0.y + s1.y);
        v[2] = make_float2(s0.x - s1.x, s0.y - s1.y);
        v[1] = make_float2(d0.x + jd1.x, d0.y + jd1.y);
        v[3] = make_float2(d0.x - jd1.x, d0.y - jd1.y);
    } else if constexpr (R == 5) {
        constexpr float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
        constexpr float s1 = SIGN * 0.95105651629515357212f, s2 = SIGN * 0.58778525229247312917f;
        const float2 a = v[0];
        const float2 t1 = make_float2(v[1].x + v[4].x, v[1].y + v[4].y), t2 = make_float2(v[2].x + v[3].x, v[2].y + v[3].y);
        const float2 d1 = make_float2(v[1].x - v[4].x, v[1].y - v[4].y), d2 = make_float2(v[2].x - v[3].x, v[2].y - v[3].y);
        v[0] = make_float2(a.x + t1.x + t2.x, a.y + t1.y + t2.y);
        const float2 m1 = make_float2(a.x + c1 * t1.x + c2 * t2.x, a.y + c1 * t1.y + c2 * t2.y);
        const float2 m2 = make_float2(a.x + c2 * t1.x + c1 * t2.x, a.y + c2 * t1.y + c1 * t2.y);
        // j*(s1 d1 + s2 d2) and j*(s2 d1 - s1 d2)
        const float2 n1 = make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);
        const float2 n2 = make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);
        v[1] = make_float2(m1.x - n1.y, m1.y + n1.x);
        v[4] = make_float2(m1.x + n1.y, m1.y - n1.x);
        v[2] = make_float2(m2.x - n2.y, m2.y + n2.x);
        v[3] = make_float2(m2.x + n2.y, m2.y - n2.x);
    } else if constexpr (R == 10) {
        // prime-factor (Good-Thomas) 2 x 5, no internal twiddles: input n = (5·n1 + 2·n2) mod 10,
        // output k ≡ k1 (mod 2), k ≡ k2 (mod 5), i.e. k = (5·k1 + 6·k2) mod 10
        float2 a[2][5];
#pragma unroll
        for (int n1 = 0; n1 < 2; n1++)
#pragma unroll
            for (int n2 = 0; n2 < 5; n2++) a[n1][n2] = v[(5 * n1 + 2 * n2) % 10];
        dft_small<5, SIGN>(a[0]);
        dft_small<5, SIGN>(a[1]);
#pragma unroll
        for (int k2 = 0; k2 < 5; k2++) {
            const float2 p = a[0][k2], q = a[1][k2];
            v[(6 * k2) % 10] = make_float2(p.x + q.x, p.y + q.y);
            v[(5 + 6 * k2) % 10] = make_float2(p.x - q.x, p.y - q.y);
        }
    } else if constexpr (R == 8) {
        // radix-8 as 2 x 4: even/odd radix-4 then combine with w8^k
        float2 e[8], o[8];
        e[0] = v[0]; e[1] = v[2]; e[2] = v[4]; e[3] = v[6];
        o[0] = v[1]; o[1] = v[3]; o[2] = v[5]; o[3] = v[7];
        dft_small<4, SIGN>(e);
        dft_small<4, SIGN>(o);
        constexpr float h = 0.70710678118654752440f;
        const float2 w[4] = {make_float2(1.f, 0.f), make_float2(h, SIGN * h), make_float2(0.f, SIGN * 1.f), make_float2(-h, SIGN * h)};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const float2 t = cmulf(o[k], w[k]);
            v[k] = make_float2(e[k].x + t.x, e[k].y + t.y);
            v[k + 4] = make_float2(e[k].x - t.x, e[k].y - t.y);
        }
    }
}

// One Stockham pass of radix R over LDS buffer `buf` (in place through registers: every thread
// loads its butterflies, barrier, stores).  tw[t] = exp(-2πi t/N); conjugated for SIGN = +1.
// Butterfly j reads buf[j + r·N/R] and writes buf[(j/Ns)·Ns·R + j%Ns + r·Ns]  (Stockham autosort).
template <int R, int SIGN>
__device__ __forceinline__ void stockham_pass(float2* __restrict__ buf, int N, int Ns, const float2* __restrict__ tw)
{
    constexpr int MAXB = (kMaxAcqN / R + kAcqThreads - 1) / kAcqThreads;  // butterflies per thread
    const int nb = N / R;
    const int tstep = N / (Ns * R);  // twiddle table stride
    float2 v[MAXB][R];
#pragma unroll
    for (int c = 0; c < MAXB; c++) {
        const int j = threadIdx.x + c * kAcqThreads;
        if (j < nb) {
            const int k = j % Ns;
#pragma unroll
            for (int r = 0; r < R; r++) {
                float2 x = buf[j + r * nb];
                if (r > 0 && k > 0) {
                    float2 w = tw[k * r * tstep];  // k·r·tstep < Ns·R·tstep = N
                    if (SIGN > 0) w.y = -w.y;
                    x = cmulf(x, w);
                }
                v[c][r] = x;
            }
            dft_small<R, SIGN>(v[c]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < MAXB; c++) {
        const int j = threadIdx.x + c * kAcqThreads;
        if (j < nb) {
            const int k = j % Ns;
            const int base = (j / Ns) * Ns * R + k;
#pragma unroll
            for (int r = 0; r < R; r++) buf[base + r * Ns] = v[c][r];
        }
    }
    __syncthreads();
}

template <int SIGN>
__device__ void fft_lds(float2* __restrict__ buf, const FftPlan& plan, const float2* __restrict__ tw)
{
    int Ns = 1;
    for (int p = 0; p < plan.n_passes; p++) {
        const int R = plan.radix[p];
        switch (R) {
        case 2: stockham_pass<2, SIGN>(buf, plan.n, Ns, tw); break;
        case 3: stockham_pass<3, SIGN>(buf, plan.n, Ns, tw); break;
        case 4: stockham_pass<4, SIGN>(buf, plan.n, Ns, tw); break;
        case 5: stockham_pass<5, SIGN>(buf, plan.n, Ns, tw); break;
        default: stockham_pass<8, SIGN>(buf, plan.n, Ns, tw); break;
        }
        Ns *= R;
    }
}

// fft_lds with the length known at compile time (ct_radix order: radix 10 where it divides, then
// odd radices): constant index arithmetic, every pass's butterflies unrolled, fewer passes
// (12500 = 10·10·5·5·5: five instead of six).  Twiddles tw[k·r·tstep] from the M-entry table.
constexpr int ct_radix(int m);
template <int MC, int NsC, int SIGN>
__device__ __forceinline__ void fft_lds_ct(float2* __restrict__ buf, const float2* __restrict__ tw)
{
    if constexpr (NsC < MC) {
        constexpr int R = ct_radix(MC / NsC);
        constexpr int nb = MC / R;
        constexpr int tstep = MC / (NsC * R);
        constexpr int MAXB = (nb + kAcqThreads - 1) / kAcqThreads;
        float2 v[MAXB][R];
#pragma unroll
        for (int c = 0; c < MAXB; c++) {
            const int j = threadIdx.x + c * kAcqThreads;
            if (j < nb) {
                const int k = j % NsC;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    float2 x = buf[j + r * nb];
                    if (r > 0 && NsC > 1) {
                        float2 w = tw[k * r * tstep];
                        if (SIGN > 0) w.y = -w.y;
                        x = cmulf(x, w);
                    }
                    v[c][r] = x;
                }
                dft_small<R, SIGN>(v[c]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < MAXB; c++) {
            const int j = threadIdx.x + c * kAcqThreads;
            if (j < nb) {
                const int k = j % NsC;
                const int base = (j / NsC) * NsC * R + k;
#pragma unroll
                for (int r = 0; r < R; r++) buf[base + r * NsC] = v[c][r];
            }
        }
        __syncthreads();
        fft_lds_ct<MC, NsC * R, SIGN>(buf, tw);
    }
}

// fft_lds_ct with the twiddles from a QUARTER table in LDS (tq[u] = exp(−2πi u/M), u < M/4): the
// M-entry table no longer fits beside an M-point row (12500 × 8 B each), and read from global
// memory its loads sat in every pass's vmcnt queue.  tw[t] for t = q·M/4 + u
// is tq[u]·(−j)^q — exact, the same float values as the full table (whose entries are rounded from
// the same double cos/sin up to the quarter-turn symmetry).
// R consecutive points from a 16-byte-aligned slot (R even): R/2 16-byte stores.  The first pass's
// outputs (slot j·R, stride R points between lanes) as 8-byte stores put 4 lanes on a bank; as
// 16-byte stores the 8 lanes of each store cycle fall on distinct banks.
template <int R>
__device__ __forceinline__ void store_run(float2* __restrict__ dst, const float2 (&v)[R])
{
    if constexpr (R % 2 == 0) {
        float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll
        for (int r = 0; r < R; r += 2) d4[r / 2] = make_float4(v[r].x, v[r].y, v[r + 1].x, v[r + 1].y);
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) dst[r] = v[r];
    }
}

// One butterfly of fft_lds_ct_q's pass at NsC: thread index j's R inputs buf[j + r·nb], twiddled,
// through the R-point DFT (the only arithmetic of the pass; its output goes to (j / NsC)·NsC·R +
// j % NsC + r·NsC).
template <int MC, int NsC, int SIGN>
__device__ __forceinline__ void ctq_bfly(const float2* __restrict__ buf, const float2* __restrict__ tq, int j, float2 (&v)[ct_radix(MC / NsC)])
{
    constexpr int R = ct_radix(MC / NsC);
    constexpr int nb = MC / R;
    constexpr int tstep = MC / (NsC * R);
    constexpr int Q = MC / 4;
    const int k = j % NsC;
    if constexpr (NsC > 1 && (NsC - 1) * tstep < Q) {
        // W^{k·r·tstep} = (W^{k·tstep})^r: one table read (k·tstep < M/4, no quarter turn),
        // the other powers as a balanced product tree (≤ 4 products deep)
        float2 w[R];
        w[1] = tq[k * tstep];
        if (SIGN > 0) w[1].y = -w[1].y;
#pragma unroll
        for (int r = 2; r < R; r++) w[r] = cmulf(w[r / 2], w[r - r / 2]);
        v[0] = buf[j];
#pragma unroll
        for (int r = 1; r < R; r++) v[r] = cmulf(buf[j + r * nb], w[r]);
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {
            float2 x = buf[j + r * nb];
            if (r > 0 && NsC > 1) {
                const int t = k * r * tstep;  // < MC
                const int q = t / Q, u = t - q * Q;
                const float2 w0 = tq[u];
                float wx = (q & 1) ? w0.y : w0.x, wy = (q & 1) ? -w0.x : w0.y;
                if (q & 2) {
                    wx = -wx;
                    wy = -wy;
                }
                if (SIGN > 0) wy = -wy;
                x = cmulf(x, make_float2(wx, wy));
            }
            v[r] = x;
        }
    }
    dft_small<R, SIGN>(v);
}

// The passes from NsC up to (not including) the one at NSTOP (NSTOP = MC: every remaining pass).
// jp10: this thread's butterfly in the NsC = 10 pass when that pass has one butterfly per thread
// (kLanePerm10 below; −1: none), else the thread index.
template <int MC, int NsC, int SIGN, int NSTOP = MC>
__device__ __forceinline__ void fft_lds_ct_q(float2* __restrict__ buf, const float2* __restrict__ tq, int tid, int jp10 = -2)
{
    static_assert(MC % 4 == 0, "quarter twiddle table");
    if constexpr (NsC < NSTOP) {
        constexpr int R = ct_radix(MC / NsC);
        constexpr int nb = MC / R;
        constexpr int MAXB = (nb + kAcqThreads - 1) / kAcqThreads;
        float2 v[MAXB][R];
#pragma unroll
        for (int c = 0; c < MAXB; c++) {
            const int j = (NsC == 10 && MAXB == 1 && jp10 != -2) ? jp10 : tid + c * kAcqThreads;
            if (j >= 0 && j < nb) ctq_bfly<MC, NsC, SIGN>(buf, tq, j, v[c]);
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < MAXB; c++) {
            const int j = (NsC == 10 && MAXB == 1 && jp10 != -2) ? jp10 : tid + c * kAcqThreads;
            if (j >= 0 && j < nb) {
                const int k = j % NsC;
                const int base = (j / NsC) * NsC * R + k;
                if constexpr (NsC == 1) {
                    store_run<R>(buf + base, v[c]);
                } else {
#pragma unroll
                    for (int r = 0; r < R; r++) buf[base + r * NsC] = v[c][r];
                }
            }
        }
        __syncthreads();
        fft_lds_ct_q<MC, NsC * R, SIGN, NSTOP>(buf, tq, tid, jp10);
    }
}

// The stride before the last pass of the compile-time plan (its NsC): MC / (the last radix).
constexpr int ct_last_ns(int m, int ns = 1) { return ns * ct_radix(m / ns) >= m ? ns : ct_last_ns(m, ns * ct_radix(m / ns)); }

// Transforms of up to kTwLdsMax points read their twiddles from LDS: the N-entry table is staged
// next to the data once per workgroup (every Stockham pass otherwise waits on L2 for its R − 1
// twiddle loads, with only one or two butterflies per thread to hide them).
constexpr int kTwLdsMax = 4096;

__device__ __forceinline__ const float2* stage_twiddles(float2* dst, const float2* __restrict__ tw, int n)
{
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = tw[i];
    return dst;  // visible after the caller's next barrier
}

// dst[i] = a[i] ⊙ b[i] (b == nullptr: a[i]), i < n, by threads tid, tid + nt, … with a runtime n:
// the loads go in batches of kLdsBatch per thread (index clamped in bounds, the store guarded), so a
// batch is in flight together instead of one load-wait-store round trip per element.
constexpr int kLdsBatch = 8;
__device__ __forceinline__ void lds_load_prod(float2* __restrict__ dst, const float2* __restrict__ a, const float2* __restrict__ b, int n,
    int tid, int nt)
{
    for (int base = tid; base < n; base += kLdsBatch * nt) {
        float2 av[kLdsBatch], bv[kLdsBatch];
#pragma unroll
        for (int u = 0; u < kLdsBatch; u++) {
            const int i = base + u * nt;
            av[u] = a[i < n ? i : n - 1];
        }
        if (b) {
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int i = base + u * nt;
                bv[u] = b[i < n ? i : n - 1];
            }
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) av[u] = cmulf(av[u], bv[u]);
        }
#pragma unroll
        for (int u = 0; u < kLdsBatch; u++) {
            const int i = base + u * nt;
            if (i < n) dst[i] = av[u];
        }
    }
}

// rows[b] = FFT(sig ⊙ mult[b])  (mult == nullptr: FFT(sig)); conj_out: store conj (code FFT).
template <int FMT>
__global__ __launch_bounds__(kAcqThreads) void acq_fft_rows_kernel(const void* __restrict__ sig, const float2* __restrict__ mult,
    FftPlan plan, const float2* __restrict__ tw, float2* __restrict__ rows, int conj_out, int n_valid)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int N = plan.n;
    const float2* m = mult ? mult + static_cast<int64_t>(b) * N : nullptr;
    const float2* twl = N <= kTwLdsMax ? stage_twiddles(lds + N, tw, N) : tw;
    const int last = n_valid > 0 ? n_valid - 1 : 0;
    for (int base = threadIdx.x; base < N; base += kLdsBatch * blockDim.x) {  // batches of loads in flight
        float2 xv[kLdsBatch];
#pragma unroll
        for (int u = 0; u < kLdsBatch; u++) {
            const int i = base + u * blockDim.x;
            const float2 x = load_if<FMT>(sig, i < n_valid ? i : last);
            xv[u] = i < n_valid ? x : make_float2(0.0f, 0.0f);  // zero-padded past the consumed samples
        }
        if (m) {
            float2 wv[kLdsBatch];
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int i = base + u * blockDim.x;
                wv[u] = m[i < N ? i : N - 1];
            }
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) xv[u] = cmulf(xv[u], wv[u]);  // volk_32fc_x2_multiply_32fc(in, wipeoff)
        }
#pragma unroll
        for (int u = 0; u < kLdsBatch; u++) {
            const int i = base + u * blockDim.x;
            if (i < N) lds[i] = xv[u];
        }
    }
    __syncthreads();
    fft_lds<-1>(lds, plan, twl);
    float2* out = rows + static_cast<int64_t>(b) * N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        float2 y = lds[i];
        if (conj_out) y.y = -y.y;
        out[i] = y;
    }
}

// ---------------------------------------------------------------------------------------------
// Large transforms (kMaxAcqN < N ≤ 32768, e.g. the 25000-point transform of a 1 ms GPS code at
// 25 Msps): four-step, N = P·M, M ≤ 1024 rows of the LDS stage and P ≤ 32 points per thread in
// registers.  Thread t owns column t: x[t + M·q], q < P.
//   forward:  X[kq + P·k] = Σ_t W_M^{t·k} · W_N^{t·kq} · Σ_q x[t + M·q] W_P^{q·kq}
//             (register P-point DFT and twiddle in one launch, then the M-point row DFTs in place
//             in a second, one wave per row, each wave running its row's passes in LDS with no
//             workgroup barrier);
//             stored row-major TRANSPOSED: XT[kq·M + k] = X[kq + P·k].
//   inverse:  y[t + M·q] = Σ_kq W_P^{−q·kq} · W_N^{−t·kq} · Σ_k Z[kq + P·k] W_M^{−t·k}
//             reads Z in the same transposed layout (rows first, registers last) and so returns
//             natural order.  Point-wise products between two transposed spectra need no reorder.
// Pass twiddles come from the N-entry table: exp(−2πi m/M) = tw[m·P].
// ---------------------------------------------------------------------------------------------
constexpr int first_radix(int m)
{
    return (m % 8 == 0) ? 8 : (m % 5 == 0) ? 5 : (m % 4 == 0) ? 4 : (m % 3 == 0) ? 3 : 2;
}

// Wave-level row transforms: each wave owns whole rows of the four-step and runs every Stockham
// pass of its row in place, with no workgroup barrier — a pass loads all of the lane's butterflies
// into registers before any store, and a wave's LDS operations complete in program order (the fence
// keeps the compiler from moving a store above the loads).  The workgroup meets only at the
// column↔row transposes.  tw[m] = exp(−2πi m/M) (the row table staged in LDS).
constexpr int kWaveRows = kAcqThreads / 64;  // rows transformed per round (one per wave)

template <int R, int SIGN>
__device__ __forceinline__ void wave_pass(float2* __restrict__ buf, int M, int Ns, const float2* __restrict__ tw, int lane)
{
    constexpr int MAXB = (kAcqThreads / R + 63) / 64;  // butterflies per lane for M ≤ 1024
    const int nb = M / R;
    const int tstep = M / (Ns * R);
    float2 v[MAXB][R];
#pragma unroll
    for (int c = 0; c < MAXB; c++) {
        const int j = lane + 64 * c;
        if (j < nb) {
            const int k = j % Ns;
#pragma unroll
            for (int r = 0; r < R; r++) {
                float2 x = buf[j + r * nb];
                if (r > 0 && k > 0) {
                    float2 w = tw[k * r * tstep];
                    if (SIGN > 0) w.y = -w.y;
                    x = cmulf(x, w);
                }
                v[c][r] = x;
            }
            dft_small<R, SIGN>(v[c]);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < MAXB; c++) {
        const int j = lane + 64 * c;
        if (j < nb) {
            const int k = j % Ns;
            const int base = (j / Ns) * Ns * R + k;
#pragma unroll
            for (int r = 0; r < R; r++) buf[base + r * Ns] = v[c][r];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The same passes with the row length known at compile time (MC > 0): radices first_radix(M / Ns)
// in order, every index split j / Ns, j % Ns and twiddle stride a constant (the runtime form spends
// more VALU on integer division than on the butterflies).
// Radix order of the compile-time rows: odd radices first.  The first Stockham pass (Ns = 1) writes
// butterfly j's outputs at R·j…R·j+R−1, a lane stride of 8R bytes: 16-way LDS bank conflicts for
// R = 8 (64 B), 2-way for R = 5 (40 B); the radix-8 pass goes last, where its writes are contiguous.
// Radix 10 (a twiddle-free 2 x 5 prime-factor butterfly) where it divides: 1000 = 10·10·10 runs in
// three passes instead of four (5·5·5·8), a quarter fewer LDS round trips per row.
constexpr int ct_radix(int m)
{
    return (m % 10 == 0) ? 10 : (m % 5 == 0) ? 5 : (m % 3 == 0) ? 3 : (m % 8 == 0) ? 8 : (m % 4 == 0) ? 4 : 2;
}

// Twiddles of the compile-time rows, one table per pass laid out [r − 1][k] (k < Ns, 1 ≤ r < R):
// consecutive lanes (consecutive k) read consecutive entries, where the single M-entry table read at
// k·r·tstep put up to eight lanes of a wave on one LDS bank.  Same values (tw[k·r·tstep]), so the
// transform is bit-identical.  ct_tw_count(M, Ns) = entries of the passes from Ns on (< M in total).
constexpr int ct_tw_count(int m, int ns)
{
    return ns >= m ? 0 : (ns > 1 ? (ct_radix(m / ns) - 1) * ns : 0) + ct_tw_count(m, ns * ct_radix(m / ns));
}

// dst[pass table] = exp(−2πi·k·r·tstep/M) = tw[k·r·tstep·stride]  (tw: the N-entry table, stride = N/M)
template <int MC, int NsC>
__device__ __forceinline__ void fill_row_pass_tw(float2* __restrict__ dst, const float2* __restrict__ tw, int stride, int tid, int nt)
{
    if constexpr (NsC < MC) {
        constexpr int R = ct_radix(MC / NsC);
        constexpr int tstep = MC / (NsC * R);
        if constexpr (NsC > 1) {
            constexpr int off = ct_tw_count(MC, 1) - ct_tw_count(MC, NsC);
            for (int i = tid; i < (R - 1) * NsC; i += nt) {
                const int r = 1 + i / NsC, k = i % NsC;
                dst[off + i] = tw[k * r * tstep * stride];
            }
        }
        fill_row_pass_tw<MC, NsC * R>(dst, tw, stride, tid, nt);
    }
}

template <int MC, int NsC, int SIGN>
__device__ __forceinline__ void wave_fft_row_ct(float2* __restrict__ buf, const float2* __restrict__ tw, int lane)
{
    if constexpr (NsC < MC) {
        constexpr int R = ct_radix(MC / NsC);
        constexpr int nb = MC / R;
        constexpr int MAXB = (nb + 63) / 64;
        constexpr int off = ct_tw_count(MC, 1) - ct_tw_count(MC, NsC);
        float2 v[MAXB][R];
#pragma unroll
        for (int c = 0; c < MAXB; c++) {
            const int j = lane + 64 * c;
            if (j < nb) {
                const int k = j % NsC;
                if constexpr (NsC > 1) {
                    // W^{k·r·tstep} = (W^{k·tstep})^r: one table read (the pass table's r = 1 row), the
                    // other powers as a balanced product tree (≤ 4 products deep) — the LDS pipe, which
                    // the CU's waves share, carried a third of the row traffic as twiddle reads
                    float2 w[R];
                    w[1] = tw[off + k];
                    if (SIGN > 0) w[1].y = -w[1].y;
#pragma unroll
                    for (int r = 2; r < R; r++) w[r] = cmulf(w[r / 2], w[r - r / 2]);
                    v[c][0] = buf[j];
#pragma unroll
                    for (int r = 1; r < R; r++) v[c][r] = cmulf(buf[j + r * nb], w[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < R; r++) v[c][r] = buf[j + r * nb];
                }
                dft_small<R, SIGN>(v[c]);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < MAXB; c++) {
            const int j = lane + 64 * c;
            if (j < nb) {
                const int k = j % NsC;
                const int base = (j / NsC) * NsC * R + k;
                if constexpr (NsC == 1) {
                    store_run<R>(buf + base, v[c]);
                } else {
#pragma unroll
                    for (int r = 0; r < R; r++) buf[base + r * NsC] = v[c][r];
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_sched_barrier(0);  // keep the next pass's loads from being hoisted into this one (register pressure)
        wave_fft_row_ct<MC, NsC * R, SIGN>(buf, tw, lane);
    }
}

template <int SIGN>
__device__ __forceinline__ void wave_fft_row(float2* __restrict__ row, const FftPlan& plan, const float2* __restrict__ tw, int lane)
{
    int Ns = 1;
    for (int p = 0; p < plan.n_passes; p++) {
        switch (plan.radix[p]) {
        case 2: wave_pass<2, SIGN>(row, plan.n, Ns, tw, lane); break;
        case 3: wave_pass<3, SIGN>(row, plan.n, Ns, tw, lane); break;
        case 4: wave_pass<4, SIGN>(row, plan.n, Ns, tw, lane); break;
        case 5: wave_pass<5, SIGN>(row, plan.n, Ns, tw, lane); break;
        default: wave_pass<8, SIGN>(row, plan.n, Ns, tw, lane); break;
        }
        Ns *= plan.radix[p];
    }
}


// cos/sin of 2π·m/L in double by Taylor series, for compile-time register-DFT twiddles (L ≤ 32).
constexpr double ct_sin_red(double x)
{
    double term = x, sum = x;
    for (int i = 1; i < 30; i++) {
        term *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
        sum += term;
    }
    return sum;
}
constexpr double ct_cos_red(double x)
{
    double term = 1.0, sum = 1.0;
    for (int i = 1; i < 30; i++) {
        term *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
        sum += term;
    }
    return sum;
}
constexpr double kPi = 3.14159265358979323846;
constexpr double ct_angle(int m, int L)
{
    // reduce 2π·m/L into (−π, π]
    const int mm = m % L;
    const int ms = (2 * mm > L) ? mm - L : mm;
    return 2.0 * kPi * static_cast<double>(ms) / static_cast<double>(L);
}

// In-register Stockham DFT of length P (compile-time, fully unrolled).  Pass twiddles
// exp(SIGN·2πi·m/(Ns·R)) are literal constants.
template <int P, int Ns, int SIGN>
__device__ __forceinline__ void dft_reg(float2* x, const float2* __restrict__ tw, int N)
{
    if constexpr (Ns < P) {
        constexpr int R = first_radix(P / Ns);
        constexpr int nb = P / R;
        float2 y[P];
#pragma unroll
        for (int j = 0; j < nb; j++) {
            const int k = j % Ns;
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                float2 a = x[j + r * nb];
                if (r > 0 && k > 0) {
                    const double ang = ct_angle(k * r, Ns * R);
                    const float2 w = make_float2(static_cast<float>(ct_cos_red(ang)), static_cast<float>(SIGN * ct_sin_red(ang)));
                    a = cmulf(a, w);
                }
                v[r] = a;
            }
            dft_small<R, SIGN>(v);
#pragma unroll
            for (int r = 0; r < R; r++) y[(j / Ns) * Ns * R + k + r * Ns] = v[r];
        }
#pragma unroll
        for (int i = 0; i < P; i++) x[i] = y[i];
        dft_reg<P, Ns * R, SIGN>(x, tw, N);
    }
}

// In-place register DFT for P = R1·R2 (R1 = first_radix(P), R2 a supported radix): with
// n = R2·n1 + n2,  X[k1 + R1·k2] = Σ_n2 W_P^{n2·k1} W_R2^{n2·k2} Σ_n1 x[R2·n1 + n2] W_R1^{n1·k1}.
// Stage 1 writes the R1-point results back into the slots they came from, stage 2 likewise, so only
// one butterfly's values are live beside the P points (the Stockham form above holds a second P-point
// array and spills at 128 VGPRs).  Output X[q] is left in slot reg_slot<P>(q) = R2·(q mod R1) + q/R1.
constexpr bool small_radix(int r) { return r == 2 || r == 3 || r == 4 || r == 5 || r == 8; }
template <int P>
constexpr bool two_factor() { return small_radix(first_radix(P)) && small_radix(P / first_radix(P)) && first_radix(P) * (P / first_radix(P)) == P; }
template <int P>
constexpr int reg_slot(int q)
{
    if constexpr (two_factor<P>()) {
        constexpr int R1 = first_radix(P), R2 = P / R1;
        return R2 * (q % R1) + q / R1;
    } else {
        return q;
    }
}

template <int P, int SIGN>
__device__ __forceinline__ void dft_reg_inplace(float2* x, const float2* __restrict__ tw, int N)
{
    if constexpr (two_factor<P>()) {
        constexpr int R1 = first_radix(P), R2 = P / R1;
#pragma unroll
        for (int n2 = 0; n2 < R2; n2++) {
            float2 v[R1];
#pragma unroll
            for (int n1 = 0; n1 < R1; n1++) v[n1] = x[R2 * n1 + n2];
            dft_small<R1, SIGN>(v);
#pragma unroll
            for (int k1 = 0; k1 < R1; k1++) {
                float2 a = v[k1];
                if (n2 > 0 && k1 > 0) {
                    const double ang = ct_angle(n2 * k1, P);
                    a = cmulf(a, make_float2(static_cast<float>(ct_cos_red(ang)), static_cast<float>(SIGN * ct_sin_red(ang))));
                }
                x[R2 * k1 + n2] = a;
            }
        }
#pragma unroll
        for (int k1 = 0; k1 < R1; k1++) {
            float2 v[R2];
#pragma unroll
            for (int n2 = 0; n2 < R2; n2++) v[n2] = x[R2 * k1 + n2];
            dft_small<R2, SIGN>(v);
#pragma unroll
            for (int k2 = 0; k2 < R2; k2++) x[R2 * k1 + k2] = v[k2];
        }
    } else {
        dft_reg<P, 1, SIGN>(x, tw, N);
    }
}

// rowsT[b] = transposed FFT(sig ⊙ mult[b]) in two launches over the whole chip (one workgroup per
// transform would occupy n_bins CUs): the column stage writes each column's register P-point DFT,
// twiddled by W_N^{t·kq}, to row kq of the output, then the row stage transforms every row in
// place, one wave per row.  The same operations in the same order as the one-workgroup-per-transform
// form this replaces (and as the inverse in acq_search_big_kernel, mirrored).
constexpr int kBigColThreads = 64;
constexpr int kBigRowWaves = 4;

template <int FMT, int P>
__global__ __launch_bounds__(kBigColThreads) void acq_fft_big_cols_kernel(const void* __restrict__ sig, const float2* __restrict__ mult, int M,
    const float2* __restrict__ tw, float2* __restrict__ rowsT, int n_valid)
{
    const int N = P * M;
    const int t = blockIdx.x * kBigColThreads + threadIdx.x;
    const int b = blockIdx.y;
    if (t >= M) return;
    float2 v[P];
    // branch-free loads (every load of the column in flight at once): past the consumed samples the
    // index is clamped in bounds and the value replaced by zero (the zero padding)
    const int last = n_valid > 0 ? n_valid - 1 : 0;
#pragma unroll
    for (int q = 0; q < P; q++) {
        const int i = t + M * q;
        const float2 x = load_if<FMT>(sig, i < n_valid ? i : last);
        v[q] = i < n_valid ? x : make_float2(0.0f, 0.0f);
    }
    if (mult) {  // uniform: the Doppler wipeoff of bin b (volk_32fc_x2_multiply_32fc(in, wipeoff))
        const float2* m = mult + static_cast<int64_t>(b) * N;
        float2 w[P];
#pragma unroll
        for (int q = 0; q < P; q++) w[q] = m[t + M * q];
#pragma unroll
        for (int q = 0; q < P; q++) v[q] = cmulf(v[q], w[q]);
    }
    dft_reg_inplace<P, -1>(v, tw, N);  // X[kq] in v[reg_slot<P>(kq)]
    float2* out = rowsT + static_cast<int64_t>(b) * N;
    // W_N^{t·kq} = (W_N^t)^kq: one coalesced table read and a balanced product tree (≤ 5 products
    // deep) instead of P − 1 reads gathered at stride kq from the N-entry table
    float2 w[P];
    w[0] = make_float2(1.0f, 0.0f);
    if constexpr (P > 1) w[1] = tw[t];
#pragma unroll
    for (int kq = 2; kq < P; kq++) w[kq] = cmulf(w[kq / 2], w[kq - kq / 2]);
#pragma unroll
    for (int kq = 0; kq < P; kq++) {
        const float2 xk = v[reg_slot<P>(kq)];
        out[kq * M + t] = kq ? cmulf(xk, w[kq]) : xk;
    }
}

// grid: ceil(n_bins·P / kBigRowWaves); row r = b·P + kq of rowsT, transformed in place.
template <int MC>
__global__ __launch_bounds__(kBigRowWaves * 64) void acq_fft_big_rows_kernel(FftPlan row_plan, int P, const float2* __restrict__ tw,
    float2* __restrict__ rowsT, int n_rows_total, int conj_out)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int M = MC > 0 ? MC : row_plan.n;  // compile-time for the C3 plan: the row copies unroll (loads in flight together)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float2* rtw = lds + kBigRowWaves * M;  // row twiddles exp(−2πi m/M) = tw[m·P], m < M (per-pass tables for MC > 0)
    if constexpr (MC > 0) fill_row_pass_tw<MC, 1>(rtw, tw, P, threadIdx.x, kBigRowWaves * 64);
    else for (int i = threadIdx.x; i < M; i += kBigRowWaves * 64) rtw[i] = tw[i * P];
    const int r = blockIdx.x * kBigRowWaves + wave;
    float2* row = lds + wave * M;
    float2* g = rowsT + static_cast<int64_t>(r) * M;  // rows are contiguous: b·N + kq·M = (b·P + kq)·M
    if constexpr (MC > 0 && MC % 2 == 0) {  // 16-byte pairs (rows start 16-byte aligned)
        const float4* g4 = reinterpret_cast<const float4*>(g);
        float4* row4 = reinterpret_cast<float4*>(row);
        if (r < n_rows_total) {
#pragma unroll
            for (int i = lane; i < MC / 2; i += 64) row4[i] = g4[i];
        }
    } else {
        if (r < n_rows_total)
            for (int i = lane; i < M; i += 64) row[i] = g[i];
    }
    __syncthreads();
    if (r >= n_rows_total) return;
    if constexpr (MC > 0) wave_fft_row_ct<MC, 1, -1>(row, rtw, lane);
    else wave_fft_row<-1>(row, row_plan, rtw, lane);
    if constexpr (MC > 0 && MC % 2 == 0) {
        const float4* row4 = reinterpret_cast<const float4*>(row);
        float4* g4 = reinterpret_cast<float4*>(g);
#pragma unroll
        for (int i = lane; i < MC / 2; i += 64) {
            float4 y = row4[i];
            if (conj_out) {
                y.y = -y.y;
                y.w = -y.w;
            }
            g4[i] = y;
        }
    } else {
        for (int i = lane; i < M; i += 64) {
            float2 y = row[i];
            if (conj_out) y.y = -y.y;
            g[i] = y;
        }
    }
}

struct MaxIdx {
    float v;
    int i;
};

__device__ __forceinline__ MaxIdx better(MaxIdx a, MaxIdx b)
{
    // strict greater wins; ties → smaller index (volk_gnsssdr_32f_index_max_32u: first index of max)
    if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
    return a;
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// Wave reductions: within each 16-lane row by DPP (quad xor 1, xor 2, half-row mirror, row mirror —
// each step pairs two already-reduced groups), across the four rows by two shuffles.
__device__ __forceinline__ MaxIdx wave_argmax(MaxIdx m)
{
    m = better(m, MaxIdx{dpp_f<0xB1>(m.v), dpp_i<0xB1>(m.i)});    // quad_perm [1,0,3,2]
    m = better(m, MaxIdx{dpp_f<0x4E>(m.v), dpp_i<0x4E>(m.i)});    // quad_perm [2,3,0,1]
    m = better(m, MaxIdx{dpp_f<0x141>(m.v), dpp_i<0x141>(m.i)});  // row_half_mirror
    m = better(m, MaxIdx{dpp_f<0x140>(m.v), dpp_i<0x140>(m.i)});  // row_mirror
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) m = better(m, MaxIdx{__shfl_xor(m.v, o, 64), __shfl_xor(m.i, o, 64)});
    return m;
}

__device__ __forceinline__ float wave_sum_f(float s)
{
    s += dpp_f<0xB1>(s);
    s += dpp_f<0x4E>(s);
    s += dpp_f<0x141>(s);
    s += dpp_f<0x140>(s);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    return s;
}

template <int NW>  // waves per workgroup, = blockDim.x / 64 (the cross-wave loops unroll)
__device__ __forceinline__ MaxIdx block_argmax(MaxIdx m, MaxIdx* red)
{
    m = wave_argmax(m);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = m;
    __syncthreads();
    MaxIdx r = red[0];
#pragma unroll
    for (int w = 1; w < NW; w++) r = better(r, red[w]);
    __syncthreads();
    return r;
}

template <int NW>  // waves per workgroup, = blockDim.x / 64 (the cross-wave loops unroll)
__device__ __forceinline__ float block_sum(float s, float* red)
{
    s = wave_sum_f(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = s;
    __syncthreads();
    float r = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; w++) r += red[w];
    __syncthreads();
    return r;
}

__device__ __forceinline__ float wave_max_f(float s)
{
    s = fmaxf(s, dpp_f<0xB1>(s));
    s = fmaxf(s, dpp_f<0x4E>(s));
    s = fmaxf(s, dpp_f<0x141>(s));
    s = fmaxf(s, dpp_f<0x140>(s));
    s = fmaxf(s, __shfl_xor(s, 16, 64));
    s = fmaxf(s, __shfl_xor(s, 32, 64));
    return s;
}

// Block maximum of values (no index): the second peak keeps only its value.
template <int NW>  // waves per workgroup, = blockDim.x / 64 (the cross-wave loops unroll)
__device__ __forceinline__ float block_max(float s, float* red)
{
    s = wave_max_f(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = s;
    __syncthreads();
    float r = red[0];
#pragma unroll
    for (int w = 1; w < NW; w++) r = fmaxf(r, red[w]);
    return r;
}

// Both at once (one barrier pair): the row maximum with its first index and the row sum.
template <int NW>  // waves per workgroup, = blockDim.x / 64 (the cross-wave loops unroll)
__device__ __forceinline__ void block_argmax_sum(MaxIdx& m, float& s, MaxIdx* redm, float* reds)
{
    m = wave_argmax(m);
    s = wave_sum_f(s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        redm[wave] = m;
        reds[wave] = s;
    }
    __syncthreads();
    MaxIdx r = redm[0];
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        if (w) r = better(r, redm[w]);
        t += reds[w];
    }
    __syncthreads();
    m = r;
    s = t;
}

// grid: (n_bins, n_prns).  rowstat[(p*n_bins + b)] ; grid_out optional [p][b][row_len].
// Row = |Y[row_off + i]|², i < row_len (the second half of the transform with bit_transition_flag,
// pcps_acquisition.cc:663-664); the second-peak window wraps modulo win_mod (d_fft_size, :573-580).
__global__ __launch_bounds__(kAcqThreads) void acq_search_kernel(const float2* __restrict__ X, const float2* __restrict__ codes_fft,
    FftPlan plan, const float2* __restrict__ tw, int n_bins, RowSpec rs, int accumulate, RowStat* __restrict__ rowstat,
    float* __restrict__ grid_out)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ MaxIdx red_m[kAcqThreads / 64];
    __shared__ float red_s[kAcqThreads / 64];
    const int b = blockIdx.x, p = blockIdx.y;
    const int N = plan.n;
    const float2* x = X + static_cast<int64_t>(b) * N;
    const float2* c = codes_fft + static_cast<int64_t>(p) * N;
    const float2* twl = N <= kTwLdsMax ? stage_twiddles(lds + N, tw, N) : tw;
    lds_load_prod(lds, x, c, N, threadIdx.x, blockDim.x);  // ×conj(code FFT)
    __syncthreads();
    fft_lds<+1>(lds, plan, twl);
    // |Y|² in place (as float in the .x slot) + optional grid row (accumulated over dwells)
    float* row = grid_out ? grid_out + (static_cast<int64_t>(p) * n_bins + b) * rs.row_len : nullptr;
    MaxIdx m{-1.0f, 0x7fffffff};
    float s = 0.0f;
    for (int i = threadIdx.x; i < rs.row_len; i += blockDim.x) {
        const float2 y = lds[rs.row_off + i];
        float mag = __fadd_rn(__fmul_rn(y.x, y.x), __fmul_rn(y.y, y.y));  // volk_32fc_magnitude_squared_32f
        if (row) {
            if (accumulate) mag = __fadd_rn(row[i], mag);  // volk_32f_x2_add_32f
            row[i] = mag;
        }
        lds[rs.row_off + i].x = mag;
        m = better(m, MaxIdx{mag, i});
        s += mag;
    }
    block_argmax_sum<kAcqThreads / 64>(m, s, red_m, red_s);
    const MaxIdx best = m;
    const float sum = s;
    // second peak outside the circular window [best-spc, best+spc) (first_vs_second_peak_statistic :566-593)
    int e1 = best.i - rs.spc, e2 = best.i + rs.spc;
    if (e1 < 0) e1 += rs.win_mod; else if (e2 >= rs.win_mod) e2 -= rs.win_mod;
    MaxIdx m2{0.0f, 0x7fffffff};
    for (int i = threadIdx.x; i < rs.row_len; i += blockDim.x) {
        const bool in_win = (e1 < e2) ? (i >= e1 && i < e2) : (i >= e1 || i < e2);
        const float v = in_win ? 0.0f : lds[rs.row_off + i].x;
        m2 = better(m2, MaxIdx{v, i});
    }
    const MaxIdx second = block_argmax<kAcqThreads / 64>(m2, red_m);
    if (threadIdx.x == 0) {
        RowStat r;
        r.max = best.v;
        r.argmax = best.i;
        r.sum = sum;
        r.second = second.v;
        rowstat[static_cast<int64_t>(p) * n_bins + b] = r;
    }
}

// Large-N search: Y = IFFT(XT_b ⊙ CT_p) by the transposed four-step (rows in LDS, then the
// register P-point stage), |Y|² and the same row statistics as acq_search_kernel.  Thread t holds
// y[t + M·q] for q < P, i.e. the natural index n = t + M·q.
// NT threads per workgroup (NT ≥ M; NT/64 rows per round).  (A 40 × 625 layout of the C3 transform
// in 640 threads, two workgroups per CU, needs ≤ 96 VGPRs and spills: 0.50 ms per C3 sweep; at one
// workgroup per CU it ties 25 × 1000.)
// dst[i] = x[i] ⊙ c[i], i < n, by threads tid, tid + nt, …  With an even compile-time row length
// (MC > 0) the pairs of points go as 16-byte loads and stores (rows start 16-byte aligned), the trip
// count is known and the loads are issued back to back.
template <int MC>
__device__ __forceinline__ void load_rows_prod(float2* __restrict__ dst, const float2* __restrict__ x, const float2* __restrict__ c, int n,
    int tid, int nt)
{
    if constexpr (MC > 0 && MC % 2 == 0) {
        const float4* x4 = reinterpret_cast<const float4*>(x);
        const float4* c4 = reinterpret_cast<const float4*>(c);
        float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll 4
        for (int i = tid; i < n / 2; i += nt) {
            const float4 a = x4[i], b = c4[i];
            const float2 p0 = cmulf(make_float2(a.x, a.y), make_float2(b.x, b.y));
            const float2 p1 = cmulf(make_float2(a.z, a.w), make_float2(b.z, b.w));
            d4[i] = make_float4(p0.x, p0.y, p1.x, p1.y);
        }
    } else {
        for (int i = tid; i < n; i += nt) dst[i] = cmulf(x[i], c[i]);
    }
}

template <int P, int MC = 0, int NT = kAcqThreads>
__global__ __launch_bounds__(NT) void acq_search_big_kernel(const float2* __restrict__ XT,
    const float2* __restrict__ codesT, FftPlan row_plan, const float2* __restrict__ tw, int n_bins, RowSpec rs, int accumulate,
    RowStat* __restrict__ rowstat, float* __restrict__ grid_out)
{
    constexpr int kRoundRows = NT / 64;  // rows transformed per round (one per wave)
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ MaxIdx red_m[NT / 64];
    __shared__ float red_s[NT / 64];
    const int b = blockIdx.x, p = blockIdx.y;
    const int M = MC > 0 ? MC : row_plan.n;  // compile-time for the C3 plan: the load loops unroll
    const int N = P * M;
    const int t = threadIdx.x;
    const float2* x = XT + static_cast<int64_t>(b) * N;
    const float2* c = codesT + static_cast<int64_t>(p) * N;
    float2 v[P];
    float2* rtw = lds + kRoundRows * M;  // row twiddles exp(−2πi m/M) = tw[m·P], m < M
    if constexpr (MC > 0) fill_row_pass_tw<MC, 1>(rtw, tw, P, t, NT);  // per-pass tables (conflict-free reads)
    else for (int i = t; i < M; i += NT) rtw[i] = tw[i * P];
    const int lane = t & 63, wave = t >> 6;
    // the short round first: the v[kq] of finished rounds stay live in registers through the later
    // rounds' row passes, so the fewer of them the better (P = 25: 9 rows, then 16)
    constexpr int kFirst = P - kRoundRows * ((P - 1) / kRoundRows);
    constexpr int kRounds = 1 + (P - kFirst) / kRoundRows;
    // Two rounds with a short first one: the waves with no row in round 0 load rows kFirst..kRoundRows−1
    // of round 1 into their own (free) slots meanwhile; round 1 then loads only rows kRoundRows..P−1,
    // into slots 0..kFirst−1.  Slot kk of round 1 holds row kk (kk ≥ kFirst) or kk + kRoundRows.
    constexpr bool kPrefetch = kRounds == 2 && kFirst < kRoundRows;
    GNSSHIP_ACQ_STAMP(0);
#pragma unroll
    for (int rr = 0; rr < kRounds; rr++) {  // constant trip count: unrolled, v[] indices compile-time
        const int r0 = rr == 0 ? 0 : kFirst + (rr - 1) * kRoundRows;
        const int nrows = rr == 0 ? kFirst : kRoundRows;
        if (kPrefetch && rr == 1) {
            load_rows_prod<MC>(lds, x + kRoundRows * M, c + kRoundRows * M, kFirst * M, t, NT);  // ×conj(code FFT)
        } else {
            load_rows_prod<MC>(lds, x + r0 * M, c + r0 * M, nrows * M, t, NT);
        }
        __syncthreads();
        GNSSHIP_ACQ_STAMP(r0 == 0 ? 1 : 4);
        if (wave < nrows) {
            // an opaque copy of the lane id per round: the row's index arithmetic is recomputed rather
            // than kept live across rounds by common-subexpression elimination (register pressure)
            int lane_r = lane;
            asm volatile("" : "+v"(lane_r));
            if constexpr (MC > 0) wave_fft_row_ct<MC, 1, +1>(lds + wave * M, rtw, lane_r);
            else wave_fft_row<+1>(lds + wave * M, row_plan, rtw, lane);
        } else if (kPrefetch && rr == 0) {
            load_rows_prod<MC>(lds + wave * M, x + wave * M, c + wave * M, M, lane, 64);
        }
        __syncthreads();
        GNSSHIP_ACQ_STAMP(r0 == 0 ? 2 : 5);
        if (t < M) {
            // MC > 0: W_N^{t·kq} as powers of W_N^t (one table read, a product tree ≤ 5 deep) — the
            // two-table form read 2 LDS entries per point
            float2 wp[P];
            if constexpr (MC > 0) {
                wp[0] = make_float2(1.0f, 0.0f);
                wp[1] = tw[t];
#pragma unroll
                for (int q = 2; q < P; q++) wp[q] = cmulf(wp[q / 2], wp[q - q / 2]);
            }
#pragma unroll
            for (int kk = 0; kk < kRoundRows; kk++) {
                const int kq = (kPrefetch && rr == 1) ? (kk < kFirst ? kk + kRoundRows : kk) : r0 + kk;
                if (kk < nrows) {
                    float2 w;
                    if constexpr (MC > 0) {
                        w = wp[kq];
                    } else {
                        w = tw[t * kq];
                    }
                    w.y = -w.y;  // W_N^{−t·kq}
                    v[kq] = kq ? cmulf(lds[kk * M + t], w) : lds[kk * M + t];
                }
            }
        }
        __syncthreads();
        GNSSHIP_ACQ_STAMP(r0 == 0 ? 3 : 6);
    }
    // |y|² stays in registers (g[], the thread's own P points) for the rare second-peak rescan below.
    MaxIdx m{-1.0f, 0x7fffffff};
    float s = 0.0f;
    float g[P];
    if (t < M) {
        dft_reg_inplace<P, +1>(v, tw, N);  // y[t + M·q] in v[reg_slot<P>(q)]
        GNSSHIP_ACQ_STAMP_LANE(10, 0);
        GNSSHIP_ACQ_STAMP_LANE(11, 960);
        // |y|² first (the complex points die as their magnitudes appear), then the optional grid
        // row and the row statistics in separate branch-light loops
#pragma unroll
        for (int q = 0; q < P; q++) {
            const float2 y = v[reg_slot<P>(q)];
            g[q] = __fadd_rn(__fmul_rn(y.x, y.x), __fmul_rn(y.y, y.y));  // volk_32fc_magnitude_squared_32f
        }
        if (grid_out) {
            float* row = grid_out + (static_cast<int64_t>(p) * n_bins + b) * rs.row_len;
#pragma unroll
            for (int q = 0; q < P; q++) {
                const int i = t + M * q - rs.row_off;
                if (i >= 0 && i < rs.row_len) {
                    if (accumulate) g[q] = __fadd_rn(row[i], g[q]);  // volk_32f_x2_add_32f
                    row[i] = g[q];
                }
            }
        }
        // The thread's best and its row sum, branch-free (selects, no divergent exec masks).  A
        // thread's row indices rise with q, so "x beats m" in better() order (strict >, ties to the
        // smaller index) is plain x > m for every earlier m; a point outside the row adds +0 to s.
        auto stat = [&](int q, bool valid) {
            const float x = g[q];
            const int i = t + M * q - rs.row_off;
            const bool gt = valid && x > m.v;
            m.v = gt ? x : m.v;
            m.i = gt ? i : m.i;
            s += valid ? x : 0.0f;
        };
        if (rs.row_off == 0 && rs.row_len == N) {  // the whole transform is the row (uniform branch)
#pragma unroll
            for (int q = 0; q < P; q++) stat(q, true);
        } else {
#pragma unroll
            for (int q = 0; q < P; q++) {
                const int i = t + M * q - rs.row_off;
                stat(q, i >= 0 && i < rs.row_len);
            }
        }
    }
    GNSSHIP_ACQ_STAMP(7);
    GNSSHIP_ACQ_STAMP_LANE(12, 960);
    const MaxIdx m1t = m;  // this thread's best, before the block reduction
    block_argmax_sum<NT / 64>(m, s, red_m, red_s);
    const MaxIdx best = m;
    const float sum = s;
    GNSSHIP_ACQ_STAMP(8);
    int e1 = best.i - rs.spc, e2 = best.i + rs.spc;
    if (e1 < 0) e1 += rs.win_mod; else if (e2 >= rs.win_mod) e2 -= rs.win_mod;
    // Second peak outside the window (first_vs_second_peak_statistic :566-593): only its value is
    // kept, i.e. max(0, the largest |y|² outside the window).  The window spans 2·spc < M
    // consecutive indices, so it holds at most one or two of a thread's indices: a thread whose best
    // lies outside it contributes that best, and only the few threads whose best lies inside rescan
    // their P values.
    auto in_win = [&](int i) { return (e1 < e2) ? (i >= e1 && i < e2) : (i >= e1 || i < e2); };
    float v2 = 0.0f;  // only the value is kept: max(0, …)
    if (m1t.i != 0x7fffffff && !in_win(m1t.i)) {
        v2 = m1t.v;
    } else if (m1t.i != 0x7fffffff) {
        // this thread's indices (natural t + M·q, row-shifted) outside the window; the window's
        // form (one interval, or two at the wrap) is uniform over the block
        if (e1 < e2) {
            const unsigned w = static_cast<unsigned>(e2 - e1);
#pragma unroll
            for (int q = 0; q < P; q++) {
                const int i = t + M * q - rs.row_off;
                const bool out = i >= 0 && i < rs.row_len && static_cast<unsigned>(i - e1) >= w;
                v2 = out ? fmaxf(v2, g[q]) : v2;
            }
        } else {
#pragma unroll
            for (int q = 0; q < P; q++) {
                const int i = t + M * q - rs.row_off;
                const bool out = i >= 0 && i < rs.row_len && i < e1 && i >= e2;
                v2 = out ? fmaxf(v2, g[q]) : v2;
            }
        }
    }
    const float second = block_max<NT / 64>(v2, red_s);  // values ≥ 0: max(0, the largest outside the window)
    GNSSHIP_ACQ_STAMP(9);
    if (t == 0) {
        RowStat r;
        r.max = best.v;
        r.argmax = best.i;
        r.sum = sum;
        r.second = second;
        rowstat[static_cast<int64_t>(p) * n_bins + b] = r;
    }
}

// One thread per PRN: the reference's row scan (strict >, ascending bin) and decision values.
// Step two of make_2_steps (step2.active): Doppler = (int)(center + (bin − floor(nb/2))·step2) in float
// and the CFAR input power left at its step-one value (pcps_acquisition.cc:516-525).
__global__ __launch_bounds__(64) void acq_decide_kernel(const RowStat* __restrict__ rowstat, int n_prns, int n_bins, int N, int doppler_max,
    int doppler_step, int doppler_center, int dwells, int use_cfar, float samples_per_code, float resampler_ratio, uint32_t resampler_latency,
    Step2Spec step2, gnsship_acq_result* __restrict__ out)
{
    // one wave per PRN: lane b scans bins b, b + 64, …, then a wave arg-max.  The reference's scan
    // (gmax = 0; strict >, ascending bin) selects the first bin holding the row maximum, and none
    // (bin 0, peak 0) when no row maximum exceeds 0: better() with ties to the smaller index, from a
    // start of {0, −1} that an equal 0 never displaces.
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const RowStat* rs = rowstat + static_cast<int64_t>(p) * n_bins;
    MaxIdx m{0.0f, -1};
    for (int b = lane; b < n_bins; b += 64) m = better(m, MaxIdx{rs[b].max, b});
    m = wave_argmax(m);
    if (lane != 0) return;
    const float gmax = m.i < 0 ? 0.0f : m.v;
    const int bi = m.i < 0 ? 0 : m.i;
    const int ti = m.i < 0 ? 0 : rs[bi].argmax;
    gnsship_acq_result r;
    r.doppler_index = static_cast<uint32_t>(bi);
    r.code_index = static_cast<uint32_t>(ti);
    r.doppler_hz = -doppler_max + doppler_center + doppler_step * bi;
    if (step2.active)
        r.doppler_hz = static_cast<int32_t>(step2.center + (static_cast<float>(bi) - static_cast<float>(floor(n_bins / 2.0))) * step2.step);
    r.peak = gmax;
    if (use_cfar && step2.active) {
        r.input_power = step2.input_power;
        r.test_statistic = gmax / r.input_power;
    } else if (use_cfar) {
        const int opp = (bi + n_bins / 2) % n_bins;
        // (float)(sum / N / 2.0 / dwells)  (pcps_acquisition.cc:518)
        const float s = rs[opp].sum;
        r.input_power = static_cast<float>(static_cast<double>(s / static_cast<float>(N)) / 2.0 / static_cast<double>(dwells));
        r.test_statistic = gmax / r.input_power;
    } else {
        r.input_power = rs[bi].second;
        r.test_statistic = gmax / rs[bi].second;
    }
    // :686-687: the delay at the resampled rate scaled back to input samples, minus the FIR latency
    r.acq_delay_samples = static_cast<double>(fmodf(static_cast<float>(ti), samples_per_code)) * static_cast<double>(resampler_ratio);
    r.acq_delay_samples -= static_cast<double>(resampler_latency);
    out[p] = r;
}

// ---------------------------------------------------------------------------------------------
// Huge transforms (N > 32768: Galileo E1 at 25 Msps, N = 100000; 1 ms GPS/B1I at 50 Msps,
// N = 50000; E1 at 50 Msps, N = 200000): N = P·M with the M-point rows LDS-resident
// (M ≤ 16384) and P ≤ 32 register points per column, the two stages as separate kernels through
// HBM (the spectrum of one bin is 8N bytes, far beyond one workgroup's LDS):
//   forward:  huge_cols_fwd  T[kq·M + m] = W_N^{m·kq} Σ_q x[m + M·q] W_P^{q·kq}     (registers)
//             huge_rows      XT[kq·M + k] = Σ_m T[kq·M + m] W_M^{m·k}                 (LDS rows)
//             → the same TRANSPOSED layout as the four-step above: XT[kq·M + k] = X[kq + P·k]
//   inverse:  huge_rows      U[kq·M + m] = Σ_k (XT ⊙ CT)[kq·M + k] W_M^{−m·k}          (LDS rows)
//             huge_cols_inv  y[m + M·q] = Σ_kq W_P^{−q·kq} W_N^{−m·kq} U[kq·M + m]   (registers)
//             |y|² into the grid row + per-tile max/argmax/sum, then huge_finalize per row:
//             the reference's first-index maximum, the row sum and the second peak outside
//             ±samples_per_chip (pcps_acquisition.cc:496-597).
// ---------------------------------------------------------------------------------------------
constexpr int kHugeColThreads = 256;
#define GNSSHIP_HUGE_P_LIST(X) X(4) X(5) X(8) X(10) X(16) X(20) X(25) X(32)

// W_N^{m·kq} for kq < P from the column-layout table twC[kq·M + m]: the kq = 1 entry read (coalesced)
// and the other powers as a balanced product tree (≤ 5 products deep) — the other P − 2 reads were
// as many bytes of L2 traffic per column as the column's own data.
template <int P>
__device__ __forceinline__ void col_twiddles(const float2* __restrict__ twC, int M, int m, float2 (&w)[P])
{
    w[0] = make_float2(1.0f, 0.0f);
    if constexpr (P > 1) w[1] = twC[M + m];
#pragma unroll
    for (int kq = 2; kq < P; kq++) w[kq] = cmulf(w[kq / 2], w[kq - kq / 2]);
}

template <int FMT, int P>
__global__ __launch_bounds__(kHugeColThreads) void acq_huge_cols_fwd_kernel(const void* __restrict__ sig, const float2* __restrict__ mult,
    int M, const float2* __restrict__ twN, float2* __restrict__ T, int n_valid)
{
    const int m = blockIdx.x * kHugeColThreads + threadIdx.x;
    const int b = blockIdx.y;
    const int N = P * M;
    if (m >= M) return;
    float2 v[P];
    const int last = n_valid > 0 ? n_valid - 1 : 0;  // branch-free loads, zero padding past n_valid
#pragma unroll
    for (int q = 0; q < P; q++) {
        const int i = m + M * q;
        const float2 x = load_if<FMT>(sig, i < n_valid ? i : last);
        v[q] = i < n_valid ? x : make_float2(0.0f, 0.0f);
    }
    if (mult) {  // uniform: volk_32fc_x2_multiply_32fc(in, wipeoff)
        const float2* w = mult + static_cast<int64_t>(b) * N;
        float2 wv[P];
#pragma unroll
        for (int q = 0; q < P; q++) wv[q] = w[m + M * q];
#pragma unroll
        for (int q = 0; q < P; q++) v[q] = cmulf(v[q], wv[q]);
    }
    dft_reg<P, 1, -1>(v, twN, N);
    float2* out = T + static_cast<int64_t>(b) * N + m;
    float2 wt[P];
    col_twiddles<P>(twN, M, m, wt);
#pragma unroll
    for (int kq = 0; kq < P; kq++) out[kq * M] = kq ? cmulf(v[kq], wt[kq]) : v[kq];  // W_N^{m·kq}
}

// One LDS-resident M-point transform per block: row blockIdx.x of cell (blockIdx.y, blockIdx.z).
// src row = A + y·a_sy + z·a_sz + x·M (times B + z·b_sz + y·b_sy + x·M when B is given);
// dst row = D + y·d_sy + z·d_sz + x·M.  conj_out stores the conjugate (the code spectrum).
template <int SIGN, int MC = 0>
__global__ __launch_bounds__(kAcqThreads) void acq_huge_rows_kernel(const float2* __restrict__ A, int64_t a_sy, int64_t a_sz,
    const float2* __restrict__ B, int64_t b_sy, int64_t b_sz, float2* __restrict__ D, int64_t d_sy, int64_t d_sz, FftPlan plan,
    const float2* __restrict__ twM, int conj_out)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int M = plan.n;
    const int64_t row = static_cast<int64_t>(blockIdx.x) * M;
    const float2* a = A + blockIdx.y * a_sy + blockIdx.z * a_sz + row;
    const float2* bb = B ? B + blockIdx.y * b_sy + blockIdx.z * b_sz + row : nullptr;
    if constexpr (MC > 0) {  // the quarter twiddle table beside the row (M + M/4 entries of LDS)
        for (int i = threadIdx.x; i < MC / 4; i += kAcqThreads) lds[MC + i] = twM[i];
    }
    lds_load_prod(lds, a, bb, M, threadIdx.x, kAcqThreads);  // ×conj(code FFT)
    __syncthreads();
    if constexpr (MC > 0) fft_lds_ct_q<MC, 1, SIGN>(lds, lds + MC, threadIdx.x);
    else fft_lds<SIGN>(lds, plan, twM);
    float2* d = D + blockIdx.y * d_sy + blockIdx.z * d_sz + row;
    for (int i = threadIdx.x; i < M; i += kAcqThreads) {
        float2 y = lds[i];
        if (conj_out) y.y = -y.y;
        d[i] = y;
    }
}

// Column m of the inverse column stage for one cell: v[q] = y[m + M·q] (the same instructions in
// the column kernel and in the finalize kernel's recomputation, so the |y|² agree bit for bit).
template <int P>
__device__ __forceinline__ void huge_col_inv(const float2* __restrict__ u, int m, int M, const float2* __restrict__ twN, float2 (&v)[P])
{
    const int N = P * M;
    float2 wt[P];
    col_twiddles<P>(twN, M, m, wt);
#pragma unroll
    for (int kq = 0; kq < P; kq++) {
        float2 x = u[kq * M];
        if (kq) {
            float2 w = wt[kq];  // W_N^{−m·kq}
            w.y = -w.y;
            x = cmulf(x, w);
        }
        v[kq] = x;
    }
    dft_reg<P, 1, +1>(v, twN, N);
}

// The compile-time-length rows of the search (inverse) stage as a persistent pipeline: block b
// transforms rows b, b + grid, …; the next row's XT and code-spectrum loads (13 + 13 per thread) are
// issued before the current row's transform and land during it, so with one workgroup per CU (the
// 12500-point row and its quarter twiddle table fill 125 KB of LDS) the row reads no longer stall
// each transform.  Row index r = x + P·(y + ny·z) as acq_huge_rows_kernel's (x, y, z) blocks.
template <int SIGN, int MC>
__global__ __launch_bounds__(kAcqThreads) void acq_huge_rows_pipe_kernel(const float2* __restrict__ A, int64_t a_sy, int64_t a_sz,
    const float2* __restrict__ B, int64_t b_sy, int64_t b_sz, float2* __restrict__ D, int64_t d_sy, int64_t d_sz, const float2* __restrict__ twM,
    int P, int ny, int nz)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int PER = (MC + kAcqThreads - 1) / kAcqThreads;
    // the 10000-point rows (10 samples per thread) prefetch the code-spectrum row as well; the
    // 12500-point rows (13) keep it out of the registers the transform needs
    constexpr bool kPrefB = PER <= 10;
    const int total = P * ny * nz;
    const int tid = threadIdx.x;
    for (int i = tid; i < MC / 4; i += kAcqThreads) lds[MC + i] = twM[i];
    float2 av[PER];                   // the next row's XT samples
    float2 bp[kPrefB ? PER : 1];      // and its code-spectrum samples (kPrefB)
    auto issue = [&](int r) {
        const int x = r % P, yz = r / P, y = yz % ny, z = yz / ny;
        const float2* a = A + y * a_sy + z * a_sz + static_cast<int64_t>(x) * MC;
#pragma unroll
        for (int u = 0; u < PER; u++) av[u] = a[min(tid + u * kAcqThreads, MC - 1)];
        if constexpr (kPrefB) {
            const float2* b = B + y * b_sy + z * b_sz + static_cast<int64_t>(x) * MC;
#pragma unroll
            for (int u = 0; u < PER; u++) bp[u] = b[min(tid + u * kAcqThreads, MC - 1)];
        }
    };
    int r = blockIdx.x;
    if (r < total) issue(r);
    for (; r < total; r += gridDim.x) {
        {
            const int x = r % P, yz = r / P, y = yz % ny, z = yz / ny;
            const float2* b = B + y * b_sy + z * b_sz + static_cast<int64_t>(x) * MC;
            float2 bv[PER];
#pragma unroll
            for (int u = 0; u < PER; u++) bv[u] = kPrefB ? bp[kPrefB ? u : 0] : b[min(tid + u * kAcqThreads, MC - 1)];
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int i = tid + u * kAcqThreads;
                if (i < MC) lds[i] = cmulf(av[u], bv[u]);  // XT ⊙ conj(code FFT)
            }
        }
        __syncthreads();
        if (r + static_cast<int>(gridDim.x) < total) issue(r + gridDim.x);  // in flight during this transform
        // the transform's index arithmetic is loop-invariant; recomputed per row (an opaque thread id)
        // rather than hoisted into registers that would spill
        int tid_r = tid;
        asm volatile("" : "+v"(tid_r));
        fft_lds_ct_q<MC, 1, SIGN>(lds, lds + MC, tid_r);
        const int x = r % P, yz = r / P, y = yz % ny, z = yz / ny;
        float2* d = D + y * d_sy + z * d_sz + static_cast<int64_t>(x) * MC;
        for (int i = tid; i < MC; i += kAcqThreads) d[i] = lds[i];
        __syncthreads();  // the row is read out before the next one is written
    }
}

// kLanePerm10: the butterflies of the 10000-point rows' NsC = 10 pass (radix 10, 1000 butterflies
// j = 10a + b) dealt to the 1024 threads so that each 16-lane group reads buf[j + 1000r] and writes
// buf[100a + b + 10r] on 16 distinct bank pairs — j mod 32 and (4a + b) mod 32 distinct in the group
// (thread order made two lanes of a group write one bank pair: 58 % LDS conflict cycles in the rows).
// Greedy in increasing j: 62 full groups and one of 8; −1 marks an idle thread.  Set once per device.
__device__ int16_t g_lane_perm10[kAcqThreads];

static std::vector<int16_t> lane_perm10_table()
{
    std::vector<int16_t> perm(kAcqThreads, -1);
    std::vector<int> rest(1000);
    for (int j = 0; j < 1000; j++) rest[j] = j;
    int slot = 0;
    while (!rest.empty()) {
        std::vector<int> left;
        unsigned long long used_r = 0, used_w = 0;
        int n = 0;
        for (int j : rest) {
            const int kr = j % 32, kw = (4 * (j / 10) + j % 10) % 32;
            if (n < 16 && !((used_r >> kr) & 1) && !((used_w >> kw) & 1)) {
                used_r |= 1ull << kr;
                used_w |= 1ull << kw;
                perm[slot + n++] = static_cast<int16_t>(j);
            } else {
                left.push_back(j);
            }
        }
        slot += 16;
        rest.swap(left);
    }
    return perm;
}

hipError_t ensure_lane_perm10()
{
    static bool done[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 64 && done[dev]) return hipSuccess;
    static const std::vector<int16_t> perm = lane_perm10_table();
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_lane_perm10), perm.data(), sizeof(int16_t) * kAcqThreads);
    if (e == hipSuccess && dev < 64) done[dev] = true;
    return e;
}

// The pipelined search rows when the plan's first and last passes take one butterfly per thread
// (10000 = 10⁴: 1000 butterflies of radix 10 in every pass): thread j < MC / R1 loads its first-pass
// inputs XT[j + r·nb] and code[j + r·nb] straight from memory (the next row's prefetched during the
// transform), forms their products and the first pass's butterfly in registers, and the last pass
// stores its outputs d[j + r·NsC_last] straight to memory — two LDS passes and two barriers per row
// fewer than staging the row in LDS, with the same operations in the same order (bit-identical).
template <int SIGN, int MC, bool HAS_B = true>
__global__ __launch_bounds__(kAcqThreads) void acq_huge_rows_reg_kernel(const float2* __restrict__ A, int64_t a_sy, int64_t a_sz,
    const float2* __restrict__ B, int64_t b_sy, int64_t b_sz, float2* __restrict__ D, int64_t d_sy, int64_t d_sz, const float2* __restrict__ twM,
    int P, int ny, int nz, int conj_out = 0)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    constexpr int R1 = ct_radix(MC), NB1 = MC / R1;
    constexpr int NL = ct_last_ns(MC), RL = MC / NL;
    static_assert(NB1 <= kAcqThreads && NL <= kAcqThreads && MC / RL == NL, "one butterfly per thread in the first and last passes");
    const int total = P * ny * nz;
    const int tid = threadIdx.x;
    for (int i = tid; i < MC / 4; i += kAcqThreads) lds[MC + i] = twM[i];
    const bool first = tid < NB1, last = tid < NL;
    // the stride-10 pass's butterfly for this thread (kLanePerm10): every 16-lane group's reads and
    // writes on distinct bank pairs
    const int jp10 = (MC == 10000) ? static_cast<int>(g_lane_perm10[tid]) : -2;
    float2 av[R1], bv[R1];  // the next row's first-pass inputs
    auto issue = [&](int r) {
        const int x = r % P, yz = r / P, y = yz % ny, z = yz / ny;
        const float2* a = A + y * a_sy + z * a_sz + static_cast<int64_t>(x) * MC;
        const int j = first ? tid : 0;
#pragma unroll
        for (int u = 0; u < R1; u++) av[u] = a[j + u * NB1];
        if constexpr (HAS_B) {
            const float2* b = B + y * b_sy + z * b_sz + static_cast<int64_t>(x) * MC;
#pragma unroll
            for (int u = 0; u < R1; u++) bv[u] = b[j + u * NB1];
        }
    };
    int r = blockIdx.x;
    if (r < total) issue(r);
    for (; r < total; r += gridDim.x) {
        float2 v[R1];
#pragma unroll
        for (int u = 0; u < R1; u++) v[u] = HAS_B ? cmulf(av[u], bv[u]) : av[u];  // XT ⊙ conj(code FFT) (search rows)
        if (r + static_cast<int>(gridDim.x) < total) issue(r + gridDim.x);  // in flight during this transform
        dft_small<R1, SIGN>(v);  // the first pass (NsC = 1: no twiddles)
        __syncthreads();         // the previous row's last pass has read the LDS
        if (first) store_run<R1>(lds + tid * R1, v);
        __syncthreads();
        int tid_r = tid;  // an opaque thread id: the passes' index arithmetic is not hoisted into registers
        asm volatile("" : "+v"(tid_r));
        fft_lds_ct_q<MC, R1, SIGN, NL>(lds, lds + MC, tid_r, jp10);
        const int x = r % P, yz = r / P, y = yz % ny, z = yz / ny;
        float2* d = D + y * d_sy + z * d_sz + static_cast<int64_t>(x) * MC;
        if (last) {
            float2 w[RL];
            ctq_bfly<MC, NL, SIGN>(lds, lds + MC, tid_r, w);  // the last pass
#pragma unroll
            for (int u = 0; u < RL; u++) {
                if (conj_out) w[u].y = -w[u].y;
                d[tid + u * NL] = w[u];
            }
        }
    }
}

// Inverse column stage + |y|² for cell (prn blockIdx.z, bin blockIdx.y): tile statistics, and the
// grid row g = grid + (z·n_bins + y)·N (accumulated over dwells when `accumulate`) only when a grid
// is kept — without one the |y|² never reach HBM (finalize recomputes the few columns it rescans).
template <int P>
__global__ __launch_bounds__(kHugeColThreads) void acq_huge_cols_inv_kernel(const float2* __restrict__ U, int M, int n_bins,
    const float2* __restrict__ twN, float* __restrict__ grid, int accumulate, TileStat* __restrict__ tiles, RowSpec rs)
{
    __shared__ MaxIdx red_m[kHugeColThreads / 64];
    __shared__ float red_s[kHugeColThreads / 64];
    const int m = blockIdx.x * kHugeColThreads + threadIdx.x;
    const int N = P * M;
    const int64_t cell = static_cast<int64_t>(blockIdx.z) * n_bins + blockIdx.y;
    MaxIdx best{-1.0f, 0x7fffffff};
    float s = 0.0f;
    if (m < M) {
        float2 v[P];
        huge_col_inv<P>(U + cell * N + m, m, M, twN, v);
        float* g = grid ? grid + cell * rs.row_len : nullptr;
#pragma unroll
        for (int q = 0; q < P; q++) {
            const int n = m + M * q - rs.row_off;  // index in the row
            if (n < 0 || n >= rs.row_len) continue;
            float mag = __fadd_rn(__fmul_rn(v[q].x, v[q].x), __fmul_rn(v[q].y, v[q].y));  // volk_32fc_magnitude_squared_32f
            if (g) {
                if (accumulate) mag = __fadd_rn(g[n], mag);  // volk_32f_x2_add_32f
                g[n] = mag;
            }
            best = better(best, MaxIdx{mag, n});
            s += mag;
        }
    }
    const MaxIdx bm = block_argmax<kHugeColThreads / 64>(best, red_m);
    const float bs = block_sum<kHugeColThreads / 64>(s, red_s);
    if (threadIdx.x == 0) tiles[cell * gridDim.x + blockIdx.x] = TileStat{bm.v, bm.i, bs, 0};
}

// Row statistics of cell (prn blockIdx.y, bin blockIdx.x) from its tiles and grid row.  Tile i
// holds columns m ∈ [256·i, 256·i + 256) of every register point q, i.e. row indices
// n = m + M·q − row_off.  The second peak (the largest |y|² outside the window around the peak,
// first_vs_second_peak_statistic :566-593) takes the maximum of every tile that misses the window
// from its tile statistic and rescans from the grid only the few tiles the window meets (the window
// is 2·spc consecutive indices: one or two column runs), instead of the whole row.
constexpr int kHugeFlagMax = 64;
// The finalize's work is the tile statistics of one cell (40-49 tiles) and the recomputation of the one
// or two tiles the window meets (one column per thread): 256 threads, four workgroups per CU (1024
// threads left 768 idle and held a CU per cell).
constexpr int kHugeFinThreads = 256;  // tiles met by the window that are rescanned together (more: full-row fallback)

__device__ __forceinline__ bool interval_meets(int a0, int a1, int b0, int b1) { return a0 < b1 && b0 < a1; }

// |y|² of row index n's column tile recomputed from U (grid-free mode): thread t of the block takes
// column lo + t % 256 and register point q = t / 256 … the whole tile's P·256 values, each thread
// folding the ones outside the window into v2.
template <int P>
__device__ __forceinline__ float huge_tile_max_outside(const float2* __restrict__ Ucell, int lo, int M, const float2* __restrict__ twN, RowSpec rs,
    int e1, int e2)
{
    float v2 = 0.0f;
    for (int c = threadIdx.x; c < kHugeColThreads; c += kHugeFinThreads) {
        const int mm = lo + c;
        if (mm >= M) continue;
        float2 v[P];
        huge_col_inv<P>(Ucell + mm, mm, M, twN, v);
#pragma unroll
        for (int q = 0; q < P; q++) {
            const int n = mm + M * q - rs.row_off;
            if (n < 0 || n >= rs.row_len) continue;
            const bool in_win = (e1 < e2) ? (n >= e1 && n < e2) : (n >= e1 || n < e2);
            const float mag = __fadd_rn(__fmul_rn(v[q].x, v[q].x), __fmul_rn(v[q].y, v[q].y));
            if (!in_win) v2 = fmaxf(v2, mag);
        }
    }
    return v2;
}

__global__ __launch_bounds__(kHugeFinThreads) void acq_huge_finalize_kernel(const float* __restrict__ grid, const TileStat* __restrict__ tiles,
    int n_tiles, int n_bins, int prn_offset, RowSpec rs, int M, int P, RowStat* __restrict__ rowstat, const float2* __restrict__ U,
    const float2* __restrict__ twN)
{
    __shared__ MaxIdx red_m[kHugeFinThreads / 64];
    __shared__ float red_s[kHugeFinThreads / 64];
    __shared__ int flag_list[kHugeFlagMax];
    __shared__ int n_flag;
    const int64_t cell = static_cast<int64_t>(blockIdx.y) * n_bins + blockIdx.x;
    const TileStat* ts = tiles + cell * n_tiles;
    if (threadIdx.x == 0) n_flag = 0;
    MaxIdx m{-1.0f, 0x7fffffff};
    float s = 0.0f;
    for (int i = threadIdx.x; i < n_tiles; i += kHugeFinThreads) {
        m = better(m, MaxIdx{ts[i].max, ts[i].argmax});
        s += ts[i].sum;
    }
    block_argmax_sum<kHugeFinThreads / 64>(m, s, red_m, red_s);  // its barriers also publish n_flag = 0
    const MaxIdx best = m;
    const float sum = s;
    int e1 = best.i - rs.spc, e2 = best.i + rs.spc;
    if (e1 < 0) e1 += rs.win_mod; else if (e2 >= rs.win_mod) e2 -= rs.win_mod;
    // the window as one or two row-index intervals
    const int w0a = e1 < e2 ? e1 : e1, w0b = e1 < e2 ? e2 : rs.win_mod;
    const int w1a = 0, w1b = e1 < e2 ? 0 : e2;
    float v2 = 0.0f;  // max(0, …): the reference's second peak starts from 0
    for (int i = threadIdx.x; i < n_tiles; i += kHugeFinThreads) {
        const int lo = i * kHugeColThreads, hi = min(M, lo + kHugeColThreads);
        bool meets = false;
        for (int q = 0; q < P; q++) {
            const int a0 = max(0, lo + M * q - rs.row_off), a1 = min(rs.row_len, hi + M * q - rs.row_off);
            if (a0 < a1 && (interval_meets(a0, a1, w0a, w0b) || interval_meets(a0, a1, w1a, w1b))) meets = true;
        }
        if (meets) {
            const int k = atomicAdd(&n_flag, 1);
            if (k < kHugeFlagMax) flag_list[k] = i;
        } else {
            v2 = fmaxf(v2, ts[i].max);
        }
    }
    __syncthreads();
    auto in_win = [&](int i) { return (e1 < e2) ? (i >= e1 && i < e2) : (i >= e1 || i < e2); };
    const int nf = n_flag;
    if (!grid) {  // grid-free: the met tiles (or, past kHugeFlagMax of them, every tile) recomputed from U
        const float2* Ucell = U + cell * static_cast<int64_t>(P) * M;
        const int cnt = nf <= kHugeFlagMax ? nf : n_tiles;
        for (int f = 0; f < cnt; f++) {
            const int lo = (nf <= kHugeFlagMax ? flag_list[f] : f) * kHugeColThreads;
            float t = 0.0f;
#define GNSSHIP_P_CASE(p) \
    case p: t = huge_tile_max_outside<p>(Ucell, lo, M, twN, rs, e1, e2); break;
            switch (P) { GNSSHIP_HUGE_P_LIST(GNSSHIP_P_CASE) default: break; }
#undef GNSSHIP_P_CASE
            v2 = fmaxf(v2, t);
        }
        const float second = block_max<kHugeFinThreads / 64>(v2, red_s);
        if (threadIdx.x == 0) rowstat[(static_cast<int64_t>(prn_offset) + blockIdx.y) * n_bins + blockIdx.x] = RowStat{best.v, best.i, sum, second};
        return;
    }
    const float* g = grid + cell * rs.row_len;
    if (nf <= kHugeFlagMax) {
        for (int f = 0; f < nf; f++) {
            const int lo = flag_list[f] * kHugeColThreads;
            for (int j = threadIdx.x; j < kHugeColThreads * P; j += kHugeFinThreads) {
                const int mm = lo + j % kHugeColThreads, q = j / kHugeColThreads;
                const int n = mm + M * q - rs.row_off;
                if (mm < M && n >= 0 && n < rs.row_len && !in_win(n)) v2 = fmaxf(v2, g[n]);
            }
        }
    } else {  // more tiles met than listed: scan the whole row
        for (int i = threadIdx.x; i < rs.row_len; i += kHugeFinThreads)
            if (!in_win(i)) v2 = fmaxf(v2, g[i]);
    }
    const float second = block_max<kHugeFinThreads / 64>(v2, red_s);
    if (threadIdx.x == 0) rowstat[(static_cast<int64_t>(prn_offset) + blockIdx.y) * n_bins + blockIdx.x] = RowStat{best.v, best.i, sum, second};
}


bool huge_ct_rows(int M) { return M == 10000 || M == 12500; }

bool huge_p_supported(int P)
{
#define GNSSHIP_P_CASE(p) \
    case p: return true;
    switch (P) { GNSSHIP_HUGE_P_LIST(GNSSHIP_P_CASE) default: return false; }
#undef GNSSHIP_P_CASE
}

hipError_t launch_acq_fft_huge(const void* sig, int fmt, const float2* mult, int n_rows, int P, const FftPlan& row_plan, const float2* twN,
    const float2* twM, float2* scratch, float2* rowsT, int conj_out, int n_valid, hipStream_t stream)
{
    const int M = row_plan.n;
    const int64_t N = static_cast<int64_t>(P) * M;
    const dim3 cgrid((M + kHugeColThreads - 1) / kHugeColThreads, n_rows);
#define GNSSHIP_P_CASE(p)                                                                                                                 \
    case p:                                                                                                                               \
        if (fmt == GNSSHIP_FMT_CF32)                                                                                                      \
            hipLaunchKernelGGL((acq_huge_cols_fwd_kernel<GNSSHIP_FMT_CF32, p>), cgrid, dim3(kHugeColThreads), 0, stream, sig, mult, M, twN, \
                scratch, n_valid);                                                                                                                 \
        else if (fmt == GNSSHIP_FMT_CI16)                                                                                                 \
            hipLaunchKernelGGL((acq_huge_cols_fwd_kernel<GNSSHIP_FMT_CI16, p>), cgrid, dim3(kHugeColThreads), 0, stream, sig, mult, M, twN, \
                scratch, n_valid);                                                                                                                 \
        else if (fmt == GNSSHIP_FMT_CI8)                                                                                                  \
            hipLaunchKernelGGL((acq_huge_cols_fwd_kernel<GNSSHIP_FMT_CI8, p>), cgrid, dim3(kHugeColThreads), 0, stream, sig, mult, M, twN,  \
                scratch, n_valid);                                                                                                                 \
        else                                                                                                                              \
            return hipErrorInvalidValue;                                                                                                  \
        break;
    switch (P) {
        GNSSHIP_HUGE_P_LIST(GNSSHIP_P_CASE)
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_P_CASE
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds = sizeof(float2) * static_cast<size_t>(M);
    const size_t lds_q = sizeof(float2) * static_cast<size_t>(M + M / 4);  // + the quarter twiddle table
    // the compile-time rows (huge_ct_rows): Galileo E1 at 25 Msps (N = 100000 = 10 × 10000), GPS/B1I at
    // 50 Msps (5 × 10000), E1 at 50 Msps (20 × 10000); 12500-point rows where 10000 does not divide N
#define GNSSHIP_CT_ROWS(mc)                                                                                                               \
    if (M == mc)                                                                                                                          \
        hipLaunchKernelGGL((acq_huge_rows_kernel<-1, mc>), dim3(P, n_rows, 1), dim3(kAcqThreads), lds_q, stream, scratch, N, int64_t(0), \
            static_cast<const float2*>(nullptr), int64_t(0), int64_t(0), rowsT, N, int64_t(0), row_plan, twM, conj_out);                  \
    else
    if (M == 10000) {  // persistent, first and last passes in registers (as the search rows)
        if (hipError_t pe = ensure_lane_perm10(); pe != hipSuccess) return pe;
        int n_cu = 256;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n_cu = 256;
        const int total = P * n_rows;
        hipLaunchKernelGGL((acq_huge_rows_reg_kernel<-1, 10000, false>), dim3(total < n_cu ? total : n_cu), dim3(kAcqThreads), lds_q, stream, scratch, N,
            int64_t(0), static_cast<const float2*>(nullptr), int64_t(0), int64_t(0), rowsT, N, int64_t(0), twM, P, n_rows, 1, conj_out);
    } else
    GNSSHIP_CT_ROWS(12500)
#undef GNSSHIP_CT_ROWS
        hipLaunchKernelGGL((acq_huge_rows_kernel<-1>), dim3(P, n_rows, 1), dim3(kAcqThreads), lds, stream, scratch, N, int64_t(0),
            static_cast<const float2*>(nullptr), int64_t(0), int64_t(0), rowsT, N, int64_t(0), row_plan, twM, conj_out);
    return hipGetLastError();
}

hipError_t launch_acq_search_huge(const float2* XT, const float2* codesT, int prn_offset, int n_prns, int n_bins, int P, const FftPlan& row_plan,
    const float2* twN, const float2* twM, float2* U, float* grid, int accumulate, TileStat* tiles, RowSpec rs, RowStat* rowstat,
    hipStream_t stream)
{
    const int M = row_plan.n;
    const int64_t N = static_cast<int64_t>(P) * M;
    const size_t lds = sizeof(float2) * static_cast<size_t>(M);
    const size_t lds_q = sizeof(float2) * static_cast<size_t>(M + M / 4);
    // rows: blockIdx.y = bin (XT row set), blockIdx.z = prn (code spectrum), U cell = z·n_bins + y
    if (huge_ct_rows(M)) {
        // persistent: one workgroup per CU (100 or 125 KB of LDS each), rows pipelined through it
        int n_cu = 256;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n_cu = 256;
        const int total = P * n_bins * n_prns;
        const int blocks = total < n_cu ? total : n_cu;
        if (M == 10000 && ensure_lane_perm10() != hipSuccess) return hipErrorInvalidValue;
        if (M == 10000)
            hipLaunchKernelGGL((acq_huge_rows_reg_kernel<+1, 10000>), dim3(blocks), dim3(kAcqThreads), lds_q, stream, XT, N, int64_t(0),
                codesT + static_cast<int64_t>(prn_offset) * N, int64_t(0), N, U, N, N * n_bins, twM, P, n_bins, n_prns);
        else
            hipLaunchKernelGGL((acq_huge_rows_pipe_kernel<+1, 12500>), dim3(blocks), dim3(kAcqThreads), lds_q, stream, XT, N, int64_t(0),
                codesT + static_cast<int64_t>(prn_offset) * N, int64_t(0), N, U, N, N * n_bins, twM, P, n_bins, n_prns);
    }
    else
        hipLaunchKernelGGL((acq_huge_rows_kernel<+1>), dim3(P, n_bins, n_prns), dim3(kAcqThreads), lds, stream, XT, N, int64_t(0),
            codesT + static_cast<int64_t>(prn_offset) * N, int64_t(0), N, U, N, N * n_bins, row_plan, twM, 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int n_tiles = (M + kHugeColThreads - 1) / kHugeColThreads;
    const dim3 cgrid(n_tiles, n_bins, n_prns);
#define GNSSHIP_P_CASE(p)                                                                                                              \
    case p:                                                                                                                            \
        hipLaunchKernelGGL((acq_huge_cols_inv_kernel<p>), cgrid, dim3(kHugeColThreads), 0, stream, U, M, n_bins, twN, grid, accumulate, \
            tiles, rs);                                                                                                                    \
        break;
    switch (P) {
        GNSSHIP_HUGE_P_LIST(GNSSHIP_P_CASE)
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_P_CASE
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(acq_huge_finalize_kernel, dim3(n_bins, n_prns), dim3(kHugeFinThreads), 0, stream, grid, tiles, n_tiles, n_bins, prn_offset, rs,
        M, P, rowstat, U, twN);
    return hipGetLastError();
}

hipError_t launch_acq_fft_rows(const void* sig, int fmt, const float2* mult, int n_rows, const FftPlan& plan, const float2* tw, float2* rows,
    int conj_out, int n_valid, hipStream_t stream)
{
    const size_t lds = sizeof(float2) * static_cast<size_t>(plan.n) * (plan.n <= kTwLdsMax ? 2 : 1);
    switch (fmt) {
    case GNSSHIP_FMT_CF32:
        hipLaunchKernelGGL(acq_fft_rows_kernel<GNSSHIP_FMT_CF32>, dim3(n_rows), dim3(kAcqThreads), lds, stream, sig, mult, plan, tw, rows, conj_out, n_valid);
        break;
    case GNSSHIP_FMT_CI16:
        hipLaunchKernelGGL(acq_fft_rows_kernel<GNSSHIP_FMT_CI16>, dim3(n_rows), dim3(kAcqThreads), lds, stream, sig, mult, plan, tw, rows, conj_out, n_valid);
        break;
    case GNSSHIP_FMT_CI8:
        hipLaunchKernelGGL(acq_fft_rows_kernel<GNSSHIP_FMT_CI8>, dim3(n_rows), dim3(kAcqThreads), lds, stream, sig, mult, plan, tw, rows, conj_out, n_valid);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_acq_search(const float2* X, const float2* codes_fft, int n_prns, int n_bins, const FftPlan& plan, const float2* tw,
    RowSpec rs, int accumulate, RowStat* rowstat, float* grid, hipStream_t stream)
{
    const size_t lds = sizeof(float2) * static_cast<size_t>(plan.n) * (plan.n <= kTwLdsMax ? 2 : 1);
    hipLaunchKernelGGL(acq_search_kernel, dim3(n_bins, n_prns), dim3(kAcqThreads), lds, stream, X, codes_fft, plan, tw, n_bins,
        rs, accumulate, rowstat, grid);
    return hipGetLastError();
}

#define GNSSHIP_BIG_P_LIST(X) X(16) X(18) X(20) X(24) X(25) X(27) X(30) X(32)

bool big_p_supported(int P)
{
#define GNSSHIP_P_CASE(p) \
    case p: return true;
    switch (P) { GNSSHIP_BIG_P_LIST(GNSSHIP_P_CASE) default: return false; }
#undef GNSSHIP_P_CASE
}

hipError_t launch_acq_fft_big(const void* sig, int fmt, const float2* mult, int n_rows, int P, const FftPlan& row_plan, const float2* tw,
    float2* rowsT, int conj_out, int n_valid, hipStream_t stream)
{
    const int M = row_plan.n;
    if (M > kAcqThreads) return hipErrorInvalidValue;
    const dim3 cgrid((M + kBigColThreads - 1) / kBigColThreads, n_rows);
#define GNSSHIP_P_CASE(p)                                                                                                            \
    case p:                                                                                                                          \
        if (fmt == GNSSHIP_FMT_CF32)                                                                                                 \
            hipLaunchKernelGGL((acq_fft_big_cols_kernel<GNSSHIP_FMT_CF32, p>), cgrid, dim3(kBigColThreads), 0, stream, sig, mult, M, tw, \
                rowsT, n_valid);                                                                                                     \
        else if (fmt == GNSSHIP_FMT_CI16)                                                                                            \
            hipLaunchKernelGGL((acq_fft_big_cols_kernel<GNSSHIP_FMT_CI16, p>), cgrid, dim3(kBigColThreads), 0, stream, sig, mult, M, tw, \
                rowsT, n_valid);                                                                                                     \
        else if (fmt == GNSSHIP_FMT_CI8)                                                                                             \
            hipLaunchKernelGGL((acq_fft_big_cols_kernel<GNSSHIP_FMT_CI8, p>), cgrid, dim3(kBigColThreads), 0, stream, sig, mult, M, tw,  \
                rowsT, n_valid);                                                                                                     \
        else                                                                                                                         \
            return hipErrorInvalidValue;                                                                                             \
        break;
    switch (P) {
        GNSSHIP_BIG_P_LIST(GNSSHIP_P_CASE)
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_P_CASE
    const int rows_total = n_rows * P;
    const size_t lds = (static_cast<size_t>(kBigRowWaves) + 1) * sizeof(float2) * M;
    const dim3 rgrid((rows_total + kBigRowWaves - 1) / kBigRowWaves);
    if (M == 1000)  // C3: N = 25000 (GPS 1 ms at 25 Msps), compile-time row plan
        hipLaunchKernelGGL((acq_fft_big_rows_kernel<1000>), rgrid, dim3(kBigRowWaves * 64), lds, stream, row_plan, P, tw, rowsT, rows_total, conj_out);
    else if (M == 250)  // C1: N = 4000 (GPS 1 ms at 4 Msps) as 16 × 250
        hipLaunchKernelGGL((acq_fft_big_rows_kernel<250>), rgrid, dim3(kBigRowWaves * 64), lds, stream, row_plan, P, tw, rowsT, rows_total, conj_out);
    else
        hipLaunchKernelGGL((acq_fft_big_rows_kernel<0>), rgrid, dim3(kBigRowWaves * 64), lds, stream, row_plan, P, tw, rowsT, rows_total, conj_out);
    return hipGetLastError();
}

hipError_t launch_acq_search_big(const float2* XT, const float2* codesT, int n_prns, int n_bins, int P, const FftPlan& row_plan,
    const float2* tw, RowSpec rs, int accumulate, RowStat* rowstat, float* grid, hipStream_t stream)
{
    const size_t lds = (static_cast<size_t>(kWaveRows) + 1) * sizeof(float2) * row_plan.n;
    if (row_plan.n > kAcqThreads) return hipErrorInvalidValue;
    if (P == 25 && row_plan.n == 1000) {  // C3: N = 25000
        hipLaunchKernelGGL((acq_search_big_kernel<25, 1000>), dim3(n_bins, n_prns), dim3(kAcqThreads), lds, stream, XT, codesT, row_plan, tw, n_bins,
            rs, accumulate, rowstat, grid);
        return hipGetLastError();
    }
    if (P == 16 && row_plan.n == 250) {  // C1: N = 4000 in 256-thread workgroups (several per CU)
        constexpr int kNT = 256;
        const size_t lds_c1 = (static_cast<size_t>(kNT / 64) + 1) * sizeof(float2) * 250;
        hipLaunchKernelGGL((acq_search_big_kernel<16, 250, kNT>), dim3(n_bins, n_prns), dim3(kNT), lds_c1, stream, XT, codesT, row_plan, tw, n_bins,
            rs, accumulate, rowstat, grid);
        return hipGetLastError();
    }
#define GNSSHIP_P_CASE(p)                                                                                                            \
    case p:                                                                                                                          \
        hipLaunchKernelGGL((acq_search_big_kernel<p>), dim3(n_bins, n_prns), dim3(kAcqThreads), lds, stream, XT, codesT, row_plan, tw, \
            n_bins, rs, accumulate, rowstat, grid);                                                                    \
        break;
    switch (P) {
        GNSSHIP_BIG_P_LIST(GNSSHIP_P_CASE)
    default: return hipErrorInvalidValue;
    }
#undef GNSSHIP_P_CASE
    return hipGetLastError();
}

hipError_t launch_acq_decide(const RowStat* rowstat, int n_prns, int n_bins, int N, int doppler_max, int doppler_step, int doppler_center,
    int dwells, int use_cfar, float samples_per_code, float resampler_ratio, uint32_t resampler_latency, Step2Spec step2, gnsship_acq_result* out,
    hipStream_t stream)
{
    hipLaunchKernelGGL(acq_decide_kernel, dim3(n_prns), dim3(64), 0, stream, rowstat, n_prns, n_bins, N, doppler_max, doppler_step,
        doppler_center, dwells, use_cfar, samples_per_code, resampler_ratio, resampler_latency, step2, out);
    return hipGetLastError();
}

}  // namespace gnsship

#ifdef GNSSHIP_CORR_PROFILE
extern "C" int gnsship_debug_acq_profile(void* dev_buf)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(gnsship::g_acq_prof), &dev_buf, sizeof(void*)) == hipSuccess ? 0 : -3;
}
#endif
