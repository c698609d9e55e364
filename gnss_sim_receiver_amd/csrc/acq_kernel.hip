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
#include "acq_engine.h"

namespace gnsship {

__device__ __forceinline__ float2 cmulf(float2 a, float2 b)
{
    return make_float2(__fsub_rn(__fmul_rn(a.x, b.x), __fmul_rn(a.y, b.y)), __fadd_rn(__fmul_rn(a.x, b.y), __fmul_rn(a.y, b.x)));
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
                    float2 w = tw[(k * r * tstep) % N];
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

// rows[b] = FFT(sig ⊙ mult[b])  (mult == nullptr: FFT(sig)); conj_out: store conj (code FFT).
template <int FMT>
__global__ __launch_bounds__(kAcqThreads) void acq_fft_rows_kernel(const void* __restrict__ sig, const float2* __restrict__ mult,
    FftPlan plan, const float2* __restrict__ tw, float2* __restrict__ rows, int conj_out)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int N = plan.n;
    const float2* m = mult ? mult + static_cast<int64_t>(b) * N : nullptr;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        float2 x = load_if<FMT>(sig, i);
        if (m) x = cmulf(x, m[i]);  // volk_32fc_x2_multiply_32fc(in, wipeoff)
        lds[i] = x;
    }
    __syncthreads();
    fft_lds<-1>(lds, plan, tw);
    float2* out = rows + static_cast<int64_t>(b) * N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        float2 y = lds[i];
        if (conj_out) y.y = -y.y;
        out[i] = y;
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

__device__ __forceinline__ MaxIdx block_argmax(MaxIdx m, MaxIdx* red)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        MaxIdx q;
        q.v = __shfl_xor(m.v, o, 64);
        q.i = __shfl_xor(m.i, o, 64);
        m = better(m, q);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = m;
    __syncthreads();
    MaxIdx r = red[0];
    for (int w = 1; w < static_cast<int>(blockDim.x >> 6); w++) r = better(r, red[w]);
    __syncthreads();
    return r;
}

__device__ __forceinline__ float block_sum(float s, float* red)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = s;
    __syncthreads();
    float r = 0.0f;
    for (int w = 0; w < static_cast<int>(blockDim.x >> 6); w++) r += red[w];
    __syncthreads();
    return r;
}

// grid: (n_bins, n_prns).  rowstat[(p*n_bins + b)] ; grid_out optional [p][b][N].
__global__ __launch_bounds__(kAcqThreads) void acq_search_kernel(const float2* __restrict__ X, const float2* __restrict__ codes_fft,
    FftPlan plan, const float2* __restrict__ tw, int n_bins, int samples_per_chip, int accumulate, RowStat* __restrict__ rowstat,
    float* __restrict__ grid_out)
{
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ MaxIdx red_m[kAcqThreads / 64];
    __shared__ float red_s[kAcqThreads / 64];
    const int b = blockIdx.x, p = blockIdx.y;
    const int N = plan.n;
    const float2* x = X + static_cast<int64_t>(b) * N;
    const float2* c = codes_fft + static_cast<int64_t>(p) * N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) lds[i] = cmulf(x[i], c[i]);  // ×conj(code FFT)
    __syncthreads();
    fft_lds<+1>(lds, plan, tw);
    // |Y|² in place (as float in the .x slot) + optional grid row (accumulated over dwells)
    float* row = grid_out ? grid_out + (static_cast<int64_t>(p) * n_bins + b) * N : nullptr;
    MaxIdx m{-1.0f, 0x7fffffff};
    float s = 0.0f;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const float2 y = lds[i];
        float mag = __fadd_rn(__fmul_rn(y.x, y.x), __fmul_rn(y.y, y.y));  // volk_32fc_magnitude_squared_32f
        if (row) {
            if (accumulate) mag = __fadd_rn(row[i], mag);  // volk_32f_x2_add_32f
            row[i] = mag;
        }
        lds[i].x = mag;
        m = better(m, MaxIdx{mag, i});
        s += mag;
    }
    const MaxIdx best = block_argmax(m, red_m);
    const float sum = block_sum(s, red_s);
    // second peak outside the circular window [best-spc, best+spc) (first_vs_second_peak_statistic :566-593)
    int e1 = best.i - samples_per_chip, e2 = best.i + samples_per_chip;
    if (e1 < 0) e1 += N; else if (e2 >= N) e2 -= N;
    MaxIdx m2{0.0f, 0x7fffffff};
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const bool in_win = (e1 < e2) ? (i >= e1 && i < e2) : (i >= e1 || i < e2);
        const float v = in_win ? 0.0f : lds[i].x;
        m2 = better(m2, MaxIdx{v, i});
    }
    const MaxIdx second = block_argmax(m2, red_m);
    if (threadIdx.x == 0) {
        RowStat r;
        r.max = best.v;
        r.argmax = best.i;
        r.sum = sum;
        r.second = second.v;
        rowstat[static_cast<int64_t>(p) * n_bins + b] = r;
    }
}

// One thread per PRN: the reference's row scan (strict >, ascending bin) and decision values.
__global__ void acq_decide_kernel(const RowStat* __restrict__ rowstat, int n_prns, int n_bins, int N, int doppler_max, int doppler_step,
    int doppler_center, int dwells, int use_cfar, float samples_per_code, gnsship_acq_result* __restrict__ out)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_prns) return;
    const RowStat* rs = rowstat + static_cast<int64_t>(p) * n_bins;
    float gmax = 0.0f;
    int bi = 0, ti = 0;
    for (int b = 0; b < n_bins; b++) {
        if (rs[b].max > gmax) {
            gmax = rs[b].max;
            bi = b;
            ti = rs[b].argmax;
        }
    }
    gnsship_acq_result r;
    r.doppler_index = static_cast<uint32_t>(bi);
    r.code_index = static_cast<uint32_t>(ti);
    r.doppler_hz = -doppler_max + doppler_center + doppler_step * bi;
    r.peak = gmax;
    if (use_cfar) {
        const int opp = (bi + n_bins / 2) % n_bins;
        // (float)(sum / N / 2.0 / dwells)  (pcps_acquisition.cc:518)
        const float s = rs[opp].sum;
        r.input_power = static_cast<float>(static_cast<double>(s / static_cast<float>(N)) / 2.0 / static_cast<double>(dwells));
        r.test_statistic = gmax / r.input_power;
    } else {
        r.input_power = rs[bi].second;
        r.test_statistic = gmax / rs[bi].second;
    }
    r.acq_delay_samples = static_cast<double>(fmodf(static_cast<float>(ti), samples_per_code));
    out[p] = r;
}

hipError_t launch_acq_fft_rows(const void* sig, int fmt, const float2* mult, int n_rows, const FftPlan& plan, const float2* tw, float2* rows,
    int conj_out, hipStream_t stream)
{
    const size_t lds = sizeof(float2) * static_cast<size_t>(plan.n);
    switch (fmt) {
    case GNSSHIP_FMT_CF32:
        hipLaunchKernelGGL(acq_fft_rows_kernel<GNSSHIP_FMT_CF32>, dim3(n_rows), dim3(kAcqThreads), lds, stream, sig, mult, plan, tw, rows, conj_out);
        break;
    case GNSSHIP_FMT_CI16:
        hipLaunchKernelGGL(acq_fft_rows_kernel<GNSSHIP_FMT_CI16>, dim3(n_rows), dim3(kAcqThreads), lds, stream, sig, mult, plan, tw, rows, conj_out);
        break;
    case GNSSHIP_FMT_CI8:
        hipLaunchKernelGGL(acq_fft_rows_kernel<GNSSHIP_FMT_CI8>, dim3(n_rows), dim3(kAcqThreads), lds, stream, sig, mult, plan, tw, rows, conj_out);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_acq_search(const float2* X, const float2* codes_fft, int n_prns, int n_bins, const FftPlan& plan, const float2* tw,
    int samples_per_chip, int accumulate, RowStat* rowstat, float* grid, hipStream_t stream)
{
    const size_t lds = sizeof(float2) * static_cast<size_t>(plan.n);
    hipLaunchKernelGGL(acq_search_kernel, dim3(n_bins, n_prns), dim3(kAcqThreads), lds, stream, X, codes_fft, plan, tw, n_bins,
        samples_per_chip, accumulate, rowstat, grid);
    return hipGetLastError();
}

hipError_t launch_acq_decide(const RowStat* rowstat, int n_prns, int n_bins, int N, int doppler_max, int doppler_step, int doppler_center,
    int dwells, int use_cfar, float samples_per_code, gnsship_acq_result* out, hipStream_t stream)
{
    hipLaunchKernelGGL(acq_decide_kernel, dim3((n_prns + 63) / 64), dim3(64), 0, stream, rowstat, n_prns, n_bins, N, doppler_max, doppler_step,
        doppler_center, dwells, use_cfar, samples_per_code, out);
    return hipGetLastError();
}

}  // namespace gnsship
