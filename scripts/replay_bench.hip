// Microbenchmark: shader cycles of trk_fast.hip's phasor replay (fast_replay, same code) on one wave
// of a lone workgroup, with and without its slot stores and normalisations.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude -Ignss_sim_receiver_amd/csrc \
//       scripts/replay_bench.hip -o scripts/replay_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "corr_device.h"

#ifndef POLL_SLEEP
#define POLL_SLEEP 0
#endif

using namespace gnsship;

template <int G, bool STORE, bool NORM>
__device__ __forceinline__ f2 replay(f2 z, f2 dz, int S, uint64_t* __restrict__ Zs, int l)
{
    constexpr int kTB = 64 / G;
    const int full = (S - 1) / kTB;
    uint64_t* p = Zs + l;
#pragma unroll 1
    for (int b = 0; b < full; b++) {
#pragma unroll
        for (int u = 0; u < kTB; u++) {
            if (STORE) __hip_atomic_store(p, __builtin_bit_cast(uint64_t, z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p += kAvxLanes;
            if (u == 0 && NORM)
                z = cmul_pow_s<G - 1>(normalise_avx(cmul_exact_s(z, dz)), dz);
            else
                z = cmul_pow_s<G>(z, dz);
        }
    }
#pragma unroll 1
    for (int t = full * kTB; t < S - 1; t++) {
        if (STORE) __hip_atomic_store(p, __builtin_bit_cast(uint64_t, z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        p += kAvxLanes;
        z = cmul_exact_s(z, dz);
        if (t == full * kTB && NORM) z = normalise_avx(z);
        z = cmul_pow_s<G - 1>(z, dz);
    }
    return z;
}

// Two lanes per phasor chain (lane 2l: re, lane 2l + 1: im): per product one plain multiply, one DPP
// multiply by the neighbour lane's component and one add; 2 wait states between the add and the next
// DPP read of its result.  The slot store is a 32-bit half per lane, issued in the same block.
#define PSTEP(X, Y)                                                          \
    "v_mul_f32 %[t], %[c], " X "\n\t"                                     \
    "s_nop 0\n\t"                                                          \
    "v_mul_f32_dpp %[u], " X ", %[k2] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t" \
    "v_add_f32 " Y ", %[t], %[u]\n\t"

template <int G, bool STORE, bool NORM>
__device__ __forceinline__ float replay2(float x, float c, float k2, int S, uint32_t* __restrict__ Zh, int lane)
{
    constexpr int kTB = 64 / G;
    static_assert(G == 4, "bench: G = 4");
    const int full = (S - 1) / kTB;
    uint32_t* p = Zh + lane;  // 32-bit halves: chain l's slot = halves 2l, 2l + 1
    float t, u, w, v;
#pragma unroll 1
    for (int b = 0; b < full; b++) {
#pragma unroll
        for (int q = 0; q < kTB; q++) {
            if (q == 0 && NORM) {
                if (STORE) __hip_atomic_store(p, __builtin_bit_cast(uint32_t, x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                asm volatile(PSTEP("%[x]", "%[x]") "s_nop 1\n\t" : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u) : [c] "s"(c), [k2] "v"(k2));
                const float s2 = __fmul_rn(x, x);
                const float m = __fsqrt_rn(__fadd_rn(s2, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s2), 0xB1, 0xF, 0xF, false))));
                x = __fdiv_rn(x, m);
                asm volatile(PSTEP("%[x]", "%[w]") PSTEP("%[w]", "%[v]") PSTEP("%[v]", "%[x]")
                             : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [v] "=&v"(v)
                             : [c] "s"(c), [k2] "v"(k2));
            } else if (STORE) {
                asm volatile(PSTEP("%[x]", "%[w]") "ds_write_b32 %[p], %[x] offset:0\n\t"
                             PSTEP("%[w]", "%[v]") PSTEP("%[v]", "%[w]") PSTEP("%[w]", "%[x]")
                             : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [v] "=&v"(v)
                             : [c] "s"(c), [k2] "v"(k2), [p] "v"(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)))
                             : "memory");
            } else {
                asm volatile(PSTEP("%[x]", "%[w]") PSTEP("%[w]", "%[v]") PSTEP("%[v]", "%[w]") PSTEP("%[w]", "%[x]")
                             : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w), [v] "=&v"(v)
                             : [c] "s"(c), [k2] "v"(k2));
            }
            p += 2 * kAvxLanes;
        }
    }
    return x;
}

template <bool STORE, bool NORM>
__global__ void k2(float* out, unsigned long long* cyc, float dzr, float dzi, int S, int busy = 0, int prio = 0)
{
    __shared__ uint64_t Zs[64 * 16 * 4];
    __shared__ int done;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (threadIdx.x >= 64) {  // pollers (launched with 256 threads): spin on LDS until wave 0 is done
        uint64_t acc = 0;
        float f0 = threadIdx.x * 1e-3f, f1 = f0 + 1.0f, f2v = f0 + 2.0f, f3 = f0 + 3.0f;
        while (__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
            if (busy) {  // VALU-bound neighbours (the correlating waves' load): independent FMA chains
#pragma unroll
                for (int i = 0; i < 64; i++) {
                    f0 = __builtin_fmaf(f0, 0.999f, 1e-3f);
                    f1 = __builtin_fmaf(f1, 0.999f, 1e-3f);
                    f2v = __builtin_fmaf(f2v, 0.999f, 1e-3f);
                    f3 = __builtin_fmaf(f3, 0.999f, 1e-3f);
                }
            } else {
                acc += __hip_atomic_load(Zs + (threadIdx.x & 255), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (POLL_SLEEP >= 0) __builtin_amdgcn_s_sleep(POLL_SLEEP > 0 ? POLL_SLEEP : 0);
            }
        }
        out[threadIdx.x] = static_cast<float>(acc) + f0 + f1 + f2v + f3;
        return;
    }
    if (prio) __builtin_amdgcn_s_setprio(3);
    float x = (lane & 1) ? (lane >> 1) * 1e-3f : 1.0f - (lane >> 1) * 1e-3f;
    const float c = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, dzr)));
    const float k2v = (lane & 1) ? dzi : -dzi;
    unsigned long long t0 = clock64();
    if (lane < 32) x = replay2<4, STORE, NORM>(x, c, k2v, S, reinterpret_cast<uint32_t*>(Zs), lane);
    unsigned long long t1 = clock64();
    out[lane] = x + (STORE ? __builtin_bit_cast(float, static_cast<uint32_t>(Zs[lane * 7])) : 0.0f);
    if (lane == 0) *cyc = t1 - t0;
    if (lane == 0) __hip_atomic_store(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool STORE, bool NORM>
__global__ void k(float* out, unsigned long long* cyc, float dzr, float dzi, int S)
{
    __shared__ uint64_t Zs[64 * 16 * 4];
    const int lane = threadIdx.x;
    f2 z = f2{1.0f - lane * 1e-3f, lane * 1e-3f};
    const f2 dz = f2{__builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, dzr))),
        __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, dzi)))};
    __syncthreads();
    unsigned long long t0 = clock64();
    if (lane < 16) z = replay<4, STORE, NORM>(z, dz, S, Zs, lane);
    unsigned long long t1 = clock64();
    out[lane] = z.x + z.y + (STORE ? __builtin_bit_cast(float, static_cast<uint32_t>(Zs[lane * 7])) : 0.0f);
    if (lane == 0) *cyc = t1 - t0;
}

int main()
{
    float* out;
    unsigned long long* cyc;
    if (hipMalloc(&out, 256 * sizeof(float)) != hipSuccess || hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
    const int S = 63;  // C2: 4000 samples, 250 iterations, 4-iteration tasks
    for (int v = 0; v < 13; v++) {
        unsigned long long best = ~0ull;
        for (int rep = 0; rep < 5; rep++) {
            switch (v) {
            case 0: hipLaunchKernelGGL((k<true, true>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 1: hipLaunchKernelGGL((k<false, true>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 2: hipLaunchKernelGGL((k<true, false>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 3: hipLaunchKernelGGL((k<false, false>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 4: hipLaunchKernelGGL((k2<true, true>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 5: hipLaunchKernelGGL((k2<false, true>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 6: hipLaunchKernelGGL((k2<true, false>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 7: hipLaunchKernelGGL((k2<false, false>), 1, 64, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 8: hipLaunchKernelGGL((k2<true, true>), 1, 256, 0, 0, out, cyc, 0.99f, 0.14f, S); break;
            case 9: hipLaunchKernelGGL((k2<false, false>), 1, 256, 0, 0, out, cyc, 0.99f, 0.14f, S, 0, 0); break;
            case 10: hipLaunchKernelGGL((k2<true, true>), 1, 256, 0, 0, out, cyc, 0.99f, 0.14f, S, 1, 0); break;
            case 11: hipLaunchKernelGGL((k2<true, true>), 1, 256, 0, 0, out, cyc, 0.99f, 0.14f, S, 1, 1); break;
            default: hipLaunchKernelGGL((k2<true, true>), 1, 256, 0, 0, out, cyc, 0.99f, 0.14f, S, 0, 1); break;
            }
            unsigned long long c = 0;
            if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 2;
            if (c < best) best = c;
        }
        printf("%s stores %d normalise %d: %llu cycles for 250 iterations (%.1f / iteration)\n",
            v < 4 ? "1-lane" : v < 8 ? "2-lane DPP" : v < 10 ? "2-lane DPP + 3 polling waves" : v == 10 ? "2-lane DPP + 3 VALU-busy waves" : v == 11 ? "2-lane DPP + 3 VALU-busy waves, setprio 3" : "2-lane DPP + 3 polling waves, setprio 3",
            v == 8 || v >= 10 || (v < 8 && (v & 1) == 0), v == 8 || v >= 10 || (v < 8 && (v & 3) < 2),
            best, best / 250.0);
    }
    return 0;
}
