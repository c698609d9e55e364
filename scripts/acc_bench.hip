// Microbenchmark: shader cycles of trk_fast.hip's accumulator pattern on one wave of a lone workgroup —
// dependent v_add_f32 chains (1, 2 or 4 interleaved per lane) over 16-byte LDS loads, per 32-iteration
// group, with the flag read between groups; and the bare dependent-add latency.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/acc_bench.hip -o scripts/acc_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// NS interleaved serial chains per lane, G groups of 32 iterations, each group 8·NS b128 loads
template <int NS, bool FLAG>
__global__ void acc_k(float* out, unsigned long long* cyc, int groups)
{
    __shared__ __attribute__((aligned(16))) float P[2 * 6 * 16 * 36];
    __shared__ int ready[16];
    const int lane = threadIdx.x;
    for (int i = lane; i < 2 * 6 * 16 * 36; i += 64) P[i] = 1e-3f * (i & 7);
    if (lane < 16) ready[lane] = 1;
    __syncthreads();
    const int l = lane & 15, r = lane >> 4;
    float acc[NS];
    int off[NS];
    for (int k = 0; k < NS; k++) {
        acc[k] = 0.0f;
        off[k] = (r + 4 * k) % 6 * 576 + l * 36;
    }
    unsigned long long t0 = clock64();
    for (int g = 0; g < groups; g++) {
        if (FLAG)
            while (__hip_atomic_load(ready + (g & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 1) __builtin_amdgcn_s_sleep(0);
        asm volatile("" ::: "memory");
        const float* src = P + (g & 1) * 3456;
        f4 v[8][NS];
#pragma unroll
        for (int q = 0; q < 8; q++)
#pragma unroll
            for (int k = 0; k < NS; k++) v[q][k] = *reinterpret_cast<const f4*>(src + off[k] + 4 * q);
#pragma unroll
        for (int q = 0; q < 8; q++)
#pragma unroll
            for (int k = 0; k < NS; k++)
#pragma unroll
                for (int u = 0; u < 4; u++) acc[k] = __fadd_rn(acc[k], v[q][k][u]);
#pragma unroll
        for (int k = 0; k < NS; k++) asm volatile("" ::"v"(acc[k]) : "memory");
    }
    unsigned long long t1 = clock64();
    float s = 0.0f;
    for (int k = 0; k < NS; k++) s += acc[k];
    out[lane] = s;
    if (lane == 0) *cyc = t1 - t0;
}

// bare dependent chain: N v_add_f32 in one asm block (no loads)
template <int CH>
__global__ void chain_k(float* out, unsigned long long* cyc, float x)
{
    float a0 = x + threadIdx.x, a1 = a0 + 1.0f, a2 = a0 + 2.0f, a3 = a0 + 3.0f;
    unsigned long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < 64; i++) {
        if constexpr (CH == 1)
            asm volatile(".rept 32\n\tv_add_f32 %0, %0, %1\n\t.endr" : "+v"(a0) : "v"(x));
        else if constexpr (CH == 2)
            asm volatile(".rept 16\n\tv_add_f32 %0, %0, %2\n\tv_add_f32 %1, %1, %2\n\t.endr" : "+v"(a0), "+v"(a1) : "v"(x));
        else
            asm volatile(".rept 8\n\tv_add_f32 %0, %0, %4\n\tv_add_f32 %1, %1, %4\n\tv_add_f32 %2, %2, %4\n\tv_add_f32 %3, %3, %4\n\t.endr"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                         : "v"(x));
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = a0 + a1 + a2 + a3;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main()
{
    float* out;
    unsigned long long* cyc;
    if (hipMalloc(&out, 256 * sizeof(float)) != hipSuccess || hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
    auto best = [&](auto launch) {
        unsigned long long b = ~0ull;
        for (int rep = 0; rep < 5; rep++) {
            launch();
            unsigned long long c = 0;
            if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return ~0ull;
            if (c < b) b = c;
        }
        return b;
    };
    const int G = 64;
    unsigned long long c;
    c = best([&] { hipLaunchKernelGGL((chain_k<1>), 1, 64, 0, 0, out, cyc, 1e-7f); });
    printf("bare chain 1 x 32 adds: %.2f cycles per dependent add (%.2f per add issued)\n", c / (64.0 * 32), c / (64.0 * 32));
    c = best([&] { hipLaunchKernelGGL((chain_k<2>), 1, 64, 0, 0, out, cyc, 1e-7f); });
    printf("bare chains 2 x 16 adds: %.2f cycles per add issued\n", c / (64.0 * 32));
    c = best([&] { hipLaunchKernelGGL((chain_k<4>), 1, 64, 0, 0, out, cyc, 1e-7f); });
    printf("bare chains 4 x 8 adds: %.2f cycles per add issued\n", c / (64.0 * 32));
    c = best([&] { hipLaunchKernelGGL((acc_k<1, false>), 1, 64, 0, 0, out, cyc, G); });
    printf("acc NS=1 (8 b128 + 32 adds per group): %.1f cycles per group\n", c / double(G));
    c = best([&] { hipLaunchKernelGGL((acc_k<1, true>), 1, 64, 0, 0, out, cyc, G); });
    printf("acc NS=1 + flag poll: %.1f cycles per group\n", c / double(G));
    c = best([&] { hipLaunchKernelGGL((acc_k<2, true>), 1, 64, 0, 0, out, cyc, G); });
    printf("acc NS=2 + flag poll (16 b128 + 64 adds): %.1f cycles per group\n", c / double(G));
    return 0;
}
