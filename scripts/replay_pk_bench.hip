// Microbenchmark: shader cycles per step of the phasor chain z <- z*dz on one lone wave, in two forms:
//   dpp: trk_fast.hip's two lanes per chain (v_mul, s_nop, v_mul_dpp, v_add);
//   pk : one lane per chain with z in a VGPR pair (v_pk_mul, v_pk_mul with swapped halves, v_pk_add).
// Both compute re' = fl(fl(re*c) + fl(im*(-d))), im' = fl(fl(im*c) + fl(re*d)); the bench checks that
// their chains agree bit for bit after the run.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/replay_pk_bench.hip -o scripts/replay_pk_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#pragma clang fp contract(off)

typedef float f2v __attribute__((ext_vector_type(2)));

#define PSTEP(X, Y)                                                          \
    "v_mul_f32 %[t], %[c], " X "\n\t"                                     \
    "s_nop 0\n\t"                                                          \
    "v_mul_f32_dpp %[u], " X ", %[k2] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t" \
    "v_add_f32 " Y ", %[t], %[u]\n\t"

__global__ void k_dpp(float* out, unsigned long long* cyc, float dzr, float dzi, int steps)
{
    const int lane = threadIdx.x;
    float x = (lane & 1) ? (lane >> 1) * 1e-3f : 1.0f - (lane >> 1) * 1e-3f;
    const float c = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, dzr)));
    const float k2 = (lane & 1) ? dzi : -dzi;
    float t, u, w;
    const unsigned long long t0 = clock64();
    if (lane < 32) {
#pragma unroll 1
        for (int i = 0; i < steps; i += 8)
            asm volatile(PSTEP("%[x]", "%[w]") PSTEP("%[w]", "%[x]") PSTEP("%[x]", "%[w]") PSTEP("%[w]", "%[x]")
                             PSTEP("%[x]", "%[w]") PSTEP("%[w]", "%[x]") PSTEP("%[x]", "%[w]") PSTEP("%[w]", "%[x]")
                         : [x] "+v"(x), [t] "=&v"(t), [u] "=&v"(u), [w] "=&v"(w)
                         : [c] "s"(c), [k2] "v"(k2));
    }
    const unsigned long long t1 = clock64();
    out[lane] = x;
    if (lane == 0) *cyc = t1 - t0;
}

__device__ __forceinline__ f2v pk_step(f2v x, f2v cc, f2v kk)
{
    const f2v t = x * cc;                                   // {re*c, im*c}
    const f2v u = __builtin_shufflevector(x, x, 1, 0) * kk;  // {im*(-d), re*d}
    return t + u;
}

__global__ void k_pk(float* out, unsigned long long* cyc, float dzr, float dzi, int steps)
{
    const int lane = threadIdx.x;
    f2v x = f2v{1.0f - lane * 1e-3f, lane * 1e-3f};
    const f2v cc = f2v{dzr, dzr};
    const f2v kk = f2v{-dzi, dzi};
    const unsigned long long t0 = clock64();
    if (lane < 16) {
#pragma unroll 1
        for (int i = 0; i < steps; i += 8) {
#pragma unroll
            for (int j = 0; j < 8; j++) x = pk_step(x, cc, kk);
        }
    }
    const unsigned long long t1 = clock64();
    out[2 * lane] = x.x;
    out[2 * lane + 1] = x.y;
    if (lane == 0) *cyc = t1 - t0;
}

int main()
{
    float *o1, *o2;
    unsigned long long* cyc;
    if (hipMalloc(&o1, 128 * sizeof(float)) != hipSuccess || hipMalloc(&o2, 128 * sizeof(float)) != hipSuccess ||
        hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess)
        return 1;
    const int steps = 1024;
    unsigned long long best[2] = {~0ull, ~0ull};
    for (int rep = 0; rep < 7; rep++) {
        for (int v = 0; v < 2; v++) {
            if (v == 0) hipLaunchKernelGGL(k_dpp, 1, 64, 0, 0, o1, cyc, 0.99f, 0.14f, steps);
            else hipLaunchKernelGGL(k_pk, 1, 64, 0, 0, o2, cyc, 0.99f, 0.14f, steps);
            unsigned long long c = 0;
            if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 2;
            if (c < best[v]) best[v] = c;
        }
    }
    float h1[64], h2[64];
    if (hipMemcpy(h1, o1, sizeof(h1), hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(h2, o2, sizeof(h2), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int same = 0;
    for (int l = 0; l < 16; l++) same += memcmp(&h1[2 * l], &h2[2 * l], 8) == 0;
    printf("dpp (2 lanes/chain): %.2f cycles/step; pk (1 lane/chain): %.2f cycles/step; chains bit-identical: %d/16\n",
        best[0] / double(steps), best[1] / double(steps), same);
    return same == 16 ? 0 : 4;
}
