// Microbenchmark: cycles per step of the AVX rotator's serial phasor chain z <- z·dz (bit-exact
// roundings) in three instruction forms, one wave, 16 chains.  Diagnostic only (not in the library).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/chain_bench.hip -o scripts/chain_bench
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ f2 cmul_pk(f2 a, f2 b)
{
    const f2 t = f2{a.x, a.x} * b;
    const f2 u = f2{a.y, a.y} * f2{-b.y, b.x};
    return t + u;
}

__device__ __forceinline__ f2 cmul_sc(f2 a, f2 b)
{
    const float p0 = __fmul_rn(a.x, b.x), p1 = __fmul_rn(a.y, b.y), p2 = __fmul_rn(a.x, b.y), p3 = __fmul_rn(a.y, b.x);
    return f2{__fsub_rn(p0, p1), __fadd_rn(p2, p3)};
}

template <int MODE>
__global__ void chain(const float* in, float* out, long long* cyc, int steps)
{
    const int lane = threadIdx.x;
    f2 dz = f2{in[0], in[1]};
    f2 z = f2{in[2 + (lane & 15)], in[3]};
    float v = (lane & 3) < 2 ? z.x : z.y;
    const int r = lane & 3;
    const float dq = r == 0 ? dz.x : r == 1 ? -dz.y : r == 2 ? dz.y : dz.x;
    __syncthreads();
    const long long t0 = clock64();
    if constexpr (MODE == 0) {
        for (int s = 0; s < steps; s += 16) {
#pragma unroll
            for (int u = 0; u < 16; u++) z = cmul_pk(z, dz);
        }
    } else if constexpr (MODE == 1) {
        for (int s = 0; s < steps; s += 16) {
#pragma unroll
            for (int u = 0; u < 16; u++) z = cmul_sc(z, dz);
        }
    } else {
        for (int s = 0; s < steps; s += 16) {
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const float p = __fmul_rn(dpp_mov<0xD8>(v), dq);
                v = __fadd_rn(dpp_mov<0xB1>(p), p);
            }
        }
        z = f2{v, v};
    }
    const long long t1 = clock64();
    out[lane * 2] = z.x;
    out[lane * 2 + 1] = z.y;
    if (lane == 0) cyc[MODE] = t1 - t0;
}

int main()
{
    float h[32];
    for (int i = 0; i < 32; i++) h[i] = 0.7f + 0.001f * i;
    h[0] = 0.99995f;
    h[1] = 0.0099f;
    float *din, *dout;
    long long* dc;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 64 * 2 * sizeof(float));
    hipMalloc(&dc, 4 * sizeof(long long));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const int steps = 4096;
    for (int rep = 0; rep < 3; rep++) {
        chain<0><<<1, 64>>>(din, dout, dc, steps);
        chain<1><<<1, 64>>>(din, dout, dc, steps);
        chain<2><<<1, 64>>>(din, dout, dc, steps);
    }
    long long c[3];
    hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    printf("cycles/step (clock64): packed %.1f  scalar %.1f  dpp-quad %.1f\n", c[0] / double(steps), c[1] / double(steps), c[2] / double(steps));
    return 0;
}
