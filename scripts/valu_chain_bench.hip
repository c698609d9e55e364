// Microbenchmark: shader cycles per step of a serial complex-product chain z ← z·q on one wave
// (the AVX phasor replay's critical path, trk_fast.hip), in several instruction forms.
//   hipcc --offload-arch=gfx950 -O3 scripts/valu_chain_bench.hip -o scripts/valu_chain_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kSteps = 4096;

#define STEP6                      \
    "v_mul_f32 %2, %6, %0\n\t"     \
    "v_mul_f32 %4, %7, %0\n\t"     \
    "v_mul_f32 %3, %7, %1\n\t"     \
    "v_mul_f32 %5, %6, %1\n\t"     \
    "v_sub_f32 %0, %2, %3\n\t"     \
    "v_add_f32 %1, %4, %5\n\t"
#define STEP6x4 STEP6 STEP6 STEP6 STEP6

// the packed form the compiler emits for cmul_exact
#define STEPPK                                                         \
    "v_pk_mul_f32 %2, %0, %4 op_sel_hi:[0,1]\n\t"                      \
    "v_pk_mul_f32 %3, %0, %5 op_sel:[1,0] op_sel_hi:[1,1]\n\t"         \
    "s_nop 0\n\t"                                                      \
    "v_pk_add_f32 %0, %2, %3\n\t"                                      \
    "s_nop 0\n\t"

// quad-DPP form: lanes (4j..4j+3) of chain j hold x·k for (a·c, b·(−d), b·c, a·d)
#define STEPDPP                                                                          \
    "v_mul_f32_dpp %0, %1, %2 quad_perm:[0,2,2,0] row_mask:0xf bank_mask:0xf\n\t"        \
    "s_nop 1\n\t"                                                                        \
    "v_add_f32_dpp %1, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"       \
    "s_nop 1\n\t"

template <int V>
__global__ void chain(float* out, unsigned long long* cyc, float qx, float qy, int active)
{
    const int lane = threadIdx.x;
    float re = 1.0f + lane * 1e-3f, im = 0.5f, ac, bd, ad, bc;
    float re2 = 0.7f, im2 = 0.1f;
    if (lane >= active) return;
    unsigned long long t0 = clock64();
    if constexpr (V == 0) {  // 6 single-rate ops, one chain
        for (int i = 0; i < kSteps / 4; i++)
            asm volatile(STEP6x4 : "+v"(re), "+v"(im), "=&v"(ac), "=&v"(bd), "=&v"(ad), "=&v"(bc) : "s"(qx), "s"(qy));
    } else if constexpr (V == 1) {  // two independent chains interleaved per block
        float ac2, bd2, ad2, bc2;
        for (int i = 0; i < kSteps / 4; i++) {
            asm volatile(STEP6x4 : "+v"(re), "+v"(im), "=&v"(ac), "=&v"(bd), "=&v"(ad), "=&v"(bc) : "s"(qx), "s"(qy));
            asm volatile(STEP6x4 : "+v"(re2), "+v"(im2), "=&v"(ac2), "=&v"(bd2), "=&v"(ad2), "=&v"(bc2) : "s"(qx), "s"(qy));
        }
        re += re2;
    } else if constexpr (V == 2) {  // packed
        f2 z = f2{re, im}, t, u;
        const f2 q = f2{qx, qy}, qn = f2{-qy, qx};
        for (int i = 0; i < kSteps / 4; i++)
            asm volatile(STEPPK STEPPK STEPPK STEPPK : "+v"(z), "=&v"(t), "=&v"(u) : "v"(z), "v"(q), "v"(qn));
        re = z.x;
        im = z.y;
    } else if constexpr (V == 3) {  // quad DPP, 2 VALU per step
        const int ql = lane & 3;
        float k = ql == 0 ? qx : ql == 1 ? -qy : ql == 2 ? qx : qy;
        float x = (ql == 0 || ql == 3) ? re : im, p = 0.0f, s = x;
        for (int i = 0; i < kSteps / 4; i++)
            asm volatile(STEPDPP STEPDPP STEPDPP STEPDPP : "+v"(p), "+v"(s) : "v"(k));
        re = s;
    } else if constexpr (V == 4) {  // quad DPP without the nops (timing only: hazard not honoured)
        const int ql = lane & 3;
        float k = ql == 0 ? qx : ql == 1 ? -qy : ql == 2 ? qx : qy;
        float p = 0.0f, s = re;
        for (int i = 0; i < kSteps / 4; i++)
            asm volatile(
                "v_mul_f32_dpp %0, %1, %2 quad_perm:[0,2,2,0] row_mask:0xf bank_mask:0xf\n\t"
                "v_add_f32_dpp %1, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                "v_mul_f32_dpp %0, %1, %2 quad_perm:[0,2,2,0] row_mask:0xf bank_mask:0xf\n\t"
                "v_add_f32_dpp %1, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                "v_mul_f32_dpp %0, %1, %2 quad_perm:[0,2,2,0] row_mask:0xf bank_mask:0xf\n\t"
                "v_add_f32_dpp %1, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                "v_mul_f32_dpp %0, %1, %2 quad_perm:[0,2,2,0] row_mask:0xf bank_mask:0xf\n\t"
                "v_add_f32_dpp %1, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                : "+v"(p), "+v"(s)
                : "v"(k));
        re = s;
    } else if constexpr (V == 5) {  // 6 independent single-rate ops per step (pure issue rate)
        float a0 = re, a1 = im, a2 = re2, a3 = im2, a4 = 0.3f, a5 = 0.2f;
        for (int i = 0; i < kSteps / 4; i++)
            asm volatile(
                "v_mul_f32 %0, %6, %0\n\tv_mul_f32 %1, %6, %1\n\tv_mul_f32 %2, %6, %2\n\tv_mul_f32 %3, %6, %3\n\tv_mul_f32 %4, %6, %4\n\tv_mul_f32 %5, %6, %5\n\t"
                "v_mul_f32 %0, %6, %0\n\tv_mul_f32 %1, %6, %1\n\tv_mul_f32 %2, %6, %2\n\tv_mul_f32 %3, %6, %3\n\tv_mul_f32 %4, %6, %4\n\tv_mul_f32 %5, %6, %5\n\t"
                "v_mul_f32 %0, %6, %0\n\tv_mul_f32 %1, %6, %1\n\tv_mul_f32 %2, %6, %2\n\tv_mul_f32 %3, %6, %3\n\tv_mul_f32 %4, %6, %4\n\tv_mul_f32 %5, %6, %5\n\t"
                "v_mul_f32 %0, %6, %0\n\tv_mul_f32 %1, %6, %1\n\tv_mul_f32 %2, %6, %2\n\tv_mul_f32 %3, %6, %3\n\tv_mul_f32 %4, %6, %4\n\tv_mul_f32 %5, %6, %5\n\t"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5)
                : "s"(qx));
        re = a0 + a1 + a2 + a3 + a4 + a5;
    } else if constexpr (V == 6) {  // a fully dependent chain of single-rate muls (latency)
        for (int i = 0; i < kSteps / 4; i++)
            asm volatile(
                "v_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\t"
                "v_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\t"
                "v_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\t"
                "v_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\tv_mul_f32 %0, %1, %0\n\t"
                : "+v"(re)
                : "s"(qx));
    }
    unsigned long long t1 = clock64();
    out[lane] = re + im;
    if (lane == 0) *cyc = t1 - t0;
}

int main()
{
    float* out;
    unsigned long long* cyc;
    if (hipMalloc(&out, 256 * sizeof(float)) != hipSuccess || hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
    const char* names[] = {"6 ops, 1 chain", "6 ops, 2 chains interleaved (per step of each)", "packed 3 ops + 2 nops", "quad DPP + nops",
        "quad DPP no nops (timing only)", "6 independent muls per step (issue rate)", "6 dependent muls per step (latency)"};
    for (int active : {64, 16}) {
        for (int v = 0; v < 7; v++) {
            unsigned long long best = ~0ull;
            for (int rep = 0; rep < 5; rep++) {
                switch (v) {
                case 0: hipLaunchKernelGGL(chain<0>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                case 1: hipLaunchKernelGGL(chain<1>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                case 2: hipLaunchKernelGGL(chain<2>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                case 3: hipLaunchKernelGGL(chain<3>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                case 4: hipLaunchKernelGGL(chain<4>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                case 5: hipLaunchKernelGGL(chain<5>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                default: hipLaunchKernelGGL(chain<6>, 1, 64, 0, 0, out, cyc, 0.999f, 0.01f, active); break;
                }
                unsigned long long c = 0;
                if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 2;
                if (c < best) best = c;
            }
            printf("active %2d  %-50s %7.2f cycles/step\n", active, names[v], static_cast<double>(best) / kSteps);
        }
    }
    return 0;
}
