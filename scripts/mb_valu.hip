// Micro-benchmark: VALU issue on gfx950.
//   mode 0: v_mul_f32, 8 independent chains / wave   mode 1: v_pk_mul_f32, 8 chains
//   mode 2: v_fma_f32, 8 chains                         mode 3: v_mul_f32, ONE dependent chain
//   mode 4: v_mul_f32, 2 chains                         mode 5: 8 chains + a uniform s_cbranch per 8 ops
//   mode 6: v_pk_fma_f32, 8 chains                      mode 7: v_pk_mul_f32, 4 chains (dependent pairs)
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float float2_t __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0+4, a5=a0+5, a6=a0+6, a7=a0+7;
    float2_t p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4={a1,a0}, p5={a3,a2}, p6={a5,a4}, p7={a7,a6};
    float2_t ss = {s, s};
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0 || MODE == 5) {
            a0 *= s; a1 *= s; a2 *= s; a3 *= s; a4 *= s; a5 *= s; a6 *= s; a7 *= s;
            if (MODE == 5 && a0 == 12345.0f) a1 = a2 + 1.0f;  // divergent-capable branch
        } else if (MODE == 1) {
            p0 *= ss; p1 *= ss; p2 *= ss; p3 *= ss; p4 *= ss; p5 *= ss; p6 *= ss; p7 *= ss;
        } else if (MODE == 2) {
            a0 = __builtin_fmaf(a0, s, s); a1 = __builtin_fmaf(a1, s, s); a2 = __builtin_fmaf(a2, s, s); a3 = __builtin_fmaf(a3, s, s);
            a4 = __builtin_fmaf(a4, s, s); a5 = __builtin_fmaf(a5, s, s); a6 = __builtin_fmaf(a6, s, s); a7 = __builtin_fmaf(a7, s, s);
        } else if (MODE == 6) {
#define PKFMA(p) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p) : "v"(ss))
            PKFMA(p0); PKFMA(p1); PKFMA(p2); PKFMA(p3); PKFMA(p4); PKFMA(p5); PKFMA(p6); PKFMA(p7);
        } else if (MODE == 7) {
#define PKMUL(p) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p) : "v"(ss))
            PKMUL(p0); PKMUL(p1); PKMUL(p2); PKMUL(p3); PKMUL(p0); PKMUL(p1); PKMUL(p2); PKMUL(p3);
        } else if (MODE == 3) {
            a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s;
        } else {
            a0 *= s; a1 *= s; a0 *= s; a1 *= s; a0 *= s; a1 *= s; a0 *= s; a1 *= s;
        }
    }
    float r = a0+a1+a2+a3+a4+a5+a6+a7 + p0.x+p0.y+p1.x+p1.y+p2.x+p2.y+p3.x+p3.y+p4.x+p4.y+p5.x+p5.y+p6.x+p6.y+p7.x+p7.y;
    if (r == 1234.5f) out[0] = r;
}
int main(int argc, char** argv) {
    float* out; (void)hipMalloc(&out, 4);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    int wpb = argc > 1 ? atoi(argv[1]) : 4;  // waves per block -> occupancy
    int blocks = argc > 2 ? atoi(argv[2]) : 2048;
    int iters = argc > 3 ? atoi(argv[3]) : 20000;
    int only = argc > 4 ? atoi(argv[4]) : -1;
    const char* names[8] = {"mul x8 chains", "pk_mul x8 chains", "fma x8 chains", "mul 1 chain", "mul 2 chains", "mul x8 + branch", "pk_fma x8 chains", "pk_mul x4 chains"};
    for (int m = 0; m < 8; ++m) {
        if (only >= 0 && m != only) continue;
        for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(a);
        dim3 g(blocks), t(64 * wpb);
        switch (m) {
            case 0: hipLaunchKernelGGL(k<0>, g, t, 0, 0, out, iters, 0.999f); break;
            case 1: hipLaunchKernelGGL(k<1>, g, t, 0, 0, out, iters, 0.999f); break;
            case 2: hipLaunchKernelGGL(k<2>, g, t, 0, 0, out, iters, 0.999f); break;
            case 3: hipLaunchKernelGGL(k<3>, g, t, 0, 0, out, iters, 0.999f); break;
            case 4: hipLaunchKernelGGL(k<4>, g, t, 0, 0, out, iters, 0.999f); break;
            case 5: hipLaunchKernelGGL(k<5>, g, t, 0, 0, out, iters, 0.999f); break;
            case 6: hipLaunchKernelGGL(k<6>, g, t, 0, 0, out, iters, 0.999f); break;
            case 7: hipLaunchKernelGGL(k<7>, g, t, 0, 0, out, iters, 0.999f); break;
        }
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        double instr = (double)blocks * wpb * iters * 8;  // wave-instructions of the measured op
        if (rep) printf("%-18s waves/blk %d blocks %d iters %d  %8.3f ms  %.3f T wave-instr/s\n", names[m], wpb, blocks, iters, ms, instr / ms / 1e9);
        }
    }
    return 0;
}
