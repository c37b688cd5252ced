// Micro-benchmark: cost of lane selects on gfx950 in the forms the compiler emits
// (v_cmp + v_cndmask on VCC) against explicit SGPR-pair masks.  8 chains per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP>
__global__ __launch_bounds__(256) void k(float *out, int iters, float seed) {
    float c0 = threadIdx.x * 0.37f + seed, c1 = seed * 0.5f;
    float r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = c0 + i;
    for (int it = 0; it < iters; ++it) {
        if (OP == 0) {  // one VCC write per iteration, eight VOP2 selects reading it
            asm volatile("v_cmp_lt_f32 vcc, %0, %1" ::"v"(c0), "v"(c1) : "vcc");
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(c0) : "vcc");
        }
        if (OP == 1) {  // the same with an SGPR-pair mask (VOP3)
            unsigned long long m;
            asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(c0), "v"(c1));
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(r[i]) : "v"(c0), "s"(m));
        }
        if (OP == 2) {  // compiler-generated compare + select per chain
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = r[i] < c1 ? r[i] + c0 : r[i] * 0.5f;
        }
        if (OP == 3) {  // compiler: plain f32 mul + add per chain (reference)
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = r[i] * 0.5f + c0;
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += r[i];
    if (s == 1234.5f) out[0] = s;
}

template <int OP>
void run(const char *name, float *out, double per_iter) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 256 * 8 * 4, iters = 4000;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.25f);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double wi = (double)blocks * 4 * iters * per_iter / 1024.0;
        if (rep) printf("%-44s %7.3f ms  %6.2f cyc/wave-instr/SIMD (%g instr/iter)\n", name, ms, ms * 1e-3 * 2.4e9 / wi, per_iter);
    }
}

int main() {
    float *out;
    (void)hipMalloc(&out, 4);
    run<0>("v_cmp vcc + 8x v_cndmask_b32 vcc", out, 9);
    run<1>("v_cmp_e64 sgpr + 8x v_cndmask_b32_e64 sgpr", out, 9);
    run<2>("compiler: 8x (cmp, add, mul, select)", out, 32);
    run<3>("compiler: 8x (mul, add)", out, 16);
    return 0;
}
