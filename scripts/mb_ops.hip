// Micro-benchmark: throughput of individual gfx950 VALU instructions, 8
// independent chains per wave, many waves per SIMD.  Prints cycles per
// wave-instruction per SIMD (2.0 = a full-rate wave64 f32 op).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define OP8(body)                                                              \
    asm volatile(body : "+v"(r0) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r1) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r2) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r3) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r4) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r5) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r6) : "v"(c0), "v"(c1));                          \
    asm volatile(body : "+v"(r7) : "v"(c0), "v"(c1));

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, int iters, unsigned seed) {
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    unsigned c0 = threadIdx.x * 7u + seed, c1 = seed ^ 0x9e3779b9u;
    if (OP >= 100) {  // 64-bit destination ops
        unsigned long long r0 = c0, r1 = c0 + 1, r2 = c0 + 2, r3 = c0 + 3, r4 = c0 + 4, r5 = c0 + 5, r6 = c0 + 6, r7 = c0 + 7;
        for (int i = 0; i < iters; ++i) {
            if (OP == 100) { OP8("v_mad_u64_u32 %0, vcc, %1, %2, %0") }
            if (OP == 101) { OP8("v_lshrrev_b64 %0, %1, %0") }
            if (OP == 102) { OP8("v_pk_fma_f32 %0, %0, %0, %0") }
            if (OP == 103) { OP8("v_pk_mul_f32 %0, %0, %0") }
            if (OP == 104) { OP8("v_fma_f64 %0, %0, %0, %0") }
            if (OP == 105) { OP8("v_mul_f64 %0, %0, %0") }
        }
        unsigned long long r = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
        if ((unsigned)r == 0x12345u) out[0] = (unsigned)r;
        return;
    }
    unsigned r0 = c0, r1 = c0 + 1, r2 = c0 + 2, r3 = c0 + 3, r4 = c0 + 4, r5 = c0 + 5, r6 = c0 + 6, r7 = c0 + 7;
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) { OP8("v_add_f32 %0, %0, %1") }
        if (OP == 1) { OP8("v_fma_f32 %0, %0, %1, %2") }
        if (OP == 2) { OP8("v_mul_lo_u32 %0, %0, %1") }
        if (OP == 3) { OP8("v_mul_hi_u32 %0, %0, %1") }
        if (OP == 4) { OP8("v_sqrt_f32 %0, %0") }
        if (OP == 5) { OP8("v_rcp_f32 %0, %0") }
        if (OP == 6) { OP8("v_cvt_f32_u32 %0, %0") }
        if (OP == 7) { OP8("v_xor_b32 %0, %0, %1") }
        if (OP == 8) { OP8("v_alignbit_b32 %0, %0, %1, %2") }
        if (OP == 9) { OP8("v_mul_u32_u24 %0, %0, %1") }
        if (OP == 10) { OP8("v_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 11) { OP8("v_div_scale_f32 %0, vcc, %0, %1, %0") }
        if (OP == 12) { OP8("v_div_fmas_f32 %0, %0, %1, %2") }
        if (OP == 13) { OP8("v_frexp_exp_i32_f32 %0, %0") }
        if (OP == 14) { OP8("v_add3_u32 %0, %0, %1, %2") }
        if (OP == 15) { OP8("v_mad_u32_u24 %0, %0, %1, %2") }
    }
    unsigned r = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
    if (r == 0x12345u) out[0] = r;
}

template <int OP>
void run(const char *name, unsigned *out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 256 * 8 * 4, iters = 4000;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 12345u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        // wave-instructions per SIMD: blocks*4 waves*iters*8 over 1024 SIMDs; clock ~2.4 GHz
        const double wi = (double)blocks * 4 * iters * 8 / 1024.0;
        if (rep) printf("%-28s %7.3f ms  %6.2f cyc/wave-instr/SIMD (at 2.4 GHz)\n", name, ms, ms * 1e-3 * 2.4e9 / wi);
    }
}

int main() {
    unsigned *out;
    (void)hipMalloc(&out, 4);
    run<0>("v_add_f32", out);
    run<1>("v_fma_f32", out);
    run<2>("v_mul_lo_u32", out);
    run<3>("v_mul_hi_u32", out);
    run<4>("v_sqrt_f32", out);
    run<5>("v_rcp_f32", out);
    run<6>("v_cvt_f32_u32", out);
    run<7>("v_xor_b32", out);
    run<8>("v_alignbit_b32", out);
    run<9>("v_mul_u32_u24", out);
    run<10>("v_cndmask_b32 (vcc)", out);
    run<11>("v_div_scale_f32", out);
    run<12>("v_div_fmas_f32", out);
    run<13>("v_frexp_exp_i32_f32", out);
    run<14>("v_add3_u32", out);
    run<15>("v_mad_u32_u24", out);
    run<100>("v_mad_u64_u32", out);
    run<101>("v_lshrrev_b64", out);
    run<102>("v_pk_fma_f32", out);
    run<103>("v_pk_mul_f32", out);
    run<104>("v_fma_f64", out);
    run<105>("v_mul_f64", out);
    return 0;
}
