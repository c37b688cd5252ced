// Micro-benchmark (second set): issue cost of the gfx950 VALU forms the trace kernel's
// hot blocks use, 8 independent chains per wave, many waves per SIMD.  Prints cycles per
// wave-instruction per SIMD (scripts/mb_ops.hip measured v_add_f32 2.8, v_pk_fma_f32 4.2).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define OP8(body)                                                              \
    asm volatile(body : "+v"(r0) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r1) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r2) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r3) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r4) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r5) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r6) : "v"(c0), "v"(c1), "s"(m));                  \
    asm volatile(body : "+v"(r7) : "v"(c0), "v"(c1), "s"(m));
#define CMP8(body)                                                             \
    asm volatile(body : "=s"(q0) : "v"(r0), "v"(c1));                          \
    asm volatile(body : "=s"(q1) : "v"(r1), "v"(c1));                          \
    asm volatile(body : "=s"(q2) : "v"(r2), "v"(c1));                          \
    asm volatile(body : "=s"(q3) : "v"(r3), "v"(c1));                          \
    asm volatile(body : "=s"(q4) : "v"(r4), "v"(c1));                          \
    asm volatile(body : "=s"(q5) : "v"(r5), "v"(c1));                          \
    asm volatile(body : "=s"(q6) : "v"(r6), "v"(c1));                          \
    asm volatile(body : "=s"(q7) : "v"(r7), "v"(c1));

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, int iters, unsigned seed) {
    unsigned c0 = threadIdx.x * 7u + seed, c1 = seed ^ 0x9e3779b9u;
    unsigned long long m = __builtin_amdgcn_read_exec() ^ (unsigned long long)seed;
    unsigned r0 = c0, r1 = c0 + 1, r2 = c0 + 2, r3 = c0 + 3, r4 = c0 + 4, r5 = c0 + 5, r6 = c0 + 6, r7 = c0 + 7;
    unsigned long long q0 = 0, q1 = 0, q2 = 0, q3 = 0, q4 = 0, q5 = 0, q6 = 0, q7 = 0;
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) { OP8("v_mul_f32 %0, %0, %1") }
        if (OP == 1) { OP8("v_sub_f32 %0, %0, %1") }
        if (OP == 2) { OP8("v_min_f32 %0, %0, %1") }
        if (OP == 3) { OP8("v_min3_f32 %0, %0, %1, %2") }
        if (OP == 4) { OP8("v_and_b32 %0, %0, %1") }
        if (OP == 5) { OP8("v_lshlrev_b32 %0, %1, %0") }
        if (OP == 6) { OP8("v_add_u32 %0, %0, %1") }
        if (OP == 7) { OP8("v_bfe_u32 %0, %0, %1, %2") }
        if (OP == 8) { OP8("v_cndmask_b32_e64 %0, %0, %1, %3") }
        if (OP == 9) { OP8("v_fmac_f32 %0, %1, %2") }
        if (OP == 10) { OP8("v_fma_f32 %0, -%0, %1, %2") }
        if (OP == 11) { OP8("v_mul_f32 %0, %0, 0.5") }
        if (OP == 12) { OP8("v_sub_u32 %0, %0, %1") }
        if (OP == 13) { OP8("v_mov_b32 %0, %1") }
        if (OP == 14) { OP8("v_med3_f32 %0, %0, %1, %2") }
        if (OP == 15) { OP8("v_max_f32 %0, |%0|, %1") }
        if (OP == 16) { CMP8("v_cmp_lt_f32_e64 %0, %1, %2") }
        if (OP == 17) { CMP8("v_cmp_eq_u32_e64 %0, %1, %2") }
        if (OP == 18) { OP8("v_xad_u32 %0, %0, %1, %2") }
        if (OP == 19) { OP8("v_lshl_add_u32 %0, %0, 3, %1") }
        if (OP == 20) { OP8("v_exp_f32 %0, %0") }
        if (OP == 21) { OP8("v_rsq_f32 %0, %0") }
        if (OP == 22) { OP8("v_cvt_f32_u32 %0, %0") }
        if (OP == 23) { OP8("v_ldexp_f32 %0, %0, %1") }
    }
    unsigned r = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ (unsigned)(q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7);
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
        const double wi = (double)blocks * 4 * iters * 8 / 1024.0;
        if (rep) printf("%-34s %7.3f ms  %6.2f cyc/wave-instr/SIMD (at 2.4 GHz)\n", name, ms, ms * 1e-3 * 2.4e9 / wi);
    }
}

int main() {
    unsigned *out;
    (void)hipMalloc(&out, 4);
    run<0>("v_mul_f32", out);
    run<1>("v_sub_f32", out);
    run<2>("v_min_f32", out);
    run<3>("v_min3_f32", out);
    run<4>("v_and_b32", out);
    run<5>("v_lshlrev_b32", out);
    run<6>("v_add_u32", out);
    run<7>("v_bfe_u32", out);
    run<8>("v_cndmask_b32_e64 (sgpr mask)", out);
    run<9>("v_fmac_f32", out);
    run<10>("v_fma_f32 (neg)", out);
    run<11>("v_mul_f32 (inline const)", out);
    run<12>("v_sub_u32", out);
    run<13>("v_mov_b32", out);
    run<14>("v_med3_f32", out);
    run<15>("v_max_f32 (abs)", out);
    run<16>("v_cmp_lt_f32_e64 (sgpr dst)", out);
    run<17>("v_cmp_eq_u32_e64 (sgpr dst)", out);
    run<18>("v_xad_u32", out);
    run<19>("v_lshl_add_u32", out);
    run<20>("v_exp_f32", out);
    run<21>("v_rsq_f32", out);
    run<22>("v_cvt_f32_u32", out);
    run<23>("v_ldexp_f32", out);
    return 0;
}
