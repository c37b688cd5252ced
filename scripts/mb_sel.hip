// Micro-benchmark: lane-select (v_cndmask) costs on gfx950 by mask source, against
// full-rate references; 8 independent chains per wave, many waves per SIMD.
// Prints cycles per wave-instruction per SIMD (2.0 = a full-rate wave64 f32 op).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define OP8S(body)                                                                        \
    asm volatile(body : "+v"(r0) : "v"(c0), "v"(c1), "s"(m)); asm volatile(body : "+v"(r1) : "v"(c0), "v"(c1), "s"(m)); \
    asm volatile(body : "+v"(r2) : "v"(c0), "v"(c1), "s"(m)); asm volatile(body : "+v"(r3) : "v"(c0), "v"(c1), "s"(m)); \
    asm volatile(body : "+v"(r4) : "v"(c0), "v"(c1), "s"(m)); asm volatile(body : "+v"(r5) : "v"(c0), "v"(c1), "s"(m)); \
    asm volatile(body : "+v"(r6) : "v"(c0), "v"(c1), "s"(m)); asm volatile(body : "+v"(r7) : "v"(c0), "v"(c1), "s"(m));

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, int iters, unsigned seed) {
    unsigned c0 = threadIdx.x * 7u + seed, c1 = seed ^ 0x9e3779b9u;
    unsigned long long m = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    unsigned r0 = c0, r1 = c0 + 1, r2 = c0 + 2, r3 = c0 + 3, r4 = c0 + 4, r5 = c0 + 5, r6 = c0 + 6, r7 = c0 + 7;
    if (OP == 3 || OP == 6) asm volatile("s_mov_b64 vcc, %0" :: "s"(m) : "vcc");
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) { OP8S("v_max_f32 %0, %0, %1") }
        if (OP == 1) { OP8S("v_cndmask_b32_e64 %0, %0, %1, %3") }
        if (OP == 2) { OP8S("v_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 3) { OP8S("v_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 4) { OP8S("v_cmp_lt_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 5) { OP8S("v_cmp_lt_f32_e64 %3, %0, %1\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %0, %1, %3") }
        if (OP == 6) { OP8S("v_cndmask_b32_e64 %0, %0, %1, vcc") }
        if (OP == 7) { OP8S("v_med3_f32 %0, %0, %1, %2") }
        if (OP == 8) { OP8S("v_min_f32 %0, %0, %1") }
        if (OP == 9) { OP8S("v_bfi_b32 %0, %0, %1, %2") }
        if (OP == 10) { OP8S("v_cmp_lt_f32_e64 %3, %0, %1") }
        if (OP == 11) { OP8S("v_mov_b32_dpp %0, %1 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf") }
        if (OP == 12) { OP8S("v_xad_u32 %0, %0, %1, %2") }
        if (OP == 13) { OP8S("v_add_f32 %0, %0, %1") }
        if (OP == 14) { OP8S("v_cmp_lt_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc\n\tv_cndmask_b32 %0, %0, %2, vcc\n\tv_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 15) { OP8S("v_cmp_lt_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %0, %1, vcc\n\tv_cndmask_b32_e64 %0, %0, %2, vcc\n\tv_cndmask_b32_e64 %0, %0, %1, vcc") }
        if (OP == 16) { OP8S("v_cmp_lt_f32 vcc, %0, %1\n\tv_add_f32 %0, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 19) { OP8S("v_cmp_lt_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc\n\tv_add_f32 %0, %0, %1\n\tv_cndmask_b32 %0, %0, %2, vcc\n\tv_add_f32 %0, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 20) { OP8S("v_cndmask_b32 %0, %0, %1, vcc\n\tv_add_f32 %0, %0, %1") }
        if (OP == 21) { OP8S("v_addc_co_u32 %0, vcc, %0, %1, vcc") }
        if (OP == 22) { OP8S("v_cmp_lt_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 17) { OP8S("v_mul_f32 %0, %0, %1") }
        if (OP == 18) { OP8S("v_add_u32 %0, %0, %1") }
    }
    unsigned r = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
    if (r == 0x12345u) out[0] = r;
}

template <int OP>
void run(const char *name, unsigned *out, int per) {
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
        const double wi = (double)blocks * 4 * iters * 8 * per / 1024.0;
        if (rep) printf("%-44s %7.3f ms  %6.2f cyc/wave-instr/SIMD (at 2.4 GHz)\n", name, ms, ms * 1e-3 * 2.4e9 / wi);
    }
}

int main() {
    unsigned *out;
    (void)hipMalloc(&out, 4);
    run<0>("v_max_f32", out, 1);
    run<1>("v_cndmask_b32_e64 (sgpr pair)", out, 1);
    run<2>("v_cndmask_b32 (vcc, never written)", out, 1);
    run<3>("v_cndmask_b32 (vcc, written once)", out, 1);
    run<4>("v_cmp vcc + s_nop 1 + v_cndmask vcc (per 2)", out, 2);
    run<5>("v_cmp sgpr + s_nop 1 + v_cndmask sgpr (per 2)", out, 2);
    run<6>("v_cndmask_b32_e64 (vcc)", out, 1);
    run<7>("v_med3_f32", out, 1);
    run<8>("v_min_f32", out, 1);
    run<9>("v_bfi_b32", out, 1);
    run<10>("v_cmp_lt_f32_e64 sgpr", out, 1);
    run<11>("v_mov_b32_dpp quad_perm", out, 1);
    run<12>("v_xad_u32", out, 1);
    run<13>("v_add_f32", out, 1);
    run<14>("v_cmp vcc + nop + 3 x v_cndmask_e32 vcc (per 4)", out, 4);
    run<15>("v_cmp vcc + nop + 3 x v_cndmask_e64 vcc (per 4)", out, 4);
    run<16>("v_cmp vcc + v_add + v_cndmask_e32 vcc (per 3)", out, 3);
    run<17>("v_mul_f32", out, 1);
    run<19>("cmp vcc; nop; 3 x (cndmask_e32 vcc; add) (per 6)", out, 6);
    run<20>("cndmask_e32 vcc; add (per 2)", out, 2);
    run<21>("v_addc_co_u32 vcc", out, 1);
    run<22>("cmp vcc; nop 1; cndmask_e32 vcc (per 2, same wave chain)", out, 2);
    run<18>("v_add_u32", out, 1);
    return 0;
}
