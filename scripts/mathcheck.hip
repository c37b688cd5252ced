// GPU verification of the short exact-rounding sequences considered for the
// trace kernel, against the compiler's IEEE sequences (-ffp-contract=off):
//   rcp:  y = RN(1/b) from v_rcp_f32 + one Newton step       (exhaustive mantissas x exponent range)
//   sqrt: RN(sqrt(x)) from v_sqrt_f32 + +-1ulp residual fix   (exhaustive mantissas x exponent range)
//         and from v_rsq_f32 + one fma correction (Markstein; the kernel's sqrt_rn since round 6, mode 6)
//   div:  RN(a/b) = fma(r, y, q0), q0 = a*y, r = fma(-q0, b, a), y = RN(1/b)  (random + edge pairs)
// Prints mismatch counts and the first few mismatching inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ float rcp_fast(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}
__device__ __forceinline__ float sqrt_fast(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = s;
    if (__builtin_fmaf(-sm, s, x) <= 0.0f) r = sm;
    if (__builtin_fmaf(-sp, s, x) > 0.0f) r = sp;
    return r;
}
__device__ __forceinline__ float sqrt_down(float x) {  // the residual fix toward zero only
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    return __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
}
__device__ __forceinline__ float sqrt_up(float x) {  // the residual fix away from zero only
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    return __builtin_fmaf(-sp, s, x) > 0.0f ? sp : s;
}
__device__ __forceinline__ float sqrt_markstein(float x) {  // v_rsq_f32 + one fma correction
    const float y = __builtin_fminf(__builtin_amdgcn_rsqf(x), 0x1p64f);  // x = 0 -> 0
    const float g = x * y, h = 0.5f * y;
    const float r = __builtin_fmaf(-g, g, x);
    return __builtin_fmaf(r, h, g);
}
__device__ __forceinline__ float sqrt_markstein2(float x) {  // v_rsq_f32, one Goldschmidt step, then the correction
    const float y = __builtin_amdgcn_rsqf(x);
    float g = x * y, h = 0.5f * y;
    const float e = __builtin_fmaf(-g, h, 0.5f);
    g = __builtin_fmaf(g, e, g);
    h = __builtin_fmaf(h, e, h);
    const float r = __builtin_fmaf(-g, g, x);
    return __builtin_fmaf(r, h, g);
}
__device__ __forceinline__ float sqrt_vsqrt_fma(float x) {  // v_sqrt_f32 + one correction with h = 0.5 v_rsq
    const float s = __builtin_amdgcn_sqrtf(x);
    const float h = 0.5f * __builtin_amdgcn_rsqf(x);
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, h, s);
}
__device__ __forceinline__ float div_fast(float a, float b, float y) {
    const float q0 = a * y;
    const float r = __builtin_fmaf(-q0, b, a);
    return __builtin_fmaf(r, y, q0);
}

__device__ unsigned long long g_hist[256];  // mismatches per biased exponent of the input (unary modes)
__device__ void report(unsigned long long *cnt, uint32_t *bad, uint32_t a, uint32_t b) {
    atomicAdd(&g_hist[(a >> 23) & 0xFFu], 1ull);
    const unsigned long long i = atomicAdd(cnt, 1ull);
    if (i < 8) { bad[2 * i] = a; bad[2 * i + 1] = b; }
}

// mode 0: rcp, 1: sqrt over u = (e0 + blockIdx.y) << 23 | mantissa
__global__ void k_unary(int mode, int e0, unsigned long long *cnt, uint32_t *bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const uint32_t u = ((uint32_t)(e0 + (int)blockIdx.y) << 23) | m;
    const float x = __uint_as_float(u);
    float got, want;
    if (mode == 0) { got = rcp_fast(x); want = 1.0f / x; }
    else if (mode == 1) { got = sqrt_fast(x); want = __builtin_sqrtf(x); }
    else if (mode == 2) { got = __builtin_amdgcn_sqrtf(x); want = __builtin_sqrtf(x); }   // raw v_sqrt_f32
    else if (mode == 3) { got = sqrt_down(x); want = __builtin_sqrtf(x); }               // only the -1ulp fix
    else if (mode == 4) { got = sqrt_up(x); want = __builtin_sqrtf(x); }                 // only the +1ulp fix
    else if (mode == 6) { got = sqrt_markstein(x); want = __builtin_sqrtf(x); }
    else if (mode == 9) {  // RN(1/len), len = RN(sqrt(x)), by one Newton step from v_rsq_f32(x) (normalize's reciprocal)
        const float len = sqrt_markstein(x);
        const float y = __builtin_fminf(__builtin_amdgcn_rsqf(x), 0x1p64f);
        got = __builtin_fmaf(__builtin_fmaf(-len, y, 1.0f), y, y);
        want = 1.0f / len;
    }
    else if (mode == 10) {  // mode 9 with the kernel's fallback: len's mantissa all ones -> rcp + Newton
        const float len = sqrt_markstein(x);
        const float y = __builtin_fminf(__builtin_amdgcn_rsqf(x), 0x1p64f);
        got = __builtin_fmaf(__builtin_fmaf(-len, y, 1.0f), y, y);
        if ((__float_as_uint(len) & 0x7FFFFFu) == 0x7FFFFFu) got = rcp_fast(len);
        want = 1.0f / len;
    }
    else if (mode == 7) { got = sqrt_markstein2(x); want = __builtin_sqrtf(x); }
    else if (mode == 8) { got = sqrt_vsqrt_fma(x); want = __builtin_sqrtf(x); }
    else { got = __builtin_amdgcn_rcpf(x); want = 1.0f / x; }                            // raw v_rcp_f32
    if (__float_as_uint(got) != __float_as_uint(want)) report(cnt, bad, u, 0);
}

__device__ __forceinline__ uint32_t pcg(uint64_t &s) {
    const uint64_t old = s;
    s = old * 6364136223846793005ULL + 1442695040888963407ULL;
    const uint32_t v = (uint32_t)(old >> 32) ^ (uint32_t)old;
    return __builtin_amdgcn_alignbit(v, v, (uint32_t)(old >> 59));
}

// division pairs: b from an exponent window [eb0, eb0+16), a anywhere in
// [ea0, ea0+64) exponents, random mantissas (plus every 16th pair with b's
// mantissa near 1 or 2 and a's near a multiple of b)
__global__ void k_div(uint64_t seed, int iters, int ea0, int eb0, unsigned long long *cnt, uint32_t *bad) {
    uint64_t s = seed ^ ((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B97F4A7C15ULL);
    for (int it = 0; it < iters; ++it) {
        const uint32_t r0 = pcg(s), r1 = pcg(s), r2 = pcg(s);
        uint32_t mb = r1 & 0x7FFFFFu;
        if ((r2 & 15u) == 0) mb = (r2 & 16u) ? (r1 & 0xFFu) : (0x7FFFFFu - (r1 & 0xFFu));
        const uint32_t ub = ((uint32_t)(eb0 + (int)((r2 >> 8) & 15u)) << 23) | mb;
        const float b = __uint_as_float(ub);
        uint32_t ua = ((uint32_t)(ea0 + (int)((r2 >> 12) & 63u)) << 23) | (r0 & 0x7FFFFFu);
        if ((r2 & 0xF0000u) == 0) {  // a close to k*b: quotient near a representable value
            const float k = (float)((r0 >> 9) | 1u);
            ua = __float_as_uint(k * b) + ((r2 >> 24) & 3u) - 1u;
        }
        if (r2 >> 31) ua |= 0x80000000u;
        const float a = __uint_as_float(ua);
        const float y = 1.0f / b;
        const float got = div_fast(a, b, y), want = a / b;
        if (__float_as_uint(got) != __float_as_uint(want) && !(got != got && want != want)) report(cnt, bad, ua, ub);
    }
}

int main() {
    unsigned long long *cnt;
    uint32_t *bad;
    (void)hipMalloc(&cnt, 8);
    (void)hipMalloc(&bad, 64);
    bool hist = true;
    auto run = [&](const char *name, auto launch) {
        (void)hipMemset(cnt, 0, 8);
        (void)hipMemset(bad, 0, 64);
        launch();
        (void)hipDeviceSynchronize();
        unsigned long long c;
        uint32_t h[16];
        (void)hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h, bad, 64, hipMemcpyDeviceToHost);
        printf("%-34s mismatches %llu", name, c);
        for (int i = 0; i < 8 && i < (int)c; ++i) printf("  [%08x %08x]", h[2 * i], h[2 * i + 1]);
        printf("\n");
        unsigned long long hh[256];
        (void)hipMemcpyFromSymbol(hh, HIP_SYMBOL(g_hist), sizeof(hh));
        if (c && hist) {  // where the mismatches lie (x in [2^(e-127), 2^(e-126)))
            printf("    by input exponent:");
            for (int e = 0; e < 256; ++e)
                if (hh[e]) printf(" 2^%d:%llu", e - 127, hh[e]);
            printf("\n");
        }
        unsigned long long z[256] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_hist), z, sizeof(z));
    };
    // exponents 127-40 .. 127+40: x in [2^-40, 2^40)
    run("rcp  rcp+Newton, 2^-40..2^40", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 80), dim3(256), 0, 0, 0, 87, cnt, bad); });
    run("sqrt v_sqrt+fix, 2^-60..2^60", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 1, 67, cnt, bad); });
    // is either fix-up step ever needed? (raw instructions and one-sided fixes, same range)
    run("sqrt raw v_sqrt_f32, 2^-60..2^60", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 2, 67, cnt, bad); });
    run("sqrt v_sqrt + down fix only", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 3, 67, cnt, bad); });
    run("sqrt v_sqrt + up fix only", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 4, 67, cnt, bad); });
    run("sqrt v_rsq + fma correction", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 6, 67, cnt, bad); });
    // the whole normal range 2^-126 .. 2^128 (exponents 1..254): beyond the kernel's proven callers
    run("rcp  1/RN(sqrt x) by Newton from v_rsq(x), 2^-60..2^100", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 160), dim3(256), 0, 0, 9, 67, cnt, bad); });
    run("rcp  same + all-ones-mantissa fallback, 2^-60..2^100", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 160), dim3(256), 0, 0, 10, 67, cnt, bad); });
    run("sqrt v_rsq + fma correction, all normals", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 254), dim3(256), 0, 0, 6, 1, cnt, bad); });
    run("sqrt v_sqrt+fix, all normals", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 254), dim3(256), 0, 0, 1, 1, cnt, bad); });
    run("sqrt v_rsq + Goldschmidt + correction", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 7, 67, cnt, bad); });
    run("sqrt v_sqrt + fma correction (rsq h)", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 120), dim3(256), 0, 0, 8, 67, cnt, bad); });
    run("rcp  raw v_rcp_f32, 2^-40..2^40", [&] { hipLaunchKernelGGL(k_unary, dim3(1 << 15, 80), dim3(256), 0, 0, 5, 87, cnt, bad); });
    // b in [2^-8, 2^8), a in [2^-40, 2^24): quotients 2^-48 .. 2^32 (normal)
    for (int rep = 0; rep < 4; ++rep)
        run("div  q0+fma, b 2^-8..2^8", [&] { hipLaunchKernelGGL(k_div, dim3(16384), dim3(256), 0, 0, 0x1234567ull + rep, 512, 87, 119, cnt, bad); });
    return 0;
}
