/* Captures the x86 rsqrtss table this repo uses to emulate
 * InverseSquareRoot / v3::NormalizeFast (reference x64_math.h:71-74,246-257)
 * bit-exactly on the GPU and in the oracle.
 *
 * Run on an Intel host (the reference's probe host family):
 *   gcc -O2 -msse2 make_rsqrt_lut.c -o make_lut && ./make_lut rsqrt_lut_intel.bin
 * It writes lut[par*1024 + k] = rsqrtss(2^par * (1 + k/1024)) and then
 * verifies, for EVERY float in [1e-9, 1e9], that
 *   rsqrtss(x) == lut[par(x)*1024 + top10(x)] * 2^-((e(x)-par(x))/2)
 * i.e. that the hardware result depends only on the exponent parity and the
 * top 10 mantissa bits.  Exit status 1 if any input disagrees. */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float rsq(float x) { return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x))); }
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float bf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char **argv)
{
    static float lut[2048];
    for (uint32_t e = 0; e < 2; ++e)
        for (uint32_t k = 0; k < 1024; ++k) lut[e * 1024 + k] = rsq(bf(((127u + e) << 23) | (k << 13)));
    long bad = 0, n = 0;
    for (uint32_t u = fb(1e-9f); u < fb(1e9f); ++u, ++n) {
        int32_t e = (int32_t)(u >> 23) - 127;
        uint32_t par = (uint32_t)e & 1u;
        uint32_t base = fb(lut[par * 1024 + ((u >> 13) & 1023u)]);
        uint32_t pred = base - ((uint32_t)((e - (int32_t)par) / 2) << 23);
        if (pred != fb(rsq(bf(u)))) ++bad;
    }
    printf("checked %ld inputs, %ld disagree\n", n, bad);
    FILE *f = fopen(argc > 1 ? argv[1] : "rsqrt_lut_intel.bin", "wb");
    if (!f) return 2;
    fwrite(lut, 4, 2048, f);
    fclose(f);
    return bad ? 1 : 0;
}
