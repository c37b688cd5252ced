// rt_kernel.hip — CDNA4 (gfx950) trace kernel for the brute-force sphere path.
//
// Replaces the reference's tile callback RenderTile / RenderTileScalar
// (main.cpp:348-495 / 497-640) and its lane-4 math layer (x64_math.h,
// base.h:474-887).  A wave owns a small pixel tile with P lanes per pixel;
// each lane traces its pixel's samples k = j, j+P, ... and the pixel's owner
// lane folds every finished sample into the running mean strictly in sample
// order, so the result is bit-identical to one thread per pixel folding all
// of this launch's frames.  The reference's 4-wide SIMD lanes become the four
// per-residue-class minima each lane carries.
//
// Exactness: built with -ffp-contract=off (every op rounds separately, as the
// reference's SSE lane ops do), IEEE f32 denormals, correctly rounded sqrt and
// division (short verified sequences where their range is guaranteed); the
// one FMA the reference's -mfma build emits (Reflectance, main.cpp:299) is an
// explicit fmaf; rsqrtss is reproduced by table.
//
// Work shape: lanes alternate between starting primary rays
// and gathering secondary segments; primary rays test only the sphere groups
// their tile's cone can reach (tiles whose cone reaches none fold their
// samples without tracing); secondary rays run an FMA prefilter with a proven
// error bound and re-test exactly only the sphere pairs it flags.  Sphere
// groups are wave-uniform: read through the scalar cache into SGPRs (SRC_SMEM)
// or, for A/B, from the block's LDS copy (SRC_LDS); per-lane gathers (winning
// sphere, material, r^2 of flagged groups, rsqrt table) hit the LDS copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_kernel.h"

namespace rtk {

constexpr float kEps = 1e-4f;   // base.h:889 F32Epsilon
constexpr float kFMax = 1e30f;  // base.h:891 F32Max
constexpr float kPfDirTol = 1.0f / 65536.0f;  // |1 - |D|^2| bound of the secondary prefilter (host: rt_host.cpp)
// RandomFloat's (Max-Min)/(f64)(u32)-1 rounded to f32 (base.h:985), for the
// three ranges the path uses: (-0.5,0.5) and (0,1) -> 1, (-1,1) -> 2.
constexpr float kInvRange1 = (float)(1.0 / 4294967295.0);
constexpr float kInvRange2 = (float)(2.0 / 4294967295.0);

__device__ __forceinline__ uint32_t pcg(uint64_t &s) {  // base.h:954-963
    const uint64_t old = s;
    s = old * 6364136223846793005ULL + 1442695040888963407ULL;
    const uint32_t v = (uint32_t)(old >> 32) ^ (uint32_t)old;
    return __builtin_amdgcn_alignbit(v, v, (uint32_t)(old >> 59));  // RotateRight32
}

__device__ __forceinline__ float rand_float(uint64_t &s, float lo, float inv) {  // base.h:983-989
    const float r = (float)pcg(s) * inv;
    return r + lo;
}

__device__ __forceinline__ uint64_t seed_mix(uint64_t i) {  // main.cpp:668-675
    uint64_t s = 0x420247153476526ULL * i;
    s += 0x8442885C91A5C8DULL;
    s ^= s >> ((7u + i) % 64u);
    s ^= s << 23;
    s ^= s >> ((0x29u ^ i) % 64u);
    s = (s * 0x11C19226CEB4769AULL) + 0x1105404122082911ULL;
    s ^= s << 19;
    s ^= s >> 13;
    return s;
}

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    const float px = ax * bx, py = ay * by, pz = az * bz;  // x64_math.h:224-227
    return (px + py) + pz;
}

// Short correctly rounded sequences (each checked against the compiler's
// IEEE sequence by scripts/mathcheck.hip on gfx950: rcp_rn and sqrt_rn
// exhaustively over every f32 in [2^-40, 2^40] / [2^-60, 2^60], div_rn on
// 8.6e9 random and edge-case pairs; all bit-identical).
// RN(1/b) for b in [2^-40, 2^40]: v_rcp_f32 (< 1 ulp) + one Newton step.
__device__ __forceinline__ float rcp_rn(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}

// RN(sqrt(x)) for x = 0 or x in [2^-60, 2^60] (Markstein): y = v_rsq_f32(x),
// g = RN(x y), h = y / 2, r = x - g^2 (one fma, exact), result RN(g + r h).
// scripts/mathcheck.hip finds it bit-identical to the IEEE sqrt on every f32 of
// the range (mode 6, profiles/r06q_mathcheck.txt).  x = 0: v_rsq gives +inf,
// clamped to 2^64 so g = 0 and the result is +0 (the range's y is below 2^30).
// Five full-rate ops besides the transcendental, against eight for v_sqrt_f32
// and its two +-1 ulp residual tests (round 5's form, RTK_SQRT_FIX=2 in
// experiment builds): C2 +2.5 %, RTWeekend +2.3 % (profiles/r06q_sqrt_ab.txt).
#ifndef RTK_SQRT_FIX
#define RTK_SQRT_FIX 4
#endif
__device__ __forceinline__ float sqrt_rn(float x, float *rsq = nullptr) {
    if (RTK_SQRT_FIX == 4) {
        const float y = __builtin_fminf(__builtin_amdgcn_rsqf(x), 0x1p64f);
        if (rsq) *rsq = y;
        const float g = x * y, h = 0.5f * y;
        return __builtin_fmaf(__builtin_fmaf(-g, g, x), h, g);
    }
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = s;
    if (RTK_SQRT_FIX == 1 || RTK_SQRT_FIX == 2) r = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
    if (RTK_SQRT_FIX == 2 || RTK_SQRT_FIX == 3) r = __builtin_fmaf(-sp, s, x) > 0.0f ? sp : r;
    return r;
}

// RN(a/b) from y = RN(1/b) (Markstein: q0 = a*y, exact residual, one fma
// correction) for b > 0 and a == +0 or |a/b| >= 2^-100 (no underflow in the
// residual).  a == -0 would come out +0: neither caller divides one (the film
// numerator is never -0; normalize sends any zero quotient to its IEEE path).
__device__ __forceinline__ float div_rn(float a, float b, float y) {
    const float q0 = a * y;
    return __builtin_fmaf(__builtin_fmaf(-q0, b, a), y, q0);
}

// The running-mean weights of the frame after pc folded ones (main.cpp:484-487):
// {RN(1 / (f32)(pc + 1)), RN((f32)pc / (f32)(pc + 1))}, the reference's f32
// divisions, by the short sequences: n = (f32)(pc + 1) is in [1, 2^32], inside
// rcp_rn's verified range, so RN(1/n) is rcp_rn(n) itself, and pc / n is +0 or
// >= 1/2 (div_rn's condition).  (The host keeps pc + 1 below 2^32: rt_trace.)
__device__ __forceinline__ float2 fold_weights(uint32_t pc) {
    const float n = (float)(pc + 1u);
    const float y = rcp_rn(n);
    return make_float2(y, div_rn((float)pc, n, y));
}

// v3::Normalize (x64_math.h:234-245): IEEE divide by the correctly rounded
// sqrt, zero when len^2 <= 1e-4.  Fast path: one reciprocal shared by the
// three quotients; lanes outside its proven range (a quotient below 2^-99
// or len above 2^40) take the compiler's IEEE sequence.
__device__ __forceinline__ void normalize(float &x, float &y, float &z) {
    const float l2 = dot3(x, y, z, x, y, z);
    const bool keep = l2 > kEps;
#ifndef RTK_NORM_RSQ
#define RTK_NORM_RSQ 0
#endif
    float rq = 0.0f;
    const float len = sqrt_rn(l2, RTK_NORM_RSQ ? &rq : nullptr);
    float inv;
    if (RTK_NORM_RSQ) {
        // RN(1/len) by one Newton step from sqrt_rn's v_rsq_f32(l2); exact except when len's mantissa is all
        // ones (len just under a power of two, 1/len next to a midpoint): those lanes take rcp_rn
        inv = __builtin_fmaf(__builtin_fmaf(-len, rq, 1.0f), rq, rq);
        if (__builtin_expect((__float_as_uint(len) & 0x7FFFFFu) == 0x7FFFFFu, 0)) {
            asm volatile("");
            inv = rcp_rn(len);
        }
    } else {
        inv = rcp_rn(len);
    }
    float qx = div_rn(x, len, inv), qy = div_rn(y, len, inv), qz = div_rn(z, len, inv);
    // (a zero component also takes the IEEE path: rare, and exact either way)
    const float m = __builtin_fminf(__builtin_fminf(__builtin_fabsf(qx), __builtin_fabsf(qy)), __builtin_fabsf(qz));
    if (__builtin_expect(keep && (m < 0x1p-99f || len > 0x1p40f), 0)) {
        qx = x / len;
        qy = y / len;
        qz = z / len;
    }
    x = keep ? qx : 0.0f;
    y = keep ? qy : 0.0f;
    z = keep ? qz : 0.0f;
}

// rsqrtss (x64_math.h:71-74) from the 2x1024 table: exponent parity + top
// 10 mantissa bits pick the entry, the remaining even exponent scales it.
// The table sits in the block's LDS image, or (large scenes, in_lds false:
// the LDS budget goes to occupancy) is read from HBM through the caches.
struct Lut {
    const float *lds, *glob;
    bool in_lds;  // wave-uniform
};

// For a positive normal v with unbiased exponent e: the entry is
// (e & 1) * 1024 + mantissa[22:13], i.e. bits [23:13] of v with bit 23 (the
// biased exponent's parity, the opposite of e's) flipped; the scale is
// floor(e / 2), which is (int)(bits(v) - bits(1.0f)) >> 24 (the mantissa adds
// less than half a unit of that shift).  Checked against the direct form on
// every positive normal f32 (index and result bits): two bit-field ops instead
// of five, most of them the half-rate shift class.
__device__ __forceinline__ float rsqrt_x86(const Lut &lut, float v) {
    const uint32_t u = __float_as_uint(v);
    const uint32_t idx = ((u >> 13) & 2047u) ^ 1024u;
    const float base = lut.in_lds ? lut.lds[idx] : lut.glob[idx];
    const int32_t sh = (int32_t)(u - 0x3F800000u) >> 24;
    return __uint_as_float(__float_as_uint(base) - ((uint32_t)sh << 23));
}

__device__ __forceinline__ float saturate(float v) {  // x64_math.h:97-101
    if (v < 0.0f) return 0.0f;
    if (v > 1.0f) return 1.0f;
    return v;
}

__device__ __forceinline__ uint32_t to_u8(float v) {  // main.cpp:341-343
    const float s = saturate(v) * 255.0f;
    if (s != s) return 0u;
    return (uint32_t)(int32_t)s & 0xFFu;
}

__device__ __forceinline__ float linear_to_srgb(float l) {  // main.cpp:312-329
    l = saturate(l);
    return l < 0.0031308f ? l * 12.92f : sqrt_rn(l);  // l in [0.0031308, 1]
}

// The exact-pow branch of LinearToSRGB (main.cpp:320-321, '#if 0' in the
// reference; RT_FLAG_SRGB_POW).  powf there is libm's (musl in the WASM build,
// glibc on Linux: the same algorithm, not correctly rounded); here the f64
// pow rounded once to f32.  The two differ in the last f32 bit on ~46k of the
// 70.4M inputs in [0.0031308, 1], and the RGBA8 byte on none of them
// (exhaustive: tests/test_srgb_pow.py on the CPU, and the GPU's own bytes
// against the oracle's over the same range in tests/test_gpu_parity.py).
// Unfused, as wasm32 has no FMA.
__device__ __forceinline__ float linear_to_srgb_pow(float l) {
    l = saturate(l);
    if (l < 0.0031308f) return l * 12.92f;
    const float p = (float)pow((double)l, (double)(1.0f / 2.4f));
    return 1.055f * p - 0.055f;
}

// ColorFromV4(LinearToSRGB(v)) (main.cpp:340-346, 490).
__device__ __forceinline__ uint32_t rgba8(float x, float y, float z, bool pw) {
    if (pw)
        return to_u8(linear_to_srgb_pow(x)) | (to_u8(linear_to_srgb_pow(y)) << 8) |
               (to_u8(linear_to_srgb_pow(z)) << 16) | (255u << 24);
    return to_u8(linear_to_srgb(x)) | (to_u8(linear_to_srgb(y)) << 8) | (to_u8(linear_to_srgb(z)) << 16) |
           (255u << 24);
}

// r0 = ((1 - eta)/(1 + eta))^2 comes from the sphere record: the host's IEEE
// division and product per material and side (rt_host.cpp put_material), the
// same bits as the kernel's own (RTWeekend +0.4 %, its 8-rank share +1.3 %,
// profiles/r06s_diel_tab_ab.txt)
__device__ __forceinline__ float reflectance(float cos_t, float r0) {  // main.cpp:292-300
    float r1 = 1.0f - cos_t;
    r1 = r1 * r1 * r1 * r1 * r1;
    return __builtin_fmaf(1.0f - r0, r1, r0);  // contracted by the reference's -mfma build
}

typedef float f2 __attribute__((ext_vector_type(2)));

struct Sample {
    f2 rx, ry, rz;     // {origin, direction} per axis (the packed pair test reads them in place)
    float ax, ay, az;  // attenuation
    float cx, cy, cz;  // output colour
    uint64_t rng;
    uint32_t bounce;
};

// Jittered primary ray (main.cpp:375-385).
// The kernel's by-value TraceArgs re-read from the kernarg segment (scalar
// loads, K$ hits) at each use: the camera fields start_sample needs are then
// not held in SGPRs across the trace loop, where they were spilled to VGPR
// lanes and restored with ~30 v_readlane per primary round.
typedef const __attribute__((address_space(4))) TraceArgs cargs_t;
__device__ __forceinline__ cargs_t &kernel_args() {
    cargs_t *p = (cargs_t *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));  // opaque per use: the loads stay at the use site
    return *p;
}

template <typename Args>
__device__ __forceinline__ void start_sample(const Args &a, uint32_t x, uint32_t y, uint32_t frame, Sample &p) {
    p.rng = seed_mix(((uint64_t)frame * a.height + y) * a.width + x);
    const float jx = rand_float(p.rng, -0.5f, kInvRange1);
    const float jy = rand_float(p.rng, -0.5f, kInvRange1);
    // ((x + Jx) * 2) / W with W's reciprocal RN(1/W) from the host: the
    // numerator is +0 or >= 2^-24 (Jx = -0.5 + r is never -0), so div_rn's
    // range condition holds
    const float fx = -1.0f + div_rn(((float)x + jx) * 2.0f, (float)a.width, a.inv_width);
    const float fy = -1.0f + div_rn(((float)y + jy) * 2.0f, (float)a.height, a.inv_height);
    const float kx = (fx * a.film_w) * 0.5f;
    const float ky = (fy * a.film_h) * 0.5f;
    const float px = (a.film_center[0] + kx * a.cam_x[0]) + ky * a.cam_y[0];
    const float py = (a.film_center[1] + kx * a.cam_x[1]) + ky * a.cam_y[1];
    const float pz = (a.film_center[2] + kx * a.cam_x[2]) + ky * a.cam_y[2];
    p.rx.x = a.cam_pos[0];
    p.ry.x = a.cam_pos[1];
    p.rz.x = a.cam_pos[2];
    float dx = px - p.rx.x, dy = py - p.ry.x, dz = pz - p.rz.x;
    normalize(dx, dy, dz);
    p.rx.y = dx;
    p.ry.y = dy;
    p.rz.y = dz;
    p.ax = p.ay = p.az = 1.0f;
    p.cx = p.cy = p.cz = 0.0f;
    p.bounce = 0;
}

// Emission, attenuation and the next direction (main.cpp:446-481).
__device__ __forceinline__ void shade(const Lut &lut, float4 col_spec, float4 emis_ior, const float4 *diel, float hx,
                                      float hy, float hz, bool inside, Sample &p) {
    p.cx = p.cx + emis_ior.x * p.ax;
    p.cy = p.cy + emis_ior.y * p.ay;
    p.cz = p.cz + emis_ior.z * p.az;
    p.ax = p.ax * col_spec.x;
    p.ay = p.ay * col_spec.y;
    p.az = p.az * col_spec.z;
    float nx = hx, ny = hy, nz = hz;
    normalize(nx, ny, nz);
    const float k2 = 2.0f * dot3(p.rx.y, p.ry.y, p.rz.y, nx, ny, nz);
    const float bx = p.rx.y - k2 * nx, by = p.ry.y - k2 * ny, bz = p.rz.y - k2 * nz;  // PureBounce
    if (inside) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
    const float ior = emis_ior.w;
    if (ior == 0.0f) {
        float rx = rand_float(p.rng, -1.0f, kInvRange2);
        float ry = rand_float(p.rng, -1.0f, kInvRange2);
        float rz = rand_float(p.rng, -1.0f, kInvRange2);
        const float l2 = dot3(rx, ry, rz, rx, ry, rz);  // v3::NormalizeFast
        const bool keep = l2 > kEps;
        const float inv = rsqrt_x86(lut, l2);
        rx = keep ? rx * inv : 0.0f;
        ry = keep ? ry * inv : 0.0f;
        rz = keep ? rz * inv : 0.0f;
        const float s = col_spec.w;
        const float om = 1.0f - s;
        float dx = om * (nx + rx) + s * bx;
        float dy = om * (ny + ry) + s * by;
        float dz = om * (nz + rz) + s * bz;
        normalize(dx, dy, dz);
        p.rx.y = dx;
        p.ry.y = dy;
        p.rz.y = dz;
    } else {
        // {1/IOR, r0 outside, r0 inside} of the record's row 3 (dielectric lanes only)
        const float4 dq = *diel;
        const float eta = inside ? ior : dq.x;
        const float dd = dot3(-p.rx.y, -p.ry.y, -p.rz.y, nx, ny, nz);
        const float cos_t = dd < 1.0f ? dd : 1.0f;  // _mm_min_ss
        // 1 - c*c and |1 - q.q| are 0 or >= 2^-25 (or NaN): inside sqrt_rn's range
        const float sin_t = sqrt_rn(1.0f - cos_t * cos_t);
        const bool cant = eta * sin_t > 1.0f;
        const float qx = eta * (p.rx.y + cos_t * nx);
        const float qy = eta * (p.ry.y + cos_t * ny);
        const float qz = eta * (p.rz.y + cos_t * nz);
        const float q = -sqrt_rn(__builtin_fabsf(1.0f - dot3(qx, qy, qz, qx, qy, qz)));
        float rx = qx + q * nx, ry = qy + q * ny, rz = qz + q * nz;
        normalize(rx, ry, rz);
        bool refl = cant;
        if (!refl) refl = reflectance(cos_t, inside ? dq.z : dq.y) > rand_float(p.rng, 0.0f, kInvRange1);
        if (refl && !inside) {
            p.rx.y = bx;
            p.ry.y = by;
            p.rz.y = bz;
        } else {
            p.rx.y = rx;
            p.ry.y = ry;
            p.rz.y = rz;
        }
    }
}

struct Group {
    float x[4], y[4], z[4], r2[4];
    float r2p[4];  // prefilter threshold r^2 + E (see pair_prefilter)
};

__device__ __forceinline__ void group_rows(Group &G, float4 x, float4 y, float4 z, float4 r2p, float4 r2) {
    G.x[0] = x.x; G.x[1] = x.y; G.x[2] = x.z; G.x[3] = x.w;
    G.y[0] = y.x; G.y[1] = y.y; G.y[2] = y.z; G.y[3] = y.w;
    G.z[0] = z.x; G.z[1] = z.y; G.z[2] = z.z; G.z[3] = z.w;
    G.r2p[0] = r2p.x; G.r2p[1] = r2p.y; G.r2p[2] = r2p.z; G.r2p[3] = r2p.w;
    G.r2[0] = r2.x; G.r2[1] = r2.y; G.r2[2] = r2.z; G.r2[3] = r2.w;
}

// Group rows from the constant address space: read-only for the kernel's
// lifetime, so a wave-uniform address always becomes s_loads into SGPRs
// (immediate offsets from one base: rows 0-3 one dwordx16, row 4 a dwordx4).
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) v4f_t cv4f_t;
__device__ __forceinline__ float4 f4(v4f_t v) { return make_float4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ Group load_group_at(cv4f_t *cg) {
    Group G;
    group_rows(G, f4(cg[kRowX]), f4(cg[kRowY]), f4(cg[kRowZ]), f4(cg[kRowR2P]), f4(cg[kRowR2]));
    return G;
}

template <int SRC>
__device__ __forceinline__ Group load_group(const TraceArgs &a, const float4 *lds_groups, uint32_t g) {
    if (SRC == kSrcSmem) return load_group_at((cv4f_t *)a.groups + kGroupF4 * g);
    Group G;
    const float4 *r = lds_groups + kGroupF4 * g;
    group_rows(G, r[kRowX], r[kRowY], r[kRowZ], r[kRowR2P], r[kRowR2]);
    return G;
}

// The shared part of one sphere test: T, |C - D*T|^2 (main.cpp:401-407).
__device__ __forceinline__ void sphere_core(const Sample &p, float sx, float sy, float sz, float &T, float &dist) {
    const float cx = sx - p.rx.x, cy = sy - p.ry.x, cz = sz - p.rz.x;
    T = dot3(cx, cy, cz, p.rx.y, p.ry.y, p.rz.y);
    const float qx = cx - p.rx.y * T, qy = cy - p.ry.y * T, qz = cz - p.rz.y * T;
    dist = dot3(qx, qy, qz, qx, qy, qz);
}

// Per-lane hit state.  SIMD rules: the reference's four lane minima
// (MinT / MaterialIndex / InsideSphere, main.cpp:394-396), one per residue
// class s & 3.  Scalar rules use slot 0 only (main.cpp:541-545).
struct Hit {
    float t0, t1, t2, t3;
    uint32_t g0, g1, g2, g3;
    uint32_t ins;
};

__device__ __forceinline__ void hit_reset(Hit &h) {
    h.t0 = h.t1 = h.t2 = h.t3 = kFMax;
    h.g0 = h.g1 = h.g2 = h.g3 = 0;
    h.ins = 0;
}

// Exact intersection of one candidate sphere (main.cpp:413-429 / 561-578),
// given its T and |C - D*T|^2 from the packed distance test.
// fast: the host proved every hittable r^2 is 0 or in [2^-36, 2^60], so
// r^2 - dist (positive, hence >= ulp(r^2)/2, or exactly 0) is inside sqrt_rn's
// verified range.
template <bool SIMD, int L>
__device__ __forceinline__ void candidate(Hit &h, uint32_t g, float T, float dist, float r2, bool fast) {
    const float X = fast ? sqrt_rn(r2 - dist) : __builtin_sqrtf(r2 - dist);
    float it = T - X;
    const bool in = it < kEps;
    if (in) it = T + X;
    if (SIMD) {
        float &tl = L == 0 ? h.t0 : L == 1 ? h.t1 : L == 2 ? h.t2 : h.t3;
        uint32_t &gl = L == 0 ? h.g0 : L == 1 ? h.g1 : L == 2 ? h.g2 : h.g3;
        if (it < tl && it > kEps) {  // strict: the earliest group keeps a tie
            tl = it;
            gl = g;
            h.ins |= (in ? 1u : 0u) << L;  // sticky OR (main.cpp:425)
        }
    } else {
        if (!(it > h.t0) && !(it < kEps)) {  // the later sphere wins a tie
            h.t0 = it;
            h.g0 = 4u * g + (uint32_t)L;
            h.ins = in ? 1u : 0u;
        }
    }
}


// T and |C - D*T|^2 for two spheres of a group at once: every f32 op of
// main.cpp:401-407 becomes one packed v_pk_{add,mul}_f32 over the pair (same
// IEEE rounding per element; a packed op issues at the cost of a scalar one
// on gfx950, so this halves the sphere loop's VALU instructions).
// The ray as three {origin, direction} register pairs: a packed op can then
// broadcast either half to both lanes with op_sel / op_sel_hi, so the pair
// test needs no duplicated (splat) copies of the ray.
struct RayPk {
    f2 x, y, z;  // {o, d} per axis
};

__device__ __forceinline__ f2 pair_dist(const RayPk &r, f2 sx, f2 sy, f2 sz, f2 &T) {
    f2 cx, cy, cz, t, d;
    // c = s - o ; T = (cx*dx + cy*dy) + cz*dz ; q = c - d*T (in c) ;
    // dist = (qx*qx + qy*qy) + qz*qz  -- op for op the reference's f32 sequence
    asm("v_pk_add_f32 %[cx], %[sx], %[rx] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[cy], %[sy], %[ry] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[cz], %[sz], %[rz] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[t], %[cx], %[rx] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_mul_f32 %[d], %[cy], %[ry] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[T], %[t], %[d]\n\t"
        "v_pk_mul_f32 %[t], %[cz], %[rz] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[T], %[T], %[t]\n\t"
        "v_pk_mul_f32 %[t], %[rx], %[T] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[cx], %[cx], %[t] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[t], %[ry], %[T] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[cy], %[cy], %[t] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[t], %[rz], %[T] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[cz], %[cz], %[t] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[d], %[cx], %[cx]\n\t"
        "v_pk_mul_f32 %[t], %[cy], %[cy]\n\t"
        "v_pk_add_f32 %[d], %[d], %[t]\n\t"
        "v_pk_mul_f32 %[t], %[cz], %[cz]\n\t"
        "v_pk_add_f32 %[d], %[d], %[t]"
        : [cx] "=&v"(cx), [cy] "=&v"(cy), [cz] "=&v"(cz), [t] "=&v"(t), [T] "=&v"(T), [d] "=&v"(d)
        : [sx] "s"(sx), [sy] "s"(sy), [sz] "s"(sz), [rx] "v"(r.x), [ry] "v"(r.y), [rz] "v"(r.z));
    return d;
}

// Secondary-ray prefilter: an FMA estimate of |C - D*T|^2 for two spheres
// in 10 packed ops instead of the exact test's 19:
//   C = S - O ;  cc = |C|^2 ;  T = C.D ;  e = cc - T*T      (fused)
// For |D|^2 within K = 2^-16 of 1 and every origin on a sphere of the scene
// (true for all secondary rays: NextRayOrigin is a hit point), |e - dist|
// where dist is the reference's exactly-rounded value (main.cpp:401-407) is
// below E_j = M_j (32u + 1.01K), u = 2^-24, M_j a bound on |C|^2 for
// sphere j over every such origin (derivation: DESIGN.md).  The host stores
// r2p_j >= r^2_j + E_j (rounded up), so e >= r2p proves dist > r^2 -- the
// sphere is missed under both rule sets -- and only groups where some lane
// fails that proof run the exact test.  A wave with any lane outside the
// |D|^2 bound runs the exact loop instead.
__device__ __forceinline__ f2 pair_prefilter(const RayPk &r, f2 sx, f2 sy, f2 sz, f2 &T, f2 &cc) {
    f2 cx, cy, cz, e;
    asm("v_pk_add_f32 %[cx], %[sx], %[rx] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[cy], %[sy], %[ry] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[cz], %[sz], %[rz] op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[cc], %[cz], %[cz]\n\t"
        "v_pk_fma_f32 %[cc], %[cy], %[cy], %[cc]\n\t"
        "v_pk_fma_f32 %[cc], %[cx], %[cx], %[cc]\n\t"
        "v_pk_mul_f32 %[T], %[cx], %[rx] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_fma_f32 %[T], %[cy], %[ry], %[T] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[T], %[cz], %[rz], %[T] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[e], %[T], %[T], %[cc] neg_lo:[1,0,0] neg_hi:[1,0,0]"
        : [cx] "=&v"(cx), [cy] "=&v"(cy), [cz] "=&v"(cz), [cc] "=&v"(cc), [T] "=&v"(T), [e] "=&v"(e)
        : [sx] "s"(sx), [sy] "s"(sy), [sz] "s"(sz), [rx] "v"(r.x), [ry] "v"(r.y), [rz] "v"(r.z));
    return e;
}

// Group g for a secondary ray through the prefilter: one wave branch per
// group, and inside it one per sphere pair a lane could hit -- only such a pair
// reruns the exact packed test (same ops as test_group) and the exact candidate
// logic decides, so results are identical.  (Measured: +5.5 % on C2 over one
// exact recheck of both pairs per flagged group.)
// The prefilter needs rows 0-3 only (SGPRs); r^2 of a flagged group comes
// from the block's LDS copy.
// The exact recheck of one group's flagged sphere pairs (f01, f23): only such
// a pair reruns the exact packed test (same ops as test_group) and the exact
// candidate logic decides, so results are identical.
// GS (scenes beyond the LDS image, rt_kernel.h kMaxLdsGroups): the group's r^2
// row (wave-uniform g) comes through the scalar cache instead of LDS.
template <bool SIMD, bool GS>
__device__ __forceinline__ void recheck_pairs(const TraceArgs &a, const float4 *lds_groups, const Group &G, uint32_t g,
                                              const RayPk &p, Hit &h, bool f01, bool f23) {
    const float4 r2 = GS ? f4(((cv4f_t *)a.groups)[kGroupF4 * g + kRowR2]) : lds_groups[kGroupF4 * g + kRowR2];
    if (f01) {
        f2 T01;
        const f2 d01 = pair_dist(p, f2{G.x[0], G.x[1]}, f2{G.y[0], G.y[1]}, f2{G.z[0], G.z[1]}, T01);
        const uint32_t s0 = 4u * g;
        const bool h0 = SIMD ? d01.x < r2.x : s0 + 0u < a.n_spheres && !(d01.x > r2.x);
        const bool h1 = SIMD ? d01.y < r2.y : s0 + 1u < a.n_spheres && !(d01.y > r2.y);
        if (h0) candidate<SIMD, 0>(h, g, T01.x, d01.x, r2.x, a.fast_sqrt != 0u);
        if (h1) candidate<SIMD, 1>(h, g, T01.y, d01.y, r2.y, a.fast_sqrt != 0u);
    }
    if (f23) {
        f2 T23;
        const f2 d23 = pair_dist(p, f2{G.x[2], G.x[3]}, f2{G.y[2], G.y[3]}, f2{G.z[2], G.z[3]}, T23);
        const uint32_t s0 = 4u * g;
        const bool h2 = SIMD ? d23.x < r2.z : s0 + 2u < a.n_spheres && !(d23.x > r2.z);
        const bool h3 = SIMD ? d23.y < r2.w : s0 + 3u < a.n_spheres && !(d23.y > r2.w);
        if (h2) candidate<SIMD, 2>(h, g, T23.x, d23.x, r2.z, a.fast_sqrt != 0u);
        if (h3) candidate<SIMD, 3>(h, g, T23.y, d23.y, r2.w, a.fast_sqrt != 0u);
    }
}

// Per-lane ("relative") prefilter threshold: t = RN(cc * 2^-15 + r^2) with
// cc = the lane's computed |C|^2, where row 3 holds r^2 (-inf: never hit).
// The error bound of e (and of the reference-rounded dist) scales with the
// lane's own |C|^2 instead of the scene-wide M_j, so the test still proves
// misses in scenes whose M_j bound is useless (RTWeekend's ground sphere
// makes M ~ 1.6e4 against r^2 ~ 1.6e-4).  Proof: with
// |C|^2 <= cc (1 + 5u) and E = 23.5u + K(1+K) the combined error of e and of
// the reference's dist relative to |C|^2, e >= t gives dist > r^2 whenever
// cc >= r^2 / 232 (then cc (2^-15 (1-u) - (1+5u) E) >= u r^2 covers t's own
// rounding); and when cc < r^2 / 232, e <= cc < t, so nothing is skipped.
constexpr float kPfRel = 0x1p-15f;

// Prefilter flags of group G's two sphere pairs for this lane's ray.
template <bool REL>
__device__ __forceinline__ void prefilter_group(const Group &G, const RayPk &p, bool &f01, bool &f23) {
    f2 T01, T23, c01, c23;
    const f2 e01 = pair_prefilter(p, f2{G.x[0], G.x[1]}, f2{G.y[0], G.y[1]}, f2{G.z[0], G.z[1]}, T01, c01);
    const f2 e23 = pair_prefilter(p, f2{G.x[2], G.x[3]}, f2{G.y[2], G.y[3]}, f2{G.z[2], G.z[3]}, T23, c23);
    if (REL) {
        f01 = !(e01.x >= __builtin_fmaf(c01.x, kPfRel, G.r2p[0])) | !(e01.y >= __builtin_fmaf(c01.y, kPfRel, G.r2p[1]));
        f23 = !(e23.x >= __builtin_fmaf(c23.x, kPfRel, G.r2p[2])) | !(e23.y >= __builtin_fmaf(c23.y, kPfRel, G.r2p[3]));
    } else {
        f01 = !(e01.x >= G.r2p[0]) | !(e01.y >= G.r2p[1]);
        f23 = !(e23.x >= G.r2p[2]) | !(e23.y >= G.r2p[3]);
    }
}

// Group g for a secondary ray through the prefilter: one wave branch per
// group, and inside it one per flagged pair.  (Measured: +5.5 % on C2 over
// one exact recheck of both pairs per flagged group.)
struct PfStats {
    uint32_t groups, cl_tested, pairs, cl_top_entered, lane_pairs;
};

template <bool SIMD, bool GS, bool REL>
__device__ __forceinline__ void test_group_pf(const TraceArgs &a, const float4 *lds_groups, const Group &G, uint32_t g,
                                              const RayPk &p, Hit &h, PfStats *ps = nullptr) {
    bool f01, f23;
    prefilter_group<REL>(G, p, f01, f23);
    if (ps) {
        ps->groups += __ballot(f01 | f23) != 0;
        ps->pairs += (__ballot(f01) != 0) + (__ballot(f23) != 0);
        ps->lane_pairs += __builtin_popcountll(__ballot(f01)) + __builtin_popcountll(__ballot(f23));
    }
    if (f01 | f23) recheck_pairs<SIMD, GS>(a, lds_groups, G, g, p, h, f01, f23);
}

template <bool SIMD>
__device__ __forceinline__ void test_group(const TraceArgs &a, const Group &G, uint32_t g, const RayPk &p, Hit &h,
                                           uint32_t *hit_groups);

// Rows 0-3 only (one s_load_dwordx16): what the prefilter reads.
__device__ __forceinline__ Group load_group_pf_at(cv4f_t *cg) {
    Group G;
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    group_rows(G, f4(cg[kRowX]), f4(cg[kRowY]), f4(cg[kRowZ]), f4(cg[kRowR2P]), z4);
    return G;
}

// The full sphere loop over all groups from SGPRs.  PF: secondary rays
// through the prefilter; else the exact test.
template <bool SIMD, bool PF, bool GS, bool REL = false>
__device__ __forceinline__ void all_groups_smem(const TraceArgs &a, const float4 *lds_groups, const RayPk &ray, Hit &h,
                                                uint32_t *hit_groups, PfStats *ps = nullptr) {
    cv4f_t *gp = (cv4f_t *)a.groups;
    // one group in SGPRs at a time: its s_load (scalar-cache hit) is covered
    // by the other waves on the SIMD -- measured as fast as a ping-pong
    // prefetch, at half the SGPRs (and two groups per trip under one branch
    // measured 2 % slower)
    for (uint32_t g = 0; g < a.n_groups; ++g, gp += kGroupF4) {
        const Group G = PF ? load_group_pf_at(gp) : load_group_at(gp);
        if (PF) test_group_pf<SIMD, GS, REL>(a, lds_groups, G, g, ray, h, ps);
        else test_group<SIMD>(a, G, g, ray, h, hit_groups);
    }
}

// The clustered prefilter (secondary rays; rt_host.cpp cluster_table proves
// it).  A wave tests the ray against about sqrt(n) cluster bounding volumes,
// two per packed prefilter, and only the members of a cluster some lane may
// reach run the per-sphere prefilter; a sphere pair some lane may hit sets
// bit (slot >> 1) of the wave's pair mask (W u64 words, SGPRs only; W = 1
// tables carry the bit itself, W = 2 tables the pair index).  The
// exact recheck then walks the flagged groups in ascending order -- the
// reference's order, so the per-class minima, tie rules and sticky inside flags
// come out as in the full loop.  The recheck runs on every lane: a lane whose
// own estimate cleared the pair has a proven miss there, which its exact test
// reproduces, so no per-lane flags are needed.
constexpr int kClWords = 4;  // pair-mask words (n_groups <= 128)
// Per-lane thresholds (pf_relative, rt_host.cpp cluster_table "relative"):
// cluster: e_c >= RN(cc kClRel + R_c); sphere: e >= RN(cc kPfRel + r^2) (kPfRel
// below); behind: T < RN(b - cc kBehindRel).
constexpr float kClRel = 9.2e-4f;               // >= (a + a^2 + E1)(1 + 6u), a = 8.917e-4
constexpr float kBehindRel = 4.5f * 0x1p-24f;    // >= 4.3u (|Q|, |C_j| <= (1 + cc)/2)

// ballot(a && b) as ballot(a) & ballot(b): the backend folds the ballot of a
// single compare into the v_cmp's own lane mask, but materialises the ballot of
// a conjunction through v_cndmask + v_cmp_ne (two VALU per ballot)
__device__ __forceinline__ uint64_t ballot_and(bool a, bool b) {
    return __builtin_amdgcn_ballot_w64(a) & __builtin_amdgcn_ballot_w64(b);
}

// Entry e of the cluster table at byte offset off (a 32-bit offset from the
// table's base keeps the per-entry address arithmetic to one SALU add).
__device__ __forceinline__ cv4f_t *cl_entry(cv4f_t *ct, uint32_t off) {
    return (cv4f_t *)((const __attribute__((address_space(4))) char *)ct + off);
}

// The member pairs [first, first + count) of an entered cluster: a sphere pair
// some lane may hit ORs its word-w bits into every word w of the wave's pair
// mask (rt_kernel.h: the entry's row of word w holds the bit or 0).  The walk is
// SALU-heavy (ballots, mask merges, loop control issue on the CU's one scalar
// unit): C5's member loop at 48 SALU per entry ran 17 % slower than at 34.
// wave[w] |= f ? bits[w] : 0 for every word under one compare of the ballot f:
// s_cselect_b64 per word (the compiler's lowering selects 32-bit halves, two
// per word) -- the merge runs on the CU's one scalar unit for every member.
template <int W>
__device__ __forceinline__ void merge_words(uint64_t (&wave)[kClWords], uint64_t f, const uint64_t (&bits)[W]) {
    uint64_t t0, t1;
    if constexpr (W == 2) {
        asm("s_cmp_lg_u64 %[f], 0\n\t"
            "s_cselect_b64 %[t0], %[b0], 0\n\t"
            "s_cselect_b64 %[t1], %[b1], 0\n\t"
            "s_or_b64 %[w0], %[w0], %[t0]\n\t"
            "s_or_b64 %[w1], %[w1], %[t1]"
            : [w0] "+s"(wave[0]), [w1] "+s"(wave[1]), [t0] "=&s"(t0), [t1] "=&s"(t1)
            : [f] "s"(f), [b0] "s"(bits[0]), [b1] "s"(bits[1])
            : "scc");
    } else {
        static_assert(W == 4, "pair-mask words");
        uint64_t t2, t3;
        asm("s_cmp_lg_u64 %[f], 0\n\t"
            "s_cselect_b64 %[t0], %[b0], 0\n\t"
            "s_cselect_b64 %[t1], %[b1], 0\n\t"
            "s_cselect_b64 %[t2], %[b2], 0\n\t"
            "s_cselect_b64 %[t3], %[b3], 0\n\t"
            "s_or_b64 %[w0], %[w0], %[t0]\n\t"
            "s_or_b64 %[w1], %[w1], %[t1]\n\t"
            "s_or_b64 %[w2], %[w2], %[t2]\n\t"
            "s_or_b64 %[w3], %[w3], %[t3]"
            : [w0] "+s"(wave[0]), [w1] "+s"(wave[1]), [w2] "+s"(wave[2]), [w3] "+s"(wave[3]), [t0] "=&s"(t0),
              [t1] "=&s"(t1), [t2] "=&s"(t2), [t3] "=&s"(t3)
            : [f] "s"(f), [b0] "s"(bits[0]), [b1] "s"(bits[1]), [b2] "s"(bits[2]), [b3] "s"(bits[3])
            : "scc");
    }
}

// an SGPR pointer the compiler cannot see through: loads through it stay where they are written
__device__ __forceinline__ cv4f_t *opaque(cv4f_t *p) {
    asm volatile("" : "+s"(p));
    return p;
}

// The per-lane thresholds of per-lane (REL) tables, both members of an entry
// per packed FMA.  The constants sit in VGPR pairs (kc = {kClRel, kBehindRel},
// kp = {kPfRel, kSlabRel}, aux = {slab_e0, |D.y|}) and op_sel broadcasts one
// half to both lanes: an f32 FMA with a literal and an SGPR row lowered to
// v_mov + v_fmamk, two VALU per threshold where this is half of one.  Every
// value is the same single-rounded FMA as fmaf, so the bits are unchanged.
struct ClConst {
    f2 kc, kp, aux;
};

// A constant in a VGPR, written where the walk starts: a plain constant is
// hoisted to the kernel's entry and held across every loop, which pushed other
// values into scratch.
__device__ __forceinline__ float walk_const(float c) {
    float r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(c));
    return r;
}

// t = cc * kPfRel + r (a member pair's near-line thresholds)
__device__ __forceinline__ f2 member_thr(f2 cc, const ClConst &k, f2 r) {
    f2 t;
    asm("v_pk_fma_f32 %[t], %[cc], %[kp], %[r] op_sel_hi:[1,0,1]" : [t] "=v"(t) : [cc] "v"(cc), [kp] "v"(k.kp), [r] "s"(r));
    return t;
}

// A cluster pair's near-line thresholds t = cc kClRel + R, behind bounds
// b = beta - cc kBehindRel, and the height-slab distance d = |O.y + D.y T - ymid|
// (before the abs) with its limit thr = |D.y| srho + (yhalf + E),
// E = cc kSlabRel + slab_e0 (cluster_pair below).
__device__ __forceinline__ void cluster_thr(f2 cc, const ClConst &k, f2 r, f2 beta, f2 &t, f2 &b) {
    asm("v_pk_fma_f32 %[t], %[cc], %[kc], %[r] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[b], %[cc], %[kc], %[beta] op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[0,1,0] neg_hi:[0,1,0]"
        : [t] "=&v"(t), [b] "=&v"(b)
        : [cc] "v"(cc), [kc] "v"(k.kc), [r] "s"(r), [beta] "s"(beta));
}
__device__ __forceinline__ void cluster_slab(f2 cc, f2 T, const RayPk &ray, const ClConst &k, f2 srho, f2 ymid,
                                             f2 yhalf, f2 &d, f2 &thr) {
    asm("v_pk_fma_f32 %[thr], %[cc], %[kp], %[aux] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "v_pk_add_f32 %[thr], %[yhalf], %[thr]\n\t"
        "v_pk_fma_f32 %[thr], %[aux], %[srho], %[thr] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[d], %[ry], %[T], %[ry] op_sel:[1,0,0] op_sel_hi:[1,1,0]\n\t"
        "v_pk_add_f32 %[d], %[d], %[ymid] neg_lo:[0,1] neg_hi:[0,1]"
        : [thr] "=&v"(thr), [d] "=&v"(d)
        : [cc] "v"(cc), [kp] "v"(k.kp), [aux] "v"(k.aux), [yhalf] "s"(yhalf), [srho] "s"(srho), [ry] "v"(ray.y),
          [T] "v"(T), [ymid] "s"(ymid));
}

template <int W, bool REL>
__device__ __forceinline__ void member_pairs(cv4f_t *ct, uint32_t first, uint32_t count, const RayPk &ray,
                                             uint64_t (&wave)[kClWords], const ClConst &k, PfStats *ps) {
    constexpr uint32_t kEntryBytes = 16u * cl_entry_f4(W, REL);
    if (ps) ps->groups += count;
    const uint32_t end = (first + count) * kEntryBytes;
    for (uint32_t off = first * kEntryBytes; off != end; off += kEntryBytes) {
        cv4f_t *e = cl_entry(ct, off);
        const v4f_t r0 = e[0], r1 = e[1];
        const v4f_t r3 = e[3];
        const v4f_t r2 = W <= 2 ? e[2] : v4f_t{0.0f, 0.0f, 0.0f, 0.0f};
        f2 T, cc;
        const f2 v = pair_prefilter(ray, f2{r0.x, r0.y}, f2{r0.z, r0.w}, f2{r1.x, r1.y}, T, cc);
        // a lane may hit the sphere: near the line, and not wholly behind the origin
        const f2 tr = REL ? member_thr(cc, k, f2{r1.z, r1.w}) : f2{r1.z, r1.w};
        const float t0 = tr.x, t1 = tr.y;
        const float b0 = REL ? __builtin_fmaf(cc.x, -kBehindRel, r3.x) : r3.x;
        const float b1 = REL ? __builtin_fmaf(cc.y, -kBehindRel, r3.y) : r3.y;
        // Members of per-lane (REL) tables take the near-line test only: their behind
        // threshold is a per-lane FMA, and the rule stays at the cluster level
        // (RTWeekend +2.7 % same box; C2's scene-wide table loses 1.7 % without it).
        // Either way a skipped pair is a proven miss.
        constexpr bool kBehind = !REL;
        const uint64_t f0m = kBehind ? ballot_and(!(v.x >= t0), !(T.x < b0)) : __builtin_amdgcn_ballot_w64(!(v.x >= t0));
        const uint64_t f1m = kBehind ? ballot_and(!(v.y >= t1), !(T.y < b1)) : __builtin_amdgcn_ballot_w64(!(v.y >= t1));
        const bool f0 = f0m != 0, f1 = f1m != 0;
        if constexpr (W == 1) {
            const uint64_t b0 = (uint64_t)__float_as_uint(r2.x) | ((uint64_t)__float_as_uint(r2.y) << 32);
            const uint64_t b1 = (uint64_t)__float_as_uint(r2.z) | ((uint64_t)__float_as_uint(r2.w) << 32);
            wave[0] |= (f0 ? b0 : 0ull) | (f1 ? b1 : 0ull);
        } else if constexpr (W == 2) {
            uint64_t bw0[W], bw1[W];  // member 0 and 1 bits in word w
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const v4f_t rb = w == 0 ? r2 : e[3 + w];
                bw0[w] = (uint64_t)__float_as_uint(rb.x) | ((uint64_t)__float_as_uint(rb.y) << 32);
                bw1[w] = (uint64_t)__float_as_uint(rb.z) | ((uint64_t)__float_as_uint(rb.w) << 32);
            }
            merge_words<W>(wave, f0m, bw0);
            merge_words<W>(wave, f1m, bw1);
        } else {
            // four-word tables: a member's four bit rows are read only when some lane flagged it (a
            // uniform branch), so they do not hold 16 SGPRs across every entry's prefilter (RTWeekend
            // +0.7 %; the two-word form keeps its selects: C5 -0.5 % this way, profiles/r05u_lazy_bits_ab.txt)
            if (f0 | f1) {
                cv4f_t *eb = opaque(e);
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    const v4f_t rb = w == 0 ? eb[2] : eb[3 + w];
                    if (f0) wave[w] |= (uint64_t)__float_as_uint(rb.x) | ((uint64_t)__float_as_uint(rb.y) << 32);
                    if (f1) wave[w] |= (uint64_t)__float_as_uint(rb.z) | ((uint64_t)__float_as_uint(rb.w) << 32);
                }
            }
        }
    }
}

// One cluster-pair entry (both levels of the table share the row layout):
// the wave's lanes that may reach cluster 0 / 1 (near the line, not wholly
// behind the origin, and for per-lane tables inside the height slab).
// Height slab (per-lane tables): the line's height over the t range that can
// reach the cluster is c +- |D.y| srho with c = O.y + D.y T; it cannot meet a
// member when that range clears [ymid - yhalf, ymid + yhalf] by the lane's
// margin E (a ground-plane scene: rays leaving the ground cross the thin layer
// of small spheres only near their origin).
template <bool REL, bool SLAB = true, bool BEHIND = true>
__device__ __forceinline__ void cluster_pair(cv4f_t *e, const RayPk &ray, const ClConst &k, uint64_t &m0,
                                             uint64_t &m1) {
    const v4f_t r0 = e[0], r1 = e[1], r3 = e[3];
    f2 T, cc;
    const f2 v = pair_prefilter(ray, f2{r0.x, r0.y}, f2{r0.z, r0.w}, f2{r1.x, r1.y}, T, cc);
    if constexpr (REL) {
        f2 t, b;
        cluster_thr(cc, k, f2{r1.z, r1.w}, f2{r3.x, r3.y}, t, b);
        if (BEHIND) {
            m0 = ballot_and(!(v.x >= t.x), !(T.x < b.x));
            m1 = ballot_and(!(v.y >= t.y), !(T.y < b.y));
        } else {
            m0 = __builtin_amdgcn_ballot_w64(!(v.x >= t.x));
            m1 = __builtin_amdgcn_ballot_w64(!(v.y >= t.y));
        }
        if constexpr (SLAB) {
            const v4f_t r4 = e[4];
            f2 d, thr;
            cluster_slab(cc, T, ray, k, f2{r3.z, r3.w}, f2{r4.x, r4.y}, f2{r4.z, r4.w}, d, thr);
            m0 &= __builtin_amdgcn_ballot_w64(!(__builtin_fabsf(d.x) > thr.x));
            m1 &= __builtin_amdgcn_ballot_w64(!(__builtin_fabsf(d.y) > thr.y));
        }
    } else {
        m0 = ballot_and(!(v.x >= r1.z), !(T.x < r3.x));
        m1 = ballot_and(!(v.y >= r1.w), !(T.y < r3.y));
    }
}

// ps (RTK_STATS): groups += member-pair entries tested, pairs += sphere pairs
// rechecked exactly, lane_pairs += clusters entered (per wave, both levels),
// cl_tested += cluster-pair entries tested (both levels), cl_top_entered += top
// clusters entered (two-level tables).
// Tables of two or more mask words (more than 32 groups) have two levels: a
// top cluster's entry ranges index sub-cluster entries of a few spheres each,
// whose ranges index the member entries (rt_host.cpp cluster_table); the bound
// of a cluster covers every sphere under it, so a skipped top cluster skips
// its sub-clusters' members too.
template <bool SIMD, int W, bool GS, bool REL>
__device__ __forceinline__ void clustered_groups(const TraceArgs &a, const float4 *lds_groups, const RayPk &ray,
                                                 Hit &h, PfStats *ps) {
    cv4f_t *ct = (cv4f_t *)a.clusters;
    uint64_t wave[kClWords] = {0ull, 0ull, 0ull, 0ull};
    constexpr uint32_t kEntryBytes = 16u * cl_entry_f4(W, REL);
    constexpr bool kTwoLevels = W >= 2;
    // per-lane part of the height-slab margin (REL tables; rt_host.cpp cluster_table)
    const float oy = ray.y.x, dy = ray.y.y;
    const float slab_e0 = REL ? __builtin_fmaf(__builtin_fabsf(oy), 0x1p-21f, kSlabRel) : 0.0f;
    ClConst k;
    if constexpr (REL) {
        k.kc = f2{walk_const(kClRel), walk_const(kBehindRel)};
        k.kp = f2{walk_const(kPfRel), walk_const(kSlabRel)};
        k.aux = f2{slab_e0, __builtin_fabsf(dy)};
    }
    // the member pairs of an entered (sub-)cluster pair entry
    auto members = [&](cv4f_t *e, bool in0, bool in1) {
        const v4f_t r2 = e[2];
        if (ps) ps->lane_pairs += (in0 ? 1u : 0u) + (in1 ? 1u : 0u);
        if (in0) member_pairs<W, REL>(ct, __float_as_uint(r2.x), __float_as_uint(r2.y), ray, wave, k, ps);
        if (in1) member_pairs<W, REL>(ct, __float_as_uint(r2.z), __float_as_uint(r2.w), ray, wave, k, ps);
    };
    // the sub-cluster pair entries [first, first + count) of an entered top cluster
    auto subs = [&](uint32_t first, uint32_t count) {
        if (ps) ps->cl_tested += count;
        for (uint32_t off = first * kEntryBytes, end = (first + count) * kEntryBytes; off != end; off += kEntryBytes) {
            cv4f_t *e = cl_entry(ct, off);
            uint64_t m0, m1;
#ifndef RTK_EXP_SUB
#define RTK_EXP_SUB true, true
#endif
            cluster_pair<REL, RTK_EXP_SUB>(e, ray, k, m0, m1);
            members(e, m0 != 0, m1 != 0);
        }
    };
    if (ps) ps->cl_tested += a.n_cpairs;
    for (uint32_t off = 0, end = a.n_cpairs * kEntryBytes; off != end; off += kEntryBytes) {
        cv4f_t *e = cl_entry(ct, off);
        uint64_t m0, m1;
#ifndef RTK_EXP_TOP
#define RTK_EXP_TOP true, true
#endif
        cluster_pair<REL, RTK_EXP_TOP>(e, ray, k, m0, m1);
        if constexpr (kTwoLevels) {
            const v4f_t r2 = e[2];
            if (ps) ps->lane_pairs += (m0 != 0 ? 1u : 0u) + (m1 != 0 ? 1u : 0u);
            if (ps) ps->cl_top_entered += (m0 != 0 ? 1u : 0u) + (m1 != 0 ? 1u : 0u);
            if (m0 != 0) subs(__float_as_uint(r2.x), __float_as_uint(r2.y));
            if (m1 != 0) subs(__float_as_uint(r2.z), __float_as_uint(r2.w));
        } else {
            members(e, m0 != 0, m1 != 0);
        }
    }
    cv4f_t *gp = (cv4f_t *)a.groups;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        uint64_t m = wave[w];
        while (m) {
            const uint32_t q = (uint32_t)__builtin_ctzll(m) & ~1u;  // first pair of the lowest flagged group
            const uint32_t g = 32u * (uint32_t)w + (q >> 1);
            const bool f01 = (m >> q) & 1u, f23 = (m >> (q + 1u)) & 1u;
            m &= ~(3ull << q);
            if (ps) ps->pairs += (f01 ? 1u : 0u) + (f23 ? 1u : 0u);
            recheck_pairs<SIMD, GS>(a, lds_groups, load_group_pf_at(gp + kGroupF4 * g), g, ray, h, f01, f23);
        }
    }
}

// All four spheres of group g; one wave-level branch per group, nested
// branches only for the (rare) lanes that pass the distance test.
template <bool SIMD>
__device__ __forceinline__ void test_group(const TraceArgs &a, const Group &G, uint32_t g, const RayPk &p, Hit &h,
                                           uint32_t *hit_groups) {
    f2 T01, T23;
    const f2 d01 = pair_dist(p, f2{G.x[0], G.x[1]}, f2{G.y[0], G.y[1]}, f2{G.z[0], G.z[1]}, T01);
    const f2 d23 = pair_dist(p, f2{G.x[2], G.x[3]}, f2{G.y[2], G.y[3]}, f2{G.z[2], G.z[3]}, T23);
    bool h0, h1, h2, h3;
    if (SIMD) {  // HitMask = d < r^2 (main.cpp:409)
        h0 = d01.x < G.r2[0];
        h1 = d01.y < G.r2[1];
        h2 = d23.x < G.r2[2];
        h3 = d23.y < G.r2[3];
    } else {  // !(d > r^2) over the Count real spheres only (main.cpp:547,557)
        const uint32_t s0 = 4u * g;
        h0 = s0 + 0u < a.n_spheres && !(d01.x > G.r2[0]);
        h1 = s0 + 1u < a.n_spheres && !(d01.y > G.r2[1]);
        h2 = s0 + 2u < a.n_spheres && !(d23.x > G.r2[2]);
        h3 = s0 + 3u < a.n_spheres && !(d23.y > G.r2[3]);
    }
    if (hit_groups && __ballot(h0 | h1 | h2 | h3)) *hit_groups += 1;
    if (h0 | h1 | h2 | h3) {
        if (h0) candidate<SIMD, 0>(h, g, T01.x, d01.x, G.r2[0], a.fast_sqrt != 0u);
        if (h1) candidate<SIMD, 1>(h, g, T01.y, d01.y, G.r2[1], a.fast_sqrt != 0u);
        if (h2) candidate<SIMD, 2>(h, g, T23.x, d23.x, G.r2[2], a.fast_sqrt != 0u);
        if (h3) candidate<SIMD, 3>(h, g, T23.y, d23.y, G.r2[3], a.fast_sqrt != 0u);
    }
}

// pair_dist for rays that all start at the camera (primary rounds): C = S - O
// is the same on every lane, so its three packed subtractions come from the
// cull pass's table (TraceArgs.prim, computed with the same single f32
// rounding) and the C operands stay in SGPRs -- 16 packed ops instead of 19.
__device__ __forceinline__ f2 pair_dist_c(const RayPk &r, f2 cx, f2 cy, f2 cz, f2 &T) {
    f2 qx, qy, qz, t, d;
    asm("v_pk_mul_f32 %[t], %[cx], %[rx] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_mul_f32 %[d], %[cy], %[ry] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[T], %[t], %[d]\n\t"
        "v_pk_mul_f32 %[t], %[cz], %[rz] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[T], %[T], %[t]\n\t"
        "v_pk_mul_f32 %[t], %[rx], %[T] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[qx], %[cx], %[t] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[t], %[ry], %[T] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[qy], %[cy], %[t] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[t], %[rz], %[T] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f32 %[qz], %[cz], %[t] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_mul_f32 %[d], %[qx], %[qx]\n\t"
        "v_pk_mul_f32 %[t], %[qy], %[qy]\n\t"
        "v_pk_add_f32 %[d], %[d], %[t]\n\t"
        "v_pk_mul_f32 %[t], %[qz], %[qz]\n\t"
        "v_pk_add_f32 %[d], %[d], %[t]"
        : [qx] "=&v"(qx), [qy] "=&v"(qy), [qz] "=&v"(qz), [t] "=&v"(t), [T] "=&v"(T), [d] "=&v"(d)
        : [cx] "s"(cx), [cy] "s"(cy), [cz] "s"(cz), [rx] "v"(r.x), [ry] "v"(r.y), [rz] "v"(r.z));
    return d;
}

// One sphere pair of a primary round (spheres L0, L0 + 1 of group g, camera-relative rows from
// TraceArgs.prim): test_group's two halves as separate pair tests.
template <bool SIMD, int L0>
__device__ __forceinline__ void test_half_prim(const TraceArgs &a, uint32_t g, const RayPk &p, Hit &h, f2 cx, f2 cy,
                                               f2 cz, float r2a, float r2b) {
    f2 T;
    const f2 d = pair_dist_c(p, cx, cy, cz, T);
    bool ha, hb;
    if (SIMD) {  // HitMask = d < r^2 (main.cpp:409)
        ha = d.x < r2a;
        hb = d.y < r2b;
    } else {  // !(d > r^2) over the Count real spheres only (main.cpp:547,557)
        const uint32_t s0 = 4u * g + (uint32_t)L0;
        ha = s0 < a.n_spheres && !(d.x > r2a);
        hb = s0 + 1u < a.n_spheres && !(d.y > r2b);
    }
    if (ha | hb) {
        if (ha) candidate<SIMD, L0>(h, g, T.x, d.x, r2a, a.fast_sqrt != 0u);
        if (hb) candidate<SIMD, L0 + 1>(h, g, T.y, d.y, r2b, a.fast_sqrt != 0u);
    }
}

// Pair pr of a primary round's pair mask (half pr & 1 of group pr >> 1); the mask's pairs come in
// ascending order, the reference's sphere order, so the per-class minima and tie rules are those of
// the full group loop.
template <bool SIMD>
__device__ __forceinline__ void test_pair_prim(const TraceArgs &a, cv4f_t *prim, uint32_t pr, const RayPk &p, Hit &h) {
    const uint32_t g = pr >> 1;
    cv4f_t *pg = prim + kPrimF4 * g;
    const v4f_t cx = pg[0], cy = pg[1], cz = pg[2], r2 = pg[3];
    if (pr & 1u) test_half_prim<SIMD, 2>(a, g, p, h, f2{cx.z, cx.w}, f2{cy.z, cy.w}, f2{cz.z, cz.w}, r2.z, r2.w);
    else test_half_prim<SIMD, 0>(a, g, p, h, f2{cx.x, cx.y}, f2{cy.x, cy.y}, f2{cz.x, cz.y}, r2.x, r2.y);
}

// Conservative per-wave culling for primary rays.  All primary rays of a
// tile start at CameraPosition and point into the tile's film rectangle
// (+-0.5 px jitter), i.e. inside a cone (axis A, half-angle theta).  A sphere
// can pass the exact test d < r^2 only if the LINE through the camera along
// some cone direction comes within r of its centre, i.e. if the angle between
// +-C and A is below theta + asin(r/|C|).  The cone and the test are computed
// in f64, so their own rounding is negligible; the margins cover the f32 path
// the kernel actually traces: each traced direction lies within ~1e-6 rad of
// the ideal cone (film point and Normalize rounding; |jitter| <= 0.5 + 1e-7 px,
// covered by the 0.501 px bound), and the reference-rounded distance is within
// 13.3u|C|^2 of the exact one -- the test uses a 1e-5 rad
// angular margin and r'^2 = r^2 (1 + 1e-5) + 1e-5 |C|^2, ten times both.  A
// group it rejects is one every lane's exact test misses: skipping it changes
// nothing.
struct Cone {
    double ax, ay, az;     // axis
    double cos_t, sin_t;   // inflated half-angle
};

__device__ __forceinline__ Cone tile_cone(const TraceArgs &a, double u0, double u1, double v0, double v1) {
    const double fcx = (double)a.film_center[0] - a.cam_pos[0];
    const double fcy = (double)a.film_center[1] - a.cam_pos[1];
    const double fcz = (double)a.film_center[2] - a.cam_pos[2];
    const double aa[2] = {(-1.0 + (u0 * 2.0) / a.width) * a.film_w * 0.5, (-1.0 + (u1 * 2.0) / a.width) * a.film_w * 0.5};
    const double bb[2] = {(-1.0 + (v0 * 2.0) / a.height) * a.film_h * 0.5,
                          (-1.0 + (v1 * 2.0) / a.height) * a.film_h * 0.5};
    double cx[4], cy[4], cz[4];
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int i = 0; i < 4; ++i) {
        const double ka = aa[i & 1], kb = bb[i >> 1];
        const double x = fcx + ka * a.cam_x[0] + kb * a.cam_y[0];
        const double y = fcy + ka * a.cam_x[1] + kb * a.cam_y[1];
        const double z = fcz + ka * a.cam_x[2] + kb * a.cam_y[2];
        const double inv = 1.0 / __builtin_sqrt(x * x + y * y + z * z);
        cx[i] = x * inv;
        cy[i] = y * inv;
        cz[i] = z * inv;
        sx += cx[i];
        sy += cy[i];
        sz += cz[i];
    }
    Cone c;
    const double inv = 1.0 / __builtin_sqrt(sx * sx + sy * sy + sz * sz);
    c.ax = sx * inv;
    c.ay = sy * inv;
    c.az = sz * inv;
    double ct = 1.0;
    for (int i = 0; i < 4; ++i) ct = fmin(ct, c.ax * cx[i] + c.ay * cy[i] + c.az * cz[i]);
    const double st = __builtin_sqrt(fmax(0.0, 1.0 - ct * ct));
    const double cd = 0.99999999995, sd = 1e-5;  // cos/sin of the 1e-5 rad margin
    c.cos_t = ct * cd - st * sd;
    c.sin_t = st * cd + ct * sd;
    return c;
}

__device__ __forceinline__ bool cone_may_hit(const TraceArgs &a, const Cone &c, float px, float py, float pz, float r2) {
    if (!(r2 >= 0.0f)) return false;  // padding lanes of the scalar packing (-inf)
    const double qx = (double)px - a.cam_pos[0], qy = (double)py - a.cam_pos[1], qz = (double)pz - a.cam_pos[2];
    const double c2 = qx * qx + qy * qy + qz * qz;
    const double rr = (double)r2 * (1.0 + 1e-5) + 1e-5 * c2;
    if (rr >= c2) return true;  // the camera is (nearly) inside: never cull
    const double sb = __builtin_sqrt(rr / c2), cb = __builtin_sqrt(1.0 - rr / c2);
    if (c.cos_t <= 0.0) return true;  // cone wider than 90 degrees: no culling
    const double cos_lim = c.cos_t * cb - c.sin_t * sb;  // cos(theta + beta)
    const double cos_phi = fabs(c.ax * qx + c.ay * qy + c.az * qz) / __builtin_sqrt(c2);
    return cos_phi >= cos_lim - 1e-12;
}

// Scheduling counters (RT_STATS=1) are compiled in only with -DRTK_STATS
// (the diagnostic build, `make variant NAME=stats KFLAGS=-DRTK_STATS`): the
// production kernel carries no per-trip checks for them.
#ifdef RTK_STATS
constexpr bool kStats = true;
#else
constexpr bool kStats = false;
#endif

constexpr int kWavesPerBlock = 4;
// primary pair mask words per wave tile (rtk_mask_words): the LDS-image kernels keep this
// small (it is static LDS, and C2's blocks fill the CU's 160 KB 7 times)
template <bool GS>
struct MaskWords {
    static constexpr int N = GS ? (int)((2u * kMaxGroups + 63u) / 64u) : (int)((2u * kMaxLdsGroups + 63u) / 64u);
};
constexpr uint32_t kFoldTable = 256;
// Per-pixel out-of-order sample slots (LDS ring): at least P (every sample
// lane holds one sample in flight) plus slack: 16 per pixel at P <= 4 (12 and
// 32 measured slower), 2 per sample lane above.  A multiple of 4, so a
// whole-batch fold never wraps.
template <int P>
struct Ring {
    static constexpr uint32_t N = P <= 4 ? 16u : 2u * (uint32_t)P;
};

#ifndef RTK_SOLO_WAVES_PER_SIMD  // the same target for the one-wave kernels (A/B: make variant KFLAGS=-DRTK_SOLO_WAVES_PER_SIMD=8)
#define RTK_SOLO_WAVES_PER_SIMD 7
#endif
#ifndef RTK_MIN_WAVES_PER_SIMD  // occupancy target (VGPR budget) of the production (SMEM) kernels;
#define RTK_MIN_WAVES_PER_SIMD 7   // 7 waves = 72 VGPRs, no VGPR spills: measured best on C2 with the
#endif                             // cluster walk (w6 116.5k, w7 120.0-121.1k, w8 118.2k Mrays/s, w8 spills)

// Work shape.  A wave owns a small pixel tile and P lanes per pixel: the
// lanes of a pixel take its samples in order as they free up (kDynamic in
// trace_kernel), park each finished sample's radiance in a per-pixel LDS
// ring, and the pixel's owner lane (j == 0) folds the ring into the running
// mean strictly in sample order (main.cpp:484-487), so results are
// bit-identical to one lane tracing the samples one after another.  P > 1
// splits the long per-pixel sample chains of pixels that see geometry over
// several lanes: the heaviest waves get P times shorter, which removes most
// of the kernel's tail.  Tiles: P=1 8x8, P=2 8x4, P=4 4x4 pixels per wave.
// P = 0 is the other direction, for launches of one frame (the reference's
// OnRender unit): one lane per pixel and kPixelsPerLane pixels per lane over a
// 16x16 wave tile (slot q of lane l: the 8x8 quadrant q, pixel l of it).  A
// lane whose path ends starts its next pixel's sample in the next primary
// round, so a wave stays full instead of draining after one pass, and a
// launch has a quarter of the waves (each of which pays the wave's setup once).
constexpr uint32_t kPixelsPerLane = 4;
template <int P>
struct Shape {
    static constexpr uint32_t LP = P == 0 ? 1u : (uint32_t)P;         // lanes per pixel
    static constexpr uint32_t Q = P == 0 ? kPixelsPerLane : 1u;       // pixels per lane
    static constexpr uint32_t TW = P == 0 ? 16u : P <= 2 ? 8u : P <= 8 ? 4u : 2u;
    static constexpr uint32_t TH = P == 0 ? 16u : P == 1 ? 8u : P <= 4 ? 4u : P <= 16 ? 2u : 1u;
    static_assert(TW * TH * LP == 64u * Q, "a wave is 64 lanes");
};

// GS: the scene (groups + materials) stays in HBM and per-lane gathers read it
// through the caches (scenes beyond the LDS image, or RT_SCENE_GLOBAL=1).
// SOLO: one wave per workgroup (block b traces quadrant b & 3 of block tile
// tile_order[b >> 2]).  A 4-wave workgroup's slots are held until its last wave
// ends, and a new workgroup needs four free slots at once: at C2 about a fifth
// of the wave slots sat idle mid-launch (scripts/wave_tail.py).  A one-wave
// workgroup is replaced as soon as it ends.  It keeps no LDS image (the scene
// and both tables are read through the caches, measured as fast at C2), only
// its ring and mask.
// WALK: the secondary-ray sphere walk compiled into the kernel (rt_kernel.h
// kWalk*): every variant selected at run time (kWalkAny), the per-group loops
// only (kWalkGroups), or one cluster walk (pair-mask words, per-lane or
// scene-wide thresholds).  One walk per kernel keeps the code and the SGPR
// pressure of the others out of the trace loop (C2 +4 % with only the W = 1
// walk compiled in).  The exact all-groups loop stays in every variant (rounds
// whose directions leave the prefilter's |D|^2 bound).
// Occupancy target of the one-wave kernels per secondary walk: the two-word
// scene-wide cluster walk (C5: 256 spheres) takes 8 waves/SIMD (63 VGPRs, the
// cull mask in dynamic LDS leaves room for 32 workgroups per CU): C5 +2.7 %
// same-box, while C2 (one word) and RTWeekend (four per-lane words) lose
// 1.5 % and 0.5 % at 8 and keep 7.
#ifndef RTK_SOLO_WAVES_CL2
#define RTK_SOLO_WAVES_CL2 8
#endif
constexpr int solo_waves(int walk) { return walk == kWalkCl2 ? RTK_SOLO_WAVES_CL2 : RTK_SOLO_WAVES_PER_SIMD; }

template <int WALK> struct Walk {
    // the per-group walk (small scenes) may merge primary and secondary rounds
    static constexpr bool MERGEABLE = WALK == kWalkAny || WALK == kWalkGroups;
    static constexpr int W = WALK == kWalkCl2 || WALK == kWalkCl2Rel ? 2 : WALK == kWalkCl4 || WALK == kWalkCl4Rel ? 4 : 1;
    static constexpr bool REL = WALK == kWalkCl1Rel || WALK == kWalkCl2Rel || WALK == kWalkCl4Rel;
    static constexpr bool CLUSTERS = WALK >= kWalkCl1;
};

// Tile of this block: heaviest-first order from the previous launch's
// measured costs when the host supplies one (tile_order), so the long
// waves do not start last and form the launch's tail.  One-wave kernels
// rank waves (unit 4 * tile + quadrant), four-wave ones block tiles.
template <bool SOLO, typename Args>
__device__ __forceinline__ void wave_unit(const Args &a, uint32_t tid, uint32_t &tile, uint32_t &wave) {
    if (SOLO && a.unit_waves != 0u) {
        const uint32_t u = a.tile_order ? a.tile_order[blockIdx.x] : blockIdx.x;
        tile = u >> 2;
        wave = u & 3u;
    } else {
        const uint32_t blk = SOLO ? blockIdx.x >> 2 : blockIdx.x;
        tile = a.tile_order ? a.tile_order[blk] : blk;
        wave = SOLO ? blockIdx.x & 3u : tid >> 6;
    }
}

template <bool SIMD, int SRC, bool CULL, int P, bool GS, bool SOLO = false, int WALK = kWalkAny>
__global__ __launch_bounds__(SOLO ? 64 : 256, SOLO ? solo_waves(WALK) : SRC == kSrcSmem ? RTK_MIN_WAVES_PER_SIMD : 1)
void trace_kernel(TraceArgs a) {
    static_assert(!GS || SRC == kSrcSmem, "a scene in HBM is read through the scalar cache");
    static_assert(!SOLO || GS, "a one-wave workgroup keeps no LDS image");
    constexpr uint32_t kWB = SOLO ? 1u : (uint32_t)kWavesPerBlock;  // waves (LDS slots) per workgroup
    constexpr uint32_t TW = Shape<P>::TW, TH = Shape<P>::TH, LP = Shape<P>::LP, Q = Shape<P>::Q;
    constexpr uint32_t NPIX = 64u / LP;  // pixels traced at a time
    constexpr bool kMergeable = Walk<WALK>::MERGEABLE;
    constexpr uint32_t kRing = Ring<LP>::N;
    extern __shared__ float4 smem[];
    // first launch of a key: the host has not read the live-tile count back, so
    // the grid covers every tile (live first) and blocks past the count leave
    if (a.live_total && (SOLO ? blockIdx.x >> 2 : blockIdx.x) >= (uint32_t)*a.live_total) return;
    const uint64_t st_entry = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;
    // LDS image: [rsqrt table 512 float4][fold table 128 float4]
    //            [groups kGroupF4*n_groups float4][sphere records kSphereF4*4*n_groups float4]
    // the wave tile's primary group mask: one-wave workgroups keep no LDS image,
    // so theirs is the dynamic LDS the host sizes to the scene's words (static
    // kMaxGroups / 64 words would cost 512 B of every workgroup's allocation)
    __shared__ uint64_t s_mask_st[SOLO ? 1 : kWB][SOLO ? 1 : MaskWords<GS>::N];
    uint64_t *const s_maskw = SOLO ? reinterpret_cast<uint64_t *>(smem) : s_mask_st[SOLO ? 0u : threadIdx.x >> 6];
    // ring slot s of pixel pl at s * kRingStride + pl: the sample lanes of a
    // pixel (different slots) fall on different LDS banks (stride NPIX + 1)
    constexpr uint32_t kRingStride = NPIX + 1u;
    __shared__ float4 s_ring[LP > 1 ? kWB * kRing * kRingStride : 1];
    // (one-wave kernels keep no LDS image: both tables are theirs from HBM at compile time, so the
    // rsqrt gather is a global load with a scalar base, not a flat one through a selected pointer)
    const bool lut_lds = !SOLO && a.lut_in_lds != 0u;
    const uint32_t lut_f4 = lut_lds ? 512u : 0u;  // see rtk_lds_bytes
    const Lut lut = {reinterpret_cast<const float *>(smem), a.rsqrt_lut, lut_lds};
    float2 *fold = reinterpret_cast<float2 *>(smem + lut_f4);
    // running-mean weights of the first kFoldTable frames (large scenes: none, computed per sample)
    const uint32_t fold_n = !SOLO && a.fold_in_lds ? kFoldTable : 0u;
    float4 *lds_groups = smem + lut_f4 + fold_n / 2;
    float4 *lds_mats = lds_groups + kGroupF4 * a.n_groups;
    // per-lane gathers of the winner's centre and material: LDS image or HBM (GS)
    const float4 *mat_src = GS ? a.materials : lds_mats;
    {
        const float4 *glut = reinterpret_cast<const float4 *>(a.rsqrt_lut);
        for (uint32_t i = threadIdx.x; i < lut_f4; i += blockDim.x) smem[i] = glut[i];
        if (!GS) {
            for (uint32_t i = threadIdx.x; i < kGroupF4 * a.n_groups; i += blockDim.x) lds_groups[i] = a.groups[i];
            for (uint32_t i = threadIdx.x; i < 4u * kSphereF4 * a.n_groups; i += blockDim.x) lds_mats[i] = a.materials[i];
        }
        // running-mean weights of frame k (main.cpp:484-487): 1/(p+1), p/(p+1)
        for (uint32_t i = threadIdx.x; i < fold_n; i += blockDim.x) {
            const uint32_t pc = a.prev_count + i;
            fold[i] = make_float2(1.0f / (float)(pc + 1u), (float)pc / (float)(pc + 1u));
        }
    }

    // wave: quadrant of the block tile; sw: the wave's LDS slot in its workgroup
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t sw = SOLO ? 0u : tid >> 6;
    uint32_t tile, wave;
    wave_unit<SOLO>(a, tid, tile, wave);
    const uint32_t tile_x = tile % a.tiles_x, tile_y = tile / a.tiles_x;
    // The wave's start times go to memory and LDS, and the end of the kernel re-derives its tile
    // (wave_unit through the kernarg segment): nothing of the bookkeeping is held in SGPRs across the
    // trip loop, where the four-word walk spilled it around every secondary round.
    __shared__ uint64_t s_cost0[SOLO ? 1 : kWB];
    if (a.wave_times && lane == 0) a.wave_times[2u * ((uint64_t)tile * 4u + wave)] = __builtin_amdgcn_s_memrealtime();
    if (a.tile_cost && lane == 0) s_cost0[sw] = __builtin_amdgcn_s_memtime();
    const uint64_t t_cost0 = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t pl = lane / LP, j = lane % LP;  // pixel of the tile, sample lane of the pixel
    // wave tile: a TW x TH quadrant of the block tile, or (interleave) every
    // other pixel and row of the whole block tile, parity (wave & 1, wave >> 1);
    // Q > 1: pixel slot q of the lane is pixel pl of the tile's 8x8 quadrant q
    auto pixel_x = [&](uint32_t q) -> uint32_t {
        if (Q > 1) return tile_x * (2u * TW) + (wave & 1u) * TW + (pl & 7u) + 8u * (q & 1u);
        return a.interleave ? tile_x * (2u * TW) + 2u * (pl % TW) + (wave & 1u)
                            : tile_x * (2u * TW) + (wave & 1u) * TW + pl % TW;
    };
    auto pixel_ly = [&](uint32_t q) -> uint32_t {
        if (Q > 1) return tile_y * (2u * TH) + (wave >> 1) * TH + (pl >> 3) + 8u * (q >> 1);
        return a.interleave ? tile_y * (2u * TH) + 2u * (pl / TW) + (wave >> 1)
                            : tile_y * (2u * TH) + (wave >> 1) * TH + pl / TW;
    };
    uint32_t q_slot = 0;  // Q > 1: the lane's current pixel slot
    uint32_t x = pixel_x(0), ly = pixel_ly(0);
    bool valid = x < a.width && ly < a.local_rows;
    // (slot 0 outside the image puts every slot of the lane outside it: the
    // slots lie right of and below slot 0)
    auto global_y = [&](uint32_t l) -> uint32_t {
        return ((l / a.band_rows) * a.band_count + a.band_index) * a.band_rows + l % a.band_rows;
    };
    uint32_t y = global_y(ly);
    // pixels dealt to the block's waves by cost (rtk_launch_pixel_sort): wave-uniform
    const uint8_t *perm = Q == 1 && a.pix_perm && !a.interleave ? a.pix_perm + (size_t)tile * 64u : nullptr;
    const bool permuted = perm && perm[0] != 0xFFu;
    if (permuted) {
        const uint32_t li = perm[wave * NPIX + pl];
        x = tile_x * (2u * TW) + li % (2u * TW);
        ly = tile_y * (2u * TH) + li / (2u * TW);
        valid = x < a.width && ly < a.local_rows;
        y = global_y(ly);
    }
    const bool owner = j == 0;
    // The running mean of a pixel is one sequential chain per colour channel, so
    // with P >= 4 its lanes j = 0, 1, 2 each fold ONE channel (kept in accx) in
    // lockstep: a fold step then costs one multiply and one add per lane, and a
    // wave folds 3 chains per pixel at once (at P = 16 the owner's three-channel
    // fold was ~15 % of the wave's VALU instructions).  The owner gathers the
    // other two channels by DPP for the final store.
    constexpr bool FOLD3 = LP >= 4;
    const bool folder = FOLD3 ? j < 3u : owner;
    // the channel a lane reads from a ring slot (lanes j >= 3 of the whole-batch fold
    // read the ratio word and discard their sums)
    const uint32_t jc = j < 3u ? j : 3u;
    // every lane of a pixel keeps the fold cursor (whole-batch frontier fold)
    constexpr bool kCursorPerLane = LP > 1;
    float4 *ring = s_ring + sw * kRing * kRingStride + pl;

    const uint32_t n_words = rtk_mask_words(a.n_groups);
    // the wave tile's primary pair mask, from the cull pass (rtk_launch_cull)
    // (a permuted wave's pixels come from all four quadrants: the union of their masks)
    if (CULL)
        for (uint32_t wd = lane; wd < n_words; wd += 64u) {
            uint64_t m = a.masks[((size_t)tile * 4u + wave) * n_words + wd];
            if (permuted)
                for (uint32_t q = 0; q < 4u; ++q) m |= a.masks[((size_t)tile * 4u + q) * n_words + wd];
            s_maskw[wd] = m;
        }
    const uint64_t st_c1 = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;
    __syncthreads();
    const uint64_t st_c2 = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;

    float accx = 0.0f, accy = 0.0f, accz = 0.0f;  // FOLD3: accx = this folding lane's channel j
    // the running mean so far of the lane's current pixel (main.cpp:485)
    auto load_mean = [&]() {
        accx = accy = accz = 0.0f;
        if (valid && folder && a.prev_count > 0 && !(a.flags & kFlagAccumZero)) {
            const float4 pv = a.prev[(size_t)ly * a.width + x];
            if (FOLD3) {
                accx = j == 0u ? pv.x : j == 1u ? pv.y : pv.z;
            } else {
                accx = pv.x;
                accy = pv.y;
                accz = pv.z;
            }
        }
    };
    load_mean();
    // the blended mean and its RGBA8 (main.cpp:488-492) of the current pixel
    // (Q > 1 stores inside the trace loop, where the f64 pow of RT_FLAG_SRGB_POW
    // would cost registers: the host launches that flag with Q = 1 only)
    auto store_pixel = [&]() {
        const size_t pix = (size_t)ly * a.width + x;
        a.prev[pix] = make_float4(accx, accy, accz, 1.0f);
        if (!a.skip_cur) a.cur[pix] = rgba8(accx, accy, accz, Q == 1 && (a.flags & kFlagSrgbPow) != 0u);
    };

    // owner lanes of in-image pixels (they fold until every frame is folded)
    const uint64_t folding = ballot_and(owner, valid);
    // lane mode: 0 = next sample pending, 1 = path continues (secondary), 2 = no samples left
    // The P lanes of a pixel take its samples in order as they free up (kDynamic):
    // each trip the lanes wanting a sample are ranked inside the slice and take
    // next, next + 1, ...  A lane whose samples run short no longer idles while its
    // neighbours trace theirs: only the pixel's last few samples leave lanes idle.
    constexpr bool kDynamic = LP > 1;
    uint32_t k = j;            // this lane's next (or current) sample
    uint32_t next = 0;         // kDynamic: the pixel's first unassigned sample (same on its lanes)
    uint32_t folded = 0;       // owner: samples folded so far
    uint32_t mode = (valid && k < a.frames) ? 0u : 2u;
    const uint32_t slice_base = lane - j;

    uint64_t nrays = 0;  // wave total (uniform): segments traced by this wave
    uint32_t pseg = 0;   // segments this lane traced (pix_cost)
    uint32_t st_pri_it = 0, st_pri_lanes = 0, st_sec_it = 0, st_sec_lanes = 0, st_groups = 0, st_sec_hit = 0;
    uint32_t st_sparse_it = 0, st_sparse_lanes = 0, st_tail_it = 0;
    uint32_t st_pri_blocked = 0, st_pri_waitsec = 0, st_pri_done = 0;
    uint32_t st_sec_done = 0, st_sec_waitpri = 0, st_done_trips = 0, st_done_lanes = 0;
    uint32_t st_sec_exact = 0, st_sec_badlanes = 0, st_sec_zerodir = 0;
    uint64_t st_cyc_pri = 0, st_cyc_sec = 0, st_cyc_fold = 0, st_cyc_setup = 0;
    uint64_t st_cyc_cull = 0, st_cyc_sync = 0, st_cyc_post = 0;
    PfStats st_pf = {0, 0, 0, 0, 0};
    uint32_t st_pf_rounds = 0;
    Sample p;
    p.bounce = 0;
    p.cx = p.cy = p.cz = 0.0f;

    // Empty tile: no sphere group passes the tile's (conservative) cone test,
    // so every primary ray of every sample misses; without a sky term each
    // sample's Out is exactly 0 (main.cpp:433-440), its one segment still
    // counts (main.cpp:390), and its blend is Final = 0*(1/n) + Prev*((n-1)/n)
    // = RN(Prev*((n-1)/n)) -- folded here without generating the rays.
    bool empty_tile = CULL && !a.use_sky && a.max_bounce != 0;
    if (CULL)
        for (uint32_t w = 0; w < n_words; ++w) empty_tile = empty_tile && s_maskw[w] == 0;
    // (an all-zero running mean stays exactly zero: nothing to fold)
    auto fold_zero_frames = [&]() {
        if (valid && folder && (accx != 0.0f || accy != 0.0f || accz != 0.0f)) {
            for (uint32_t q = 0; q < a.frames; ++q) {
                float ratio;
                if (q < fold_n) {
                    ratio = fold[q].y;
                } else {
                    ratio = fold_weights(a.prev_count + q).y;
                }
                accx = 0.0f + accx * ratio;
                accy = 0.0f + accy * ratio;
                accz = 0.0f + accz * ratio;
            }
        }
    };
    if (empty_tile) {
        if (Q > 1) {  // every pixel slot of the lane, each stored here
            for (uint32_t q = 0; q < Q; ++q) {
                if (q > 0) {
                    x = pixel_x(q);
                    ly = pixel_ly(q);
                    valid = x < a.width && ly < a.local_rows;
                    load_mean();
                }
                fold_zero_frames();
                nrays += (uint64_t)__builtin_popcountll(__ballot(valid)) * a.frames;
                if (valid) store_pixel();
            }
            valid = false;  // (nothing left for the final store)
        } else {
            fold_zero_frames();
            nrays = (uint64_t)__builtin_popcountll(__ballot(valid && owner)) * a.frames;
        }
        folded = a.frames;
        mode = 2u;
    }

    if (kStats && a.stats) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        st_cyc_setup = t_cost0 - st_entry;  // LDS image loads issued, tile picked
        st_cyc_cull = st_c1 - t_cost0;
        st_cyc_sync = st_c2 - st_c1;
        st_cyc_post = t - st_c2;
    }
    // Re-derive the winner's HitNormal / NextRayOrigin exactly as they were
    // formed at acceptance (main.cpp:423-429), then shade and bounce.
    auto shade_hit = [&](float tmin, uint32_t sidx, bool inside) {
        // the winner's record (rt_kernel.h kSphereF4): one shift of the sphere index addresses its
        // centre and both material rows
        const float4 *rec = mat_src + kSphereF4 * sidx;
        const float4 sc = rec[0];
        const float sx = sc.x, sy = sc.y, sz = sc.z;
        const float cx = sx - p.rx.x, cy = sy - p.ry.x, cz = sz - p.rz.x;
        const float ipx = p.rx.y * tmin, ipy = p.ry.y * tmin, ipz = p.rz.y * tmin;
        const float hx = ipx - cx, hy = ipy - cy, hz = ipz - cz;
        p.rx.x = p.rx.x + ipx;
        p.ry.x = p.ry.x + ipy;
        p.rz.x = p.rz.x + ipz;
        const float4 cs = rec[1];
        const float4 ei = rec[2];
        shade(lut, cs, ei, rec + 3, hx, hy, hz, inside, p);
        p.bounce += 1;
    };
    // the pixel's owner lane's fold cursor (first of its P-lane slice) via DPP
    auto fold_cursor = [&]() -> uint32_t {
        return kCursorPerLane ? folded
               : LP == 4 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)folded, 0x00, 0xf, 0xf, false)    // quad_perm 0,0,0,0
               : LP == 2 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)folded, 0xA0, 0xf, 0xf, false)  // quad_perm 0,0,2,2
               : LP > 4 ? (uint32_t)__shfl((int)folded, (int)(lane - j), 64)
                        : folded;
    };
    // The pixel's parked frontier: every sample below it is in the ring.  A lane's
    // samples below its cursor k are parked (mode 0: k not started yet; 1: k in
    // flight; 2: k >= frames), so it is the minimum of k over the pixel's P lanes
    // -- a DPP reduction inside the lane slice (quads, half rows, rows; a
    // cross-row shuffle only for P = 32), run with every lane active.
    auto parked_frontier = [&]() -> uint32_t {
        // (kDynamic: samples below next are all assigned; those not in flight are parked)
        uint32_t f = kDynamic && mode != 1u ? next : k;
#define RTK_DMIN(CTRL) f = min(f, (uint32_t)__builtin_amdgcn_update_dpp((int)f, (int)f, CTRL, 0xf, 0xf, false))
        if (LP >= 2) RTK_DMIN(0xB1);   // quad_perm 1,0,3,2 (lane ^ 1)
        if (LP >= 4) RTK_DMIN(0x4E);   // quad_perm 2,3,0,1 (lane ^ 2)
        if (LP >= 8) RTK_DMIN(0x141);  // row_half_mirror (the other quad of the 8)
        if (LP >= 16) RTK_DMIN(0x140); // row_mirror (the other half of the row)
#undef RTK_DMIN
        if (LP >= 32) f = min(f, (uint32_t)__shfl_xor((int)f, 16, 64));
        return min(f, a.frames);
    };
    auto fold_ring = [&]() {
        if (LP == 1) return;
        // ---- running-mean blend (main.cpp:484-489) of every parked sample, in
        // order: Final = Out*(1/n) + Prev*((n-1)/n), the first product done by the
        // sample's lane.  Slots [folded, F) are all parked: no per-slot flags, no
        // clearing writes.  Whole batches of four slots aligned to 4 (kRing is a
        // multiple of 4, so a batch never wraps; its LDS reads take immediate
        // offsets), each slot folded straight with no per-slot test; the ragged end
        // once every sample is parked.  A lane that waits for ring space still gets
        // it: the lane holding the frontier sample F < folded + 4 <= folded + kRing
        // is never blocked, so the frontier keeps moving.  Every lane of the pixel
        // runs the loop (F is uniform over them), so each keeps the fold cursor
        // itself; only the folding lanes' sums are used.
        const uint32_t F = parked_frontier();  // (every lane active: a DPP reduction)
        if (!valid) return;
        const uint32_t Fb = F >= a.frames ? F : (F & ~3u);
        while (folded + 4u <= Fb) {
            const float4 *base = ring + (folded % kRing) * kRingStride;
            float v[4], w[4];
            float4 r4[4];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
                if (FOLD3) {
                    const float *slot = reinterpret_cast<const float *>(base + i * kRingStride);
                    v[i] = slot[jc];
                    w[i] = slot[3];
                } else {
                    r4[i] = base[i * kRingStride];
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
                if (FOLD3) {
                    accx = v[i] + accx * -w[i];
                } else {
                    accx = r4[i].x + accx * -r4[i].w;
                    accy = r4[i].y + accy * -r4[i].w;
                    accz = r4[i].z + accz * -r4[i].w;
                }
            }
            folded += 4u;
        }
        while (folded < Fb) {
            const float4 *s4 = ring + (folded % kRing) * kRingStride;
            if (FOLD3) {
                const float *slot = reinterpret_cast<const float *>(s4);
                accx = slot[jc] + accx * -slot[3];
            } else {
                const float4 r = *s4;
                accx = r.x + accx * -r.w;
                accy = r.y + accy * -r.w;
                accz = r.z + accz * -r.w;
            }
            folded += 1u;
        }
    };
    for (;;) {
        // ring space: sample k may start once k < folded + kRing (the oldest
        // unfolded sample's lane is never blocked, so this cannot deadlock)
        // the pixel's owner lane (first of its P-lane quad slice) via DPP
        uint32_t folded_g = fold_cursor();
        uint32_t want_n = 0;  // kDynamic: the slice's lanes wanting a sample
        if (kDynamic) {
            const uint32_t sw_bits = (uint32_t)((__builtin_amdgcn_ballot_w64(mode == 0u) >> slice_base) & ((1ull << LP) - 1ull));
            want_n = __builtin_popcount(sw_bits);
            if (mode == 0u) {
                k = next + __builtin_popcount(sw_bits & ((1u << j) - 1u));
                if (k >= a.frames) mode = 2u;
            }
        }
        // (lane masks from single compares: see ballot_and)
        bool ring_ok = LP == 1 || k < folded_g + kRing;
        bool can_start = mode == 0u && ring_ok;
        uint64_t pri = LP == 1 ? __builtin_amdgcn_ballot_w64(mode == 0u) : ballot_and(mode == 0u, ring_ok);
        const uint64_t sec = __builtin_amdgcn_ballot_w64(mode == 1u);
        // (one lane per pixel folds each sample as it ends: nothing left to fold then)
        const uint64_t alive = __builtin_amdgcn_ballot_w64(mode != 2u) |
                               (LP > 1 ? folding & __builtin_amdgcn_ballot_w64(folded < a.frames) : 0ull);
        if (alive == 0) break;
        const uint64_t st_t0 = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;
        // Secondary segments run the full sphere loop; let them gather until
        // enough lanes share one (or no primary work is ready).  Merged rounds
        // (scenes of one or two groups, TraceArgs.merge_rounds): every round
        // starts new samples AND continues paths, all through the exact loop.
        const bool merged = kMergeable && a.merge_rounds != 0u;
        const bool do_sec = !merged && sec != 0 && (pri == 0 || __builtin_popcountll(sec) >= a.sec_threshold);
        // (lazy: only when some lane waits for ring space, or nothing else is left)
        const bool fold_now = !do_sec && ((pri | sec) == 0 || (__builtin_amdgcn_ballot_w64(mode == 0u) & ~pri) != 0);
        if (fold_now) {
            // the owners fold only before a primary round (or when nothing is left to
            // trace): a secondary round starts no sample, so it needs no ring space
            const uint64_t st_f0 = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;
            fold_ring();
            if (kStats && a.stats) st_cyc_fold += __builtin_amdgcn_s_memtime() - st_f0;
            folded_g = fold_cursor();
            ring_ok = LP == 1 || k < folded_g + kRing;
            can_start = mode == 0u && ring_ok;
            pri = LP == 1 ? __builtin_amdgcn_ballot_w64(mode == 0u) : ballot_and(mode == 0u, ring_ok);
        }
        if (merged) pri |= sec;  // (the lanes a merged round traces)
        if ((pri | sec) != 0) {
            if (kStats && a.stats) {
                if (do_sec) { st_sec_it += 1; st_sec_lanes += __builtin_popcountll(sec); }
                if (do_sec && __builtin_popcountll(sec) < 16) { st_sparse_it += 1; st_sparse_lanes += __builtin_popcountll(sec); }
                if (do_sec && __ballot(mode == 0u) == 0) st_tail_it += 1;  // no lane has a sample to start
                if (do_sec) {  // a secondary round: where the other lanes are
                    st_sec_done += __builtin_popcountll(__ballot(mode == 2u));
                    st_sec_waitpri += __builtin_popcountll(__ballot(mode == 0u));
                }
                // trips with finished pixels (every sample started and traced) beside live ones
                const uint32_t nd = __builtin_popcountll(__ballot(mode == 2u));
                if (nd) { st_done_trips += 1; st_done_lanes += nd; }
                if (!do_sec) {  // a primary round: where the other lanes are
                    st_pri_it += 1;
                    st_pri_lanes += __builtin_popcountll(pri);
                    st_pri_blocked += __builtin_popcountll(__ballot(mode == 0u && !can_start));
                    st_pri_waitsec += __builtin_popcountll(sec);
                    st_pri_done += __builtin_popcountll(__ballot(mode == 2u));
                }
            }
            // do_sec ? mode == 1 : can_start, as one compare against a uniform mode
            // and a uniform override of the ring test (no lane-mask select)
            const bool traces = merged ? (mode == 0u && ring_ok) || mode == 1u
                                       : mode == (do_sec ? 1u : 0u) && (do_sec || ring_ok);
            if (a.max_bounce != 0) nrays += __builtin_popcountll(do_sec ? sec : pri);
            // the slice's lanes that start now are its lowest-ranked wanting ones
            if (kDynamic && !do_sec) next = min(next + want_n, min(a.frames, folded_g + kRing));
            if (traces) {
                pseg += 1u;
                if (!do_sec && mode == 0u) start_sample(kernel_args(), x, y, a.prev_count + k, p);
                bool done;
                if (a.max_bounce == 0) {
                    done = true;  // no segment is traced; the frame folds black
                } else {
                    Hit h;
                    hit_reset(h);
                    const RayPk ray = {p.rx, p.ry, p.rz};
                    if (CULL && !do_sec && !merged) {
                        // (the table's address is loaded here from the kernarg segment, as
                        // the camera fields are: held in an SGPR pair across the trip loop it
                        // cost the RTWeekend kernel SGPR spills, v_readlane in the loop)
                        cv4f_t *prim = (cv4f_t *)kernel_args().prim;
                        for (uint32_t w = 0; w < n_words; ++w) {
                            // (readfirstlane returns int: widen each half as u32, or
                            // bit 31 would sign-extend into groups 32..63)
                            const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)s_maskw[w]);
                            const uint32_t hi =
                                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(s_maskw[w] >> 32));
                            uint64_t m = (uint64_t)lo | ((uint64_t)hi << 32);
                            if (kStats && a.stats) st_groups += __builtin_popcountll(m);
                            while (m) {  // the tile's sphere pairs, in the reference's order
                                const uint32_t pr = w * 64u + (uint32_t)__builtin_ctzll(m);
                                m &= m - 1;
                                test_pair_prim<SIMD>(a, prim, pr, ray, h);
                            }
                        }
                    } else {
                        // Secondary rays: the prefiltered loop, whose error bound
                        // needs |D|^2 within 2^-16 of 1 on every lane (else exact).
                        const float u2 = __builtin_fmaf(p.rx.y, p.rx.y, __builtin_fmaf(p.ry.y, p.ry.y, p.rz.y * p.rz.y));
                        // (a cluster-walk kernel runs only with the prefilter and a cluster table: rt_host.cpp)
                        const bool pf = do_sec && (Walk<WALK>::CLUSTERS || a.prefilter) &&
                                        !__ballot(!(__builtin_fabsf(1.0f - u2) <= kPfDirTol));
                        if (kStats && a.stats && do_sec && !pf) {
                            st_sec_exact += 1;
                            st_sec_badlanes += __builtin_popcountll(__ballot(!(__builtin_fabsf(1.0f - u2) <= kPfDirTol)));
                            st_sec_zerodir += __builtin_popcountll(__ballot(u2 == 0.0f));
                        }
                        if (SRC == kSrcSmem && pf && (Walk<WALK>::CLUSTERS || a.n_cpairs)) {
                            if (kStats && a.stats) st_pf_rounds += 1;
                            PfStats *ps = kStats && a.stats ? &st_pf : nullptr;
                            if constexpr (Walk<WALK>::CLUSTERS) {
                                clustered_groups<SIMD, Walk<WALK>::W, GS, Walk<WALK>::REL>(a, lds_groups, ray, h, ps);
                            } else if constexpr (WALK == kWalkGroups) {
                                __builtin_unreachable();  // the host runs kWalkGroups kernels without a cluster table
                            } else if (a.pf_relative) {
                                if (a.cl_words == 1u) clustered_groups<SIMD, 1, GS, true>(a, lds_groups, ray, h, ps);
                                else if (a.cl_words == 2u) clustered_groups<SIMD, 2, GS, true>(a, lds_groups, ray, h, ps);
                                else clustered_groups<SIMD, 4, GS, true>(a, lds_groups, ray, h, ps);
                            } else {
                                if (a.cl_words == 1u) clustered_groups<SIMD, 1, GS, false>(a, lds_groups, ray, h, ps);
                                else if (a.cl_words == 2u) clustered_groups<SIMD, 2, GS, false>(a, lds_groups, ray, h, ps);
                                else clustered_groups<SIMD, 4, GS, false>(a, lds_groups, ray, h, ps);
                            }
                        } else if (SRC == kSrcSmem && pf && a.pf_relative && !Walk<WALK>::CLUSTERS) {
                            if (kStats && a.stats) st_pf_rounds += 1;
                            all_groups_smem<SIMD, true, GS, true>(a, lds_groups, ray, h, nullptr,
                                                                  kStats && a.stats ? &st_pf : nullptr);
                        } else if (SRC == kSrcSmem && pf && !Walk<WALK>::CLUSTERS) {
                            if (kStats && a.stats) st_pf_rounds += 1;
                            all_groups_smem<SIMD, true, GS>(a, lds_groups, ray, h, nullptr,
                                                        kStats && a.stats ? &st_pf : nullptr);
                        } else if (SRC == kSrcSmem) {
                            all_groups_smem<SIMD, false, GS>(a, lds_groups, ray, h,
                                                             kStats && a.stats ? &st_sec_hit : nullptr);
                        } else {
                            // software-pipelined: group g+1's load is in flight while
                            // g is tested (the array carries padding groups)
                            Group next = load_group<SRC>(a, lds_groups, 0);
                            for (uint32_t g = 0; g < a.n_groups; ++g) {
                                const Group G = next;
                                next = load_group<SRC>(a, lds_groups, g + 1u);
                                test_group<SIMD>(a, G, g, ray, h, kStats && a.stats ? &st_sec_hit : nullptr);
                            }
                        }
                    }
                    // ---- hit select (x64_math.h:579-585 HorizontalMin + first equal lane)
                    float tmin;
                    uint32_t sidx;
                    bool inside;
                    if (SIMD) {
                        const float m02 = h.t0 < h.t2 ? h.t0 : h.t2;
                        const float m13 = h.t1 < h.t3 ? h.t1 : h.t3;
                        tmin = m02 < m13 ? m02 : m13;
                        const uint32_t l = h.t0 == tmin ? 0u : h.t1 == tmin ? 1u : h.t2 == tmin ? 2u : 3u;
                        const uint32_t gsel = l == 0 ? h.g0 : l == 1 ? h.g1 : l == 2 ? h.g2 : h.g3;
                        sidx = gsel * 4u + l;
                        inside = (h.ins >> l) & 1u;
                    } else {
                        tmin = h.t0;
                        sidx = h.g0;
                        inside = h.ins != 0;
                    }
                    if (tmin == kFMax) {
                        if (a.use_sky) {  // main.cpp:434-438
                            const float s = (p.ry.y + 1.0f) * 0.5f;
                            const float w = (1.0f - s) * 1.0f;
                            p.cx = p.cx + (w + s * 0.5f) * p.ax;
                            p.cy = p.cy + (w + s * 0.7f) * p.ay;
                            p.cz = p.cz + (w + s * 1.0f) * p.az;
                        }
                        done = true;
                    } else {
                        shade_hit(tmin, sidx, inside);
                        done = p.bounce == a.max_bounce;
                    }
                }
                if (done) {
                    const float ox = a.max_bounce == 0 ? 0.0f : p.cx;
                    const float oy = a.max_bounce == 0 ? 0.0f : p.cy;
                    const float oz = a.max_bounce == 0 ? 0.0f : p.cz;
                    if (LP == 1) {
                        // ---- running-mean blend (main.cpp:484-489), in order by construction
                        const uint32_t pc = a.prev_count + k;
                        const float2 fw = SOLO ? (pc < kWeightsN ? a.weights[pc] : fold_weights(pc))
                                               : k < fold_n ? fold[k] : fold_weights(pc);
                        const float inv = fw.x, ratio = fw.y;
                        accx = ox * inv + accx * ratio;
                        accy = oy * inv + accy * ratio;
                        accz = oz * inv + accz * ratio;
                        folded = k + 1u;
                    } else {
                        // park Out*(1/n) and the ratio (n-1)/n of sample k's blend; the
                        // sign bit of .w marks the slot ready (the ratio is >= 0)
                        float2 w;
                        if (SOLO) {  // the static table of the first kWeightsN frames (TraceArgs.weights)
                            const uint32_t pc = a.prev_count + k;
                            w = pc < kWeightsN ? a.weights[pc] : fold_weights(pc);
                        } else {
                            w = fold[k < fold_n ? k : 0u];  // (fold_n = 0: an unused in-bounds read)
                            if (__builtin_expect(k >= fold_n, 0)) w = fold_weights(a.prev_count + k);
                        }
                        ring[(k % kRing) * kRingStride] = make_float4(ox * w.x, oy * w.x, oz * w.x, -w.y);
                    }
                    k += kDynamic ? 0u : LP;
                    mode = kDynamic || k < a.frames ? 0u : 2u;
                    if (Q > 1 && mode == 2u) {
                        // the pixel is complete: store it and move to the lane's next pixel
                        // slot inside the image (its samples start from k = 0)
                        store_pixel();
                        while (mode == 2u && q_slot + 1u < Q) {
                            q_slot += 1u;
                            x = pixel_x(q_slot);
                            ly = pixel_ly(q_slot);
                            if (x < a.width && ly < a.local_rows) {
                                y = global_y(ly);
                                k = 0;
                                folded = 0;
                                load_mean();
                                mode = 0u;
                            }
                        }
                    }
                } else {
                    mode = 1u;
                }
            }
        }
        const uint64_t st_t1 = kStats && a.stats ? __builtin_amdgcn_s_memtime() : 0;
        if (kStats && a.stats && (pri | sec) != 0) {
            const bool was_sec = sec != 0 && (pri == 0 || __builtin_popcountll(sec) >= a.sec_threshold);
            (was_sec ? st_cyc_sec : st_cyc_pri) += st_t1 - st_t0;
        }
    }

    if (FOLD3) {  // channels 1 and 2 from lanes j = 1, 2 of the pixel's quad (quad_perm 1,1,1,1 / 2,2,2,2)
        accy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(accx), 0x55, 0xf, 0xf, false));
        accz = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(accx), 0xAA, 0xf, 0xf, false));
    }
    if (Q == 1 && valid && owner && a.frames > 0) store_pixel();  // (Q > 1: stored as each pixel completes)

    cargs_t &ka = kernel_args();  // (the end's fields from the kernarg segment: see wave_unit above)
    if (ka.pix_cost) {  // the pixel's traced segments over its P lanes (every lane active here)
        for (uint32_t off = 1; off < LP; off <<= 1) pseg += (uint32_t)__shfl_xor((int)pseg, (int)off, 64);
        if (Q == 1 && valid && owner) ka.pix_cost[(size_t)ly * ka.width + x] = pseg;
    }
    // ---- ray counter (RaysCastInThread, main.cpp:390): one atomic per wave
    if (lane == 0 && nrays) atomicAdd(ka.rays, (unsigned long long)nrays);
    if ((ka.tile_cost || ka.wave_times) && lane == 0) {
        uint32_t tile_e, wave_e;
        wave_unit<SOLO>(ka, tid, tile_e, wave_e);
        if (ka.tile_cost) {
            const uint64_t c = __builtin_amdgcn_s_memtime() - s_cost0[sw];
            const uint32_t c32 = (uint32_t)(c < 0xFFFFFFFFull ? c : 0xFFFFFFFFull);
            if (SOLO && ka.unit_waves != 0u)
                ka.tile_cost[4u * tile_e + wave_e] = c32 | 1u;  // (>= 1: a launched wave never ranks with dead ones)
            else
                atomicMax(ka.tile_cost + tile_e, c32);
        }
        if (ka.wave_times) ka.wave_times[2u * ((uint64_t)tile_e * 4u + wave_e) + 1u] = __builtin_amdgcn_s_memrealtime();
    }
    if (kStats && a.stats && lane == 0) {
        atomicAdd(a.stats + kStatPriIters, (unsigned long long)st_pri_it);
        atomicAdd(a.stats + kStatPriLanes, (unsigned long long)st_pri_lanes);
        atomicAdd(a.stats + kStatSecIters, (unsigned long long)st_sec_it);
        atomicAdd(a.stats + kStatSecLanes, (unsigned long long)st_sec_lanes);
        atomicAdd(a.stats + kStatPriGroups, (unsigned long long)st_groups);
        atomicAdd(a.stats + kStatSecHitGroups, (unsigned long long)st_sec_hit);
        atomicAdd(a.stats + kStatSecSparseIters, (unsigned long long)st_sparse_it);
        atomicAdd(a.stats + kStatSecSparseLanes, (unsigned long long)st_sparse_lanes);
        atomicAdd(a.stats + kStatSecTailIters, (unsigned long long)st_tail_it);
        atomicAdd(a.stats + kStatPriCycles, (unsigned long long)st_cyc_pri);
        atomicAdd(a.stats + kStatSecCycles, (unsigned long long)st_cyc_sec);
        atomicAdd(a.stats + kStatFoldCycles, (unsigned long long)st_cyc_fold);
        atomicAdd(a.stats + kStatSetupCycles, (unsigned long long)st_cyc_setup);
        atomicAdd(a.stats + kStatCullCycles, (unsigned long long)st_cyc_cull);
        atomicAdd(a.stats + kStatSyncCycles, (unsigned long long)st_cyc_sync);
        atomicAdd(a.stats + kStatPostCycles, (unsigned long long)st_cyc_post);
        atomicAdd(a.stats + kStatPfRounds, (unsigned long long)st_pf_rounds);
        atomicAdd(a.stats + kStatPfGroups, (unsigned long long)st_pf.groups);
        atomicAdd(a.stats + kStatClTested, (unsigned long long)st_pf.cl_tested);
        atomicAdd(a.stats + kStatPfPairs, (unsigned long long)st_pf.pairs);
        atomicAdd(a.stats + kStatClTopEntered, (unsigned long long)st_pf.cl_top_entered);
        atomicAdd(a.stats + kStatPfLanePairs, (unsigned long long)st_pf.lane_pairs);
        atomicAdd(a.stats + kStatPriBlocked, (unsigned long long)st_pri_blocked);
        atomicAdd(a.stats + kStatPriWaitSec, (unsigned long long)st_pri_waitsec);
        atomicAdd(a.stats + kStatPriDone, (unsigned long long)st_pri_done);
        atomicAdd(a.stats + kStatSecDone, (unsigned long long)st_sec_done);
        atomicAdd(a.stats + kStatSecWaitPri, (unsigned long long)st_sec_waitpri);
        atomicAdd(a.stats + kStatDoneTrips, (unsigned long long)st_done_trips);
        atomicAdd(a.stats + kStatDoneLaneTrips, (unsigned long long)st_done_lanes);
        atomicAdd(a.stats + kStatSecExact, (unsigned long long)st_sec_exact);
        atomicAdd(a.stats + kStatSecBadLanes, (unsigned long long)st_sec_badlanes);
        atomicAdd(a.stats + kStatSecZeroDir, (unsigned long long)st_sec_zerodir);
    }
}

// Primary-ray culling of one wave tile (TW x TH pixels at x0, ly0): bit p of
// the mask is set when some sphere of pair p (sphere slots 2p, 2p + 1: half
// p & 1 of group p >> 1) may pass some primary ray's exact test
// (cone_may_hit).  One sphere per lane, 64 per ballot, folded into one bit
// per pair; word w covers pairs 64w .. 64w+63 (spheres 128w .. 128w+127).
template <int P>
__device__ __forceinline__ uint64_t wave_tile_mask(const TraceArgs &a, const Cone &c, uint32_t w, uint32_t lane) {
    const float *gf = reinterpret_cast<const float *>(a.groups);
    uint64_t gm = 0;
    for (uint32_t q = 0; q < 2u && w * 128u + q * 64u < 4u * a.n_groups; ++q) {
        const uint32_t sph = w * 128u + q * 64u + lane;  // sphere slot 4*g + l
        bool cand = false;
        if (sph < 4u * a.n_groups) {
            const float *row = gf + (size_t)(sph >> 2) * (4u * kGroupF4) + (sph & 3u);
            cand = cone_may_hit(a, c, row[4u * kRowX], row[4u * kRowY], row[4u * kRowZ], row[4u * kRowR2]);
        }
        uint64_t m = __ballot(cand);
        m = (m | (m >> 1)) & 0x5555555555555555ull;  // bit 2i: some sphere of pair 32q + i
        m = (m | (m >> 1)) & 0x3333333333333333ull;  // compress the even bits into bits 0..31
        m = (m | (m >> 2)) & 0x0F0F0F0F0F0F0F0Full;
        m = (m | (m >> 4)) & 0x00FF00FF00FF00FFull;
        m = (m | (m >> 8)) & 0x0000FFFF0000FFFFull;
        m = (m | (m >> 16)) & 0x00000000FFFFFFFFull;
        gm |= m << (32u * q);
    }
    return gm;
}

// The cull pass: one block per block tile, one wave per wave tile (the trace
// kernel's geometry).  Runs once per camera / scene / launch geometry; the
// trace launches reuse its masks and live-tile list.
// Striped launch counters of the cull pass (one atomic per block tile, spread
// over kCullStripes addresses so they do not serialise on one): [0, 64) live
// block tiles, [64, 128) image pixels of dead block tiles.
constexpr uint32_t kCullStripes = 64;

// The cull pass: one block per block tile, one wave per wave tile (the trace
// kernel's geometry).  Runs once per camera / scene / launch geometry; the
// trace launches reuse its masks and live-tile list.
template <int P>
__global__ __launch_bounds__(256) void cull_kernel(TraceArgs a, uint32_t *live, uint32_t *cost,
                                                   unsigned long long *counters, uint32_t empty_capable) {
    constexpr uint32_t TW = Shape<P>::TW, TH = Shape<P>::TH;
    __shared__ uint32_t s_any;
    const uint32_t tile = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t tile_x = tile % a.tiles_x, tile_y = tile / a.tiles_x;
    // the wave tile's pixel extent [x0, x1] x [ly0, ly1] (see trace_kernel)
    const uint32_t x0 = tile_x * (2u * TW) + (a.interleave ? (wave & 1u) : (wave & 1u) * TW);
    const uint32_t ly0 = tile_y * (2u * TH) + (a.interleave ? (wave >> 1) : (wave >> 1) * TH);
    const uint32_t x1 = x0 + (a.interleave ? 2u : 1u) * (TW - 1u), ly1 = ly0 + (a.interleave ? 2u : 1u) * (TH - 1u);
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    // the image rows of the wave tile's first and last band-local rows: the band
    // map is increasing, so every row of the tile lies between them (a tile of
    // 16 rows may span two 8-row bands, whose rows between are other devices':
    // the cone then covers them too, which only makes it wider)
    const uint32_t y0 = ((ly0 / a.band_rows) * a.band_count + a.band_index) * a.band_rows + ly0 % a.band_rows;
    const uint32_t y1 = ((ly1 / a.band_rows) * a.band_count + a.band_index) * a.band_rows + ly1 % a.band_rows;
    const Cone c = tile_cone(a, (double)x0 - 0.501, (double)x1 + 0.501, (double)y0 - 0.501, (double)y1 + 0.501);
    const uint32_t n_words = rtk_mask_words(a.n_groups);
    bool any = false;
    for (uint32_t w = 0; w < n_words; ++w) {
        const uint64_t gm = wave_tile_mask<P>(a, c, w, lane);
        if (lane == 0) const_cast<uint64_t *>(a.masks)[((size_t)tile * 4u + wave) * n_words + w] = gm;
        any = any || gm != 0;
    }
    // a wave tile entirely outside the image does no work
    if (lane == 0 && any && x0 < a.width && ly0 < a.local_rows) atomicOr(&s_any, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool l = s_any != 0 || !empty_capable;
        live[tile] = l ? 1u : 0u;
        if (a.unit_waves) {  // the one-wave kernels' order ranks waves (4 * tile + quadrant)
            for (uint32_t w = 0; w < 4u; ++w) cost[4u * tile + w] = l ? 2u : 0u;
        } else {
            cost[tile] = l ? 2u : 0u;
        }
        const uint32_t stripe = tile % kCullStripes;
        if (l) {
            atomicAdd(counters + stripe, 1ull);
        } else {
            const uint32_t bx = tile_x * 2u * TW, by = tile_y * 2u * TH;
            const uint32_t w = min(2u * TW, a.width - bx), h = min(2u * TH, a.local_rows - by);
            atomicAdd(counters + kCullStripes + stripe, (unsigned long long)w * h);
        }
    }
}

// The cull pass's striped counters summed on the device (one wave), so no
// launch needs the host to read them: counters[kCullTotals] = live block
// tiles, counters[kCullTotals + 1] = image pixels of dead block tiles.
#ifndef RTK_P16_TU
__global__ __launch_bounds__(64) void cull_total_kernel(unsigned long long *counters) {
    const uint32_t lane = threadIdx.x;
    unsigned long long live = counters[lane], dead = counters[kCullStripes + lane];
    for (int off = 32; off > 0; off >>= 1) {
        live += __shfl_xor(live, off);
        dead += __shfl_xor(dead, off);
    }
    if (lane == 0) {
        counters[kCullTotals] = live;
        counters[kCullTotals + 1] = dead;
    }
}
#endif

// Pixels of dead block tiles: no sphere group passes any of the tile's
// (conservative) cone tests, so every primary ray of every sample misses;
// without a sky term each sample's Out is exactly 0 (main.cpp:433-440), its
// one segment still counts (main.cpp:390; dead pixels x frames, the pixels
// from the cull pass's device total, added once), and its blend is
// Final = 0*(1/n) + Prev*((n-1)/n) = RN(Prev*((n-1)/n)) -- folded here without
// generating the rays (an all-zero running mean stays exactly zero).  The
// ratios are the trace kernel's fold-table values.
template <int P>
__global__ __launch_bounds__(256) void empty_kernel(TraceArgs a, const uint32_t *live,
                                                    const unsigned long long *dead_pixels) {
    constexpr uint32_t BW = 2u * Shape<P>::TW, BH = 2u * Shape<P>::TH;
    __shared__ float ratio[kFoldTable];
    const bool fold = a.prev_count > 0 && !(a.flags & kFlagAccumZero);
    if (fold)
        for (uint32_t i = threadIdx.x; i < kFoldTable; i += blockDim.x) {
            const uint32_t pc = a.prev_count + i;
            ratio[i] = (float)pc / (float)(pc + 1u);
        }
    __syncthreads();
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        const unsigned long long dead_rays = *dead_pixels * a.frames;
        if (dead_rays) atomicAdd(a.rays, dead_rays);
    }
    const uint32_t x = blockIdx.x * 256u + threadIdx.x, ly = blockIdx.y;
    if (!(x < a.width && live[(ly / BH) * a.tiles_x + x / BW] == 0u)) return;
    const size_t pix = (size_t)ly * a.width + x;
    float accx = 0.0f, accy = 0.0f, accz = 0.0f;
    if (fold) {
        const float4 pv = a.prev[pix];
        accx = pv.x;
        accy = pv.y;
        accz = pv.z;
    }
    if (accx != 0.0f || accy != 0.0f || accz != 0.0f) {
        for (uint32_t q = 0; q < a.frames; ++q) {
            float r;
            if (q < kFoldTable) {
                r = ratio[q];
            } else {
                const uint32_t pc = a.prev_count + q;
                r = (float)pc / (float)(pc + 1u);
            }
            accx = 0.0f + accx * r;
            accy = 0.0f + accy * r;
            accz = 0.0f + accz * r;
        }
    }
    a.prev[pix] = make_float4(accx, accy, accz, 1.0f);
    if (!a.skip_cur) a.cur[pix] = rgba8(accx, accy, accz, (a.flags & kFlagSrgbPow) != 0u);
}

#ifndef RTK_P16_TU  // (the P = 16 translation unit holds only its trace launches: see launch_p16)
// One wave per block tile: rank its pixels by the last launch's cost (ties by
// index), so wave w of the next launch gets ranks [NPIX w, NPIX (w + 1)).
// With pix_seg = S > 1 the ranked units are row segments of S pixels (summed
// cost), dealt whole: a wave's pixels then form S-pixel runs of a row.
template <int P>
__global__ __launch_bounds__(64) void pixel_sort_kernel(TraceArgs a, uint8_t *perm) {
    constexpr uint32_t TW = Shape<P>::TW, TH = Shape<P>::TH, BW = 2u * TW, NB = 4u * TW * TH;
    static_assert(NB <= 64, "a block tile's pixels fit one wave");
    const uint32_t tile = blockIdx.x, lane = threadIdx.x;
    const uint32_t tile_x = tile % a.tiles_x, tile_y = tile / a.tiles_x;
    uint8_t *pp = perm + (size_t)tile * 64u;
    // a quadrant without candidate groups folds without tracing: keep such blocks as they are
    if (a.masks) {
        const uint32_t n_words = rtk_mask_words(a.n_groups);
        bool live = false;
        for (uint32_t w = 0; lane < 4u && w < n_words; ++w) live = live || a.masks[((size_t)tile * 4u + lane) * n_words + w] != 0;
        if (__builtin_popcountll(__ballot(lane < 4u && live)) != 4) {
            if (lane == 0) pp[0] = 0xFFu;
            return;
        }
    }
    uint32_t c = 0;
    if (lane < NB) {
        const uint32_t x = tile_x * BW + lane % BW, ly = tile_y * (2u * TH) + lane / BW;
        c = x < a.width && ly < a.local_rows ? a.pix_cost[(size_t)ly * a.width + x] : 0u;
    }
    // segment size: a power of two dividing the block row (BW) and the wave's pixels
    constexpr uint32_t NPIX = NB / 4u;
    const uint32_t S = a.pix_seg >= 4u && NPIX >= 4u && BW % 4u == 0 ? 4u : a.pix_seg >= 2u && NPIX >= 2u ? 2u : 1u;
    for (uint32_t off = 1; off < S; off <<= 1) c += (uint32_t)__shfl_xor((int)c, (int)off, 64);  // (every lane active)
    const uint32_t seg = lane / S, nseg = NB / S;
    uint32_t rank = 0;
    for (uint32_t i = 0; i < nseg; ++i) {
        const uint32_t ci = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)(i * S));
        rank += ci < c || (ci == c && i < seg) ? 1u : 0u;
    }
    if (lane < NB) pp[rank * S + lane % S] = (uint8_t)lane;
}

// Scatter RCCL-gathered compact band images into the full framebuffer.
__global__ __launch_bounds__(256) void assemble_kernel(const uint8_t *src, uint64_t rank_stride, uint8_t *dst,
                                                       uint32_t width, uint32_t height, uint32_t elem,
                                                       uint32_t band_rows, uint32_t band_count) {
    const uint32_t y = blockIdx.y;
    const uint32_t band = y / band_rows;
    const uint32_t owner = band % band_count;
    const uint32_t ly = (band / band_count) * band_rows + y % band_rows;
    const uint8_t *s = src + owner * rank_stride + (uint64_t)ly * width * elem;
    uint8_t *d = dst + (uint64_t)y * width * elem;
    const uint32_t row_bytes = width * elem;
    if ((row_bytes & 15u) == 0 && (((uintptr_t)s | (uintptr_t)d) & 15u) == 0) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
        uint4 *d4 = reinterpret_cast<uint4 *>(d);
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < row_bytes / 16u; i += gridDim.x * blockDim.x)
            d4[i] = s4[i];
    } else {
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < row_bytes; i += gridDim.x * blockDim.x)
            d[i] = s[i];
    }
}

// ---- heaviest-first tile order for the next launch (counting sort of the
// per-tile costs this launch measured into 32 log2 buckets, descending)
// Counting sort of the tiles by log2(cost), heaviest bucket first, stable,
// without atomics, over the whole grid (a single-block version was latency
// bound at ~60 us; grid-wide device atomics on the few busy buckets ~300 us).
// A wave walks its 64 tiles visiting only the distinct buckets present
// (readlane of the first pending lane + ballot) and keeps per-bucket counters
// in lane k of one VGPR.  Blocks cover 1024 tiles:
//   tile_count_kernel: block j's kSortBuckets bucket counts -> bcount[kSortBuckets*j + k]
//   tile_scan_kernel:  exclusive scan in (bucket descending, block ascending)
//                      order, staged through LDS
//   tile_rank_kernel:  per-wave bases inside the block, the walk again ->
//                      order[rank] = tile
// Consecutive ranks keep similar cost: blocks are dealt round-robin to the 8
// XCDs, so alternating heavy and light tiles would put all heavy work on half
// of them (measured 2x slower).
constexpr uint32_t kSortBlock = 1024, kSortWaves = kSortBlock / 64, kScanLds = 16384;
constexpr uint32_t kSortBuckets = 64;  // one counter per lane

// Quarter-octave buckets of the cost (cycles): 4 log2(c) + the two bits after
// the leading one, offset so octaves 10..25 (1k..64M cycles) are resolved;
// bucket 0 is cost 0 only (dead tiles), so the live-first prefix survives.
// (Measured against whole octaves: 8-rank C2 share 1.035 -> 0.957 ms, C2
// +1.3 %; eighth-octave buckets measured the same as quarter-octave ones.)
__device__ __forceinline__ uint32_t tile_bucket(const uint32_t *cost, uint32_t i, uint32_t n) {
    if (i >= n) return kSortBuckets;  // past the end
    const uint32_t c = cost[i];
    if (c == 0u) return 0u;
    const int l = 31 - __builtin_clz(c);
    const int q = 4 * l + (l >= 2 ? (int)((c >> (l - 2)) & 3u) : 0) - 40;
    return (uint32_t)(q < 1 ? 1 : q > (int)kSortBuckets - 1 ? (int)kSortBuckets - 1 : q);
}

// lane k < kSortBuckets of the result: run[k] + (this wave's count of bucket k);
// *rank: run[b] + this lane's position among the wave's lanes with bucket b
__device__ __forceinline__ uint32_t wave_walk(uint32_t b, uint32_t run, uint32_t lane, uint32_t *rank) {
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t pend = b;
    for (uint64_t live = __ballot(pend < kSortBuckets); live; live = __ballot(pend < kSortBuckets)) {
        const uint32_t b0 = __builtin_amdgcn_readlane(pend, (int)__builtin_ctzll(live));
        const uint64_t m = __ballot(pend == b0);
        if (pend == b0) {
            *rank = __builtin_amdgcn_readlane(run, (int)b0) + (uint32_t)__popcll(m & lt);
            pend = kSortBuckets;
        }
        if (lane == b0) run += (uint32_t)__popcll(m);
    }
    return run;
}

__global__ __launch_bounds__(kSortBlock) void tile_count_kernel(const uint32_t *cost, uint32_t n, uint32_t *bcount) {
    __shared__ uint32_t wc[kSortWaves][kSortBuckets];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t rank;
    const uint32_t c = wave_walk(tile_bucket(cost, blockIdx.x * kSortBlock + threadIdx.x, n), 0u, lane, &rank);
    if (lane < kSortBuckets) wc[wave][lane] = c;
    __syncthreads();
    if (threadIdx.x < kSortBuckets) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kSortWaves; ++w) t += wc[w][threadIdx.x];
        bcount[kSortBuckets * blockIdx.x + threadIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void tile_scan_kernel(uint32_t *bcount, uint32_t n_blk) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t stage[kScanLds];
    const uint32_t len = kSortBuckets * n_blk, t = threadIdx.x, per = (len + 1023u) / 1024u;
    const bool in_lds = len <= kScanLds;
    if (in_lds)
        for (uint32_t j = t; j < len; j += 1024u) stage[j] = bcount[j];
    __syncthreads();
    uint32_t *const src = in_lds ? stage : bcount;
    // scan position p -> (bucket kSortBuckets-1 - p / n_blk, block p % n_blk)
    auto at = [&](uint32_t p) -> uint32_t & { return src[kSortBuckets * (p % n_blk) + (kSortBuckets - 1u - p / n_blk)]; };
    const uint32_t p0 = min(len, t * per), p1 = min(len, p0 + per);
    uint32_t sum = 0;
    for (uint32_t p = p0; p < p1; ++p) sum += at(p);
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {  // inclusive Hillis-Steele scan of the partials
        const uint32_t x = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t off = part[t] - sum;
    for (uint32_t p = p0; p < p1; ++p) {
        const uint32_t c = at(p);
        at(p) = off;
        off += c;
    }
    __syncthreads();
    if (in_lds)
        for (uint32_t j = t; j < len; j += 1024u) bcount[j] = stage[j];
}

__global__ __launch_bounds__(kSortBlock) void tile_rank_kernel(uint32_t *cost, uint32_t n, const uint32_t *bbase,
                                                               uint32_t *order) {
    __shared__ uint32_t wc[kSortWaves][kSortBuckets];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * kSortBlock + threadIdx.x, b = tile_bucket(cost, i, n);
    uint32_t rank = 0;
    const uint32_t c = wave_walk(b, 0u, lane, &rank);
    if (lane < kSortBuckets) wc[wave][lane] = c;
    __syncthreads();
    if (threadIdx.x < kSortBuckets) {  // the block's base -> each wave's base, in wave order
        uint32_t off = bbase[kSortBuckets * blockIdx.x + threadIdx.x];
        for (uint32_t w = 0; w < kSortWaves; ++w) {
            const uint32_t x = wc[w][threadIdx.x];
            wc[w][threadIdx.x] = off;
            off += x;
        }
    }
    __syncthreads();
    (void)wave_walk(b, lane < kSortBuckets ? wc[wave][lane] : 0u, lane, &rank);
    if (b < kSortBuckets) {
        order[rank] = i;
        cost[i] = 0;  // measured afresh by the next launch
    }
}

// ---- XCD grouping of the wave order (one-wave kernels).  Workgroups are dealt
// round-robin to the 8 XCDs (block b and b + 8 share one; MI355X_MICROARCH.md,
// "Workgroup dispatch"), so the four waves of a block tile, which store
// neighbouring pixels of the same 128-B lines, land on up to four XCDs whose
// L2s each write their part of every line back (the excess HBM writes of §4).
// Grouping keeps the per-wave heaviest-first order but moves every unit of block
// tile t into one XCD group x = grp[t] (below): the live prefix [0, L) of the sorted order is
// partitioned stably by x (each group stays heaviest first), and group x's r-th
// unit goes to position 8r + x while r < m (the smallest group's size), so block
// 8r + x runs on the group's XCD; the r >= m leftovers (the lightest units of the
// larger groups) follow at 8m + ..., group by group.  A permutation of [0, L):
// no unit is lost or repeated; [L, n) (dead tiles' units) is copied as is.
constexpr uint32_t kXgBlock = 1024, kXgWaves = kXgBlock / 64;

// The group of a block tile is its rank, among the live tiles, in the order of
// their heaviest wave (the tile's first unit in the sorted order), modulo 8: the
// groups then take every eighth tile of a cost-sorted list, so the eight XCDs get
// equal work (a group by tile & 7 measured C2 -1.2 %: its columns' costs differ).
// xg_first_kernel: first[t] = the smallest sorted position of tile t's units;
// xg_flag_count / xg_scan / xg_tile_rank: grp[t] = (rank of tile t among the live
// tiles, by first[t]) & 7 (first and grp: two n_tiles-word arrays in aux).
__device__ __forceinline__ uint32_t xg_group(const uint32_t *in, uint32_t i, uint32_t live_units,
                                             const uint32_t *grp) {
    return i < live_units ? grp[in[i] >> 2] : 8u;
}

__global__ __launch_bounds__(kXgBlock) void xg_first_kernel(const uint32_t *in, uint32_t n,
                                                            const unsigned long long *live_tiles, uint32_t *first) {
    const uint32_t i = blockIdx.x * kXgBlock + threadIdx.x;
    const uint32_t L = (uint32_t)min((unsigned long long)n, 4ull * *live_tiles);
    if (i < L) atomicMin(first + (in[i] >> 2), i);
}

// per block: the number of positions that are their tile's first (bc[blk])
__global__ __launch_bounds__(kXgBlock) void xg_flag_count_kernel(const uint32_t *in, uint32_t n,
                                                                 const unsigned long long *live_tiles,
                                                                 const uint32_t *first, uint32_t *bc) {
    __shared__ uint32_t wc[kXgWaves];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, i = blockIdx.x * kXgBlock + threadIdx.x;
    const uint32_t L = (uint32_t)min((unsigned long long)n, 4ull * *live_tiles);
    const bool f = i < L && first[in[i] >> 2] == i;
    const uint64_t m = __ballot(f);
    if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kXgWaves; ++w) t += wc[w];
        bc[blockIdx.x] = t;
    }
}

// one wave: exclusive scan of bc[0, n_blk) in place
__global__ __launch_bounds__(64) void xg_scan1_kernel(uint32_t *bc, uint32_t n_blk) {
    if (threadIdx.x != 0) return;
    uint32_t run = 0;
    for (uint32_t b = 0; b < n_blk; ++b) {
        const uint32_t c = bc[b];
        bc[b] = run;
        run += c;
    }
}

__global__ __launch_bounds__(kXgBlock) void xg_tile_rank_kernel(const uint32_t *in, uint32_t n,
                                                                const unsigned long long *live_tiles,
                                                                const uint32_t *first, const uint32_t *bc,
                                                                uint32_t *grp) {
    __shared__ uint32_t wc[kXgWaves];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, i = blockIdx.x * kXgBlock + threadIdx.x;
    const uint32_t L = (uint32_t)min((unsigned long long)n, 4ull * *live_tiles);
    const bool f = i < L && first[in[i] >> 2] == i;
    const uint64_t m = __ballot(f);
    if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (!f) return;
    uint32_t rank = bc[blockIdx.x] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    for (uint32_t w = 0; w < wave; ++w) rank += wc[w];
    grp[in[i] >> 2] = rank & 7u;
}

__global__ __launch_bounds__(kXgBlock) void xg_count_kernel(const uint32_t *in, uint32_t n,
                                                            const unsigned long long *live_tiles, const uint32_t *grp,
                                                            uint32_t *bc) {
    __shared__ uint32_t wc[kXgWaves][8];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, i = blockIdx.x * kXgBlock + threadIdx.x;
    const uint32_t L = (uint32_t)min((unsigned long long)n, 4ull * *live_tiles);
    const uint32_t x = xg_group(in, i, L, grp);
    for (uint32_t v = 0; v < 8u; ++v) {
        const uint64_t m = __ballot(x == v);
        if (lane == v) wc[wave][v] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < 8u) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kXgWaves; ++w) t += wc[w][threadIdx.x];
        bc[8u * blockIdx.x + threadIdx.x] = t;
    }
}

// one wave: per-group exclusive scan over the blocks (in place), then the group
// sizes c_x, m = min c_x and the leftover bases at bc[8 n_blk ..]
__global__ __launch_bounds__(64) void xg_scan_kernel(uint32_t *bc, uint32_t n_blk) {
    const uint32_t lane = threadIdx.x;
    uint32_t run = 0;
    if (lane < 8u)
        for (uint32_t b = 0; b < n_blk; ++b) {
            const uint32_t c = bc[8u * b + lane];
            bc[8u * b + lane] = run;
            run += c;
        }
    uint32_t m = lane < 8u ? run : 0xFFFFFFFFu;
    for (int off = 1; off < 8; off <<= 1) m = min(m, (uint32_t)__shfl_xor((int)m, off, 64));
    m = (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
    // base_x = sum over y < x of (c_y - m)
    uint32_t extra = lane < 8u ? run - m : 0u, base = 0;
    for (uint32_t y = 0; y < 8u; ++y) {
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)extra, (int)y);
        if (y < lane) base += e;
    }
    if (lane == 0) bc[8u * n_blk] = m;
    if (lane < 8u) bc[8u * n_blk + 1u + lane] = base;
}

__global__ __launch_bounds__(kXgBlock) void xg_place_kernel(const uint32_t *in, uint32_t *out, uint32_t n,
                                                            const unsigned long long *live_tiles, const uint32_t *grp,
                                                            const uint32_t *bc, uint32_t n_blk) {
    __shared__ uint32_t wc[kXgWaves][8];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, i = blockIdx.x * kXgBlock + threadIdx.x;
    const uint32_t L = (uint32_t)min((unsigned long long)n, 4ull * *live_tiles);
    const uint32_t x = xg_group(in, i, L, grp);
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t rank = 0;
    for (uint32_t v = 0; v < 8u; ++v) {
        const uint64_t m = __ballot(x == v);
        if (x == v) rank = (uint32_t)__popcll(m & lt);
        if (lane == v) wc[wave][v] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (i >= n) return;
    if (x >= 8u) {  // a dead tile's unit (or past the live prefix): unchanged
        out[i] = in[i];
        return;
    }
    for (uint32_t w = 0; w < wave; ++w) rank += wc[w][x];
    const uint32_t r = bc[8u * blockIdx.x + x] + rank;
    const uint32_t m = bc[8u * n_blk];
    const uint32_t pos = r < m ? 8u * r + x : 8u * m + bc[8u * n_blk + 1u + x] + (r - m);
    out[pos] = in[i];
}

#endif  // !RTK_P16_TU
}  // namespace rtk

#ifndef RTK_P16_TU
extern "C" size_t rtk_tile_sort_scratch(uint32_t n) {
    return rtk::kSortBuckets * 4u * (size_t)((n + rtk::kSortBlock - 1u) / rtk::kSortBlock);
}

extern "C" int rtk_launch_tile_sort(uint32_t *cost, uint32_t *order, uint32_t *scratch, uint32_t n, hipStream_t stream) {
    const uint32_t n_blk = (n + rtk::kSortBlock - 1u) / rtk::kSortBlock;
    if (n_blk == 0) return 0;
    const dim3 grid(n_blk), block(rtk::kSortBlock);
    hipLaunchKernelGGL(rtk::tile_count_kernel, grid, block, 0, stream, (const uint32_t *)cost, n, scratch);
    hipLaunchKernelGGL(rtk::tile_scan_kernel, dim3(1), dim3(1024), 0, stream, scratch, n_blk);
    hipLaunchKernelGGL(rtk::tile_rank_kernel, grid, block, 0, stream, cost, n, (const uint32_t *)scratch, order);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int rtk_launch_xcd_group(const uint32_t *order_in, uint32_t *order_out, uint32_t n_units,
                                    const unsigned long long *live_tiles, uint32_t *scratch, uint32_t *aux,
                                    hipStream_t stream) {
    const uint32_t n_blk = (n_units + rtk::kXgBlock - 1u) / rtk::kXgBlock;
    if (n_blk == 0) return 0;
    const uint32_t n_tiles = (n_units + 3u) / 4u;
    uint32_t *first = aux, *grp = aux + n_tiles;
    const dim3 grid(n_blk), block(rtk::kXgBlock);
    if (hipMemsetAsync(first, 0xFF, (size_t)n_tiles * 4u, stream) != hipSuccess) return -5;
    hipLaunchKernelGGL(rtk::xg_first_kernel, grid, block, 0, stream, order_in, n_units, live_tiles, first);
    hipLaunchKernelGGL(rtk::xg_flag_count_kernel, grid, block, 0, stream, order_in, n_units, live_tiles,
                       (const uint32_t *)first, scratch);
    hipLaunchKernelGGL(rtk::xg_scan1_kernel, dim3(1), dim3(64), 0, stream, scratch, n_blk);
    hipLaunchKernelGGL(rtk::xg_tile_rank_kernel, grid, block, 0, stream, order_in, n_units, live_tiles,
                       (const uint32_t *)first, (const uint32_t *)scratch, grp);
    hipLaunchKernelGGL(rtk::xg_count_kernel, grid, block, 0, stream, order_in, n_units, live_tiles,
                       (const uint32_t *)grp, scratch);
    hipLaunchKernelGGL(rtk::xg_scan_kernel, dim3(1), dim3(64), 0, stream, scratch, n_blk);
    hipLaunchKernelGGL(rtk::xg_place_kernel, grid, block, 0, stream, order_in, order_out, n_units, live_tiles,
                       (const uint32_t *)grp, (const uint32_t *)scratch, n_blk);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" uint32_t rtk_tiles_x(uint32_t width, int lanes_per_pixel) {
    return rtk_tile_count(width, 1u, lanes_per_pixel);
}

extern "C" uint32_t rtk_tile_count(uint32_t width, uint32_t local_rows, int lanes_per_pixel) {
    uint32_t bw = 16u, bh = 16u;  // 2*TW x 2*TH of the launch's shape
    switch (lanes_per_pixel) {
        case 32: bw = 2u * rtk::Shape<32>::TW; bh = 2u * rtk::Shape<32>::TH; break;
        case 16: bw = 2u * rtk::Shape<16>::TW; bh = 2u * rtk::Shape<16>::TH; break;
        case 8: bw = 2u * rtk::Shape<8>::TW; bh = 2u * rtk::Shape<8>::TH; break;
        case 4: bw = 2u * rtk::Shape<4>::TW; bh = 2u * rtk::Shape<4>::TH; break;
        case 2: bw = 2u * rtk::Shape<2>::TW; bh = 2u * rtk::Shape<2>::TH; break;
        case 0: bw = 2u * rtk::Shape<0>::TW; bh = 2u * rtk::Shape<0>::TH; break;
        default: bw = 2u * rtk::Shape<1>::TW; bh = 2u * rtk::Shape<1>::TH; break;
    }
    return ((width + bw - 1u) / bw) * ((local_rows + bh - 1u) / bh);
}

#endif  // !RTK_P16_TU

template <int P>
static void launch_p(const TraceArgs *a, int simd, int src, int cull, uint32_t n_blocks, hipStream_t stream) {
    const dim3 block(256), grid(n_blocks);
    const size_t lds = rtk_lds_bytes(a);
    const size_t solo_lds = 8u * rtk_mask_words(a->n_groups);  // one-wave kernels: the cull mask words
#define RTK_LAUNCH(S, R, C, G) hipLaunchKernelGGL((rtk::trace_kernel<S, R, C, P, G>), grid, block, lds, stream, *a)
#define RTK_LAUNCH_SOLO(S, C, K) \
    hipLaunchKernelGGL((rtk::trace_kernel<S, kSrcSmem, C, P, true, true, K>), dim3(4u * n_blocks), dim3(64), solo_lds, \
                       stream, *a)
    if (a->solo) {  // one wave per workgroup, no LDS image (the host clears the *_in_lds flags)
        // one walk per kernel for the culled production shapes; others dispatch at run time
        if constexpr (P == 0 || P == 4 || P == 8 || P == 16) {
            if (cull) {
#define RTK_WALKS(S)                                                          \
    switch (a->walk) {                                                        \
        case kWalkGroups: RTK_LAUNCH_SOLO(S, true, kWalkGroups); return;      \
        case kWalkCl1: RTK_LAUNCH_SOLO(S, true, kWalkCl1); return;            \
        case kWalkCl2: RTK_LAUNCH_SOLO(S, true, kWalkCl2); return;            \
        case kWalkCl4: RTK_LAUNCH_SOLO(S, true, kWalkCl4); return;            \
        case kWalkCl1Rel: RTK_LAUNCH_SOLO(S, true, kWalkCl1Rel); return;      \
        case kWalkCl2Rel: RTK_LAUNCH_SOLO(S, true, kWalkCl2Rel); return;      \
        case kWalkCl4Rel: RTK_LAUNCH_SOLO(S, true, kWalkCl4Rel); return;      \
        default: break;                                                       \
    }
                if (simd) { RTK_WALKS(true) } else { RTK_WALKS(false) }
#undef RTK_WALKS
            }
        }
        const int key = (simd ? 2 : 0) | (cull ? 1 : 0);
        switch (key) {
            case 0: RTK_LAUNCH_SOLO(false, false, kWalkAny); break;
            case 1: RTK_LAUNCH_SOLO(false, true, kWalkAny); break;
            case 2: RTK_LAUNCH_SOLO(true, false, kWalkAny); break;
            default: RTK_LAUNCH_SOLO(true, true, kWalkAny); break;
        }
        return;
    }
#undef RTK_LAUNCH_SOLO
    if (!a->scene_in_lds) {  // the scene in HBM (the host picks the SMEM source for it)
        const int key = (simd ? 2 : 0) | (cull ? 1 : 0);
        switch (key) {
            case 0: RTK_LAUNCH(false, kSrcSmem, false, true); break;
            case 1: RTK_LAUNCH(false, kSrcSmem, true, true); break;
            case 2: RTK_LAUNCH(true, kSrcSmem, false, true); break;
            default: RTK_LAUNCH(true, kSrcSmem, true, true); break;
        }
        return;
    }
    const int key = (simd ? 4 : 0) | (src == kSrcLds ? 2 : 0) | (cull ? 1 : 0);
    switch (key) {
        case 0: RTK_LAUNCH(false, kSrcSmem, false, false); break;
        case 1: RTK_LAUNCH(false, kSrcSmem, true, false); break;
        case 2: RTK_LAUNCH(false, kSrcLds, false, false); break;
        case 3: RTK_LAUNCH(false, kSrcLds, true, false); break;
        case 4: RTK_LAUNCH(true, kSrcSmem, false, false); break;
        case 5: RTK_LAUNCH(true, kSrcSmem, true, false); break;
        case 6: RTK_LAUNCH(true, kSrcLds, false, false); break;
        default: RTK_LAUNCH(true, kSrcLds, true, false); break;
    }
#undef RTK_LAUNCH
}

// The P = 16 trace kernels (the 8-GPU band shares) are compiled in
// a translation unit of their own (this file with RTK_P16_TU, Makefile
// build/rt_kernel_p16.o) under the scheduler's register-pressure trackers
// (-amdgpu-use-amdgpu-trackers): about -1.4 % on the 8-rank share over two same-box
// A/Bs (0.770 against 0.781 ms, near the noise), while the same flag
// costs the P = 4 kernel of one GPU 1.7 % (profiles/r02_sched_trackers_ab.txt).
extern "C" void rtk_launch_p16(const TraceArgs *a, int simd, int src, int cull, uint32_t n_blocks,
                               hipStream_t stream);
#ifdef RTK_P16_TU
extern "C" void rtk_launch_p16(const TraceArgs *a, int simd, int src, int cull, uint32_t n_blocks,
                               hipStream_t stream) {
    launch_p<16>(a, simd, src, cull, n_blocks, stream);
}
#else
extern "C" int rtk_launch_trace_grid(const TraceArgs *a, int simd, int src, int cull, int lanes_per_pixel,
                                     uint32_t n_blocks, hipStream_t stream) {
    if (n_blocks == 0) return 0;
    switch (lanes_per_pixel) {
        case 32: launch_p<32>(a, simd, src, cull, n_blocks, stream); break;
        case 16: rtk_launch_p16(a, simd, src, cull, n_blocks, stream); break;
        case 8: launch_p<8>(a, simd, src, cull, n_blocks, stream); break;
        case 4: launch_p<4>(a, simd, src, cull, n_blocks, stream); break;
        case 2: launch_p<2>(a, simd, src, cull, n_blocks, stream); break;
        case 0: launch_p<0>(a, simd, src, cull, n_blocks, stream); break;
        default: launch_p<1>(a, simd, src, cull, n_blocks, stream); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int rtk_launch_trace(const TraceArgs *a, int simd, int src, int cull, int lanes_per_pixel,
                                hipStream_t stream) {
    return rtk_launch_trace_grid(a, simd, src, cull, lanes_per_pixel,
                                 rtk_tile_count(a->width, a->local_rows, lanes_per_pixel), stream);
}

#define RTK_BY_P(F, ...)                                     \
    switch (lanes_per_pixel) {                               \
        case 32: F<32>(__VA_ARGS__); break;                  \
        case 16: F<16>(__VA_ARGS__); break;                  \
        case 8: F<8>(__VA_ARGS__); break;                    \
        case 4: F<4>(__VA_ARGS__); break;                    \
        case 2: F<2>(__VA_ARGS__); break;                    \
        case 0: F<0>(__VA_ARGS__); break;                    \
        default: F<1>(__VA_ARGS__); break;                   \
    }

namespace rtk {
// The primary rounds' group rows for this camera (TraceArgs.prim): one sphere
// slot per thread, c = RN(centre - CameraPosition) as main.cpp:401 rounds it
// (one f32 subtraction: no contraction, IEEE denormals), and r*r copied.
__global__ __launch_bounds__(256) void prim_kernel(TraceArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;  // sphere slot 4 g + l
    if (i >= 4u * a.n_groups) return;
    const uint32_t g = i >> 2, l = i & 3u;
    const float *src = reinterpret_cast<const float *>(a.groups + (size_t)kGroupF4 * g);
    float *dst = reinterpret_cast<float *>(a.prim + (size_t)kPrimF4 * g);
    dst[0u + l] = src[4u * kRowX + l] - a.cam_pos[0];
    dst[4u + l] = src[4u * kRowY + l] - a.cam_pos[1];
    dst[8u + l] = src[4u * kRowZ + l] - a.cam_pos[2];
    dst[12u + l] = src[4u * kRowR2 + l];
}
}  // namespace rtk

template <int P>
static void launch_cull_p(const TraceArgs *a, uint32_t *live, uint32_t *cost, unsigned long long *counters,
                          int empty_capable, hipStream_t stream) {
    const uint32_t n = rtk_tile_count(a->width, a->local_rows, P);
    if (a->n_groups)
        hipLaunchKernelGGL(rtk::prim_kernel, dim3((4u * a->n_groups + 255u) / 256u), dim3(256), 0, stream, *a);
    (void)hipMemsetAsync(counters, 0, 2u * rtk::kCullStripes * sizeof(unsigned long long), stream);
    hipLaunchKernelGGL(rtk::cull_kernel<P>, dim3(n), dim3(256), 0, stream, *a, live, cost, counters,
                       (uint32_t)(empty_capable != 0));
    hipLaunchKernelGGL(rtk::cull_total_kernel, dim3(1), dim3(64), 0, stream, counters);
}

extern "C" int rtk_launch_cull(const TraceArgs *a, int lanes_per_pixel, uint32_t *live, uint32_t *cost,
                               unsigned long long *counters, int empty_capable, hipStream_t stream) {
    if (!a->masks || !a->prim) return -1;
    RTK_BY_P(launch_cull_p, a, live, cost, counters, empty_capable, stream)
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int P>
static void launch_empty_p(const TraceArgs *a, const uint32_t *live, const unsigned long long *dead_pixels,
                           hipStream_t stream) {
    hipLaunchKernelGGL(rtk::empty_kernel<P>, dim3((a->width + 255u) / 256u, a->local_rows), dim3(256), 0, stream, *a,
                       live, dead_pixels);
}

extern "C" int rtk_launch_empty(const TraceArgs *a, int lanes_per_pixel, const uint32_t *live,
                                const unsigned long long *dead_pixels, hipStream_t stream) {
    RTK_BY_P(launch_empty_p, a, live, dead_pixels, stream)
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int P>
static void launch_pixel_sort_p(const TraceArgs *a, uint8_t *perm, hipStream_t stream) {
    const uint32_t n = rtk_tile_count(a->width, a->local_rows, P);
    hipLaunchKernelGGL(rtk::pixel_sort_kernel<P>, dim3(n), dim3(64), 0, stream, *a, perm);
}

extern "C" int rtk_launch_pixel_sort(const TraceArgs *a, int lanes_per_pixel, uint8_t *perm, hipStream_t stream) {
    switch (a->pix_cost ? lanes_per_pixel : 0) {  // (a block tile of 64 pixels at most: P >= 4)
        case 32: launch_pixel_sort_p<32>(a, perm, stream); break;
        case 16: launch_pixel_sort_p<16>(a, perm, stream); break;
        case 8: launch_pixel_sort_p<8>(a, perm, stream); break;
        case 4: launch_pixel_sort_p<4>(a, perm, stream); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
#undef RTK_BY_P

namespace rtk {
// Re-encode a resident running mean (v4 f32) as RGBA8: the store of
// main.cpp:490 on its own (rt_encode_rgba8).
__global__ __launch_bounds__(256) void encode_kernel(const float4 *accum, uint32_t *out, uint64_t n, uint32_t pw) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 v = accum[i];
        out[i] = rgba8(v.x, v.y, v.z, pw != 0u);
    }
}
}  // namespace rtk

extern "C" int rtk_launch_encode(const void *accum, void *out, uint64_t n, uint32_t pow_mode, hipStream_t stream) {
    if (n == 0) return 0;
    const uint64_t blocks = (n + 255u) / 256u;
    const uint32_t grid = (uint32_t)(blocks < 8192u ? blocks : 8192u);
    hipLaunchKernelGGL(rtk::encode_kernel, dim3(grid), dim3(256), 0, stream, (const float4 *)accum, (uint32_t *)out, n,
                       pow_mode);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void sum_u64_kernel(const uint64_t *slots, uint32_t n, uint64_t *dst) {
    if (threadIdx.x != 0) return;
    uint64_t s = 0;
    for (uint32_t i = 0; i < n; ++i) s += slots[i];
    dst[0] += s;
}

extern "C" int rtk_launch_sum_u64(const uint64_t *slots, uint32_t n, uint64_t *dst, hipStream_t stream) {
    hipLaunchKernelGGL(sum_u64_kernel, dim3(1), dim3(64), 0, stream, slots, n, dst);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int rtk_launch_assemble(const void *src, uint64_t rank_stride, void *dst, uint32_t width, uint32_t height,
                                   uint32_t elem, uint32_t band_rows, uint32_t band_count, hipStream_t stream) {
    const dim3 block(256);
    const dim3 grid(4, height);
    hipLaunchKernelGGL(rtk::assemble_kernel, grid, block, 0, stream, (const uint8_t *)src, rank_stride, (uint8_t *)dst,
                       width, height, elem, band_rows, band_count);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
#endif  // RTK_P16_TU
