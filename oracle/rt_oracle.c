/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).  CPU restatement of the
 * reference trace path, written from the behaviour of the reference, not copied.
 * Every function cites the reference file:line it restates.
 *
 * Floating-point policy (must match the reference's clang -O3 -mavx2 -mfma
 * x64 build, win32/compile.ps1:15):
 *   - built with -ffp-contract=off: every + - * / sqrt rounds separately,
 *     exactly like the SSE lane ops of x64_math.h;
 *   - the two places where that clang build DID contract are written as
 *     explicit fmaf(): Reflectance (main.cpp:299) and v3::Cross
 *     (x64_math.h:260-262, used only for the camera basis);
 *   - rsqrtss (x64_math.h:71-74, NormalizeFast) is reproduced bit-exactly
 *     by a 2x1024 table captured from an Intel host (tests/golden/).
 * Lane-4 SIMD semantics use SSE intrinsics so this also serves as the
 * reference-speed CPU baseline (bench.py cpu_baseline, kind "port").
 */
#include "rt_oracle.h"

#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define OR_TILE 32u                      /* main.cpp:9 TileSize */
#define OR_EPS 1e-4f                     /* base.h:889 F32Epsilon */
#define OR_FMAX 1e30f                    /* base.h:891 F32Max */
#define OR_PI32 3.14159265358979323846f  /* base.h:892 */
#define OR_WORLD_SCALE 0.0625f           /* main.cpp:56 (1.0 / 16.0f, exact) */

/* ------------------------------------------------------------------ PRNG */

/* base.h:954-963 (PCG variant with RotateRight32, x64_math.h:168-170). */
uint32_t or_pcg(uint64_t *state)
{
    uint64_t old = *state;
    *state = old * 6364136223846793005ULL + 1442695040888963407ULL;
    uint32_t v = (uint32_t)(old >> 32) ^ (uint32_t)old;
    uint32_t r = (uint32_t)(old >> 59);
    return (v >> r) | (v << ((32u - r) & 31u));
}

/* base.h:983-989: (Max-Min) in f32, divided in f64 by 2^32-1, rounded to f32;
 * then (f32)N * Inv and + Min, each rounded. */
float or_random_float(uint64_t *state, float lo, float hi)
{
    uint32_t n = or_pcg(state);
    float inv = (float)((double)(hi - lo) / 4294967295.0);
    float r = (float)n * inv;
    return r + lo;
}

/* main.cpp:668-675, per-thread seed; also the per-(pixel,frame) seed of the
 * 'pixel' mode with i = (k*H + y)*W + x. */
uint64_t or_seed_mix(uint64_t i)
{
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

/* ---------------------------------------------------------- rsqrt table */

static float g_rsqrt_lut[2048];

void or_set_rsqrt_lut(const float *lut2048) { memcpy(g_rsqrt_lut, lut2048, sizeof(g_rsqrt_lut)); }

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* Intel rsqrtss (x64_math.h:71-74) depends only on the exponent parity and
 * the top 10 mantissa bits; scaling the input by 4 halves the output exactly
 * (verified exhaustively over [1e-9, 1e9] by tests/golden/make_rsqrt_lut.c). */
float or_rsqrt(float x)
{
    uint32_t u = f2u(x);
    int32_t e = (int32_t)((u >> 23) & 0xFFu) - 127;
    uint32_t par = (uint32_t)e & 1u;
    float base = g_rsqrt_lut[par * 1024u + ((u >> 13) & 1023u)];
    int32_t sh = (e - (int32_t)par) / 2;
    return u2f(f2u(base) - ((uint32_t)sh << 23));
}

/* ----------------------------------------------------------- v3 helpers */

static inline float dot3(const float a[3], const float b[3])
{
    float px = a[0] * b[0], py = a[1] * b[1], pz = a[2] * b[2];
    return (px + py) + pz;  /* x64_math.h:224-227 */
}

/* x64_math.h:234-245: v / sqrt(len2) (IEEE div), zeroed if len2 <= 1e-4. */
void or_normalize(const float in[3], float out[3])
{
    float l2 = dot3(in, in);
    float len = sqrtf(l2);
    int keep = l2 > OR_EPS;
    for (int c = 0; c < 3; ++c) out[c] = keep ? in[c] / len : 0.0f;
}

/* x64_math.h:246-257: v * rsqrtss(len2), zeroed if len2 <= 1e-4. */
void or_normalize_fast(const float in[3], float out[3])
{
    float l2 = dot3(in, in);
    int keep = l2 > OR_EPS;
    float inv = keep ? or_rsqrt(l2) : 0.0f;
    for (int c = 0; c < 3; ++c) out[c] = keep ? in[c] * inv : 0.0f;
}

/* x64_math.h:258-264 as contracted by clang -mfma: x = fma(Ay,Bz,-(Az*By)). */
static void cross_fma(const float a[3], const float b[3], float out[3])
{
    out[0] = fmaf(a[1], b[2], -(a[2] * b[1]));
    out[1] = fmaf(a[2], b[0], -(a[0] * b[2]));
    out[2] = fmaf(a[0], b[1], -(a[1] * b[0]));
}

/* x64_math.h:728-746: x87 fcos/fsin on the f32 argument, result stored f32. */
static float x87_cos(float x)
{
    long double r = x;
    __asm__("fcos" : "+t"(r));
    return (float)r;
}
static float x87_sin(float x)
{
    long double r = x;
    __asm__("fsin" : "+t"(r));
    return (float)r;
}

/* ---------------------------------------------------------------- scenes */

static or_v3 v3s(float x, float y, float z) { or_v3 v = {x, y, z, 0.0f}; return v; }

/* main.cpp:57-71 CreateScalarSphere. */
static void create_sphere(or_v3 pos, float radius, or_v3 color, float spec, float ior, or_v3 emis,
                          or_sphere *s, int world_scale)
{
    memset(s, 0, sizeof(*s));
    if (world_scale) {
        s->pos = v3s(pos.x * OR_WORLD_SCALE, pos.y * OR_WORLD_SCALE, pos.z * OR_WORLD_SCALE);
        s->radius = radius * OR_WORLD_SCALE;
    } else {
        s->pos = pos;
        s->radius = radius;
    }
    s->mat.color = color;
    s->mat.specular = spec;
    s->mat.emissive = emis;
    s->mat.ior = ior;
}

/* main.cpp:73-91 ConvertScalarSpheresToSIMDSpheres (padding lanes stay 0). */
static void to_groups(const or_sphere *s, uint32_t n, or_group *g, or_material *m)
{
    uint32_t ng = (n + 3u) / 4u;
    memset(g, 0, ng * sizeof(or_group));
    memset(m, 0, (n + 1u) * sizeof(or_material));
    for (uint32_t i = 0; i < n; ++i) {
        g[i / 4].px[i % 4] = s[i].pos.x;
        g[i / 4].py[i % 4] = s[i].pos.y;
        g[i / 4].pz[i % 4] = s[i].pos.z;
        g[i / 4].r[i % 4] = s[i].radius;
        m[i] = s[i].mat;
    }
}

static void normalize_v3(or_v3 *v)
{
    float in[3] = {v->x, v->y, v->z}, out[3];
    or_normalize(in, out);
    v->x = out[0]; v->y = out[1]; v->z = out[2];
}

/* main.cpp:96-167 InitRandomizedSphereScene ("Floating Spheres", 256). */
static void scene_floating(or_sphere *sp, or_scene_info *info)
{
    uint64_t rng = 0x29D7A0A514F22432ULL;
    or_material mats[28];
    const uint32_t len = 256;
    info->default_distance = 48.0f * OR_WORLD_SCALE;
    info->default_xangle = (float)((double)(OR_PI32 * 2.65f) / 2.0);
    info->default_yheight = 0.0f;
    for (uint32_t i = 0; i < 28; ++i) {
        or_v3 color = v3s(0, 0, 0), emis = v3s(0, 0, 0);
        float spec = 0.0f;
        color.x = or_random_float(&rng, 0.15f, 1.0f);
        color.y = or_random_float(&rng, 0.1f, 0.75f);
        color.z = or_random_float(&rng, 0.15f, 1.0f);
        if (or_random_float(&rng, 0.0f, 1.0f) < 0.125f) {
            float k = or_random_float(&rng, 2.0f, 5.0f);
            emis = v3s(k * color.x, k * color.y, k * color.z);
        } else {
            float r = or_random_float(&rng, 0.0f, 1.0f);
            if (r < 0.65f) spec = 1.0f;
        }
        memset(&mats[i], 0, sizeof(mats[i]));
        mats[i].color = color;
        mats[i].emissive = emis;
        mats[i].ior = 0.0f;
        mats[i].specular = spec;
    }
    float radius = or_random_float(&rng, 2.0f, 8.0f);
    const or_material *m0 = &mats[0];
    create_sphere(v3s(1, 0, 0), radius, m0->color, m0->specular, m0->ior, m0->emissive, sp + 0, 0);
    create_sphere(v3s(8, -1, 8), radius, m0->color, m0->specular, m0->ior, m0->emissive, sp + 1, 0);
    create_sphere(v3s(-20, -4, -20), radius, m0->color, m0->specular, m0->ior, m0->emissive, sp + 2, 0);
    for (uint32_t i = 3; i < len; ++i) {
        or_v3 v = v3s(0, 0, 0);
        v.x = or_random_float(&rng, -1.0f, 1.0f);
        v.y = or_random_float(&rng, -1.0f, 1.0f);
        v.z = or_random_float(&rng, -1.0f, 1.0f);
        normalize_v3(&v);
        float r_prev = sp[i - 3].radius;
        or_v3 p = sp[i - 3].pos;
        float r = or_random_float(&rng, 1.0f, 4.0f);
        float dist = (or_random_float(&rng, 1.0f, 8.0f) + r) + r_prev;
        or_v3 pos = v3s(p.x + v.x * dist, p.y + v.y * dist, p.z + v.z * dist);
        const or_material *m = &mats[i % 28];
        create_sphere(pos, r, m->color, m->specular, m->ior, m->emissive, sp + i, 0);
    }
    for (uint32_t i = 0; i < len; ++i) {
        sp[i].radius *= OR_WORLD_SCALE;
        sp[i].pos.x *= OR_WORLD_SCALE;
        sp[i].pos.y *= OR_WORLD_SCALE;
        sp[i].pos.z *= OR_WORLD_SCALE;
    }
    info->look_at = v3s(2.0f * OR_WORLD_SCALE, 0.0f, 2.0f * OR_WORLD_SCALE);
    info->use_sky = 0;
    info->n_spheres = len;
}

/* main.cpp:171-191 InitRGBSphereScene ("RGB Glass", 5). */
static void scene_rgb(or_sphere *sp, or_scene_info *info)
{
    or_v3 z = v3s(0, 0, 0);
    info->default_distance = 16.0f * OR_WORLD_SCALE;
    info->default_xangle = (float)((double)OR_PI32 / 3.0);
    info->default_yheight = 4.0f * OR_WORLD_SCALE;
    create_sphere(v3s(0.0f, -256 - 2.0f, -15.0f), 256.0f, v3s(0.2f, 0.2f, 0.2f), 0.0f, 0.0f, z, sp + 0, 1);
    create_sphere(v3s(0.0f, 0, -10.0f), 2.0f, v3s(1, 1, 1), 0.0f, 1.5f, z, sp + 1, 1);
    create_sphere(v3s(-4.0f, 1.0f, -15.0f), 1.5f, v3s(1, 0, 0), 0.0f, 0, v3s(8, 0, 0), sp + 2, 1);
    create_sphere(v3s(0.0f, 1.0f, -15.0f), 1.5f, v3s(1, 0, 0), 0.0f, 0, v3s(0, 8, 0), sp + 3, 1);
    create_sphere(v3s(4.0f, 1.0f, -15.0f), 1.5f, v3s(1, 0, 0), 0.0f, 0, v3s(0, 0, 8), sp + 4, 1);
    info->look_at = sp[1].pos;
    info->use_sky = 0;
    info->n_spheres = 5;
}

static float len3(float x, float y, float z)
{
    float v[3] = {x, y, z};
    return sqrtf(dot3(v, v));
}

/* main.cpp:196-268 InitRTWeekendSphereScene (482 of the 488 generated spheres
 * fit the reference's array; the RNG stream is consumed for all 484 cells). */
static void scene_rtweekend(or_sphere *sp, or_scene_info *info)
{
    const uint32_t cap = 482;
    or_v3 z = v3s(0, 0, 0);
    info->default_distance = 12.0f * OR_WORLD_SCALE;
    info->default_xangle = OR_PI32 / 8;
    info->default_yheight = 2.0f * OR_WORLD_SCALE;
    uint32_t idx = 0;
    create_sphere(v3s(0, -1000, 0), 1000, v3s(0.5f, 0.5f, 0.5f), 0.0f, 0.0f, z, sp + idx++, 1);
    create_sphere(v3s(0, 1, 0), 1, v3s(1, 1, 1), 0.0f, 1.5f, z, sp + idx++, 1);
    create_sphere(v3s(-4, 1, 0), 1, v3s(0.4f, 0.2f, 0.1f), 0.0f, 0.0f, z, sp + idx++, 1);
    create_sphere(v3s(4, 1, 0), 1, v3s(0.7f, 0.6f, 0.5f), 1.0f, 0.0f, z, sp + idx++, 1);
    uint64_t rng = 0xCD46749A57ACB371ULL;
    for (int32_t i = -11; i < 11; ++i) {
        for (int32_t j = -11; j < 11; ++j) {
            float m = or_random_float(&rng, 0.0f, 1.0f);
            or_v3 c;
            int t1, t2, t3;
            do {
                c.x = (float)i + or_random_float(&rng, -1.0f, 1.0f);
                c.y = 0.2f;
                c.z = (float)j + or_random_float(&rng, -1.0f, 1.0f);
                c.w = 0.0f;
                t1 = (double)len3(c.x - 4.0f, c.y - 0.2f, c.z - 0.0f) > 0.9;
                t2 = (double)len3(c.x - 0.0f, c.y - 0.2f, c.z - 0.0f) > 0.9;
                t3 = (double)len3(c.x - -4.0f, c.y - 0.2f, c.z - 0.0f) > 0.9;
            } while (!t1 || !t2 || !t3);
            or_v3 color = v3s(0, 0, 0);
            float spec = 0.0f, ior = 0.0f;
            if ((double)m < 0.8) {
                color.x = or_random_float(&rng, 0.0f, 1.0f);
                color.y = or_random_float(&rng, 0.0f, 1.0f);
                color.z = or_random_float(&rng, 0.0f, 1.0f);
            } else if ((double)m < 0.95) {
                color.x = or_random_float(&rng, 0.0f, 1.0f);
                color.y = or_random_float(&rng, 0.0f, 1.0f);
                color.z = or_random_float(&rng, 0.0f, 1.0f);
                spec = or_random_float(&rng, 0.5f, 1.0f);
            } else {
                color = v3s(1, 1, 1);
                ior = 1.5f;
            }
            if (idx < cap) create_sphere(c, 0.2f, color, spec, ior, z, sp + idx, 1);
            idx += 1;
        }
    }
    info->look_at = sp[1].pos;
    info->use_sky = 1;
    info->n_spheres = cap;
}

int or_scene_builtin(int index, or_sphere *spheres, or_group *groups, or_material *materials, or_scene_info *info)
{
    memset(info, 0, sizeof(*info));
    if (index == 0) scene_rgb(spheres, info);
    else if (index == 1) scene_floating(spheres, info);
    else if (index == 2) scene_rtweekend(spheres, info);
    else return -1;
    info->n_groups = (info->n_spheres + 3u) / 4u;
    info->n_materials = info->n_spheres + 1u;
    to_groups(spheres, info->n_spheres, groups, materials);
    return 0;
}

/* ---------------------------------------------------------------- camera */

/* main.cpp:776-838.  The orbit clamps of :763-774 are applied by the caller. */
void or_camera_setup(const or_v3 *look_at, float distance, float xangle, float yheight,
                     uint32_t width, uint32_t height, or_camera *out)
{
    memset(out, 0, sizeof(*out));
    float xy0 = x87_cos(xangle) * distance;
    float xy1 = x87_sin(xangle) * distance;
    float pos[3] = {xy0 + look_at->x, yheight + look_at->y, xy1 + look_at->z};
    float zr[3] = {pos[0] - look_at->x, pos[1] - look_at->y, pos[2] - look_at->z};
    float cz[3], cx[3], cy[3], t[3];
    or_normalize(zr, cz);
    const float up[3] = {0.0f, 1.0f, 0.0f};
    cross_fma(up, cz, t);
    or_normalize(t, cx);
    cross_fma(cz, cx, t);
    or_normalize(t, cy);
    out->position = v3s(pos[0], pos[1], pos[2]);
    out->cam_z = v3s(cz[0], cz[1], cz[2]);
    out->cam_x = v3s(cx[0], cx[1], cx[2]);
    out->cam_y = v3s(cy[0], cy[1], cy[2]);
    out->film_center = v3s(pos[0] - cz[0], pos[1] - cz[1], pos[2] - cz[2]);
    out->film_w = 1.0f;
    out->film_h = 1.0f;
    if (width > height) out->film_h = (float)height / (float)width;
    else out->film_w = (float)width / (float)height;
    out->tiles_x = (width + OR_TILE - 1u) / OR_TILE;
}

/* ---------------------------------------------------------------- tracer */

typedef struct trace_ctx {
    const or_group *groups;
    uint32_t n_groups;
    const or_sphere *spheres;
    uint32_t n_spheres;
    const or_material *materials;
    uint32_t use_sky;
    const or_camera *cam;
    uint32_t width, height, max_bounce;
} trace_ctx;

/* main.cpp:292-300 Reflectance; the final a + b*c is one FMA in the
 * reference's -mfma build. */
static float reflectance(float cos_theta, float eta)
{
    float r0 = (1.0f - eta) / (1.0f + eta);
    r0 *= r0;
    float r1 = 1.0f - cos_theta;
    r1 = r1 * r1 * r1 * r1 * r1;
    return fmaf(1.0f - r0, r1, r0);
}

/* main.cpp:375-385: jittered primary ray through the film. */
static void primary_ray(const trace_ctx *c, uint32_t x, uint32_t y, uint64_t *rng, float o[3], float d[3])
{
    const or_camera *cam = c->cam;
    float jx = or_random_float(rng, -0.5f, 0.5f);
    float jy = or_random_float(rng, -0.5f, 0.5f);
    float fx = -1.0f + (((float)x + jx) * 2.0f) / (float)c->width;
    float fy = -1.0f + (((float)y + jy) * 2.0f) / (float)c->height;
    float ax = (fx * cam->film_w) * 0.5f;
    float ay = (fy * cam->film_h) * 0.5f;
    const float *fc = &cam->film_center.x, *cx = &cam->cam_x.x, *cy = &cam->cam_y.x, *cp = &cam->position.x;
    float v[3];
    for (int k = 0; k < 3; ++k) {
        float fp = (fc[k] + ax * cx[k]) + ay * cy[k];
        o[k] = cp[k];
        v[k] = fp - cp[k];
    }
    or_normalize(v, d);
}

/* main.cpp:446-481: emission/attenuation and the bounce direction.
 * hit_n is the un-normalised HitNormal, new_o the next origin. */
static void emit_attenuate(const float emis[3], const float color[3], float att[3], float out[3])
{
    for (int k = 0; k < 3; ++k) out[k] = out[k] + emis[k] * att[k];   /* main.cpp:446 */
    for (int k = 0; k < 3; ++k) att[k] = att[k] * color[k];           /* main.cpp:447 */
}

static void shade(const or_material *m, const float hit_n[3], int inside, uint64_t *rng,
                  float dir[3], float att[3], float out[3])
{
    emit_attenuate(&m->emissive.x, &m->color.x, att, out);
    float n[3];
    or_normalize(hit_n, n);
    float k2 = 2.0f * dot3(dir, n);
    float pb[3];
    for (int k = 0; k < 3; ++k) pb[k] = dir[k] - k2 * n[k];
    if (inside) for (int k = 0; k < 3; ++k) n[k] = -n[k];
    if (m->ior == 0.0f) {
        float r[3], rn[3], nd[3];
        r[0] = or_random_float(rng, -1.0f, 1.0f);
        r[1] = or_random_float(rng, -1.0f, 1.0f);
        r[2] = or_random_float(rng, -1.0f, 1.0f);
        or_normalize_fast(r, rn);
        float s = m->specular;
        float one_minus = 1.0f - s;  /* (1.0 - Specular) in f64 rounds to this f32 */
        for (int k = 0; k < 3; ++k) nd[k] = one_minus * (n[k] + rn[k]) + s * pb[k];
        or_normalize(nd, dir);
    } else {
        float eta = inside ? m->ior : 1.0f / m->ior;
        float nd[3] = {-dir[0], -dir[1], -dir[2]};
        float dd = dot3(nd, n);
        float cos_t = dd < 1.0f ? dd : 1.0f;          /* _mm_min_ss(a, b) */
        float sin_t = sqrtf(1.0f - cos_t * cos_t);     /* f64 1.0 - f32 rounds identically */
        int cant = eta * sin_t > 1.0f;
        float perp[3], par[3], rr[3], refr[3];
        for (int k = 0; k < 3; ++k) perp[k] = eta * (dir[k] + cos_t * n[k]);
        float q = -sqrtf(fabsf(1.0f - dot3(perp, perp)));
        for (int k = 0; k < 3; ++k) par[k] = q * n[k];
        for (int k = 0; k < 3; ++k) rr[k] = perp[k] + par[k];
        or_normalize(rr, refr);
        int refl = cant;
        if (!refl) refl = reflectance(cos_t, eta) > or_random_float(rng, 0.0f, 1.0f);
        if (refl && !inside) memcpy(dir, pb, sizeof(pb));
        else memcpy(dir, refr, sizeof(refr));
    }
}

/* main.cpp:433-440: sky term on a miss. */
static void sky(const trace_ctx *c, const float dir[3], const float att[3], float out[3])
{
    if (!c->use_sky) return;
    float a = (dir[1] + 1.0f) * 0.5f;
    const float k[3] = {0.5f, 0.7f, 1.0f};
    for (int i = 0; i < 3; ++i) {
        float s = (1.0f - a) * 1.0f + a * k[i];
        out[i] = out[i] + s * att[i];
    }
}

/* main.cpp:400-407: per group, C = P - O, T = Dot(C, D), |C - D*T|^2, R*R. */
static inline void group_core(const or_group *sg, __m128 ox, __m128 oy, __m128 oz, __m128 dx, __m128 dy, __m128 dz,
                              __m128 *cx, __m128 *cy, __m128 *cz, __m128 *t, __m128 *dist, __m128 *r2)
{
    *cx = _mm_sub_ps(_mm_loadu_ps(sg->px), ox);
    *cy = _mm_sub_ps(_mm_loadu_ps(sg->py), oy);
    *cz = _mm_sub_ps(_mm_loadu_ps(sg->pz), oz);
    *t = _mm_add_ps(_mm_add_ps(_mm_mul_ps(*cx, dx), _mm_mul_ps(*cy, dy)), _mm_mul_ps(*cz, dz));
    __m128 qx = _mm_sub_ps(*cx, _mm_mul_ps(dx, *t));
    __m128 qy = _mm_sub_ps(*cy, _mm_mul_ps(dy, *t));
    __m128 qz = _mm_sub_ps(*cz, _mm_mul_ps(dz, *t));
    *dist = _mm_add_ps(_mm_add_ps(_mm_mul_ps(qx, qx), _mm_mul_ps(qy, qy)), _mm_mul_ps(qz, qz));
    __m128 r = _mm_loadu_ps(sg->r);
    *r2 = _mm_mul_ps(r, r);
}

/* main.cpp:413-417: X = sqrt(R^2 - d), t = T - X, or T + X when t < eps. */
static inline __m128 group_hit_t(__m128 t, __m128 dist, __m128 r2, __m128 *itest)
{
    __m128 xx = _mm_sqrt_ps(_mm_sub_ps(r2, dist));
    __m128 it = _mm_sub_ps(t, xx);
    *itest = _mm_cmplt_ps(it, _mm_set1_ps(OR_EPS));
    return _mm_blendv_ps(it, _mm_add_ps(t, xx), *itest);
}

/* x64_math.h:579-585 HorizontalMin, then the lowest lane holding it
 * (FindFirstIndex, wasm_math.h:286-291 semantics). */
static inline uint32_t lane_select(__m128 min_t, float *m_out)
{
    __m128 m = _mm_min_ps(min_t, _mm_movehl_ps(min_t, min_t));
    m = _mm_min_ps(m, _mm_shuffle_ps(m, m, 0x11));
    float mv = _mm_cvtss_f32(m);
    *m_out = mv;
    int mask = _mm_movemask_ps(_mm_cmpeq_ps(min_t, _mm_set1_ps(mv)));
    return mask ? (uint32_t)__builtin_ctz((unsigned)mask) : 0u;
}

/* Exported for tests: the lane-4 group arithmetic and selection above. */
void or_group_test(const float o[3], const float d[3], const or_group *g, float dist_out[4], float t_out[4])
{
    __m128 cx, cy, cz, t, dist, r2, itest;
    group_core(g, _mm_set1_ps(o[0]), _mm_set1_ps(o[1]), _mm_set1_ps(o[2]), _mm_set1_ps(d[0]), _mm_set1_ps(d[1]),
               _mm_set1_ps(d[2]), &cx, &cy, &cz, &t, &dist, &r2);
    _mm_storeu_ps(dist_out, dist);
    _mm_storeu_ps(t_out, group_hit_t(t, dist, r2, &itest));
}

float or_horizontal_min(const float v[4], uint32_t *lane)
{
    float m;
    *lane = lane_select(_mm_loadu_ps(v), &m);
    return m;
}

void or_cross(const float a[3], const float b[3], float out[3]) { cross_fma(a, b, out); }

/* One sample with RenderTile lane-4 rules (main.cpp:375-482). */
static void trace_simd(const trace_ctx *c, uint32_t x, uint32_t y, uint64_t *rng, float out[3], uint64_t *rays)
{
    float o[3], d[3], att[3] = {1, 1, 1};
    out[0] = out[1] = out[2] = 0.0f;
    primary_ray(c, x, y, rng, o, d);
    for (uint32_t b = 0; b < c->max_bounce; ++b) {
        *rays += 1;
        __m128 ox = _mm_set1_ps(o[0]), oy = _mm_set1_ps(o[1]), oz = _mm_set1_ps(o[2]);
        __m128 dx = _mm_set1_ps(d[0]), dy = _mm_set1_ps(d[1]), dz = _mm_set1_ps(d[2]);
        __m128 hnx = _mm_setzero_ps(), hny = hnx, hnz = hnx, nox = hnx, noy = hnx, noz = hnx;
        __m128 min_t = _mm_set1_ps(OR_FMAX);
        __m128i grp = _mm_setzero_si128();
        __m128 inside = _mm_setzero_ps();
#pragma clang loop unroll_count(2)  /* as main.cpp:398 */
        for (uint32_t g = 0; g < c->n_groups; ++g) {
            __m128 cx, cy, cz, t, dist, r2;
            group_core(&c->groups[g], ox, oy, oz, dx, dy, dz, &cx, &cy, &cz, &t, &dist, &r2);
            __m128 hit = _mm_cmplt_ps(dist, r2);
            if (_mm_movemask_ps(hit) == 0) continue;
            __m128 itest, it = group_hit_t(t, dist, r2, &itest);
            __m128 mv = _mm_and_ps(_mm_and_ps(_mm_cmplt_ps(it, min_t), _mm_cmpgt_ps(it, _mm_set1_ps(OR_EPS))), hit);
            if (_mm_movemask_ps(mv) == 0) continue;
            __m128 ipx = _mm_mul_ps(dx, it), ipy = _mm_mul_ps(dy, it), ipz = _mm_mul_ps(dz, it);
            inside = _mm_or_ps(inside, _mm_and_ps(itest, mv));                 /* sticky, main.cpp:425 */
            grp = _mm_castps_si128(_mm_blendv_ps(_mm_castsi128_ps(grp), _mm_castsi128_ps(_mm_set1_epi32((int)g)), mv));
            min_t = _mm_blendv_ps(min_t, it, mv);
            hnx = _mm_blendv_ps(hnx, _mm_sub_ps(ipx, cx), mv);
            hny = _mm_blendv_ps(hny, _mm_sub_ps(ipy, cy), mv);
            hnz = _mm_blendv_ps(hnz, _mm_sub_ps(ipz, cz), mv);
            nox = _mm_blendv_ps(nox, _mm_add_ps(ox, ipx), mv);
            noy = _mm_blendv_ps(noy, _mm_add_ps(oy, ipy), mv);
            noz = _mm_blendv_ps(noz, _mm_add_ps(oz, ipz), mv);
        }
        float mv;
        uint32_t lane = lane_select(min_t, &mv);
        if (mv == OR_FMAX) {
            sky(c, d, att, out);
            break;
        }
        float lt[4], hx[4], hy[4], hz[4], nx[4], ny[4], nz[4], in4[4];
        uint32_t g4[4];
        _mm_storeu_ps(lt, min_t);
        _mm_storeu_ps(hx, hnx); _mm_storeu_ps(hy, hny); _mm_storeu_ps(hz, hnz);
        _mm_storeu_ps(nx, nox); _mm_storeu_ps(ny, noy); _mm_storeu_ps(nz, noz);
        _mm_storeu_ps(in4, inside);
        _mm_storeu_si128((__m128i *)g4, grp);
        uint32_t sidx = g4[lane] * 4u + lane;
        const or_material *mat = &c->materials[sidx];
        float hn[3] = {hx[lane], hy[lane], hz[lane]};
        int ins = f2u(in4[lane]) != 0;
        o[0] = nx[lane]; o[1] = ny[lane]; o[2] = nz[lane];
        shade(mat, hn, ins, rng, d, att, out);
    }
}

/* One sample with RenderTileScalar rules (main.cpp:524-627). */
static void trace_scalar(const trace_ctx *c, uint32_t x, uint32_t y, uint64_t *rng, float out[3], uint64_t *rays)
{
    float o[3], d[3], att[3] = {1, 1, 1};
    out[0] = out[1] = out[2] = 0.0f;
    primary_ray(c, x, y, rng, o, d);
    for (uint32_t b = 0; b < c->max_bounce; ++b) {
        *rays += 1;
        float hn[3] = {0, 0, 0}, no[3] = {0, 0, 0}, min_t = OR_FMAX;
        uint32_t sidx = 0;
        int ins = 0;
        for (uint32_t s = 0; s < c->n_spheres; ++s) {
            const or_sphere *sp = &c->spheres[s];
            float cc[3] = {sp->pos.x - o[0], sp->pos.y - o[1], sp->pos.z - o[2]};
            float t = dot3(cc, d);
            float q[3] = {cc[0] - d[0] * t, cc[1] - d[1] * t, cc[2] - d[2] * t};
            float r2 = sp->radius * sp->radius;
            float dist = dot3(q, q);
            if (dist > r2) continue;
            float xx = sqrtf(r2 - dist);
            float it = t - xx;
            int itest = it < OR_EPS;
            if (itest) it = t + xx;
            if (it > min_t) continue;
            if (it < OR_EPS) continue;
            float ip[3] = {d[0] * it, d[1] * it, d[2] * it};
            ins = itest;
            sidx = s;
            min_t = it;
            for (int k = 0; k < 3; ++k) { hn[k] = ip[k] - cc[k]; no[k] = o[k] + ip[k]; }
        }
        if (min_t == OR_FMAX) {
            sky(c, d, att, out);
            break;
        }
        const or_material *mat = &c->spheres[sidx].mat;
        memcpy(o, no, sizeof(no));
        shade(mat, hn, ins, rng, d, att, out);
    }
}

/* main.cpp:312-346: LinearToSRGB ("sqrt" variant) + ColorFromV4. */
static float saturate(float v) { if (v < 0.0f) return 0.0f; if (v > 1.0f) return 1.0f; return v; }
static uint32_t to_u8(float v)
{
    float s = saturate(v) * 255.0f;
    if (s != s) return 0u;  /* cvttss2si(NaN) = 0x80000000 -> low byte 0 */
    return (uint32_t)(int32_t)s & 0xFFu;
}
static float srgb(float l)
{
    l = saturate(l);
    return l < 0.0031308f ? l * 12.92f : sqrtf(l);
}

/* main.cpp:320-321: the exact-pow branch ('#if 0' in the reference), as the
 * WASM build would compile it: libm powf (musl there, glibc here -- the same
 * algorithm), unfused (wasm32 has no FMA). */
static float srgb_pow(float l)
{
    l = saturate(l);
    return l < 0.0031308f ? l * 12.92f : 1.055f * powf(l, 1.0f / 2.4f) - 0.055f;
}

void or_encode_rgba8(const float *v4, uint32_t *rgba, uint64_t n, int pow_mode)
{
    for (uint64_t i = 0; i < n; ++i) {
        const float *f = v4 + 4 * i;
        rgba[i] = pow_mode ? to_u8(srgb_pow(f[0])) | (to_u8(srgb_pow(f[1])) << 8) | (to_u8(srgb_pow(f[2])) << 16) | (255u << 24)
                           : to_u8(srgb(f[0])) | (to_u8(srgb(f[1])) << 8) | (to_u8(srgb(f[2])) << 16) | (255u << 24);
    }
}

float or_srgb_channel(float l, int pow_mode) { return pow_mode ? srgb_pow(l) : srgb(l); }

/* main.cpp:484-492: running-mean blend and the RGBA8 store. */
static void blend_store(uint32_t prev_count, const float out[3], float *prev4, uint32_t *px)
{
    uint32_t total = prev_count + 1u;
    float inv = 1.0f / (float)total;
    float ratio = (float)prev_count / (float)total;
    float f[3];
    for (int k = 0; k < 3; ++k) f[k] = out[k] * inv + prev4[k] * ratio;
    prev4[0] = f[0]; prev4[1] = f[1]; prev4[2] = f[2]; prev4[3] = 1.0f;
    *px = to_u8(srgb(f[0])) | (to_u8(srgb(f[1])) << 8) | (to_u8(srgb(f[2])) << 16) | (255u << 24);
}

/* ----------------------------------------------------------- tile queue */

typedef struct job {
    trace_ctx ctx;
    uint32_t prev_count, frames, simd, seed_mode;
    uint32_t row_begin, row_end, tiles_x, tile_y0, n_tiles;
    uint64_t *stream_states;
    float *prev_v4;
    uint32_t *cur;
    uint32_t frame;          /* stream mode: current frame */
    volatile uint32_t next;  /* atomic tile counter (wasm/wasm.cpp:630,641) */
    uint64_t rays[256];
} job;

typedef struct worker { job *j; uint32_t index; } worker;

static void render_tile(job *j, uint32_t tile, uint32_t ti, uint32_t frame_lo, uint32_t frame_hi)
{
    const trace_ctx *c = &j->ctx;
    uint32_t tx = tile % j->tiles_x, ty = j->tile_y0 + tile / j->tiles_x;
    uint32_t top = ty * OR_TILE, left = tx * OR_TILE;
    uint32_t bottom = top + OR_TILE, right = left + OR_TILE;
    if (bottom > c->height) bottom = c->height;
    if (right > c->width) right = c->width;
    if (top < j->row_begin) top = j->row_begin;
    if (bottom > j->row_end) bottom = j->row_end;
    uint64_t rays = 0;
    for (uint32_t f = frame_lo; f < frame_hi; ++f) {
        uint32_t pc = j->prev_count + f;
        for (uint32_t y = top; y < bottom; ++y) {
            for (uint32_t x = left; x < right; ++x) {
                uint64_t pix_rng, *rng;
                if (j->seed_mode == OR_SEED_PIXEL) {
                    pix_rng = or_seed_mix(((uint64_t)pc * c->height + y) * c->width + x);
                    rng = &pix_rng;
                } else {
                    rng = &j->stream_states[ti];
                }
                float out[3];
                if (j->simd) trace_simd(c, x, y, rng, out, &rays);
                else trace_scalar(c, x, y, rng, out, &rays);
                size_t p = (size_t)y * c->width + x;
                blend_store(pc, out, j->prev_v4 + 4 * p, j->cur + p);
            }
        }
    }
    j->rays[ti] += rays;
}

static void *worker_main(void *arg)
{
    worker *w = (worker *)arg;
    job *j = w->j;
    for (;;) {
        uint32_t t = __atomic_fetch_add(&j->next, 1u, __ATOMIC_RELAXED);
        if (t >= j->n_tiles) break;
        if (j->seed_mode == OR_SEED_PIXEL) render_tile(j, t, w->index, 0, j->frames);
        else render_tile(j, t, w->index, j->frame, j->frame + 1);
    }
    return NULL;
}

static void run_pool(job *j, uint32_t threads)
{
    j->next = 0;
    if (threads <= 1) {
        worker w = {j, 0};
        worker_main(&w);
        return;
    }
    pthread_t th[256];
    worker ws[256];
    for (uint32_t i = 0; i < threads; ++i) {
        ws[i].j = j;
        ws[i].index = i;
        pthread_create(&th[i], NULL, worker_main, &ws[i]);
    }
    for (uint32_t i = 0; i < threads; ++i) pthread_join(th[i], NULL);
}

int or_render(const or_group *groups, uint32_t n_groups,
              const or_sphere *spheres, uint32_t n_spheres,
              const or_material *materials, uint32_t use_sky,
              const or_camera *cam, uint32_t width, uint32_t height,
              uint32_t prev_count, uint32_t frames, uint32_t max_bounce,
              int simd, int seed_mode, uint32_t threads, uint64_t *stream_states,
              uint32_t row_begin, uint32_t row_end,
              float *prev_v4, uint32_t *cur_rgba, uint64_t *rays_out)
{
    if (!cam || !prev_v4 || !cur_rgba || width == 0 || height == 0) return -22;
    if (threads == 0) threads = 1;
    if (threads > 256) threads = 256;
    if (seed_mode == OR_SEED_STREAM && !stream_states) return -22;
    if (row_end == 0 || row_end > height) row_end = height;
    if (row_begin >= row_end) { if (rays_out) *rays_out = 0; return 0; }
    job *j = (job *)calloc(1, sizeof(job));
    if (!j) return -12;
    j->ctx.groups = groups;
    j->ctx.n_groups = n_groups;
    j->ctx.spheres = spheres;
    j->ctx.n_spheres = n_spheres;
    j->ctx.materials = materials;
    j->ctx.use_sky = use_sky;
    j->ctx.cam = cam;
    j->ctx.width = width;
    j->ctx.height = height;
    j->ctx.max_bounce = max_bounce;
    j->prev_count = prev_count;
    j->frames = frames;
    j->simd = simd ? 1u : 0u;
    j->seed_mode = (uint32_t)seed_mode;
    j->row_begin = row_begin;
    j->row_end = row_end;
    j->tiles_x = (width + OR_TILE - 1u) / OR_TILE;
    j->tile_y0 = row_begin / OR_TILE;
    j->n_tiles = j->tiles_x * ((row_end + OR_TILE - 1u) / OR_TILE - j->tile_y0);
    j->stream_states = stream_states;
    j->prev_v4 = prev_v4;
    j->cur = cur_rgba;
    if (seed_mode == OR_SEED_PIXEL) {
        run_pool(j, threads);
    } else {
        for (uint32_t f = 0; f < frames; ++f) {
            j->frame = f;
            run_pool(j, threads);
        }
    }
    uint64_t total = 0;
    for (uint32_t i = 0; i < threads; ++i) total += j->rays[i];
    if (rays_out) *rays_out = total;
    free(j);
    return 0;
}

uint64_t or_fnv1a64(const void *data, uint64_t nbytes)
{
    const uint8_t *p = (const uint8_t *)data;
    uint64_t h = 0xcbf29ce484222325ULL;
    for (uint64_t i = 0; i < nbytes; ++i) { h ^= p[i]; h *= 0x100000001b3ULL; }
    return h;
}

/* Exported pieces of the colour path, for differential tests against the
 * reference's own compiled main.cpp lines (oracle/_ref/librefmath.so). */
float or_reflectance(float cos_theta, float eta) { return reflectance(cos_theta, eta); }
void or_blend_store(uint32_t prev_count, const float out3[3], float prev4[4], uint32_t *px)
{
    blend_store(prev_count, out3, prev4, px);
}
void or_emit_attenuate(const float emis[3], const float color[3], float att[3], float out[3])
{
    emit_attenuate(emis, color, att, out);
}
void or_srgb_n(const float *in, float *out, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) out[i] = srgb(in[i]);
}
