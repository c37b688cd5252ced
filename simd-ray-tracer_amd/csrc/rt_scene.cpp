// rt_scene.cpp — host-side inputs of the trace path: the three built-in
// scenes, scene prefixes, the orbit camera and the pixel seed.
//
// Compiled with -ffp-contract=off; the two contractions the reference's
// clang -mfma build performs in this code (v3::Cross in the camera basis,
// x64_math.h:258-264) are written as explicit fmaf.
#include <math.h>
#include <mutex>
#include <string.h>

#include "rt_trace.h"

namespace {

constexpr float kWorldScale = 0.0625f;                 // main.cpp:56 (1.0 / 16.0f)
constexpr float kPi32 = 3.14159265358979323846f;       // base.h:892
constexpr float kEps = 1e-4f;                          // base.h:889

struct Rng {  // u32_random_state, base.h:951-997
    uint64_t seed;
    uint32_t next() {
        const uint64_t old = seed;
        seed = old * 6364136223846793005ULL + 1442695040888963407ULL;
        const uint32_t v = (uint32_t)(old >> 32) ^ (uint32_t)old;
        const uint32_t r = (uint32_t)(old >> 59);
        return (v >> r) | (v << ((32u - r) & 31u));
    }
    float uniform(float lo = -1.0f, float hi = 1.0f) {
        const uint32_t n = next();
        const float inv = (float)((double)(hi - lo) / 4294967295.0);
        const float r = (float)n * inv;
        return r + lo;
    }
};

rt_v3 V(float x, float y, float z) {
    rt_v3 v;
    v.x = x;
    v.y = y;
    v.z = z;
    v._w = 0.0f;
    return v;
}

float dot(const rt_v3 &a, const rt_v3 &b) {
    const float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
    return (px + py) + pz;
}

rt_v3 normalize(const rt_v3 &v) {  // x64_math.h:234-245
    const float l2 = dot(v, v);
    if (!(l2 > kEps)) return V(0.0f, 0.0f, 0.0f);
    const float len = sqrtf(l2);
    return V(v.x / len, v.y / len, v.z / len);
}

rt_v3 cross_mfma(const rt_v3 &a, const rt_v3 &b) {  // x64_math.h:258-264 under -mfma
    return V(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}

float x87_cos(float x) {  // x64_math.h:728-736
    long double r = x;
    __asm__("fcos" : "+t"(r));
    return (float)r;
}
float x87_sin(float x) {  // x64_math.h:738-746
    long double r = x;
    __asm__("fsin" : "+t"(r));
    return (float)r;
}

// CreateScalarSphere, main.cpp:57-71.
void make_sphere(rt_v3 pos, float radius, rt_v3 color, float specular, float ior, rt_v3 emissive,
                 rt_scalar_sphere *s, bool world_scale) {
    memset(s, 0, sizeof(*s));
    if (world_scale) {
        s->Position = V(pos.x * kWorldScale, pos.y * kWorldScale, pos.z * kWorldScale);
        s->Radius = radius * kWorldScale;
    } else {
        s->Position = pos;
        s->Radius = radius;
    }
    s->Material.Color = color;
    s->Material.Specular = specular;
    s->Material.Emissive = emissive;
    s->Material.IndexOfRefraction = ior;
}

// ConvertScalarSpheresToSIMDSpheres, main.cpp:73-91 (padding lanes zero).
void to_simd(const rt_scalar_sphere *s, uint32_t n, rt_sphere_group *g, rt_material *m) {
    const uint32_t ng = (n + 3u) / 4u;
    memset(g, 0, ng * sizeof(*g));
    memset(m, 0, (n + 1u) * sizeof(*m));
    for (uint32_t i = 0; i < n; ++i) {
        rt_sphere_group &G = g[i / 4u];
        G.X[i % 4u] = s[i].Position.x;
        G.Y[i % 4u] = s[i].Position.y;
        G.Z[i % 4u] = s[i].Position.z;
        G.Radii[i % 4u] = s[i].Radius;
        m[i] = s[i].Material;
    }
}

struct Storage {
    rt_scalar_sphere rgb[5];
    rt_sphere_group rgb_g[2];
    rt_material rgb_m[6];
    rt_scalar_sphere flt[256];
    rt_sphere_group flt_g[64];
    rt_material flt_m[257];
    rt_scalar_sphere rtw[482];
    rt_sphere_group rtw_g[121];
    rt_material rtw_m[483];
    rt_scene scenes[3];
};
Storage g_store;
std::once_flag g_once;

void set_arrays(rt_scene *sc, rt_scalar_sphere *s, uint32_t n, rt_sphere_group *g, rt_material *m) {
    sc->ScalarSpheres.Data = s;
    sc->ScalarSpheres.Count = n;
    sc->SIMDSpheres.Data = g;
    sc->SIMDSpheres.Count = (n + 3u) / 4u;
    sc->Materials.Data = m;
    sc->Materials.Count = n + 1u;
}

// InitRGBSphereScene, main.cpp:171-191.
void init_rgb(rt_scene *sc) {
    rt_scalar_sphere *s = g_store.rgb;
    const rt_v3 zero = V(0, 0, 0);
    sc->DefaultDistanceFromLookAt = 16.0f * kWorldScale;
    sc->DefaultXAngle = (float)((double)kPi32 / 3.0);
    sc->DefaultYHeight = 4.0f * kWorldScale;
    make_sphere(V(0.0f, -256 - 2.0f, -15.0f), 256.0f, V(0.2f, 0.2f, 0.2f), 0.0f, 0.0f, zero, s + 0, true);
    make_sphere(V(0.0f, 0.0f, -10.0f), 2.0f, V(1, 1, 1), 0.0f, 1.5f, zero, s + 1, true);
    make_sphere(V(-4.0f, 1.0f, -15.0f), 1.5f, V(1, 0, 0), 0.0f, 0.0f, V(8, 0, 0), s + 2, true);
    make_sphere(V(0.0f, 1.0f, -15.0f), 1.5f, V(1, 0, 0), 0.0f, 0.0f, V(0, 8, 0), s + 3, true);
    make_sphere(V(4.0f, 1.0f, -15.0f), 1.5f, V(1, 0, 0), 0.0f, 0.0f, V(0, 0, 8), s + 4, true);
    to_simd(s, 5, g_store.rgb_g, g_store.rgb_m);
    set_arrays(sc, s, 5, g_store.rgb_g, g_store.rgb_m);
    sc->LookAt = s[1].Position;
    sc->UseSkyColor = false;
}

// InitRandomizedSphereScene ("Floating Spheres"), main.cpp:96-167.
void init_floating(rt_scene *sc) {
    rt_scalar_sphere *s = g_store.flt;
    const uint32_t n = 256;
    sc->DefaultDistanceFromLookAt = 48.0f * kWorldScale;
    sc->DefaultXAngle = (float)((double)(kPi32 * 2.65f) / 2.0);
    sc->DefaultYHeight = 0.0f;
    Rng rng{0x29D7A0A514F22432ULL};
    rt_material pal[28];
    for (uint32_t i = 0; i < 28; ++i) {
        rt_v3 color = V(0, 0, 0), emissive = V(0, 0, 0);
        float specular = 0.0f;
        color.x = rng.uniform(0.15f, 1.0f);
        color.y = rng.uniform(0.1f, 0.75f);
        color.z = rng.uniform(0.15f, 1.0f);
        if (rng.uniform(0.0f) < 0.125f) {
            const float k = rng.uniform(2.0f, 5.0f);
            emissive = V(k * color.x, k * color.y, k * color.z);
        } else if (rng.uniform(0.0f) < 0.65f) {
            specular = 1.0f;
        }
        memset(&pal[i], 0, sizeof(pal[i]));
        pal[i].Color = color;
        pal[i].Emissive = emissive;
        pal[i].Specular = specular;
        pal[i].IndexOfRefraction = 0.0f;
    }
    const float r0 = rng.uniform(2.0f, 8.0f);
    const rt_material &m0 = pal[0];
    make_sphere(V(1, 0, 0), r0, m0.Color, m0.Specular, m0.IndexOfRefraction, m0.Emissive, s + 0, false);
    make_sphere(V(8, -1, 8), r0, m0.Color, m0.Specular, m0.IndexOfRefraction, m0.Emissive, s + 1, false);
    make_sphere(V(-20, -4, -20), r0, m0.Color, m0.Specular, m0.IndexOfRefraction, m0.Emissive, s + 2, false);
    for (uint32_t i = 3; i < n; ++i) {
        rt_v3 dir = V(0, 0, 0);
        dir.x = rng.uniform();
        dir.y = rng.uniform();
        dir.z = rng.uniform();
        dir = normalize(dir);
        const rt_scalar_sphere &anchor = s[i - 3];
        const float radius = rng.uniform(1.0f, 4.0f);
        const float dist = (rng.uniform(1.0f, 8.0f) + radius) + anchor.Radius;
        const rt_v3 pos = V(anchor.Position.x + dir.x * dist, anchor.Position.y + dir.y * dist,
                            anchor.Position.z + dir.z * dist);
        const rt_material &m = pal[i % 28u];
        make_sphere(pos, radius, m.Color, m.Specular, m.IndexOfRefraction, m.Emissive, s + i, false);
    }
    for (uint32_t i = 0; i < n; ++i) {
        s[i].Radius *= kWorldScale;
        s[i].Position.x *= kWorldScale;
        s[i].Position.y *= kWorldScale;
        s[i].Position.z *= kWorldScale;
    }
    to_simd(s, n, g_store.flt_g, g_store.flt_m);
    set_arrays(sc, s, n, g_store.flt_g, g_store.flt_m);
    sc->LookAt = V(2.0f * kWorldScale, 0.0f, 2.0f * kWorldScale);
    sc->UseSkyColor = false;
}

float length3(float x, float y, float z) {
    const rt_v3 v = V(x, y, z);
    return sqrtf(dot(v, v));
}

// InitRTWeekendSphereScene, main.cpp:196-268.  The reference writes 488
// spheres into a 482-entry array; only the first 482 are part of the scene.
void init_rtweekend(rt_scene *sc) {
    rt_scalar_sphere *s = g_store.rtw;
    const uint32_t cap = 482;
    const rt_v3 zero = V(0, 0, 0);
    sc->DefaultDistanceFromLookAt = 12.0f * kWorldScale;
    sc->DefaultXAngle = kPi32 / 8;
    sc->DefaultYHeight = 2.0f * kWorldScale;
    uint32_t idx = 0;
    make_sphere(V(0, -1000, 0), 1000, V(0.5f, 0.5f, 0.5f), 0.0f, 0.0f, zero, s + idx++, true);
    make_sphere(V(0, 1, 0), 1, V(1, 1, 1), 0.0f, 1.5f, zero, s + idx++, true);
    make_sphere(V(-4, 1, 0), 1, V(0.4f, 0.2f, 0.1f), 0.0f, 0.0f, zero, s + idx++, true);
    make_sphere(V(4, 1, 0), 1, V(0.7f, 0.6f, 0.5f), 1.0f, 0.0f, zero, s + idx++, true);
    Rng rng{0xCD46749A57ACB371ULL};
    for (int32_t i = -11; i < 11; ++i) {
        for (int32_t j = -11; j < 11; ++j) {
            const float choose = rng.uniform(0.0f, 1.0f);
            rt_v3 c = V(0, 0, 0);
            bool clear;
            do {
                c.x = (float)i + rng.uniform();
                c.y = 0.2f;
                c.z = (float)j + rng.uniform();
                clear = (double)length3(c.x - 4.0f, c.y - 0.2f, c.z - 0.0f) > 0.9 &&
                        (double)length3(c.x - 0.0f, c.y - 0.2f, c.z - 0.0f) > 0.9 &&
                        (double)length3(c.x + 4.0f, c.y - 0.2f, c.z - 0.0f) > 0.9;
            } while (!clear);
            rt_v3 color = V(0, 0, 0);
            float specular = 0.0f, ior = 0.0f;
            if ((double)choose < 0.8) {
                color.x = rng.uniform(0.0f, 1.0f);
                color.y = rng.uniform(0.0f, 1.0f);
                color.z = rng.uniform(0.0f, 1.0f);
            } else if ((double)choose < 0.95) {
                color.x = rng.uniform(0.0f, 1.0f);
                color.y = rng.uniform(0.0f, 1.0f);
                color.z = rng.uniform(0.0f, 1.0f);
                specular = rng.uniform(0.5f, 1.0f);
            } else {
                color = V(1, 1, 1);
                ior = 1.5f;
            }
            if (idx < cap) make_sphere(c, 0.2f, color, specular, ior, zero, s + idx, true);
            idx += 1;
        }
    }
    to_simd(s, cap, g_store.rtw_g, g_store.rtw_m);
    set_arrays(sc, s, cap, g_store.rtw_g, g_store.rtw_m);
    sc->LookAt = s[1].Position;
    sc->UseSkyColor = true;
}

void init_all() {
    memset(&g_store, 0, sizeof(g_store));
    init_rgb(&g_store.scenes[0]);
    init_floating(&g_store.scenes[1]);
    init_rtweekend(&g_store.scenes[2]);
}

}  // namespace

static_assert(sizeof(rt_v3) == 16, "v3 is 16 B (base.h:357-375)");
static_assert(sizeof(rt_material) == 48, "material is 48 B");
static_assert(offsetof(rt_material, Specular) == 32 && offsetof(rt_material, IndexOfRefraction) == 36, "material");
static_assert(sizeof(rt_scalar_sphere) == 80 && offsetof(rt_scalar_sphere, Material) == 32, "scalar_sphere");
static_assert(sizeof(rt_sphere_group) == 64, "sphere_group (SIMD_WIDTH 4)");
static_assert(sizeof(rt_array) == 16, "array<T>");
static_assert(sizeof(rt_scene) == 80 && offsetof(rt_scene, UseSkyColor) == 16 &&
                  offsetof(rt_scene, ScalarSpheres) == 32 && offsetof(rt_scene, SIMDSpheres) == 48 &&
                  offsetof(rt_scene, Materials) == 64,
              "scene");
static_assert(sizeof(rt_image) == 24, "image");
static_assert(sizeof(rt_camera_info) == 144 && offsetof(rt_camera_info, FilmW) == 80 &&
                  offsetof(rt_camera_info, TilesX) == 88 && offsetof(rt_camera_info, CurrentImage) == 96 &&
                  offsetof(rt_camera_info, PreviousImage) == 120,
              "camera_info");
static_assert(sizeof(rt_render_params) == 12, "render_params");

extern "C" int rt_scene_builtin(uint32_t index, rt_scene *out) {
    if (!out || index > 2) return RT_EINVAL;
    std::call_once(g_once, init_all);
    *out = g_store.scenes[index];
    return RT_OK;
}

extern "C" int rt_scene_prefix(const rt_scene *in, uint32_t n, rt_scene *out) {
    if (!in || !out || n == 0 || n > in->ScalarSpheres.Count) return RT_EINVAL;
    *out = *in;
    out->ScalarSpheres.Count = n;
    out->SIMDSpheres.Count = (n + 3u) / 4u;
    out->Materials.Count = n + 1u;
    return RT_OK;
}

extern "C" int rt_camera_setup(const rt_scene *scene, float distance, float x_angle, float y_height, uint32_t width,
                               uint32_t height, rt_camera_info *out) {
    if (!scene || !out || width == 0 || height == 0) return RT_EINVAL;
    memset(out, 0, sizeof(*out));
    const rt_v3 look = scene->LookAt;
    // main.cpp:776-780: v2(Cosine, Sin) * Distance, then += LookAt
    const float px = x87_cos(x_angle) * distance;
    const float pz = x87_sin(x_angle) * distance;
    const rt_v3 pos = V(px + look.x, y_height + look.y, pz + look.z);
    const rt_v3 cz = normalize(V(pos.x - look.x, pos.y - look.y, pos.z - look.z));  // main.cpp:811-813
    const rt_v3 cx = normalize(cross_mfma(V(0.0f, 1.0f, 0.0f), cz));
    const rt_v3 cy = normalize(cross_mfma(cz, cx));
    out->CameraPosition = pos;
    out->CameraZ = cz;
    out->CameraX = cx;
    out->CameraY = cy;
    out->FilmCenter = V(pos.x - cz.x, pos.y - cz.y, pos.z - cz.z);  // :814
    out->FilmW = 1.0f;                                              // :816-822
    out->FilmH = 1.0f;
    if (width > height) out->FilmH = (float)height / (float)width;
    else out->FilmW = (float)width / (float)height;
    out->TilesX = (width + 31u) / 32u;  // :824-827
    return RT_OK;
}

extern "C" uint64_t rt_pixel_seed(uint32_t x, uint32_t y, uint32_t frame, uint32_t width, uint32_t height) {
    const uint64_t i = ((uint64_t)frame * height + y) * width + x;
    uint64_t s = 0x420247153476526ULL * i;  // main.cpp:668-675
    s += 0x8442885C91A5C8DULL;
    s ^= s >> ((7u + i) % 64u);
    s ^= s << 23;
    s ^= s >> ((0x29u ^ i) % 64u);
    s = (s * 0x11C19226CEB4769AULL) + 0x1105404122082911ULL;
    s ^= s << 19;
    s ^= s >> 13;
    return s;
}

extern "C" uint32_t rt_band_local_rows(uint32_t height, uint32_t band_rows, uint32_t band_count, uint32_t band_index) {
    if (band_rows == 0 || band_count == 0 || band_index >= band_count) return 0;
    const uint32_t bands = (height + band_rows - 1u) / band_rows;
    uint32_t rows = 0;
    for (uint32_t b = band_index; b < bands; b += band_count) {
        const uint32_t top = b * band_rows;
        rows += (height - top < band_rows) ? height - top : band_rows;
    }
    return rows;
}
