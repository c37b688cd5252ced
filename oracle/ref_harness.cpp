// ORACLE test harness (test infrastructure only).  Builds the reference's own
// code -- /root/reference/base.h + x64_math.h, and main.cpp lines 7-640 (the
// scene types and generators, camera_info, Reflectance, LinearToSRGB,
// ColorFromV4, RenderTile and RenderTileScalar) -- from where it lies, and
// exposes it through extern "C" so tests can check the oracle's restatement
// against the real thing.  Nothing here is shipped or used by the product.
//
// oracle/Makefile extracts the main.cpp line ranges into oracle/_ref/*.inc at
// build time (never committed) and checks that each range still starts and
// ends where this file expects.  main.cpp as a whole is not compiled: line 5
// includes <emscripten/atomic.h>, which this image lacks, and lines 642-859
// (OnInit/OnRender) need the platform layer.  Lines 1-6 and 641-859 are the
// only parts left out; lines 7-640 need nothing but base.h.
#include "base.h"

// main.cpp's RenderTile calls three lane helpers that base.h declares
// (f32x4::FindFirstIndex / f32x4::Extract, base.h:503-504; u32x4::Extract,
// base.h:546) but the x64 layer never defines -- only the WASM layer does
// (wasm_math.h:286-323), so the reference's own x64 build of RenderTile does
// not link.  They are defined here with the WASM layer's semantics: the lowest
// lane equal to Value (ctz of the compare mask), and a lane read.  These are
// the only lines of the SIMD render path that are not the reference's text;
// RenderTileScalar needs none of them.
inline u32 f32x4::FindFirstIndex(const f32x4 &A, f32 Value) {
    for (u32 i = 0; i < 4; ++i)
        if (A[i] == Value) return i;
    return 0;  // unreachable on the path: Value is HorizontalMin(A) and not NaN
}
inline f32 f32x4::Extract(u32 Index) { return (*this)[Index]; }
inline u32 u32x4::Extract(u32 Index) { return (*this)[Index]; }

#ifndef RT_REF_PATCHED
#include "_ref/main_7_640.inc"   // main.cpp:7-640, verbatim
#else
// librefpix.so: the same lines with SURVEY §8c's two textual patches
// (oracle/Makefile, _ref/main_7_640_px.inc): MaxRayBounce = RtMaxRayBounce at
// main.cpp:387,536, and RT_PIXEL_SEED_HOOK(x, y) at the top of the pixel loops
// (main.cpp:373,522).  With RtMaxRayBounce 5 and RtPixelSeeds 0 this build is
// the verbatim one.  The pixel seed is OnInit's own mixer (main.cpp:668-675,
// extracted verbatim) applied to i = (PreviousRayCount*H + y)*W + x, i.e.
// SURVEY §8c's `pixel` seed mode; i is 64-bit (C3's index passes 2^32).
static u32 RtMaxRayBounce = 5;
static int RtPixelSeeds = 0;
static u64 RtSeedMix(u64 i) {
#include "_ref/main_668_675.inc"
    return InitialSeed;
}
#define RT_PIXEL_SEED_HOOK(x, y)                                                                              \
    if (RtPixelSeeds)                                                                                          \
        RandomState.Seed = RtSeedMix(((u64)PreviousRayCount * CurrentImage.Height + (y)) * CurrentImage.Width + (x))
#include "_ref/main_7_640_px.inc"  // main.cpp:7-640 with the two patches
#include <pthread.h>
#endif

extern "C" {
// ------------------------------------------------------- the math layer
u32 ref_pcg(u64 *state) { u32_random_state s = {*state}; u32 r = s.PCG(); *state = s.Seed; return r; }   // base.h:954-963
f32 ref_random_float(u64 *state, f32 lo, f32 hi) {                                                     // base.h:983-989
    u32_random_state s = {*state}; f32 r = s.RandomFloat(lo, hi); *state = s.Seed; return r;
}
f32 ref_rsqrt(f32 x) { return InverseSquareRoot(x); }                                                 // x64_math.h:71-74
f32 ref_sqrt(f32 x) { return SquareRoot(x); }
f32 ref_min(f32 a, f32 b) { return Min(a, b); }                                                       // x64_math.h:79-82
void ref_normalize(const f32 *in, f32 *out) { v3 r = v3::Normalize(v3(in[0], in[1], in[2])); out[0] = r.x; out[1] = r.y; out[2] = r.z; }
void ref_normalize_fast(const f32 *in, f32 *out) { v3 r = v3::NormalizeFast(v3(in[0], in[1], in[2])); out[0] = r.x; out[1] = r.y; out[2] = r.z; }
void ref_cross(const f32 *a, const f32 *b, f32 *out) {                                                 // x64_math.h:258-264
    v3 r = v3::Cross(v3(a[0], a[1], a[2]), v3(b[0], b[1], b[2])); out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
f32 ref_dot(const f32 *a, const f32 *b) { return v3::Dot(v3(a[0], a[1], a[2]), v3(b[0], b[1], b[2])); }
f32 ref_cos(f32 x) { return Cosine(x); }                                                              // x64_math.h:728-736
f32 ref_sin(f32 x) { return Sin(x); }                                                                 // x64_math.h:738-746
f32 ref_horizontal_min(const f32 *v4) {                                                               // x64_math.h:579-585
    f32x4 v; for (int i = 0; i < 4; ++i) v[i] = v4[i]; return f32x4::HorizontalMin(v);
}
// One lane-4 sphere-group test with the reference's f32x4/v3x4 operators
// (the arithmetic of main.cpp:400-417, restated over the reference types).
void ref_group_test(const f32 *o, const f32 *d, const f32 *px, const f32 *py, const f32 *pz, const f32 *r,
                    f32 *dist_out, f32 *t_out) {
    v3 O(o[0], o[1], o[2]), D(d[0], d[1], d[2]);
    v3x4 P; for (int i = 0; i < 4; ++i) { P.x[i] = px[i]; P.y[i] = py[i]; P.z[i] = pz[i]; }
    f32x4 R; for (int i = 0; i < 4; ++i) R[i] = r[i];
    v3x4 C = P - v3x4(O);
    f32x4 T = v3x4::Dot(C, v3x4(D));
    v3x4 PP = v3x4(D) * v3x4(T);
    f32x4 R2 = R * R;
    f32x4 Dist = v3x4::LengthSquared(C - PP);
    f32x4 X = f32x4::SquareRoot(R2 - Dist);
    f32x4 IT = T - X;
    f32x4 Test = IT < f32x4(F32Epsilon);
    f32x4::ConditionalMove(&IT, T + X, Test);
    for (int i = 0; i < 4; ++i) { dist_out[i] = Dist[i]; t_out[i] = IT[i]; }
}

// ------------------------------------------ main.cpp's colour path, compiled
f32 ref_reflectance(f32 cos_theta, f32 eta) { return Reflectance(cos_theta, eta); }     // main.cpp:292-300
f32 ref_linear_to_srgb(f32 l) { return LinearToSRGB(l); }                               // main.cpp:312-329
u32 ref_color_from_v4(const f32 *v) { return ColorFromV4(v4(v[0], v[1], v[2], v[3])); }  // main.cpp:340-346
// The store expression of main.cpp:492, ColorFromV4(LinearToSRGB(FinalColor)),
// over n v4 values (the v4 LinearToSRGB of main.cpp:331-338).
void ref_encode_rgba8(const f32 *v, u32 *out, u64 n) {
    for (u64 i = 0; i < n; ++i, v += 4) out[i] = ColorFromV4(LinearToSRGB(v4(v[0], v[1], v[2], v[3])));
}
void ref_linear_to_srgb_n(const f32 *in, f32 *out, u64 n) { for (u64 i = 0; i < n; ++i) out[i] = LinearToSRGB(in[i]); }

// main.cpp:484-492 verbatim: the running-mean blend into PreviousImage and the
// RGBA8 store, for one pixel whose radiance is `out3`, with the reference's
// own PreviousRayCount global (main.cpp:7) set to prev_count.
void ref_blend_store(u32 prev_count, const f32 *out3, f32 *prev4, u32 *px) {
    PreviousRayCount = prev_count;
    image PreviousImage = {}; PreviousImage.Data = prev4; PreviousImage.Width = 1; PreviousImage.Height = 1;
    image CurrentImage = {};  CurrentImage.Data = px;     CurrentImage.Width = 1;  CurrentImage.Height = 1;
    u32 x = 0, y = 0;
    v3 OutputColor = v3(out3[0], out3[1], out3[2]);
#include "_ref/main_484_492.inc"
}

// main.cpp:446-447 verbatim: the emission / attenuation update of one bounce.
void ref_emit_attenuate(const f32 *emissive, const f32 *color, f32 *att, f32 *out) {
    material Material = {};
    Material.Emissive = v3(emissive[0], emissive[1], emissive[2]);
    Material.Color = v3(color[0], color[1], color[2]);
    v3 Attenuation = v3(att[0], att[1], att[2]);
    v3 OutputColor = v3(out[0], out[1], out[2]);
#include "_ref/main_446_447.inc"
    att[0] = Attenuation.x; att[1] = Attenuation.y; att[2] = Attenuation.z;
    out[0] = OutputColor.x; out[1] = OutputColor.y; out[2] = OutputColor.z;
}

// ------------------------------------------------ the scene generators
// InitRGBSphereScene / InitRandomizedSphereScene / InitRTWeekendSphereScene
// (main.cpp:96-268), run once, as OnInit does (main.cpp:652-654).  Copies
// scene `index` out: scalar spheres (80 B each), sphere groups (64 B), the
// materials (48 B) and {LookAt.xyz, UseSkyColor, distance, x angle, y height,
// counts}.  Returns 0, or -1 when a buffer is too small.
int ref_scene_builtin(int index, void *spheres, u32 cap_spheres, void *groups, u32 cap_groups,
                      void *materials, u32 cap_materials, f32 *info) {
    static bool inited = false;
    if (!inited) {
        InitRGBSphereScene(Scenes + 0);
        InitRandomizedSphereScene(Scenes + 1);
        InitRTWeekendSphereScene(Scenes + 2);
        inited = true;
    }
    if (index < 0 || index > 2) return -1;
    const scene &S = Scenes[index];
    if (S.ScalarSpheres.Count > cap_spheres || S.SIMDSpheres.Count > cap_groups || S.Materials.Count > cap_materials)
        return -1;
    __builtin_memcpy(spheres, S.ScalarSpheres.Data, sizeof(scalar_sphere) * S.ScalarSpheres.Count);
    __builtin_memcpy(groups, S.SIMDSpheres.Data, sizeof(sphere_group) * S.SIMDSpheres.Count);
    __builtin_memcpy(materials, S.Materials.Data, sizeof(material) * S.Materials.Count);
    info[0] = S.LookAt.x; info[1] = S.LookAt.y; info[2] = S.LookAt.z;
    info[3] = S.UseSkyColor ? 1.0f : 0.0f;
    info[4] = S.DefaultDistanceFromLookAt; info[5] = S.DefaultXAngle; info[6] = S.DefaultYHeight;
    info[7] = (f32)S.ScalarSpheres.Count; info[8] = (f32)S.SIMDSpheres.Count; info[9] = (f32)S.Materials.Count;
    return 0;
}

// ------------------------------------------------------ the render itself
// `frames` frames of the reference's RenderTile (simd != 0) or
// RenderTileScalar over every 32x32 tile in order, on ThreadIndex 0, i.e. the
// reference with one worker thread: the thread's PCG stream starts at *state
// and runs on across tiles and frames, and PreviousRayCount is prev_count + k
// for frame k (OnRender, main.cpp:797-806).  The scene is the caller's arrays
// (layouts identical to main.cpp:11-26); the camera is camera_info's first 92
// bytes (main.cpp:270-278).  MaxRayBounce is the reference's literal 5
// (main.cpp:387,536) in librefmath.so, ref_set_patch's value in librefpix.so
// (which also re-seeds per pixel when asked).  *state and *rays are updated.
void ref_render(const void *spheres, u32 n_spheres, const void *groups, u32 n_groups, const void *materials,
                u32 n_materials, u32 use_sky, const f32 *cam, u32 width, u32 height, u32 prev_count, u32 frames,
                int simd, u64 *state, f32 *prev_v4, u32 *cur, u64 *rays) {
    static thread_context Context[1];
    scene Saved = Scenes[1];
    u32 SavedIndex = SceneIndex;
    scene &S = Scenes[1];
    S.UseSkyColor = use_sky != 0;
    S.ScalarSpheres.Data = (scalar_sphere *)spheres; S.ScalarSpheres.Count = n_spheres;
    S.SIMDSpheres.Data = (sphere_group *)groups;     S.SIMDSpheres.Count = n_groups;
    S.Materials.Data = (material *)materials;        S.Materials.Count = n_materials;
    SceneIndex = 1;

    __builtin_memcpy(&CameraInfo, cam, 92);
    CameraInfo.TilesX = (width + TileSize - 1) / TileSize;
    CameraInfo.CurrentImage.Data = cur;      CameraInfo.CurrentImage.Width = width;  CameraInfo.CurrentImage.Height = height;
    CameraInfo.PreviousImage.Data = prev_v4; CameraInfo.PreviousImage.Width = width; CameraInfo.PreviousImage.Height = height;

    Context[0].RandomState.Seed = *state;
    Context[0].RaysCastInThread = 0;
    ThreadContexts = Context;
    u32 Tiles = CameraInfo.TilesX * ((height + TileSize - 1) / TileSize);
    for (u32 k = 0; k < frames; ++k) {
        PreviousRayCount = prev_count + k;
        for (u32 t = 0; t < Tiles; ++t) {
            work_queue_context Work = {};
            Work.WorkEntry = t;
            Work.ThreadIndex = 0;
            if (simd) RenderTile(&Work);
            else RenderTileScalar(&Work);
        }
    }
    *state = Context[0].RandomState.Seed;
    *rays = Context[0].RaysCastInThread;
    ThreadContexts = 0;
    Scenes[1] = Saved;
    SceneIndex = SavedIndex;
}

#ifdef RT_REF_PATCHED
// The patched build's knobs: MaxRayBounce (patch i) and per-(pixel, frame)
// seeds (patch ii).
void ref_set_patch(u32 max_bounce, int pixel_seeds) { RtMaxRayBounce = max_bounce; RtPixelSeeds = pixel_seeds; }

struct RtPool { u32 tiles; u32 simd; volatile u32 next; const u32 *list; };
static void *rt_worker(void *arg) {
    void **a = (void **)arg;
    RtPool *p = (RtPool *)a[0];
    u32 index = (u32)(uintptr_t)a[1];
    for (;;) {
        u32 t = __atomic_fetch_add(&p->next, 1u, __ATOMIC_RELAXED);
        if (t >= p->tiles) break;
        work_queue_context Work = {};
        Work.WorkEntry = p->list ? p->list[t] : t;
        Work.ThreadIndex = index;
        if (p->simd) RenderTile(&Work);
        else RenderTileScalar(&Work);
    }
    return 0;
}

// ref_render with the tiles of each frame pulled by `threads` workers from
// one counter, as the reference's work queue deals them (wasm/wasm.cpp:624-694,
// main.cpp:851-856).  Only meaningful with pixel seeds on (the output is then
// independent of the schedule); *rays is the sum over the workers.
void ref_render_tile_list(const void *spheres, u32 n_spheres, const void *groups, u32 n_groups, const void *materials,
                          u32 n_materials, u32 use_sky, const f32 *cam, u32 width, u32 height, u32 prev_count,
                          u32 frames, int simd, u32 threads, const u32 *tile_list, u32 n_list, f32 *prev_v4, u32 *cur,
                          u64 *rays);

void ref_render_threads(const void *spheres, u32 n_spheres, const void *groups, u32 n_groups, const void *materials,
                        u32 n_materials, u32 use_sky, const f32 *cam, u32 width, u32 height, u32 prev_count,
                        u32 frames, int simd, u32 threads, f32 *prev_v4, u32 *cur, u64 *rays) {
    ref_render_tile_list(spheres, n_spheres, groups, n_groups, materials, n_materials, use_sky, cam, width, height,
                         prev_count, frames, simd, threads, 0, 0, prev_v4, cur, rays);
}

// ref_render_threads over a subset of the 32x32 tiles (work entries tile_list[0..n_list), row-major
// tile indices as main.cpp:362-368 decodes them), e.g. whole tile rows of a frame too large to render
// entirely (C5).  tile_list NULL: every tile.
void ref_render_tile_list(const void *spheres, u32 n_spheres, const void *groups, u32 n_groups, const void *materials,
                          u32 n_materials, u32 use_sky, const f32 *cam, u32 width, u32 height, u32 prev_count,
                          u32 frames, int simd, u32 threads, const u32 *tile_list, u32 n_list, f32 *prev_v4, u32 *cur,
                          u64 *rays) {
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    static thread_context Context[64];
    scene Saved = Scenes[1];
    u32 SavedIndex = SceneIndex;
    scene &S = Scenes[1];
    S.UseSkyColor = use_sky != 0;
    S.ScalarSpheres.Data = (scalar_sphere *)spheres; S.ScalarSpheres.Count = n_spheres;
    S.SIMDSpheres.Data = (sphere_group *)groups;     S.SIMDSpheres.Count = n_groups;
    S.Materials.Data = (material *)materials;        S.Materials.Count = n_materials;
    SceneIndex = 1;
    __builtin_memcpy(&CameraInfo, cam, 92);
    CameraInfo.TilesX = (width + TileSize - 1) / TileSize;
    CameraInfo.CurrentImage.Data = cur;      CameraInfo.CurrentImage.Width = width;  CameraInfo.CurrentImage.Height = height;
    CameraInfo.PreviousImage.Data = prev_v4; CameraInfo.PreviousImage.Width = width; CameraInfo.PreviousImage.Height = height;
    for (u32 i = 0; i < threads; ++i) { Context[i].RandomState.Seed = 0; Context[i].RaysCastInThread = 0; }
    ThreadContexts = Context;
    RtPool pool;
    pool.tiles = tile_list ? n_list : CameraInfo.TilesX * ((height + TileSize - 1) / TileSize);
    pool.list = tile_list;
    pool.simd = simd ? 1u : 0u;
    pthread_t th[64];
    void *args[64][2];
    for (u32 k = 0; k < frames; ++k) {
        PreviousRayCount = prev_count + k;
        pool.next = 0;
        for (u32 i = 0; i < threads; ++i) {
            args[i][0] = &pool; args[i][1] = (void *)(uintptr_t)i;
            pthread_create(&th[i], 0, rt_worker, args[i]);
        }
        for (u32 i = 0; i < threads; ++i) pthread_join(th[i], 0);
    }
    u64 total = 0;
    for (u32 i = 0; i < threads; ++i) total += Context[i].RaysCastInThread;
    *rays = total;
    ThreadContexts = 0;
    Scenes[1] = Saved;
    SceneIndex = SavedIndex;
}
#endif
}
