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

#include "_ref/main_7_640.inc"   // main.cpp:7-640, verbatim

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
// (main.cpp:387,536).  *state and *rays are updated.
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
}
