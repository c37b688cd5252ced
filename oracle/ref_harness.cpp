// ORACLE test harness (test infrastructure only).  Compiles the reference's
// own math layer -- /root/reference/base.h and x64_math.h, untouched, from
// where they lie -- and exposes its operations through extern "C" so tests
// can check the oracle's restated primitives against the real thing.
// main.cpp is NOT compiled (it needs <emscripten/atomic.h>, absent here).
#include "base.h"

extern "C" {
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
}
