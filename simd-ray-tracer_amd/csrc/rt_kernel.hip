// rt_kernel.hip — CDNA4 (gfx950) trace kernel for the brute-force sphere path.
//
// Replaces the reference's tile callback RenderTile / RenderTileScalar
// (main.cpp:348-495 / 497-640) and its lane-4 math layer (x64_math.h,
// base.h:474-887).  One HIP thread owns one pixel of a compact per-GPU band
// image and folds ALL of this launch's frames (samples) for that pixel in
// order, keeping the running mean in registers; the reference's 4-wide SIMD
// lanes become the four per-residue-class minima each thread carries.
//
// Exactness: built with -ffp-contract=off (every op rounds separately, as the
// reference's SSE lane ops do), IEEE f32 denormals, correctly rounded sqrt and
// division; the one FMA the reference's -mfma build emits (Reflectance,
// main.cpp:299) is an explicit fmaf; rsqrtss is reproduced by table.
//
// Work shape: a wave = one 8x8 pixel tile (coherent rays), a block = 16x16.
// Paths are regenerated per lane (a lane whose sample ends starts its next
// sample on the next loop trip) so the sphere loop never idles on lanes whose
// path already terminated.  The sphere loop reads wave-uniform sphere groups
// either through the scalar cache into SGPRs (SRC_SMEM) or from the
// block's LDS copy (SRC_LDS); per-lane gathers (winning sphere, material,
// rsqrt table) always hit the LDS copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_kernel.h"

namespace rtk {

constexpr float kEps = 1e-4f;   // base.h:889 F32Epsilon
constexpr float kFMax = 1e30f;  // base.h:891 F32Max
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

// v3::Normalize (x64_math.h:234-245): IEEE divide by the correctly rounded
// sqrt, zero when len^2 <= 1e-4.
__device__ __forceinline__ void normalize(float &x, float &y, float &z) {
    const float l2 = dot3(x, y, z, x, y, z);
    const float len = __builtin_sqrtf(l2);
    const bool keep = l2 > kEps;
    x = keep ? x / len : 0.0f;
    y = keep ? y / len : 0.0f;
    z = keep ? z / len : 0.0f;
}

// rsqrtss (x64_math.h:71-74) from the 2x1024 table: exponent parity + top
// 10 mantissa bits pick the entry, the remaining even exponent scales it.
__device__ __forceinline__ float rsqrt_x86(const float *lut, float v) {
    const uint32_t u = __float_as_uint(v);
    const int32_t e = (int32_t)((u >> 23) & 0xFFu) - 127;
    const uint32_t par = (uint32_t)e & 1u;
    const float base = lut[par * 1024u + ((u >> 13) & 1023u)];
    const int32_t sh = (e - (int32_t)par) >> 1;
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
    return l < 0.0031308f ? l * 12.92f : __builtin_sqrtf(l);
}

__device__ __forceinline__ float reflectance(float cos_t, float eta) {  // main.cpp:292-300
    float r0 = (1.0f - eta) / (1.0f + eta);
    r0 *= r0;
    float r1 = 1.0f - cos_t;
    r1 = r1 * r1 * r1 * r1 * r1;
    return __builtin_fmaf(1.0f - r0, r1, r0);  // contracted by the reference's -mfma build
}

struct Sample {
    float ox, oy, oz, dx, dy, dz;
    float ax, ay, az;  // attenuation
    float cx, cy, cz;  // output colour
    uint64_t rng;
    uint32_t bounce;
};

// Jittered primary ray (main.cpp:375-385).
__device__ __forceinline__ void start_sample(const TraceArgs &a, uint32_t x, uint32_t y, uint32_t frame, Sample &p) {
    p.rng = seed_mix(((uint64_t)frame * a.height + y) * a.width + x);
    const float jx = rand_float(p.rng, -0.5f, kInvRange1);
    const float jy = rand_float(p.rng, -0.5f, kInvRange1);
    const float fx = -1.0f + (((float)x + jx) * 2.0f) / (float)a.width;
    const float fy = -1.0f + (((float)y + jy) * 2.0f) / (float)a.height;
    const float kx = (fx * a.film_w) * 0.5f;
    const float ky = (fy * a.film_h) * 0.5f;
    const float px = (a.film_center[0] + kx * a.cam_x[0]) + ky * a.cam_y[0];
    const float py = (a.film_center[1] + kx * a.cam_x[1]) + ky * a.cam_y[1];
    const float pz = (a.film_center[2] + kx * a.cam_x[2]) + ky * a.cam_y[2];
    p.ox = a.cam_pos[0];
    p.oy = a.cam_pos[1];
    p.oz = a.cam_pos[2];
    p.dx = px - p.ox;
    p.dy = py - p.oy;
    p.dz = pz - p.oz;
    normalize(p.dx, p.dy, p.dz);
    p.ax = p.ay = p.az = 1.0f;
    p.cx = p.cy = p.cz = 0.0f;
    p.bounce = 0;
}

// Emission, attenuation and the next direction (main.cpp:446-481).
__device__ __forceinline__ void shade(const float *lut, float4 col_spec, float4 emis_ior, float hx, float hy, float hz,
                                      bool inside, Sample &p) {
    p.cx = p.cx + emis_ior.x * p.ax;
    p.cy = p.cy + emis_ior.y * p.ay;
    p.cz = p.cz + emis_ior.z * p.az;
    p.ax = p.ax * col_spec.x;
    p.ay = p.ay * col_spec.y;
    p.az = p.az * col_spec.z;
    float nx = hx, ny = hy, nz = hz;
    normalize(nx, ny, nz);
    const float k2 = 2.0f * dot3(p.dx, p.dy, p.dz, nx, ny, nz);
    const float bx = p.dx - k2 * nx, by = p.dy - k2 * ny, bz = p.dz - k2 * nz;  // PureBounce
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
        p.dx = om * (nx + rx) + s * bx;
        p.dy = om * (ny + ry) + s * by;
        p.dz = om * (nz + rz) + s * bz;
        normalize(p.dx, p.dy, p.dz);
    } else {
        const float eta = inside ? ior : 1.0f / ior;
        const float dd = dot3(-p.dx, -p.dy, -p.dz, nx, ny, nz);
        const float cos_t = dd < 1.0f ? dd : 1.0f;  // _mm_min_ss
        const float sin_t = __builtin_sqrtf(1.0f - cos_t * cos_t);
        const bool cant = eta * sin_t > 1.0f;
        const float qx = eta * (p.dx + cos_t * nx);
        const float qy = eta * (p.dy + cos_t * ny);
        const float qz = eta * (p.dz + cos_t * nz);
        const float q = -__builtin_sqrtf(__builtin_fabsf(1.0f - dot3(qx, qy, qz, qx, qy, qz)));
        float rx = qx + q * nx, ry = qy + q * ny, rz = qz + q * nz;
        normalize(rx, ry, rz);
        bool refl = cant;
        if (!refl) refl = reflectance(cos_t, eta) > rand_float(p.rng, 0.0f, kInvRange1);
        if (refl && !inside) {
            p.dx = bx;
            p.dy = by;
            p.dz = bz;
        } else {
            p.dx = rx;
            p.dy = ry;
            p.dz = rz;
        }
    }
}

struct Group {
    float x[4], y[4], z[4], r2[4];
};

template <int SRC>
__device__ __forceinline__ Group load_group(const TraceArgs &a, const float4 *lds_groups, uint32_t g) {
    Group G;
    float4 v0, v1, v2, v3;
    if (SRC == kSrcLds) {
        v0 = lds_groups[4 * g + 0];
        v1 = lds_groups[4 * g + 1];
        v2 = lds_groups[4 * g + 2];
        v3 = lds_groups[4 * g + 3];
    } else {
        v0 = a.groups[4 * g + 0];
        v1 = a.groups[4 * g + 1];
        v2 = a.groups[4 * g + 2];
        v3 = a.groups[4 * g + 3];
    }
    G.x[0] = v0.x; G.x[1] = v0.y; G.x[2] = v0.z; G.x[3] = v0.w;
    G.y[0] = v1.x; G.y[1] = v1.y; G.y[2] = v1.z; G.y[3] = v1.w;
    G.z[0] = v2.x; G.z[1] = v2.y; G.z[2] = v2.z; G.z[3] = v2.w;
    G.r2[0] = v3.x; G.r2[1] = v3.y; G.r2[2] = v3.z; G.r2[3] = v3.w;
    return G;
}

// The shared part of one sphere test: T, |C - D*T|^2 (main.cpp:401-407).
__device__ __forceinline__ void sphere_core(const Sample &p, float sx, float sy, float sz, float &T, float &dist) {
    const float cx = sx - p.ox, cy = sy - p.oy, cz = sz - p.oz;
    T = dot3(cx, cy, cz, p.dx, p.dy, p.dz);
    const float qx = cx - p.dx * T, qy = cy - p.dy * T, qz = cz - p.dz * T;
    dist = dot3(qx, qy, qz, qx, qy, qz);
}

template <bool SIMD, int SRC>
__global__ __launch_bounds__(256) void trace_kernel(TraceArgs a) {
    extern __shared__ float4 smem[];
    // LDS image: [rsqrt table 512 float4][groups 4*n_groups float4][materials 2*4*n_groups float4]
    const float *lut = reinterpret_cast<const float *>(smem);
    float4 *lds_groups = smem + 512;
    float4 *lds_mats = lds_groups + 4 * a.n_groups;
    {
        const float4 *glut = reinterpret_cast<const float4 *>(a.rsqrt_lut);
        for (uint32_t i = threadIdx.x; i < 512u; i += blockDim.x) smem[i] = glut[i];
        for (uint32_t i = threadIdx.x; i < 4u * a.n_groups; i += blockDim.x) lds_groups[i] = a.groups[i];
        for (uint32_t i = threadIdx.x; i < 8u * a.n_groups; i += blockDim.x) lds_mats[i] = a.materials[i];
        __syncthreads();
    }

    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint32_t x = blockIdx.x * 16u + (wave & 1u) * 8u + (lane & 7u);
    const uint32_t ly = blockIdx.y * 16u + (wave >> 1) * 8u + (lane >> 3);
    const bool valid = x < a.width && ly < a.local_rows;
    const uint32_t y = ((ly / a.band_rows) * a.band_count + a.band_index) * a.band_rows + ly % a.band_rows;
    const size_t pix = (size_t)ly * a.width + x;

    float accx = 0.0f, accy = 0.0f, accz = 0.0f;
    if (valid && a.prev_count > 0 && !(a.flags & kFlagAccumZero)) {
        const float4 pv = a.prev[pix];
        accx = pv.x;
        accy = pv.y;
        accz = pv.z;
    }

    uint32_t nrays = 0;
    uint32_t k = 0;
    bool active = valid && a.frames > 0;
    Sample p;
    if (active) start_sample(a, x, y, a.prev_count, p);

    while (active) {
        bool done;
        if (a.max_bounce == 0) {
            done = true;
        } else {
            nrays += 1;
            // ---- brute-force intersection against every sphere (main.cpp:392-441 / 541-588)
            float t0 = kFMax, t1 = kFMax, t2 = kFMax, t3 = kFMax;
            uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0, ins = 0;
            for (uint32_t g = 0; g < a.n_groups; ++g) {
                const Group G = load_group<SRC>(a, lds_groups, g);
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    float T, dist;
                    sphere_core(p, G.x[l], G.y[l], G.z[l], T, dist);
                    const float r2 = G.r2[l];
                    if (SIMD) {
                        // lane-4 rules: strict '<' hit, per-class strict minimum,
                        // sticky inside flag (main.cpp:409-429)
                        if (dist < r2) {
                            const float X = __builtin_sqrtf(r2 - dist);
                            float it = T - X;
                            const bool in = it < kEps;
                            if (in) it = T + X;
                            float &tl = l == 0 ? t0 : l == 1 ? t1 : l == 2 ? t2 : t3;
                            uint32_t &gl = l == 0 ? g0 : l == 1 ? g1 : l == 2 ? g2 : g3;
                            if (it < tl && it > kEps) {
                                tl = it;
                                gl = g;
                                ins |= (in ? 1u : 0u) << l;
                            }
                        }
                    } else {
                        // scalar rules: '<=' hit, later sphere wins ties, inside
                        // flag from the accepted sphere only (main.cpp:557-578)
                        if (4u * g + (uint32_t)l < a.n_spheres && !(dist > r2)) {
                            const float X = __builtin_sqrtf(r2 - dist);
                            float it = T - X;
                            const bool in = it < kEps;
                            if (in) it = T + X;
                            if (!(it > t0) && !(it < kEps)) {
                                t0 = it;
                                g0 = 4u * g + (uint32_t)l;
                                ins = in ? 1u : 0u;
                            }
                        }
                    }
                }
            }
            // ---- hit select (x64_math.h:579-585 HorizontalMin + first equal lane)
            float tmin;
            uint32_t sidx;
            bool inside;
            if (SIMD) {
                const float m02 = t0 < t2 ? t0 : t2;
                const float m13 = t1 < t3 ? t1 : t3;
                tmin = m02 < m13 ? m02 : m13;
                const uint32_t l = t0 == tmin ? 0u : t1 == tmin ? 1u : t2 == tmin ? 2u : 3u;
                const uint32_t gsel = l == 0 ? g0 : l == 1 ? g1 : l == 2 ? g2 : g3;
                sidx = gsel * 4u + l;
                inside = (ins >> l) & 1u;
            } else {
                tmin = t0;
                sidx = g0;
                inside = ins != 0;
            }
            if (tmin == kFMax) {
                if (a.use_sky) {  // main.cpp:434-438
                    const float s = (p.dy + 1.0f) * 0.5f;
                    const float w = (1.0f - s) * 1.0f;
                    p.cx = p.cx + (w + s * 0.5f) * p.ax;
                    p.cy = p.cy + (w + s * 0.7f) * p.ay;
                    p.cz = p.cz + (w + s * 1.0f) * p.az;
                }
                done = true;
            } else {
                // Re-derive the winner's HitNormal / NextRayOrigin exactly as
                // they were formed at acceptance (main.cpp:423-429).
                const float *gsph = reinterpret_cast<const float *>(lds_groups) + 16u * (sidx >> 2) + (sidx & 3u);
                const float sx = gsph[0], sy = gsph[4], sz = gsph[8];
                const float cx = sx - p.ox, cy = sy - p.oy, cz = sz - p.oz;
                const float ipx = p.dx * tmin, ipy = p.dy * tmin, ipz = p.dz * tmin;
                const float hx = ipx - cx, hy = ipy - cy, hz = ipz - cz;
                p.ox = p.ox + ipx;
                p.oy = p.oy + ipy;
                p.oz = p.oz + ipz;
                const float4 cs = lds_mats[2u * sidx + 0u];
                const float4 ei = lds_mats[2u * sidx + 1u];
                shade(lut, cs, ei, hx, hy, hz, inside, p);
                p.bounce += 1;
                done = p.bounce == a.max_bounce;
            }
        }
        if (done) {
            // ---- running-mean blend (main.cpp:484-489)
            const uint32_t pc = a.prev_count + k;
            const uint32_t total = pc + 1u;
            const float inv = 1.0f / (float)total;
            const float ratio = (float)pc / (float)total;
            const float ox = a.max_bounce == 0 ? 0.0f : p.cx;
            const float oy = a.max_bounce == 0 ? 0.0f : p.cy;
            const float oz = a.max_bounce == 0 ? 0.0f : p.cz;
            accx = ox * inv + accx * ratio;
            accy = oy * inv + accy * ratio;
            accz = oz * inv + accz * ratio;
            k += 1;
            if (k < a.frames) start_sample(a, x, y, a.prev_count + k, p);
            else active = false;
        }
    }

    if (valid && a.frames > 0) {
        a.prev[pix] = make_float4(accx, accy, accz, 1.0f);
        a.cur[pix] = to_u8(linear_to_srgb(accx)) | (to_u8(linear_to_srgb(accy)) << 8) |
                     (to_u8(linear_to_srgb(accz)) << 16) | (255u << 24);
    }

    // ---- ray counter (RaysCastInThread, main.cpp:390): wave sum, one atomic
    uint32_t sum = nrays;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    if (lane == 0 && sum) atomicAdd(a.rays, (unsigned long long)sum);
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

}  // namespace rtk

extern "C" int rtk_launch_trace(const TraceArgs *a, int simd, int src, hipStream_t stream) {
    const dim3 block(256);
    const dim3 grid((a->width + 15u) / 16u, (a->local_rows + 15u) / 16u);
    const size_t lds = rtk_lds_bytes(a->n_groups);
    if (simd) {
        if (src == kSrcLds) hipLaunchKernelGGL((rtk::trace_kernel<true, kSrcLds>), grid, block, lds, stream, *a);
        else hipLaunchKernelGGL((rtk::trace_kernel<true, kSrcSmem>), grid, block, lds, stream, *a);
    } else {
        if (src == kSrcLds) hipLaunchKernelGGL((rtk::trace_kernel<false, kSrcLds>), grid, block, lds, stream, *a);
        else hipLaunchKernelGGL((rtk::trace_kernel<false, kSrcSmem>), grid, block, lds, stream, *a);
    }
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
