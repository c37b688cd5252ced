// multi_rccl_check.cpp -- TEST PROGRAM: rt_multi's RCCL branch over N shards of
// one GPU, through the C-ABI only (include/rt_trace.h), with
// tests/loopback_rccl/librccl.so.1 (the loopback stand-in) found first on
// LD_LIBRARY_PATH.  Started by tests/conftest.py before the test process
// touches the GPU; tests/test_gpu_multi.py checks what it writes.
//
// usage: multi_rccl_check <out.json> [n_devices=8] [width=1920 height=1080 spp=256]
//
// Calls (every one through rt_multi_trace with Transport RCCL, every frame
// compared byte for byte with one rt_device tracing the whole frame):
//   A  a restart of S frames that also gathers the running mean (BASELINE C2
//      by default: its hashes go to the JSON for the golden check);
//   B  a continuation of 8 frames on the devices' resident means;
//   C  three restarts back to back with no host synchronisation (frames 4 at
//      PreviousRayCount 1000, 2000, 3000 with RT_FLAG_ACCUM_ZERO), each into
//      its own frame buffer: the two band-image slots and the sent events.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rt_trace.h"

#define CHECK(what, expr)                                                                        \
    do {                                                                                         \
        const int rc_ = (expr);                                                                  \
        if (rc_ != RT_OK) {                                                                      \
            fprintf(stderr, "multi_rccl_check: %s failed (%d): %s\n", what, rc_, rt_last_error()); \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)
#define HCHECK(expr)                                                                              \
    do {                                                                                          \
        if ((expr) != hipSuccess) {                                                               \
            fprintf(stderr, "multi_rccl_check: %s: %s\n", #expr, hipGetErrorString(hipGetLastError())); \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

template <class T>
static std::vector<T> host(const void *d, size_t n) {
    std::vector<T> v(n);
    if (hipMemcpy(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess) v.clear();
    return v;
}

static bool same_bytes(const void *da, const void *db, size_t bytes) {
    std::vector<unsigned char> a = host<unsigned char>(da, bytes), b = host<unsigned char>(db, bytes);
    return a.size() == bytes && b.size() == bytes && memcmp(a.data(), b.data(), bytes) == 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out.json> [n_devices] [width height spp]\n", argv[0]);
        return 2;
    }
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 8u;
    const uint32_t W = argc > 5 ? (uint32_t)atoi(argv[3]) : 1920u, H = argc > 5 ? (uint32_t)atoi(argv[4]) : 1080u;
    const uint32_t S = argc > 5 ? (uint32_t)atoi(argv[5]) : 256u, B = 8u;
    if (n == 0 || n > RT_MULTI_MAX_DEVICES) return 2;
    float table[2048];
    CHECK("rt_rsqrt_table_builtin", rt_rsqrt_table_builtin(table));
    rt_scene full_scene, scene;
    CHECK("rt_scene_builtin", rt_scene_builtin(1, &full_scene));
    CHECK("rt_scene_prefix", rt_scene_prefix(&full_scene, 64, &scene));
    rt_camera_info cam;
    CHECK("rt_camera_setup", rt_camera_setup(&scene, scene.DefaultDistanceFromLookAt, scene.DefaultXAngle,
                                             scene.DefaultYHeight, W, H, &cam));
    std::vector<int> devs(n, 0);
    rt_multi *m = nullptr;
    CHECK("rt_multi_create(RT_MULTI_RCCL)", rt_multi_create(devs.data(), n, RT_MULTI_RCCL, &m));
    CHECK("rt_multi_set_rsqrt_table", rt_multi_set_rsqrt_table(m, table));
    CHECK("rt_multi_scene_upload", rt_multi_scene_upload(m, &scene));
    CHECK("rt_multi_reserve", rt_multi_reserve(m, W, H, 8u, RT_MULTI_RESERVE_MEAN));
    rt_device *d = nullptr;
    CHECK("rt_device_create", rt_device_create(0, &d));
    CHECK("rt_set_rsqrt_table", rt_set_rsqrt_table(d, table));
    CHECK("rt_scene_upload", rt_scene_upload(d, &scene));
    CHECK("rt_device_reserve", rt_device_reserve(d, W, H));

    const size_t px = (size_t)W * H;
    void *m_cur[3], *m_mean, *d_cur[3], *d_prev;
    uint64_t *rays;  // [0..3] the multi calls, [4..7] the device's
    HCHECK(hipSetDevice(0));
    for (int i = 0; i < 3; ++i) {
        HCHECK(hipMalloc(&m_cur[i], px * 4));
        HCHECK(hipMalloc(&d_cur[i], px * 4));
    }
    HCHECK(hipMalloc(&m_mean, px * 16));
    HCHECK(hipMalloc(&d_prev, px * 16));
    HCHECK(hipMalloc(&rays, 16 * sizeof(uint64_t)));
    HCHECK(hipMemset(rays, 0, 16 * sizeof(uint64_t)));
    hipStream_t st;
    HCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

    rt_trace_desc desc;
    memset(&desc, 0, sizeof(desc));
    desc.Width = W;
    desc.Height = H;
    desc.MaxBounce = B;
    desc.EnableSIMD = 1;
    desc.SeedMode = RT_SEED_PIXEL;
    rt_camera_info c = cam;

    // A: S frames from scratch, frame and running mean gathered
    desc.Frames = S;
    desc.PreviousRayCount = 0;
    desc.Flags = RT_FLAG_ACCUM_ZERO;
    desc.BandRows = 8;
    c.CurrentImage.Data = m_cur[0];
    c.PreviousImage.Data = m_mean;
    CHECK("rt_multi_trace A", rt_multi_trace(m, &c, &desc, rays + 0, st));
    rt_multi_info info;
    CHECK("rt_multi_get_info", rt_multi_get_info(m, &info));
    rt_trace_desc dd = desc;
    dd.BandRows = 32;
    dd.BandCount = 1;
    rt_camera_info dc = cam;
    dc.CurrentImage.Data = d_cur[0];
    dc.PreviousImage.Data = d_prev;
    CHECK("rt_trace A", rt_trace(d, &dc, &dd, rays + 4, st));
    HCHECK(hipStreamSynchronize(st));
    std::vector<uint64_t> r = host<uint64_t>(rays, 8);
    const std::vector<uint32_t> cur_a = host<uint32_t>(m_cur[0], px);
    const std::vector<float> mean_a = host<float>(m_mean, px * 4);
    const uint64_t h_rgba = rt_frame_hash(cur_a.data(), px * 4), h_v4 = rt_frame_hash(mean_a.data(), px * 16);
    const bool eq_a = same_bytes(m_cur[0], d_cur[0], px * 4) && same_bytes(m_mean, d_prev, px * 16) && r[0] == r[4];
    const uint64_t rays_a = r[0];

    // B: a continuation of 8 frames on the resident means (the device continues its own mean)
    desc.PreviousRayCount = S;
    desc.Frames = 8;
    desc.Flags = 0;
    CHECK("rt_multi_trace B", rt_multi_trace(m, &c, &desc, rays + 1, st));
    dd.PreviousRayCount = S;
    dd.Frames = 8;
    dd.Flags = 0;
    CHECK("rt_trace B", rt_trace(d, &dc, &dd, rays + 5, st));
    HCHECK(hipStreamSynchronize(st));
    r = host<uint64_t>(rays, 8);
    const bool eq_b = same_bytes(m_cur[0], d_cur[0], px * 4) && same_bytes(m_mean, d_prev, px * 16) && r[1] == r[5];
    uint64_t resident_b = 0;
    CHECK("rt_multi_resident_frames", rt_multi_resident_frames(m, &resident_b));

    // C: three restarts back to back, no host synchronisation, each into its own frame
    bool eq_c[3];
    c.PreviousImage.Data = nullptr;
    desc.Frames = 4;
    desc.Flags = RT_FLAG_ACCUM_ZERO;
    for (int i = 0; i < 3; ++i) {
        desc.PreviousRayCount = 1000u * (uint32_t)(i + 1);
        c.CurrentImage.Data = m_cur[i];
        CHECK("rt_multi_trace C", rt_multi_trace(m, &c, &desc, rays + 8 + i, st));
    }
    HCHECK(hipStreamSynchronize(st));
    dd.Frames = 4;
    dd.Flags = RT_FLAG_ACCUM_ZERO;
    for (int i = 0; i < 3; ++i) {
        dd.PreviousRayCount = 1000u * (uint32_t)(i + 1);
        dc.CurrentImage.Data = d_cur[i];
        CHECK("rt_trace C", rt_trace(d, &dc, &dd, rays + 12 + i, st));
        HCHECK(hipStreamSynchronize(st));
    }
    r = host<uint64_t>(rays, 16);
    for (int i = 0; i < 3; ++i) eq_c[i] = same_bytes(m_cur[i], d_cur[i], px * 4) && r[8 + i] == r[12 + i];
    uint64_t resident_c = 0;
    CHECK("rt_multi_resident_frames", rt_multi_resident_frames(m, &resident_c));
    float gather_ms = 0.0f;
    CHECK("rt_multi_last_gather_ms", rt_multi_last_gather_ms(m, &gather_ms));

    FILE *f = fopen(argv[1], "w");
    if (!f) return 1;
    fprintf(f,
            "{\"transport\": \"%s\", \"devices\": %u, \"width\": %u, \"height\": %u, \"frames\": %u, \"bounces\": %u,\n"
            " \"a\": {\"rays\": %llu, \"fnv1a64_rgba8\": \"%016llx\", \"fnv1a64_v4\": \"%016llx\", \"equal_one_device\": %s},\n"
            " \"b\": {\"rays\": %llu, \"equal_one_device\": %s, \"resident_frames\": %llu},\n"
            " \"c\": {\"equal_one_device\": [%s, %s, %s], \"rays\": [%llu, %llu, %llu], \"resident_frames\": %llu},\n"
            " \"gather_ms\": %.4f}\n",
            info.Transport == RT_MULTI_RCCL ? "rccl" : "peer", n, W, H, S, B, (unsigned long long)rays_a,
            (unsigned long long)h_rgba, (unsigned long long)h_v4, eq_a ? "true" : "false",
            (unsigned long long)r[1], eq_b ? "true" : "false", (unsigned long long)resident_b,
            eq_c[0] ? "true" : "false", eq_c[1] ? "true" : "false", eq_c[2] ? "true" : "false",
            (unsigned long long)r[8], (unsigned long long)r[9], (unsigned long long)r[10],
            (unsigned long long)resident_c, gather_ms);
    fclose(f);
    rt_device_destroy(d);
    rt_multi_destroy(m);
    printf("multi_rccl_check: transport %s, A %s, B %s, C %s %s %s\n", info.Transport == RT_MULTI_RCCL ? "rccl" : "peer",
           eq_a ? "equal" : "DIFFER", eq_b ? "equal" : "DIFFER", eq_c[0] ? "equal" : "DIFFER",
           eq_c[1] ? "equal" : "DIFFER", eq_c[2] ? "equal" : "DIFFER");
    return eq_a && eq_b && eq_c[0] && eq_c[1] && eq_c[2] ? 0 : 3;
}
