// rt_app.cpp — the OnInit / OnRender frame driver (main.cpp:645-859) with
// the progressive accumulation resident in HBM, plus the rsqrtss tables.
//
// Semantics kept from the reference:
//   - one progressive frame per OnRender call, launched asynchronously;
//   - the image handed back is the previously COMPLETED frame (one-frame lag,
//     main.cpp:783-789), and OnRender returns false while a frame is in flight;
//   - a scene switch, a camera move, a resize or R resets the running mean
//     (PreviousRayCount = 0, buffers zeroed; main.cpp:791-804);
//   - *OutTotalRaysCast = bounce segments of the completed frame,
//     *OutTimeElapsed = its launch -> completion time (main.cpp:840-849).
// The reference's WASD/Space/C orbit (main.cpp:730-781) is driven by the
// RT_KEY_* bits the caller passes instead of the platform's IsDown().
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <string.h>
#include <time.h>

#include "rt_kernel.h"
#include "rt_trace.h"

#include "rsqrt_table_intel.inc"

extern "C" int rt_rsqrt_table_builtin(float out[2048]) {
    if (!out) return RT_EINVAL;
    memcpy(out, kRsqrtTableIntelBits, sizeof(kRsqrtTableIntelBits));
    return RT_OK;
}

static inline float host_rsqrtss(float x) { return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x))); }

extern "C" int rt_rsqrt_table_capture_host(float out[2048]) {
    if (!out) return RT_EINVAL;
    for (uint32_t e = 0; e < 2; ++e)
        for (uint32_t k = 0; k < 1024; ++k) {
            uint32_t u = ((127u + e) << 23) | (k << 13);
            float f;
            memcpy(&f, &u, 4);
            out[e * 1024 + k] = host_rsqrtss(f);
        }
    // Verify the table model on every mantissa of [1, 4) and a sweep of exponents.
    for (uint32_t u = 0x3F800000u; u < 0x40800000u; u += 7u) {
        for (int shift = -14; shift <= 2; shift += 2) {
            const uint32_t v = u + ((uint32_t)shift << 23);
            float x;
            memcpy(&x, &v, 4);
            const int32_t ex = (int32_t)((v >> 23) & 0xFFu) - 127;
            const uint32_t par = (uint32_t)ex & 1u;
            uint32_t base;
            memcpy(&base, &out[par * 1024u + ((v >> 13) & 1023u)], 4);
            const uint32_t pred = base - ((uint32_t)((ex - (int32_t)par) >> 1) << 23);
            const float got = host_rsqrtss(x);
            uint32_t gb;
            memcpy(&gb, &got, 4);
            if (gb != pred) return RT_EINVAL;
        }
    }
    return RT_OK;
}

namespace {

constexpr float kWorldScale = 0.0625f;
constexpr float kPi32 = 3.14159265358979323846f;

struct App {
    bool ready = false;
    rt_device *dev = nullptr;
    rt_multi *multi = nullptr;  // rt_on_init_devices with several devices
    int ordinal = 0;            // hip_devices[0]: the frame, the counter and the stream live there
    uint32_t scene_index = 0xFFFFFFFFu;
    float distance = 0.0f, x_angle = 0.0f, y_height = 0.0f;
    uint32_t prev_count = 0;
    uint32_t width = 0, height = 0;
    // Two device frames: frame k writes d_cur[k & 1] while the completed frame
    // k - 1 is handed out from the other, so a call launches the next frame
    // FIRST and then copies the previous one to the caller's image (the
    // reference's CopyImage, main.cpp:688-697) while the GPU traces.
    void *d_prev = nullptr;
    uint32_t *d_cur[2] = {nullptr, nullptr};
    // Pixels the three frame buffers hold (rt_on_render_reserve; OnInit reserves
    // its window, main.cpp:649-650).  A resize within it reuses them, as the
    // reference re-Pushes its images into the arena OnInit sized (main.cpp:
    // 658, 798-804): no call of the frame loop frees or allocates.
    size_t cap_px = 0;
    bool restart_pending = false;  // a reservation dropped the resident mean: the next call restarts it
    uint32_t slot = 0;             // d_cur slot of the last launched frame
    uint64_t *d_rays = nullptr;
    uint64_t *h_rays = nullptr;    // pinned: the last frame's count, copied after its trace
    hipEvent_t ev_start = nullptr, ev_done = nullptr;
    hipStream_t stream = nullptr;  // traces
    hipStream_t copy = nullptr;    // the hand-out DMA, beside the next frame's trace
    bool in_flight = false;
    // A caller image registered with rt_on_render_register_image is page-locked,
    // so the hand-out is one DMA straight into it.  Any other image gets the
    // frame through a pinned staging buffer the library owns (DMA, then one host
    // copy): the library never page-locks memory it was not handed explicitly.
    void *reg_ptr = nullptr;
    size_t reg_bytes = 0;
    void *staging = nullptr;
    size_t staging_bytes = 0;
    rt_camera_info cam;
    rt_on_render_profile prof;
};
App g_app;

double now_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

bool frame_complete() {
    if (!g_app.in_flight) return true;
    if (hipEventQuery(g_app.ev_done) == hipSuccess) return true;
    (void)hipGetLastError();  // "not ready" must not reach a later launch check
    return false;
}

int wait_frame() {
    if (!g_app.in_flight) return RT_OK;
    const double t = now_ms();
    if (hipEventSynchronize(g_app.ev_done) != hipSuccess) return RT_EIO;
    g_app.prof.HostWaitMs += now_ms() - t;
    return RT_OK;
}

// Frame buffers for `px` pixels: grows only beyond the capacity, keeping the
// running mean and both frames of the current geometry (device copies).
int ensure_frames(size_t px) {
    if (px <= g_app.cap_px) return RT_OK;
    void *prev = nullptr;
    uint32_t *cur[2] = {nullptr, nullptr};
    if (hipMalloc(&prev, px * 16u) != hipSuccess || hipMalloc(&cur[0], px * 4u) != hipSuccess ||
        hipMalloc(&cur[1], px * 4u) != hipSuccess) {
        (void)hipFree(prev);
        (void)hipFree(cur[0]);
        (void)hipFree(cur[1]);
        return RT_ENOMEM;
    }
    const size_t live = (size_t)g_app.width * g_app.height;
    if (live && g_app.d_prev &&
        (hipMemcpy(prev, g_app.d_prev, live * 16u, hipMemcpyDeviceToDevice) != hipSuccess ||
         hipMemcpy(cur[0], g_app.d_cur[0], live * 4u, hipMemcpyDeviceToDevice) != hipSuccess ||
         hipMemcpy(cur[1], g_app.d_cur[1], live * 4u, hipMemcpyDeviceToDevice) != hipSuccess)) {
        (void)hipFree(prev);  // the old frames stay in place
        (void)hipFree(cur[0]);
        (void)hipFree(cur[1]);
        return RT_EIO;
    }
    (void)hipFree(g_app.d_prev);
    (void)hipFree(g_app.d_cur[0]);
    (void)hipFree(g_app.d_cur[1]);
    g_app.d_prev = prev;
    g_app.d_cur[0] = cur[0];
    g_app.d_cur[1] = cur[1];
    g_app.cap_px = px;
    g_app.prof.FrameAllocations += 1;
    return RT_OK;
}

// The trace's launch buffers for a width x height frame (rt_device_reserve, or
// rt_multi_reserve over the devices' 8-row bands).  Called for every new
// geometry: a reservation already covering it grows nothing (the libraries keep
// the largest tile and pixel counts asked for), and only a new geometry gets here.
int reserve_launch(uint32_t w, uint32_t h) {
    int rc;
    if (g_app.multi) {
        rc = rt_multi_reserve(g_app.multi, w, h, 8u, 0u);
        // a reservation that grows the devices' resident means drops them (rt_multi_reserve):
        // once any frame has been traced (the mean holds frame 0 even at prev_count 0), the next
        // call must restart it rather than continue (a resize restarts it anyway)
        uint64_t held = 0;
        if (g_app.width && (rt_multi_resident_frames(g_app.multi, &held) != RT_OK || held == 0))
            g_app.restart_pending = true;
    } else {
        rc = rt_device_reserve(g_app.dev, w, h);
    }
    (void)hipSetDevice(g_app.ordinal);
    return rc;
}

void unregister_image() {
    if (g_app.reg_ptr) (void)hipHostUnregister(g_app.reg_ptr);
    (void)hipGetLastError();
    g_app.reg_ptr = nullptr;
    g_app.reg_bytes = 0;
}

// The completed frame in d_cur[slot] into the caller's image (CopyImage,
// main.cpp:688-697): one DMA on the copy stream, straight into a registered
// image, else into the library's pinned staging buffer and from there by a
// host copy.
int hand_out(const rt_image *image, uint32_t slot) {
    if (!image->Data) return RT_OK;
    const size_t bytes = (size_t)g_app.width * g_app.height * 4u;
    const double t = now_ms();
    const bool direct = image->Data == g_app.reg_ptr && bytes <= g_app.reg_bytes;
    if (!direct && bytes > g_app.staging_bytes) {
        if (g_app.staging) (void)hipHostFree(g_app.staging);
        g_app.staging = nullptr;
        g_app.staging_bytes = 0;
        if (hipHostMalloc(&g_app.staging, bytes, hipHostMallocDefault) != hipSuccess) return RT_ENOMEM;
        g_app.staging_bytes = bytes;
    }
    void *dst = direct ? image->Data : g_app.staging;
    if (hipMemcpyAsync(dst, g_app.d_cur[slot], bytes, hipMemcpyDeviceToHost, g_app.copy) != hipSuccess ||
        hipStreamSynchronize(g_app.copy) != hipSuccess)
        return RT_EIO;
    if (!direct) memcpy(image->Data, g_app.staging, bytes);
    g_app.prof.HostCopyMs += now_ms() - t;
    g_app.prof.FramesCopied += 1;
    return RT_OK;
}

}  // namespace

extern "C" int rt_on_init(rt_init_params *params) {
    const int first = 0;
    return rt_on_init_devices(params, &first, 1);
}

extern "C" int rt_on_init_devices(rt_init_params *params, const int *hip_devices, uint32_t count) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!hip_devices || count == 0) return RT_EINVAL;
    if (params) {  // main.cpp:646-650
        static const char kTitle[] = "SIMD Ray Tracer";
        params->WindowTitle = kTitle;
        params->WindowTitleSize = sizeof(kTitle) - 1u;
        params->WindowWidth = 1280;
        params->WindowHeight = 720;
    }
    if (g_app.ready) return RT_OK;
    rt_scene s;
    int rc = rt_scene_builtin(0, &s);  // builds all three scenes (main.cpp:652-654)
    if (rc) return rc;
    float table[2048];
    rt_rsqrt_table_builtin(table);
    if (count > 1) {  // WorkQueueCreate's thread pool -> the devices (main.cpp:658-665)
        rc = rt_multi_create(hip_devices, count, RT_MULTI_AUTO, &g_app.multi);
        if (rc) return rc;
        rc = rt_multi_set_rsqrt_table(g_app.multi, table);
    } else {
        rc = rt_device_create(hip_devices[0], &g_app.dev);
        if (rc) return rc;
        rc = rt_set_rsqrt_table(g_app.dev, table);
    }
    if (rc) return rc;
    g_app.ordinal = hip_devices[0];
    if (hipSetDevice(g_app.ordinal) != hipSuccess) return RT_ENODEV;
    if (hipMalloc(&g_app.d_rays, sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&g_app.h_rays, sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreate(&g_app.ev_start) != hipSuccess || hipEventCreate(&g_app.ev_done) != hipSuccess ||
        hipStreamCreateWithFlags(&g_app.stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&g_app.copy, hipStreamNonBlocking) != hipSuccess)
        return RT_ENOMEM;
    (void)hipMemset(g_app.d_rays, 0, sizeof(uint64_t));
    g_app.ready = true;
    // the window OnInit asks the platform for (main.cpp:649-650): frames up to
    // that size need no allocation in the frame loop.  Best effort: a failed
    // reservation (no memory) leaves the frames to grow on the first resize, as
    // they would without one, so the initialised driver stays usable.
    (void)rt_on_render_reserve(1280u, 720u);
    (void)hipGetLastError();
    return RT_OK;
}

extern "C" int rt_on_render_reserve(uint32_t width, uint32_t height) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!g_app.ready || width == 0 || height == 0 || width > 65536 || height > 65536)
        return RT_EINVAL;
    if (hipSetDevice(g_app.ordinal) != hipSuccess) return RT_ENODEV;
    const size_t px = (size_t)width * height;
    if (wait_frame() != RT_OK) return RT_EIO;  // growing frees buffers the frame in flight uses
    if (const int rc = ensure_frames(px)) return rc;
    return reserve_launch(width, height);
}

static int on_render(const rt_image *image, rt_render_params params, uint32_t keys, uint64_t *out_total_rays_cast,
                     double *out_time_elapsed_ms);

extern "C" int rt_on_render(const rt_image *image, rt_render_params params, uint32_t keys,
                            uint64_t *out_total_rays_cast, double *out_time_elapsed_ms) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    const double t = now_ms();
    const int rc = on_render(image, params, keys, out_total_rays_cast, out_time_elapsed_ms);
    g_app.prof.Calls += 1;
    g_app.prof.CallMs += now_ms() - t;
    return rc;
}

static int on_render(const rt_image *image, rt_render_params params, uint32_t keys, uint64_t *out_total_rays_cast,
                     double *out_time_elapsed_ms) {
    if (!g_app.ready || !image || image->Width == 0 || image->Height == 0) return RT_EINVAL;
    if (params.SceneIndex > 2) return RT_EINVAL;
    if (hipSetDevice(g_app.ordinal) != hipSuccess) return RT_ENODEV;
    bool moved = false;
    if (g_app.scene_index != params.SceneIndex) {  // main.cpp:718-727
        if (!frame_complete()) return 0;
        rt_scene sc;
        rt_scene_builtin(params.SceneIndex, &sc);
        int rc = g_app.multi ? rt_multi_scene_upload(g_app.multi, &sc) : rt_scene_upload(g_app.dev, &sc);
        if (rc) return rc;
        g_app.scene_index = params.SceneIndex;
        g_app.distance = sc.DefaultDistanceFromLookAt;
        g_app.x_angle = sc.DefaultXAngle;
        g_app.y_height = sc.DefaultYHeight;
        moved = true;
    }
    {  // main.cpp:730-775
        const float speed = 1.0f * kWorldScale;
        if (keys & RT_KEY_FORWARD) { g_app.distance -= speed; moved = true; }
        if (keys & RT_KEY_BACK) { g_app.distance += speed; moved = true; }
        if (keys & RT_KEY_RIGHT) { g_app.x_angle -= 1.0f / 16.0f; moved = true; }
        if (keys & RT_KEY_LEFT) { g_app.x_angle += 1.0f / 16.0f; moved = true; }
        if (keys & RT_KEY_UP) { g_app.y_height += speed; moved = true; }
        if (keys & RT_KEY_DOWN) { g_app.y_height -= speed; moved = true; }
        if (g_app.x_angle > kPi32 * 2.0f) g_app.x_angle -= kPi32 * 4.0f;
        if (g_app.x_angle < -(kPi32 * 2.0f)) g_app.x_angle += kPi32 * 4.0f;
        if (g_app.distance < 0.5f * kWorldScale) g_app.distance = 0.5f * kWorldScale;
        if (g_app.y_height > g_app.distance) g_app.y_height = g_app.distance;
    }
    const bool complete = frame_complete();                                          // :783
    const bool resize = image->Width != g_app.width || image->Height != g_app.height;  // :784
    bool copy_out = complete && !resize;
    if (resize || moved || (keys & RT_KEY_RESET) || g_app.restart_pending) {  // :791-804
        if (wait_frame() != RT_OK) return RT_EIO;
        copy_out = !resize;  // the completed frame still goes out (below)
        g_app.prev_count = 0;
        g_app.restart_pending = false;
        if (resize) {
            // RenderData.Reset + Push (main.cpp:798-804): the reserved buffers are
            // reused; only a frame beyond the reservation grows them
            if (const int rc = ensure_frames((size_t)image->Width * image->Height)) return rc;
            if (const int rc = reserve_launch(image->Width, image->Height)) return rc;
            g_app.restart_pending = false;  // the resize restarts the mean anyway
            g_app.width = image->Width;
            g_app.height = image->Height;
            g_app.in_flight = false;
        }
        // (the reference's arena zero-fills the new images on Push, wasm/wasm.cpp:52;
        // here the restarted frame writes every pixel of both, and PreviousRayCount 0
        // keeps the old running mean from being read, so no clear is needed)
    } else if (complete) {
        g_app.prev_count += 1;  // :805-806
    } else {
        return 0;  // :807-808
    }
    const uint32_t done_slot = g_app.slot;  // the completed frame (when copy_out)
    const uint32_t slot = g_app.in_flight ? done_slot ^ 1u : done_slot;
    rt_scene sc;
    rt_scene_builtin(g_app.scene_index, &sc);
    int rc = rt_camera_setup(&sc, g_app.distance, g_app.x_angle, g_app.y_height, g_app.width, g_app.height, &g_app.cam);
    if (rc) return rc;
    g_app.cam.CurrentImage.Data = g_app.d_cur[slot];
    g_app.cam.CurrentImage.Width = g_app.width;
    g_app.cam.CurrentImage.Height = g_app.height;
    g_app.cam.CurrentImage.Format = RT_FORMAT_R8G8B8A8_U32;
    g_app.cam.PreviousImage.Data = g_app.d_prev;
    g_app.cam.PreviousImage.Width = g_app.width;
    g_app.cam.PreviousImage.Height = g_app.height;
    g_app.cam.PreviousImage.Format = RT_FORMAT_R32B32G32A32_F32;
    if (copy_out && out_total_rays_cast) *out_total_rays_cast = g_app.in_flight ? *g_app.h_rays : 0u;  // :840-842
    {  // :848 (the previous frame has completed here: on every path above)
        float ms = 0.0f;
        if (g_app.in_flight && hipEventElapsedTime(&ms, g_app.ev_start, g_app.ev_done) != hipSuccess) {
            (void)hipGetLastError();
            ms = 0.0f;
        }
        g_app.prof.GpuFrameMs += ms;
        if (out_time_elapsed_ms) *out_time_elapsed_ms = ms;
    }
    const bool had_frame = g_app.in_flight;
    if (hipMemsetAsync(g_app.d_rays, 0, sizeof(uint64_t), g_app.stream) != hipSuccess) return RT_EIO;  // :843-846
    rt_trace_desc desc;
    memset(&desc, 0, sizeof(desc));
    desc.Width = g_app.width;
    desc.Height = g_app.height;
    desc.PreviousRayCount = g_app.prev_count;
    desc.Frames = 1;
    desc.MaxBounce = 5;  // main.cpp:387
    desc.EnableSIMD = params.EnableSIMD ? 1u : 0u;
    desc.SeedMode = RT_SEED_PIXEL;
    if (hipEventRecord(g_app.ev_start, g_app.stream) != hipSuccess) return RT_EIO;
    if (g_app.multi) {  // the running mean stays on the devices, the frame is gathered into d_cur
        desc.BandRows = 8;
        if (g_app.prev_count == 0) desc.Flags |= RT_FLAG_ACCUM_ZERO;
        g_app.cam.PreviousImage.Data = nullptr;
        rc = rt_multi_trace(g_app.multi, &g_app.cam, &desc, g_app.d_rays, g_app.stream);
    } else {
        desc.BandRows = 32;
        desc.BandCount = 1;
        rc = rt_trace(g_app.dev, &g_app.cam, &desc, g_app.d_rays, g_app.stream);
    }
    if (rc) return rc;
    if (hipMemcpyAsync(g_app.h_rays, g_app.d_rays, sizeof(uint64_t), hipMemcpyDeviceToHost, g_app.stream) != hipSuccess ||
        hipEventRecord(g_app.ev_done, g_app.stream) != hipSuccess)
        return RT_EIO;
    g_app.slot = slot;
    g_app.in_flight = true;
    g_app.prof.FramesLaunched += 1;
    // the completed frame goes out while the new one traces (it is in the other slot)
    if (copy_out) {
        if (!had_frame) {  // nothing traced yet: the zero-filled CurrentImage
            if (image->Data) memset(image->Data, 0, (size_t)g_app.width * g_app.height * 4u);
        } else if (hand_out(image, done_slot) != RT_OK) {
            return RT_EIO;
        }
    }
    return copy_out ? 1 : 0;
}

extern "C" int rt_on_render_get_profile(rt_on_render_profile *out, int reset) {
    if (!out) return RT_EINVAL;
    *out = g_app.prof;
    if (reset) g_app.prof = rt_on_render_profile{};
    return RT_OK;
}

extern "C" int rt_on_render_wait(void) { return g_app.ready ? wait_frame() : RT_OK; }

extern "C" int rt_on_render_register_image(void *data, uint64_t bytes) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!g_app.ready || !data || bytes == 0) return RT_EINVAL;
    if (hipSetDevice(g_app.ordinal) != hipSuccess) return RT_ENODEV;
    if (data == g_app.reg_ptr && bytes == g_app.reg_bytes) return RT_OK;
    // the copy stream may still be writing into the old registration only
    // inside a hand-out, which is synchronous, so it is idle here
    unregister_image();
    if (hipHostRegister(data, (size_t)bytes, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        return RT_EIO;
    }
    g_app.reg_ptr = data;
    g_app.reg_bytes = (size_t)bytes;
    return RT_OK;
}

extern "C" int rt_on_render_unregister_image(void) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!g_app.ready) return RT_OK;
    if (hipSetDevice(g_app.ordinal) != hipSuccess) return RT_ENODEV;
    unregister_image();
    return RT_OK;
}

extern "C" int rt_on_shutdown(void) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!g_app.ready) return RT_OK;
    wait_frame();
    unregister_image();
    if (g_app.staging) (void)hipHostFree(g_app.staging);
    (void)hipFree(g_app.d_prev);
    (void)hipFree(g_app.d_cur[0]);
    (void)hipFree(g_app.d_cur[1]);
    (void)hipFree(g_app.d_rays);
    if (g_app.h_rays) (void)hipHostFree(g_app.h_rays);
    (void)hipEventDestroy(g_app.ev_start);
    (void)hipEventDestroy(g_app.ev_done);
    (void)hipStreamDestroy(g_app.stream);
    if (g_app.copy) (void)hipStreamDestroy(g_app.copy);
    rt_device_destroy(g_app.dev);
    rt_multi_destroy(g_app.multi);
    g_app = App();
    return RT_OK;
}
