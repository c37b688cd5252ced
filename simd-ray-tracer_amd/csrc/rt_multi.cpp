// rt_multi.cpp — several GPUs behind the C-ABI (include/rt_trace.h):
//   rt_multi : one host process drives N devices (the reference's thread-pool
//              tiler, main.cpp:658-665 / 851-856, becomes per-device band
//              dispatch plus one gather to devices[0] per call);
//   rt_comm  : the same band gather for one-process-per-GPU launches.
// Bands are dealt round-robin (band b -> device b mod N); every
// device traces its residue with rt_trace into compact band-local images,
// the images travel to devices[0] -- RCCL grouped send/recv into a staging
// buffer, or hipMemcpyPeerAsync over xGMI -- and the assembly kernel scatters
// them into the full frame.  RCCL is loaded at run time (dlopen), so the
// library has no link-time dependency on it and reports RT_ENODEV when it is
// absent; inside a torch process the already-loaded librccl.so.1 is reused.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "rt_kernel.h"
#include "rt_trace.h"

#define MHIP(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return rt_fail(RT_EIO, "%s: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

namespace {

// ------------------------------------------------------------ RCCL (dlopen)
struct Rccl {
    bool ok = false;
    // tests/loopback_rccl's stand-in library (rtLoopbackSharedDevices): its communicators may
    // list a device twice, which the real RCCL refuses (so with it, never tried)
    bool shared_devices = false;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static bool tried = false;
    if (tried) return r;
    tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, when torch is loaded
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    bool all = true;
    auto sym = [&](auto &fn, const char *name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        all = all && fn != nullptr;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = all;
    r.shared_devices = dlsym(h, "rtLoopbackSharedDevices") != nullptr;
    return r;
}

#define NCCL_OK(expr)                                                                                  \
    do {                                                                                               \
        ncclResult_t r_ = (expr);                                                                      \
        if (r_ != ncclSuccess) return rt_fail(RT_EIO, "%s: %s", #expr, rccl().GetErrorString(r_));    \
    } while (0)

// Bytes of rank r's compact band image.
inline size_t band_bytes(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t n, uint32_t r, uint32_t elem) {
    return (size_t)rt_band_local_rows(height, band_rows, n, r) * width * elem;
}

inline uint32_t max_local_rows(uint32_t height, uint32_t band_rows, uint32_t n) {
    uint32_t m = 0;
    for (uint32_t r = 0; r < n; ++r) m = std::max(m, rt_band_local_rows(height, band_rows, n, r));
    return m;
}

template <class T>
int grow(T **p, size_t *cap, size_t bytes) {  // device allocation on the current device
    if (bytes <= *cap) return RT_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, bytes) != hipSuccess) return rt_fail(RT_ENOMEM, "rt_multi: device allocation of %zu B", bytes);
    *cap = bytes;
    return RT_OK;
}

// Calls alternate between two slots of every shard's band image and ray
// counter, so call k's gather (reading slot k & 1) overlaps call k+1's trace
// (writing the other slot); a slot is traced again only after the gather two
// calls back has read it.
constexpr int kSlots = 2;

struct Shard {
    int ordinal = 0;
    rt_device *dev = nullptr;
    hipStream_t stream = nullptr;      // traces
    hipStream_t xfer = nullptr;        // RCCL sends of this device's images (off the trace stream)
    hipEvent_t traced[kSlots] = {};    // the trace into slot b is done
    hipEvent_t sent[kSlots] = {};      // RCCL: the sends of slot b are done (slot b free again)
    hipEvent_t t0[kSlots] = {}, t1[kSlots] = {};  // timing of the trace into slot b
    float4 *prev = nullptr;            // resident running mean of this device's bands
    uint32_t *cur[kSlots] = {};        // RGBA8 of this device's bands
    uint64_t *rays[kSlots] = {};       // segments this device traced into slot b
    size_t cap_prev = 0, cap_cur = 0;
    bool launched = false;             // the last call launched a trace here (rows > 0, frames > 0)
    ncclComm_t comm = nullptr;
};

}  // namespace

struct rt_multi {
    std::vector<Shard> s;
    uint32_t transport = RT_MULTI_PEER;
    // devices[0]: staging for the gathered compact images and ray counters
    uint8_t *stage_cur = nullptr, *stage_prev = nullptr;
    size_t cap_stage_cur = 0, cap_stage_prev = 0;
    uint64_t *ray_slots = nullptr;
    hipStream_t gather = nullptr;  // devices[0]
    hipEvent_t start = nullptr, gathered = nullptr;
    // timing of the gather: from every trace done (the gather stream has waited
    // for each device's traced event) to the frame assembled on devices[0]
    hipEvent_t g0[kSlots] = {}, g1[kSlots] = {};
    hipEvent_t copied[kSlots] = {};   // peer transport: slot b's copies are done (slot b free again)
    bool slot_used[kSlots] = {};      // slot b has been gathered before (its free event is valid)
    uint32_t calls = 0;               // rt_multi_trace calls (slot = calls & 1)
    bool prev_gathered = false;       // the last call also gathered the resident running means
    // geometry the resident running means belong to, and the frames folded there
    uint32_t width = 0, height = 0, band_rows = 0;
    bool accum_valid = false;
    uint64_t resident_frames = 0;
    uint32_t last_band_rows = 0, last_max_rows = 0, last_slot = 0;
};

static void destroy_shard(Shard &sh) {
    (void)hipSetDevice(sh.ordinal);
    if (sh.stream) (void)hipStreamSynchronize(sh.stream);
    if (sh.xfer) (void)hipStreamSynchronize(sh.xfer);
    // the device first: it waits on its own event after the last trace, issued on sh.stream
    if (sh.dev) rt_device_destroy(sh.dev);
    if (sh.comm && rccl().ok) (void)rccl().CommDestroy(sh.comm);
    (void)hipFree(sh.prev);
    for (int b = 0; b < kSlots; ++b) {
        (void)hipFree(sh.cur[b]);
        (void)hipFree(sh.rays[b]);
        for (hipEvent_t e : {sh.traced[b], sh.sent[b], sh.t0[b], sh.t1[b]})
            if (e) (void)hipEventDestroy(e);
    }
    if (sh.xfer) (void)hipStreamDestroy(sh.xfer);
    if (sh.stream) (void)hipStreamDestroy(sh.stream);
    sh = Shard();
}

extern "C" int rt_multi_destroy(rt_multi *m) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m) return RT_OK;
    for (Shard &sh : m->s) {
        (void)hipSetDevice(sh.ordinal);
        if (sh.stream) (void)hipStreamSynchronize(sh.stream);
        if (sh.xfer) (void)hipStreamSynchronize(sh.xfer);
    }
    if (!m->s.empty()) {
        (void)hipSetDevice(m->s[0].ordinal);
        if (m->gather) (void)hipStreamSynchronize(m->gather);
        (void)hipFree(m->stage_cur);
        (void)hipFree(m->stage_prev);
        (void)hipFree(m->ray_slots);
        for (hipEvent_t e : {m->start, m->gathered, m->copied[0], m->copied[1], m->g0[0], m->g0[1], m->g1[0], m->g1[1]})
            if (e) (void)hipEventDestroy(e);
        if (m->gather) (void)hipStreamDestroy(m->gather);
    }
    for (Shard &sh : m->s) destroy_shard(sh);
    delete m;
    return RT_OK;
}

extern "C" int rt_multi_create(const int *hip_devices, uint32_t count, uint32_t transport, rt_multi **out) {
    return rt_multi_create_ex(hip_devices, count, transport, nullptr, out);
}

extern "C" int rt_multi_create_ex(const int *hip_devices, uint32_t count, uint32_t transport,
                                  const rt_device_options *options, rt_multi **out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!hip_devices || !out || count == 0 || count > RT_MULTI_MAX_DEVICES)
        return rt_fail(RT_EINVAL, "rt_multi_create: need 1..%u devices", RT_MULTI_MAX_DEVICES);
    if (transport > RT_MULTI_PEER) return rt_fail(RT_EINVAL, "rt_multi_create: unknown transport %u", transport);
    *out = nullptr;
    rt_multi *m = new rt_multi();
    m->s.resize(count);
    for (uint32_t i = 0; i < count; ++i) {
        Shard &sh = m->s[i];
        sh.ordinal = hip_devices[i];
        int rc = rt_device_create_ex(sh.ordinal, options, &sh.dev);
        if (rc) {
            rt_multi_destroy(m);
            return rc;
        }
        bool ok = hipSetDevice(sh.ordinal) == hipSuccess &&
                  hipStreamCreateWithFlags(&sh.stream, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&sh.xfer, hipStreamNonBlocking) == hipSuccess;
        for (int b = 0; ok && b < kSlots; ++b)
            ok = hipEventCreateWithFlags(&sh.traced[b], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&sh.sent[b], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreate(&sh.t0[b]) == hipSuccess && hipEventCreate(&sh.t1[b]) == hipSuccess &&
                 hipMalloc(&sh.rays[b], sizeof(uint64_t)) == hipSuccess;
        if (!ok) {
            rt_multi_destroy(m);
            return rt_fail(RT_ENOMEM, "rt_multi_create: stream/event/counter on device %d", sh.ordinal);
        }
    }
    const int d0 = m->s[0].ordinal;
    if (hipSetDevice(d0) != hipSuccess || hipStreamCreateWithFlags(&m->gather, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&m->start, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->gathered, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->copied[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->copied[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&m->g0[0]) != hipSuccess || hipEventCreate(&m->g0[1]) != hipSuccess ||
        hipEventCreate(&m->g1[0]) != hipSuccess || hipEventCreate(&m->g1[1]) != hipSuccess ||
        hipMalloc(&m->ray_slots, RT_MULTI_MAX_DEVICES * sizeof(uint64_t)) != hipSuccess) {
        rt_multi_destroy(m);
        return rt_fail(RT_ENOMEM, "rt_multi_create: gather resources on device %d", d0);
    }
    bool distinct = true;
    for (uint32_t i = 0; i < count; ++i)
        for (uint32_t j = 0; j < i; ++j) distinct = distinct && hip_devices[i] != hip_devices[j];
    bool use_rccl = false;
    if (transport != RT_MULTI_PEER && (distinct || rccl().shared_devices) && rccl().ok) {
        std::vector<ncclComm_t> comms(count, nullptr);
        std::vector<int> devs(hip_devices, hip_devices + count);
        if (rccl().CommInitAll(comms.data(), (int)count, devs.data()) == ncclSuccess) {
            for (uint32_t i = 0; i < count; ++i) m->s[i].comm = comms[i];
            use_rccl = true;
        }
    }
    if (transport == RT_MULTI_RCCL && !use_rccl) {
        const bool loaded = rccl().ok;
        rt_multi_destroy(m);
        return rt_fail(RT_ENODEV, "rt_multi_create: RCCL unavailable (%s)",
                       !distinct ? "a device is listed twice" : !loaded ? "librccl.so.1 not loadable"
                                                                         : "ncclCommInitAll failed");
    }
    if (!use_rccl) {  // peer copies: let devices[0] read the others over xGMI where the hardware allows
        (void)hipSetDevice(d0);
        for (uint32_t i = 1; i < count; ++i) {
            int can = 0;
            if (hip_devices[i] != d0 && hipDeviceCanAccessPeer(&can, d0, hip_devices[i]) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(hip_devices[i], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            }
        }
    }
    m->transport = use_rccl ? RT_MULTI_RCCL : RT_MULTI_PEER;
    *out = m;
    return RT_OK;
}

extern "C" int rt_multi_set_rsqrt_table(rt_multi *m, const float table[2048]) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !table) return rt_fail(RT_EINVAL, "rt_multi_set_rsqrt_table: NULL argument");
    if (const int rc = rt_multi_synchronize(m)) return rc;
    for (Shard &sh : m->s)
        if (const int rc = rt_set_rsqrt_table(sh.dev, table)) return rc;
    return RT_OK;
}

extern "C" int rt_multi_scene_upload(rt_multi *m, const rt_scene *scene) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !scene) return rt_fail(RT_EINVAL, "rt_multi_scene_upload: NULL argument");
    if (const int rc = rt_multi_synchronize(m)) return rc;
    for (Shard &sh : m->s)
        if (const int rc = rt_scene_upload(sh.dev, scene)) return rc;
    return RT_OK;
}

extern "C" int rt_multi_synchronize(rt_multi *m) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m) return rt_fail(RT_EINVAL, "rt_multi_synchronize: NULL argument");
    for (Shard &sh : m->s) {
        MHIP(hipSetDevice(sh.ordinal));
        MHIP(hipStreamSynchronize(sh.stream));
        MHIP(hipStreamSynchronize(sh.xfer));
        if (const int rc = rt_device_synchronize(sh.dev)) return rc;
    }
    MHIP(hipSetDevice(m->s[0].ordinal));
    MHIP(hipStreamSynchronize(m->gather));
    return RT_OK;
}

extern "C" int rt_multi_get_info(rt_multi *m, rt_multi_info *out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !out) return rt_fail(RT_EINVAL, "rt_multi_get_info: NULL argument");
    out->DeviceCount = (uint32_t)m->s.size();
    out->Transport = m->transport;
    out->BandRows = m->last_band_rows;
    out->MaxLocalRows = m->last_max_rows;
    // dead-tile segments of the last call: resolved per device (each may wait
    // for its cull pass's totals to reach the host, rt_trace_last_info)
    uint64_t folded = 0;
    for (Shard &sh : m->s)
        if (sh.launched) {
            rt_trace_info info;
            if (const int rc = rt_trace_last_info(sh.dev, &info)) return rc;
            folded += info.SegmentsFolded;
        }
    out->SegmentsFolded = folded;
    return RT_OK;
}

extern "C" int rt_multi_last_trace_ms(rt_multi *m, float *ms_out, uint32_t count) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !ms_out || count < m->s.size()) return rt_fail(RT_EINVAL, "rt_multi_last_trace_ms: bad argument");
    if (m->calls == 0) return rt_fail(RT_EINVAL, "rt_multi_last_trace_ms: no call yet");
    const uint32_t b = m->last_slot;
    for (size_t i = 0; i < m->s.size(); ++i) {
        Shard &sh = m->s[i];
        MHIP(hipSetDevice(sh.ordinal));
        MHIP(hipEventSynchronize(sh.t1[b]));
        MHIP(hipEventElapsedTime(&ms_out[i], sh.t0[b], sh.t1[b]));
    }
    return RT_OK;
}

extern "C" int rt_multi_last_gather_ms(rt_multi *m, float *ms_out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !ms_out) return rt_fail(RT_EINVAL, "rt_multi_last_gather_ms: NULL argument");
    if (m->calls == 0) return rt_fail(RT_EINVAL, "rt_multi_last_gather_ms: no call yet");
    MHIP(hipSetDevice(m->s[0].ordinal));
    MHIP(hipEventSynchronize(m->g1[m->last_slot]));
    MHIP(hipEventElapsedTime(ms_out, m->g0[m->last_slot], m->g1[m->last_slot]));
    return RT_OK;
}

extern "C" int rt_multi_shard_info(rt_multi *m, uint32_t index, rt_trace_info *out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !out || index >= m->s.size()) return rt_fail(RT_EINVAL, "rt_multi_shard_info: bad argument");
    if (!m->s[index].launched) return rt_fail(RT_EINVAL, "rt_multi_shard_info: device %u traced nothing in the last call", index);
    return rt_trace_last_info(m->s[index].dev, out);
}

extern "C" int rt_multi_reserve(rt_multi *m, uint32_t width, uint32_t height, uint32_t band_rows, uint32_t flags) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    const uint32_t R = band_rows ? band_rows : 8u;
    if (!m || width == 0 || height == 0 || width > 65536 || height > 65536 || R % 8u ||
        (flags & ~RT_MULTI_RESERVE_MEAN))
        return rt_fail(RT_EINVAL, "rt_multi_reserve: bad argument");
    if (const int rc = rt_multi_synchronize(m)) return rc;  // growing frees buffers in-flight calls may use
    const uint32_t n = (uint32_t)m->s.size();
    const uint32_t maxr = max_local_rows(height, R, n);
    for (Shard &sh : m->s) {
        MHIP(hipSetDevice(sh.ordinal));
        // growing a shard's resident running mean discards it (grow() does not
        // copy), so no continuation may blend onto the new buffer
        if ((size_t)maxr * width * 16u > sh.cap_prev) m->accum_valid = false;
        if (const int rc = grow(&sh.prev, &sh.cap_prev, (size_t)maxr * width * 16u)) return rc;
        size_t cap = sh.cap_cur;
        for (int b = 0; b < kSlots; ++b) {
            cap = sh.cap_cur;
            if (const int rc = grow(&sh.cur[b], &cap, (size_t)maxr * width * 4u)) return rc;
        }
        sh.cap_cur = cap;
        if (const int rc = rt_device_reserve(sh.dev, width, maxr)) return rc;
    }
    MHIP(hipSetDevice(m->s[0].ordinal));
    if (const int rc = grow(&m->stage_cur, &m->cap_stage_cur, (size_t)n * maxr * width * 4u)) return rc;
    if (flags & RT_MULTI_RESERVE_MEAN)
        if (const int rc = grow(&m->stage_prev, &m->cap_stage_prev, (size_t)n * maxr * width * 16u)) return rc;
    return RT_OK;
}

extern "C" int rt_multi_resident_frames(rt_multi *m, uint64_t *out) {
    if (!m || !out) return rt_fail(RT_EINVAL, "rt_multi_resident_frames: NULL argument");
    *out = m->accum_valid ? m->resident_frames : 0u;
    return RT_OK;
}

static int multi_trace(rt_multi *m, const rt_camera_info *cam, const rt_trace_desc *desc, uint64_t *d_rays,
                       hipStream_t caller, bool restart, bool same_geometry);

extern "C" int rt_multi_trace(rt_multi *m, const rt_camera_info *cam, const rt_trace_desc *desc, uint64_t *d_rays,
                              void *stream) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!m || !cam || !desc || !d_rays) return rt_fail(RT_EINVAL, "rt_multi_trace: NULL argument");
    if (desc->BandCount != 0 || desc->BandIndex != 0)
        return rt_fail(RT_EINVAL, "rt_multi_trace: BandCount/BandIndex must be 0 (bands are dealt over the devices)");
    const uint32_t W = desc->Width, H = desc->Height, R = desc->BandRows ? desc->BandRows : 8u;
    if (W == 0 || H == 0 || W > 65536 || H > 65536 || R % 8u)
        return rt_fail(RT_EINVAL, "rt_multi_trace: bad geometry %ux%u, BandRows %u", W, H, R);
    if (!cam->CurrentImage.Data) return rt_fail(RT_EINVAL, "rt_multi_trace: CurrentImage device pointer missing");
    const bool restart = (desc->Flags & RT_FLAG_ACCUM_ZERO) || desc->PreviousRayCount == 0;
    const bool same_geometry = m->width == W && m->height == H && m->band_rows == R;
    if (!restart && !(same_geometry && m->accum_valid))
        return rt_fail(RT_EINVAL, "rt_multi_trace: PreviousRayCount %u but no resident running mean for this geometry",
                       desc->PreviousRayCount);
    // the resident means hold resident_frames frames: a continuation must say so,
    // or its weights (main.cpp:484-487) would blend the wrong way
    if (!restart && desc->PreviousRayCount != m->resident_frames)
        return rt_fail(RT_EINVAL, "rt_multi_trace: PreviousRayCount %u but the resident running mean holds %llu frames",
                       desc->PreviousRayCount, (unsigned long long)m->resident_frames);
    const int rc = multi_trace(m, cam, desc, d_rays, (hipStream_t)stream, restart, same_geometry);
    if (rc) {  // some shards may have traced (restarting their means), others not
        m->accum_valid = false;
        return rc;
    }
    if (restart) {
        // the frames were folded with the weights of PreviousRayCount + k (an
        // ACCUM_ZERO launch may start at any count), so a continuation names
        // PreviousRayCount + Frames, exactly as for one device's rt_trace
        m->accum_valid = desc->Frames > 0;
        m->resident_frames = (uint64_t)desc->PreviousRayCount + desc->Frames;
    } else {
        m->resident_frames += desc->Frames;
    }
    return RT_OK;
}

static int multi_trace(rt_multi *m, const rt_camera_info *cam, const rt_trace_desc *desc, uint64_t *d_rays,
                       hipStream_t caller, bool restart, bool same_geometry) {
    const uint32_t n = (uint32_t)m->s.size();
    const uint32_t W = desc->Width, H = desc->Height, R = desc->BandRows ? desc->BandRows : 8u;
    const uint32_t maxr = max_local_rows(H, R, n);
    const bool want_prev = cam->PreviousImage.Data != nullptr;
    const int d0 = m->s[0].ordinal;
    // resident per-device images (a geometry change drops the running means)
    if (!same_geometry) {
        if (const int rc = rt_multi_synchronize(m)) return rc;
        m->accum_valid = false;
    }
    for (Shard &sh : m->s) {
        MHIP(hipSetDevice(sh.ordinal));
        if ((size_t)maxr * W * 16u > sh.cap_prev || (size_t)maxr * W * 4u > sh.cap_cur) {
            MHIP(hipStreamSynchronize(sh.stream));
            MHIP(hipStreamSynchronize(sh.xfer));
            if (const int rc = grow(&sh.prev, &sh.cap_prev, (size_t)maxr * W * 16u)) return rc;
            size_t cap = sh.cap_cur;
            for (int b = 0; b < kSlots; ++b) {
                cap = sh.cap_cur;
                if (const int rc = grow(&sh.cur[b], &cap, (size_t)maxr * W * 4u)) return rc;
            }
            sh.cap_cur = cap;
        }
    }
    MHIP(hipSetDevice(d0));
    {
        const size_t need_cur = (size_t)n * maxr * W * 4u, need_prev = want_prev ? (size_t)n * maxr * W * 16u : 0u;
        if (need_cur > m->cap_stage_cur || need_prev > m->cap_stage_prev) {
            MHIP(hipStreamSynchronize(m->gather));
            if (const int rc = grow(&m->stage_cur, &m->cap_stage_cur, need_cur)) return rc;
            if (need_prev)
                if (const int rc = grow(&m->stage_prev, &m->cap_stage_prev, need_prev)) return rc;
        }
    }
    m->width = W, m->height = H, m->band_rows = R;
    const uint32_t b = m->calls & 1u;
    // The traces read nothing of the caller's: they wait only until their slot
    // has been gathered (two calls back) and, when the last call gathered the
    // resident means they overwrite, until that gather is done.  Everything the
    // caller sees (frame, mean, d_rays) is written on the gather stream, after
    // the caller's prior work on `stream`.
    MHIP(hipEventRecord(m->start, caller));
    const uint32_t pb = b ^ 1u;
    for (uint32_t i = 0; i < n; ++i) {
        Shard &sh = m->s[i];
        MHIP(hipSetDevice(sh.ordinal));
        if (m->slot_used[b]) MHIP(hipStreamWaitEvent(sh.stream, m->transport == RT_MULTI_RCCL ? sh.sent[b] : m->copied[b], 0));
        if (m->prev_gathered && m->slot_used[pb])
            MHIP(hipStreamWaitEvent(sh.stream, m->transport == RT_MULTI_RCCL ? sh.sent[pb] : m->copied[pb], 0));
        MHIP(hipMemsetAsync(sh.rays[b], 0, sizeof(uint64_t), sh.stream));
        rt_camera_info c = *cam;
        c.CurrentImage.Data = sh.cur[b];
        c.PreviousImage.Data = sh.prev;
        rt_trace_desc d = *desc;
        d.BandRows = R;
        d.BandCount = n;
        d.BandIndex = i;
        if (restart) d.Flags |= RT_FLAG_ACCUM_ZERO;
        MHIP(hipEventRecord(sh.t0[b], sh.stream));
        if (const int rc = rt_trace(sh.dev, &c, &d, sh.rays[b], sh.stream)) return rc;
        MHIP(hipEventRecord(sh.t1[b], sh.stream));
        MHIP(hipEventRecord(sh.traced[b], sh.stream));
        sh.launched = rt_band_local_rows(H, R, n, i) > 0 && desc->Frames > 0;
    }
    // gather to devices[0]: compact images -> staging (rank-strided), then scatter
    const uint64_t stride_cur = (uint64_t)maxr * W * 4u, stride_prev = (uint64_t)maxr * W * 16u;
    if (m->transport == RT_MULTI_RCCL) {
        // sends leave from each device's transfer stream, so its next trace
        // (the other slot) does not queue behind them
        for (Shard &sh : m->s) {
            MHIP(hipSetDevice(sh.ordinal));
            MHIP(hipStreamWaitEvent(sh.xfer, sh.traced[b], 0));
        }
        MHIP(hipSetDevice(d0));
        for (Shard &sh : m->s) MHIP(hipStreamWaitEvent(m->gather, sh.traced[b], 0));
        MHIP(hipEventRecord(m->g0[b], m->gather));
        const Rccl &r = rccl();
        NCCL_OK(r.GroupStart());
        for (uint32_t i = 0; i < n; ++i) {
            Shard &sh = m->s[i];
            const size_t bc = band_bytes(W, H, R, n, i, 4u);
            if (bc) NCCL_OK(r.Send(sh.cur[b], bc, ncclUint8, 0, sh.comm, sh.xfer));
            if (bc && want_prev) NCCL_OK(r.Send(sh.prev, bc * 4u, ncclUint8, 0, sh.comm, sh.xfer));
            NCCL_OK(r.Send(sh.rays[b], 1, ncclUint64, 0, sh.comm, sh.xfer));
        }
        for (uint32_t i = 0; i < n; ++i) {
            const size_t bc = band_bytes(W, H, R, n, i, 4u);
            if (bc) NCCL_OK(r.Recv(m->stage_cur + i * stride_cur, bc, ncclUint8, (int)i, m->s[0].comm, m->gather));
            if (bc && want_prev)
                NCCL_OK(r.Recv(m->stage_prev + i * stride_prev, bc * 4u, ncclUint8, (int)i, m->s[0].comm, m->gather));
            NCCL_OK(r.Recv(m->ray_slots + i, 1, ncclUint64, (int)i, m->s[0].comm, m->gather));
        }
        NCCL_OK(r.GroupEnd());
        for (Shard &sh : m->s) {
            MHIP(hipSetDevice(sh.ordinal));
            MHIP(hipEventRecord(sh.sent[b], sh.xfer));
        }
        MHIP(hipSetDevice(d0));
    } else {
        MHIP(hipSetDevice(d0));
        for (Shard &sh : m->s) MHIP(hipStreamWaitEvent(m->gather, sh.traced[b], 0));
        MHIP(hipEventRecord(m->g0[b], m->gather));
        for (uint32_t i = 0; i < n; ++i) {
            Shard &sh = m->s[i];
            const size_t bc = band_bytes(W, H, R, n, i, 4u);
            if (bc) MHIP(hipMemcpyPeerAsync(m->stage_cur + i * stride_cur, d0, sh.cur[b], sh.ordinal, bc, m->gather));
            if (bc && want_prev)
                MHIP(hipMemcpyPeerAsync(m->stage_prev + i * stride_prev, d0, sh.prev, sh.ordinal, bc * 4u, m->gather));
            MHIP(hipMemcpyPeerAsync(m->ray_slots + i, d0, sh.rays[b], sh.ordinal, sizeof(uint64_t), m->gather));
        }
        MHIP(hipEventRecord(m->copied[b], m->gather));
    }
    m->slot_used[b] = true;
    m->prev_gathered = want_prev;
    MHIP(hipStreamWaitEvent(m->gather, m->start, 0));  // d_rays and the output follow the caller's prior work
    if (rtk_launch_assemble(m->stage_cur, stride_cur, cam->CurrentImage.Data, W, H, 4u, R, n, m->gather) != 0 ||
        (want_prev &&
         rtk_launch_assemble(m->stage_prev, stride_prev, cam->PreviousImage.Data, W, H, 16u, R, n, m->gather) != 0) ||
        rtk_launch_sum_u64(m->ray_slots, n, d_rays, m->gather) != 0)
        return rt_fail(RT_EIO, "rt_multi_trace: gather launch failed: %s", hipGetErrorString(hipGetLastError()));
    MHIP(hipEventRecord(m->g1[b], m->gather));
    MHIP(hipEventRecord(m->gathered, m->gather));
    MHIP(hipStreamWaitEvent(caller, m->gathered, 0));
    m->last_band_rows = R;
    m->last_max_rows = maxr;
    m->last_slot = b;
    m->calls += 1;
    return RT_OK;
}

// ------------------------------------------------------------------ rt_comm
struct rt_comm {
    int ordinal = 0;
    uint32_t nranks = 1, rank = 0;
    ncclComm_t comm = nullptr;
    uint8_t *stage = nullptr;  // rank 0: nranks compact images, rank-strided
    size_t cap_stage = 0;
};

extern "C" int rt_comm_unique_id(void *id_out) {
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id_out) return rt_fail(RT_EINVAL, "rt_comm_unique_id: NULL argument");
    if (!rccl().ok) return rt_fail(RT_ENODEV, "rt_comm_unique_id: librccl.so.1 not loadable");
    ncclUniqueId id;
    NCCL_OK(rccl().GetUniqueId(&id));
    memcpy(id_out, &id, sizeof(id));
    return RT_OK;
}

extern "C" int rt_comm_create(int hip_device, const void *id, uint32_t nranks, uint32_t rank, rt_comm **out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!id || !out || nranks == 0 || rank >= nranks) return rt_fail(RT_EINVAL, "rt_comm_create: bad argument");
    *out = nullptr;
    if (!rccl().ok) return rt_fail(RT_ENODEV, "rt_comm_create: librccl.so.1 not loadable");
    MHIP(hipSetDevice(hip_device));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = rccl().CommInitRank(&comm, (int)nranks, uid, (int)rank);
    if (r != ncclSuccess) return rt_fail(RT_ENODEV, "rt_comm_create: ncclCommInitRank: %s", rccl().GetErrorString(r));
    rt_comm *c = new rt_comm();
    c->ordinal = hip_device;
    c->nranks = nranks;
    c->rank = rank;
    c->comm = comm;
    *out = c;
    return RT_OK;
}

extern "C" int rt_comm_destroy(rt_comm *c) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c) return RT_OK;
    (void)hipSetDevice(c->ordinal);
    (void)hipDeviceSynchronize();
    if (c->comm) (void)rccl().CommDestroy(c->comm);
    (void)hipFree(c->stage);
    delete c;
    return RT_OK;
}

extern "C" int rt_comm_gather_bands(rt_comm *c, const void *d_local, void *d_full, uint32_t width, uint32_t height,
                                    uint32_t elem_bytes, uint32_t band_rows, void *stream) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c || width == 0 || height == 0 || elem_bytes == 0 || band_rows == 0 || band_rows % 8u)
        return rt_fail(RT_EINVAL, "rt_comm_gather_bands: bad argument");
    const uint32_t n = c->nranks;
    const size_t mine = band_bytes(width, height, band_rows, n, c->rank, elem_bytes);
    if ((mine && !d_local) || (c->rank == 0 && !d_full)) return rt_fail(RT_EINVAL, "rt_comm_gather_bands: NULL buffer");
    hipStream_t s = (hipStream_t)stream;
    MHIP(hipSetDevice(c->ordinal));
    const uint64_t stride = (uint64_t)max_local_rows(height, band_rows, n) * width * elem_bytes;
    if (c->rank == 0 && (size_t)n * stride > c->cap_stage) {
        MHIP(hipDeviceSynchronize());
        if (const int rc = grow(&c->stage, &c->cap_stage, (size_t)n * stride)) return rc;
    }
    const Rccl &r = rccl();
    NCCL_OK(r.GroupStart());
    if (c->rank == 0)
        for (uint32_t k = 0; k < n; ++k) {
            const size_t b = band_bytes(width, height, band_rows, n, k, elem_bytes);
            if (b) NCCL_OK(r.Recv(c->stage + k * stride, b, ncclUint8, (int)k, c->comm, s));
        }
    if (mine) NCCL_OK(r.Send(d_local, mine, ncclUint8, 0, c->comm, s));
    NCCL_OK(r.GroupEnd());
    if (c->rank == 0 && rtk_launch_assemble(c->stage, stride, d_full, width, height, elem_bytes, band_rows, n, s) != 0)
        return rt_fail(RT_EIO, "rt_comm_gather_bands: assembly launch failed");
    return RT_OK;
}
