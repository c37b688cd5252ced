// rt_host.cpp — C-ABI host side: device context, scene upload, trace launch,
// band assembly.  Plain HIP runtime; no torch types cross this boundary.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rt_kernel.h"
#include "rt_trace.h"

struct rt_device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    float *d_lut = nullptr;                // 2048 f32
    bool lut_set = false;
    // SIMD rule set (SIMDSpheres + Materials) and scalar rule set (ScalarSpheres)
    float4 *d_groups[2] = {nullptr, nullptr};
    float2 *d_weights = nullptr;  // TraceArgs.weights: kWeightsN running-mean weight pairs
    // the primary rounds' camera-relative group rows (TraceArgs.prim), written by the cull pass
    float4 *d_prim[2] = {nullptr, nullptr};
    float4 *d_mats[2] = {nullptr, nullptr};
    uint32_t n_groups[2] = {0, 0};
    uint32_t n_spheres = 0;
    size_t cap_groups[2] = {0, 0};
    bool scene_set = false;
    bool use_sky = false;
    int src = kSrcSmem;
    int cull = 1;
    uint32_t sec_threshold = 0;  // 0: per scene (rt_trace), else rt_device_options SecondaryThreshold
    int prefilter_env = -1;  // options Prefilter: -1 auto, 0 off, 1 on
    uint32_t prefilter[2] = {0, 0};  // per rule set, decided at upload
    uint32_t pf_relative[2] = {0, 0};  // per rule set: row 3 holds r^2, per-lane thresholds (rt_kernel.hip kPfRel)
    int pf_rel_env = -1;  // options PrefilterRelative: -1 auto (where the scene-wide bound does not pay), 0 never, 1 always
    uint32_t fast_sqrt[2] = {0, 0};  // per rule set: candidate sqrt in sqrt_rn's verified range
    float4 *d_clusters[2] = {nullptr, nullptr};  // clustered prefilter tables (cluster_table)
    size_t cap_clusters[2] = {0, 0};             // float4 capacity
    uint32_t n_cpairs[2] = {0, 0};               // 0: per-group prefilter loop
    uint32_t cl_words[2] = {0, 0};
    // options Clusters off (0): per-group prefilter loop only; on (2): clustered loop up to
    // kClMaxGroups groups; default 1: up to kClAutoGroups (measured: clusters
    // win 13-15 % at 16/24/32 groups on C2 geometry, and at C5's 64 groups
    // 32.4k against 28.6k Mrays/s once the behind rule and the 7-block LDS
    // image are in)
    int clusters_env = 1;
    int interleave_env = 0;  // options Interleave: wave tiles interleaved over the block tile (P >= 2)
    int scene_global_env = 0;  // options SceneInHbm: keep the scene in HBM even when the LDS image could hold it
    int tables_global_env = 0;  // options TablesInLds off: the rsqrt and fold-weight tables stay out of the LDS image
    int solo_env = 1;           // options OneWaveGroups off: four waves per workgroup sharing an LDS image (TraceArgs.solo)
    int wave_order_env = 1;     // options WaveOrder off: one-wave kernels order block tiles, not waves (A/B)
    int walk_any_env = 0;       // options WalkAny: the one-wave kernel dispatches the walk at run time (A/B)
    int lanes_per_pixel = 0;  // 0 = auto per launch (rt_trace), else forced by options LanesPerPixel
    // options PixelsPerLane: 0 auto (4 pixels per lane for one-lane-per-pixel launches of one
    // frame), 1 never, 4 for every one-lane-per-pixel launch (A/B and the parity suite)
    int pixels_per_lane_env = 0;
    // each block tile's pixels dealt to its waves by the cost the last launch
    // measured (rtk_launch_pixel_sort), at P >= 4; options PixelSort off turns it off.
    // Same box: C2 158.7-159.3k -> 164.6-166.4k Mrays/s, RTWeekend 22.4k -> 23.3k
    int pixel_sort_env = 1;
    // pixels per dealt unit (TraceArgs.pix_seg), options PixelSegment 1/2/4: 4-pixel row segments keep
    // each wave's stores to whole 64-B runs of the v4 image (HBM writes per launch: C2 20.9 ->
    // 17.5 MB, RTWeekend 80.2 -> 57.3 MB) but deal costs coarser: C2 -2.2 %, RTWeekend -4 %
    // (profiles/r05b_pixel_seg_ab.txt), so single pixels stay the default
    uint32_t pixel_seg = 1;
    // options XcdGroup: every wave of a block tile on one XCD (rtk_launch_xcd_group), so its lines'
    // partial stores merge in one L2 before they are written back
    // off/on forces it; by default it is on for launches of at most 4 lanes per pixel (the
    // whole frame, where it halves the trace kernel's HBM writes at no cost) and off for the multi-GPU shares
    // (8 and 16 lanes per pixel: small launches, whose partial-line writes are a few MB, and the 8-rank share
    // -2.3 % without it at the final kernel, profiles/r05z6_xcd_group_ab.txt)
    int xcd_group_env = -1;
    // RGBA8 encoded from the running mean by a coalesced pass after the launch (TraceArgs.skip_cur),
    // at P >= 2: trace-kernel HBM writes C2 21.0 -> 15.7 MB, RTWeekend 80.6 -> 54.1 MB, C2 +0.7 %
    // (profiles/r05e_cur_pass_ab.txt); options EncodePass off stores RGBA8 in the trace kernel
    uint32_t cur_pass = 1;
    int merge_env = -1;  // options MergeRounds: -1 auto (scenes of at most kMergeGroups groups), 0 never, 1 always
    uint8_t *d_pix_perm = nullptr;  // 64 B per block tile (TraceArgs.pix_perm)
    uint32_t *d_pix_cost = nullptr; // per band pixel (TraceArgs.pix_cost)
    size_t pix_perm_cap = 0, pix_cost_cap = 0;
    // heaviest-first tile order learned from the previous launch of the same
    // geometry (options TileOrder off disables); launches must be stream-ordered
    int tile_sched = 1;
    uint32_t n_sorts = 0;             // re-sorts done for the current tile key
    int split_env = 1;                // options SplitFirstLaunch off: a key's first launch is not split (below)
    uint32_t head_samples = 8;        // samples per lane of the split's head (options HeadSamples)
    uint32_t split_parts = 2;         // launches of a split first launch (options SplitParts, <= 8)
    uint32_t split_growth = 3;        // each leading part this many times the previous (options SplitGrowth)
    // options OrderLaunches: re-sorts per key before the order is kept.  4 (a key's split first launch
    // sorts twice, then two more launches): as fast as 6 at steady state on C2 and the 8-rank share,
    // 3 is slower (profiles/r05q_order_launches_ab.txt), and a bench's timed launches are past the
    // sorting ones after two warm-ups
    uint32_t order_launches = 4;
    uint32_t *d_tile_cost = nullptr, *d_tile_order = nullptr, *d_tile_scratch = nullptr;
    uint32_t *d_tile_order_sorted = nullptr;  // the sort's output before XCD grouping (rtk_launch_xcd_group)
    uint32_t *d_tile_aux = nullptr;           // XCD grouping: per block tile, first sorted position and group
    uint32_t *d_tile_live = nullptr;
    unsigned long long *d_cull_counters = nullptr;  // kCullCounterWords: striped counters + device totals of the cull pass
    uint64_t *d_masks = nullptr;  // cull pass output: per wave tile primary group masks
    size_t tile_cap = 0, mask_cap = 0;
    // rt_device_reserve: the most block tiles (over every lanes-per-pixel shape)
    // and band pixels of any geometry reserved so far (0: none)
    uint32_t reserve_tiles = 0;
    size_t reserve_pixels = 0;
    size_t mask_words = 0;  // words the last cull pass wrote (rt_debug_masks)
    // the launch (camera, scene, geometry) the masks / live list / order were made for
    std::vector<uint32_t> tile_key;
    bool tile_order_valid = false;
    // The cull pass's totals travel to the host asynchronously (pinned h_counts,
    // event ev_counts): a new key never blocks the host.  Until they have
    // landed (counts_known), launches size their grids for every tile and read
    // the live count on the device (TraceArgs.live_total).
    uint32_t n_live = 0;
    uint64_t dead_pixels = 0;
    bool counts_known = true;
    unsigned long long *h_counts = nullptr;  // pinned {live tiles, dead pixels}
    hipEvent_t ev_counts = nullptr;
    uint64_t scene_gen = 0;  // bumped by every rt_scene_upload
    // the last stream rt_trace ran on (a switch waits for the device: below)
    hipStream_t tile_stream = nullptr;
    bool tile_stream_set = false;
    // what rt_trace_last_info resolves lazily (the folded segments need the counts)
    uint32_t last_n_tiles = 0, last_frames = 0;
    bool last_empty_capable = false;
    uint32_t cu_count = 256;
    unsigned long long *d_stats = nullptr;  // RT_STATS=1: per-launch scheduling counters
    unsigned long long *d_wave_times = nullptr;  // RT_WAVETIMES=1: per-wave start/end of the last launch
    size_t wave_times_cap = 0;
    bool want_wave_times = false;
    rt_trace_info last{};  // what the last rt_trace launched (rt_trace_last_info)
    rt_device_options opt{};  // as created (rt_device_get_options)
    uint32_t cluster_k = 0, sub_spheres = 0;  // cluster_table's K and sub-cluster size (0: per scene)
};

static thread_local char g_err[512];

static int vfail(int code, const char *fmt, va_list ap) {
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    return code;
}

static int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

// rt_kernel.h: the error text other translation units (rt_multi.cpp) report
int rt_fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_OK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(RT_EIO, "%s: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

extern "C" const char *rt_last_error(void) { return g_err; }

extern "C" int rt_device_create(int hip_device, rt_device **out) { return rt_device_create_ex(hip_device, nullptr, out); }

// rt_device_options -> the device's switches (rt_trace.h: 0 = the default, RT_OPT_ON / RT_OPT_OFF)
static int apply_options(rt_device *d, const rt_device_options *o) {
    if (!o) return RT_OK;
    if (o->Size != 0 && o->Size != sizeof(rt_device_options))
        return fail(RT_EINVAL, "rt_device_options: Size %u, this library's is %zu", o->Size, sizeof(rt_device_options));
    const int32_t tri[] = {o->Cull, o->Prefilter, o->PrefilterRelative, o->Clusters, o->OneWaveGroups,
                           o->SphereSourceLds, o->SceneInHbm, o->TablesInLds, o->WalkAny, o->Interleave,
                           o->MergeRounds, o->TileOrder, o->WaveOrder, o->PixelSort, o->XcdGroup,
                           o->SplitFirstLaunch, o->EncodePass};
    for (const int32_t v : tri)
        if (v < -1 || v > 1) return fail(RT_EINVAL, "rt_device_options: a switch is %d (RT_OPT_DEFAULT/ON/OFF)", v);
    const int32_t lpp = o->LanesPerPixel;
    if (!(lpp == 0 || lpp == 1 || lpp == 2 || lpp == 4 || lpp == 8 || lpp == 16 || lpp == 32))
        return fail(RT_EINVAL, "rt_device_options: LanesPerPixel %d", lpp);
    if (!(o->PixelsPerLane == 0 || o->PixelsPerLane == 1 || o->PixelsPerLane == 4))
        return fail(RT_EINVAL, "rt_device_options: PixelsPerLane %d", o->PixelsPerLane);
    if (!(o->PixelSegment == 0 || o->PixelSegment == 1 || o->PixelSegment == 2 || o->PixelSegment == 4))
        return fail(RT_EINVAL, "rt_device_options: PixelSegment %d", o->PixelSegment);
    if (o->SplitParts < 0 || o->SplitParts > 8 || o->HeadSamples < 0 || o->SplitGrowth < 0 || o->OrderLaunches < -1 ||
        o->SecondaryThreshold < 0 || o->SecondaryThreshold > 64 || o->ClusterCount < 0 || o->ClusterCount == 1 ||
        o->SubClusterSpheres < 0)
        return fail(RT_EINVAL, "rt_device_options: a count is out of range");
    auto on = [](int32_t v, bool dflt) { return v == RT_OPT_DEFAULT ? dflt : v == RT_OPT_ON; };
    d->opt = *o;
    d->opt.Size = sizeof(rt_device_options);
    d->cull = on(o->Cull, true) ? 1 : 0;
    d->prefilter_env = o->Prefilter == RT_OPT_DEFAULT ? -1 : o->Prefilter == RT_OPT_ON ? 1 : 0;
    d->pf_rel_env = o->PrefilterRelative == RT_OPT_DEFAULT ? -1 : o->PrefilterRelative == RT_OPT_ON ? 1 : 0;
    d->clusters_env = o->Clusters == RT_OPT_DEFAULT ? 1 : o->Clusters == RT_OPT_ON ? 2 : 0;
    d->cluster_k = (uint32_t)o->ClusterCount;
    d->sub_spheres = (uint32_t)o->SubClusterSpheres;
    d->sec_threshold = (uint32_t)o->SecondaryThreshold;
    d->lanes_per_pixel = lpp;
    d->pixels_per_lane_env = o->PixelsPerLane;
    d->solo_env = on(o->OneWaveGroups, true) ? 1 : 0;
    d->src = on(o->SphereSourceLds, false) ? kSrcLds : kSrcSmem;
    d->scene_global_env = on(o->SceneInHbm, false) ? 1 : 0;
    d->tables_global_env = on(o->TablesInLds, true) ? 0 : 1;
    d->walk_any_env = on(o->WalkAny, false) ? 1 : 0;
    d->interleave_env = on(o->Interleave, false) ? 1 : 0;
    d->merge_env = o->MergeRounds == RT_OPT_DEFAULT ? -1 : o->MergeRounds == RT_OPT_ON ? 1 : 0;
    d->tile_sched = on(o->TileOrder, true) ? 1 : 0;
    d->wave_order_env = on(o->WaveOrder, true) ? 1 : 0;
    d->pixel_sort_env = on(o->PixelSort, true) ? 1 : 0;
    if (o->PixelSegment) d->pixel_seg = (uint32_t)o->PixelSegment;
    d->xcd_group_env = o->XcdGroup == RT_OPT_DEFAULT ? -1 : o->XcdGroup == RT_OPT_ON ? 1 : 0;
    d->split_env = on(o->SplitFirstLaunch, true) ? 1 : 0;
    if (o->HeadSamples) d->head_samples = (uint32_t)o->HeadSamples;
    if (o->SplitParts) d->split_parts = (uint32_t)o->SplitParts;
    if (o->SplitGrowth) d->split_growth = (uint32_t)o->SplitGrowth;
    if (o->OrderLaunches) d->order_launches = o->OrderLaunches < 0 ? 0u : (uint32_t)o->OrderLaunches;
    d->cur_pass = on(o->EncodePass, true) ? 1u : 0u;
    return RT_OK;
}

extern "C" int rt_device_get_options(rt_device *d, rt_device_options *out) {
    if (!d || !out) return fail(RT_EINVAL, "rt_device_get_options: NULL argument");
    *out = d->opt;
    return RT_OK;
}

extern "C" int rt_device_create_ex(int hip_device, const rt_device_options *options, rt_device **out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!out) return fail(RT_EINVAL, "rt_device_create: out is NULL");
    {  // options are checked before anything touches a device (a host-only rt_device)
        rt_device probe;
        if (const int rc = apply_options(&probe, options)) return rc;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(RT_ENODEV, "rt_device_create: no HIP device visible");
    if (hip_device < 0 || hip_device >= count) return fail(RT_EINVAL, "rt_device_create: bad device %d", hip_device);
    HIP_OK(hipSetDevice(hip_device));
    rt_device *d = new rt_device();
    d->ordinal = hip_device;
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d->d_lut, 2048 * sizeof(float)) != hipSuccess ||
        hipMalloc(&d->d_weights, kWeightsN * sizeof(float2)) != hipSuccess ||
        hipHostMalloc(&d->h_counts, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_counts, hipEventDisableTiming) != hipSuccess) {
        rt_device_destroy(d);
        return fail(RT_ENOMEM, "rt_device_create: stream/LUT/event allocation failed");
    }
    {
        // IEEE f32 divisions (this file is built with -ffp-contract=off): the bits of the kernel's
        // rcp_rn / div_rn weights, which reproduce the reference's divisions (main.cpp:484-487)
        std::vector<float2> w(kWeightsN);
        for (uint32_t n = 0; n < kWeightsN; ++n) {
            const float d1 = (float)(n + 1u);
            w[n] = make_float2(1.0f / d1, (float)n / d1);
        }
        if (hipMemcpy(d->d_weights, w.data(), kWeightsN * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
            rt_device_destroy(d);
            return fail(RT_EIO, "rt_device_create: weight table upload failed");
        }
    }
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, hip_device) == hipSuccess && prop.multiProcessorCount > 0)
            d->cu_count = (uint32_t)prop.multiProcessorCount;
    }
    if (const int rc = apply_options(d, options)) {
        rt_device_destroy(d);
        return rc;
    }
    // diagnostic hooks only (the -DRTK_STATS build's counters, per-wave timestamps): what is
    // computed, and how, is fixed by the options
    const char *wt = getenv("RT_WAVETIMES");
    d->want_wave_times = wt && wt[0] == '1';
    const char *st = getenv("RT_STATS");
    if (st && st[0] == '1' && hipMalloc(&d->d_stats, kStatSlots * sizeof(unsigned long long)) == hipSuccess)
        (void)hipMemset(d->d_stats, 0, kStatSlots * sizeof(unsigned long long));
    *out = d;
    return RT_OK;
}

extern "C" int rt_device_destroy(rt_device *d) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d) return RT_OK;
    (void)hipSetDevice(d->ordinal);
    // the caller's trace stream may already be gone: wait for the whole device
    (void)hipDeviceSynchronize();
    for (int r = 0; r < 2; ++r) {
        (void)hipFree(d->d_groups[r]);
        (void)hipFree(d->d_prim[r]);
        (void)hipFree(d->d_mats[r]);
        (void)hipFree(d->d_clusters[r]);
    }
    (void)hipFree(d->d_lut);
    (void)hipFree(d->d_weights);
    (void)hipFree(d->d_stats);
    (void)hipFree(d->d_wave_times);
    (void)hipFree(d->d_tile_cost);
    (void)hipFree(d->d_tile_order);
    (void)hipFree(d->d_tile_order_sorted);
    (void)hipFree(d->d_tile_aux);
    (void)hipFree(d->d_tile_scratch);
    (void)hipFree(d->d_tile_live);
    (void)hipFree(d->d_cull_counters);
    (void)hipFree(d->d_masks);
    (void)hipFree(d->d_pix_perm);
    (void)hipFree(d->d_pix_cost);
    if (d->h_counts) (void)hipHostFree(d->h_counts);
    if (d->ev_counts) (void)hipEventDestroy(d->ev_counts);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
    return RT_OK;
}

static int apply_reserve(rt_device *d);  // (rt_device_reserve, below)

// rt_trace is asynchronous on the caller's stream, while uploads go through
// the device's own non-blocking stream: before a buffer a trace may still
// read (scene groups, materials, cluster table, rsqrt table) is overwritten,
// every launch issued so far must have finished.  The wait is for the whole
// device, not on the caller's stream, which the caller may have destroyed
// since (and no per-launch event is recorded for it: an event marker between
// consecutive launches measured 4.6 us of dispatch gap, 0.6 % of an 8-GPU
// band share).  Uploads are rare; the extra wait for unrelated work is the price.
static int quiesce(rt_device *d) {
    (void)d;
    HIP_OK(hipDeviceSynchronize());
    return RT_OK;
}

// Brings the cull pass's totals to the host once they have landed (wait:
// block until they have).  Returns whether they are known.
static bool resolve_counts(rt_device *d, bool wait) {
    if (d->counts_known) return true;
    if (wait) {
        if (hipEventSynchronize(d->ev_counts) != hipSuccess) return false;
    } else {
        const hipError_t q = hipEventQuery(d->ev_counts);
        if (q != hipSuccess) {
            (void)hipGetLastError();  // "not ready" must not reach a later launch check
            return false;
        }
    }
    d->n_live = (uint32_t)d->h_counts[0];
    d->dead_pixels = d->h_counts[1];
    d->counts_known = true;
    return true;
}

extern "C" int rt_set_rsqrt_table(rt_device *d, const float table[2048]) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !table) return fail(RT_EINVAL, "rt_set_rsqrt_table: NULL argument");
    HIP_OK(hipSetDevice(d->ordinal));
    if (const int rc = quiesce(d)) return rc;
    HIP_OK(hipMemcpyAsync(d->d_lut, table, 2048 * sizeof(float), hipMemcpyHostToDevice, d->stream));
    HIP_OK(hipStreamSynchronize(d->stream));
    d->lut_set = true;
    return RT_OK;
}

// Packs one rule set: positions/radii as 4-wide groups with r*r precomputed,
// sphere records as {centre.xyz, 0}, {Color.xyz, Specular}, {Emissive.xyz, IOR}, {0} (kSphereF4).
static int upload_set(rt_device *d, int rs, const std::vector<float> &groups, const std::vector<float> &mats,
                      uint32_t n_groups) {
    if (n_groups > d->cap_groups[rs]) {
        (void)hipFree(d->d_groups[rs]);
        (void)hipFree(d->d_mats[rs]);
        (void)hipFree(d->d_prim[rs]);
        d->d_groups[rs] = nullptr;
        d->d_mats[rs] = nullptr;
        d->d_prim[rs] = nullptr;
        // +2 padding groups: the kernel's loops prefetch up to group g+2 while testing g
        if (hipMalloc(&d->d_groups[rs], (size_t)(n_groups + 2) * kGroupF4 * 16) != hipSuccess ||
            hipMalloc(&d->d_mats[rs], (size_t)n_groups * 64u * kSphereF4) != hipSuccess ||
            hipMalloc(&d->d_prim[rs], (size_t)n_groups * kPrimF4 * 16) != hipSuccess)
            return fail(RT_ENOMEM, "rt_scene_upload: device allocation failed");
        d->cap_groups[rs] = n_groups;
    }
    HIP_OK(hipMemsetAsync(d->d_groups[rs] + kGroupF4 * (size_t)n_groups, 0, 2 * kGroupF4 * 16, d->stream));
    HIP_OK(hipMemcpyAsync(d->d_groups[rs], groups.data(), (size_t)n_groups * kGroupF4 * 16, hipMemcpyHostToDevice,
                          d->stream));
    HIP_OK(hipMemcpyAsync(d->d_mats[rs], mats.data(), (size_t)n_groups * 64u * kSphereF4, hipMemcpyHostToDevice,
                          d->stream));
    d->n_groups[rs] = n_groups;
    return RT_OK;
}

static void put_material(float *dst, const rt_material &m) {
    dst[0] = m.Color.x;
    dst[1] = m.Color.y;
    dst[2] = m.Color.z;
    dst[3] = m.Specular;
    dst[4] = m.Emissive.x;
    dst[5] = m.Emissive.y;
    dst[6] = m.Emissive.z;
    dst[7] = m.IndexOfRefraction;
    // row 3: the dielectric path's per-material quotients, the reference's own f32 divisions done
    // once here (IEEE, as the kernel's were): eta outside = 1/IOR (main.cpp:463) and Reflectance's
    // r0 = ((1 - eta)/(1 + eta))^2 (main.cpp:292-295) for eta outside and inside (= IOR)
    if (m.IndexOfRefraction != 0.0f) {
        const float ior = m.IndexOfRefraction, eo = 1.0f / ior;
        const float ro = (1.0f - eo) / (1.0f + eo), ri = (1.0f - ior) / (1.0f + ior);
        dst[8] = eo;
        dst[9] = ro * ro;
        dst[10] = ri * ri;
    }
}

// Prefilter thresholds r2p (row 4 of each group) for the secondary-ray
// sphere loop (rt_kernel.hip, pair_prefilter).  Secondary origins are hit
// points, i.e. lie within |r_i| of a hittable sphere centre s_i, so
//   M_j = (max_i |s_i - s_j| + |r_i|)^2   (with slack for origin rounding)
// bounds |C|^2 for sphere j, and r2p_j = r^2_j + M_j (32u + 1.01K) rounded
// up (u = 2^-24, K = 2^-16) exceeds the prefilter's error bound.  Spheres
// that can never pass the exact test (SIMD r^2 <= 0, scalar padding) get
// -inf: never flagged.  Returns whether the prefilter pays for this scene
// (thresholds not far above r^2 on average).
static bool prefilter_rows(std::vector<float> &gv, uint32_t n_groups, bool simd) {
    std::vector<uint32_t> hit;
    for (uint32_t s = 0; s < 4u * n_groups; ++s) {
        const float r2 = gv[(s / 4u) * 4u * kGroupF4 + 4u * kRowR2 + s % 4u];
        if (simd ? r2 > 0.0f : r2 >= 0.0f) hit.push_back(s);
    }
    double ratio = 0.0;
    uint32_t n_ratio = 0;
    for (uint32_t j = 0; j < 4u * n_groups; ++j) {
        const uint32_t gj = (j / 4u) * 4u * kGroupF4, lj = j % 4u;
        const float r2 = gv[gj + 4u * kRowR2 + lj];
        float &r2p = gv[gj + 4u * kRowR2P + lj];
        if (!(simd ? r2 > 0.0f : r2 >= 0.0f) || !std::isfinite(r2)) {
            r2p = -INFINITY;
            continue;
        }
        double reach = 0.0;
        for (uint32_t i : hit) {
            const uint32_t gi = (i / 4u) * 4u * kGroupF4, li = i % 4u;
            const double dx = (double)gv[gi + 4u * kRowX + li] - gv[gj + 4u * kRowX + lj],
                         dy = (double)gv[gi + 4u * kRowY + li] - gv[gj + 4u * kRowY + lj],
                         dz = (double)gv[gi + 4u * kRowZ + li] - gv[gj + 4u * kRowZ + lj];
            const double ri = std::sqrt((double)gv[gi + 4u * kRowR2 + li]);
            reach = std::max(reach, std::sqrt(dx * dx + dy * dy + dz * dz) + ri);
        }
        const double m = (reach * 1.001 + 1e-3) * (reach * 1.001 + 1e-3);
        const double e = m * (32.0 * 0x1p-24 + 1.01 * 0x1p-16);
        r2p = std::nextafter((float)((double)r2 + e), INFINITY);
        ratio += std::min(e / std::max((double)r2, 1e-30), 10.0);
        n_ratio += 1;
    }
    return n_ratio > 0 && ratio / n_ratio < 0.5;
}

// Clustered prefilter table (rt_kernel.h, cl_entry_f4(words) rows per entry) for the
// secondary-ray sphere loop: the hittable spheres are grouped into about
// sqrt(n) spatial clusters (deterministic k-means; any membership -- the
// exact test still runs in the reference's group order).  A cluster c with
// centre q_c is skipped by a wave when every lane's FMA estimate
// e_c = |Q|^2 - (Q.D)^2, Q = RN(q_c - O), satisfies e_c >= rc2p_c.  Proof
// that skipping is exact (u = 2^-24, K = 2^-16, l(p) = the exact squared
// distance from point p to the ray's line; distance to a line is 1-Lipschitz):
//  - e_c is within M_c (10.2u + K(1+K)/(1-K)) of l(O + Q) (as for spheres,
//    plus the 1/|D|^2 factor of l), M_c a bound on |Q|^2 over every secondary
//    origin; so e_c >= rc2p_c = rho_c^2 + M_c (32u + 1.01K) gives
//    l(O + Q) >= rho_c^2, and |Q - (q_c - O)| <= u sqrt(M_c) moves the point
//    by at most that: sqrt(l(q_c)) >= rho_c - u sqrt(M_c);
//  - member j: sqrt(l(s_j)) >= sqrt(l(q_c)) - |s_j - q_c|, and the
//    reference's rounded C_j moves s_j by <= u sqrt(M_j) again;
//  - the reference-rounded dist_j (exact ops on C_j: >= l(O + C_j)) is within
//    13.3u M_j of its exact value, so l(O + C_j) > sigma_j^2 = r_j^2 + 13.3u M_j
//    makes dist_j > r_j^2: a miss under both rule sets.
// Hence rho_c = max_j (|s_j - q_c| + sigma_j + u sqrt(M_j)) + u sqrt(M_c),
// inflated by 1e-6 relative.  Members of a passing cluster are tested with
// their own r2p (the per-sphere bound above); a sphere pair some lane may
// hit sets its bit in the wave's pair mask, and the exact recheck walks that
// mask in group order.  Returns the number of cluster-pair entries (0: not
// used -- more than kClMaxGroups groups, too few hittable spheres); *words =
// u64 words of the pair mask.
//
// relative (the per-lane thresholds of pack_set, where the scene-wide M makes
// the bound above useless): the thresholds are formed per lane from the lane's
// own cc = |Q|^2 (rt_kernel.hip kClRel / kPfRel / kBehindRel).  With A_j =
// |Q|(1+u) + delta_j >= |C_j| (delta_j = |s_j - q_c|) the chain above reads
//   sqrt(l(O+Q)) > delta_j + sqrt(r_j^2 + 13.3u A_j^2) + 2u A_j + u|Q|
// and sqrt(r^2 + 13.3u A^2) <= r + sqrt(13.3u) A, so it holds when
//   sqrt(l(O+Q)) > rho_j + a|Q|,  rho_j = delta_j (1+s) + r_j,  s = sqrt(13.3u) + 2u,  a = s(1+u) + u;
// (rho + a|Q|)^2 <= rho^2 (1+a) + |Q|^2 (a + a^2), l(O+Q) >= e_c - E1 |Q|^2
// (E1 = 10.2u + K(1+K)/(1-K)) and |Q|^2 <= cc (1 + 5.1u), so the cluster is
// skipped when e_c >= RN(cc kClRel + R_c), R_c = rho_c^2 (1+a) rounded up,
// kClRel >= (a + a^2 + E1)(1 + 6u) (both inflated for the FMA's rounding).
// Members carry r^2 (the group rows' per-lane rule), behind thresholds lose
// their M terms (|Q|, |C_j| <= (1 + cc)/2 bound them per lane, kBehindRel):
//   cluster  -(max_j ((delta_j + r_j)(1 + 2^-15) + 4.3u delta_j) + 4.3u),
//   member   -(r_j (1 + 2^-15) + 4.3u),
// and a lane's behind test is T < RN(stored - 4.5u cc).
// k_override / sub_override: rt_device_options ClusterCount / SubClusterSpheres (0: per scene, below).
static uint32_t cluster_table(const std::vector<float> &gv, uint32_t n_groups, std::vector<float> &tab,
                              uint32_t *words, bool relative = false, uint32_t *levels = nullptr,
                              uint32_t *sub_pairs = nullptr, uint32_t k_override = 0, uint32_t sub_override = 0) {
    if (levels) *levels = 0;
    if (sub_pairs) *sub_pairs = 0;
    tab.clear();
    *words = n_groups <= 32u ? 1u : n_groups <= 64u ? 2u : 4u;
    if (n_groups > kClMaxGroups) return 0;
    struct Sph {
        uint32_t s;
        double x, y, z, r, m;
    };
    std::vector<Sph> sp;
    for (uint32_t s = 0; s < 4u * n_groups; ++s) {
        const uint32_t g = (s / 4u) * 4u * kGroupF4, l = s % 4u;
        if (!std::isfinite(gv[g + 4u * kRowR2P + l])) continue;  // never flagged (-inf)
        sp.push_back({s, gv[g + 4u * kRowX + l], gv[g + 4u * kRowY + l], gv[g + 4u * kRowZ + l],
                      std::sqrt((double)std::max(gv[g + 4u * kRowR2 + l], 0.0f)), 0.0});
    }
    const uint32_t n = (uint32_t)sp.size();
    if (n < 8u) return 0;
    // reach of every origin (a point on some hittable sphere) from point p, with
    // the same slack for origin rounding as prefilter_rows
    auto bound_m = [&](double px, double py, double pz) {
        double reach = 0.0;
        for (const Sph &o : sp)
            reach = std::max(reach, std::sqrt((o.x - px) * (o.x - px) + (o.y - py) * (o.y - py) + (o.z - pz) * (o.z - pz)) + o.r);
        return (reach * 1.001 + 1e-3) * (reach * 1.001 + 1e-3);
    };
    const double u = 0x1p-24, K = 0x1p-16;
    if (!relative)
        for (Sph &o : sp) o.m = bound_m(o.x, o.y, o.z);
    auto sigma = [&](const Sph &o) {
        return relative ? o.r : std::sqrt(o.r * o.r + 13.3 * u * o.m) + u * std::sqrt(o.m);
    };
    const double s_rel = std::sqrt(13.3 * u) + 2.0 * u, a_rel = s_rel * (1.0 + u) + u;
    // max(1.25 sqrt(n), n/8) clusters: measured on C2 (N = 64) K = 6/8/10/12/16 ->
    // 112.4k/113.8k/114.6k/114.5k/111.4k Mrays/s; at 200 spheres K = 17/28 ->
    // 45.0k/46.9k; at C5 (256) K = 20/26/32/40 -> 30.1k/31.3k/32.4k/32.4k
    // per-lane tables carry the height-slab test, which culls most clusters of a
    // ground-plane scene, so fewer (larger) clusters pay there: RTWeekend (482
    // spheres) K = 32/40/60/90 -> 17.8k/18.5k/17.8k/16.7k Mrays/s, hence n/12
    // Two-level tables (two or more mask words, below) take fewer, larger top
    // clusters over sub-clusters of 3 (scene-wide) or 4 (per-lane) spheres:
    // RTWeekend K/S = 40/4, 28/3, 28/4, 24/4 -> 21.1k/21.9k/21.9k/21.7k (one level
    // at K 40: 19.6k); C5 at 512 spp K/S = 32/4, 24/3, 28/3, 24/2 -> 47.4k/48.2k/
    // 48.3k/48.3k (one level: 46.3k).
    // two levels for tables of two or more mask words only: the kernel walks
    // one-word tables (at most 32 groups) as one level (rt_kernel.hip clustered_groups)
    const bool two_levels = *words >= 2u;
    const uint32_t div = two_levels ? (relative ? 17u : 10u) : (relative ? 12u : 8u);
    uint32_t k = std::max(2u, std::max((uint32_t)std::lround(1.25 * std::sqrt((double)n)), n / div));
    if (k_override) k = std::min(n, std::max(2u, k_override));  // A/B (rt_device_options ClusterCount)
    // k-means (f64, fixed LCG restarts) of the spheres idx into k clusters,
    // minimising the sum of rho_c^2; returns each sphere's label
    uint64_t lcg = 0x9E3779B97F4A7C15ull;
    auto rnd = [&](uint32_t m) {
        lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)((lcg >> 33) % m);
    };
    auto kmeans = [&](const std::vector<uint32_t> &idx, uint32_t k, int restarts) {
        const uint32_t m = (uint32_t)idx.size();
        std::vector<uint32_t> best_lab(m, 0u);
        double best_cost = INFINITY;
        std::vector<double> cx(k), cy(k), cz(k);
        std::vector<uint32_t> lab(m);
        for (int restart = 0; restart < restarts; ++restart) {
            for (uint32_t c = 0; c < k; ++c) {  // k-means++ style seeding (farthest of a few random picks)
                uint32_t pick = rnd(m);
                double far = -1.0;
                for (int t = 0; t < 4 && c > 0; ++t) {
                    const uint32_t cand = rnd(m);
                    const Sph &o = sp[idx[cand]];
                    double dmin = INFINITY;
                    for (uint32_t q = 0; q < c; ++q)
                        dmin = std::min(dmin, (o.x - cx[q]) * (o.x - cx[q]) + (o.y - cy[q]) * (o.y - cy[q]) +
                                                  (o.z - cz[q]) * (o.z - cz[q]));
                    if (dmin > far) {
                        far = dmin;
                        pick = cand;
                    }
                }
                const Sph &o = sp[idx[pick]];
                cx[c] = o.x;
                cy[c] = o.y;
                cz[c] = o.z;
            }
            for (int it = 0; it < 40; ++it) {
                for (uint32_t i = 0; i < m; ++i) {
                    const Sph &o = sp[idx[i]];
                    double dmin = INFINITY;
                    for (uint32_t c = 0; c < k; ++c) {
                        const double d2 = (o.x - cx[c]) * (o.x - cx[c]) + (o.y - cy[c]) * (o.y - cy[c]) +
                                          (o.z - cz[c]) * (o.z - cz[c]);
                        if (d2 < dmin) {
                            dmin = d2;
                            lab[i] = c;
                        }
                    }
                }
                std::vector<double> sx(k, 0.0), sy(k, 0.0), sz(k, 0.0), cnt(k, 0.0);
                for (uint32_t i = 0; i < m; ++i) {
                    sx[lab[i]] += sp[idx[i]].x;
                    sy[lab[i]] += sp[idx[i]].y;
                    sz[lab[i]] += sp[idx[i]].z;
                    cnt[lab[i]] += 1.0;
                }
                for (uint32_t c = 0; c < k; ++c)
                    if (cnt[c] > 0.0) {
                        cx[c] = sx[c] / cnt[c];
                        cy[c] = sy[c] / cnt[c];
                        cz[c] = sz[c] / cnt[c];
                    }
            }
            std::vector<double> rho(k, 0.0);
            for (uint32_t i = 0; i < m; ++i) {
                const Sph &o = sp[idx[i]];
                const uint32_t c = lab[i];
                const double d = std::sqrt((o.x - cx[c]) * (o.x - cx[c]) + (o.y - cy[c]) * (o.y - cy[c]) +
                                           (o.z - cz[c]) * (o.z - cz[c]));
                rho[c] = std::max(rho[c], d + sigma(o));
            }
            double cost = 0.0;
            for (uint32_t c = 0; c < k; ++c) cost += rho[c] * rho[c];
            if (cost < best_cost) {
                best_cost = cost;
                best_lab = lab;
            }
        }
        return best_lab;
    };
    // final clusters: f32 centres (what the kernel subtracts), exact thresholds
    struct Cl {
        float qx, qy, qz, t;
        float b;                    // behind threshold (below)
        float srho = 0.0f, ymid = 0.0f, yhalf = INFINITY;  // height-slab bound (relative tables, below)
        std::vector<uint32_t> mem;  // sphere slots, ascending
    };
    // Behind thresholds: a member j cannot be accepted by a ray whose computed
    // T_j + X_j stays below eps (it = T - X or T + X < eps), and X_j <= r_j(1+2u).
    // With T_j within 4.2u sqrt(M_j)|D| of (S_j - O).D (one rounding in C_j, three
    // in the dot) and the prefilter's FMA T_c within 4u sqrt(M_c)|D| of (q_c - O).D,
    // (S_j - O).D <= (q_c - O).D + |S_j - q_c||D| gives: T_c < -b_c with
    //   b_c = max_j (|S_j - q_c| + r_j)(1 + 2^-15) + 4.3u (sqrt(M_c) + sqrt(M_j))
    // proves every member is behind every origin-side candidate (|D| <= 1 + 2^-17
    // under the |D|^2 bound).  Per sphere (q_c = S_j): b_j = r_j(1 + 2^-15) + 8.6u sqrt(M_j).
    std::vector<float> beta_of_slot(4u * n_groups, 0.0f);
    for (const Sph &o : sp)
        beta_of_slot[o.s] = relative ? std::nextafter((float)(-(o.r * (1.0 + 0x1p-15) + 4.3 * u) * (1.0 + 1e-6)), -INFINITY)
                                     : std::nextafter((float)-(o.r * (1.0 + 0x1p-15) + 8.6 * u * std::sqrt(o.m)), -INFINITY);
    // The bound rows of a cluster over the spheres idx (any set: a top cluster's
    // bound covers every sphere under it, as a sub-cluster's covers its members).
    auto make_cl = [&](const std::vector<uint32_t> &idx) {
        Cl C;
        double sx = 0.0, sy = 0.0, sz = 0.0;
        for (uint32_t i : idx) {
            sx += sp[i].x;
            sy += sp[i].y;
            sz += sp[i].z;
        }
        C.qx = (float)(sx / idx.size());
        C.qy = (float)(sy / idx.size());
        C.qz = (float)(sz / idx.size());
        const double qx = C.qx, qy = C.qy, qz = C.qz;
        auto delta = [&](uint32_t i) {
            return std::sqrt((sp[i].x - qx) * (sp[i].x - qx) + (sp[i].y - qy) * (sp[i].y - qy) +
                             (sp[i].z - qz) * (sp[i].z - qz));
        };
        if (relative) {
            double rho = 0.0, bmax = 0.0;
            for (uint32_t i : idx) {
                rho = std::max(rho, delta(i) * (1.0 + s_rel) + sp[i].r);
                bmax = std::max(bmax, (delta(i) + sp[i].r) * (1.0 + 0x1p-15) + 4.3 * u * delta(i));
            }
            C.t = std::nextafter((float)(rho * rho * (1.0 + a_rel) * (1.0 + 1e-6)), INFINITY);
            C.b = std::nextafter((float)(-(bmax + 4.3 * u) * (1.0 + 1e-6)), -INFINITY);
            // Height slab.  A lane can accept member j only if its exact line passes
            // within sigma_j = sqrt(r_j^2 + 13.3u |C_j|^2) <= r_j + k_s |C_j| of s_j
            // (k_s = sqrt(13.3u) = 8.9e-4; the reference-rounded dist error, as above),
            // so at some t with |O + tD - q_c| <= rho_s + k_s |C_j|, rho_s = max_j
            // (delta_j + r_j), and height within [y_lo - k_s|C_j|, y_hi + k_s|C_j|]
            // (y_lo/y_hi the members' extent).  Along the line the height O.y + t D.y
            // over that t range lies within c +- |D.y| rho' (c = O.y + D.y T, T the
            // projection of q_c): if |c - ymid| > yhalf + |D.y| rho' + E the line misses
            // every member.  |C_j| <= |Q| + delta_j, |Q| <= (1 + cc)/2: the delta_j part
            // is folded into srho / yhalf here, the |Q| part (twice, for height and t
            // range) and the rounding of T, c, d and thr (< 2^-14 (1 + cc) + u |O.y|)
            // into the kernel's per-lane E = cc kSlabRel + |O.y| 2^-21 + kSlabRel,
            // kSlabRel = 2^-9 >= 2 (8.9e-4 (1.0001) / 2 + 2^-14).
            double rs = 0.0, yhi = -INFINITY, ylo = INFINITY;
            for (uint32_t i : idx) {
                rs = std::max(rs, delta(i) + sp[i].r);
                yhi = std::max(yhi, sp[i].y + sp[i].r);
                ylo = std::min(ylo, sp[i].y - sp[i].r);
            }
            const double ks = 8.91e-4;
            C.srho = std::nextafter((float)(rs * (1.0 + ks) * (1.0 + 0x1p-12)), INFINITY);
            C.ymid = (float)((yhi + ylo) * 0.5);
            const double half = std::max(yhi - (double)C.ymid, (double)C.ymid - ylo) + ks * rs;
            C.yhalf = std::nextafter((float)(half * (1.0 + 0x1p-12)), INFINITY);
        } else {
            double rho = 0.0;
            for (uint32_t i : idx) rho = std::max(rho, delta(i) + sigma(sp[i]));
            const double mc = bound_m(qx, qy, qz);
            rho = (rho + u * std::sqrt(mc)) * (1.0 + 1e-6);
            C.t = std::nextafter((float)(rho * rho + mc * (32.0 * u + 1.01 * K)), INFINITY);
            double bmax = 0.0;
            for (uint32_t i : idx)
                bmax = std::max(bmax, (delta(i) + sp[i].r) * (1.0 + 0x1p-15) + 4.3 * u * (std::sqrt(mc) + std::sqrt(sp[i].m)));
            C.b = std::nextafter((float)-bmax, -INFINITY);
        }
        for (uint32_t i : idx) C.mem.push_back(sp[i].s);
        return C;
    };
    const Cl pad_cl{0.0f, 0.0f, 0.0f, -INFINITY, 0.0f, 0.0f, 0.0f, INFINITY, {}};  // never entered
    // top clusters
    std::vector<uint32_t> all(n);
    for (uint32_t i = 0; i < n; ++i) all[i] = i;
    const std::vector<uint32_t> top_lab = kmeans(all, k, 16);
    std::vector<std::vector<uint32_t>> tops;
    for (uint32_t c = 0; c < k; ++c) {
        std::vector<uint32_t> idx;
        for (uint32_t i = 0; i < n; ++i)
            if (top_lab[i] == c) idx.push_back(i);
        if (!idx.empty()) tops.push_back(std::move(idx));
    }
    std::vector<Cl> cl;
    for (const auto &idx : tops) cl.push_back(make_cl(idx));
    if (cl.size() & 1u) cl.push_back(pad_cl);
    // Second level (tables of two or more mask words): each top cluster's spheres
    // in sub-clusters of about kSubSpheres (k-means inside the top cluster), their
    // pair entries contiguous per top cluster, padded to whole pairs.
    const bool two = two_levels;
    uint32_t sub_spheres = relative ? 4u : 3u;
    if (sub_override) sub_spheres = sub_override;  // A/B (rt_device_options SubClusterSpheres)
    std::vector<std::vector<Cl>> sub(cl.size());
    if (two)
        for (size_t c = 0; c < tops.size(); ++c) {
            const std::vector<uint32_t> &idx = tops[c];
            const uint32_t k2 = std::min((uint32_t)idx.size(), ((uint32_t)idx.size() + sub_spheres - 1u) / sub_spheres);
            if (k2 <= 1u) {
                sub[c].push_back(make_cl(idx));
            } else {
                const std::vector<uint32_t> lab = kmeans(idx, k2, 8);
                for (uint32_t q = 0; q < k2; ++q) {
                    std::vector<uint32_t> part;
                    for (size_t i = 0; i < idx.size(); ++i)
                        if (lab[i] == q) part.push_back(idx[i]);
                    if (!part.empty()) sub[c].push_back(make_cl(part));
                }
            }
            if (sub[c].size() & 1u) sub[c].push_back(pad_cl);
        }
    for (Cl &C : cl) std::sort(C.mem.begin(), C.mem.end());
    for (auto &v : sub)
        for (Cl &C : v) std::sort(C.mem.begin(), C.mem.end());
    const uint32_t n_cp = (uint32_t)cl.size() / 2u;
    uint32_t n_sp = 0, n_mp = 0;
    for (size_t c = 0; c < cl.size(); ++c) {
        if (two) {
            n_sp += (uint32_t)sub[c].size() / 2u;
            for (const Cl &S : sub[c]) n_mp += ((uint32_t)S.mem.size() + 1u) / 2u;
        } else {
            n_mp += ((uint32_t)cl[c].mem.size() + 1u) / 2u;
        }
    }
    const uint32_t ef = cl_entry_f4(*words, relative) * 4u;  // floats per entry
    tab.assign((size_t)(n_cp + n_sp + n_mp) * ef, 0.0f);
    auto put_u = [&](size_t at, uint32_t v) { memcpy(&tab[at], &v, 4); };
    auto sphere_xyz = [&](uint32_t s, int axis) {
        const uint32_t g = (s / 4u) * 4u * kGroupF4, l = s % 4u;
        return gv[g + 4u * (uint32_t)axis + l];
    };
    // member threshold: the scene-wide r2p, or r^2 for the per-lane rule
    auto sphere_r2p = [&](uint32_t s) {
        return gv[(s / 4u) * 4u * kGroupF4 + 4u * (relative ? kRowR2 : kRowR2P) + s % 4u];
    };
    // the bound rows of a cluster pair entry (both levels)
    auto put_pair = [&](uint32_t p, const Cl &A, const Cl &B) {
        float *e = &tab[(size_t)p * ef];
        e[0] = A.qx, e[1] = B.qx, e[2] = A.qy, e[3] = B.qy, e[4] = A.qz, e[5] = B.qz, e[6] = A.t, e[7] = B.t;
        e[12] = A.b, e[13] = B.b;
        if (relative) {  // the height-slab bound (rt_kernel.h: row 3 zw, row 4)
            e[14] = A.srho, e[15] = B.srho;
            e[16] = A.ymid, e[17] = B.ymid, e[18] = A.yhalf, e[19] = B.yhalf;
        }
    };
    uint32_t next_sub = n_cp, next = n_cp + n_sp;
    // the member pair entries of cluster C from entry `next` on; returns their count
    auto put_members = [&](const Cl &C) {
        const uint32_t cnt = ((uint32_t)C.mem.size() + 1u) / 2u;
        for (uint32_t q = 0; q < cnt; ++q, ++next) {
            float *m = &tab[(size_t)next * ef];
            const size_t mb = (size_t)next * ef;
            for (int w = 0; w < 2; ++w) {
                const uint32_t idx = 2u * q + (uint32_t)w;
                if (idx < C.mem.size()) {
                    const uint32_t s = C.mem[idx];
                    m[0 + w] = sphere_xyz(s, kRowX);
                    m[2 + w] = sphere_xyz(s, kRowY);
                    m[4 + w] = sphere_xyz(s, kRowZ);
                    m[6 + w] = sphere_r2p(s);
                    m[12 + w] = beta_of_slot[s];
                    // the u64 bit of pair q = s >> 1 in the row of word q >> 6 (row 2
                    // for word 0, row 3 + w for word w >= 1; the other words' rows stay 0)
                    const uint64_t bit = 1ull << ((s >> 1) & 63u);
                    const uint32_t word = (s >> 1) >> 6;
                    const size_t row = word == 0u ? 8u : 4u * (3u + word);
                    put_u(mb + row + 2u * w, (uint32_t)bit);
                    put_u(mb + row + 1u + 2u * w, (uint32_t)(bit >> 32));
                } else {
                    m[6 + w] = -INFINITY;  // padding member: never flagged, no bit
                }
            }
        }
        return cnt;
    };
    for (uint32_t p = 0; p < n_cp; ++p) {
        put_pair(p, cl[2u * p], cl[2u * p + 1u]);
        for (int h = 0; h < 2; ++h) {
            const size_t c = 2u * p + (uint32_t)h;
            if (!two) {
                put_u((size_t)p * ef + 8u + 2u * h, next);
                put_u((size_t)p * ef + 9u + 2u * h, put_members(cl[c]));
                continue;
            }
            // a top cluster: its sub-cluster pair entries, then their members
            const uint32_t first = next_sub, cnt = (uint32_t)sub[c].size() / 2u;
            put_u((size_t)p * ef + 8u + 2u * h, first);
            put_u((size_t)p * ef + 9u + 2u * h, cnt);
            next_sub += cnt;
            for (uint32_t q = 0; q < cnt; ++q) {
                const uint32_t e = first + q;
                put_pair(e, sub[c][2u * q], sub[c][2u * q + 1u]);
                for (int h2 = 0; h2 < 2; ++h2) {
                    put_u((size_t)e * ef + 8u + 2u * h2, next);
                    put_u((size_t)e * ef + 9u + 2u * h2, put_members(sub[c][2u * q + (uint32_t)h2]));
                }
            }
        }
    }
    if (levels) *levels = two ? 2u : 1u;
    if (sub_pairs) *sub_pairs = n_sp;
    return n_cp;
}

// Whether every r^2 the exact test can accept is 0 or in [2^-36, 2^60]: then
// a passing candidate's r^2 - dist is 0 or >= 2^-60 (it is >= ulp(r^2)/2 when
// positive), the range where the kernel's short sqrt is verified exact.
static uint32_t sqrt_range_ok(const std::vector<float> &gv, uint32_t n_groups, bool simd) {
    for (uint32_t s = 0; s < 4u * n_groups; ++s) {
        const float r2 = gv[(s / 4u) * 4u * kGroupF4 + 4u * kRowR2 + s % 4u];
        if (!(simd ? r2 > 0.0f : r2 >= 0.0f)) continue;  // never accepted (padding)
        if (r2 != 0.0f && !(r2 >= 0x1p-36f && r2 <= 0x1p60f)) return 0u;
    }
    return 1u;
}

// One rule set of a scene in the kernel's layout (see rt_kernel.h): rs 0 =
// SIMD rules from SIMDSpheres (main.cpp:399-400) + Materials[4g+l]
// (main.cpp:443-444); rs 1 = scalar rules from ScalarSpheres[s].Position/
// Radius/Material (main.cpp:547-590), padding lanes r^2 = -inf (the kernel
// also skips them by its s < n_spheres test: the scalar loop runs to Count).
struct PackedSet {
    std::vector<float> groups, mats;
    uint32_t n_groups = 0;
    bool prefilter_pays = false;
    bool relative = false;  // row 3 rewritten to r^2 / -inf for the per-lane threshold
    uint32_t fast_sqrt = 0;
    std::vector<float> clusters;  // cluster_table
    uint32_t n_cpairs = 0, cl_words = 0;
    uint32_t cl_levels = 0, cl_sub_pairs = 0;  // two-level tables (cl_words >= 2)
};

static int pack_set(const rt_scene *scene, int rs, PackedSet &p, int pf_rel_env = -1, uint32_t cluster_k = 0,
                    uint32_t sub_spheres = 0) {
    const uint32_t ng = scene->SIMDSpheres.Count;
    const uint32_t ns = scene->ScalarSpheres.Count;
    if (ng == 0 || !scene->SIMDSpheres.Data || !scene->Materials.Data || ns == 0 || !scene->ScalarSpheres.Data)
        return fail(RT_EINVAL, "scene: empty scene");
    const uint32_t ngs = (ns + 3u) / 4u;
    if (ng > kMaxGroups || ngs > kMaxGroups)
        return fail(RT_EINVAL, "scene: %u spheres exceed the limit of %u", ns, 4u * kMaxGroups);
    const uint32_t n = rs == 0 ? ng : ngs;
    p.n_groups = n;
    p.groups.assign((size_t)n * 4 * kGroupF4, 0.0f);
    p.mats.assign((size_t)n * 16u * kSphereF4, 0.0f);  // sphere records (rt_kernel.h kSphereF4)
    std::vector<float> &gv = p.groups;
    if (rs == 0) {
        const rt_sphere_group *g = (const rt_sphere_group *)scene->SIMDSpheres.Data;
        const rt_material *m = (const rt_material *)scene->Materials.Data;
        for (uint32_t i = 0; i < ng; ++i) {
            for (int l = 0; l < 4; ++l) {
                gv[i * 4 * kGroupF4 + 4 * kRowX + l] = g[i].X[l];
                gv[i * 4 * kGroupF4 + 4 * kRowY + l] = g[i].Y[l];
                gv[i * 4 * kGroupF4 + 4 * kRowZ + l] = g[i].Z[l];
                gv[i * 4 * kGroupF4 + 4 * kRowR2 + l] = g[i].Radii[l] * g[i].Radii[l];
                const uint32_t s = 4u * i + (uint32_t)l;
                float *rec = &p.mats[(size_t)s * 4u * kSphereF4];
                rec[0] = g[i].X[l];
                rec[1] = g[i].Y[l];
                rec[2] = g[i].Z[l];
                if (s < scene->Materials.Count) put_material(rec + 4, m[s]);
            }
        }
    } else {
        const rt_scalar_sphere *s = (const rt_scalar_sphere *)scene->ScalarSpheres.Data;
        for (uint32_t i = 0; i < ns; ++i) {
            const uint32_t gi = i / 4u, l = i % 4u;
            gv[gi * 4 * kGroupF4 + 4 * kRowX + l] = s[i].Position.x;
            gv[gi * 4 * kGroupF4 + 4 * kRowY + l] = s[i].Position.y;
            gv[gi * 4 * kGroupF4 + 4 * kRowZ + l] = s[i].Position.z;
            gv[gi * 4 * kGroupF4 + 4 * kRowR2 + l] = s[i].Radius * s[i].Radius;
            float *rec = &p.mats[(size_t)i * 4u * kSphereF4];
            rec[0] = s[i].Position.x;
            rec[1] = s[i].Position.y;
            rec[2] = s[i].Position.z;
            put_material(rec + 4, s[i].Material);
        }
        for (uint32_t i = ns; i < ngs * 4u; ++i) gv[(i / 4u) * 4 * kGroupF4 + 4 * kRowR2 + (i % 4u)] = -__builtin_inff();
    }
    p.prefilter_pays = prefilter_rows(gv, n, rs == 0);
    p.fast_sqrt = sqrt_range_ok(gv, n, rs == 0);
    // Where the scene-wide bound M_j makes r2p useless (a huge sphere: RTWeekend's
    // ground), the thresholds are formed per lane from the lane's own |C|^2 instead
    // (rt_kernel.hip kPfRel, kClRel): the cluster table is built for that rule, and
    // row 3 then holds r^2 (-inf: never hit).
    p.relative = pf_rel_env == 1 || (pf_rel_env < 0 && !p.prefilter_pays);
    p.n_cpairs = cluster_table(gv, n, p.clusters, &p.cl_words, p.relative, &p.cl_levels, &p.cl_sub_pairs, cluster_k,
                               sub_spheres);
    if (p.relative)
        for (uint32_t sl = 0; sl < 4u * n; ++sl) {
            const size_t base = (size_t)(sl / 4u) * 4u * kGroupF4 + sl % 4u;
            gv[base + 4u * kRowR2P] = std::isfinite(gv[base + 4u * kRowR2P]) ? gv[base + 4u * kRowR2] : -INFINITY;
        }
    return RT_OK;
}

extern "C" int rt_scene_upload(rt_device *d, const rt_scene *scene) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !scene) return fail(RT_EINVAL, "rt_scene_upload: NULL argument");
    PackedSet ps[2];
    for (int rs = 0; rs < 2; ++rs) {
        const int rc = pack_set(scene, rs, ps[rs], d->pf_rel_env, d->cluster_k, d->sub_spheres);
        if (rc) return rc;
    }
    HIP_OK(hipSetDevice(d->ordinal));
    if (const int rc = quiesce(d)) return rc;
    for (int rs = 0; rs < 2; ++rs) {
        d->prefilter[rs] = d->prefilter_env < 0 ? ((ps[rs].prefilter_pays || ps[rs].relative) ? 1u : 0u)
                                                : (uint32_t)d->prefilter_env;
        d->pf_relative[rs] = ps[rs].relative ? 1u : 0u;
        d->fast_sqrt[rs] = ps[rs].fast_sqrt;
        const int rc = upload_set(d, rs, ps[rs].groups, ps[rs].mats, ps[rs].n_groups);
        if (rc) return rc;
        const size_t nf4 = ps[rs].clusters.size() / 4u;
        d->n_cpairs[rs] = 0;
        if (nf4 > d->cap_clusters[rs]) {
            HIP_OK(hipStreamSynchronize(d->stream));
            (void)hipFree(d->d_clusters[rs]);
            d->d_clusters[rs] = nullptr;
            d->cap_clusters[rs] = 0;
            if (hipMalloc(&d->d_clusters[rs], nf4 * 16u) != hipSuccess)
                return fail(RT_ENOMEM, "rt_scene_upload: device allocation failed");
            d->cap_clusters[rs] = nf4;
        }
        if (nf4) {
            HIP_OK(hipMemcpyAsync(d->d_clusters[rs], ps[rs].clusters.data(), nf4 * 16u, hipMemcpyHostToDevice,
                                  d->stream));
            d->n_cpairs[rs] = ps[rs].n_cpairs;
            d->cl_words[rs] = ps[rs].cl_words;
        }
    }
    HIP_OK(hipStreamSynchronize(d->stream));
    d->n_spheres = scene->ScalarSpheres.Count;
    d->use_sky = scene->UseSkyColor;
    d->scene_set = true;
    d->scene_gen += 1;
    // a reserved geometry keeps its promise for the new scene's mask words (the
    // device is quiescent here: the upload waited for every launch).  The scene
    // is committed by now, so a failure here does not fail the upload: the
    // reservation is dropped and later launches grow their buffers lazily.
    if (apply_reserve(d) != RT_OK) {
        (void)hipGetLastError();
        d->reserve_tiles = 0;
        d->reserve_pixels = 0;
    }
    return RT_OK;
}

extern "C" int rt_scene_prefilter(const rt_scene *scene, uint32_t enable_simd, float *out_r2, float *out_r2p,
                                  uint32_t capacity, uint32_t *out_count, uint32_t *out_flags) {
    if (!scene || !out_count) return fail(RT_EINVAL, "rt_scene_prefilter: NULL argument");
    PackedSet p;
    const int rc = pack_set(scene, enable_simd ? 0 : 1, p);
    if (rc) return rc;
    const uint32_t n = 4u * p.n_groups;
    *out_count = n;
    if (out_flags) *out_flags = (p.prefilter_pays ? 1u : 0u) | (p.fast_sqrt ? 2u : 0u) | (p.relative ? 4u : 0u);
    if ((out_r2 || out_r2p) && capacity < n) return fail(RT_EINVAL, "rt_scene_prefilter: capacity %u < %u", capacity, n);
    for (uint32_t s = 0; s < n; ++s) {
        const size_t base = (size_t)(s / 4u) * 4u * kGroupF4 + s % 4u;
        if (out_r2) out_r2[s] = p.groups[base + 4u * kRowR2];
        if (out_r2p) out_r2p[s] = p.groups[base + 4u * kRowR2P];
    }
    return RT_OK;
}

extern "C" int rt_scene_clusters(const rt_scene *scene, uint32_t enable_simd, float *out, uint32_t capacity_f4,
                                 uint32_t *out_f4, uint32_t *out_cpairs) {
    if (!scene || !out_f4 || !out_cpairs) return fail(RT_EINVAL, "rt_scene_clusters: NULL argument");
    PackedSet p;
    const int rc = pack_set(scene, enable_simd ? 0 : 1, p);
    if (rc) return rc;
    const uint32_t nf4 = (uint32_t)(p.clusters.size() / 4u);
    *out_f4 = nf4;
    *out_cpairs = p.n_cpairs;
    if (out) {
        if (capacity_f4 < nf4) return fail(RT_EINVAL, "rt_scene_clusters: capacity %u < %u", capacity_f4, nf4);
        memcpy(out, p.clusters.data(), (size_t)nf4 * 16u);
    }
    return RT_OK;
}

extern "C" int rt_scene_cluster_layout(const rt_scene *scene, uint32_t enable_simd, uint32_t *out_levels,
                                       uint32_t *out_sub_pairs) {
    if (!scene || !out_levels || !out_sub_pairs) return fail(RT_EINVAL, "rt_scene_cluster_layout: NULL argument");
    PackedSet p;
    const int rc = pack_set(scene, enable_simd ? 0 : 1, p);
    if (rc) return rc;
    *out_levels = p.n_cpairs ? p.cl_levels : 0u;
    *out_sub_pairs = p.cl_sub_pairs;
    return RT_OK;
}

// Launch buffers for n_tiles block tiles (cost, order, live flags, sort
// scratch, cull counters) and for mask_words cull-mask words.  Growing frees
// buffers earlier launches may still read, so `sync` (the caller's stream, or
// the whole device when NULL) is waited for first; growing clears the tile key.
static int ensure_tile_buffers(rt_device *d, uint32_t n_tiles, hipStream_t sync, bool device_wide) {
    if (n_tiles <= d->tile_cap && d->d_cull_counters) return RT_OK;
    if (device_wide) HIP_OK(hipDeviceSynchronize());
    else HIP_OK(hipStreamSynchronize(sync));
    if (n_tiles > d->tile_cap) {
        for (uint32_t **b : {&d->d_tile_cost, &d->d_tile_order, &d->d_tile_scratch, &d->d_tile_live,
                             &d->d_tile_order_sorted, &d->d_tile_aux}) {
            (void)hipFree(*b);
            *b = nullptr;
        }
        d->tile_cap = 0;
        // cost / order / sort scratch per unit: up to 4 per block tile (wave units)
        if (hipMalloc(&d->d_tile_cost, 4u * n_tiles * 4u) != hipSuccess ||
            hipMalloc(&d->d_tile_order, 4u * n_tiles * 4u) != hipSuccess ||
            hipMalloc(&d->d_tile_order_sorted, 4u * n_tiles * 4u) != hipSuccess ||
            hipMalloc(&d->d_tile_aux, 2u * n_tiles * 4u) != hipSuccess ||
            hipMalloc(&d->d_tile_live, n_tiles * 4u) != hipSuccess ||
            hipMalloc(&d->d_tile_scratch, rtk_tile_sort_scratch(4u * n_tiles)) != hipSuccess)
            return fail(RT_ENOMEM, "rt_trace: tile order buffers");
        d->tile_cap = n_tiles;
        d->last.BufferGrowths += 1;
    }
    if (!d->d_cull_counters && hipMalloc(&d->d_cull_counters, kCullCounterWords * 8u) != hipSuccess)
        return fail(RT_ENOMEM, "rt_trace: tile order buffers");
    d->tile_key.clear();
    return RT_OK;
}

static int ensure_masks(rt_device *d, size_t mask_words, hipStream_t sync, bool device_wide) {
    if (mask_words <= d->mask_cap) return RT_OK;
    if (device_wide) HIP_OK(hipDeviceSynchronize());
    else HIP_OK(hipStreamSynchronize(sync));
    (void)hipFree(d->d_masks);
    d->d_masks = nullptr;
    d->mask_cap = 0;
    if (hipMalloc(&d->d_masks, mask_words * 8u) != hipSuccess) return fail(RT_ENOMEM, "rt_trace: cull masks");
    d->mask_cap = mask_words;
    d->last.BufferGrowths += 1;
    d->tile_key.clear();
    return RT_OK;
}

static int ensure_pixel_sort(rt_device *d, uint32_t n_tiles, size_t pixels, hipStream_t sync, bool device_wide) {
    if ((size_t)n_tiles * 64u <= d->pix_perm_cap && pixels * 4u <= d->pix_cost_cap) return RT_OK;
    if (device_wide) HIP_OK(hipDeviceSynchronize());
    else HIP_OK(hipStreamSynchronize(sync));
    if ((size_t)n_tiles * 64u > d->pix_perm_cap) {
        (void)hipFree(d->d_pix_perm);
        d->d_pix_perm = nullptr;
        d->pix_perm_cap = 0;
        if (hipMalloc(&d->d_pix_perm, (size_t)n_tiles * 64u) != hipSuccess) return fail(RT_ENOMEM, "rt_trace: pixel order");
        d->pix_perm_cap = (size_t)n_tiles * 64u;
    }
    if (pixels * 4u > d->pix_cost_cap) {
        (void)hipFree(d->d_pix_cost);
        d->d_pix_cost = nullptr;
        d->pix_cost_cap = 0;
        if (hipMalloc(&d->d_pix_cost, pixels * 4u) != hipSuccess) return fail(RT_ENOMEM, "rt_trace: pixel costs");
        d->pix_cost_cap = pixels * 4u;
    }
    d->last.BufferGrowths += 1;
    d->tile_key.clear();
    return RT_OK;
}

// The buffers of every launch rt_trace may make at the reserved geometry:
// the most block tiles over every lanes-per-pixel shape (rt_trace picks P per
// launch) and the current scene's mask words, so no later launch allocates.
static int apply_reserve(rt_device *d) {
    if (!d->reserve_tiles) return RT_OK;
    const uint32_t n_tiles = d->reserve_tiles;
    uint32_t n_words = 1;
    if (d->scene_set)
        for (int rs = 0; rs < 2; ++rs) n_words = std::max(n_words, rtk_mask_words(d->n_groups[rs]));
    if (const int rc = ensure_tile_buffers(d, n_tiles, nullptr, true)) return rc;
    if (d->pixel_sort_env)
        if (const int rc = ensure_pixel_sort(d, n_tiles, d->reserve_pixels, nullptr, true))
            return rc;
    return ensure_masks(d, (size_t)n_tiles * 4u * n_words, nullptr, true);
}

extern "C" int rt_device_reserve(rt_device *d, uint32_t width, uint32_t local_rows) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || width == 0 || local_rows == 0 || width > 65536 || local_rows > 65536)
        return fail(RT_EINVAL, "rt_device_reserve: bad argument");
    HIP_OK(hipSetDevice(d->ordinal));
    uint32_t n_tiles = 0;
    for (const int p : {1, 2, 4, 8, 16, 32}) n_tiles = std::max(n_tiles, rtk_tile_count(width, local_rows, p));
    d->reserve_tiles = std::max(d->reserve_tiles, n_tiles);
    d->reserve_pixels = std::max(d->reserve_pixels, (size_t)width * local_rows);
    return apply_reserve(d);
}

extern "C" int rt_trace(rt_device *d, const rt_camera_info *cam, const rt_trace_desc *desc, uint64_t *d_rays,
                        void *stream) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !cam || !desc || !d_rays) return fail(RT_EINVAL, "rt_trace: NULL argument");
    if (!d->lut_set) return fail(RT_EINVAL, "rt_trace: rsqrt table not set (rt_set_rsqrt_table)");
    if (!d->scene_set) return fail(RT_EINVAL, "rt_trace: no scene uploaded (rt_scene_upload)");
    if (desc->SeedMode != RT_SEED_PIXEL) return fail(RT_EINVAL, "rt_trace: only RT_SEED_PIXEL runs on the GPU");
    if (desc->Flags & ~(RT_FLAG_ACCUM_ZERO | RT_FLAG_SRGB_POW))
        return fail(RT_EINVAL, "rt_trace: unknown Flags 0x%x", desc->Flags);
    if (desc->Width == 0 || desc->Height == 0 || desc->Width > 65536 || desc->Height > 65536)
        return fail(RT_EINVAL, "rt_trace: bad image size %ux%u", desc->Width, desc->Height);
    const uint32_t band_rows = desc->BandRows ? desc->BandRows : 32u;
    const uint32_t band_count = desc->BandCount ? desc->BandCount : 1u;
    if (desc->BandIndex >= band_count) return fail(RT_EINVAL, "rt_trace: BandIndex >= BandCount");
    if (band_rows % 8u) return fail(RT_EINVAL, "rt_trace: BandRows must be a multiple of 8");
    if ((uint64_t)desc->PreviousRayCount + desc->Frames > 0xFFFFFFFFull)
        return fail(RT_EINVAL, "rt_trace: PreviousRayCount + Frames exceeds the u32 frame count");
    const uint32_t local_rows = rt_band_local_rows(desc->Height, band_rows, band_count, desc->BandIndex);
    if (desc->Frames == 0 || local_rows == 0) return RT_OK;
    if (!cam->CurrentImage.Data || !cam->PreviousImage.Data)
        return fail(RT_EINVAL, "rt_trace: CurrentImage/PreviousImage device pointers missing");
    const int rs = desc->EnableSIMD ? 0 : 1;
    TraceArgs a;
    memset(&a, 0, sizeof(a));
    a.groups = d->d_groups[rs];
    a.materials = d->d_mats[rs];
    a.rsqrt_lut = d->d_lut;
    a.weights = d->d_weights;
    a.prev = (float4 *)cam->PreviousImage.Data;
    a.cur = (uint32_t *)cam->CurrentImage.Data;
    a.rays = (unsigned long long *)d_rays;
    const rt_v3 *v[4] = {&cam->CameraPosition, &cam->CameraX, &cam->CameraY, &cam->FilmCenter};
    float *dst[4] = {a.cam_pos, a.cam_x, a.cam_y, a.film_center};
    for (int i = 0; i < 4; ++i) {
        dst[i][0] = v[i]->x;
        dst[i][1] = v[i]->y;
        dst[i][2] = v[i]->z;
    }
    a.film_w = cam->FilmW;
    a.film_h = cam->FilmH;
    a.width = desc->Width;
    a.height = desc->Height;
    // f64 division then rounding to f32 is the correctly rounded f32 quotient
    // (53 >= 2*24 + 2: double rounding is innocuous for division)
    a.inv_width = (float)(1.0 / (double)(float)desc->Width);
    a.inv_height = (float)(1.0 / (double)(float)desc->Height);
    a.local_rows = local_rows;
    a.prev_count = desc->PreviousRayCount;
    a.frames = desc->Frames;
    a.max_bounce = desc->MaxBounce;
    a.n_groups = d->n_groups[rs];
    a.n_spheres = d->n_spheres;
    a.use_sky = d->use_sky ? 1u : 0u;
    a.flags = ((desc->Flags & RT_FLAG_ACCUM_ZERO) ? kFlagAccumZero : 0u) |
              ((desc->Flags & RT_FLAG_SRGB_POW) ? kFlagSrgbPow : 0u);
    a.band_rows = band_rows;
    a.band_count = band_count;
    a.band_index = desc->BandIndex;
    a.prefilter = d->prefilter[rs];
    a.pf_relative = d->pf_relative[rs];
    a.fast_sqrt = d->fast_sqrt[rs];
    if (a.prefilter && d->n_cpairs[rs] &&
        (d->clusters_env == 2 || (d->clusters_env == 1 && d->n_groups[rs] <= kClAutoGroups))) {
        a.clusters = d->d_clusters[rs];
        a.n_cpairs = d->n_cpairs[rs];
        a.cl_words = d->cl_words[rs];
    }
    // Lanes that must wait before a secondary round runs: the dearer a wave's
    // secondary round (cluster pairs, or groups without clusters), the more it
    // pays to fill it first.  Measured (same box, Mrays/s, threshold 16/32/40/48):
    // RTWeekend (20 cluster pairs) 18.6k/19.4k/19.5k/19.5k, C5 at 512 spp (16)
    // 44.7k/46.3k/46.4k/46.4k, C2 (5) 153.8k/151.2k/150.4k/149.9k.  Round 4 (in-pixel
    // sample hand-out, 40/44/48/52): RTWeekend (per-lane thresholds) 25.61k/25.73k/25.74k/
    // 25.71k, C5 (scene-wide) 52.74k/52.44k/52.58k/52.38k: 48 for per-lane walks.
    a.merge_rounds = d->merge_env == 1 || (d->merge_env == -1 && d->n_groups[rs] <= kMergeGroups) ? 1u : 0u;
    // Round 5 (primary table, steady state): 24 for the small walks, against 16 / 32: C2 +1.2 %, C3 +1.0 %, the
    // 4-rank share -2.7 %, the 8-rank share -0.8 % (profiles/r05r_sec_threshold_ab.txt).
    a.sec_threshold = d->sec_threshold;
    if (a.sec_threshold == 0)
        a.sec_threshold = (a.clusters ? a.n_cpairs : a.n_groups) >= 12u ? (a.pf_relative ? 48u : 40u) : 24u;
    a.stats = d->d_stats;
    HIP_OK(hipSetDevice(d->ordinal));
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
    // Lanes per pixel (measured on MI355X at 1/2/4/8-way band splits of C2,
    // bench.py --sim-ranks, heaviest-first order at every P): 4 while the band
    // has >= 6k pixels per CU, 8 down to 3k, else 16 (round 4, with the in-pixel
    // sample hand-out: the 4-rank share 1.19-1.23 ms at P = 16 against 1.25-1.28
    // at P = 8; the 2-rank share 2.26-2.27 at P = 8, 2.29 at P = 16; more lanes per pixel
    // shorten the per-lane sample chains that form the launch tail; C2 rank
    // shares: 1 GPU P=4 6.21 ms (P=8 6.29, P=16 6.62); 2 ranks P=8 3.26 ms
    // (P=4 3.35); 4 ranks P=8 = P=16 1.81 ms; 8 ranks P=16 1.02 ms (P=8
    // 1.47)); never more lanes than frames.
    int lpp = d->lanes_per_pixel;
    const bool auto_lpp = lpp == 0;
    if (lpp == 0) {
        const uint64_t pixels = (uint64_t)desc->Width * local_rows;
        lpp = pixels >= (uint64_t)d->cu_count * 6144u ? 4 : pixels >= (uint64_t)d->cu_count * 3072u ? 8 : 16;
        while (lpp > 1 && (uint32_t)lpp / 2u >= desc->Frames) lpp /= 2;
    }
    // One lane per pixel, and one frame (the reference's OnRender unit): each lane
    // takes kPixelsPerLane pixels in turn (launch shape 0, rt_kernel.hip Shape<0>),
    // so a wave stays full after its first pass and the launch has a quarter of
    // the waves.  Measured on the 1080p OnRender frame: see DESIGN.md §6a.
    const uint32_t pixels_per_lane =
        lpp == 1 && !(desc->Flags & RT_FLAG_SRGB_POW) &&
                (d->pixels_per_lane_env == 4 || (d->pixels_per_lane_env == 0 && auto_lpp && desc->Frames == 1))
            ? 4u : 1u;
    const uint32_t lanes = (uint32_t)lpp;  // lanes per pixel (the sample chains of a pixel)
    if (pixels_per_lane > 1) lpp = 0;      // the launch shape code of rtk_* (0: pixels per lane)
    // Tile scheduling.  Block tiles (2TW x 2TH pixels) are traced in the order
    // tile_order[0 .. n_live): with culling, the cull pass (once per camera /
    // scene / geometry) writes every wave tile's primary group mask and a
    // live-first order, and dead tiles (no candidate group anywhere, no sky)
    // never reach the trace kernel -- rtk_launch_empty folds their pixels.
    // With heaviest-first scheduling each launch also measures its tiles and
    // re-sorts them for the next launch (live tiles keep costs > 0, dead ones
    // 0, so the live prefix is preserved).
    if (d->want_wave_times) {  // one {start, end} per wave of this launch's tile shape
        const size_t waves = (size_t)rtk_tile_count(desc->Width, local_rows, lpp) * 4u;
        if (waves > d->wave_times_cap) {
            (void)hipFree(d->d_wave_times);
            d->d_wave_times = nullptr;
            if (hipMalloc(&d->d_wave_times, waves * 16u) != hipSuccess) return fail(RT_ENOMEM, "wave_times");
            d->wave_times_cap = waves;
        }
        a.wave_times = d->d_wave_times;
    }
    a.interleave = d->interleave_env && lpp >= 2 ? 1u : 0u;
    // The rsqrt and fold tables (10 KB) leave the LDS image at P = 16, whose 4-wave
    // ring (10 KB) would otherwise cap a CU at 6 blocks: measured on the 8-rank C2
    // share 0.900-0.903 against 0.914-0.922 ms; at P = 4 they stay (C2 -1.8 % without)
    const bool tables = !d->tables_global_env && lpp <= 8;
    a.lut_in_lds = rtk_lut_in_lds(a.n_groups) && tables ? 1u : 0u;
    a.fold_in_lds = rtk_fold_in_lds(a.n_groups) && tables ? 1u : 0u;
    a.scene_in_lds = a.n_groups <= kMaxLdsGroups && !d->scene_global_env ? 1u : 0u;
    if (d->solo_env && d->src == kSrcSmem) {  // one-wave workgroups keep no LDS image
        a.solo = 1u;
        a.lut_in_lds = a.fold_in_lds = a.scene_in_lds = 0u;
        if (!a.clusters) a.walk = kWalkGroups;
        else if (a.cl_words == 1u) a.walk = a.pf_relative ? kWalkCl1Rel : kWalkCl1;
        else if (a.cl_words == 2u) a.walk = a.pf_relative ? kWalkCl2Rel : kWalkCl2;
        else a.walk = a.pf_relative ? kWalkCl4Rel : kWalkCl4;
        if (d->walk_any_env) a.walk = kWalkAny;
    }
    const int src = a.scene_in_lds ? d->src : kSrcSmem;  // a scene in HBM is read through the scalar cache
    const uint32_t n_tiles = rtk_tile_count(desc->Width, local_rows, lpp);
    // Units of the heaviest-first order: waves for the one-wave kernels (each wave
    // its own workgroup, so each is placed by its own cost), block tiles otherwise
    a.unit_waves = a.solo && d->wave_order_env ? 1u : 0u;
    const uint32_t n_units = a.unit_waves ? 4u * n_tiles : n_tiles;
    const uint32_t n_words = rtk_mask_words(a.n_groups);
    const bool cull = d->cull != 0;
    const bool empty_capable = cull && !d->use_sky && desc->MaxBounce != 0;
    const bool sched = d->tile_sched != 0;
    a.tiles_x = rtk_tiles_x(desc->Width, lpp);
    std::vector<uint32_t> key = {desc->Width, desc->Height, local_rows, band_rows, band_count, desc->BandIndex,
                                 (uint32_t)lpp, (uint32_t)rs, (uint32_t)cull, (uint32_t)empty_capable, (uint32_t)sched,
                                 a.interleave, a.unit_waves,
                                 (uint32_t)d->scene_gen, (uint32_t)(d->scene_gen >> 32)};
    for (const float *f : {a.cam_pos, a.cam_x, a.cam_y, a.film_center}) {
        for (int i = 0; i < 3; ++i) {
            uint32_t u;
            memcpy(&u, f + i, 4);
            key.push_back(u);
        }
    }
    for (const float f : {a.film_w, a.film_h}) {
        uint32_t u;
        memcpy(&u, &f, 4);
        key.push_back(u);
    }
    if (!d->tile_stream_set || s != d->tile_stream) {
        // order, masks and costs are written and read in stream order: on a new
        // stream, every launch issued on the previous one must have finished (the
        // previous stream may be gone, so the wait is for the device; switching
        // streams is rare -- every caller here keeps one per device)
        if (d->tile_stream_set) HIP_OK(hipDeviceSynchronize());
        d->tile_stream = s;
        d->tile_stream_set = true;
    }
    // (no allocation here once rt_device_reserve has sized the buffers for this geometry)
    if (const int rc = ensure_tile_buffers(d, n_tiles, s, false)) return rc;
    const size_t mask_words = (size_t)n_tiles * 4u * n_words;
    if (cull)
        if (const int rc = ensure_masks(d, mask_words, s, false)) return rc;
    // pixels dealt to waves by cost (options PixelSort): block tiles of at most 64 pixels
    const bool pixel_sort = d->pixel_sort_env && sched && lpp >= 4 && !a.interleave;
    if (pixel_sort)
        if (const int rc = ensure_pixel_sort(d, n_tiles, (size_t)desc->Width * local_rows, s, false)) return rc;
    const bool new_key = key != d->tile_key;
    // (the table is written by the key's cull pass: the key holds the camera and the scene)
    a.prim = cull ? d->d_prim[rs] : nullptr;
    uint32_t head_frames = 0;  // > 0: split this launch (first launch of a key, below): frames of the leading parts
    uint32_t split[8], n_split = 0;
    if (new_key) {
        d->tile_key = key;
        d->n_sorts = 0;
        if (pixel_sort) HIP_OK(hipMemsetAsync(d->d_pix_perm, 0xFF, (size_t)n_tiles * 64u, s));  // identity
        if (cull) {
            a.masks = d->d_masks;
            d->mask_words = mask_words;
            if (rtk_launch_cull(&a, lpp, d->d_tile_live, d->d_tile_cost, d->d_cull_counters, empty_capable ? 1 : 0, s) !=
                    0 ||
                rtk_launch_tile_sort(d->d_tile_cost, d->d_tile_order, d->d_tile_scratch, n_units, s) != 0)
                return fail(RT_EIO, "rt_trace: cull pass launch failed: %s", hipGetErrorString(hipGetLastError()));
            // the totals follow asynchronously (resolve_counts); no host wait here
            HIP_OK(hipMemcpyAsync(d->h_counts, d->d_cull_counters + kCullTotals, 2 * sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, s));
            HIP_OK(hipEventRecord(d->ev_counts, s));
            d->counts_known = false;
            d->tile_order_valid = true;
            // The first launch of a key has no measured tile costs, and in the cull
            // pass's live-first order its heavy tiles start late and form the tail
            // (C2 cold 7.7 ms against 5.4 warm).  A long launch is therefore split:
            // its first head_samples samples per lane (1/8 of C2's work) run in that
            // order and measure the tile costs, and the remaining frames continue the
            // running mean heaviest-first.  Splitting a launch at a frame boundary
            // changes no bit: the owner lane folds frames in order either way, and
            // frame k's seed and weights depend on PreviousRayCount + k only.
            const uint32_t split_min = 4u * d->head_samples * lanes;
            if (sched && d->split_env && desc->Frames >= split_min) {
                // leading parts of head_samples, x split_growth, ... samples per lane
                // while the rest keeps at least half the frames
                uint32_t f = d->head_samples * lanes, used = 0;
                for (uint32_t i = 0; i + 1 < d->split_parts && used + f <= desc->Frames / 2u; ++i) {
                    split[n_split++] = f;
                    used += f;
                    f *= d->split_growth;
                }
                head_frames = used;
            }
        } else {
            HIP_OK(hipMemsetAsync(d->d_tile_cost, 0, n_units * 4u, s));
            // no cull pass: every block tile is live, and the totals word the XCD grouping reads
            // (rtk_launch_xcd_group) says so (u64 little-endian: low word n_tiles, the rest 0)
            HIP_OK(hipMemsetAsync(d->d_cull_counters + kCullTotals, 0, 2 * sizeof(unsigned long long), s));
            HIP_OK(hipMemsetD32Async((hipDeviceptr_t)(d->d_cull_counters + kCullTotals), n_tiles, 1, s));
            d->n_live = n_tiles;
            d->dead_pixels = 0;
            d->counts_known = true;
            d->tile_order_valid = false;  // identity until a measured sort exists
        }
    }
    // live-tile count: on the host once the cull totals have landed, else read
    // by the kernels from the device (grid over every tile, early exit)
    const bool known = resolve_counts(d, false);
    const uint32_t grid_tiles = known ? d->n_live : n_tiles;
    a.live_total = known ? nullptr : d->d_cull_counters + kCullTotals;
    const bool any_live = !known || d->n_live > 0;
    const bool any_dead = empty_capable && (!known || d->n_live < n_tiles);
    a.masks = cull ? d->d_masks : nullptr;
    a.tile_order = d->tile_order_valid ? d->d_tile_order : nullptr;
    a.tile_cost = sched ? d->d_tile_cost : nullptr;
    a.pix_perm = pixel_sort ? d->d_pix_perm : nullptr;
    a.pix_seg = d->pixel_seg;
    // (multi-frame launches only: a one-frame launch, OnRender's, keeps its store and one kernel fewer)
    a.skip_cur = d->cur_pass && lpp >= 2 ? 1u : 0u;
    d->last.PixelsSorted = pixel_sort && !new_key && d->n_sorts > 0 ? 1u : 0u;
    d->last_n_tiles = n_tiles;
    d->last_frames = desc->Frames;
    d->last_empty_capable = empty_capable;
    d->last.LanesPerPixel = lanes;
    d->last.PixelsPerLane = pixels_per_lane;
    d->last.TilesTotal = n_tiles;
    d->last.CullPassRan = cull && new_key ? 1u : 0u;
    d->last.OrderedLaunches = d->n_sorts;
    d->last.ClusteredWalk = a.clusters ? 1u : 0u;
    d->last.GroupsPerRuleSet = a.n_groups;
    d->last.OneWaveGroups = a.solo;
    d->last.Walk = a.walk;
    // one launch, or the split of a key's first launch (above): the leading
    // parts, then the rest, each continuing the running mean heaviest-first
    split[n_split++] = desc->Frames - head_frames;
    uint32_t done_frames = 0;
    for (uint32_t part = 0; part < n_split; ++part) {
        if (part > 0) {
            a.prev_count = desc->PreviousRayCount + done_frames;
            a.flags &= ~kFlagAccumZero;
            a.tile_order = d->d_tile_order;
        }
        a.frames = split[part];
        done_frames += split[part];
        const bool resort = sched && any_live && (d->n_sorts < d->order_launches || part + 1 < n_split);
        a.pix_cost = pixel_sort && resort ? d->d_pix_cost : nullptr;
        // wave costs only for a launch whose costs are sorted: once the order is kept, the
        // per-wave 4-B cost stores (scattered partial lines, ~8 MB of HBM writes per 1080p
        // launch at P = 4) would feed nothing
        a.tile_cost = resort ? d->d_tile_cost : nullptr;
        if (rtk_launch_trace_grid(&a, desc->EnableSIMD ? 1 : 0, src, cull ? 1 : 0, lpp, grid_tiles, s) != 0)
            return fail(RT_EIO, "rt_trace: kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
        if (any_dead && rtk_launch_empty(&a, lpp, d->d_tile_live, d->d_cull_counters + kCullTotals + 1, s) != 0)
            return fail(RT_EIO, "rt_trace: empty-tile launch failed: %s", hipGetErrorString(hipGetLastError()));
        // the learned order settles within a few launches (C2: 7.7, 6.3, 6.1, 5.9,
        // 5.8 ms); after order_launches re-sorts (RT_ORDER_LAUNCHES, default 4)
        // the order is kept and the three sort kernels (~14 us per launch, 1.5 %
        // of an 8-rank C2 share) are skipped
        if (resort) {
            d->n_sorts += 1;
            // one-wave kernels: sort, then group each block tile's waves onto one XCD
            const bool group = a.unit_waves && (d->xcd_group_env == 1 || (d->xcd_group_env < 0 && lpp <= 4));
            if (rtk_launch_tile_sort(d->d_tile_cost, group ? d->d_tile_order_sorted : d->d_tile_order,
                                     d->d_tile_scratch, n_units, s) != 0 ||
                (group && rtk_launch_xcd_group(d->d_tile_order_sorted, d->d_tile_order, n_units,
                                               d->d_cull_counters + kCullTotals, d->d_tile_scratch, d->d_tile_aux,
                                               s) != 0))
                return fail(RT_EIO, "rt_trace: tile sort launch failed: %s", hipGetErrorString(hipGetLastError()));
            if (pixel_sort && rtk_launch_pixel_sort(&a, lpp, d->d_pix_perm, s) != 0)
                return fail(RT_EIO, "rt_trace: pixel sort launch failed: %s", hipGetErrorString(hipGetLastError()));
            d->tile_order_valid = true;
        }
    }
    // options EncodePass: the RGBA8 band image from the running mean the kernels stored (main.cpp:490's
    // store on its own, the same bits), written by one coalesced pass
    if (a.skip_cur && desc->Frames > 0 &&
        rtk_launch_encode(a.prev, a.cur, (uint64_t)local_rows * desc->Width, (a.flags & kFlagSrgbPow) ? 1u : 0u, s) != 0)
        return fail(RT_EIO, "rt_trace: RGBA8 encode launch failed: %s", hipGetErrorString(hipGetLastError()));
    d->last.SplitHeadFrames = head_frames;
    return RT_OK;
}

extern "C" int rt_assemble_bands(const void *d_compact, uint64_t rank_stride_bytes, void *d_dst, uint32_t width,
                                 uint32_t height, uint32_t elem_bytes, uint32_t band_rows, uint32_t band_count,
                                 void *stream) {
    if (!d_compact || !d_dst || width == 0 || height == 0 || elem_bytes == 0 || band_rows == 0 || band_count == 0)
        return fail(RT_EINVAL, "rt_assemble_bands: bad argument");
    for (uint32_t r = 0; r < band_count; ++r)
        if ((uint64_t)rt_band_local_rows(height, band_rows, band_count, r) * width * elem_bytes > rank_stride_bytes)
            return fail(RT_EINVAL, "rt_assemble_bands: rank stride too small for rank %u", r);
    if (rtk_launch_assemble(d_compact, rank_stride_bytes, d_dst, width, height, elem_bytes, band_rows, band_count,
                            (hipStream_t)stream) != 0)
        return fail(RT_EIO, "rt_assemble_bands: launch failed");
    return RT_OK;
}

extern "C" int rt_encode_rgba8(const float *d_accum_v4, uint32_t *d_rgba8, uint64_t n_pixels, uint32_t flags,
                               void *stream) {
    if ((!d_accum_v4 || !d_rgba8) && n_pixels) return fail(RT_EINVAL, "rt_encode_rgba8: NULL buffer");
    if (flags & ~RT_FLAG_SRGB_POW) return fail(RT_EINVAL, "rt_encode_rgba8: unknown flags 0x%x", flags);
    if (rtk_launch_encode(d_accum_v4, d_rgba8, n_pixels, (flags & RT_FLAG_SRGB_POW) ? 1u : 0u, (hipStream_t)stream) != 0)
        return fail(RT_EIO, "rt_encode_rgba8: launch failed");
    return RT_OK;
}

extern "C" int rt_trace_last_info(rt_device *d, rt_trace_info *out) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !out) return fail(RT_EINVAL, "rt_trace_last_info: NULL argument");
    // the live/dead totals of the last launch's key: waits for them if they
    // are still on their way from the device (the only blocking part)
    HIP_OK(hipSetDevice(d->ordinal));
    if (!resolve_counts(d, true)) return fail(RT_EIO, "rt_trace_last_info: cull totals: %s",
                                              hipGetErrorString(hipGetLastError()));
    d->last.TilesTraced = d->n_live;
    d->last.SegmentsFolded = d->last_empty_capable && d->n_live < d->last_n_tiles
                                 ? d->dead_pixels * d->last_frames : 0u;
    *out = d->last;
    return RT_OK;
}

extern "C" int rt_device_synchronize(rt_device *d) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d) return fail(RT_EINVAL, "rt_device_synchronize: NULL device");
    HIP_OK(hipSetDevice(d->ordinal));
    return quiesce(d);
}

extern "C" int rt_debug_stats(rt_device *d, uint64_t out[32], int reset) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !out) return fail(RT_EINVAL, "rt_debug_stats: NULL argument");
    memset(out, 0, 32 * sizeof(uint64_t));
    if (!d->d_stats) return 0;
    HIP_OK(hipSetDevice(d->ordinal));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, d->d_stats, kStatSlots * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (reset) HIP_OK(hipMemset(d->d_stats, 0, kStatSlots * sizeof(unsigned long long)));
    return 1;
}

extern "C" int64_t rt_debug_masks(rt_device *d, uint64_t *out, uint64_t max_words) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !out) return fail(RT_EINVAL, "rt_debug_masks: NULL argument");
    if (!d->d_masks || d->tile_key.empty() || !d->mask_words) return 0;
    const uint64_t n = max_words < d->mask_words ? max_words : d->mask_words;
    HIP_OK(hipSetDevice(d->ordinal));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, d->d_masks, n * 8u, hipMemcpyDeviceToHost));
    return (int64_t)n;
}

extern "C" int64_t rt_debug_wave_times(rt_device *d, uint64_t *out, uint64_t max_waves) {
    DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!d || !out) return fail(RT_EINVAL, "rt_debug_wave_times: NULL argument");
    if (!d->d_wave_times) return 0;
    const uint64_t n = max_waves < d->wave_times_cap ? max_waves : d->wave_times_cap;
    HIP_OK(hipSetDevice(d->ordinal));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, d->d_wave_times, n * 16u, hipMemcpyDeviceToHost));
    return (int64_t)n;
}
