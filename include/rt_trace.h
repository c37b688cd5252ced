/*
 * rt_trace.h — C-ABI of the MI355X-native brute-force sphere trace path.
 *
 * Drop-in boundary for the per-pixel trace loop of Ne0nWinds/SIMD-Ray-Tracer
 * (reference @ 2025-01-03).  The reference has no FFI; its path boundary is
 *   (a) the tile callback launched by WorkQueueStart(RenderTile | RenderTileScalar,
 *       TilesX*TilesY, ThreadCount)                     main.cpp:851-856, base.h:166-178
 *       reading the globals CameraInfo, Scenes[SceneIndex], PreviousRayCount,
 *       ThreadContexts                                   main.cpp:7, 53-54, 289-290
 *   (b) the app entry points OnInit / OnRender           base.h:163-164, main.cpp:645-859
 * Every entry point below names the reference interface it replaces.
 *
 * Conventions: plain C types, pointers and sizes only.  Functions return 0 on
 * success or a negative errno-style code (RT_E*).  Calls on one rt_device are
 * single-threaded; each device owns one HIP stream unless a stream is passed.
 * Structs marked "byte-compatible" have the reference's exact layout
 * (offsets asserted in simd-ray-tracer_amd/csrc/rt_host.cpp and tests/).
 */
#ifndef RT_TRACE_H
#define RT_TRACE_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_TRACE_ABI_VERSION 1u
#define RT_ALIGN16 __attribute__((aligned(16)))

/* Error codes (negative errno values). */
#define RT_OK 0
#define RT_EINVAL (-22)  /* bad argument / shape */
#define RT_ENOMEM (-12)  /* allocation failed */
#define RT_ENODEV (-19)  /* no HIP device / HIP runtime error */
#define RT_EBUSY (-16)   /* previous frame still in flight */
#define RT_EIO (-5)      /* HIP/RCCL error while running */

/* ------------------------------------------------ byte-compatible structs */

/* v3: base.h:357-375 (4 floats, 16-byte aligned, _w padding lane). */
typedef struct rt_v3 {
    float x, y, z, _w;
} RT_ALIGN16 rt_v3;

/* material: main.cpp:11-16 — 48 B. */
typedef struct rt_material {
    rt_v3 Color;
    rt_v3 Emissive;
    float Specular;
    float IndexOfRefraction; /* 0 = diffuse/specular, else dielectric */
} rt_material;

/* scalar_sphere: main.cpp:17-21 — 80 B. */
typedef struct rt_scalar_sphere {
    rt_v3 Position;
    float Radius;
    rt_material Material;
} rt_scalar_sphere;

/* sphere_group: main.cpp:23-26 with SIMD_WIDTH = 4 (v3x4 + f32x4) — 64 B. */
typedef struct rt_sphere_group {
    float X[4], Y[4], Z[4], Radii[4];
} RT_ALIGN16 rt_sphere_group;

/* array<T>: main.cpp:28-40 — 16 B. */
typedef struct rt_array {
    void *Data;
    uint32_t Count;
} rt_array;

/* scene: main.cpp:42-51 — 80 B. */
typedef struct rt_scene {
    rt_v3 LookAt;
    bool UseSkyColor;
    float DefaultDistanceFromLookAt;
    float DefaultXAngle;
    float DefaultYHeight;
    rt_array ScalarSpheres; /* rt_scalar_sphere[Count] */
    rt_array SIMDSpheres;   /* rt_sphere_group[Count]  */
    rt_array Materials;     /* rt_material[Count]      */
} rt_scene;

/* format / image: base.h:117-136 — 24 B. */
#define RT_FORMAT_R32B32G32A32_F32 1u
#define RT_FORMAT_R8G8B8A8_U32 2u
typedef struct rt_image {
    void *Data;
    uint32_t Width, Height;
    uint32_t Format;
} rt_image;

/* camera_info: main.cpp:270-282 — 144 B. */
typedef struct rt_camera_info {
    rt_v3 CameraPosition;
    rt_v3 CameraZ;
    rt_v3 CameraX;
    rt_v3 CameraY;
    rt_v3 FilmCenter;
    float FilmW;
    float FilmH;
    uint32_t TilesX;
    rt_image CurrentImage;  /* RGBA8 u32 per pixel   */
    rt_image PreviousImage; /* v4 f32 running mean   */
} rt_camera_info;

/* render_params: base.h:157-161 — 12 B. */
typedef struct rt_render_params {
    uint32_t ThreadCount; /* ignored on the GPU (kept for the signature) */
    bool EnableSIMD;      /* true: RenderTile rules, false: RenderTileScalar rules */
    uint32_t SceneIndex;
} rt_render_params;

/* init_params: base.h:152-155 (string8 = {char*, u32}). */
typedef struct rt_init_params {
    uint32_t WindowWidth, WindowHeight;
    const char *WindowTitle;
    uint32_t WindowTitleSize;
} rt_init_params;

/* ------------------------------------------------------ host-side inputs */

/* Built-in scenes 0 RGB Glass, 1 Floating Spheres, 2 RTWeekend, generated
 * exactly as InitRGBSphereScene / InitRandomizedSphereScene /
 * InitRTWeekendSphereScene (main.cpp:96-268).  The returned scene points at
 * library-owned static storage (like the reference's static arrays). */
int rt_scene_builtin(uint32_t index, rt_scene *out);

/* First `n_spheres` spheres of `in` (the BASELINE "N-sphere" synthetic
 * scenes are prefixes of scene 1): counts become n, ceil(n/4), n+1; the
 * data pointers are shared. */
int rt_scene_prefix(const rt_scene *in, uint32_t n_spheres, rt_scene *out);

/* Camera basis + film for an orbit around scene->LookAt, exactly as
 * OnRender computes it (main.cpp:763-838, x87 fcos/fsin).  Image fields
 * of `out` are zeroed; the caller fills them. */
int rt_camera_setup(const rt_scene *scene, float distance_from_look_at, float x_angle, float y_height,
                    uint32_t width, uint32_t height, rt_camera_info *out);

/* Per-(pixel, frame) seed of the GPU's 'pixel' seed mode: the per-thread
 * mixer of main.cpp:668-675 applied to i = (k*H + y)*W + x. */
uint64_t rt_pixel_seed(uint32_t x, uint32_t y, uint32_t frame, uint32_t width, uint32_t height);

/* -------------------------------------------------------- device context */

typedef struct rt_device rt_device;

/* Replaces OnInit's allocation + WorkQueueCreate (main.cpp:658-665).  The
 * device runs the default kernels (every field of rt_device_options 0); the
 * library reads no environment variable that changes what it computes or
 * how (only the diagnostic RT_STATS / RT_WAVETIMES hooks, below). */
int rt_device_create(int hip_device, rt_device **out);
int rt_device_destroy(rt_device *dev);

/* Kernel and schedule choices of one device, fixed at creation.  Every
 * choice gives the same bits (each is parity-tested against the oracle); they
 * exist for A/B measurements and for the brute-force roofline (Cull and
 * Prefilter RT_OPT_OFF: every counted segment tests every sphere, as
 * main.cpp:399-430 does).  The reference's only run-time knobs are
 * render_params (base.h:157-161: ThreadCount, EnableSIMD, SceneIndex), which
 * rt_trace_desc carries.  Tri-state fields: RT_OPT_DEFAULT (0), RT_OPT_ON (1),
 * RT_OPT_OFF (-1); numeric fields: 0 = the default.  A zero-filled struct is
 * rt_device_create's behaviour. */
#define RT_OPT_DEFAULT 0
#define RT_OPT_ON 1
#define RT_OPT_OFF (-1)
typedef struct rt_device_options {
    uint32_t Size;               /* sizeof(rt_device_options), or 0                                  */
    int32_t Cull;                /* primary-ray cone cull and dead-tile fold (default on)            */
    int32_t Prefilter;           /* secondary-ray prefilter (default: per scene)                     */
    int32_t PrefilterRelative;   /* per-lane prefilter thresholds (default: per scene)               */
    int32_t Clusters;            /* cluster walk (default: scenes of <= 64 groups; ON: any size)     */
    int32_t ClusterCount;        /* k-means top clusters K >= 2 (0: ~1.25 sqrt(n) or n / 8..17)      */
    int32_t SubClusterSpheres;   /* spheres per sub-cluster of two-level tables (0: 3, per-lane 4)   */
    int32_t SecondaryThreshold;  /* lanes a secondary round waits for (0: 24/40/48 by walk size)     */
    int32_t LanesPerPixel;       /* 1/2/4/8/16/32 sample chains per pixel (0: per launch)            */
    int32_t PixelsPerLane;       /* 1 never, 4 always (0: 4 for one-frame one-lane launches)         */
    int32_t OneWaveGroups;       /* one wave per workgroup, no LDS image (default on)                */
    int32_t SphereSourceLds;     /* four-wave kernels read spheres from LDS, not SMEM (default off)  */
    int32_t SceneInHbm;          /* four-wave kernels keep the scene out of LDS (default off)        */
    int32_t TablesInLds;         /* four-wave kernels' rsqrt / fold tables in LDS at P <= 8 (on)     */
    int32_t WalkAny;             /* the one-wave kernel picks its walk at run time (default off)     */
    int32_t Interleave;          /* wave tiles interleaved over the block tile (default off)         */
    int32_t MergeRounds;         /* primary + secondary rays in every round (default: <= 2 groups)   */
    int32_t TileOrder;           /* heaviest-first order learned from earlier launches (default on)  */
    int32_t WaveOrder;           /* one-wave kernels order waves, not block tiles (default on)       */
    int32_t PixelSort;           /* a block tile's pixels dealt to its waves by cost (default on)    */
    int32_t PixelSegment;        /* pixels per dealt unit: 1, 2 or 4 (0: 1)                          */
    int32_t XcdGroup;            /* a block tile's waves on one XCD (default: launches at P <= 4)    */
    int32_t SplitFirstLaunch;    /* a key's first long launch measures costs first (default on)      */
    int32_t HeadSamples;         /* samples per lane of that split's head (0: 8)                     */
    int32_t SplitParts;          /* launches of the split, 1..8 (0: 2)                               */
    int32_t SplitGrowth;         /* each leading part this many times the previous (0: 3)            */
    int32_t OrderLaunches;       /* re-sorts per key before the order is kept (0: 4; -1: none)       */
    int32_t EncodePass;          /* RGBA8 by a coalesced pass after multi-frame launches (default on) */
} rt_device_options;

/* rt_device_create with options (NULL: the defaults).  RT_EINVAL for a value
 * out of range or a Size this library does not know. */
int rt_device_create_ex(int hip_device, const rt_device_options *options, rt_device **out);
/* The options the device was created with (as given, defaults left 0). */
int rt_device_get_options(rt_device *dev, rt_device_options *out);

/* x86 rsqrtss reproduction table (2 x 1024 f32): makes
 * v3::NormalizeFast (x64_math.h:246-257) bit-exact on the GPU. Required. */
int rt_set_rsqrt_table(rt_device *dev, const float table[2048]);

/* The built-in table: rsqrtss as captured on an Intel host (the parity
 * target; tests/golden/rsqrt_lut_intel.bin). */
int rt_rsqrt_table_builtin(float table_out[2048]);

/* Captures this host CPU's own rsqrtss into a table (x86 only).  Returns
 * RT_EINVAL when the host's rsqrtss is not representable by a parity +
 * 10-bit table (checked on a sample of inputs). */
int rt_rsqrt_table_capture_host(float table_out[2048]);

/* Uploads Scenes[SceneIndex] (read by RenderTile at main.cpp:370) into
 * HBM: SIMDSpheres/Materials for the SIMD rules, ScalarSpheres for the
 * scalar rules.  The scene is copied; the caller keeps ownership.  The
 * default one-wave kernels read every scene from HBM through the caches; the
 * four-wave kernels (rt_device_options OneWaveGroups off) also stage scenes of up to 656 spheres (164
 * groups) in each block's LDS.  Up to RT_MAX_SPHERES.
 * RT_EINVAL for a scene with no spheres (every built-in scene has some) or
 * more than RT_MAX_SPHERES. */
#define RT_MAX_SPHERES 16384u
int rt_scene_upload(rt_device *dev, const rt_scene *scene);

/* --------------------------------------------------------------- tracing */

#define RT_SEED_PIXEL 1u        /* per-(pixel, frame) PCG seed (GPU parity mode) */
#define RT_FLAG_ACCUM_ZERO 1u   /* PreviousImage treated as all-zero (not read) */
#define RT_FLAG_SRGB_POW 2u     /* RGBA8 through LinearToSRGB's exact-pow branch (main.cpp:320-321, '#if 0'
                                   in the reference) instead of its sqrt one; PreviousImage is unaffected */

typedef struct rt_trace_desc {
    uint32_t Width, Height;   /* full image (CurrentImage.Width/Height)          */
    uint32_t PreviousRayCount;/* frames already folded into PreviousImage (main.cpp:7) */
    uint32_t Frames;          /* progressive frames (samples/pixel) to fold now  */
    uint32_t MaxBounce;       /* the reference literal is 5 (main.cpp:387)       */
    uint32_t EnableSIMD;      /* 1 RenderTile rules, 0 RenderTileScalar rules    */
    uint32_t SeedMode;        /* RT_SEED_PIXEL                                   */
    uint32_t BandRows;        /* row-band height, a multiple of 8 (bench: 8)     */
    uint32_t BandCount;       /* bands are dealt round-robin over BandCount GPUs */
    uint32_t BandIndex;       /* this GPU's residue                              */
    uint32_t Flags;           /* RT_FLAG_*                                       */
} rt_trace_desc;

/* Number of image rows owned by band residue `band_index` (the compact
 * per-GPU framebuffer height). */
uint32_t rt_band_local_rows(uint32_t height, uint32_t band_rows, uint32_t band_count, uint32_t band_index);

/* Replaces WorkQueueStart(RenderTile|RenderTileScalar, TilesX*TilesY, N)
 * (main.cpp:851-856) for `Frames` consecutive frames: traces every pixel
 * of this GPU's bands, folds each frame into the running mean and stores
 * the sRGB RGBA8 of the last one.  cam->CurrentImage.Data and
 * cam->PreviousImage.Data are DEVICE pointers to compact band-local images
 * (rt_band_local_rows x Width).  `d_rays` (device u64) is incremented by
 * the bounce segments traced (RaysCastInThread, main.cpp:390).
 * Asynchronous on `stream` (hipStream_t; NULL = the HIP null stream): the
 * host never waits.  The first launch for a new camera / scene / geometry on
 * this device runs the primary-ray cull pass; its live-tile count stays on
 * the device (the trace grid covers every tile and blocks past the count
 * exit) until it has reached the host asynchronously, after which launches
 * of the same key size their grids exactly.  Launches of one device are meant
 * for one stream: when the stream changes between launches, the call first
 * waits for the device (host-side), as it does when it grows its buffers for
 * a larger geometry than any before.  PreviousRayCount + Frames must fit a u32. */
int rt_trace(rt_device *dev, const rt_camera_info *cam, const rt_trace_desc *desc,
             uint64_t *d_rays, void *stream);

/* What the last rt_trace on `dev` launched.  Host-side bookkeeping, except
 * that TilesTraced and SegmentsFolded need the cull pass's totals: when the
 * last launch's key is new and they have not reached the host yet, this call
 * waits for them (the only blocking part).  The reference counts every bounce segment, misses
 * included (RaysCastInThread, main.cpp:390); segments of pixels whose every
 * sample provably misses (no primary ray of their tile can reach a sphere,
 * no sky term) are counted analytically and folded by a pixel kernel rather
 * than traced: SegmentsFolded of the launch's ray count are such segments. */
typedef struct rt_trace_info {
    uint64_t SegmentsFolded;  /* dead-tile segments counted, not traced      */
    uint32_t LanesPerPixel;   /* P of the launch (sample chains per pixel)   */
    uint32_t TilesTotal;      /* block tiles of the band geometry            */
    uint32_t TilesTraced;     /* live tiles launched on the trace kernel     */
    uint32_t CullPassRan;     /* 1: this launch ran the primary-ray cull pass */
    uint32_t OrderedLaunches; /* heaviest-first re-sorts done for this key   */
    uint32_t ClusteredWalk;   /* 1: secondary rays used the cluster walk     */
    uint32_t GroupsPerRuleSet;/* sphere groups of the rule set traced        */
    uint32_t SplitHeadFrames; /* > 0: a key's first launch ran as two trace
                                 launches, these frames first in the cull
                                 pass's order (measuring tile costs), the rest
                                 heaviest-first; the same bits as one launch  */
    uint32_t OneWaveGroups;   /* 1: one wave per workgroup (no LDS image)    */
    uint32_t Walk;            /* secondary walk compiled into the kernel: 0
                                 run-time dispatch, 1 per-group loops, 2/3/4
                                 cluster walk with 1/2/4 mask words, 5/6/7
                                 the same with per-lane thresholds           */
    uint32_t PixelsPerLane;   /* 4: each lane traced 4 pixels in turn (one-lane-
                                 per-pixel launches of one frame), else 1     */
    uint32_t PixelsSorted;    /* 1: the block tiles' pixels were dealt to their
                                 waves by the previous launch's costs (P >= 4;
                                 PixelSort off disables)                      */
    uint32_t BufferGrowths;   /* launch-buffer (re)allocations on this device
                                 so far (tile lists, cull masks): constant
                                 across launches that rt_device_reserve covers */
} rt_trace_info;
int rt_trace_last_info(rt_device *dev, rt_trace_info *out);

/* Pre-sizes the device's launch buffers (tile order / cost / live lists, the
 * cull pass's masks and counters) for bands of up to `width` x `local_rows`
 * pixels under every lanes-per-pixel shape rt_trace may pick, so that no later
 * rt_trace of such a band allocates or waits for the device (growing a buffer
 * otherwise synchronises the launch's stream).  Successive calls keep the
 * largest tile and pixel counts over the geometries asked for (not the largest
 * width times the largest height).  Masks are sized for the current scene;
 * rt_scene_upload re-applies the reservation for a larger one (if that fails,
 * the upload still succeeds and the reservation is dropped: later launches
 * grow their buffers as they need).  Waits for the device.  (New; the reference's arena is sized once in OnInit,
 * main.cpp:658.) */
int rt_device_reserve(rt_device *dev, uint32_t width, uint32_t local_rows);

/* ColorFromV4(LinearToSRGB(v)) (main.cpp:312-346, the store at :490) over a
 * device-resident running mean: n_pixels v4 f32 -> RGBA8, both DEVICE
 * pointers, enqueued on `stream` (NULL: the null stream).  flags: 0 or
 * RT_FLAG_SRGB_POW.  rt_trace already stores the RGBA8 of every frame it
 * folds; this re-encodes a gathered or saved accumulation without tracing. */
int rt_encode_rgba8(const float *d_accum_v4, uint32_t *d_rgba8, uint64_t n_pixels, uint32_t flags, void *stream);

/* Multi-GPU gather helper: scatters `band_count` compact band images
 * (device, `elem_bytes` per pixel; rank r's image starts at byte
 * r * rank_stride_bytes of `d_compact`, as an RCCL gather of padded
 * per-rank buffers lays them out) into the full image `d_dst` (device). */
int rt_assemble_bands(const void *d_compact, uint64_t rank_stride_bytes, void *d_dst, uint32_t width,
                      uint32_t height, uint32_t elem_bytes, uint32_t band_rows, uint32_t band_count,
                      void *stream);

int rt_device_synchronize(rt_device *dev);

/* ------------------------------------------- several GPUs, one host process */

/* Replaces the reference's thread-pool tiler (WorkQueueCreate/WorkQueueStart,
 * main.cpp:658-665, 851-856; wasm/wasm.cpp:651-678) with N GPUs driven from
 * one host thread: the frame is dealt in interleaved BandRows-row bands,
 * band b -> device b mod N, each device traces its bands on its
 * own stream, and the band images are gathered to devices[0] over xGMI --
 * RCCL grouped send/recv (ncclCommInitAll over the N devices) or, where RCCL
 * cannot be used (a device listed twice, no librccl), peer copies
 * (hipMemcpyPeerAsync) -- then scattered into the full frame.  Samples are
 * never split across devices (the running-mean fold is order dependent,
 * main.cpp:484-487), so the gathered frame is bit-identical to one device's. */
typedef struct rt_multi rt_multi;

#define RT_MULTI_AUTO 0u  /* RCCL when the devices are distinct and RCCL initialises, else peer copies */
#define RT_MULTI_RCCL 1u  /* RCCL only (rt_multi_create fails if it cannot be used) */
#define RT_MULTI_PEER 2u  /* peer copies only */
#define RT_MULTI_MAX_DEVICES 16u

int rt_multi_create(const int *hip_devices, uint32_t count, uint32_t transport, rt_multi **out);
/* rt_multi_create whose devices take `options` (rt_device_create_ex; NULL: the defaults). */
int rt_multi_create_ex(const int *hip_devices, uint32_t count, uint32_t transport, const rt_device_options *options,
                       rt_multi **out);
int rt_multi_destroy(rt_multi *m);
/* rt_set_rsqrt_table / rt_scene_upload on every device. */
int rt_multi_set_rsqrt_table(rt_multi *m, const float table[2048]);
int rt_multi_scene_upload(rt_multi *m, const rt_scene *scene);

/* rt_trace over the N devices.  The running mean stays resident on the
 * devices (each keeps its own bands'): desc->PreviousRayCount frames are
 * already folded there by earlier calls of the same geometry, or
 * RT_FLAG_ACCUM_ZERO (or PreviousRayCount 0) starts a new mean.
 *   cam->CurrentImage.Data : DEVICE pointer on devices[0], the full
 *                            Width x Height RGBA8 frame (written).
 *   cam->PreviousImage.Data: NULL, or a DEVICE pointer on devices[0] that
 *                            receives the full-frame v4 f32 running mean.
 *   desc->BandRows         : band height, a multiple of 8 (0 = 8);
 *                            desc->BandCount / BandIndex must be 0.
 *   d_rays                 : DEVICE u64 on devices[0], incremented by the
 *                            segments every device traced.
 * Everything the caller sees (frame, mean, d_rays) is written after prior
 * work on `stream` (a stream of devices[0]; NULL = the null stream), and work
 * enqueued on `stream` afterwards sees the gathered frame.  The traces read
 * nothing of the caller's and do not wait for that prior work: each device
 * alternates between two band-image slots, so call k's gather overlaps call
 * k+1's traces.  A continuation's PreviousRayCount must equal the count the
 * resident means were left at (RT_EINVAL otherwise): after a call with
 * PreviousRayCount P and Frames F that is P + F -- also for a restart with
 * RT_FLAG_ACCUM_ZERO and P > 0, whose frames were folded with the weights of
 * P, P + 1, ... (main.cpp:484-487), as rt_trace does.  A failed call drops
 * the resident means.  Every entry point that switches devices restores the
 * caller's current HIP device before it returns. */
int rt_multi_trace(rt_multi *m, const rt_camera_info *cam, const rt_trace_desc *desc, uint64_t *d_rays,
                   void *stream);
int rt_multi_synchronize(rt_multi *m);

typedef struct rt_multi_info {
    uint32_t DeviceCount;
    uint32_t Transport;      /* RT_MULTI_RCCL or RT_MULTI_PEER */
    uint32_t BandRows;       /* of the last trace */
    uint32_t MaxLocalRows;   /* rows of the largest device share */
    uint64_t SegmentsFolded; /* dead-tile segments counted, not traced (last trace, all devices;
                                may wait for each device's cull totals, as rt_trace_last_info) */
} rt_multi_info;
int rt_multi_get_info(rt_multi *m, rt_multi_info *out);

/* Each device's trace time (ms, HIP events around its rt_trace on its own
 * stream) of the last rt_multi_trace call, devices[i] -> ms_out[i]; count >=
 * the device count.  Waits for those traces to finish. */
int rt_multi_last_trace_ms(rt_multi *m, float *ms_out, uint32_t count);

/* The last call's gather time (ms, HIP events on devices[0]'s gather stream):
 * from the moment every device's trace has finished to the frame (and mean)
 * assembled -- the band transfer (RCCL or peer copies) plus the scatter. */
int rt_multi_last_gather_ms(rt_multi *m, float *ms_out);

/* rt_trace_last_info of devices[index] for the last call (RT_EINVAL when that
 * device traced nothing); may wait for its cull totals. */
int rt_multi_shard_info(rt_multi *m, uint32_t index, rt_trace_info *out);

/* Pre-sizes every device's band images and launch buffers (rt_device_reserve)
 * and devices[0]'s gather staging for frames up to width x height in
 * band_rows-row bands (0 = 8), so no rt_multi_trace of that geometry
 * allocates; RT_MULTI_RESERVE_MEAN also sizes the staging of the gathered
 * running mean (cam->PreviousImage).  Waits for the devices.  A reservation
 * that grows the devices' resident running means discards them: the next
 * call must restart the mean (PreviousRayCount 0 or RT_FLAG_ACCUM_ZERO), a
 * continuation is RT_EINVAL. */
#define RT_MULTI_RESERVE_MEAN 1u
int rt_multi_reserve(rt_multi *m, uint32_t width, uint32_t height, uint32_t band_rows, uint32_t flags);

/* Frames folded into the devices' resident running means, i.e. the
 * PreviousRayCount a continuation must name; 0 when no mean is resident
 * (none traced yet, a failed call, a geometry change, or a reservation that
 * grew the means). */
int rt_multi_resident_frames(rt_multi *m, uint64_t *out);

/* ----------------------------------- several GPUs, one process per GPU (RCCL) */

/* The band gather for one-process-per-GPU launches (torch.distributed.run /
 * mpirun): every rank traces its band residue with rt_trace (BandCount =
 * nranks, BandIndex = rank) and rt_comm_gather_bands brings the compact band
 * images to rank 0 over RCCL and scatters them into the full frame.  Rank 0
 * makes the id (rt_comm_unique_id) and the launcher shares its
 * RT_COMM_ID_BYTES bytes with every rank before rt_comm_create (which blocks
 * until all ranks have joined).  RT_ENODEV when librccl cannot be loaded or
 * RCCL refuses the communicator (e.g. two ranks on one GPU). */
typedef struct rt_comm rt_comm;
#define RT_COMM_ID_BYTES 128u
int rt_comm_unique_id(void *id_out);
int rt_comm_create(int hip_device, const void *id, uint32_t nranks, uint32_t rank, rt_comm **out);
int rt_comm_destroy(rt_comm *c);
/* d_local: this rank's compact band image (rt_band_local_rows(height,
 * band_rows, nranks, rank) x width x elem_bytes, device); d_full: rank 0's
 * full frame (width x height x elem_bytes, device; ignored elsewhere).
 * Enqueued on `stream` (NULL = the null stream) on every rank. */
int rt_comm_gather_bands(rt_comm *c, const void *d_local, void *d_full, uint32_t width, uint32_t height,
                         uint32_t elem_bytes, uint32_t band_rows, void *stream);

/* Scheduling counters accumulated over trace launches when the library is the
 * diagnostic build (`make -C simd-ray-tracer_amd variant NAME=stats
 * KFLAGS=-DRTK_STATS`, loaded via RT_TRACE_LIB) and the process runs with
 * RT_STATS=1: [0] primary wave-iterations, [1] primary lane-segments,
 * [2] secondary wave-iterations, [3] secondary lane-segments, [4] sphere
 * groups tested by primary iterations after culling, [5] secondary groups
 * (exact loop) where some lane passed the distance test, [6]/[7] secondary
 * iterations with < 16 lanes and their lanes, [8] secondary iterations with
 * no sample left to start, [9]-[15] wave-resident s_memtime cycles in
 * primary iterations, secondary iterations, the owner fold, block init,
 * mask load, barrier, and post-barrier setup, [16] prefiltered secondary
 * wave-iterations, [17]/[18] (wave, group) pairs the prefilter flagged, with
 * and without flags on the sphere a diffuse ray just left, [19]/[20] the same
 * per sphere pair, [21] lane-level flagged pairs (clustered loop: [17] member
 * pairs tested, [19] pairs rechecked, [21] clusters entered); [22]-[24] lanes of
 * primary rounds blocked by the sample ring, waiting for a secondary round,
 * and done; [25, 32) reserved.
 * Returns 1 when enabled, 0 when not (out zeroed), < 0 on error. */
int rt_debug_stats(rt_device *dev, uint64_t out[32], int reset);

/* With RT_WAVETIMES=1: {start, end} s_memrealtime (100 MHz) of every wave of
 * the last trace launch, wave id = block tile * 4 + w (dead tiles are not written).
 * Returns the number of waves copied (0 when disabled), < 0 on error. */
int64_t rt_debug_wave_times(rt_device *dev, uint64_t *out, uint64_t max_waves);

/* The cull pass's primary masks of the last culled launch geometry, one bit
 * per sphere pair (bit p: spheres 2p and 2p + 1, i.e. half p & 1 of group
 * p >> 1): word ((tile * 4 + wave) * n_words + w), n_words = ceil(2 groups / 64).
 * Returns the number of words copied (0 when no cull pass ran), < 0 on error.
 * Test hook: tests/test_gpu_parity.py checks them against a CPU restatement. */
int64_t rt_debug_masks(rt_device *dev, uint64_t *out, uint64_t max_words);

/* Host-side view of what rt_scene_upload derives for one rule set (no GPU
 * needed): per sphere slot s = 4*group + lane, the r^2 the exact test uses
 * and the secondary-ray prefilter threshold r2p (any ray whose
 * origin lies on a scene sphere and |D|^2 is within 2^-16 of 1 that passes
 * the exact test d < r^2 (d <= r^2 for the scalar rules) has prefilter
 * estimate e < r2p).  *out_flags: bit 0 = the scene-wide threshold pays
 * for this scene, bit 1 = candidate sqrt in the short sequence's range, bit 2
 * = per-lane thresholds instead (where bit 0 is clear): r2p then holds r^2
 * (-inf: never hit) and a lane skips a sphere when e >= RN(cc 2^-15 + r2p),
 * cc its computed |C|^2.
 * Arrays may be NULL to query the count. */
int rt_scene_prefilter(const rt_scene *scene, uint32_t enable_simd, float *out_r2, float *out_r2p, uint32_t capacity,
                       uint32_t *out_count, uint32_t *out_flags);
/* The clustered secondary-ray prefilter table rt_scene_upload builds for one
 * rule set (layout: rt_kernel.h, kClEntryF4 = 4 float4 rows per entry;
 * cluster-pair entries first).  *out_f4 = float4 rows, *out_cpairs = cluster
 * pairs (0: the scene uses the per-group prefilter loop).  out may be NULL to
 * query the size.  Test/inspection hook: the kernel's skip proof is checked
 * against it on the CPU (tests/test_prefilter_bound.py). */
int rt_scene_clusters(const rt_scene *scene, uint32_t enable_simd, float *out, uint32_t capacity_f4,
                      uint32_t *out_f4, uint32_t *out_cpairs);
/* The table's levels (test/inspection hook): *out_levels = 1 (cluster-pair
 * entries index member entries), 2 (tables of two or more pair-mask words: the
 * *out_cpairs top entries index *out_sub_pairs sub-cluster pair entries, which
 * index the member entries) or 0 (no table). */
int rt_scene_cluster_layout(const rt_scene *scene, uint32_t enable_simd, uint32_t *out_levels,
                            uint32_t *out_sub_pairs);
const char *rt_last_error(void);

/* ----------------------------------------------- OnInit / OnRender driver */

/* OnInit (main.cpp:645-679): window defaults, built-in scenes, device 0. */
int rt_on_init(rt_init_params *params);
/* OnInit on `count` devices: with more than one, rt_on_render drives them
 * through rt_multi (bands dealt over the devices, the running mean resident
 * on each, the frame gathered to hip_devices[0]). */
int rt_on_init_devices(rt_init_params *params, const int *hip_devices, uint32_t count);

/* Input state for the orbit camera (the reference polls IsDown(key) at
 * main.cpp:732-761).  Bits: */
#define RT_KEY_FORWARD 0x01u  /* W / ArrowUp    */
#define RT_KEY_BACK 0x02u     /* S / ArrowDown  */
#define RT_KEY_RIGHT 0x04u    /* D / ArrowRight */
#define RT_KEY_LEFT 0x08u     /* A / ArrowLeft  */
#define RT_KEY_UP 0x10u       /* Space          */
#define RT_KEY_DOWN 0x20u     /* C / LeftControl*/
#define RT_KEY_RESET 0x40u    /* R              */

/* OnRender (main.cpp:705-859) with the accumulation resident in HBM: one
 * progressive frame per call, one-frame output lag, reset on
 * move/resize/scene change/R.  `image` is a HOST RGBA8 image.  Returns 1
 * when `image` received a completed frame, 0 when not (previous frame
 * still running), negative on error. */
int rt_on_render(const rt_image *image, rt_render_params params, uint32_t keys,
                 uint64_t *out_total_rays_cast, double *out_time_elapsed_ms);

/* Blocks until the in-flight frame (if any) has completed
 * (WorkQueueWaitUntilCompletion, base.h:175). */
int rt_on_render_wait(void);
int rt_on_shutdown(void);

/* Opt-in fast hand-out.  By default rt_on_render copies a completed frame
 * into `image` through a pinned staging buffer the library owns (one DMA,
 * then one host copy; the reference's CopyImage, main.cpp:688-697).  A caller
 * that renders into the same host buffer every frame (the platform's image,
 * wasm/wasm.cpp:179) may register it: the library page-locks the `bytes` at
 * `data`, and frames for an image whose Data is `data` then arrive by one DMA
 * straight into it.  The caller must keep the buffer allocated until
 * rt_on_render_unregister_image or rt_on_shutdown, which unlock it.  A second
 * registration replaces the first.  Returns RT_OK, RT_EINVAL (not initialised,
 * NULL, 0 bytes) or RT_EIO (the driver refused to page-lock it). */
int rt_on_render_register_image(void *data, uint64_t bytes);
int rt_on_render_unregister_image(void);

/* Where rt_on_render's time goes (cumulative since init or the last reset).
 * A frame is handed out by rt_on_render after the next frame is launched, so
 * the copy runs beside that frame's trace. */
typedef struct rt_on_render_profile {
    uint64_t Calls;          /* rt_on_render calls                                   */
    uint64_t FramesLaunched; /* frames started (trace + its copies to the host)      */
    uint64_t FramesCopied;   /* completed frames handed to the caller's image        */
    double CallMs;           /* host time inside rt_on_render                         */
    double HostCopyMs;       /* of which: frame -> caller image (CopyImage: DMA [+ host copy]) */
    double HostWaitMs;       /* of which: waiting for an in-flight frame (reset/move) */
    double GpuFrameMs;       /* sum of completed frames' launch -> done GPU time      */
    uint64_t FrameAllocations; /* frame-buffer (re)allocations by rt_on_init /
                                  rt_on_render_reserve / a resize beyond them      */
} rt_on_render_profile;
int rt_on_render_get_profile(rt_on_render_profile *out, int reset);

/* Sizes the frame driver's device frames (running mean + two RGBA8 frames)
 * and the trace's launch buffers for images up to width x height, so a later
 * resize within that size frees and allocates nothing: it re-uses them, as
 * the reference re-Pushes its images into the arena OnInit sized (main.cpp:
 * 658, 798-804).  rt_on_init reserves its 1280x720 window (main.cpp:649-650).
 * Keeps the current frames on one device; on several devices (rt_on_init_devices)
 * the call restarts the running mean at the next rt_on_render, as a resize does,
 * since growing the devices' resident means drops them.  New. */
int rt_on_render_reserve(uint32_t width, uint32_t height);

/* ----------------------------------------------------------- output path */

/* The RGBA8 frame (RT_FORMAT_R8G8B8A8_U32, host memory) written as a binary
 * PPM (P6, RGB) or an 8-bit RGBA PNG (stored deflate blocks), in place of
 * the reference's WebGL texture upload of Image.Data (wasm/wasm.cpp:216-218).
 * RT_IMAGE_FLIP_Y writes image row Height-1 first: the texture's row 0 is the
 * bottom of the window, so that is the on-screen orientation.
 * Returns RT_OK, RT_EINVAL (bad image / format / path) or RT_EIO. */
#define RT_IMAGE_FLIP_Y 1u
int rt_image_write_ppm(const rt_image *image, const char *path, uint32_t flags);
int rt_image_write_png(const rt_image *image, const char *path, uint32_t flags);

/* FNV-1a 64 of `nbytes` host bytes (offset basis 0xcbf29ce484222325, prime
 * 0x100000001b3): the frame checksum the committed fixtures hold
 * (tests/golden, *.json), so a caller can check a rendered frame -- RGBA8 or
 * the v4 running mean copied to the host -- against a golden without the
 * checker.  New; the reference has no frame checksum. */
uint64_t rt_frame_hash(const void *data, uint64_t nbytes);

#ifdef __cplusplus
}
#endif
#endif /* RT_TRACE_H */
