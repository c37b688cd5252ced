// rt_kernel.h — launch contract between the C-ABI host (rt_host.cpp) and the
// gfx950 trace kernel (rt_kernel.hip).  Internal; not part of include/.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

enum { kSrcSmem = 0, kSrcLds = 1 };  // where the sphere loop reads its groups
constexpr uint32_t kGroupF4 = 5;      // float4 rows per sphere group:
constexpr uint32_t kRowX = 0, kRowY = 1, kRowZ = 2;  //   centres
constexpr uint32_t kRowR2P = 3;       //   prefilter thresholds (rows 0-3 = one s_load_dwordx16)
constexpr uint32_t kRowR2 = 4;        //   r*r
constexpr uint32_t kSphereF4 = 4;     // float4 rows per sphere record (TraceArgs.materials)
enum { kFlagAccumZero = 1, kFlagSrgbPow = 2 };
// Clustered secondary-ray prefilter (rt_host.cpp cluster_table): entries of
// cl_entry_f4(W) float4 rows, read through the scalar cache --
//   cluster pair c : {qx0 qx1 qy0 qy1} {qz0 qz1 rc2p0 rc2p1} {first0 count0 first1 count1} {b0 b1 0 0} [padding]
//   member pair m  : {x0 x1 y0 y1}     {z0 z1 r2p0 r2p1}     {word-0 bits of member 0 (lo, hi), of member 1}
//                    {b0 b1 0 0}  then one row per further word w = 1 .. W-1: {word-w bits of member 0, of member 1}
// (b = behind threshold: a lane whose prefilter T = (centre - O).D is below
// it cannot accept any member -- rt_host.cpp cluster_table)
// (first/count index member-pair entries; a member's pair q = sphere slot >> 1
// is its sphere pair in group order, the bit it sets in the wave's pair mask).
// The wave mask is kept in SGPRs, W = cl_words u64 words of it (1: n_groups <= 32,
// 2: <= 64, 4: <= 128): member k's pair q sets bit q & 63 of word q >> 6, and its
// entry holds that bit in the row of word q >> 6 and 0 in the others, so the kernel
// merges a flagged member into every word with one select and one OR each.
// With pf_relative the thresholds are per lane: rc2p / r2p hold R_c / r^2 and
// b the M-free behind bases (rt_host.cpp cluster_table, "relative"), and a
// cluster pair also carries its height-slab bound (rt_kernel.hip slab test):
//   row 3 = {b0 b1 srho0 srho1}, row 4 = {ymid0 ymid1 yhalf0 yhalf1}
// (entries then have at least 5 rows; member entries leave row 4 to the bits).
// padding members: threshold -inf, bits 0.
constexpr uint32_t cl_entry_f4(uint32_t words, bool relative = false) {
    return words == 1u ? (relative ? 5u : 4u) : 3u + words;
}
constexpr float kSlabRel = 0x1p-9f;  // the slab test's per-lane margin per unit of cc (rt_host.cpp cluster_table)
constexpr uint32_t kClMaxGroups = 128;   // table built up to this many groups
constexpr uint32_t kClAutoGroups = 128;  // used by default up to this many (rt_host.cpp clusters_env; RTWeekend's
                                         // 121 groups: 11.3k Mrays/s clustered against 9.4k per group)

// HBM layout of an uploaded scene (per rule set):
//   groups    : n_groups x 5 float4 = {x[4]}, {y[4]}, {z[4]}, {r2p[4]}, {r*r[4]}  (80 B/group)
//               r2p = prefilter threshold of the secondary-ray sphere loop (rt_host.cpp);
//               with pf_relative, r*r again (-inf: never hit) and the threshold is formed per lane
//   spheres   : 4*n_groups records of kSphereF4 float4 = {centre.xyz, 0}, {Color.xyz, Specular},
//               {Emissive.xyz, IOR}, {1/IOR, r0 outside, r0 inside, 0} (dielectrics; else 0)
//               (64 B/sphere: what shading gathers for the winning sphere,
//               addressed by one shift of its index; TraceArgs.materials)
// r*r is precomputed on the host with the same f32 multiply the reference
// repeats per test (main.cpp:406), so it is bit-identical.
struct TraceArgs {
    const float4 *groups;
    const float4 *materials;
    const float *rsqrt_lut;      // 2048 f32
    float4 *prev;                // compact band image, local_rows x width
    uint32_t *cur;               // compact band image, local_rows x width
    unsigned long long *rays;    // accumulated bounce segments
    float cam_pos[3], cam_x[3], cam_y[3], film_center[3];
    float film_w, film_h;
    float inv_width, inv_height;  // RN(1/(f32)width), RN(1/(f32)height)
    uint32_t width, height, local_rows;
    uint32_t prev_count, frames, max_bounce;
    uint32_t n_groups, n_spheres, use_sky, flags;  // n_spheres: scalar rule set only
    uint32_t band_rows, band_count, band_index;
    uint32_t sec_threshold;      // lanes that must wait for a secondary iteration
    uint32_t prefilter;          // secondary sphere loop: FMA prefilter + exact recheck (r2p valid)
    uint32_t fast_sqrt;          // every hittable r^2 is 0 or in [2^-36, 2^60] (candidate sqrt_rn)
    unsigned long long *stats;   // optional (RT_STATS): kStat* counters, NULL = off
    unsigned long long *wave_times;  // optional (RT_WAVETIMES): per-wave {start, end} s_memrealtime
    const uint32_t *tile_order;  // optional: block -> tile map (heaviest first), NULL = identity
    uint32_t *tile_cost;         // optional: per-tile cost (max wave shader cycles), atomicMax'd
    const uint64_t *masks;       // CULL: per wave tile (4*tile + wave) n_words primary group masks
    uint32_t tiles_x;            // block tiles per row (2TW x 2TH pixels each)
    const float4 *clusters;      // optional: clustered prefilter table (cl_entry_f4(cl_words) rows per entry)
    uint32_t n_cpairs;           // cluster-pair entries at its start; 0 = per-group prefilter loop
    uint32_t cl_words;           // u64 words of the clustered loop's pair mask (1 or 2)
    uint32_t interleave;         // wave tiles interleave over the block tile (P >= 2 only)
    uint32_t lut_in_lds;         // rsqrt table in the LDS image (else read from HBM: rtk_lut_in_lds)
    uint32_t fold_in_lds;        // running-mean weight table in the LDS image (else computed: rtk_fold_in_lds)
    uint32_t scene_in_lds;       // groups + materials copied into the LDS image (else read from HBM: GS kernels)
    uint32_t pf_relative;        // prefilter: row 3 holds r^2 and the threshold is per lane (rt_kernel.hip kPfRel)
    uint32_t solo;               // one wave per workgroup (4 x tiles workgroups of 64 threads; needs no LDS image)
    uint32_t walk;               // kWalk*: the one-wave kernel specialised for this launch's secondary walk
    // optional: live block tiles of the cull pass, on the device (kCullTotals).  Set while the host
    // has not read the count back: the grid then covers every tile and blocks past the count exit.
    const unsigned long long *live_total;
    // one-wave kernels (solo): tile_order / tile_cost index WAVES (4 * block tile + quadrant),
    // so the heaviest-first order ranks every wave on its own cost (rt_host.cpp unit_waves)
    uint32_t unit_waves;
    // optional (rt_device_options PixelSort): the block tile's pixels dealt to its four waves by cost,
    // cheapest first: pix_perm[64 * tile + NPIX * wave + pl] = the pixel's index in the
    // block tile (row-major, 2TW wide); pix_perm[64 * tile] == 0xFF: not permuted
    const uint8_t *pix_perm;
    // optional: segments each pixel traced in this launch (band-local rows x width), the
    // cost the next launch's permutation sorts by (rtk_launch_pixel_sort)
    uint32_t *pix_cost;
    // 1: every round starts new samples and continues paths together through the exact
    // sphere loop (scenes of at most kMergeGroups groups: the cull mask and the prefilter
    // save nothing there, and split rounds leave most lanes idle at one frame per launch)
    uint32_t merge_rounds;
    // pixels per dealt unit of the pixel sort (1, 2 or 4; capped at the wave's pixel count): the
    // sort ranks row segments of pix_seg pixels by their summed cost, so each wave's owner
    // lanes store whole 4-pixel runs (a 64-B half line of the v4 image) instead of single
    // pixels of lines other waves -- on other XCDs -- also write
    uint32_t pix_seg;
    // 1: the trace and empty-tile kernels store only the running mean; the RGBA8 image is
    // encoded from it by one coalesced pass after the launch (rtk_launch_encode), so its 4-B
    // pixels are not written as scattered partial lines from several XCDs (rt_device_options EncodePass)
    uint32_t skip_cur;
    // CULL (required): the primary rounds' group rows, written by the cull pass for its camera
    // (rtk_launch_cull): per group kPrimF4 float4 = {cx[4]}, {cy[4]}, {cz[4]}, {r*r[4]} with
    // c = RN(centre - CameraPosition), the first three f32 ops of every primary sphere test
    // (main.cpp:401), identical on every lane of a primary round (one s_load_dwordx16)
    float4 *prim;
    // the running-mean weights {RN(1/(n+1)), RN(n/(n+1))} of frames n < kWeightsN (main.cpp:484-487),
    // one table per device computed once (rt_device_create): a finished sample's two weights are one
    // gather instead of two conversions, a reciprocal and a division (one-wave kernels)
    const float2 *weights;
};
constexpr uint32_t kWeightsN = 65536;
constexpr uint32_t kPrimF4 = 4;
constexpr uint32_t kMergeGroups = 2;
// Cull pass counters (rtk_launch_cull): [0, 64) striped live block tiles, [64, 128)
// striped image pixels of dead block tiles, then the two totals at kCullTotals
// (live tiles, dead pixels), summed on the device after the pass.
constexpr uint32_t kCullCounterWords = 132;
constexpr uint32_t kCullTotals = 128;
// Secondary-ray walk variants (rt_kernel.hip Walk<>): any (run-time dispatch),
// the per-group loops, or a cluster walk with 1/2/4 pair-mask words and
// scene-wide or per-lane ("Rel") thresholds
enum { kWalkAny = 0, kWalkGroups, kWalkCl1, kWalkCl2, kWalkCl4, kWalkCl1Rel, kWalkCl2Rel, kWalkCl4Rel };
enum { kStatPriIters = 0, kStatPriLanes, kStatSecIters, kStatSecLanes, kStatPriGroups, kStatSecHitGroups,
       kStatSecSparseIters, kStatSecSparseLanes, kStatSecTailIters, kStatPriCycles, kStatSecCycles, kStatFoldCycles,
       kStatSetupCycles, kStatCullCycles, kStatSyncCycles, kStatPostCycles, kStatPfRounds, kStatPfGroups,
       kStatClTested, kStatPfPairs, kStatClTopEntered, kStatPfLanePairs, kStatPriBlocked, kStatPriWaitSec,
       kStatPriDone, kStatSecDone, kStatSecWaitPri, kStatDoneTrips, kStatDoneLaneTrips,
       kStatSecExact, kStatSecBadLanes, kStatSecZeroDir, kStatCount = 32 };
constexpr uint32_t kStatSlots = 32;  // rt_debug_stats copies this many

// Dynamic LDS per block: [rsqrt table] + fold table + groups + materials.
// The 8 KB table stays in LDS up to 32 groups; a larger scene's image would
// cost occupancy (C5's 64 groups: 5 -> 7 blocks per CU without it and the
// weight table), so the table is then read from HBM through the caches.
// The 2 KB weight table of the first 256 frames goes the same way (the
// weights are then two divisions per sample): C5 fits 7 blocks per CU.
// The cull pass's primary masks hold one bit per sphere PAIR (spheres 2p, 2p + 1: half p & 1 of group
// p >> 1), so a primary round tests only the pairs its tile's cone may reach -- half of the group-level
// masks' pair tests at C2 (1.17 of 2.33 pairs per live 4x4 tile); words per wave tile:
static inline __host__ __device__ uint32_t rtk_mask_words(uint32_t n_groups) { return (2u * n_groups + 63u) / 64u; }
static inline bool rtk_lut_in_lds(uint32_t n_groups) { return n_groups <= 32u; }
static inline bool rtk_fold_in_lds(uint32_t n_groups) { return n_groups <= 32u; }
static inline size_t rtk_scene_lds_bytes(uint32_t n_groups) {
    return (size_t)n_groups * (16u * kGroupF4 + 64u * kSphereF4);
}
static inline size_t rtk_lds_bytes(const TraceArgs *a) {
    return (a->lut_in_lds ? 8192u : 0u) + (a->fold_in_lds ? 2048u : 0u) +
           (a->scene_in_lds ? rtk_scene_lds_bytes(a->n_groups) : 0u);
}
// The largest scene the LDS image holds (64 KB of dynamic LDS per block with
// the two tables): 265 groups = 1,060 spheres.  Larger scenes stay in HBM
// (scene_in_lds = 0): the sphere loop reads groups through the scalar cache as
// always, and the per-lane gathers go through L1/L2.  Up to kMaxGroups groups
// (the primary cull masks are rtk_mask_words(kMaxGroups) = 128 words per wave tile).
static const uint32_t kMaxLdsGroups = (65536u - 8192u - 2048u) / (16u * kGroupF4 + 64u * kSphereF4);  // 164 groups
static const uint32_t kMaxGroups = 4096u;                                                    // 16,384 spheres

extern "C" int rtk_launch_trace(const TraceArgs *a, int simd, int src, int cull, int lanes_per_pixel,
                                hipStream_t stream);
// Heaviest-first tile order for the next launch from this launch's costs
// (resets the costs); n = rtk_tile_count(...) of the launch geometry.
// scratch: rtk_tile_sort_scratch(n) bytes of device memory
extern "C" size_t rtk_tile_sort_scratch(uint32_t n);
extern "C" int rtk_launch_tile_sort(uint32_t *cost, uint32_t *order, uint32_t *scratch, uint32_t n, hipStream_t stream);
// One-wave kernels' wave order: the live prefix (4 x live_tiles[0] units) of a sorted
// order_in partitioned stably by XCD group (every eighth live tile by its heaviest
// wave's rank) and interleaved so that every wave of a block tile runs on one XCD
// (rt_kernel.hip, "XCD grouping"); the rest copied.  scratch: rtk_tile_sort_scratch(
// n_units) bytes (8 n_blk + 9 words used); aux: 2 x n_units / 4 words.
extern "C" int rtk_launch_xcd_group(const uint32_t *order_in, uint32_t *order_out, uint32_t n_units,
                                    const unsigned long long *live_tiles, uint32_t *scratch, uint32_t *aux,
                                    hipStream_t stream);
extern "C" uint32_t rtk_tile_count(uint32_t width, uint32_t local_rows, int lanes_per_pixel);
extern "C" uint32_t rtk_tiles_x(uint32_t width, int lanes_per_pixel);
// grid: blocks of the trace launch (tile_order[0..grid) when tile_order is set)
extern "C" int rtk_launch_trace_grid(const TraceArgs *a, int simd, int src, int cull, int lanes_per_pixel,
                                     uint32_t grid, hipStream_t stream);
// Primary-ray cone culling of every wave tile -> a->masks, and the camera-relative
// group rows of the primary rounds -> a->prim (both must be set);
// per block tile live[t] (some wave tile has a candidate group, or
// !empty_capable) and cost[t] = live ? 2 : 0 (so a tile sort puts live tiles
// first); counters[0, 64) sum to the live tiles, counters[64, 128) to the
// image pixels of dead tiles (zeroed by the call), and counters[kCullTotals],
// counters[kCullTotals + 1] receive the two sums (kCullCounterWords words).
extern "C" int rtk_launch_cull(const TraceArgs *a, int lanes_per_pixel, uint32_t *live, uint32_t *cost,
                               unsigned long long *counters, int empty_capable, hipStream_t stream);
// Pixels of dead block tiles (live[t] == 0): every sample misses with no sky,
// so fold zeros into the running mean, store both images; adds
// dead_pixels[0] x a->frames segments to the ray counter once (dead_pixels:
// the cull pass's device total, so the host need not read it back).
extern "C" int rtk_launch_empty(const TraceArgs *a, int lanes_per_pixel, const uint32_t *live,
                                const unsigned long long *dead_pixels, hipStream_t stream);
// Per block tile, deal its pixels to its four waves by the costs the last launch
// measured (TraceArgs.pix_cost), cheapest to wave 0, so each wave's pixels finish
// their samples at about the same time; blocks with a quadrant the cull pass
// left empty keep their pixels (that quadrant's wave folds without tracing).
// perm: 64 bytes per block tile (TraceArgs.pix_perm).  P in {4, 8, 16, 32}.
extern "C" int rtk_launch_pixel_sort(const TraceArgs *a, int lanes_per_pixel, uint8_t *perm, hipStream_t stream);
// dst[0] += sum of slots[0, n) (the gathered per-device ray counters)
extern "C" int rtk_launch_sum_u64(const uint64_t *slots, uint32_t n, uint64_t *dst, hipStream_t stream);
// Restores the caller's current HIP device when a C-ABI entry point returns:
// entry points switch to their device's ordinal (hipSetDevice), and the
// caller's own HIP work must keep targeting the device it had selected.
struct DeviceGuard {
    int saved = -1;
    DeviceGuard() {
        if (hipGetDevice(&saved) != hipSuccess) {
            saved = -1;
            (void)hipGetLastError();
        }
    }
    ~DeviceGuard() {
        if (saved >= 0) (void)hipSetDevice(saved);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};
// sets rt_last_error()'s text and returns `code` (rt_host.cpp)
int rt_fail(int code, const char *fmt, ...);
extern "C" int rtk_launch_encode(const void *accum, void *out, uint64_t n, uint32_t pow_mode, hipStream_t stream);
extern "C" int rtk_launch_assemble(const void *src, uint64_t rank_stride, void *dst, uint32_t width, uint32_t height,
                                   uint32_t elem, uint32_t band_rows, uint32_t band_count, hipStream_t stream);
