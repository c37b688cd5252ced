"""simd_ray_tracer_amd — Python mirror of the reference trace path's interface.

Thin ctypes layer over the in-tree C-ABI library ``librt_trace.so`` (HIP
kernels for gfx950 + C++ host, see ``include/rt_trace.h``).  It mirrors the
reference's names and argument meaning:

* ``scene_builtin`` / ``scene_prefix``  — Scenes[] of main.cpp:93-268
* ``camera_setup``                      — the camera block of OnRender, main.cpp:776-838
* ``Device.trace``                      — WorkQueueStart(RenderTile|RenderTileScalar, ...), main.cpp:851-856
* ``on_init`` / ``on_render``           — OnInit / OnRender, base.h:163-164

The library is REQUIRED: every entry point raises if it is missing or if no
HIP device is present.  There is no CPU fallback on this path (the CPU
restatement under ``oracle/`` is test infrastructure, never imported here).
"""
from __future__ import annotations

import ctypes
import os
import pathlib
from ctypes import POINTER, c_bool, c_char_p, c_double, c_float, c_int, c_uint32, c_uint64, c_void_p
from typing import Optional

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
# RT_TRACE_LIB selects an alternative in-tree build (kernel A/B experiments)
LIB_PATH = _HERE / os.environ.get("RT_TRACE_LIB", "librt_trace.so")

RT_SEED_PIXEL = 1
RT_MAX_SPHERES = 16384
RT_FLAG_ACCUM_ZERO = 1
RT_FLAG_SRGB_POW = 2
RT_FORMAT_R32B32G32A32_F32 = 1
RT_FORMAT_R8G8B8A8_U32 = 2
KEY_FORWARD, KEY_BACK, KEY_RIGHT, KEY_LEFT, KEY_UP, KEY_DOWN, KEY_RESET = (1, 2, 4, 8, 16, 32, 64)


# ----------------------------------------------------------- C structs
class RtV3(ctypes.Structure):
    _fields_ = [("x", c_float), ("y", c_float), ("z", c_float), ("_w", c_float)]


class RtMaterial(ctypes.Structure):  # main.cpp:11-16, 48 B (16-byte aligned in C)
    _fields_ = [("Color", RtV3), ("Emissive", RtV3), ("Specular", c_float), ("IndexOfRefraction", c_float),
                ("_pad", c_float * 2)]


class RtScalarSphere(ctypes.Structure):  # main.cpp:17-21, 80 B
    _fields_ = [("Position", RtV3), ("Radius", c_float), ("_pad", c_float * 3), ("Material", RtMaterial)]


class RtSphereGroup(ctypes.Structure):  # main.cpp:23-26, 64 B
    _fields_ = [("X", c_float * 4), ("Y", c_float * 4), ("Z", c_float * 4), ("Radii", c_float * 4)]


class RtArray(ctypes.Structure):  # main.cpp:28-40
    _fields_ = [("Data", c_void_p), ("Count", c_uint32)]


class RtScene(ctypes.Structure):  # main.cpp:42-51, 80 B
    _fields_ = [("LookAt", RtV3), ("UseSkyColor", c_bool), ("DefaultDistanceFromLookAt", c_float),
                ("DefaultXAngle", c_float), ("DefaultYHeight", c_float), ("ScalarSpheres", RtArray),
                ("SIMDSpheres", RtArray), ("Materials", RtArray)]


class RtImage(ctypes.Structure):  # base.h:132-136
    _fields_ = [("Data", c_void_p), ("Width", c_uint32), ("Height", c_uint32), ("Format", c_uint32)]


class RtCameraInfo(ctypes.Structure):  # main.cpp:270-282, 144 B
    _fields_ = [("CameraPosition", RtV3), ("CameraZ", RtV3), ("CameraX", RtV3), ("CameraY", RtV3),
                ("FilmCenter", RtV3), ("FilmW", c_float), ("FilmH", c_float), ("TilesX", c_uint32),
                ("CurrentImage", RtImage), ("PreviousImage", RtImage)]


class RtRenderParams(ctypes.Structure):  # base.h:157-161
    _fields_ = [("ThreadCount", c_uint32), ("EnableSIMD", c_bool), ("SceneIndex", c_uint32)]


class RtInitParams(ctypes.Structure):  # base.h:152-155
    _fields_ = [("WindowWidth", c_uint32), ("WindowHeight", c_uint32), ("WindowTitle", c_char_p),
                ("WindowTitleSize", c_uint32)]


class RtTraceDesc(ctypes.Structure):
    _fields_ = [(n, c_uint32) for n in ("Width", "Height", "PreviousRayCount", "Frames", "MaxBounce", "EnableSIMD",
                                        "SeedMode", "BandRows", "BandCount", "BandIndex", "Flags")]


class RtTraceInfo(ctypes.Structure):  # rt_trace_last_info
    _fields_ = [("SegmentsFolded", c_uint64)] + [(n, c_uint32) for n in (
        "LanesPerPixel", "TilesTotal", "TilesTraced", "CullPassRan", "OrderedLaunches", "ClusteredWalk",
        "GroupsPerRuleSet", "SplitHeadFrames", "OneWaveGroups", "Walk", "PixelsPerLane", "PixelsSorted", "BufferGrowths")]


OPTION_FIELDS = ("Cull", "Prefilter", "PrefilterRelative", "Clusters", "ClusterCount", "SubClusterSpheres",
                 "SecondaryThreshold", "LanesPerPixel", "PixelsPerLane", "OneWaveGroups", "SphereSourceLds",
                 "SceneInHbm", "TablesInLds", "WalkAny", "Interleave", "MergeRounds", "TileOrder", "WaveOrder",
                 "PixelSort", "PixelSegment", "XcdGroup", "SplitFirstLaunch", "HeadSamples", "SplitParts",
                 "SplitGrowth", "OrderLaunches", "EncodePass")
RT_OPT_DEFAULT, RT_OPT_ON, RT_OPT_OFF = 0, 1, -1


class RtDeviceOptions(ctypes.Structure):  # rt_device_options: kernel / schedule choices, 0 = default
    _fields_ = [("Size", c_uint32)] + [(n, ctypes.c_int32) for n in OPTION_FIELDS]


def device_options(options: Optional[dict]) -> Optional[RtDeviceOptions]:
    """rt_device_options from {"Cull": RT_OPT_OFF, "LanesPerPixel": 16, ...} (None: the defaults).
    Switches also take True / False for RT_OPT_ON / RT_OPT_OFF."""
    if not options:
        return None
    o = RtDeviceOptions()
    o.Size = ctypes.sizeof(RtDeviceOptions)
    for k, v in options.items():
        if k not in OPTION_FIELDS:
            raise KeyError(f"unknown device option {k!r} (rt_device_options: {', '.join(OPTION_FIELDS)})")
        setattr(o, k, (RT_OPT_ON if v else RT_OPT_OFF) if isinstance(v, bool) else int(v))
    return o


def parse_options(items) -> dict:
    """["Cull=off", "LanesPerPixel=16", ...] (bench.py --opt) -> an options dict."""
    out = {}
    for it in items or ():
        k, _, v = it.partition("=")
        v = v.strip().lower()
        out[k.strip()] = {"on": RT_OPT_ON, "off": RT_OPT_OFF, "default": RT_OPT_DEFAULT}.get(v, None)
        if out[k.strip()] is None:
            out[k.strip()] = int(v)
    return out


class RtMultiInfo(ctypes.Structure):  # rt_multi_get_info
    _fields_ = [(n, c_uint32) for n in ("DeviceCount", "Transport", "BandRows", "MaxLocalRows")] + [
        ("SegmentsFolded", c_uint64)]


class RtOnRenderProfile(ctypes.Structure):  # rt_on_render_get_profile
    _fields_ = [(n, c_uint64) for n in ("Calls", "FramesLaunched", "FramesCopied")] + [
        (n, c_double) for n in ("CallMs", "HostCopyMs", "HostWaitMs", "GpuFrameMs")] + [
        ("FrameAllocations", c_uint64)]


RT_MULTI_AUTO, RT_MULTI_RCCL, RT_MULTI_PEER = 0, 1, 2
RT_MULTI_RESERVE_MEAN = 1
RT_COMM_ID_BYTES = 128

for _t, _n in ((RtV3, 16), (RtMaterial, 48), (RtScalarSphere, 80), (RtSphereGroup, 64), (RtArray, 16),
               (RtScene, 80), (RtImage, 24), (RtCameraInfo, 144), (RtRenderParams, 12)):
    assert ctypes.sizeof(_t) == _n, (_t.__name__, ctypes.sizeof(_t), _n)

# Every symbol include/rt_trace.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "rt_scene_builtin": (c_int, [c_uint32, POINTER(RtScene)]),
    "rt_scene_prefix": (c_int, [POINTER(RtScene), c_uint32, POINTER(RtScene)]),
    "rt_camera_setup": (c_int, [POINTER(RtScene), c_float, c_float, c_float, c_uint32, c_uint32,
                                POINTER(RtCameraInfo)]),
    "rt_pixel_seed": (c_uint64, [c_uint32, c_uint32, c_uint32, c_uint32, c_uint32]),
    "rt_device_create": (c_int, [c_int, POINTER(c_void_p)]),
    "rt_device_create_ex": (c_int, [c_int, POINTER(RtDeviceOptions), POINTER(c_void_p)]),
    "rt_device_get_options": (c_int, [c_void_p, POINTER(RtDeviceOptions)]),
    "rt_device_destroy": (c_int, [c_void_p]),
    "rt_set_rsqrt_table": (c_int, [c_void_p, c_void_p]),
    "rt_rsqrt_table_builtin": (c_int, [c_void_p]),
    "rt_rsqrt_table_capture_host": (c_int, [c_void_p]),
    "rt_scene_upload": (c_int, [c_void_p, POINTER(RtScene)]),
    "rt_band_local_rows": (c_uint32, [c_uint32, c_uint32, c_uint32, c_uint32]),
    "rt_trace": (c_int, [c_void_p, POINTER(RtCameraInfo), POINTER(RtTraceDesc), c_void_p, c_void_p]),
    "rt_assemble_bands": (c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32, c_uint32,
                                  c_void_p]),
    "rt_trace_last_info": (c_int, [c_void_p, POINTER(RtTraceInfo)]),
    "rt_encode_rgba8": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p]),
    "rt_device_synchronize": (c_int, [c_void_p]),
    "rt_multi_create": (c_int, [POINTER(c_int), c_uint32, c_uint32, POINTER(c_void_p)]),
    "rt_multi_create_ex": (c_int, [POINTER(c_int), c_uint32, c_uint32, POINTER(RtDeviceOptions), POINTER(c_void_p)]),
    "rt_multi_resident_frames": (c_int, [c_void_p, POINTER(c_uint64)]),
    "rt_multi_destroy": (c_int, [c_void_p]),
    "rt_multi_set_rsqrt_table": (c_int, [c_void_p, c_void_p]),
    "rt_multi_scene_upload": (c_int, [c_void_p, POINTER(RtScene)]),
    "rt_multi_trace": (c_int, [c_void_p, POINTER(RtCameraInfo), POINTER(RtTraceDesc), c_void_p, c_void_p]),
    "rt_multi_synchronize": (c_int, [c_void_p]),
    "rt_multi_get_info": (c_int, [c_void_p, POINTER(RtMultiInfo)]),
    "rt_multi_last_trace_ms": (c_int, [c_void_p, c_void_p, c_uint32]),
    "rt_multi_last_gather_ms": (c_int, [c_void_p, POINTER(c_float)]),
    "rt_multi_shard_info": (c_int, [c_void_p, c_uint32, POINTER(RtTraceInfo)]),
    "rt_multi_reserve": (c_int, [c_void_p, c_uint32, c_uint32, c_uint32, c_uint32]),
    "rt_device_reserve": (c_int, [c_void_p, c_uint32, c_uint32]),
    "rt_comm_unique_id": (c_int, [c_void_p]),
    "rt_comm_create": (c_int, [c_int, c_void_p, c_uint32, c_uint32, POINTER(c_void_p)]),
    "rt_comm_destroy": (c_int, [c_void_p]),
    "rt_comm_gather_bands": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32,
                                     c_void_p]),
    "rt_debug_stats": (c_int, [c_void_p, c_void_p, c_int]),
    "rt_debug_wave_times": (ctypes.c_int64, [c_void_p, c_void_p, c_uint64]),
    "rt_debug_masks": (ctypes.c_int64, [c_void_p, c_void_p, c_uint64]),
    "rt_scene_prefilter": (c_int, [POINTER(RtScene), c_uint32, c_void_p, c_void_p, c_uint32, POINTER(c_uint32),
                                   POINTER(c_uint32)]),
    "rt_scene_clusters": (c_int, [POINTER(RtScene), c_uint32, c_void_p, c_uint32, POINTER(c_uint32),
                                  POINTER(c_uint32)]),
    "rt_scene_cluster_layout": (c_int, [POINTER(RtScene), c_uint32, POINTER(c_uint32), POINTER(c_uint32)]),
    "rt_last_error": (c_char_p, []),
    "rt_on_init": (c_int, [POINTER(RtInitParams)]),
    "rt_on_init_devices": (c_int, [POINTER(RtInitParams), POINTER(c_int), c_uint32]),
    "rt_on_render": (c_int, [POINTER(RtImage), RtRenderParams, c_uint32, POINTER(c_uint64), POINTER(c_double)]),
    "rt_on_render_wait": (c_int, []),
    "rt_on_render_register_image": (c_int, [c_void_p, c_uint64]),
    "rt_on_render_unregister_image": (c_int, []),
    "rt_on_shutdown": (c_int, []),
    "rt_on_render_get_profile": (c_int, [POINTER(RtOnRenderProfile), c_int]),
    "rt_on_render_reserve": (c_int, [c_uint32, c_uint32]),
    "rt_image_write_ppm": (c_int, [POINTER(RtImage), c_char_p, c_uint32]),
    "rt_image_write_png": (c_int, [POINTER(RtImage), c_char_p, c_uint32]),
    "rt_frame_hash": (c_uint64, [c_void_p, c_uint64]),
}

_LIB: Optional[ctypes.CDLL] = None


class RtError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Loads librt_trace.so (built by __graft_entry__.build()); raises if absent."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RtError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        try:  # share torch's HIP runtime when torch is present: its libamdhip64 carries the
            import torch  # noqa: F401  same soname, so loading it first keeps ONE runtime per process
        except ImportError:
            pass
        L = ctypes.CDLL(str(LIB_PATH))
        ab_build = "RT_TRACE_LIB" in os.environ  # an older A/B build may lack newer inspection hooks
        for name, (res, args) in SIGNATURES.items():
            if ab_build and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _check(rc: int, what: str) -> None:
    if rc < 0:
        msg = lib().rt_last_error()
        raise RtError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


# ------------------------------------------------------- host-side inputs
def scene_builtin(index: int) -> RtScene:
    s = RtScene()
    _check(lib().rt_scene_builtin(index, ctypes.byref(s)), "rt_scene_builtin")
    return s


def scene_prefix(scene: RtScene, n_spheres: int) -> RtScene:
    out = RtScene()
    _check(lib().rt_scene_prefix(ctypes.byref(scene), n_spheres, ctypes.byref(out)), "rt_scene_prefix")
    out._keep = getattr(scene, "_keep", None)
    return out


def scene_from_spheres(spheres: np.ndarray, look_at=(0.0, 0.0, 0.0), use_sky: bool = False,
                       distance: float = 1.0, x_angle: float = 0.0, y_height: float = 0.0) -> RtScene:
    """Scene from an (N, 20) f32 array of scalar_sphere records (main.cpp:17-21),
    converted to SIMD groups as ConvertScalarSpheresToSIMDSpheres does (main.cpp:73-91)."""
    sp = np.ascontiguousarray(spheres, dtype=np.float32).reshape(-1, 20)
    n = sp.shape[0]
    ng = (n + 3) // 4
    groups = np.zeros((ng, 16), np.float32)
    mats = np.zeros((n + 1, 12), np.float32)
    for i in range(n):
        g, l = divmod(i, 4)
        groups[g, l], groups[g, 4 + l], groups[g, 8 + l], groups[g, 12 + l] = sp[i, 0], sp[i, 1], sp[i, 2], sp[i, 4]
        mats[i] = sp[i, 8:20]
    s = RtScene()
    s.LookAt = RtV3(*look_at, 0.0)
    s.UseSkyColor = bool(use_sky)
    s.DefaultDistanceFromLookAt = distance
    s.DefaultXAngle = x_angle
    s.DefaultYHeight = y_height
    s.ScalarSpheres = RtArray(sp.ctypes.data, n)
    s.SIMDSpheres = RtArray(groups.ctypes.data, ng)
    s.Materials = RtArray(mats.ctypes.data, n + 1)
    s._keep = (sp, groups, mats)
    return s


def scene_arrays(scene: RtScene):
    """(spheres (N,20), groups (G,16), materials (M,12)) f32 copies of a scene."""
    def arr(a: RtArray, width: int):
        buf = (ctypes.c_float * (a.Count * width)).from_address(a.Data)
        return np.frombuffer(buf, dtype=np.float32).reshape(a.Count, width).copy()
    return arr(scene.ScalarSpheres, 20), arr(scene.SIMDSpheres, 16), arr(scene.Materials, 12)


def camera_setup(scene: RtScene, width: int, height: int, distance: Optional[float] = None,
                 x_angle: Optional[float] = None, y_height: Optional[float] = None) -> RtCameraInfo:
    cam = RtCameraInfo()
    d = scene.DefaultDistanceFromLookAt if distance is None else distance
    a = scene.DefaultXAngle if x_angle is None else x_angle
    h = scene.DefaultYHeight if y_height is None else y_height
    _check(lib().rt_camera_setup(ctypes.byref(scene), d, a, h, width, height, ctypes.byref(cam)), "rt_camera_setup")
    return cam


def camera_floats(cam: RtCameraInfo) -> np.ndarray:
    """The 24-float camera record the oracle consumes (position, Z, X, Y, film centre, W, H, tiles)."""
    raw = np.frombuffer(ctypes.string_at(ctypes.addressof(cam), 96), dtype=np.float32).copy()
    return raw


def pixel_seed(x: int, y: int, frame: int, width: int, height: int) -> int:
    return int(lib().rt_pixel_seed(x, y, frame, width, height))


def band_local_rows(height: int, band_rows: int, band_count: int, band_index: int) -> int:
    return int(lib().rt_band_local_rows(height, band_rows, band_count, band_index))


def scene_prefilter(scene: RtScene, simd: bool = True):
    """(r2, r2p, flags) per sphere slot 4*group+lane as rt_scene_upload packs
    them: the exact test's r^2, the secondary-ray prefilter threshold, and
    flags bit 0 = prefilter on by default, bit 1 = short candidate sqrt."""
    n, fl = c_uint32(), c_uint32()
    _check(lib().rt_scene_prefilter(ctypes.byref(scene), int(simd), None, None, 0, ctypes.byref(n), ctypes.byref(fl)),
           "rt_scene_prefilter")
    r2 = np.zeros(n.value, np.float32)
    r2p = np.zeros(n.value, np.float32)
    _check(lib().rt_scene_prefilter(ctypes.byref(scene), int(simd), r2.ctypes.data, r2p.ctypes.data, n.value,
                                    ctypes.byref(n), ctypes.byref(fl)), "rt_scene_prefilter")
    return r2, r2p, int(fl.value)


def scene_clusters(scene: RtScene, simd: bool = True):
    """The clustered prefilter table rt_scene_upload builds: (table (n, rows, 4)
    f32, n_cpairs) with rows = 4 for a one-word pair mask (<= 32 groups), else
    3 + words (rt_kernel.h cl_entry_f4); n_cpairs == 0 means the per-group loop
    is used."""
    nf4, ncp = c_uint32(), c_uint32()
    _check(lib().rt_scene_clusters(ctypes.byref(scene), int(simd), None, 0, ctypes.byref(nf4), ctypes.byref(ncp)),
           "rt_scene_clusters")
    tab = np.zeros((nf4.value, 4), np.float32)
    if nf4.value:
        _check(lib().rt_scene_clusters(ctypes.byref(scene), int(simd), tab.ctypes.data, nf4.value, ctypes.byref(nf4),
                                       ctypes.byref(ncp)), "rt_scene_clusters")
    # the pair-mask words follow the rule set's group count (rt_host.cpp pack_set):
    # SIMDSpheres groups for the SIMD rules, ceil(ScalarSpheres / 4) for the scalar ones;
    # per-lane ("relative") tables carry a fifth row at one word (the height slab)
    groups = scene.SIMDSpheres.Count if simd else (scene.ScalarSpheres.Count + 3) // 4
    words = 1 if groups <= 32 else 2 if groups <= 64 else 4
    relative = bool(scene_prefilter(scene, simd)[2] & 4)
    rows = (5 if relative else 4) if words == 1 else 3 + words
    return tab.reshape(-1, rows, 4), int(ncp.value)


def scene_cluster_layout(scene: RtScene, simd: bool = True):
    """(levels, sub_pairs) of the clustered prefilter table (rt_scene_cluster_layout):
    levels 2 means the first n_cpairs entries index sub_pairs sub-cluster pair
    entries, which index the member entries."""
    lv, sp = c_uint32(), c_uint32()
    _check(lib().rt_scene_cluster_layout(ctypes.byref(scene), int(simd), ctypes.byref(lv), ctypes.byref(sp)),
           "rt_scene_cluster_layout")
    return int(lv.value), int(sp.value)


def rsqrt_table_builtin() -> np.ndarray:
    t = np.zeros(2048, np.float32)
    _check(lib().rt_rsqrt_table_builtin(t.ctypes.data), "rt_rsqrt_table_builtin")
    return t


# ---------------------------------------------------------------- device
class Device:
    """One GPU: rsqrt table, uploaded scene, trace launches (rt_device)."""

    def __init__(self, ordinal: int = 0, rsqrt_table: Optional[np.ndarray] = None, options: Optional[dict] = None):
        h = c_void_p()
        o = device_options(options)
        _check(lib().rt_device_create_ex(ordinal, ctypes.byref(o) if o is not None else None, ctypes.byref(h)),
               "rt_device_create")
        self.handle = h
        table = rsqrt_table_builtin() if rsqrt_table is None else np.ascontiguousarray(rsqrt_table, np.float32)
        _check(lib().rt_set_rsqrt_table(self.handle, table.ctypes.data), "rt_set_rsqrt_table")
        self._scene = None

    def upload_scene(self, scene: RtScene) -> None:
        _check(lib().rt_scene_upload(self.handle, ctypes.byref(scene)), "rt_scene_upload")
        self._scene = scene

    def options(self) -> dict:
        """The non-default rt_device_options the device was created with."""
        o = RtDeviceOptions()
        _check(lib().rt_device_get_options(self.handle, ctypes.byref(o)), "rt_device_get_options")
        return {n: int(getattr(o, n)) for n in OPTION_FIELDS if getattr(o, n)}

    def trace(self, cam: RtCameraInfo, *, width: int, height: int, prev_ptr: int, cur_ptr: int, rays_ptr: int,
              prev_count: int = 0, frames: int = 1, max_bounce: int = 5, simd: bool = True,
              band_rows: int = 32, band_count: int = 1, band_index: int = 0, accum_zero: bool = False,
              srgb_pow: bool = False, stream: Optional[int] = None) -> None:
        """Traces `frames` progressive frames into device images (raw device pointers)
        on the HIP stream handle `stream` (None/0 = the null stream)."""
        c = RtCameraInfo()
        ctypes.pointer(c)[0] = cam
        c.CurrentImage = RtImage(cur_ptr, width, height, RT_FORMAT_R8G8B8A8_U32)
        c.PreviousImage = RtImage(prev_ptr, width, height, RT_FORMAT_R32B32G32A32_F32)
        d = RtTraceDesc(width, height, prev_count, frames, max_bounce, 1 if simd else 0, RT_SEED_PIXEL,
                        band_rows, band_count, band_index,
                        (RT_FLAG_ACCUM_ZERO if accum_zero else 0) | (RT_FLAG_SRGB_POW if srgb_pow else 0))
        _check(lib().rt_trace(self.handle, ctypes.byref(c), ctypes.byref(d), c_void_p(rays_ptr),
                              c_void_p(stream or 0)), "rt_trace")

    def last_info(self) -> dict:
        """What the last trace launched (rt_trace_last_info): segments counted
        but folded analytically (dead tiles), P, tiles traced / total, whether
        the cull pass ran."""
        info = RtTraceInfo()
        _check(lib().rt_trace_last_info(self.handle, ctypes.byref(info)), "rt_trace_last_info")
        return {n: int(getattr(info, n)) for n, _ in RtTraceInfo._fields_}

    def reserve(self, width: int, local_rows: int) -> None:
        """rt_device_reserve: pre-size the launch buffers for bands up to width x local_rows."""
        _check(lib().rt_device_reserve(self.handle, width, local_rows), "rt_device_reserve")

    def debug_stats(self, reset: bool = True):
        """RT_STATS=1 scheduling counters (see rt_debug_stats), or None when disabled."""
        out = np.zeros(32, np.uint64)
        rc = lib().rt_debug_stats(self.handle, out.ctypes.data, int(reset))
        _check(rc, "rt_debug_stats")
        if rc == 0:
            return None
        keys = ["pri_iters", "pri_lanes", "sec_iters", "sec_lanes", "pri_groups", "sec_hit_groups",
                "sec_sparse_iters", "sec_sparse_lanes", "sec_tail_iters", "pri_cycles", "sec_cycles",
                "fold_cycles", "init_cycles", "cull_cycles", "sync_cycles", "post_cycles", "pf_iters", "pf_groups",
                "cl_tested", "pf_pairs", "cl_top_entered", "pf_lane_pairs", "pri_blocked", "pri_waitsec",
                "pri_done", "sec_done", "sec_waitpri", "done_trips", "done_lane_trips",
                "sec_exact", "sec_badlanes", "sec_zerodir"]
        return {k: int(v) for k, v in zip(keys, out) if not k.startswith("_")}

    def debug_wave_times(self, max_waves: int = 1 << 22):
        """RT_WAVETIMES=1: (n, 2) array of per-wave {start, end} (100 MHz ticks), or None."""
        out = np.zeros(2 * max_waves, np.uint64)
        n = int(lib().rt_debug_wave_times(self.handle, out.ctypes.data, max_waves))
        _check(n, "rt_debug_wave_times")
        return out[: 2 * n].reshape(-1, 2) if n else None

    def debug_masks(self, max_words: int = 1 << 24):
        """Primary group masks of the last cull pass (see rt_debug_masks), or None."""
        out = np.zeros(max_words, np.uint64)
        n = int(lib().rt_debug_masks(self.handle, out.ctypes.data, max_words))
        _check(n, "rt_debug_masks")
        return out[:n].copy() if n else None

    def synchronize(self) -> None:
        _check(lib().rt_device_synchronize(self.handle), "rt_device_synchronize")

    def close(self) -> None:
        if self.handle:
            lib().rt_device_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """Several GPUs from one process (rt_multi): interleaved row bands, one
    device each, gathered to devices[0] over RCCL or peer copies."""

    def __init__(self, devices, transport: int = RT_MULTI_AUTO, rsqrt_table: Optional[np.ndarray] = None,
                 options: Optional[dict] = None):
        devs = (c_int * len(devices))(*devices)
        h = c_void_p()
        o = device_options(options)
        _check(lib().rt_multi_create_ex(devs, len(devices), transport, ctypes.byref(o) if o is not None else None,
                                        ctypes.byref(h)), "rt_multi_create")
        self.handle = h
        table = rsqrt_table_builtin() if rsqrt_table is None else np.ascontiguousarray(rsqrt_table, np.float32)
        _check(lib().rt_multi_set_rsqrt_table(self.handle, table.ctypes.data), "rt_multi_set_rsqrt_table")

    def upload_scene(self, scene: RtScene) -> None:
        _check(lib().rt_multi_scene_upload(self.handle, ctypes.byref(scene)), "rt_multi_scene_upload")

    def trace(self, cam: RtCameraInfo, *, width: int, height: int, cur_ptr: int, rays_ptr: int, prev_ptr: int = 0,
              prev_count: int = 0, frames: int = 1, max_bounce: int = 5, simd: bool = True, band_rows: int = 8,
              accum_zero: bool = False, srgb_pow: bool = False, stream: Optional[int] = None) -> None:
        """Full-frame RGBA8 (and, with prev_ptr, the gathered running mean) on devices[0]."""
        c = RtCameraInfo()
        ctypes.pointer(c)[0] = cam
        c.CurrentImage = RtImage(cur_ptr, width, height, RT_FORMAT_R8G8B8A8_U32)
        c.PreviousImage = RtImage(prev_ptr or None, width, height, RT_FORMAT_R32B32G32A32_F32)
        d = RtTraceDesc(width, height, prev_count, frames, max_bounce, 1 if simd else 0, RT_SEED_PIXEL, band_rows, 0, 0,
                        (RT_FLAG_ACCUM_ZERO if accum_zero else 0) | (RT_FLAG_SRGB_POW if srgb_pow else 0))
        _check(lib().rt_multi_trace(self.handle, ctypes.byref(c), ctypes.byref(d), c_void_p(rays_ptr),
                                    c_void_p(stream or 0)), "rt_multi_trace")

    def last_trace_ms(self, n_devices: int) -> list:
        """Each device's trace time (ms) of the last trace call (waits for them)."""
        out = (c_float * n_devices)()
        _check(lib().rt_multi_last_trace_ms(self.handle, out, n_devices), "rt_multi_last_trace_ms")
        return [float(v) for v in out]

    def last_gather_ms(self) -> float:
        """The last call's gather (transfer + scatter) time on devices[0] (waits for it)."""
        ms = c_float(0.0)
        _check(lib().rt_multi_last_gather_ms(self.handle, ctypes.byref(ms)), "rt_multi_last_gather_ms")
        return float(ms.value)

    def shard_info(self, index: int) -> dict:
        """rt_trace_last_info of devices[index] for the last call."""
        info = RtTraceInfo()
        _check(lib().rt_multi_shard_info(self.handle, index, ctypes.byref(info)), "rt_multi_shard_info")
        return {n: int(getattr(info, n)) for n, _ in RtTraceInfo._fields_}

    def reserve(self, width: int, height: int, band_rows: int = 8, mean: bool = False) -> None:
        """rt_multi_reserve: pre-size every buffer a call of this geometry needs."""
        _check(lib().rt_multi_reserve(self.handle, width, height, band_rows, RT_MULTI_RESERVE_MEAN if mean else 0),
               "rt_multi_reserve")

    def resident_frames(self) -> int:
        """Frames folded into the devices' resident means (0: none resident, rt_multi_resident_frames)."""
        n = c_uint64(0)
        _check(lib().rt_multi_resident_frames(self.handle, ctypes.byref(n)), "rt_multi_resident_frames")
        return int(n.value)

    def info(self) -> dict:
        i = RtMultiInfo()
        _check(lib().rt_multi_get_info(self.handle, ctypes.byref(i)), "rt_multi_get_info")
        return {n: int(getattr(i, n)) for n, _ in RtMultiInfo._fields_}

    def synchronize(self) -> None:
        _check(lib().rt_multi_synchronize(self.handle), "rt_multi_synchronize")

    def close(self) -> None:
        if self.handle:
            lib().rt_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(RT_COMM_ID_BYTES)
    _check(lib().rt_comm_unique_id(buf), "rt_comm_unique_id")
    return buf.raw


class Comm:
    """The RCCL band gather of a one-process-per-GPU launch (rt_comm)."""

    def __init__(self, device: int, uid: bytes, nranks: int, rank: int):
        assert len(uid) == RT_COMM_ID_BYTES
        h = c_void_p()
        buf = ctypes.create_string_buffer(uid, RT_COMM_ID_BYTES)
        _check(lib().rt_comm_create(device, buf, nranks, rank, ctypes.byref(h)), "rt_comm_create")
        self.handle = h

    def gather_bands(self, local_ptr: int, full_ptr: int, width: int, height: int, elem_bytes: int, band_rows: int,
                     stream: Optional[int] = None) -> None:
        _check(lib().rt_comm_gather_bands(self.handle, c_void_p(local_ptr or None), c_void_p(full_ptr or None), width,
                                          height, elem_bytes, band_rows, c_void_p(stream or 0)),
               "rt_comm_gather_bands")

    def close(self) -> None:
        if self.handle:
            lib().rt_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def assemble_bands(compact_ptr: int, rank_stride_bytes: int, dst_ptr: int, width: int, height: int,
                   elem_bytes: int, band_rows: int, band_count: int, stream: Optional[int] = None) -> None:
    _check(lib().rt_assemble_bands(c_void_p(compact_ptr), rank_stride_bytes, c_void_p(dst_ptr), width, height,
                                   elem_bytes, band_rows, band_count, c_void_p(stream or 0)),
           "rt_assemble_bands")


def encode_rgba8(accum_ptr: int, rgba8_ptr: int, n_pixels: int, srgb_pow: bool = False,
                 stream: Optional[int] = None) -> None:
    """ColorFromV4(LinearToSRGB(v)) over a device-resident running mean (main.cpp:312-346)."""
    _check(lib().rt_encode_rgba8(c_void_p(accum_ptr), c_void_p(rgba8_ptr), n_pixels,
                                 RT_FLAG_SRGB_POW if srgb_pow else 0, c_void_p(stream or 0)), "rt_encode_rgba8")


# ------------------------------------------------- OnInit / OnRender mirror
def on_init(devices=None) -> RtInitParams:
    """OnInit; `devices` (a list of HIP ordinals) drives several GPUs through rt_multi."""
    p = RtInitParams()
    if devices is None:
        _check(lib().rt_on_init(ctypes.byref(p)), "rt_on_init")
    else:
        devs = (c_int * len(devices))(*devices)
        _check(lib().rt_on_init_devices(ctypes.byref(p), devs, len(devices)), "rt_on_init_devices")
    return p


def on_render(image: np.ndarray, scene_index: int, enable_simd: bool = True, keys: int = 0):
    """OnRender(Image, RenderParams, &Rays, &Time): `image` is an (H, W) uint32
    RGBA8 host array.  Returns (completed, total_rays_cast, time_elapsed_ms)."""
    assert image.dtype == np.uint32 and image.ndim == 2 and image.flags.c_contiguous
    img = RtImage(image.ctypes.data, image.shape[1], image.shape[0], RT_FORMAT_R8G8B8A8_U32)
    rays = c_uint64(0)
    ms = c_double(0.0)
    rc = lib().rt_on_render(ctypes.byref(img), RtRenderParams(0, enable_simd, scene_index), keys,
                            ctypes.byref(rays), ctypes.byref(ms))
    _check(rc, "rt_on_render")
    return bool(rc), int(rays.value), float(ms.value)


def on_render_register_image(image: np.ndarray) -> None:
    """rt_on_render_register_image: page-lock `image` so frames handed to it
    arrive by one DMA; keep it alive until on_render_unregister_image()."""
    assert image.dtype == np.uint32 and image.flags.c_contiguous
    _check(lib().rt_on_render_register_image(c_void_p(image.ctypes.data), c_uint64(image.nbytes)),
           "rt_on_render_register_image")


def on_render_unregister_image() -> None:
    _check(lib().rt_on_render_unregister_image(), "rt_on_render_unregister_image")


def on_render_reserve(width: int, height: int) -> None:
    """rt_on_render_reserve: frames up to width x height need no allocation in the frame loop."""
    _check(lib().rt_on_render_reserve(width, height), "rt_on_render_reserve")


def on_render_wait() -> None:
    _check(lib().rt_on_render_wait(), "rt_on_render_wait")


def on_shutdown() -> None:
    _check(lib().rt_on_shutdown(), "rt_on_shutdown")


def on_render_profile(reset: bool = False) -> dict:
    """Where rt_on_render's time went (rt_on_render_get_profile): calls, frames
    launched / handed out, host ms in the call, its frame copies and waits,
    and the frames' GPU time."""
    p = RtOnRenderProfile()
    _check(lib().rt_on_render_get_profile(ctypes.byref(p), int(reset)), "rt_on_render_get_profile")
    return {n: (int(getattr(p, n)) if t is c_uint64 else float(getattr(p, n))) for n, t in RtOnRenderProfile._fields_}


# ------------------------------------------------------------ output path
RT_IMAGE_FLIP_Y = 1


def write_image(image: np.ndarray, path, flip_y: bool = True) -> None:
    """Writes an (H, W) uint32 RGBA8 host frame (rt_on_render / rt_trace's
    CurrentImage) as PPM or PNG by the path's suffix (rt_image_write_ppm /
    rt_image_write_png); flip_y: on-screen orientation (row H-1 first)."""
    assert image.dtype == np.uint32 and image.ndim == 2 and image.flags.c_contiguous
    img = RtImage(image.ctypes.data, image.shape[1], image.shape[0], RT_FORMAT_R8G8B8A8_U32)
    path = str(path)
    fn = lib().rt_image_write_png if path.lower().endswith(".png") else lib().rt_image_write_ppm
    name = "rt_image_write_png" if path.lower().endswith(".png") else "rt_image_write_ppm"
    _check(fn(ctypes.byref(img), path.encode(), RT_IMAGE_FLIP_Y if flip_y else 0), name)


def code_object_hash(path=None) -> str:
    """SHA-256 (first 16 hex digits) of the gfx950 code objects a library
    carries: the bytes of its ELF `.hip_fatbin` section (every kernel
    translation unit's offload bundle).  Host-only changes leave it alone; any
    kernel change moves it.  bench.py uses a committed PMC record only when
    the record's `binary_hash` equals the loaded library's.  Reads the file
    (no GPU, no load)."""
    import hashlib
    import struct
    data = pathlib.Path(path or LIB_PATH).read_bytes()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise RtError(f"{path or LIB_PATH}: not an ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    for name, _, _, _, off, size in secs:
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise RtError(f"{path or LIB_PATH}: no .hip_fatbin section")


def frame_hash(a) -> int:
    """FNV-1a 64 of a host array's bytes (rt_frame_hash): the golden fixtures' frame checksum."""
    a = np.ascontiguousarray(a)
    return int(lib().rt_frame_hash(c_void_p(a.ctypes.data), a.nbytes))
