"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/liboracle.so, the plain-C restatement of the
reference trace path (see rt_oracle.h for the file:line map).  Imported only
by tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke(), and only
as the checker.  The product package never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess
from ctypes import c_float, c_int, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
REF_PATH = HERE / "_ref" / "librefmath.so"
LUT_PATH = HERE.parent / "tests" / "golden" / "rsqrt_lut_intel.bin"

_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE), "liboracle.so"], check=True)


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        L.or_pcg.restype = c_uint32
        L.or_pcg.argtypes = [c_void_p]
        L.or_random_float.restype = c_float
        L.or_random_float.argtypes = [c_void_p, c_float, c_float]
        L.or_seed_mix.restype = c_uint64
        L.or_seed_mix.argtypes = [c_uint64]
        L.or_set_rsqrt_lut.argtypes = [c_void_p]
        L.or_rsqrt.restype = c_float
        L.or_rsqrt.argtypes = [c_float]
        L.or_normalize.argtypes = [c_void_p, c_void_p]
        L.or_normalize_fast.argtypes = [c_void_p, c_void_p]
        L.or_scene_builtin.restype = c_int
        L.or_scene_builtin.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_void_p]
        L.or_camera_setup.argtypes = [c_void_p, c_float, c_float, c_float, c_uint32, c_uint32, c_void_p]
        L.or_render.restype = c_int
        L.or_render.argtypes = [c_void_p, c_uint32, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p, c_uint32,
                                c_uint32, c_uint32, c_uint32, c_uint32, c_int, c_int, c_uint32, c_void_p, c_uint32,
                                c_uint32, c_void_p, c_void_p, c_void_p]
        L.or_fnv1a64.restype = c_uint64
        L.or_fnv1a64.argtypes = [c_void_p, c_uint64]
        L.or_group_test.argtypes = [c_void_p] * 5
        L.or_horizontal_min.restype = c_float
        L.or_horizontal_min.argtypes = [c_void_p, c_void_p]
        L.or_cross.argtypes = [c_void_p] * 3
        L.or_encode_rgba8.argtypes = [c_void_p, c_void_p, c_uint64, c_int]
        L.or_srgb_channel.restype = c_float
        L.or_srgb_channel.argtypes = [c_float, c_int]
        L.or_reflectance.restype = c_float
        L.or_reflectance.argtypes = [c_float, c_float]
        L.or_blend_store.argtypes = [c_uint32, c_void_p, c_void_p, c_void_p]
        L.or_emit_attenuate.argtypes = [c_void_p] * 4
        L.or_srgb_n.argtypes = [c_void_p, c_void_p, c_uint64]
        _L = L
        set_lut(np.fromfile(LUT_PATH, dtype=np.float32))
    return _L


def set_lut(lut: np.ndarray) -> None:
    global _LUT
    _LUT = np.ascontiguousarray(lut, dtype=np.float32)
    assert _LUT.size == 2048
    lib().or_set_rsqrt_lut(_LUT.ctypes.data)


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


class Scene:
    """Oracle-side scene: spheres (N,20), groups (G,16), materials (M,12) f32 + metadata."""

    def __init__(self, spheres, groups, materials, look_at=(0.0, 0.0, 0.0), use_sky=False,
                 distance=1.0, x_angle=0.0, y_height=0.0):
        self.spheres = np.ascontiguousarray(spheres, np.float32).reshape(-1, 20)
        self.groups = np.ascontiguousarray(groups, np.float32).reshape(-1, 16)
        self.materials = np.ascontiguousarray(materials, np.float32).reshape(-1, 12)
        self.look_at = np.array([*look_at[:3], 0.0], np.float32)
        self.use_sky = bool(use_sky)
        self.distance, self.x_angle, self.y_height = float(distance), float(x_angle), float(y_height)

    def prefix(self, n: int) -> "Scene":
        """First n spheres, as the survey's synthetic scenes (counts n, ceil(n/4), n+1; shared data)."""
        ng = (n + 3) // 4
        return Scene(self.spheres[:n], self.groups[:ng], self.materials[:n + 1], self.look_at, self.use_sky,
                     self.distance, self.x_angle, self.y_height)


def scene_builtin(index: int) -> Scene:
    L = lib()
    sp = np.zeros((482, 20), np.float32)
    gr = np.zeros((121, 16), np.float32)
    ma = np.zeros((483, 12), np.float32)
    info = np.zeros(16, np.uint32)
    assert L.or_scene_builtin(index, _p(sp), _p(gr), _p(ma), _p(info)) == 0
    f = info.view(np.float32)
    n, ng, nm = int(info[8]), int(info[9]), int(info[10])
    return Scene(sp[:n], gr[:ng], ma[:nm], tuple(f[:3]), bool(info[4]), f[5], f[6], f[7])


def camera(scene: Scene, width: int, height: int, distance=None, x_angle=None, y_height=None) -> np.ndarray:
    cam = np.zeros(24, np.float32)
    lib().or_camera_setup(_p(scene.look_at), scene.distance if distance is None else distance,
                          scene.x_angle if x_angle is None else x_angle,
                          scene.y_height if y_height is None else y_height, width, height, _p(cam))
    return cam


SEED_STREAM, SEED_PIXEL = 0, 1


def render(scene: Scene, cam: np.ndarray, width: int, height: int, *, prev_count: int = 0, frames: int = 1,
           max_bounce: int = 5, simd: bool = True, seed_mode: int = SEED_PIXEL, threads: int = 1,
           prev: np.ndarray | None = None, cur: np.ndarray | None = None, rows=(0, 0), stream_states=None):
    """Returns (prev_v4 (H*W,4) f32, cur (H*W,) u32, rays)."""
    L = lib()
    if prev is None:
        prev = np.zeros((width * height, 4), np.float32)
    if cur is None:
        cur = np.zeros(width * height, np.uint32)
    rays = np.zeros(1, np.uint64)
    st = stream_states
    if seed_mode == SEED_STREAM and st is None:
        st = np.array([L.or_seed_mix(i) for i in range(max(threads, 1))], np.uint64)
    cam = np.ascontiguousarray(cam, np.float32)
    rc = L.or_render(_p(scene.groups), scene.groups.shape[0], _p(scene.spheres), scene.spheres.shape[0],
                     _p(scene.materials), int(scene.use_sky), _p(cam), width, height, prev_count, frames,
                     max_bounce, int(simd), seed_mode, threads, _p(st) if st is not None else None,
                     rows[0], rows[1], _p(prev), _p(cur), _p(rays))
    assert rc == 0, rc
    return prev, cur, int(rays[0])


def encode_rgba8(prev_v4: np.ndarray, srgb_pow: bool = False) -> np.ndarray:
    """main.cpp:312-346: RGBA8 (u32) of running means (..., 4) f32; srgb_pow picks
    LinearToSRGB's exact-pow branch (main.cpp:320-321)."""
    v = np.ascontiguousarray(prev_v4, np.float32).reshape(-1, 4)
    out = np.empty(len(v), np.uint32)
    lib().or_encode_rgba8(_p(v), _p(out), len(v), 1 if srgb_pow else 0)
    return out


def fnv1a64(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a)
    return int(lib().or_fnv1a64(_p(a), a.nbytes))


def seed_mix(i: int) -> int:
    return int(lib().or_seed_mix(i))


def cpu_threads() -> int:
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1
