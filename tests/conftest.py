"""Shared fixtures.  `gpu`-marked tests need a real MI355X (run via gpurun);
everything else runs on the CPU-only container."""
import os
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import __graft_entry__ as graft  # noqa: E402


MULTIRANK_OUT = ROOT / "gpurun_out" / "multirank_check.json"
_multirank = {}


def _selects_gpu(config) -> bool:
    expr = (config.option.markexpr or "").replace(" ", "")
    return "gpu" in expr and "notgpu" not in expr


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run on the GPU box")
    # bench.py's multi-rank path runs as child processes (torchrun); they are
    # started here, before this process touches the GPU, and
    # tests/test_multirank_bench.py collects their result.
    if _selects_gpu(config) and os.environ.get("RT_SKIP_MULTIRANK") != "1":
        import subprocess
        MULTIRANK_OUT.parent.mkdir(exist_ok=True)
        if MULTIRANK_OUT.exists():
            MULTIRANK_OUT.unlink()
        log = open(MULTIRANK_OUT.with_suffix(".log"), "w")
        _multirank["proc"] = subprocess.Popen([sys.executable, str(ROOT / "scripts" / "multirank_check.py"),
                                               str(MULTIRANK_OUT)], cwd=ROOT, stdout=log, stderr=subprocess.STDOUT)


    # the plain-C host (examples/c_host/render) on one device and on three
    # bands of the same device, also started before this process touches the
    # GPU; tests/test_c_host.py compares its frames with the oracle's
    if _selects_gpu(config) and C_HOST_BIN.exists():
        import subprocess
        C_HOST_OUT.mkdir(parents=True, exist_ok=True)
        for name, devs in C_HOST_RUNS.items():
            for old in C_HOST_OUT.glob(name + ".*"):
                old.unlink()
            log = open(C_HOST_OUT / (name + ".log"), "w")
            _c_host[name] = subprocess.Popen([str(C_HOST_BIN), str(C_HOST_W), str(C_HOST_H), str(C_HOST_FRAMES),
                                              str(C_HOST_SCENE), str(C_HOST_OUT / name), devs],
                                             cwd=ROOT, stdout=log, stderr=subprocess.STDOUT)


    # rt_multi's RCCL branch over eight shards of this GPU, through the test-only
    # loopback librccl.so.1 (tests/loopback_rccl, first on LD_LIBRARY_PATH of that
    # child only); tests/test_gpu_multi.py checks its frames
    if _selects_gpu(config) and LOOPBACK_BIN.exists():
        import subprocess
        if LOOPBACK_OUT.exists():
            LOOPBACK_OUT.unlink()
        LOOPBACK_OUT.parent.mkdir(exist_ok=True)
        env = dict(os.environ)
        env["LD_LIBRARY_PATH"] = os.pathsep.join(p for p in (str(LOOPBACK_BIN.parent), env.get("LD_LIBRARY_PATH"))
                                                 if p)
        log = open(LOOPBACK_OUT.with_suffix(".log"), "w")
        _loopback["proc"] = subprocess.Popen([str(LOOPBACK_BIN), str(LOOPBACK_OUT), "8"], cwd=ROOT, env=env,
                                             stdout=log, stderr=subprocess.STDOUT)


LOOPBACK_BIN = ROOT / "tests" / "loopback_rccl" / "multi_rccl_check"
LOOPBACK_OUT = ROOT / "gpurun_out" / "multi_rccl_check.json"
_loopback = {}


@pytest.fixture(scope="session")
def loopback_rccl_result():
    """(exit code, JSON) of tests/loopback_rccl/multi_rccl_check (waits for it)."""
    import json
    p = _loopback.get("proc")
    if p is None:
        pytest.skip("loopback RCCL run not started (run with -m gpu after build())")
    rc = p.wait(timeout=280)
    return rc, (json.loads(LOOPBACK_OUT.read_text()) if LOOPBACK_OUT.exists() else None)


def pytest_unconfigure(config):
    for p in [_multirank.get("proc"), _loopback.get("proc")] + list(_c_host.values()):
        if p is not None and p.poll() is None:
            try:
                p.wait(timeout=300)
            except Exception:
                p.kill()


C_HOST_BIN = ROOT / "examples" / "c_host" / "render"
C_HOST_OUT = ROOT / "gpurun_out" / "c_host"
C_HOST_RUNS = {"one_device": "0", "three_bands": "0,0,0"}
C_HOST_W, C_HOST_H, C_HOST_FRAMES, C_HOST_SCENE = 72, 40, 3, 0
_c_host = {}


@pytest.fixture(scope="session")
def c_host_runs():
    """{run name: (exit code, output prefix)} of the plain-C host runs (waits for them)."""
    if not _c_host:
        pytest.skip("C host runs not started (run with -m gpu after build())")
    out = {}
    for name, p in _c_host.items():
        out[name] = (p.wait(timeout=280), C_HOST_OUT / name)
    return out


@pytest.fixture(scope="session")
def multirank_result():
    """Result list of scripts/multirank_check.py (waits for it)."""
    import json
    p = _multirank.get("proc")
    if p is None:
        pytest.skip("multi-rank rehearsal not started (run with -m gpu)")
    p.wait(timeout=280)
    return json.loads(MULTIRANK_OUT.read_text())


def _ensure_built():
    lib = ROOT / "simd-ray-tracer_amd" / "librt_trace.so"
    orc = ROOT / "oracle" / "liboracle.so"
    if not lib.exists() or not orc.exists():
        graft.build()


@pytest.fixture(scope="session")
def rt():
    _ensure_built()
    pkg = graft.load_package()
    pkg.lib()
    return pkg


@pytest.fixture(scope="session")
def orc():
    _ensure_built()
    from oracle import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def refmath():
    """The reference's own code (base.h + x64_math.h and main.cpp:7-640,
    compiled from /root/reference by `make -C oracle ref`); only present in the
    build container."""
    import ctypes
    path = ROOT / "oracle" / "_ref" / "librefmath.so"
    if not path.exists():
        pytest.skip("oracle/_ref/librefmath.so not built (needs /root/reference)")
    L = ctypes.CDLL(str(path))
    f, v, u32, u64p, u64 = ctypes.c_float, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64
    for name, res, args in [("ref_pcg", u32, [u64p]), ("ref_random_float", f, [u64p, f, f]), ("ref_rsqrt", f, [f]),
                            ("ref_sqrt", f, [f]), ("ref_min", f, [f, f]), ("ref_normalize", None, [v, v]),
                            ("ref_normalize_fast", None, [v, v]), ("ref_cross", None, [v, v, v]),
                            ("ref_dot", f, [v, v]), ("ref_cos", f, [f]), ("ref_sin", f, [f]),
                            ("ref_horizontal_min", f, [v]), ("ref_group_test", None, [v, v, v, v, v, v, v, v]),
                            ("ref_reflectance", f, [f, f]), ("ref_linear_to_srgb", f, [f]),
                            ("ref_color_from_v4", u32, [v]), ("ref_encode_rgba8", None, [v, v, u64]),
                            ("ref_linear_to_srgb_n", None, [v, v, u64]), ("ref_blend_store", None, [u32, v, v, v]),
                            ("ref_emit_attenuate", None, [v, v, v, v]),
                            ("ref_scene_builtin", ctypes.c_int, [ctypes.c_int, v, u32, v, u32, v, u32, v]),
                            ("ref_render", None, [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int,
                                                  v, v, v, v])]:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


@pytest.fixture(scope="session")
def refpix():
    """The reference's main.cpp:7-640 with SURVEY §8c's two textual patches
    (bounce count, per-pixel seeds) on a temporary copy (`make -C oracle ref`,
    oracle/_ref/librefpix.so); only present in the build container."""
    import ctypes
    path = ROOT / "oracle" / "_ref" / "librefpix.so"
    if not path.exists():
        pytest.skip("oracle/_ref/librefpix.so not built (needs /root/reference)")
    L = ctypes.CDLL(str(path))
    v, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.ref_set_patch.restype = None
    L.ref_set_patch.argtypes = [u32, ctypes.c_int]
    L.ref_render.restype = None
    L.ref_render.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, v, v, v, v]
    L.ref_render_threads.restype = None
    L.ref_render_threads.argtypes = [v, u32, v, u32, v, u32, u32, v, u32, u32, u32, u32, ctypes.c_int, u32, v, v, v]
    yield L
    L.ref_set_patch(5, 0)


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def host_is_intel() -> bool:
    try:
        return "GenuineIntel" in pathlib.Path("/proc/cpuinfo").read_text()
    except OSError:
        return False
