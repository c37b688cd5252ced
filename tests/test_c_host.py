"""The plain-C host of the C-ABI (examples/c_host/render.c): a C99 program that
drives OnInit / OnRender (main.cpp:645-859) through include/rt_trace.h only,
as the reference's platform layers do.

CPU: the header and the host compile as strict C99 and link against the
library.  GPU: tests/conftest.py starts the host before this process touches
the GPU, on one device and on three bands of the same device
(rt_on_init_devices -> rt_multi); each completed progressive frame must equal
the oracle's frame bit for bit (OnRender's reference literal of 5 bounces)."""
import pathlib
import shutil
import subprocess

import numpy as np
import pytest

from conftest import C_HOST_FRAMES, C_HOST_H, C_HOST_SCENE, C_HOST_W, ROOT


def test_c_host_compiles_as_c99(tmp_path):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    lib = ROOT / "simd-ray-tracer_amd" / "librt_trace.so"
    if not lib.exists():
        pytest.skip("librt_trace.so not built")
    out = tmp_path / "render"
    subprocess.run([gcc, "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", "-I", str(ROOT / "include"),
                    str(ROOT / "examples" / "c_host" / "render.c"), "-L", str(lib.parent), "-lrt_trace",
                    "-o", str(out)], check=True)
    assert out.exists()


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["one_device", "three_bands"])
def test_c_host_frames_match_oracle(c_host_runs, orc, name):
    rc, prefix = c_host_runs[name]
    log = pathlib.Path(str(prefix) + ".log")
    assert rc == 0, log.read_text() if log.exists() else rc
    lines = [l for l in log.read_text().splitlines() if l.startswith("frame ")]
    assert len(lines) == C_HOST_FRAMES, lines
    o = orc.scene_builtin(C_HOST_SCENE)
    ocam = orc.camera(o, C_HOST_W, C_HOST_H)
    for k in range(C_HOST_FRAMES):
        got = np.fromfile(f"{prefix}.{k}.rgba", dtype=np.uint32)
        _, ocur, orays = orc.render(o, ocam, C_HOST_W, C_HOST_H, frames=k + 1, max_bounce=5)
        assert np.array_equal(got, ocur), (name, k)
    png = pathlib.Path(str(prefix) + ".png")
    assert png.exists() and png.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
