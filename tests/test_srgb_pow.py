"""LinearToSRGB's exact-pow branch (main.cpp:320-321, '#if 0' in the
reference; RT_FLAG_SRGB_POW) on the CPU.

The reference's powf is libm's (musl in its WASM build, glibc here: the same
algorithm, not correctly rounded).  The kernel takes the f64 pow rounded once
to f32 (rt_kernel.hip linear_to_srgb_pow).  These tests pin that choice
exhaustively over every f32 the branch sees, [0.0031308, 1]: the f32 values may
differ in the last bit, the RGBA8 bytes never do.  The GPU's own bytes are
checked against the oracle over the same inputs in
tests/test_gpu_parity.py::test_encode_rgba8_exhaustive.
"""
import numpy as np

F = np.float32
Y = np.float64(F(1.0) / F(2.4))  # 1.0f / 2.4f, as the reference writes it


def every_f32_in_pow_branch() -> np.ndarray:
    lo = np.array([0.0031308], F).view(np.uint32)[0]
    return np.arange(lo, 0x3F800000 + 1, dtype=np.uint32).view(F)


def u8(v: np.ndarray) -> np.ndarray:
    """main.cpp:341-343: (u8)(Saturate(v) * 255) by truncation."""
    s = np.clip(v, F(0), F(1)) * F(255)
    return s.astype(np.int32) & 0xFF


def kernel_model(L: np.ndarray) -> np.ndarray:
    """rt_kernel.hip linear_to_srgb_pow, op for op (f64 pow, f32 rest, unfused)."""
    p = np.power(L.astype(np.float64), Y).astype(F)
    return F(1.055) * p - F(0.055)


def oracle_bytes(orc, L: np.ndarray, pow_mode: bool) -> np.ndarray:
    v = np.zeros((len(L), 4), F)
    v[:, 0] = L
    return orc.encode_rgba8(v, srgb_pow=pow_mode) & 0xFF


def test_pow_branch_bytes_match_libm_powf_exhaustively(orc):
    L = every_f32_in_pow_branch()
    assert len(L) == 70_439_397
    for i in range(0, len(L), 1 << 23):
        c = L[i:i + (1 << 23)]
        assert np.array_equal(u8(kernel_model(c)), oracle_bytes(orc, c, True)), f"RGBA8 differs in chunk {i}"
    # (the f32 values themselves differ on 45,775 of these inputs: DESIGN.md §9)
    probe = L[:: 1 << 16]
    o = np.array([orc.lib().or_srgb_channel(F(x), 1) for x in probe], F)
    assert np.max(np.abs(kernel_model(probe).view(np.int32) - o.view(np.int32))) <= 1


def test_pow_branch_edges(orc):
    below = np.array([-1.0, -0.0, 0.0, 1e-30, 0.001, np.nextafter(F(0.0031308), F(0)), -np.inf, np.nan], F)
    assert np.array_equal(oracle_bytes(orc, below, True), oracle_bytes(orc, below, False))
    assert list(oracle_bytes(orc, below[-2:], True)) == [0, 0]  # NaN -> 0 (cvttss2si)
    # saturated white: 1.055f * 1 - 0.055f = 0.99999994f, so the pow curve stores 254
    white = np.array([1.0, 2.0, np.inf], F)
    assert list(oracle_bytes(orc, white, True)) == [254] * 3 and list(oracle_bytes(orc, white, False)) == [255] * 3
    assert list(u8(kernel_model(white[:1]))) == [254]


def test_sqrt_mode_encode_equals_the_render_store(orc):
    o = orc.scene_builtin(1).prefix(16)
    W, H = 24, 16
    prev, cur, _ = orc.render(o, orc.camera(o, W, H), W, H, frames=3, max_bounce=4)
    assert np.array_equal(orc.encode_rgba8(prev), cur.reshape(-1))
    pw = orc.encode_rgba8(prev, srgb_pow=True)
    assert not np.array_equal(pw, cur.reshape(-1))  # the two curves do differ
    assert np.all(pw >> 24 == 255)
