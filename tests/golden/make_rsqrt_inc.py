"""Regenerates simd-ray-tracer_amd/csrc/rsqrt_table_intel.inc (the library's
built-in rsqrtss table) from the captured fixture rsqrt_lut_intel.bin."""
import pathlib

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]


def render() -> str:
    lut = np.fromfile(ROOT / "tests/golden/rsqrt_lut_intel.bin", dtype=np.uint32)
    assert lut.size == 2048
    lines = [
        "// Generated from tests/golden/rsqrt_lut_intel.bin by tests/golden/make_rsqrt_inc.py — do not edit.",
        "// x86 rsqrtss results captured on an Intel host: [parity*1024 + top10(mantissa)], see DESIGN.md.",
        "static const uint32_t kRsqrtTableIntelBits[2048] = {",
    ]
    for i in range(0, 2048, 8):
        lines.append("    " + ", ".join(f"0x{v:08x}u" for v in lut[i:i + 8]) + ",")
    lines.append("};")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    (ROOT / "simd-ray-tracer_amd/csrc/rsqrt_table_intel.inc").write_text(render())
