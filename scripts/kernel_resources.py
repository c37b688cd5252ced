"""Per-kernel VGPR / SGPR / spill / LDS / occupancy of a HIP source's gfx950
build, from the compiler's kernel-resource-usage remarks, optionally diffed
against another source (e.g. an A/B copy of rt_kernel.hip).

usage: python scripts/kernel_resources.py <src.hip> [name filter] [--diff other.hip] [--flags "-DX=1"]
"""
import re
import subprocess
import sys

HIPCC = "/opt/rocm/bin/hipcc"
BASE = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-Iinclude",
        "-Isimd-ray-tracer_amd/csrc", "-fno-slp-vectorize", "--offload-device-only", "-c", "-o", "/dev/null",
        "-Rpass-analysis=kernel-resource-usage"]


def resources(src, flags):
    err = subprocess.run([HIPCC, *BASE, *flags, src], capture_output=True, text=True).stderr
    out, cur = {}, None
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark: .*?(VGPRs|SGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)",
                      line)
        if m and cur:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def fmt(v):
    return (f"v{v.get('VGPRs', -1):4d} s{v.get('SGPRs', -1):4d} vsp{v.get('VGPRs Spill', -1):3d} "
            f"ssp{v.get('SGPRs Spill', -1):3d} lds{v.get('LDS Size [bytes/block]', -1):6d} "
            f"occ{v.get('Occupancy [waves/SIMD]', -1):2d}")


def main():
    argv = sys.argv[1:]
    flags = argv[argv.index("--flags") + 1].split() if "--flags" in argv else []
    other = argv[argv.index("--diff") + 1] if "--diff" in argv else None
    pos = [a for i, a in enumerate(argv) if not a.startswith("--") and (i == 0 or argv[i - 1] not in ("--flags", "--diff"))]
    src, filt = pos[0], (pos[1] if len(pos) > 1 else "")
    r = resources(src, flags)
    o = resources(other, flags) if other else {}
    for name in sorted(r):
        if filt not in name:
            continue
        line = f"{name[:88]:88s} {fmt(r[name])}"
        if other:
            if name not in o:
                line += "   (new)"
            elif o[name] != r[name]:
                line += f"   was {fmt(o[name])}"
            else:
                continue
        print(line)


if __name__ == "__main__":
    main()
