"""Per-kernel register/spill/occupancy summary of rt_kernel.hip.
Usage: python scripts/kres.py [extra hipcc flags]"""
import pathlib
import re
import subprocess
import sys

pkg = pathlib.Path(__file__).resolve().parents[1] / "simd-ray-tracer_amd"
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
       "-I../include", *sys.argv[1:], "-c", "csrc/rt_kernel.hip", "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, cwd=pkg, capture_output=True, text=True)
cur, rows = None, {}
for l in out.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+):\s*(\d+)", l)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
if out.returncode:
    print(out.stderr[-3000:])
for k, v in rows.items():
    g = v.get
    print(f"{k[-40:]:40s} V={g('VGPRs')} S={g('SGPRs')} Vsp={g('VGPRs Spill')} Ssp={g('SGPRs Spill')} "
          f"occ={g('Occupancy [waves/SIMD]')} lds={g('LDS Size [bytes/block]')}")
