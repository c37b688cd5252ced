"""Per-instruction response of the SQ VALU counters, from rocprofv3 --pmc runs
of scripts/mb_ops (one kernel per instruction, 8 independent chains, known
instruction count).  Prints, per kernel, every counter divided by the number of
wave-instructions the kernel issues (so 1.0 = the counter counts that
instruction once per wave; ACTIVE_INST_* are quad-cycles per wave-instruction).

usage: python scripts/pmc_calib.py gpurun_out <prefix>
"""
import collections
import csv
import glob
import sys

root, prefix = sys.argv[1:3]
BLOCKS, ITERS = 256 * 8 * 4, 4000
WAVE_INSTR = BLOCKS * 4 * ITERS * 8
val = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/{prefix}*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        val[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in val.values() for c in k})
for kern in sorted(val, key=lambda s: (len(s), s)):
    cs = val[kern]
    row = " ".join(f"{c.replace('SQ_INSTS_VALU_', 'V.').replace('SQ_', '')}={sum(v) / len(v) / WAVE_INSTR:.3f}"
                   for c, v in sorted(cs.items()) if c != "GRBM_GUI_ACTIVE")
    g = cs.get("GRBM_GUI_ACTIVE")
    cyc = f" cyc/wi/SIMD={sum(g) / len(g) / 8 * 1024 / WAVE_INSTR:.2f}" if g else ""
    print(f"{kern[:40]:40s}{cyc} {row}")
