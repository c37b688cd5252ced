"""Basic-block instruction mix of one kernel in a hipcc -S listing.

usage: python scripts/asm_blocks.py /tmp/k.s <kernel-symbol-substring> [min_instrs] [label-to-dump]
Prints, per block: label, line, VALU (of which packed / transcendental),
SALU, branches, LDS, SMEM, and the loop comment hipcc attaches.
"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
min_n = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dump = sys.argv[4] if len(sys.argv) > 4 else None
text = open(path).read()
start = None
for m in re.finditer(r"^(\S+):\s*(;.*)?$", text, flags=re.M):
    if sym in m.group(1) and not m.group(1).startswith("."):
        start = m.end()
        break
end = text.index(".Lfunc_end", start)
lines = text[start:end].splitlines()
blocks, cur = [], {"label": "entry", "line": 0, "note": "", "ins": []}
for i, l in enumerate(lines):
    m = re.match(r"^(\.LBB\S+):\s*(;.*)?$", l)
    if m:
        blocks.append(cur)
        cur = {"label": m.group(1), "line": i, "note": (m.group(2) or "").strip("; "), "ins": []}
        continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur["ins"].append(s.split()[0])
    cur.setdefault("text", []).append(s)
blocks.append(cur)
trans = ("v_sqrt", "v_rcp", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32")
tot = {}
for b in blocks:
    ins = b["ins"]
    c = {
        "valu": sum(1 for x in ins if x.startswith("v_")),
        "pk": sum(1 for x in ins if x.startswith("v_pk_")),
        "trans": sum(1 for x in ins if x.startswith(trans)),
        "salu": sum(1 for x in ins if x.startswith("s_") and not x.startswith(("s_cbranch", "s_branch", "s_load", "s_waitcnt", "s_nop", "s_memtime"))),
        "br": sum(1 for x in ins if x.startswith(("s_cbranch", "s_branch"))),
        "lds": sum(1 for x in ins if x.startswith("ds_")),
        "smem": sum(1 for x in ins if x.startswith("s_load")),
        "nop": sum(1 for x in ins if x.startswith("s_nop")),
        "wait": sum(1 for x in ins if x.startswith("s_waitcnt")),
    }
    for k, v in c.items():
        tot[k] = tot.get(k, 0) + v
    if len(ins) >= min_n:
        print(f"{b['label']:>12s} L{b['line']:<5d} n={len(ins):4d} valu={c['valu']:3d} pk={c['pk']:3d} tr={c['trans']:2d} "
              f"salu={c['salu']:3d} br={c['br']:2d} lds={c['lds']:2d} smem={c['smem']:2d} nop={c['nop']:2d} wait={c['wait']:2d}  {b['note'][:60]}")
print("TOTAL", tot)
if dump:
    for b in blocks:
        if b["label"] == dump:
            print("\n".join(b.get("text", [])))
