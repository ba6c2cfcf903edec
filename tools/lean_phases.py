#!/usr/bin/env python3
"""Static instruction mix per phase of lean_kernel<LDS_FACES, GM> from a device asm built with
-DSMCRT_ASM_MARKERS (hipcc --cuda-device-only -S). No GPU needed.
usage: lean_phases.py file.s [ILb1ELi2E]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
inst = sys.argv[2] if len(sys.argv) > 2 else "ILb1ELi2E"
m = re.search(r"^(_ZN5smcrt11lean_kernel" + inst + r"\w+):", s, re.M)
start = m.start()
end = s.index(".Lfunc_end", start)
phase = "pre"
stats = collections.defaultdict(collections.Counter)
for l in s[start:end].splitlines():
    l = l.strip()
    mm = re.search(r"@@(LPHASE \d+|DDA_BEGIN|DDA_END)", l)
    if mm:
        tag = mm.group(1)
        phase = {"DDA_BEGIN": "dda", "DDA_END": "post-dda"}.get(tag, tag)
        continue
    if not l or l.startswith((".", ";", "_")) or l.endswith(":"):
        continue
    op = l.split()[0]
    stats[phase][op] += 1


def cls(op):
    if op.startswith("v_"):
        if "f64" in op or "_b64" in op or "u64" in op or "i64" in op:
            return "v64"
        return "v32"
    if op.startswith("s_"):
        return "s"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


for ph, c in stats.items():
    agg = collections.Counter()
    for op, n in c.items():
        agg[cls(op)] += n
    print(f"== {ph}: total {sum(c.values())} " + " ".join(f"{k}={v}" for k, v in sorted(agg.items())))
    if "-v" in sys.argv:
        for op, n in c.most_common(25):
            print(f"   {op} {n}")
