#!/usr/bin/env python3
"""Static ISA breakdown of ws_kernel<F, G> (or transport_kernel) by region (no GPU needed).

Compiles rsmcrt_amd/csrc/kinst.hip for one (LDS faces, grid mode) slice (the part that holds the
kernel, with build.py's flags for it) with
-DSMCRT_ASM_MARKERS, which turns ws.h's WS_MARK(i) region starts into `; @@LPHASE i` comments
in the device assembly, takes the kernel's body and counts its instructions per region and
class (ws.h: 1 photon waves, 2 event waves, 10-15 the walker waves: setup, claim + take,
crossing step, record emit, finish, exit; 16 the counters flush). Static counts: what the code holds,
not how often it runs (DESIGN.md §4.3b has the dynamic shares).

usage: isa_phases.py [--kernel ws|wsx|transport] [--f 1] [--g 2] [extra hipcc flags...]
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ws_kernel (ws.h WS_MARK): the walker loop's regions
WS_NAMES = {0: "prologue", 1: "photon", 2: "event", 10: "w:setup", 11: "w:claim+take", 12: "w:dda", 13: "w:emit",
            14: "w:finish", 15: "w:exit", 16: "epilogue"}


def classify(op):
    if op.startswith("v_"):
        if re.search(r"_f64", op):
            if re.search(r"v_(rcp|rsq|sqrt|div_scale|div_fmas|div_fixup|frexp|ldexp|trig|fract|floor|ceil|rndne|trunc)", op):
                return "valu_f64_other"
            return "valu_f64_arith"
        if re.search(r"_(u64|i64|b64)", op) or op.startswith(("v_lshl_add_u64", "v_mad_u64", "v_mad_i64")):
            return "valu_64bit_int"
        if op.startswith("v_cndmask"):
            return "valu_cndmask"
        if op.startswith(("v_cmp", "v_cmpx")):
            return "valu_cmp"
        if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            return "valu_lane_xfer"
        if op.startswith(("v_mov", "v_accvgpr")):
            return "valu_mov"
        return "valu_32bit_other"
    if op.startswith("s_"):
        if op.startswith("s_waitcnt"):
            return "s_waitcnt"
        if op.startswith(("s_cbranch", "s_branch")):
            return "salu_branch"
        if op.startswith(("s_load", "s_buffer_load")):
            return "smem_load"
        return "salu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main(argv):
    kern, f, g, extra = "ws", "1", "2", []
    i = 0
    while i < len(argv):
        if argv[i] in ("--kernel", "--f", "--g"):
            val = argv[i + 1]
            if argv[i] == "--kernel":
                kern = val
            elif argv[i] == "--f":
                f = val
            else:
                g = val
            i += 2
        else:
            extra.append(argv[i])
            i += 1
    out = f"/tmp/isa_phases_{f}{g}.s"
    # the plain ws_kernel lives in kinst.hip's part 1 with build.py's flags for it
    sys.path.insert(0, ROOT)
    from rsmcrt_amd.build import PLAIN_WS_FLAGS
    part = ["-DKI_P=1", *PLAIN_WS_FLAGS] if kern == "ws" else ["-DKI_P=0"]
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                    "--offload-arch=gfx950", "--cuda-device-only", "-S", f"-DKI_F={f}", f"-DKI_G={g}", *part,
                    "-DSMCRT_ASM_MARKERS", "-o", out, os.path.join(ROOT, "rsmcrt_amd", "csrc", "kinst.hip")] + extra,
                   check=True, cwd="/tmp", stderr=subprocess.DEVNULL)
    s = open(out).read()
    pat = r"^(_ZN5smcrt9ws_kernelILb\d+ELi\d+ELb" + ("1" if kern == "wsx" else "0") + r"E\w+):" if kern.startswith("ws") else r"^(_Z16transport_kernel\w+):"
    m = re.search(pat, s, re.M)
    start = m.start()
    end = s.index(".Lfunc_end", start)
    body = s[start:end].splitlines()
    meta = re.search(re.escape(m.group(1)) + r"\.num_vgpr, (\d+)", s)
    scratch = re.search(r"; ScratchSize: (\d+)", s[end:])
    phase = 0
    per = collections.defaultdict(collections.Counter)
    for line in body:
        t = line.strip()
        mk = re.match(r"; @@LPHASE (\d+)", t)
        if mk:
            i = int(mk.group(1))
            phase = i  # region i starts at marker i
            continue
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        per[phase][classify(t.split()[0])] += 1
    classes = ["valu_f64_arith", "valu_f64_other", "valu_64bit_int", "valu_32bit_other", "valu_cmp", "valu_cndmask",
               "valu_mov", "valu_lane_xfer", "salu_other", "salu_branch", "s_waitcnt", "smem_load", "lds", "vmem",
               "other"]
    print(f"# {m.group(1)}: {meta.group(1) if meta else '?'} VGPRs, scratch {scratch.group(1) if scratch else '?'} B")
    print("phase".ljust(10) + "".join(c.replace("valu_", "v.").replace("salu_", "s.").rjust(12) for c in classes)
          + "total".rjust(8))
    tot = collections.Counter()
    for p in sorted(per):
        c = per[p]
        tot.update(c)
        print((WS_NAMES if kern.startswith("ws") else {}).get(p, str(p)).ljust(10) + "".join(str(c[k]).rjust(12) for k in classes) + str(sum(c.values())).rjust(8))
    print("all".ljust(10) + "".join(str(tot[k]).rjust(12) for k in classes) + str(sum(tot.values())).rjust(8))


if __name__ == "__main__":
    main(sys.argv[1:])
