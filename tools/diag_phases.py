"""Per-phase wave time of transport_kernel from a -DSMCRT_DIAG build (SMCRT_LIB=...): one
launch of N photons of a bench.py workload, then the s_memtime share of each phase and the
lane-state occupancy.
usage: SMCRT_LIB=tools/diag_libs/libsmcrt_diag.so python tools/diag_phases.py [N] [workload]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsmcrt_amd import abi, builders, scene  # noqa: E402
from rsmcrt_amd.engine import Engine, load_library  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
wl = sys.argv[2] if len(sys.argv) > 2 else "m1"
import bench  # noqa: E402
sc, g, src, dets, _, _ = bench.workload(wl, 0)
L = load_library()
L.smcrt_diag_read.argtypes = [C.POINTER(C.c_ulonglong)]
with Engine(sc, g, dets) as eng:
    eng.run(src, min(n, 300_000))
    buf = (C.c_ulonglong * 81)()
    L.smcrt_diag_read(buf)
    r = eng.run(src, n)
    L.smcrt_diag_read(buf)
t = list(buf[72:81])
names = ["-", "fetch", "EVAL", "P3", "P4", "DDA", "P5/P6", "P7 events", "P8+loop"]
tot = sum(t)
if not tot:
    sys.exit(0)  # the library printed its per-launch summary at each launch
for i in range(1, 9):
    print(f"{names[i]:10s} {100.0 * t[i] / tot:6.2f} %")
trips = buf[64]
print("trips", trips, "trips with a segment", buf[65], "trips with an EVAL", buf[66], "event rounds", buf[67])
print("waves", buf[70], "max wave iterations", buf[68], "mean", trips / max(1, buf[70]),
      "max wave ticks", buf[69], "mean", tot / max(1, buf[70]))
occ = sorted(((buf[c], c) for c in range(64) if buf[c]), reverse=True)
lanes = sum(o[0] for o in occ)
print("lane-slot classes (seg*32 + state):", [(c, round(100.0 * v / max(1, lanes), 2)) for v, c in occ[:12]])
print("counters", r.counters_dict(engine=True))
