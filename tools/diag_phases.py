"""Per-phase wave time of transport_kernel from a -DSMCRT_DIAG build (SMCRT_LIB=...): one M1
launch of N photons, then the s_memtime share of each phase and the lane-state occupancy.
usage: SMCRT_LIB=tools/diag_libs/libsmcrt_diag.so python tools/diag_phases.py [N]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsmcrt_amd import abi, builders, scene  # noqa: E402
from rsmcrt_amd.engine import Engine, load_library  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
L = load_library()
L.smcrt_diag_read.argtypes = [C.POINTER(C.c_ulonglong)]
with Engine(builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0), scene.grid(128, 128, 128, 1, 1, 1)) as eng:
    eng.run(scene.point_source(), 300_000)
    buf = (C.c_ulonglong * 81)()
    L.smcrt_diag_read(buf)
    r = eng.run(scene.point_source(), n)
    L.smcrt_diag_read(buf)
t = list(buf[72:81])
names = ["-", "fetch", "EVAL", "P3", "P4", "DDA", "P5/P6", "P7 events", "P8+loop"]
tot = sum(t)
for i in range(1, 9):
    print(f"{names[i]:10s} {100.0 * t[i] / tot:6.2f} %")
trips = buf[64]
print("trips", trips, "trips with a segment", buf[65], "trips with an EVAL", buf[66], "event rounds", buf[67])
print("counters", r.counters_dict(engine=True))
