"""Per-photon completion profile of one launch (is a workload bound by its
bulk or by its last photons?). Needs the diagnostic library (tools/variants.sh diag
"-DSMCRT_DIAG"), which records each photon's completion time (s_memrealtime) when
SMCRT_DIAG_DONE=1.

usage: SMCRT_LIB=tools/diag_libs/libsmcrt_diag.so SMCRT_DIAG_DONE=1 \
           python tools/tail_profile.py WORKLOAD N OUT.json
Prints and writes: the launch's duration (HIP events), the completion-time quantiles, the
share of the launch after 99 / 99.9 / 99.99 % of the photons were done, the bulk rate (photons
completed between the 1 % and 99 % marks per second) and the SDF evaluations per second over the
launch, plus a 200-bin histogram of completion times.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsmcrt_amd.engine import Engine, load_library  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "m2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25_600_000
out_path = sys.argv[3] if len(sys.argv) > 3 else f"gpurun_out/tail_{wl}.json"
import bench  # noqa: E402

sc, g, src, dets, _, _ = bench.workload(wl, 0)
L = load_library()
L.smcrt_diag_done_times.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_uint64, C.POINTER(C.c_int32)]
with Engine(sc, g, dets) as eng:
    eng.run(src, min(n, 1 << 18))  # (the scene's calibration launch, first)
    eng.set_timing(True)
    eng.kernel_times()
    r = eng.run(src, n, first_photon=1 << 40)
    kt = eng.kernel_times()
    t = np.zeros(n, dtype=np.uint64)
    khz = C.c_int32()
    st = L.smcrt_diag_done_times(eng._h, t.ctypes.data_as(C.POINTER(C.c_ulonglong)), n, C.byref(khz))
    assert st == 0, st
slow = np.argsort(t)[-64:][::-1]  # the 64 last photons (indices from first_photon = 2^40)
done = t[t > 0].astype(np.float64)
assert done.size == n, (done.size, n)
ms = (done - done.min()) / khz.value  # ms after the first completion
ms.sort()
q = {f"{p}": float(np.percentile(ms, p)) for p in (1, 10, 50, 90, 99, 99.9, 99.99, 100)}
span = ms[-1]
launch_ms = kt["transport_ms"]
bulk = (0.98 * n) / max(1e-9, (q["99"] - q["1"]) * 1e-3)
cd = r.counters_dict(engine=True)
res = {
    "workload": wl, "photons": n, "launches": kt["launches"], "transport_ms": launch_ms,
    "completion_span_ms": span, "quantiles_ms": q,
    "share_after": {f"{p}%": (span - q[str(p)]) / span for p in (99, 99.9, 99.99)},
    "bulk_photons_per_s": bulk, "photons_per_s_launch": n / (launch_ms * 1e-3),
    "sdf_evals_per_s": cd["sdf_evals"] / (launch_ms * 1e-3), "sdf_evals_per_photon": cd["sdf_evals"] / n,
    "far_steps": kt.get("far_steps"),
    "slowest_photons": [int(i) + (1 << 40) for i in slow],
    "slowest_ms": [float((t[i] - t[t > 0].min()) / khz.value) for i in slow],
    "hist_ms": np.histogram(ms, bins=200)[0].tolist(), "hist_edges_ms": [0.0, float(span)],
}
print(json.dumps({k: v for k, v in res.items() if not k.startswith("hist") and not k.startswith("slowest")}, indent=1))
print("slowest photons (index, ms):", list(zip(res["slowest_photons"][:8], [round(x, 2) for x in res["slowest_ms"][:8]])))
os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
with open(out_path, "w") as f:
    json.dump(res, f)
