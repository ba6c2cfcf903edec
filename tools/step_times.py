"""Per-step timing of a bench.py workload (diagnostic): each step is synchronised and its
transport/fold event times and launch count printed.
usage: python tools/step_times.py WORKLOAD BATCH STEPS"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from rsmcrt_amd import abi  # noqa: E402
from rsmcrt_amd.engine import Engine  # noqa: E402

wl, B, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
torch.cuda.set_device(0)
sc, g, src, dets, _, _ = bench.workload(wl, 0)
eng = Engine(sc, g, dets)
nv = g.nx * g.ny * g.nz
dev = torch.device("cuda", 0)
jm, ab = torch.zeros(nv, dtype=torch.float64, device=dev), torch.zeros(nv, dtype=torch.float64, device=dev)
ns, ctr = torch.zeros(1, dtype=torch.float64, device=dev), torch.zeros(abi.NCOUNTERS, dtype=torch.int64, device=dev)
db = torch.zeros(4096, dtype=torch.float64, device=dev)
t = abi.DeviceTallies()
t.jmean, t.absorb, t.nscatt, t.counters = jm.data_ptr(), ab.data_ptr(), ns.data_ptr(), ctr.data_ptr()
if dets:
    t.det_bins = db.data_ptr()
st = torch.cuda.current_stream()
eng.set_timing(True)
for k in range(K):
    t0 = time.perf_counter()
    eng.run_device(src, Engine.config(B, first_photon=k * B, flags=abi.FLAG_PATHLENGTH), t, st.cuda_stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kt = eng.kernel_times()
    print(f"step {k}: {dt * 1e3:.1f} ms wall, {kt['launches']} launches, transport {kt['transport_ms']:.1f} ms, "
          f"fold {kt['deposit_ms']:.1f} ms", flush=True)
eng.close()
