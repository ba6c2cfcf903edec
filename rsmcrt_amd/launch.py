"""One process per GPU without an external launcher.

`python bench.py --gpus N` (no torchrun) must still measure N GPUs. The parent process never
initialises HIP: it counts the devices from the KFD topology in sysfs (or amdsmi), fails
loudly when fewer than N are visible or when neither can count them, then starts N copies of the
same command with the environment torch.distributed.run would give them (RANK, LOCAL_RANK,
WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and exits with the first
non-zero child status (0 when every rank succeeds). Children inherit stdout/stderr, so rank
0's JSON line is the parent's output.

The reference's equivalent is the OpenMP team of run_MCRT (kernelsMod.f90:1833-1861) plus
the intended MPI reduce (:2351-2357); here each rank is one GPU.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


class LaunchError(RuntimeError):
    pass


def under_launcher() -> bool:
    """True when a launcher (torch.distributed.run, mpirun wrapper, or this module) already
    set the rank environment."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _can_open(path: str) -> bool:
    try:
        fd = os.open(path, os.O_RDWR | os.O_CLOEXEC)
    except OSError:
        return False
    os.close(fd)
    return True


def _kfd_gpu_count():
    """GPU agents in the KFD topology (sysfs text files; nothing is opened under /dev), or
    None when the topology is not there. A node is a GPU when its simd_count is non-zero
    (CPU nodes report 0) and this process can open its render node /dev/dri/renderD<minor>
    read-write: a container sees the host's whole topology but only its own GPUs' render nodes,
    which is the filter the HSA runtime applies too. The node is opened and closed at once
    (os.access would check only the file mode, not the device cgroup's allow-list); opening a
    DRM render node starts neither HSA nor HIP."""
    try:
        nodes = os.listdir(KFD_NODES)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(KFD_NODES, d, "properties")) as f:
                props = dict(l.split(None, 1) for l in f.read().splitlines() if " " in l)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) <= 0:
            continue
        minor = props.get("drm_render_minor", "").strip()
        if minor and not _can_open(f"/dev/dri/renderD{minor}"):
            continue
        n += 1
    return n


def _amdsmi_gpu_count():
    """GPUs amdsmi reports (it reads the driver's device files, never the HSA runtime), or
    None when amdsmi is missing or fails."""
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        try:
            return len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:
        return None


def visible_gpus() -> int:
    """Visible GPUs, counted without initialising HIP or HSA in this process (a parent that did
    would hold the device while its ranks start, and on this pool must never exec afterwards):
    the KFD topology in sysfs, else amdsmi, capped by ROCR_/HIP_/CUDA_VISIBLE_DEVICES. Raises
    LaunchError when neither source answers (torch.cuda.device_count() is not used: it falls
    back to hipGetDeviceCount when amdsmi fails)."""
    n = _kfd_gpu_count()
    if n is None:
        n = _amdsmi_gpu_count()
    if n is None:
        raise LaunchError("cannot count GPUs: no KFD topology under /sys/class/kfd and no working amdsmi")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    return env


def spawn(world: int, argv, need_gpus: bool = True, timeout: float | None = None, env=None) -> int:
    """Run `argv` as `world` ranks on this node and wait for them. Returns the exit status
    (the first non-zero one; the other ranks are then terminated). Raises LaunchError when
    need_gpus and fewer than `world` GPUs are visible."""
    if world < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {world})")
    if need_gpus:
        n = visible_gpus()
        if n < world:
            raise LaunchError(f"--gpus {world} asked for {world} GPUs but only {n} "
                              f"{'is' if n == 1 else 'are'} visible on this node")
    port = free_port()
    procs = [subprocess.Popen(list(argv), env=rank_env(r, world, port, env), start_new_session=True)
             for r in range(world)]
    t0 = time.monotonic()
    status = 0
    live = set(range(world))
    try:
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and status == 0:
                    status = rc
                    print(f"[launch] rank {r} exited with status {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:  # (each rank leads its own process group)
                        try:
                            os.killpg(procs[q].pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            if timeout is not None and time.monotonic() - t0 > timeout:
                for q in live:
                    try:
                        os.killpg(procs[q].pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                for q in live:
                    procs[q].wait()
                raise LaunchError(f"ranks {sorted(live)} still running after {timeout} s")
            if live:
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.wait()
    if status < 0:  # killed by a signal: report it as a shell would
        status = 128 - status
    return status
