"""bench.py's own rank launcher (rsmcrt_amd/launch.py), CPU only: it starts one process per
rank with the torch.distributed.run environment, the ranks shard the photons as bench.py
does and reduce with one collective, and the sum equals one single-process run. Also: asking
for more GPUs than are visible fails loudly before any rank starts."""
import json
import os
import subprocess
import sys

import numpy as np

from rsmcrt_amd import abi, builders, scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS, BATCH, GRID = 2, 200, 20


def test_launcher_two_ranks_match_single_process(lib_path):
    from oracle import pyoracle as O
    code = ("import sys; from rsmcrt_amd import launch; "
            f"sys.exit(launch.spawn(2, [sys.executable, {os.path.join(ROOT, 'tests', 'launch_worker.py')!r}, "
            f"'{STEPS}', '{BATCH}', '{GRID}'], need_gpus=False, timeout=240))")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    got = json.loads(lines[0])
    assert got["n_ranks"] == 2
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(GRID, GRID, GRID, 1.0, 1.0, 1.0)
    ref = O.run(sc, g, scene.point_source(), STEPS * 2 * BATCH)
    assert got["counters"] == [int(c) for c in ref.counters]
    assert got["counters"][abi.CTR["photons"]] == STEPS * 2 * BATCH
    np.testing.assert_allclose(got["jmean_sum"], ref.jmean.sum(), rtol=1e-12)
    np.testing.assert_allclose(got["jmean_max"], ref.jmean.max(), rtol=1e-12)


def test_launcher_failing_rank_stops_the_job():
    code = ("import sys; from rsmcrt_amd import launch; "
            "sys.exit(launch.spawn(2, [sys.executable, '-c', "
            "'import os, sys, time; sys.exit(3) if os.environ[\"RANK\"] == \"1\" else time.sleep(60)'], "
            "need_gpus=False, timeout=50))")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.returncode == 3, (out.returncode, out.stderr)
    assert "rank 1 exited with status 3" in out.stderr


def test_bench_more_gpus_than_visible_fails_loudly():
    """`bench.py --gpus N` with fewer than N visible GPUs exits non-zero with a clear message
    (here no GPU is visible; on a 1-GPU box --gpus 2 takes the same path)."""
    import torch
    if torch.cuda.device_count() >= 64:
        return
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--no-cpu"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 2, out
    # (this container has no KFD topology and no GPU for amdsmi: the count itself fails loudly)
    assert "--gpus 64 asked for 64 GPUs but only" in out.stderr or "cannot count GPUs" in out.stderr, out.stderr
    assert out.stdout.strip() == ""  # no JSON line


def _fake_kfd(tmp_path, nodes):
    """A KFD topology: one directory per node with its properties file."""
    for i, (simd, minor) in enumerate(nodes):
        d = tmp_path / "nodes" / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndrm_render_minor {minor}\n")
    return str(tmp_path / "nodes")


def test_visible_gpus_from_kfd_topology(tmp_path, monkeypatch):
    """The launcher counts GPUs from sysfs text only: GPU nodes (simd_count > 0) whose render
    node this process may open, capped by the *_VISIBLE_DEVICES lists; no topology and no
    amdsmi is an error, never a silent 0 or a HIP call."""
    from rsmcrt_amd import launch
    monkeypatch.setattr(launch, "KFD_NODES", _fake_kfd(tmp_path, [(0, 0), (1216, 128), (1216, 136), (1216, 999)]))
    monkeypatch.setattr(launch, "_can_open", lambda path: not path.endswith("renderD999"))
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert launch.visible_gpus() == 2  # (the CPU node and the inaccessible GPU are not counted)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert launch.visible_gpus() == 1
    monkeypatch.setattr(launch, "KFD_NODES", str(tmp_path / "absent"))
    monkeypatch.setattr(launch, "_amdsmi_gpu_count", lambda: None)
    import pytest
    with pytest.raises(launch.LaunchError, match="cannot count GPUs"):
        launch.visible_gpus()


def test_launcher_parent_never_maps_kfd():
    """Counting GPUs in the launcher's parent opens nothing under /dev/kfd (the HSA runtime
    maps it when it starts): after visible_gpus() the process's memory map holds no kfd
    mapping and torch.cuda was never initialised. On a GPU box the count is also >= 1."""
    code = ("import sys; sys.path.insert(0, %r); from rsmcrt_amd import launch\n"
            "try:\n    n = launch.visible_gpus()\nexcept launch.LaunchError:\n    n = -1\n"
            "maps = open('/proc/self/maps').read()\n"
            "print(n, int('/dev/kfd' in maps), int('torch' in sys.modules))\n") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    n, kfd, torch_loaded = map(int, out.stdout.split())
    assert kfd == 0 and torch_loaded == 0, out.stdout
    if os.path.exists("/dev/kfd"):
        assert n >= 1, out.stdout


def test_bench_gpus_must_match_launcher_world():
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--no-cpu"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr, out


import pytest  # noqa: E402


@pytest.mark.gpu
def test_launcher_parent_never_maps_kfd_on_gpu_box():
    """The same check on the GPU box, where /dev/kfd exists and the count must be >= 1, and the
    launcher's count equals the GPUs this lease gives the process (HIP's count, taken in a
    separate process after the launcher's)."""
    assert os.path.exists("/dev/kfd")
    test_launcher_parent_never_maps_kfd()
    code = ("import sys; sys.path.insert(0, %r); from rsmcrt_amd import launch; print(launch.visible_gpus())" % ROOT)
    n = int(subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                           check=True).stdout.split()[-1])
    hip = int(subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                             capture_output=True, text=True, timeout=300, check=True).stdout.split()[-1])
    assert n == hip, (n, hip)


def test_bench_n_rank_cpu_leg_and_parity():
    """The CPU leg and parity of an N > 1 bench line (bench.sharded_cpu_parity), two gloo
    ranks through the launcher: the line carries cpu_baseline (value, unit, cores, kind,
    sample), parity over the same photons summed across the ranks (counters bit-exact, the
    jmean differences at rounding level) and the communicator's rank count."""
    code = ("import sys; from rsmcrt_amd import launch; "
            f"sys.exit(launch.spawn(2, [sys.executable, {os.path.join(ROOT, 'tests', 'bench_parity_worker.py')!r}], "
            "need_gpus=False, timeout=240))")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    cb, par = line["cpu_baseline"], line["parity"]
    assert cb["value"] > 0 and cb["unit"] == "photon packets/s" and cb["cores"] == 2 and cb["kind"] == "port"
    assert "photons [0," in cb["sample"]
    assert par["counters_bit_exact_vs_cpu"] is True and par["photons_compared"] > 0
    assert par["jmean_max_rel_diff_vs_cpu"] < 1e-12 and "2 ranks" in par["gpu_side"]
    assert line["rccl_ranks"] == 2
    # the per-rank breakdown (bench.rank_row / attach_rank_breakdown)
    rows, summ = line["ranks"], line["rank_summary"]
    assert [r["rank"] for r in rows] == [0, 1] and [r["photons"] for r in rows] == [200, 400]
    assert all(r["seconds"] >= r["transport_s"] > 0 and r["reduce_ms"] >= 0 for r in rows)
    assert summ["photons_total"] == 600 and summ["slowest_rank"] in (0, 1)
    assert summ["transport_s_max"] >= summ["transport_s_min"] > 0 and summ["transport_imbalance"] >= 0
    assert summ["reduce_ms_max"] == max(r["reduce_ms"] for r in rows) and 0 <= summ["reduce_share_of_step_time"] < 1
