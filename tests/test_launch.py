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
    assert "--gpus 64 asked for 64 GPUs but only" in out.stderr
    assert out.stdout.strip() == ""  # no JSON line


def test_bench_gpus_must_match_launcher_world():
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--no-cpu"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr, out
