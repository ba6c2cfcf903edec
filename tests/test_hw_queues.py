"""The package raises GPU_MAX_HW_QUEUES to at least 8 (rsmcrt_amd/__init__.py): the GPU boxes
export HIP's default of 4, with which two overlapped launch streams share a hardware queue."""
from rsmcrt_amd import _raise_hw_queues


def test_hw_queues_raised_when_unset_or_low():
    for before, after, logged in ((None, "8", False), ("4", "8", True), ("", "8", False), ("x", "8", True),
                                  ("8", "8", False), ("16", "16", False), ("64", "32", True), ("32", "32", False)):
        env = {} if before is None else {"GPU_MAX_HW_QUEUES": before}
        msgs = []
        assert _raise_hw_queues(env, log=msgs.append) == int(after)
        assert env["GPU_MAX_HW_QUEUES"] == after, (before, env)
        assert bool(msgs) == logged, (before, msgs)


def test_bench_imports_the_package_helper():
    """bench.py raises the queues through the package helper (clamped, logged), before torch."""
    src = open(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "bench.py")).read()
    head = src[:src.index("def log(")]
    assert "_raise_hw_queues" in head and "import torch" not in head
