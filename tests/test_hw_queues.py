"""The package raises GPU_MAX_HW_QUEUES to at least 8 (rsmcrt_amd/__init__.py): the GPU boxes
export HIP's default of 4, with which two overlapped launch streams share a hardware queue."""
from rsmcrt_amd import _raise_hw_queues


def test_hw_queues_raised_when_unset_or_low():
    for before, after in ((None, "8"), ("4", "8"), ("", "8"), ("x", "8"), ("8", "8"), ("16", "16")):
        env = {} if before is None else {"GPU_MAX_HW_QUEUES": before}
        _raise_hw_queues(env)
        assert env["GPU_MAX_HW_QUEUES"] == after, (before, env)
