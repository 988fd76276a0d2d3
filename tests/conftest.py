import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # under pytest-xdist every worker would start one intra-op thread per CPU: share them instead
    workers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1") or 1)
    if workers > 1:
        import torch

        torch.set_num_threads(max(1, (os.cpu_count() or 1) // workers))
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "no_guard: cannot run under the guard-page allocator (graph capture)")
    # RTSEG_GUARD=tail|head: every device tensor borders an unmapped guard page, so any
    # out-of-bounds kernel access faults deterministically (utils/guard.py)
    mode = os.environ.get("RTSEG_GUARD")
    if mode:
        import torch

        if torch.cuda.is_available():
            from realtime_semantic_segmentation_pytorch_amd.utils import guard

            guard.install(mode)


def pytest_sessionstart(session):
    import _faultlog

    _faultlog.bind(session.config)


def pytest_runtest_logstart(nodeid, location):
    # GPU runs only: a test that aborts the process is named above the faulthandler dump
    import torch

    if torch.cuda.is_available():
        import _faultlog

        _faultlog.write(f"start {nodeid}")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        if os.environ.get("RTSEG_GUARD"):
            skip = pytest.mark.skip(reason="graph capture / child processes: not under the guard allocator")
            for item in items:
                if "no_guard" in item.keywords:
                    item.add_marker(skip)
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _isolate_miopen_find_mode():
    """A trainer built by one test turns MIOpen find mode on for the process (utils/runtime.py);
    it must not leak into later tests, whose models may have geometries find mode is not
    verified on (LEDNet / CFPNet degenerate dilated convs)."""
    import torch

    saved = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = False
    yield
    torch.backends.cudnn.benchmark = saved
