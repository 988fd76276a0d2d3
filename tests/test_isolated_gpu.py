"""GPU checks that run in child processes (tests/isolated/*_check.py):

* graph capture around whole training steps (SegTrainer.graph_step, the graph-captured KD
  teacher), so capture / MIOpen / graph-pool state never carries over into the rest of the suite;
* the whole-zoo checks of tests/test_zoo.py under the guard-page allocator (a pluggable
  allocator must be installed before the process's first CUDA allocation).

Reference: core/seg_trainer.py:38-119 (train step), models/* (the zoo)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.timeout(600)
@pytest.mark.no_guard
@pytest.mark.parametrize("script", ["graph_step_check.py", "kd_teacher_check.py"])
def test_isolated(script):
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "isolated", script)], capture_output=True,
                       text=True, timeout=560)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    assert ": ok" in r.stdout


@pytest.mark.timeout(1200)
@pytest.mark.no_guard
def test_zoo_under_guard_page_allocator():
    """Every zoo model's fp32 and bf16 HIP training checks with every device tensor placed
    against an unmapped guard page (utils/guard.py, csrc/tools/guard_alloc.cpp): an
    out-of-bounds read or write of any kernel faults on its first launch, independent of what
    the caching allocator happens to place next to the tensor -- the deterministic form of the
    round-2 intermittent illegal-address fault (profiles/r3_fault/README.md).  Fresh memory is
    NaN-filled, so a kernel that consumes memory it never wrote fails the numerics checks."""
    env = dict(os.environ, RTSEG_GUARD="tail", RTSEG_GUARD_FILL="nan")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "isolated", "zoo_gpu_check.py")],
                       capture_output=True, text=True, timeout=1150, env=env)
    assert r.returncode == 0, r.stdout[-6000:] + r.stderr[-3000:]
    assert "zoo checks done: 0 failed" in r.stdout
