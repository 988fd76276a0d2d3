"""GPU checks that run in child processes (tests/isolated/*_check.py):

* graph capture around whole training steps (SegTrainer.graph_step, the graph-captured KD
  teacher), so capture / MIOpen / graph-pool state never carries over into the rest of the suite;

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
