"""GPU checks that capture HIP graphs around whole training steps (SegTrainer.graph_step, the
graph-captured KD teacher) run in a child process: graph capture, MIOpen's find / module state
and the caching allocator's graph pools then never carry over into the rest of the GPU suite
(tests/isolated/*_check.py hold the checks; reference core/seg_trainer.py:38-119)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("script", ["graph_step_check.py", "kd_teacher_check.py"])
def test_isolated(script):
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "isolated", script)], capture_output=True,
                       text=True, timeout=560)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    assert ": ok" in r.stdout
