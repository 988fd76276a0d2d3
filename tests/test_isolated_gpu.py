"""GPU checks that run in child processes (tests/isolated/*_check.py):

* graph capture around whole training steps (SegTrainer.graph_step, the graph-captured KD
  teacher), so capture / MIOpen / graph-pool state never carries over into the rest of the suite;
* the whole-zoo checks of tests/test_zoo.py (fp32 HIP vs torch vs fp64, bf16 train step): after
  ~800 GPU tests in one process, the fp32 zoo check faulted with an illegal address on a
  different model each time (LEDNet, RegSeg, LiteSeg) while the same checks pass in a fresh
  process -- an allocator-layout-dependent fault not localised yet (profiles/r2_verify/README.md);
  a fresh process per check group is also how a training job runs.

Reference: core/seg_trainer.py:38-119 (train step), models/* (the zoo)."""
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


def _zoo_chunks(n=4):
    sys.path.insert(0, HERE)
    from test_zoo import KEYS

    return [",".join(KEYS[i::n]) for i in range(n)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("models", _zoo_chunks())
def test_zoo_in_child_process(models):
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "isolated", "zoo_gpu_check.py")],
                       capture_output=True, text=True, timeout=850, env=dict(os.environ, ZOO_ONLY=models))
    assert r.returncode == 0, r.stdout[-6000:] + r.stderr[-3000:]
    assert "zoo checks done: 0 failed" in r.stdout
