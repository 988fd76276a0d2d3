"""Host-side AddressSanitizer + UBSan run over the HIP kernels' launch planners (tile / slab /
workspace sizing, FastDiv magic numbers) -- tools/sanitize/run.sh builds the kernel sources
host-only (no device code, no GPU) with ``-Xarch_host -fsanitize=...`` and runs the checks."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_planners_clean_under_asan_ubsan(tmp_path):
    if shutil.which("bash") is None:
        pytest.skip("needs bash")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "run.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host planning checks passed" in r.stdout
