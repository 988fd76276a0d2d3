"""MI355X-native real-time semantic segmentation (PyTorch-ROCm + HIP/CDNA4 kernels + RCCL).

Importing the package points ``MIOPEN_USER_DB_PATH`` at the in-tree ``miopen_db/`` find
database (gfx950 solver choices for the zoo's shapes), so a fresh machine reuses them (an
explicit environment value wins).

MIOpen's "naive" direct-convolution solvers stay enabled here: they are the fallback for
degenerate geometries -- e.g. CFPNet's (3, 1) convs with dilation 16 on a 16-row map, where
the remaining NHWC bf16 solvers return non-finite outputs or fault.  ``bench.py`` and
``tools/test_speed.py`` (DDRNet-style shapes at 1024x2048, where the naive solvers only
slow MIOpen's find) exclude them for their own process.
"""
import os as _os

_db = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "miopen_db")
if _os.path.isdir(_db):
    _os.environ.setdefault("MIOPEN_USER_DB_PATH", _db)
