"""MI355X-native real-time semantic segmentation (PyTorch-ROCm + HIP/CDNA4 kernels + RCCL).

Importing the package sets two MIOpen defaults before any convolution runs (an explicit
environment value always wins):

* the reference "naive" direct-convolution solvers are excluded from MIOpen's find -- with
  ``cudnn.benchmark`` they are timed too and take ~15 ms per call at 1024x2048, never win,
  and turned a 30 s warm-up into minutes;
* ``MIOPEN_USER_DB_PATH`` points at the in-tree ``miopen_db/`` find database (gfx950 solver
  choices for the zoo's shapes), so a fresh machine reuses them.
"""
import os as _os

for _k in ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
           "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW"):
    _os.environ.setdefault(_k, "0")
_db = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "miopen_db")
if _os.path.isdir(_db):
    _os.environ.setdefault("MIOPEN_USER_DB_PATH", _db)
