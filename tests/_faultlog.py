"""Progress lines on the file descriptor pytest's faulthandler dumps to.

pytest captures fd 2 per test (``-q``, no ``-s``), and a process that aborts (a GPU memory
fault: HSA prints the fault and calls ``abort()``) loses the captured text.  The faulthandler
plugin keeps a dup of the ORIGINAL stderr for its crash dump; lines written there survive an
abort and land right above the dump in the driver's ``pytest.log``, so an abort names its test
and the phase inside it (``tests/conftest.py`` writes the node id, ``tests/test_zoo.py`` the
phase).
"""
import os

_CONFIG = [None]


def bind(config) -> None:
    _CONFIG[0] = config


def _fd():
    config = _CONFIG[0]
    if config is None:
        return None
    try:
        from _pytest.faulthandler import fault_handler_stderr_fd_key
    except ImportError:  # pragma: no cover - older pytest
        return None
    return config.stash.get(fault_handler_stderr_fd_key, None)


def write(text: str) -> None:
    fd = _fd()
    if fd is None:
        return
    try:
        os.write(fd, f"[rtseg] {text}\n".encode())
    except OSError:
        pass
