"""In-tree build of the rtseg HIP extension for MI355X (gfx950).

The extension is one shared library, ``_C/librtseg_hip.so``, loaded with
``torch.ops.load_library`` and exposing ``torch.ops.rtseg.*``.  It is built by
driving ``hipcc`` directly (no hipify, no CUDA sources):

* ``csrc/kernels/*.hip`` -- the device kernels; they include only
  ``rtseg_common.h`` / ``rtseg_launch.h`` and compile in seconds each;
* ``csrc/binding*.cpp``  -- torch.library registrations (torch headers);
* everything is linked against the torch/ROCm libraries that ship with the
  installed PyTorch, so the same HIP runtime instance is shared with torch.

Objects are cached by content hash of (source, headers, flags), so rebuilding
after editing one kernel recompiles only that kernel.  ``python -m
realtime_semantic_segmentation_pytorch_amd.ops.build`` builds from the shell.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(CSRC, "build")
LIB_DIR = os.path.join(PKG_DIR, "_C")
LIB_PATH = os.path.join(LIB_DIR, "librtseg_hip.so")
GUARD_LIB_PATH = os.path.join(LIB_DIR, "librtseg_guard.so")
ARCH = os.environ.get("RTSEG_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    path = os.path.join(rocm, "bin", "hipcc")
    if not os.path.exists(path):
        raise RuntimeError(f"hipcc not found at {path}; the rtseg HIP extension needs ROCm")
    return path


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "include", "*.h")))


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _kernel_flags():
    return [
        "-c", "-fPIC", "-O3", "-std=c++20", f"--offload-arch={ARCH}", "-mcode-object-version=5",
        "-ffp-contract=fast", "-munsafe-fp-atomics", "-Wno-unused-result",
        "-I", os.path.join(CSRC, "include"),
    ]


def _binding_flags():
    inc, _, abi = _torch_paths()
    flags = [
        "-c", "-fPIC", "-O2", "-std=c++17", "-x", "c++",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-parameter", "-Wno-deprecated-declarations",
        "-I", os.path.join(CSRC, "include"), "-I", "/opt/rocm/include",
    ]
    for p in inc:
        flags += ["-isystem", p]
    py_inc = sysconfig.get_paths()["include"]
    flags += ["-isystem", py_inc]
    return flags


def _compile(cmd_prefix, src, flags, out_o, verbose):
    cmd = [cmd_prefix] + flags + ["-o", out_o, src]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return out_o


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> str:
    """Compile every kernel + binding and link ``librtseg_hip.so``. Returns its path."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = _hipcc()
    hdrs = _headers()
    kflags = _kernel_flags()
    bflags = _binding_flags()
    tasks = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        tag = _digest([src] + hdrs, kflags)
        out = os.path.join(BUILD_DIR, os.path.basename(src) + f".{tag}.o")
        tasks.append((hipcc, src, kflags, out))
    gxx = os.environ.get("CXX", "g++")
    for src in sorted(glob.glob(os.path.join(CSRC, "binding*.cpp"))):
        tag = _digest([src] + hdrs, bflags)
        out = os.path.join(BUILD_DIR, os.path.basename(src) + f".{tag}.o")
        tasks.append((gxx, src, bflags, out))

    todo = [t for t in tasks if force or not os.path.exists(t[3])]
    if jobs is None:
        jobs = int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 1)))
        jobs = max(1, min(jobs, 16))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, c, s, f, o, verbose) for (c, s, f, o) in todo]
            for fu in futs:
                fu.result()
    objs = [t[3] for t in tasks]
    link_tag = _digest(objs, [ARCH])
    stamp = LIB_PATH + ".stamp"
    if not force and os.path.exists(LIB_PATH) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == link_tag:
                return LIB_PATH
    _, tlib, _ = _torch_paths()
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
        "-L", tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
        f"-Wl,-rpath,{tlib}",
    ]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    with open(stamp, "w") as f:
        f.write(link_tag)
    # drop stale objects from previous source versions
    keep = set(objs)
    for o in glob.glob(os.path.join(BUILD_DIR, "*.o")):
        if o not in keep:
            try:
                os.remove(o)
            except OSError:
                pass
    return LIB_PATH


def build_guard(verbose: bool = False) -> str:
    """Build ``_C/librtseg_guard.so``: the guard-page debugging allocator
    (``csrc/tools/guard_alloc.cpp``, host code over the HIP virtual-memory API)."""
    os.makedirs(LIB_DIR, exist_ok=True)
    src = os.path.join(CSRC, "tools", "guard_alloc.cpp")
    flags = ["-shared", "-fPIC", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-I", "/opt/rocm/include"]
    tag = _digest([src], flags)
    stamp = GUARD_LIB_PATH + ".stamp"
    if os.path.exists(GUARD_LIB_PATH) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == tag:
                return GUARD_LIB_PATH
    tmp = GUARD_LIB_PATH + ".tmp"
    cmd = [os.environ.get("CXX", "g++")] + flags + ["-o", tmp, src, "-L", "/opt/rocm/lib", "-lamdhip64",
                                                      "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"guard allocator build failed\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, GUARD_LIB_PATH)
    with open(stamp, "w") as f:
        f.write(tag)
    return GUARD_LIB_PATH


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print(p)
    print(build_guard(verbose="-v" in sys.argv))
