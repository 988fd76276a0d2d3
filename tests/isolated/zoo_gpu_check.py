"""Every zoo model on the GPU (run as a child process by tests/test_isolated_gpu.py):
fp32 eval/train HIP path vs the torch path and an fp64 reference, and a bf16 channels-last
train step with OHEM + aux heads (checks in tests/test_zoo.py)."""
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))                   # tests/
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # repo root

import pytest  # noqa: E402

import test_zoo as Z  # noqa: E402


def main():
    if os.environ.get("RTSEG_GUARD"):  # guard-page allocator: OOB accesses fault deterministically
        from realtime_semantic_segmentation_pytorch_amd.utils import guard

        guard.install(os.environ["RTSEG_GUARD"])
        print(f"guard allocator: {os.environ['RTSEG_GUARD']}", flush=True)
    only = [k for k in os.environ.get("ZOO_ONLY", "").split(",") if k]
    bad = []
    for key in only or Z.KEYS:
        for name, fn in (("hip_vs_torch", lambda k: Z.check_zoo_hip_matches_torch_path(k, mp)),
                         ("bf16_train", Z.check_zoo_bf16_channels_last_train_step)):
            mp = pytest.MonkeyPatch()
            try:
                fn(key)
                print(f"{key} {name}: ok", flush=True)
            except pytest.skip.Exception as e:
                print(f"{key} {name}: skipped ({e})", flush=True)
            except Exception:  # noqa: BLE001 - report every model, then fail
                bad.append(f"{key} {name}")
                print(f"{key} {name}: FAILED\n{traceback.format_exc()}", flush=True)
                if "illegal memory access" in traceback.format_exc():
                    break  # the device is unusable after a fault
            finally:
                mp.undo()
        else:
            continue
        break
    if os.environ.get("RTSEG_GUARD"):
        from realtime_semantic_segmentation_pytorch_amd.utils import guard

        print(f"guard stats: {guard.stats()}", flush=True)
    print(f"zoo checks done: {len(bad)} failed {bad}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
