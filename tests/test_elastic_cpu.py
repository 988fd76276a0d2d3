"""Failure detection / recovery end to end on CPU: a 2-rank gloo job under torchrun with
``--max-restarts 1`` loses a rank at the start of epoch 1 (injected fault), torchrun tears the
group down and restarts it, every rank auto-resumes from ``last.pth`` (reference
core/base_trainer.py:66-89 resume flow) and the run finishes all epochs.  Rendezvous on
127.0.0.1; the restarted generation joins through its own store prefix (parallel/ddp.py)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(900)
def test_torchrun_restart_resumes_from_last_checkpoint(tmp_path):
    save = tmp_path / "save"
    sentinel = tmp_path / "fault_fired"
    env = dict(os.environ, RTSEG_FAULT_EPOCH="1", RTSEG_FAULT_SENTINEL=str(sentinel), OMP_NUM_THREADS="2", GLOO_SOCKET_IFNAME="lo",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--max-restarts=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "main.py"),
           "--train", "--model", "enet", "--no_aux", "--synthetic_data", "--synthetic_len", "8", "--crop_size", "32",
           "--train_bs", "2", "--val_bs", "2", "--total_epoch", "3", "--device", "cpu", "--base_workers", "0",
           "--save_dir", str(save), "--load_ckpt_path", str(save / "last.pth"), "--use_tb"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert sentinel.exists(), "the injected fault never fired"
    ck = torch.load(save / "last.pth", map_location="cpu", weights_only=True)
    assert ck["cur_epoch"] == 2  # epochs 1 and 2 ran after the restart
    assert (save / "best.pth").exists()
    log = (save / "seg_trainer.log").read_text()
    assert "Resume training" in log and "Epoch:2/3" in log


@pytest.mark.timeout(600)
def test_main_spawns_single_node_ddp_without_a_launcher(tmp_path):
    """The reference's DP mode (several GPUs, no launcher) maps onto one process per device:
    main.py spawns the workers itself and they train as DDP (gloo on CPU here)."""
    save = tmp_path / "save"
    env = dict(os.environ, OMP_NUM_THREADS="2", GLOO_SOCKET_IFNAME="lo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "main.py"), "--train", "--model", "enet", "--no_aux", "--synthetic_data",
           "--synthetic_len", "8", "--crop_size", "32", "--train_bs", "2", "--val_bs", "2", "--total_epoch", "1",
           "--device", "cpu", "--base_workers", "0", "--save_dir", str(save), "--load_ckpt_path",
           str(save / "last.pth"), "--use_tb", "--spawn_procs", "2"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=550)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    log = (save / "seg_trainer.log").read_text()
    assert "gpu_num: 2" in log and "DDP: True" in log
