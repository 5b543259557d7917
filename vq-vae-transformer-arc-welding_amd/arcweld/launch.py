"""Process-group setup and the CSV logger the entry scripts use.

Multi-GPU runs are one process per GPU started by ``python -m torch.distributed.run --nproc-per-node N``
(Lightning's DDPStrategy spawns them itself in the reference, train_transformer_mtasks.py:31); the process group
is RCCL ("nccl" on ROCm) over xGMI, or gloo for CPU-only plumbing tests.
"""
from __future__ import annotations

import csv
import json
import os

import torch
import torch.distributed as dist


def init_distributed(backend=None, enable=True):
    """-> (rank, world, device).  Initialises the default process group when launched with WORLD_SIZE > 1 (and
    ``enable``; a process started by torchrun with enable=False trains alone on its LOCAL_RANK device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if enable and world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend)
    rank = dist.get_rank() if dist.is_initialized() else 0
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    return rank, (dist.get_world_size() if dist.is_initialized() else 1), dev


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()


class CSVLogger:
    """lightning CSVLogger(save_dir, name): <save_dir>/<name>/version_<k>/{hparams.json, metrics.csv}."""

    def __init__(self, save_dir="logs", name="default"):
        base = os.path.join(save_dir, name)
        os.makedirs(base, exist_ok=True)
        k = 0
        while os.path.exists(os.path.join(base, f"version_{k}")):
            k += 1
        self.log_dir = os.path.join(base, f"version_{k}")
        self.rows = []
        self._rank0 = not dist.is_initialized() or dist.get_rank() == 0
        if self._rank0:
            os.makedirs(self.log_dir, exist_ok=True)

    def log_hyperparams(self, params):
        if not self._rank0:
            return
        params = vars(params) if hasattr(params, "__dict__") and not isinstance(params, dict) else dict(params)
        with open(os.path.join(self.log_dir, "hparams.json"), "w") as f:
            json.dump({k: (v if isinstance(v, (int, float, str, bool, type(None))) else str(v))
                       for k, v in params.items()}, f, indent=1)

    def log_metrics(self, metrics, step=None):
        if not self._rank0:
            return
        row = {"step": step, **metrics}
        self.rows.append(row)
        keys = sorted({k for r in self.rows for k in r})
        with open(os.path.join(self.log_dir, "metrics.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            w.writerows(self.rows)
