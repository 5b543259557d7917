"""HIP-graph capture of the training step (the launch-bound loop: ~200 kernel launches per step from Python).

A step is captured as two graphs on the current stream:
  g_fwd_bwd : forward + backward of one micro-batch (gradients accumulate into the flat buffer)
  g_update  : clip-norm + RAdam + zero_grad
With data parallelism the RCCL all-reduce of the flat gradient buffer runs eagerly between the two.  Replay
needs no host values: dropout masks come from a device counter (aw_gemm_args.seed_ptr), the RAdam step number
and clip coefficient live on the device.  Inputs are copied into static buffers before each replay.

The first `warmup` calls run eagerly on their own batches (lazy device state -- RNG counters, optimizer
buffers -- is created there); the next call captures and replays, so every call is exactly one step on the
batch it was given.
"""
from __future__ import annotations

import torch


def _clone_static(batch):
    if isinstance(batch, torch.Tensor):
        return batch.clone()
    return type(batch)(_clone_static(b) for b in batch)


def _copy_into(dst, src):
    if isinstance(dst, torch.Tensor):
        dst.copy_(src, non_blocking=True)
        return
    for d, s in zip(dst, src):
        _copy_into(d, s)


class StepGraphs:
    def __init__(self, trainer, model, scale, allreduce, warmup=2):
        self.trainer, self.model, self.scale, self.allreduce = trainer, model, scale, allreduce
        self.warmup = warmup
        self.calls = 0
        self.static = None

    def _capture(self, batch):
        self.static = _clone_static(batch)
        torch.cuda.synchronize()
        self.g1, self.g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(self.g1, pool=pool):
            self.loss = self.trainer.micro_step(self.model, self.static, 0, self.scale)
        with torch.cuda.graph(self.g2, pool=pool):
            self.trainer._update(self.model)

    def run(self, batch):
        self.calls += 1
        if self.calls <= self.warmup:
            loss = self.trainer.micro_step(self.model, batch, 0, self.scale)
            self.allreduce()
            self.trainer._update(self.model)
            self.trainer.global_step += 1
            return loss
        if self.static is None:
            self._capture(batch)
        else:
            _copy_into(self.static, batch)
        self.g1.replay()
        self.allreduce()
        self.g2.replay()
        self.trainer.global_step += 1
        return self.loss
