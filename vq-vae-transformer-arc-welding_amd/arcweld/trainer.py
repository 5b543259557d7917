"""Training loop equivalent to the Lightning Trainer configuration the reference uses.

* train_reconstruction_embedding.py:190-197  Trainer(devices=1, gradient_clip_val=0.7) + RAdam
* train_transformer_mtasks.py:23-33          Trainer(gradient_clip_val=0.8, accumulate_grad_batches=5,
                                             DDPStrategy(find_unused_parameters=True) if n_gpus > 1)

Step semantics (Lightning automatic optimisation): each micro-batch loss is divided by
``accumulate_grad_batches``; every ``accumulate_grad_batches`` micro-batches the gradients are averaged over
data-parallel ranks, clipped to ``gradient_clip_val`` (L2 over all gradients that exist) and RAdam steps.

Data parallelism is one process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Gradients live
in ONE flat fp32 buffer (arcweld.optim.RAdam), so the average is a handful of bucketed all-reduces over xGMI;
the 1/world factor is folded into the loss scale, so the all-reduce is a plain SUM.  Parameters of the
task head that is not used in the current stage are excluded from the clip norm and the update (the
find_unused_parameters=True behaviour: their grad stays None in the reference).
"""
from __future__ import annotations

import math
import time

import torch
import torch.distributed as dist

BUCKET_ELEMS = 8 * 1024 * 1024          # 32 MiB fp32 buckets


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_flat(flat: torch.Tensor, bucket: int = BUCKET_ELEMS):
    """SUM all-reduce of a flat buffer in large buckets (RCCL rings are link-bound; few large messages)."""
    if world() == 1:
        return
    n = flat.numel()
    works = [dist.all_reduce(flat[o:min(o + bucket, n)], async_op=True) for o in range(0, n, bucket)]
    for w in works:
        w.wait()


def broadcast_params(model: torch.nn.Module):
    if world() == 1:
        return
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src=0)


class Trainer:
    def __init__(self, devices=1, num_nodes=1, max_epochs=1, max_steps=-1, logger=None, callbacks=None,
                 gradient_clip_val=None, strategy="auto", accumulate_grad_batches=1, log_every_n_steps=50,
                 fused_grad_sink=True, **_ignored):
        self.max_epochs = max_epochs
        self.max_steps = max_steps
        self.logger = logger
        self.callbacks = callbacks
        self.gradient_clip_val = gradient_clip_val
        self.accumulate = max(1, int(accumulate_grad_batches))
        self.log_every = log_every_n_steps
        self.fused_grad_sink = fused_grad_sink
        self.global_step = 0
        self.history = []
        self.optimizer = None

    # ------------------------------------------------------------------------------ loop pieces
    def setup_optimizer(self, model):
        opt = model.configure_optimizers()
        if isinstance(opt, (list, tuple)):
            opt = opt[0]
        opt.flatten()
        active = model.active_parameters() if hasattr(model, "active_parameters") else None
        opt.set_active(active)
        if self.fused_grad_sink:
            # fused autograd nodes accumulate straight into the flat gradient views (no extra add)
            model._grad_sink = {p: p.grad for p in model.parameters()}
        broadcast_params(model)
        self.optimizer = opt
        return opt

    def micro_step(self, model, batch, batch_idx, scale):
        out = model.training_step(batch, batch_idx)
        loss = out["loss"] if isinstance(out, dict) else out
        (loss * scale).backward()
        return loss

    def optimizer_step(self, model):
        opt = self.optimizer
        allreduce_flat(opt.flat_grad)
        if self.gradient_clip_val:
            opt.clip_grad_norm_(float(self.gradient_clip_val))
        opt.step()
        opt.zero_grad()
        self.global_step += 1

    def fit(self, model, datamodule=None, train_dataloaders=None):
        if datamodule is not None:
            datamodule.setup("fit")
            loader = datamodule.train_dataloader()
        else:
            loader = train_dataloaders
        model.train()
        model.trainer = self
        self.setup_optimizer(model)
        dev = next(model.parameters()).device
        scale = 1.0 / (self.accumulate * world())
        t0 = time.time()
        for epoch in range(self.max_epochs):
            if hasattr(loader, "set_epoch"):
                loader.set_epoch(epoch)
            for i, batch in enumerate(loader):
                batch = _to_device(batch, dev)
                loss = self.micro_step(model, batch, i, scale)
                if (i + 1) % self.accumulate == 0:
                    self.optimizer_step(model)
                    if self.global_step % self.log_every == 0:
                        self.history.append((self.global_step, float(loss.detach()), time.time() - t0))
                    if 0 < self.max_steps <= self.global_step:
                        break
            if 0 < self.max_steps <= self.global_step:
                break
        model._grad_sink = None
        return self

    @torch.no_grad()
    def evaluate(self, model, loader, stage="val"):
        model.eval()
        dev = next(model.parameters()).device
        tot, n = 0.0, 0
        for i, batch in enumerate(loader):
            batch = _to_device(batch, dev)
            out = (model.validation_step if stage == "val" else model.test_step)(batch, i)
            loss = out["loss"] if isinstance(out, dict) else out
            tot += float(loss)
            n += 1
        model.train()
        return tot / max(n, 1)

    def test(self, model, datamodule=None, dataloaders=None):
        if datamodule is not None:
            datamodule.setup("test")
            loader = datamodule.test_dataloader()
        else:
            loader = dataloaders
        return self.evaluate(model, loader, stage="test")


def _to_device(batch, dev):
    if isinstance(batch, torch.Tensor):
        return batch.to(dev, non_blocking=True)
    if isinstance(batch, (list, tuple)):
        return type(batch)(_to_device(b, dev) for b in batch)
    if isinstance(batch, dict):
        return {k: _to_device(v, dev) for k, v in batch.items()}
    return batch


def cosine(x):  # pragma: no cover - helper kept for schedulers
    return 0.5 * (1 + math.cos(math.pi * x))
