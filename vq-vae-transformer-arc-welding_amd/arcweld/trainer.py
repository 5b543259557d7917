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

import os

import math
import time

import torch
import torch.distributed as dist

BUCKET_ELEMS = 8 * 1024 * 1024          # 32 MiB fp32 buckets


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _collectives_off():
    """No collective at world size 1 -- unless ARCWELD_FORCE_COLLECTIVES=1 under an initialised process group: the
    RCCL test (tests/test_rccl_gpu.py) runs the bucketed all-reduce on a one-rank RCCL group, so the async work
    handles and their stream ordering against the captured step graphs run on the real backend."""
    if world() > 1:
        return False
    return not (os.environ.get("ARCWELD_FORCE_COLLECTIVES") == "1" and dist.is_available() and dist.is_initialized())


def allreduce_flat(flat: torch.Tensor, bucket: int = BUCKET_ELEMS, lo: int = 0, hi: int = None, wait: bool = True):
    """SUM all-reduce of flat[lo:hi] in large buckets (RCCL rings are link-bound; few large messages).  With
    wait=False the async work handles are returned (the collectives are ordered after the work already queued on
    the current stream and run on RCCL's stream)."""
    if _collectives_off():
        return []
    hi = flat.numel() if hi is None else hi
    works = [dist.all_reduce(flat[o:min(o + bucket, hi)], async_op=True) for o in range(lo, hi, bucket)]
    if wait:
        for w in works:
            w.wait()
        return []
    return works


def allreduce_spans(flat: torch.Tensor, spans, bucket: int = BUCKET_ELEMS):
    """Async SUM all-reduce of the [a, b) ranges of a flat buffer, each cut into buckets; returns the work handles."""
    if _collectives_off():
        return []
    n = flat.numel()
    # every span ends on a 256-B boundary: segments start 256-B aligned, so the rounding only takes in the zero
    # padding before the next segment, and RCCL moves whole 16-B packs (an odd-length tail measured unscaled by the
    # one-rank pre-multiplied sum of tests/test_rccl_gpu.py)
    spans = [(a, min(n, (b + 63) // 64 * 64)) for a, b in spans]
    return [dist.all_reduce(flat[o:min(o + bucket, b)], async_op=True) for a, b in spans for o in range(a, b, bucket)]


def _spans(opt, lo=0, hi=None):
    if hasattr(opt, "live_spans"):
        return opt.live_spans(lo, hi)
    return [(lo, opt.flat_grad.numel() if hi is None else hi)]


def broadcast_params(model: torch.nn.Module, opt=None):
    """Rank 0's parameters and buffers to every rank (DDP's initial broadcast).  Parameters packed into the
    optimizer's flat buffer go as that one buffer (some are strided views, which collectives do not take)."""
    if world() == 1:
        return
    packed = set()
    if opt is not None and hasattr(opt, "live_spans"):
        flat_p = opt.flatten()[0]
        dist.broadcast(flat_p, src=0)
        packed = set(id(p) for p in opt._flat["params"])
    for t in list(model.parameters()) + list(model.buffers()):
        if id(t) not in packed:
            dist.broadcast(t.data, src=0)
    from . import operands
    operands.invalidate(model)      # the flat buffer changed behind the parameters' version counters


class Trainer:
    def __init__(self, devices="auto", num_nodes=1, max_epochs=1, max_steps=-1, logger=None, callbacks=None,
                 gradient_clip_val=None, strategy="auto", accumulate_grad_batches=1, log_every_n_steps=50,
                 fused_grad_sink=True, hip_graphs=False, **_ignored):
        self.max_epochs = max_epochs
        self.max_steps = max_steps
        # devices=1 under an initialised process group trains this rank alone (no sharding, no all-reduce), as a
        # Lightning Trainer(devices=1) does; "auto" / N > 1 use every rank of the group
        self.devices = devices
        self.data_parallel = not (isinstance(devices, int) and devices == 1)
        self.logger = logger
        self.gradient_clip_val = gradient_clip_val
        self.accumulate = max(1, int(accumulate_grad_batches))
        self.log_every = log_every_n_steps
        self.fused_grad_sink = fused_grad_sink
        self.bucket_elems = BUCKET_ELEMS   # all-reduce bucket (fp32 elements)
        self.hip_graphs = hip_graphs   # capture the step (fixed batch shape; accumulation groups replay per micro-batch)
        self.global_step = 0
        self.history = []
        self.optimizer = None
        self.callbacks = [] if callbacks is None else (list(callbacks) if isinstance(callbacks, (list, tuple))
                                                       else [callbacks])
        self.logged_metrics = {}
        self.should_stop = False
        self.current_epoch = 0

    # ------------------------------------------------------------------------------ loop pieces
    def setup_optimizer(self, model):
        opt = model.configure_optimizers()
        if isinstance(opt, (list, tuple)):
            opt = opt[0]
        if hasattr(model, "centre_tap_parameters") and hasattr(opt, "declare_centre_tap"):
            opt.declare_centre_tap(model.centre_tap_parameters())
        if hasattr(model, "tap_major_parameters") and hasattr(opt, "declare_tap_major") \
                and os.environ.get("ARCWELD_TAP_MAJOR", "1") != "0":     # 0: the reference layout (A/B only)
            opt.declare_tap_major(model.tap_major_parameters())
        opt.flatten()
        active = model.active_parameters() if hasattr(model, "active_parameters") else None
        opt.set_active(active)
        if self.fused_grad_sink:
            # fused autograd nodes accumulate straight into the flat gradient views (no extra add)
            model._grad_sink = {p: p.grad for p in model.parameters()}
        if self.data_parallel:
            broadcast_params(model, opt)
        if hasattr(model, "operand_set") and hasattr(opt, "attach_operands"):
            opt.attach_operands(model.operand_set())     # the update kernel keeps the GEMM operand copies current
        # residual-VQ codebooks synchronise across ranks only when the ranks train one model together: a devices=1
        # Trainer under an initialised process group turns the sync off for the time it trains the model
        # (teardown() restores the previous setting, so a model later trained data-parallel by other code is not
        # left with drifting per-rank codebooks); data-parallel mode leaves it to follow the process group
        self.teardown()
        self._sync_saved = [(mod, mod.sync_codebooks) for mod in model.modules() if hasattr(mod, "sync_codebooks")]
        for mod, _ in self._sync_saved:
            mod.sync_codebooks = None if self.data_parallel else False
        self.optimizer = opt
        self._graphs = None          # a captured step belongs to one optimizer
        self._graph_shape = None
        self._late_key = None        # the late/early all-reduce spans follow this optimizer's flat offsets
        return opt

    def teardown(self):
        """Restore what setup_optimizer changed on the model outside the optimizer (the residual-VQ codebook
        sync mode); fit() calls it when training ends."""
        for mod, prev in getattr(self, "_sync_saved", ()):
            mod.sync_codebooks = prev
        self._sync_saved = []

    def micro_step(self, model, batch, batch_idx, scale):
        out = model.training_step(batch, batch_idx)
        loss = out["loss"] if isinstance(out, dict) else out
        (loss * scale).backward()
        return loss

    def _update(self, model):
        opt = self.optimizer
        if self.gradient_clip_val:
            opt.clip_grad_norm_(float(self.gradient_clip_val))
        if hasattr(opt, "attach_operands"):     # arcweld RAdam: zero_grad fused into the update pass
            opt.step(zero_grad=True)
        else:
            opt.step()
        opt.zero_grad()

    def world(self):
        return world() if self.data_parallel else 1

    def optimizer_step(self, model):
        works = allreduce_spans(self.optimizer.flat_grad, _spans(self.optimizer), self.bucket_elems) \
            if self.data_parallel else []
        for w in works:
            w.wait()
        self._update(model)
        self.global_step += 1

    def graphed_step(self, model, batch, scale):
        """One full optimizer step replayed from captured HIP graphs: `batch` is one micro-batch, or the list of
        micro-batches of one accumulation group (their forward/backward graph replayed once each, then one update).
        The first calls warm up eagerly and capture.  Returns the (static) loss tensor."""
        from .graphs import StepGraphs
        if getattr(self, "_graphs", None) is None or self._graphs.model is not model:
            self._graphs = StepGraphs(self, model, scale, lambda region: self._allreduce_region(model, region),
                                      collective=self.data_parallel and not _collectives_off())
        return self._graphs.run(batch)

    def _allreduce_region(self, model, region):
        """Async all-reduce of the flat gradients: "all", or split by the model's backward_late_parameters() into
        "late" (those parameters: final at the fused step's mid-backward hook, reduced while the rest of the
        backward runs) and "early" (every other live gradient)."""
        opt = self.optimizer
        flat = opt.flat_grad
        if not self.data_parallel:
            return []
        if region == "all" or not hasattr(model, "backward_late_parameters"):
            return allreduce_spans(flat, _spans(opt), self.bucket_elems) if region in ("all", "late") else []
        key = (id(model), getattr(model, "task", None))      # the late set of the decoder follows its task
        if getattr(self, "_late_key", None) != key:
            late = opt.param_spans(model.backward_late_parameters())
            self._late_spans, self._early_spans, self._late_key = late, opt.live_spans_excluding(late), key
        return allreduce_spans(flat, self._late_spans if region == "late" else self._early_spans, self.bucket_elems)

    def fit(self, model, datamodule=None, train_dataloaders=None, val_dataloaders=None):
        if datamodule is not None:
            datamodule.setup("fit")
            loader = datamodule.train_dataloader()
            val_loader = datamodule.val_dataloader() if hasattr(datamodule, "val_dataloader") else None
        else:
            loader, val_loader = train_dataloaders, val_dataloaders
        model.train()
        model.trainer = self
        self.setup_optimizer(model)
        self.should_stop = False
        dev = next(model.parameters()).device
        if not self.data_parallel:
            for ld in (loader, val_loader):
                if hasattr(ld, "rank") and hasattr(ld, "world"):
                    ld.rank, ld.world = 0, 1
        scale = 1.0 / (self.accumulate * self.world())
        t0 = time.time()
        for epoch in range(self.max_epochs):
            self.current_epoch = epoch
            if hasattr(loader, "set_epoch"):
                loader.set_epoch(epoch)
            n = len(loader) if hasattr(loader, "__len__") else None
            group = []          # micro-batches of the current accumulation group (captured path)
            for i, batch in enumerate(loader):
                batch = _to_device(batch, dev)
                # a residual-VQ model synchronises its codebooks with host-issued collectives in the forward
                # (arcweld/residual_vq.py): eager steps when data parallel
                graphable = not (getattr(model, "use_improved_vq", False) and self.world() > 1)
                graphed = self.hip_graphs and graphable and _fixed_shape(self, batch)
                if not graphed and group:
                    # a batch the captured step cannot take (e.g. a ragged last batch): the group so far runs
                    # eagerly, accumulating into the same gradients, and the eager path below takes over
                    for j, b in enumerate(group):
                        self.micro_step(model, b, j, scale)
                    group = []
                if graphed:
                    # Lightning steps on every accumulate-th batch and on the last batch of the epoch
                    group.append(batch)
                    if len(group) < self.accumulate and not (n is not None and i + 1 == n):
                        continue
                    batch, group = (group if self.accumulate > 1 else group[0]), []
                    loss = self.graphed_step(model, batch, scale)
                    if self.global_step % self.log_every == 0:
                        # the captured step's static loss tensor holds this replay's value
                        lv = float(loss.detach())
                        self.history.append((self.global_step, lv, time.time() - t0))
                        if self.logger is not None and hasattr(self.logger, "log_metrics"):
                            self.logger.log_metrics({"train/loss": lv}, step=self.global_step)
                    if 0 < self.max_steps <= self.global_step:
                        break
                    continue
                loss = self.micro_step(model, batch, i, scale)
                # Lightning steps on every accumulate-th batch and on the last batch of the epoch
                if (i + 1) % self.accumulate == 0 or (n is not None and i + 1 == n):
                    self.optimizer_step(model)
                    if self.global_step % self.log_every == 0:
                        lv = float(loss.detach())
                        self.history.append((self.global_step, lv, time.time() - t0))
                        if self.logger is not None and hasattr(self.logger, "log_metrics"):
                            self.logger.log_metrics({"train/loss": lv}, step=self.global_step)
                    if 0 < self.max_steps <= self.global_step:
                        break
            if val_loader is not None:
                metrics = self.evaluate(model, val_loader, "val")
                self.logged_metrics.update(metrics)
                if self.logger is not None and hasattr(self.logger, "log_metrics"):
                    self.logger.log_metrics({"epoch": epoch, **metrics}, step=self.global_step)
                for cb in self.callbacks:
                    if hasattr(cb, "on_validation_end"):
                        cb.on_validation_end(self, model, metrics)
            if self.should_stop or 0 < self.max_steps <= self.global_step:
                break
        model._grad_sink = None
        self.teardown()
        return self

    @torch.no_grad()
    def evaluate(self, model, loader, stage="val"):
        """Runs validation_step/test_step over the loader; every logged scalar is averaged over the epoch
        (weighted by batch size, Lightning's on_epoch reduction) and, under DDP, over ranks."""
        model.eval()
        dev = next(model.parameters()).device
        sums, total = {}, 0
        for i, batch in enumerate(loader):
            batch = _to_device(batch, dev)
            model._logged = {}
            (model.validation_step if stage == "val" else model.test_step)(batch, i)
            bs = len(batch[0]) if isinstance(batch, (list, tuple)) else len(batch)
            for k, v in model.logged.items():
                v = v.float() if isinstance(v, torch.Tensor) else torch.tensor(float(v), device=dev)
                sums[k] = sums.get(k, 0.0) + v * bs
            total += bs
        model.train()
        if not sums:
            return {}
        keys = sorted(sums)
        vec = torch.stack([sums[k] for k in keys] + [torch.tensor(float(total), device=dev)])
        if self.world() > 1 and stage == "val":
            dist.all_reduce(vec)
        vec = vec.cpu()
        return {k: float(vec[j] / vec[-1]) for j, k in enumerate(keys)}

    def validate(self, model, datamodule=None, dataloaders=None):
        if datamodule is not None:
            datamodule.setup("fit")
            dataloaders = datamodule.val_dataloader()
        return self.evaluate(model, dataloaders, "val")

    def test(self, model, datamodule=None, dataloaders=None):
        if datamodule is not None:
            datamodule.setup("test")
            loader = datamodule.test_dataloader()
        else:
            loader = dataloaders
        metrics = self.evaluate(model, loader, stage="test")
        self.logged_metrics.update(metrics)
        if self.logger is not None and hasattr(self.logger, "log_metrics"):
            self.logger.log_metrics(metrics, step=self.global_step)
        return [metrics]


class EarlyStopping:
    """lightning EarlyStopping(monitor, min_delta, patience, mode) evaluated at the end of each validation."""

    def __init__(self, monitor, min_delta=0.0, patience=3, verbose=False, mode="min"):
        self.monitor, self.min_delta, self.patience, self.mode = monitor, abs(min_delta), patience, mode
        self.best, self.wait = None, 0

    def on_validation_end(self, trainer, model, metrics):
        if self.monitor not in metrics:
            return
        v = metrics[self.monitor]
        better = (self.best is None or (v < self.best - self.min_delta if self.mode == "min"
                                        else v > self.best + self.min_delta))
        if better:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait >= self.patience:
                trainer.should_stop = True


class ModelCheckpoint:
    """Saves the best (by ``monitor``) and, with save_last, the last model as Lightning-layout checkpoints
    (rank 0 only)."""

    def __init__(self, dirpath, monitor=None, mode="min", filename="best", save_last=False):
        self.dirpath, self.monitor, self.mode, self.filename, self.save_last = dirpath, monitor, mode, filename, \
            save_last
        self.best, self.best_model_path = None, None

    def on_validation_end(self, trainer, model, metrics):
        import os
        if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            return
        os.makedirs(self.dirpath, exist_ok=True)
        if self.monitor in metrics:
            v = metrics[self.monitor]
            if self.best is None or (v < self.best if self.mode == "min" else v > self.best):
                self.best = v
                self.best_model_path = os.path.join(self.dirpath, self.filename + ".ckpt")
                model.save_checkpoint(self.best_model_path)
        if self.save_last:
            model.save_checkpoint(os.path.join(self.dirpath, "last.ckpt"))


def _shapes(batch):
    if isinstance(batch, torch.Tensor):
        return (tuple(batch.shape), batch.dtype)
    return tuple(_shapes(b) for b in batch)


def _fixed_shape(trainer, batch):
    """Graph replay needs the captured shapes; a ragged last batch runs eagerly."""
    sh = _shapes(batch)
    if getattr(trainer, "_graph_shape", None) is None:
        trainer._graph_shape = sh
    return sh == trainer._graph_shape


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
