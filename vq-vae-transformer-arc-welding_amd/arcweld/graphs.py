"""HIP-graph capture of the training step (the launch-bound loop: ~200 kernel launches per step from Python).

A step is captured as graphs on the current stream:
  g_fwd_bwd : forward + backward of one micro-batch (gradients accumulate into the flat buffer)
  g_update  : clip-norm + RAdam + zero_grad (captured into the last forward/backward piece when no collective and
              no accumulation separate them)
With data parallelism the RCCL all-reduce of the flat gradient buffer runs eagerly between the two.  A model
with ``fused_train_step`` (VQVAEPatch, MyTransformerDecoder) is captured as TWO forward/backward graphs split
where its ``backward_late_parameters()`` are final (VQ-VAE: the decoder side; Transformer: the task head, ln_f and
the later half of the blocks): their all-reduce is launched (async, RCCL stream) between the two replays and
overlaps the rest of the backward; the remaining gradients' all-reduce follows.  Replay needs no host values: dropout masks come from
a device counter (aw_gemm_args.seed_ptr), the RAdam step number and clip coefficient live on the device.  Inputs
are copied into static buffers before each replay; with gradient accumulation the forward/backward graphs are
replayed once per micro-batch before the update -- or, for a model with ``grouped_accumulation`` (the Transformer
decoder), the group's micro-batches are copied side by side into one static batch and the step is captured as ONE
forward/backward over all of them (``fused_train_step(groups=G)``: each micro-batch keeps its own loss mean), so the
reference's 16-sequence micro-batches (train_transformer_mtasks.py:32) no longer run as five under-filled passes.

The first `warmup` calls run eagerly on their own batches (lazy device state -- RNG counters, optimizer
buffers -- is created there); the next call captures and replays, so every call is exactly one step on the
batch it was given.
"""
from __future__ import annotations

import os

import torch

# Capture mode "thread_local": only this thread's unsafe calls are refused while it captures.  The default
# ("global") also refuses every other thread's -- including the RCCL process group's watchdog, which polls the
# completion events of earlier all-reduces from its own thread and terminates the process when the poll is refused
# (seen on the GPU box: "operation not permitted when stream is capturing" from WorkNCCL::isCompleted).
_MODE = "thread_local"


def _clone_static(batch):
    if isinstance(batch, torch.Tensor):
        return batch.clone()
    return type(batch)(_clone_static(b) for b in batch)


def _flatten(batch, out):
    if isinstance(batch, torch.Tensor):
        out.append(batch)
    else:
        for b in batch:
            _flatten(b, out)
    return out


def _concat(batches):
    """The micro-batches of a group side by side (dim 0 of every tensor)."""
    if isinstance(batches[0], torch.Tensor):
        return torch.cat(batches, 0)
    return type(batches[0])(_concat([b[i] for b in batches]) for i in range(len(batches[0])))


def _same_shapes(batches):
    shp = lambda b: [(t.shape, t.dtype) for t in _flatten(b, [])]  # noqa: E731
    return all(shp(b) == shp(batches[0]) for b in batches[1:])


def _copy_group_into(dst, batches):
    """The group's micro-batches into their row slices of the static buffers: one multi-tensor copy launch."""
    d, s = [], []
    for t_dst, *t_src in zip(_flatten(dst, []), *[_flatten(b, []) for b in batches]):
        n = t_src[0].shape[0]
        for j, t in enumerate(t_src):
            d.append(t_dst[j * n:(j + 1) * n])
            s.append(t)
    if all(a.dtype == b.dtype and a.device == b.device for a, b in zip(d, s)):
        torch._foreach_copy_(d, s, non_blocking=True)
    else:
        for a, b in zip(d, s):
            a.copy_(b, non_blocking=True)


def _copy_into(dst, src):
    """The batch into the static input buffers: one multi-tensor copy launch for all of its tensors (the decoder's
    ids / condition / targets took three copy launches)."""
    d, s = _flatten(dst, []), _flatten(src, [])
    if len(d) == 1:
        d[0].copy_(s[0], non_blocking=True)
    elif all(a.dtype == b.dtype and a.device == b.device for a, b in zip(d, s)):
        torch._foreach_copy_(d, s, non_blocking=True)
    else:
        for a, b in zip(d, s):
            a.copy_(b, non_blocking=True)


class StepGraphs:
    """allreduce(region) launches the SUM all-reduce of a flat-gradient region ("all", "late" = the part final at
    the mid-backward split, "early" = the rest) and returns the async work handles; collective=False (no process
    group) lets the model defer the late weight gradients past the split (model._wgrad_merge)."""

    def __init__(self, trainer, model, scale, allreduce, warmup=2, collective=True):
        self.trainer, self.model, self.scale, self.allreduce = trainer, model, scale, allreduce
        self.warmup = warmup
        self.calls = 0
        self.static = None
        # The forward/backward is captured as two graphs split at the model's mid-backward hook, with or without a
        # collective between them: the split measured faster on its own (VQ-VAE step 3.152 / 3.167 vs 3.222 / 3.202
        # ms unsplit, same box).  Without a collective nothing needs the late gradients at the hook, so the decoder
        # issues the weight gradients of all its blocks as one batch at the end (model._wgrad_merge, arcweld/decoder.py
        # backward).  ARCWELD_SPLIT_GRAPHS=0 captures one graph (A/B runs).
        self.split = hasattr(model, "fused_train_step") and hasattr(model, "backward_late_parameters") and \
            os.environ.get("ARCWELD_SPLIT_GRAPHS") != "0"
        model.__dict__["_wgrad_merge"] = not collective and os.environ.get("ARCWELD_WGRAD_MERGE") != "0"
        # an accumulation group as one captured batch (see the module docstring); ARCWELD_GROUP_ACCUM=0 replays the
        # per-micro-batch graph instead (A/B runs)
        self.group_accum = self.split and getattr(model, "grouped_accumulation", False) and \
            getattr(trainer, "accumulate", 1) > 1 and os.environ.get("ARCWELD_GROUP_ACCUM") != "0"
        self.G = 1
        # Without a collective and without accumulation nothing runs between the last forward/backward piece and the
        # update, so the update is captured into that piece: one graph launch (and its ~8.5 us gap on the stream)
        # fewer per step.  ARCWELD_FUSE_UPDATE=0 keeps it a graph of its own (A/B runs).
        self.fuse_update = self.split and not collective and \
            (getattr(trainer, "accumulate", 1) == 1 or self.group_accum) and os.environ.get("ARCWELD_FUSE_UPDATE") != "0"

    def _capture(self, batch, G=1):
        self.static = _clone_static(batch)
        if hasattr(self.model, "_loss_scale_tensor"):       # persistent scalars are made outside the capture
            dev = next(self.model.parameters()).device
            self.model._loss_scale_tensor(float(self.scale), dev)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        self.g2 = torch.cuda.CUDAGraph()
        if self.split:
            # the forward/backward as a list of graph pieces, cut at the mid-backward hook (the late all-reduce is
            # launched after that piece).  A further cut between the VQ-VAE forward and backward measured even
            # (3.086-3.091 vs 3.084-3.100 ms, same box) and is not made.
            self.pieces, self.late_after = [torch.cuda.CUDAGraph()], None
            state = {"ctx": torch.cuda.graph(self.pieces[0], pool=pool, capture_error_mode=_MODE)}
            state["ctx"].__enter__()

            def cut():
                state["ctx"].__exit__(None, None, None)
                self.pieces.append(torch.cuda.CUDAGraph())
                state["ctx"] = torch.cuda.graph(self.pieces[-1], pool=pool, capture_error_mode=_MODE)
                state["ctx"].__enter__()

            def mid():   # the decoder-side gradients are final here: the late all-reduce follows this piece
                self.late_after = len(self.pieces) - 1
                cut()

            try:
                kw = {"groups": G} if G > 1 else {}
                self.loss = self.model.fused_train_step(self.static, self.scale, mid_hook=mid, **kw)
                if self.fuse_update:
                    self.trainer._update(self.model)
            finally:
                state["ctx"].__exit__(None, None, None)
            if self.fuse_update:
                return
        else:
            self.g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g1, pool=pool, capture_error_mode=_MODE):
                self.loss = self.trainer.micro_step(self.model, self.static, 0, self.scale)
        with torch.cuda.graph(self.g2, pool=pool, capture_error_mode=_MODE):
            self.trainer._update(self.model)

    def _eager(self, batches):
        """One optimizer step over the micro-batches without the graphs (warm-up calls, groups the capture cannot
        take): each micro-batch's forward/backward, the all-reduce of every live gradient, the update."""
        for j, b in enumerate(batches):
            loss = self.trainer.micro_step(self.model, b, j, self.scale)
        for w in self.allreduce("all"):
            w.wait()
        self.trainer._update(self.model)
        self.trainer.global_step += 1
        return loss

    def run(self, batch):
        """One optimizer step over `batch`, or over a list of micro-batches (accumulate_grad_batches > 1: the
        forward/backward graph is replayed once per micro-batch, gradients accumulating in the flat buffer; the
        all-reduce runs once, split around the last micro-batch's backward -- DDP's no_sync accumulation)."""
        batches = batch if isinstance(batch, list) else [batch]
        G = len(batches) if len(batches) > 1 and self.group_accum and _same_shapes(batches) else 1
        self.calls += 1
        if self.calls <= self.warmup:
            return self._eager(batches)
        # A group the captured step cannot replay runs eagerly on the same gradients and optimizer state: the short
        # last group of an epoch (Lightning steps on the epoch's last batch whatever the group size), micro-batches
        # of different shapes, or more than one micro-batch where the update is captured with the backward.  The
        # graphs are captured on the first full group only, so a short group never fixes the captured size.
        full = getattr(self.trainer, "accumulate", 1) if self.group_accum else 1
        if (self.group_accum and G != full) or (self.fuse_update and G == 1 and len(batches) > 1) or \
                (self.static is not None and G != self.G):
            return self._eager(batches)
        if self.static is None:
            self.G = G
            self._capture(_concat(batches) if G > 1 else batches[0], G)
        if G > 1:
            _copy_group_into(self.static, batches)
            batches = [None]      # one replay of the group's forward/backward
        last = len(batches) - 1
        works = []
        for j, b in enumerate(batches):
            if b is not None:
                _copy_into(self.static, b)    # ordered after the previous replay on this stream
            if self.split:
                for i, g in enumerate(self.pieces):
                    g.replay()
                    if j == last and i == self.late_after:
                        works = self.allreduce("late")   # decoder side: overlaps the encoder-side backward below
                if j == last:
                    if self.late_after is None:
                        works = self.allreduce("late")
                    works += self.allreduce("early")
            else:
                self.g1.replay()
                if j == last:
                    works = self.allreduce("all")
        for w in works:
            w.wait()
        if not self.fuse_update:
            self.g2.replay()
        self.trainer.global_step += 1
        return self.loss
