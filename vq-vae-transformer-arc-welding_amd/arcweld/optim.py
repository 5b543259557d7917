"""Flat-buffer multi-tensor RAdam + global-norm clip on the HIP kernels.

Drop-in for ``torch.optim.RAdam`` as the reference builds it (model/autencoder_lightning_base.py:122-124;
model/transformer_decoder.py:64-114 -- two parameter groups that differ only in weight decay).  On the first
step the parameters of all groups are packed into ONE contiguous fp32 buffer and every ``p.data`` / ``p.grad``
is re-bound to a view of it, so that

* the optimizer update is one kernel over the flat buffer (segments carry per-group weight decay and an
  "active" flag -- a parameter that produced no gradient this stage is skipped, like torch skips grad None),
* the gradient all-reduce of data parallelism is a few large RCCL calls over the flat gradient buffer,
* the clip coefficient (Lightning ``gradient_clip_val``) is computed on device and fed to the update kernel:
  no host synchronisation anywhere in the step.

``zero_grad`` keeps the gradient views attached (it zeroes the flat buffer); ``set_to_none`` is ignored.
"""
from __future__ import annotations

import torch

from . import kernels as K


class RAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._flat = None
        self._step_count = 0
        self._coef = None
        self._pending_active = None

    # ------------------------------------------------------------------ flat layout
    def _build(self):
        params = [p for g in self.param_groups for p in g["params"]]
        dev = params[0].device
        if not all(p.device == dev and p.dtype == torch.float32 for p in params):
            raise RuntimeError("arcweld RAdam needs all parameters as float32 on one device")
        if dev.type != "cuda":
            raise RuntimeError("arcweld RAdam runs on the GPU only (no CPU fallback)")
        offs, lens, wds, owner = [], [], [], []
        total = 0
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                offs.append(total)
                lens.append(p.numel())
                wds.append(float(g["weight_decay"]))
                owner.append(gi)
                total += (p.numel() + 63) // 64 * 64        # 256-B aligned segments
        flat_p = torch.zeros(total, device=dev)
        flat_g = torch.zeros(total, device=dev)
        for p, o in zip(params, offs):
            n = p.numel()
            flat_p[o:o + n].copy_(p.detach().reshape(-1))
            if p.grad is not None:
                flat_g[o:o + n].copy_(p.grad.reshape(-1))
            p.data = flat_p[o:o + n].view_as(p)
            p.grad = flat_g[o:o + n].view_as(p)
        self._flat = dict(params=params, p=flat_p, g=flat_g, m=torch.zeros(total, device=dev),
                          v=torch.zeros(total, device=dev), total=total, owner=owner, offs=offs, lens=lens,
                          off_d=torch.tensor(offs, device=dev, dtype=torch.int64),
                          len_d=torch.tensor(lens, device=dev, dtype=torch.int64),
                          wd_d=torch.tensor(wds, device=dev, dtype=torch.float32),
                          ws=torch.zeros(1, device=dev, dtype=torch.float64),
                          norm=torch.zeros((), device=dev), coef=torch.ones((), device=dev),
                          step=torch.full((1,), self._step_count, device=dev, dtype=torch.int64))
        self.set_active(self._pending_active)

    def flatten(self):
        """Pack now (idempotent).  Returns the flat parameter and gradient buffers."""
        if self._flat is None:
            self._build()
        return self._flat["p"], self._flat["g"]

    def set_active(self, params):
        """Restrict clip-norm and update to ``params`` (None = all): the find_unused_parameters semantics of the
        reference's task switching (an unused head keeps grad None -> no update, no decay)."""
        if self._flat is None:
            self._pending_active = params
            return
        F = self._flat
        keep = None if params is None else set(id(p) for p in params)
        act = [1 if keep is None or id(p) in keep else 0 for p in F["params"]]
        dev = F["p"].device
        F["act_d"] = torch.tensor(act, device=dev, dtype=torch.int32)
        F["act_group"] = [torch.tensor([a if o == gi else 0 for a, o in zip(act, F["owner"])], device=dev,
                                       dtype=torch.int32) for gi in range(len(self.param_groups))]

    def flat_offset(self, param):
        """Element offset of ``param``'s segment in the flat buffers."""
        self.flatten()
        F = self._flat
        for p, o in zip(F["params"], F["offs"]):
            if p is param:
                return o
        raise KeyError("parameter is not managed by this optimizer")

    @property
    def flat_grad(self):
        return self.flatten()[1]

    # ------------------------------------------------------------------ torch.optim API
    def zero_grad(self, set_to_none: bool = True):
        if self._flat is None:
            for g in self.param_groups:
                for p in g["params"]:
                    p.grad = None
            return
        self._flat["g"].zero_()

    def clip_grad_norm_(self, max_norm):
        """L2 norm over the active gradients; the clip coefficient is applied inside the next step().
        Returns the (pre-clip) total norm as a device scalar."""
        self.flatten()
        F = self._flat
        K.grad_norm_clip(F["g"], F["off_d"], F["len_d"], F["act_d"], len(F["params"]), max_norm, F["ws"], F["norm"],
                         F["coef"])
        self._coef = F["coef"]
        return F["norm"]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.flatten()
        F = self._flat
        self._step_count += 1
        # the step number also lives on the device, so a captured step graph replays with the right bias
        # corrections; one launch per group (groups may differ in lr/betas/eps), other groups' segments masked
        K.counter_add(F["step"], 1)
        # groups that differ only in weight decay (per segment already) share one launch
        for (lr, (b1, b2), eps), act in self._launch_groups():
            K.radam_step(F["p"], F["g"], F["m"], F["v"], F["off_d"], F["len_d"], F["wd_d"], act, len(F["params"]),
                         F["total"], self._step_count, lr, b1, b2, eps, gscale=self._coef, step_ptr=F["step"])
        self._coef = None
        return loss

    def _launch_groups(self):
        F = self._flat
        keys = [(float(g["lr"]), tuple(g["betas"]), float(g["eps"])) for g in self.param_groups]
        if len(set(keys)) == 1:
            return [(keys[0], F["act_d"])]
        return [(k, F["act_group"][gi]) for gi, k in enumerate(keys)]

    def state_dict(self):
        sd = super().state_dict()
        if self._flat is not None:
            sd["arcweld_flat"] = {"m": self._flat["m"].cpu(), "v": self._flat["v"].cpu(),
                                  "step": int(self._flat["step"].item())}
        return sd
