"""Flat-buffer multi-tensor RAdam + global-norm clip on the HIP kernels.

Drop-in for ``torch.optim.RAdam`` as the reference builds it (model/autencoder_lightning_base.py:122-124;
model/transformer_decoder.py:64-114 -- two parameter groups that differ only in weight decay).  On the first
step the parameters of all groups are packed into ONE contiguous fp32 buffer and every ``p.data`` / ``p.grad``
is re-bound to a view of it, so that

* the optimizer update is one kernel over the flat buffer (segments carry per-group weight decay and an
  "active" flag -- a parameter that produced no gradient this stage is skipped, like torch skips grad None),
* the gradient all-reduce of data parallelism is a few large RCCL calls over the flat gradient buffer,
* conv weights declared centre-tap (declare_centre_tap) keep their provably-dead side taps out of the
  all-reduce, the norm and the update,
* k = 3 conv weights declared tap-major (declare_tap_major) are stored (O, 3, I) in their segment, so that the
  weight-gradient GEMM accumulates whole contiguous rows [O][3I] (the reference's (O, I, 3) order would scatter
  every atomic over three times the cache lines) and the forward operand [O][3I] is a plain cast of the segment,
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
        self._grads_zeroed = False

    # ------------------------------------------------------------------ flat layout
    def declare_centre_tap(self, params):
        """Conv weights (O, I, 3) whose side taps provably receive an exactly-zero gradient (a k = 3, pad = 1
        conv applied to length-1 inputs: the per-token encoder ResBlocks, model/vq_vae_patch_embedd.py:60-74,108-110).
        With weight decay 0 their side taps never change under RAdam (zero m, zero v -> zero update), so they are
        stored tap-major in one block [3][n][O][I] and only the centre-tap block is reduced, clipped and updated.
        The parameters become strided views (shape and values unchanged).  Call before the first flatten()."""
        if self._flat is not None:
            raise RuntimeError("declare_centre_tap must precede flatten()")
        self._centre = [p for p in params]

    def declare_tap_major(self, params):
        """k = 3 conv weights (O, I, 3) to store tap-major: each keeps its own segment of 3*O*I elements, laid out
        (O, 3, I); the parameter becomes the strided view .permute(0, 2, 1) of it (shape, values and state_dict
        unchanged).  RAdam, clip norm and all-reduce are elementwise over the segment, so nothing else changes.  Call
        before the first flatten()."""
        if self._flat is not None:
            raise RuntimeError("declare_tap_major must precede flatten()")
        self._tap_major = [p for p in params]

    def _build(self):
        params = [p for g in self.param_groups for p in g["params"]]
        dev = params[0].device
        if not all(p.device == dev and p.dtype == torch.float32 for p in params):
            raise RuntimeError("arcweld RAdam needs all parameters as float32 on one device")
        if dev.type != "cuda":
            raise RuntimeError("arcweld RAdam runs on the GPU only (no CPU fallback)")
        owner_of = {id(p): gi for gi, g in enumerate(self.param_groups) for p in g["params"]}
        centre = [p for p in getattr(self, "_centre", []) if id(p) in owner_of]
        if centre and not (all(p.dim() == 3 and p.shape == centre[0].shape and p.shape[2] == 3 for p in centre)
                           and len(set(owner_of[id(p)] for p in centre)) == 1
                           and float(self.param_groups[owner_of[id(centre[0])]]["weight_decay"]) == 0.0):
            centre = []          # the exactness argument needs one group, wd 0 and one (O, I, 3) shape
        cidx = {id(p): j for j, p in enumerate(centre)}
        tmaj = set(id(p) for p in getattr(self, "_tap_major", []) if id(p) in owner_of and id(p) not in cidx
                   and p.dim() == 3 and p.shape[2] == 3)
        al = lambda n: (n + 63) // 64 * 64      # 256-B aligned segments  # noqa: E731
        # segments: (param, offset, length, weight decay, group); a centre-tap param has ONE segment (its centre)
        segs, place, total, blk = [], {}, 0, None
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                if id(p) in cidx:
                    if blk is None:
                        blk = total
                        total += al(3 * len(centre) * centre[0][:, :, 0].numel())
                    oi = centre[0][:, :, 0].numel()
                    segs.append((p, blk + (len(centre) + cidx[id(p)]) * oi, oi, float(g["weight_decay"]), gi))
                    continue
                place[id(p)] = total
                segs.append((p, total, p.numel(), float(g["weight_decay"]), gi))
                total += al(p.numel())
        segs.sort(key=lambda s: s[1])          # the kernels find a segment by binary search over offsets
        flat_p = torch.zeros(total, device=dev)
        flat_g = torch.zeros(total, device=dev)

        def view(buf, p):
            if id(p) in cidx:
                O, I, _ = p.shape
                return buf[blk:blk + 3 * len(centre) * O * I].view(3, len(centre), O, I)[:, cidx[id(p)]].permute(1, 2, 0)
            o = place[id(p)]
            if id(p) in tmaj:
                O, I, _ = p.shape
                return buf[o:o + p.numel()].view(O, 3, I).permute(0, 2, 1)
            return buf[o:o + p.numel()].view_as(p)

        for p in params:
            view(flat_p, p).copy_(p.detach())
            if p.grad is not None:
                view(flat_g, p).copy_(p.grad)
            p.data = view(flat_p, p)
            p.grad = view(flat_g, p)
        # contiguous ranges holding every segment (alignment padding included, dead side-tap blocks excluded)
        spans = []
        for _, o, n, _, _ in segs:
            if spans and o <= al(spans[-1][1]):
                spans[-1][1] = max(spans[-1][1], o + n)
            else:
                spans.append([o, o + n])
        offs = [s[1] for s in segs]
        lens = [s[2] for s in segs]
        self._flat = dict(params=params, segs=segs, spans=[tuple(s) for s in spans], p=flat_p, g=flat_g,
                          m=torch.zeros(total, device=dev), v=torch.zeros(total, device=dev), total=total,
                          owner=[s[4] for s in segs], offs=offs, lens=lens,
                          off_d=torch.tensor(offs, device=dev, dtype=torch.int64),
                          len_d=torch.tensor(lens, device=dev, dtype=torch.int64),
                          wd_d=torch.tensor([s[3] for s in segs], device=dev, dtype=torch.float32),
                          ws=torch.zeros(K.NORM_WS, device=dev, dtype=torch.float64),
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
        self._grads_zeroed = False       # the fused zeroing covered the previous active set only
        keep = None if params is None else set(id(p) for p in params)
        act = [1 if keep is None or id(s[0]) in keep else 0 for s in F["segs"]]
        dev = F["p"].device
        F["act_d"] = torch.tensor(act, device=dev, dtype=torch.int32)
        F["act_group"] = [torch.tensor([a if o == gi else 0 for a, o in zip(act, F["owner"])], device=dev,
                                       dtype=torch.int32) for gi in range(len(self.param_groups))]

    def flat_offset(self, param):
        """Element offset of ``param``'s (first) segment in the flat buffers."""
        self.flatten()
        for s in self._flat["segs"]:
            if s[0] is param:
                return s[1]
        raise KeyError("parameter is not managed by this optimizer")

    def live_spans(self, lo=0, hi=None):
        """Contiguous [a, b) ranges of the flat buffers that hold gradients, clipped to [lo, hi): what a gradient
        all-reduce must move (the dead side-tap blocks of declare_centre_tap are left out)."""
        self.flatten()
        hi = self._flat["total"] if hi is None else hi
        return [(max(a, lo), min(b, hi)) for a, b in self._flat["spans"] if min(b, hi) > max(a, lo)]

    def param_spans(self, params):
        """Merged [a, b) ranges of the flat buffers holding the (live) segments of ``params``: what an all-reduce
        of just those gradients moves (alignment padding between adjacent segments included)."""
        self.flatten()
        keep = set(id(p) for p in params)
        al = lambda n: (n + 63) // 64 * 64   # noqa: E731
        spans = []
        for p, o, n, _, _ in self._flat["segs"]:
            if id(p) not in keep:
                continue
            if spans and o <= al(spans[-1][1]):
                spans[-1][1] = max(spans[-1][1], o + n)
            else:
                spans.append([o, o + n])
        return [tuple(x) for x in spans]

    def live_spans_excluding(self, spans):
        """live_spans() minus the given [a, b) ranges, each taken with its end rounded up to 64 elements as
        arcweld.trainer.allreduce_spans moves it: the zero padding after an excluded range is not all-reduced twice."""
        al = lambda n: (n + 63) // 64 * 64   # noqa: E731
        out = []
        for a, b in self.live_spans():
            cur = a
            for x, y in sorted((x, al(y)) for x, y in spans):
                if y <= cur or x >= b:
                    continue
                if x > cur:
                    out.append((cur, x))
                cur = max(cur, y)
            if cur < b:
                out.append((cur, b))
        return out

    def attach_operands(self, opset):
        """Keep the GEMM operand copies of ``opset`` (arcweld.operands.OperandSet) current from the update kernel
        (aw_radam_step_ops): each updated element is also cast into the copies of its parameter, so the step needs no
        relayout launch.  Returns False (and leaves the set refreshed per forward) when a copy's parameter is not in
        this optimizer or one parameter feeds more than AW_OPS_PER_SEG copies."""
        import ctypes
        from . import _native as nat
        self.flatten()
        F = self._flat
        seg_of = {id(sg[0]): i for i, sg in enumerate(F["segs"])}
        per = [[] for _ in F["segs"]]
        for j in opset.jobs:
            i = seg_of.get(id(j.param))
            if i is None:
                return False
            per[i].append(j)
        if any(len(x) > nat.OPS_PER_SEG for x in per):
            return False
        table = (nat.OperandDesc * (nat.OPS_PER_SEG * len(per)))()
        for i, js in enumerate(per):
            for k in range(nat.OPS_PER_SEG):
                d = table[nat.OPS_PER_SEG * i + k]
                if k >= len(js):
                    d.mode = -1
                    continue
                j = js[k]
                # the segment stores the parameter (O, I, k) contiguous, or only its [O][I] centre (declared
                # centre-tap: the job's source is then that centre view, k = 1)
                if j.src.numel() != F["segs"][i][2]:
                    return False
                _, O, I, k_, tap, mode, _, ldo = j.relayout_job()     # the mode for the source's storage order
                d.out = j.out.data_ptr()
                d.O, d.I, d.k, d.tap, d.mode, d.ldo = O, I, k_, tap, mode, ldo
                d.dtype = K.dtype_code(j.out.dtype)
        raw = torch.frombuffer(bytearray(bytes(table)), dtype=torch.uint8)
        F["ops_d"] = raw.to(F["p"].device)
        F["opset"] = opset
        opset.maintained = True
        return True

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
        if self._grads_zeroed:
            # the last step(zero_grad=True) zeroed every active segment; inactive ones carry no gradient
            self._grads_zeroed = False
            return
        g = self._flat["g"]
        for a, b in self._flat["spans"]:
            g[a:b].zero_()

    def clip_grad_norm_(self, max_norm):
        """L2 norm over the active gradients; the clip coefficient is applied inside the next step().
        Returns the (pre-clip) total norm as a device scalar."""
        self.flatten()
        F = self._flat
        K.grad_norm_clip(F["g"], F["off_d"], F["len_d"], F["act_d"], len(F["segs"]), max_norm, F["ws"], F["norm"],
                         F["coef"])
        self._coef = F["coef"]
        return F["norm"]

    @torch.no_grad()
    def step(self, closure=None, zero_grad=False):
        """torch.optim.RAdam.step; zero_grad=True also zeroes the gradients of the updated (active) segments in the
        same kernel pass, and the next zero_grad() call is then free (the Trainer's step + zero_grad pair)."""
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
            K.radam_step(F["p"], F["g"], F["m"], F["v"], F["off_d"], F["len_d"], F["wd_d"], act, len(F["segs"]),
                         F["total"], self._step_count, lr, b1, b2, eps, gscale=self._coef, step_ptr=F["step"],
                         ops=F.get("ops_d"), zero_grad=zero_grad)
        self._coef = None
        self._grads_zeroed = bool(zero_grad)
        return loss

    def _launch_groups(self):
        F = self._flat
        keys = [(float(g["lr"]), tuple(g["betas"]), float(g["eps"])) for g in self.param_groups]
        if len(set(keys)) == 1:
            return [(keys[0], F["act_d"])]
        return [(k, F["act_group"][gi]) for gi, k in enumerate(keys)]

    def state_dict(self):
        """torch's state_dict (param_groups; 'state' stays empty) plus 'arcweld_flat': the flat first/second moments
        and the device step counter, in this optimizer's flat layout (same parameters, same groups, same order)."""
        sd = super().state_dict()
        if self._flat is not None:
            sd["arcweld_flat"] = {"m": self._flat["m"].cpu(), "v": self._flat["v"].cpu(),
                                  "step": int(self._flat["step"].item()), "total": int(self._flat["total"])}
        return sd

    def load_state_dict(self, state_dict):
        """Restores the hyper-parameters of every group and, when present, the flat RAdam moments and step count
        (packing the parameters first).  The flat layout must be the one that wrote them."""
        sd = dict(state_dict)
        flat = sd.pop("arcweld_flat", None)
        super().load_state_dict(sd)
        if flat is None:
            return
        self.flatten()
        F = self._flat
        m, v = flat["m"], flat["v"]
        if m.numel() != F["total"] or v.numel() != F["total"] or int(flat.get("total", F["total"])) != F["total"]:
            raise ValueError(f"optimizer state holds a flat layout of {m.numel()} elements, this optimizer packs "
                             f"{F['total']} (different parameters, groups or centre-tap declaration)")
        F["m"].copy_(m.to(F["m"].device, torch.float32))
        F["v"].copy_(v.to(F["v"].device, torch.float32))
        self._step_count = int(flat["step"])
        F["step"].fill_(self._step_count)
