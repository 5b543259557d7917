"""Latent-token Transformer decoder -- drop-in for model/transformer_decoder.py:13-230 of the reference.

Same constructor, module tree / state_dict keys, initialisation, optimizer groups, task switching, step methods
and log keys.  One opt-in extension: ``pe_len`` (default 512, the reference's hard-coded positional table,
:22-23) sizes the sinusoidal table from its closed form (model/embedding.py:10-18) so that sequences longer than
512 tokens -- the stress configuration's T = 1025 -- can run; at the default the state_dict is the reference's.  forward() runs the fused HIP engine (arcweld.decoder): embedding, the pre-LN blocks (flash-style
causal attention, GEMM epilogues carrying bias/GELU/dropout/residual), ln_f and the task head; the losses are the
HIP cross-entropy kernels.
"""
import math

import torch
from torch import nn

from arcweld import decoder as engine
from arcweld.lightning import LightningModule
from arcweld.optim import RAdam
from model.embedding import LatentEmbedding
from model.transformer_block import Block


def _binary_scores(preds, y):
    """accuracy (multiclass, 2 classes, micro) and binary F1 of predicted labels (torchmetrics semantics)."""
    acc = (preds == y).float().mean()
    tp = ((preds == 1) & (y == 1)).sum().float()
    fp = ((preds == 1) & (y == 0)).sum().float()
    fn = ((preds == 0) & (y == 1)).sum().float()
    den = 2 * tp + fp + fn
    f1 = torch.where(den > 0, 2 * tp / den.clamp_min(1), torch.zeros_like(den))
    return acc, f1


class MyTransformerDecoder(LightningModule):

    def __init__(self, d_model: int = 64, n_classes: int = 131, seq_len: int = 100, n_blocks: int = 2,
                 n_head: int = 6, res_dropout=0.1, att_dropout=0.0, learning_rate: float = 1e-3,
                 class_h_bias: bool = False, class_h_dropout: bool = False, pe_len: int = 512):
        super().__init__()
        self.task = "generate"
        self.learning_rate = learning_rate
        self.betas = (0.9, 0.95)
        self.weight_decay = 0.1
        self.seq_len = seq_len
        self.d_model = d_model
        self.n_head = n_head
        self.n_classes = n_classes
        self.res_dropout = res_dropout
        self.embedding = LatentEmbedding(input_size=n_classes, d_model=d_model, seq_len=int(pe_len))
        self.transformer = nn.ModuleDict(dict(
            drop=nn.Dropout(res_dropout),
            h=nn.ModuleList([Block(d_model=d_model, seq_len=seq_len, n_head=n_head, res_dropout=res_dropout,
                                   att_dropout=att_dropout) for _ in range(n_blocks)]),
            ln_f=nn.LayerNorm(d_model),
        ))
        self.lm_head = nn.Linear(d_model, n_classes, bias=False)
        head = dict(linear_1=nn.Linear(d_model, 1, bias=class_h_bias), activation=nn.GELU(),
                    linear_2=nn.Linear(seq_len, 2, bias=class_h_bias))
        if class_h_dropout:
            head['dropout'] = nn.Dropout(p=0.1)      # registered but never applied (reference :38-39, :127-129)
        self.class_head = nn.ModuleDict(head)
        self.apply(self._init_weights)
        for pn, p in self.named_parameters():
            if pn.endswith('c_proj.weight'):
                torch.nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * n_blocks))
        n_params = sum(p.numel() for p in self.transformer.parameters())
        print("number of parameters: %.4fM" % (n_params / 1e6,))
        self.save_hyperparameters()

    def _init_weights(self, module):
        if isinstance(module, nn.Linear):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                torch.nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)
        elif isinstance(module, nn.LayerNorm):
            torch.nn.init.zeros_(module.bias)
            torch.nn.init.ones_(module.weight)

    def configure_optimizers(self):
        """Two RAdam groups: Linear weights decayed (0.1, L2 as torch.optim.RAdam), everything else not
        (reference :64-114)."""
        decay, no_decay = set(), set()
        for mn, m in self.named_modules():
            for pn, p in m.named_parameters():
                fpn = '%s.%s' % (mn, pn) if mn else pn
                if pn.endswith('bias'):
                    no_decay.add(fpn)
                elif pn.endswith('weight') and isinstance(m, nn.Linear):
                    decay.add(fpn)
                elif pn.endswith('weight') and isinstance(m, (nn.LayerNorm, nn.Embedding)):
                    no_decay.add(fpn)
        param_dict = dict(self.named_parameters())
        assert not (decay & no_decay), "parameters %s made it into both decay/no_decay sets!" % (decay & no_decay,)
        missing = param_dict.keys() - (decay | no_decay)
        assert not missing, "parameters %s were not separated into either decay/no_decay set!" % (missing,)
        groups = [
            {"params": [param_dict[pn] for pn in sorted(decay)], "weight_decay": self.weight_decay},
            {"params": [param_dict[pn] for pn in sorted(no_decay)], "weight_decay": 0.0},
        ]
        return RAdam(groups, lr=self.learning_rate, betas=self.betas)

    def _task_params(self, generate):
        ps = [self.embedding.latent_embedding.weight]
        for mod in list(self.transformer.h) + [self.transformer.ln_f]:
            ps += list(mod.parameters())
        if generate:
            ps.append(self.lm_head.weight)
        else:
            ps += list(self.class_head.parameters())
        return ps

    def active_parameters(self):
        """Parameters that receive a gradient in the current task (the other head is unused: its grad stays None
        under DDP(find_unused_parameters=True), train_transformer_mtasks.py:30)."""
        return self._task_params(self.task == "generate")

    def _next_seed(self):
        """Host part of the dropout seed: fixed per (torch seed, rank).  The per-call variation comes from the
        module's device-side counter (arcweld.vqvae.rng_snapshot), so eager calls and replays of a captured step
        graph draw the same sequence of masks."""
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        return (torch.initial_seed() * 1000003 + 7919 + (rank << 40)) & 0x7FFFFFFFFFFFFFFF

    def forward(self, x, generate: bool = True):
        """ids (B, T) -> logits (B, T, n_classes) [generate] or (B, 2) [classification] (reference :116-131)."""
        B, T = x.size()
        mask_len = self.transformer.h[0].attn.bias.shape[-1] if len(self.transformer.h) else T
        if T > mask_len:
            raise RuntimeError(f"The size of tensor a ({mask_len}) must match the size of tensor b ({T}) at "
                               "non-singleton dimension 3 (causal mask has seq_len rows, transformer_block.py:53)")
        params = tuple(self._task_params(generate))
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return engine.DecoderFunction.apply(self, x, generate, self._next_seed(), *params)
        out, _ = engine.forward(self, x, generate, self.training, need_backward=False, seed=self._next_seed())
        return out

    def _loss_scale_tensor(self, scale, dev):
        """Persistent device scalar holding the loss scale, one per (scale, device) and never freed: the step graphs
        make it before their capture (the captured step has no fill launch for it) and keep reading its address, so a
        later call with another scale gets a tensor of its own instead of replacing one a graph still holds."""
        cache = self.__dict__.setdefault("_gscale", {})
        key = (float(scale), str(dev))
        if key not in cache:
            cache[key] = torch.full((1,), scale, device=dev)
        return cache[key]

    # the captured step may run a whole accumulation group as one batch (fused_train_step(groups=G),
    # arcweld.graphs.StepGraphs)
    grouped_accumulation = True

    @torch.no_grad()
    def fused_train_step(self, batch, scale, mid_hook=None, groups=1):
        """One training micro-step on the kernels without autograd: training_step followed by
        ``(loss * scale).backward()``.  Gradients accumulate into each parameter's ``.grad`` (the flat optimizer
        views when a Trainer installed ``_grad_sink``); ``mid_hook`` runs once backward_late_parameters() are final
        (arcweld.decoder.backward).  groups = G: `batch` is the G micro-batches of an accumulation group concatenated
        along the sequences, each with its own loss mean (arcweld.decoder.fused_step).  Returns the loss."""
        sink = getattr(self, "_grad_sink", None)

        def slot(p):
            if sink is not None and p in sink:
                return sink[p]
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            return p.grad

        loss, logits = engine.fused_step(self, batch, scale, slot, mid_hook=mid_hook, groups=groups)
        if self.task == "generate":
            self.log('train/loss', loss, prog_bar=True)
        else:
            self.log_classification_results(loss, logits, batch[1], "train")
        return loss

    def operand_set(self):
        """The persistent GEMM operand copies of the training step (arcweld.operands), for the optimizer to keep
        current (arcweld.optim.RAdam.attach_operands)."""
        return engine.operand_set(self)

    def backward_late_parameters(self):
        """Parameters whose gradients are final at fused_train_step's mid_hook (the task head, ln_f, the later half
        of the blocks): a data-parallel step all-reduces them while the earlier blocks' backward runs."""
        return engine.late_parameters(self, self.task == "generate")

    def switch_to_generate(self):
        self.task = "generate"

    def switch_to_classification(self):
        self.task = "classification"

    def _step(self, batch):
        if self.task == "generate":
            return self.step_task_gen(batch)
        elif self.task == "classification":
            return self.step_task_class(batch)

    def step_task_gen(self, batch):
        x, _, y = batch
        logits = self(x, generate=True)
        loss = self.loss_gen(logits, y)
        return loss, logits, y

    def step_task_class(self, batch):
        x, cond, _ = batch
        logits = self(x, generate=False)
        loss = self.loss_class(logits, cond)
        return loss, logits, cond

    def log_classification_results(self, loss, logits, y, ds_type):
        preds = logits.argmax(dim=1)         # argmax(log_softmax) == argmax(logits)
        acc, f1score = _binary_scores(preds, y)
        sync_dist = on_epoch = ds_type in ("val", "test")
        self.log(f'{ds_type}/cl/loss', loss, sync_dist=sync_dist, on_epoch=on_epoch)
        self.log(f'{ds_type}/cl/acc', acc, prog_bar=False, sync_dist=sync_dist, on_epoch=on_epoch)
        self.log(f'{ds_type}/cl/f1_score', f1score, prog_bar=True, sync_dist=sync_dist, on_epoch=on_epoch)

    def training_step(self, batch, batch_idx):
        loss, logits, labels = self._step(batch)
        if self.task == "generate":
            self.log('train/loss', loss, prog_bar=True)
        else:
            self.log_classification_results(loss, logits, labels, "train")
        return loss

    def validation_step(self, batch, batch_idx):
        loss, logits, labels = self._step(batch)
        if self.task == "generate":
            self.log('val/loss', loss, prog_bar=True, sync_dist=True)
        else:
            self.log_classification_results(loss, logits, labels, "val")
        return loss

    def test_step(self, batch, batch_idx):
        loss, logits, labels = self._step(batch)
        if self.task == "generate":
            self.log('test/loss', loss, prog_bar=True)
        else:
            self.log_classification_results(loss, logits, labels, "test")
        return loss

    def generate(self, x, do_sample=False, top_k=None, use_cache=True):
        """Autoregressive continuation by seq_len tokens (reference :203-224): greedy (top-1) or multinomial
        sampling, context cropped to the last seq_len tokens.

        use_cache (default): the prompt is prefilled once and each new token is one cached decode step
        (arcweld.decoder.forward_cached, aw_attn_decode); once the context is cropped every position moves, so
        those steps re-prefill the window -- what the reference computes at every step.  use_cache=False runs
        the reference's full recompute through forward()."""
        if use_cache:
            return self._generate_cached(x, do_sample, top_k)
        with torch.no_grad():
            for _ in range(self.seq_len):
                x_cond = x if x.size(1) <= self.seq_len else x[:, -self.seq_len:]
                logits = self(x_cond)
                if top_k is not None:
                    logits = logits.clone()
                    v, _ = torch.topk(logits, top_k)
                    logits[logits < v[:, [-1]]] = -float('Inf')
                probs = torch.softmax(logits, dim=-1)[:, -1]
                if do_sample:
                    idx_next = torch.multinomial(probs, num_samples=1)
                else:
                    _, idx_next = torch.topk(probs, k=1, dim=-1)
                x = torch.cat([x, idx_next], dim=-1)
        return x

    @torch.no_grad()
    def _generate_cached(self, x, do_sample, top_k):
        cache = engine.KVCache(self, x.size(0), self.seq_len)
        filled = 0                      # positions of x[:, :filled] are in the cache
        for _ in range(self.seq_len):
            L = x.size(1)
            if L > self.seq_len:        # cropped window: every position shifted, prefill it again
                logits = engine.forward_cached(self, x[:, -self.seq_len:], cache, 0)
                filled = 0
            elif filled == 0:
                logits = engine.forward_cached(self, x, cache, 0)
                filled = L
            else:
                logits = engine.forward_cached(self, x[:, filled:], cache, filled)
                filled = L
            if top_k is not None:
                v, _ = torch.topk(logits, top_k)
                logits = logits.masked_fill(logits < v[:, [-1]], -float('Inf'))
            probs = torch.softmax(logits, dim=-1)
            if do_sample:
                idx_next = torch.multinomial(probs, num_samples=1)
            else:
                _, idx_next = torch.topk(probs, k=1, dim=-1)
            x = torch.cat([x, idx_next], dim=-1)
        return x

    def loss_gen(self, logits, labels):
        return engine.cross_entropy(logits.view(-1, logits.size(-1)), labels.view(-1), ignore_index=-1)

    def loss_class(self, logits, labels):
        return engine.cross_entropy(logits, labels)
