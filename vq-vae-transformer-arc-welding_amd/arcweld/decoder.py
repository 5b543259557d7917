"""Fused latent-Transformer (MyTransformerDecoder) forward/backward on the HIP kernels.

Reference: model/transformer_decoder.py:13-131 (+ model/transformer_block.py, model/embedding.py).
Rows are the R = B*T tokens of a batch, row = b*T + t.  Per block:

  a   = LN1(x)                       aw_layernorm_fwd (operand dtype)
  qkv = a . Wqkv^T + b               aw_gemm                        [R][3d]
  y   = causal attention(qkv)        aw_attn_fwd (flash-style, lse saved; the T x T matrix never exists)
  x1  = x + drop(y . Wo^T + bo)      aw_gemm (bias + dropout + residual fused)
  a2  = LN2(x1)
  h   = a2 . Wfc^T + bfc             aw_gemm, C = h (f32, for GELU') and C2 = GELU_tanh(h) (f32 operands); bf16:
                                     C = GELU_tanh(h) and C2 = GELU_tanh'(h) (c2_mode 4, the backward's multiplier)
  x2  = x1 + drop(g . Wp^T + bp)     aw_gemm

Heads: lm_head (logits [R][V], ld padded to 8) + cross-entropy(ignore_index=-1), or the classification head
(linear_1 -> GELU(erf) -> linear_2 over the sequence axis) + cross-entropy.  The backward mirrors the forward;
dropout masks are regenerated from (seed, element), LayerNorm backward emits the masked operand of the preceding
projection's gradient GEMMs directly.
"""
from __future__ import annotations

import torch

from . import kernels as K
from . import operands
from .vqvae import _mix, operand_dtype, rng_snapshot

F32 = torch.float32


def _pad8(n):
    return (n + 7) // 8 * 8


class DecSaved:
    pass


def _cast(t, T):
    if t.dtype == T:
        return t
    out = torch.empty(t.shape, device=t.device, dtype=T)
    K.cast(t, out)
    return out


def _operand_jobs(m, T_):
    """Operand copies of the training step: the blocks' Linear weights in the operand dtype (when it is not f32)
    and the lm head zero-padded to a multiple of 8 rows."""
    from .operands import OperandJob as J
    jobs = []
    for i, blk in enumerate(m.transformer.h):
        for nm, lin in (("qkv", blk.attn.c_attn), ("o", blk.attn.c_proj), ("fc", blk.mlp.c_fc), ("p", blk.mlp.c_proj)):
            w = lin.weight
            if w.dtype != T_:
                jobs.append(J(f"b{i}_{nm}", w, w.shape[0], w.shape[1], 1, 0, 5,
                              torch.empty(w.shape, device=w.device, dtype=T_)))
    w = m.lm_head.weight
    jobs.append(J("Wlm", w, w.shape[0], w.shape[1], 1, 0, 5,
                  torch.zeros(_pad8(w.shape[0]), w.shape[1], device=w.device, dtype=T_)))
    return jobs


def operand_set(m, T=None):
    """The OperandSet the training step of `m` reads (for arcweld.optim.RAdam.attach_operands)."""
    T_ = operand_dtype(T)
    return operands.peek(m, ("decoder", T_), lambda: _operand_jobs(m, T_))


def forward(m, ids, generate: bool, training: bool, need_backward: bool, seed: int = 0, dtype=None, zero=None):
    """ids (B, T) int64 -> logits (B, T, V) [generate] or (B, 2) [classify]."""
    T_ = operand_dtype(dtype)
    B, T = ids.shape
    d = m.d_model
    nh = m.n_head
    R = B * T
    dev = ids.device
    V = m.n_classes
    pe = m.embedding.positional_embedding.pe
    if T > pe.shape[1]:
        raise RuntimeError(f"The size of tensor a ({T}) must match the size of tensor b ({pe.shape[1]}) at "
                           f"non-singleton dimension 1 (positional table capped at {pe.shape[1]} rows, "
                           "model/embedding.py:49-50)")
    if (not generate) and T != m.seq_len:
        raise RuntimeError(f"classification head expects T == seq_len ({m.seq_len}), got {T}")
    e = lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
    p_drop = float(m.res_dropout) if training else 0.0
    sv = DecSaved()
    sv.B, sv.T, sv.R, sv.d, sv.nh, sv.V, sv.Tdt, sv.generate = B, T, R, d, nh, V, T_, generate
    sv.p_drop = p_drop
    nb = len(m.transformer.h)
    # attention-probability dropout (CausalSelfAttention.attn_dropout; reference default 0.0)
    sv.p_att = float(m.transformer.h[0].attn.attn_pdrop) if (training and nb) else 0.0
    sv.seed_attn = [_mix(seed, 300 + i) for i in range(nb)]
    sv.seed_mlp = [_mix(seed, 400 + i) for i in range(nb)]
    sv.seed_probs = [_mix(seed, 500 + i) for i in range(nb)]
    sv.ctr = rng_snapshot(m, dev, max(p_drop, sv.p_att), zero=zero)   # zero: a caller's f64 accumulators
    ids = ids.contiguous()

    x = e(R, d)
    # the first block's ln_1 runs inside the embedding launch when the vector LayerNorm form applies (d_model
    # 256..1024): the same arithmetic, without re-reading x
    ln0 = None
    if nb and d in (256, 512, 768, 1024):
        l1 = m.transformer.h[0].ln_1
        ln0 = (e(R, d, dt=T_), e(R), e(R))
        K.embed_ln_fwd(ids, m.embedding.latent_embedding.weight, pe[0], x, l1.weight, l1.bias, l1.eps, *ln0)
    else:
        K.embed_fwd(ids, m.embedding.latent_embedding.weight, pe[0], x)
    # operand copies of every block's Linear weights and the padded lm head (f32 Linear operands are used as they
    # are): persistent, re-cast only when a weight changed outside the optimizer (arcweld/operands.py)
    ops = operands.get(m, ("decoder", T_), lambda: _operand_jobs(m, T_))
    wops = [[ops.get(f"b{i}_{nm}", lin.weight)
             for nm, lin in (("qkv", blk.attn.c_attn), ("o", blk.attn.c_proj), ("fc", blk.mlp.c_fc),
                             ("p", blk.mlp.c_proj))] for i, blk in enumerate(m.transformer.h)]
    blocks = []
    for i, blk in enumerate(m.transformer.h):
        at, mlp = blk.attn, blk.mlp
        Wqkv, Wo, Wfc, Wp = wops[i]
        if i == 0 and ln0 is not None:
            a, mu1, rs1 = ln0
        else:
            a, mu1, rs1 = e(R, d, dt=T_), e(R), e(R)
            K.layernorm_fwd(x, blk.ln_1.weight, blk.ln_1.bias, blk.ln_1.eps, a, mu1, rs1)
        qkv = e(R, 3 * d, dt=T_)
        K.gemm(a, Wqkv, R, 3 * d, d, bias=at.c_attn.bias, C=qkv)
        y, lse = e(R, d, dt=T_), e(B * nh * T)
        K.attn_fwd(qkv, B, T, nh, d, y, lse, drop=(sv.p_att, sv.seed_probs[i]), seed_ptr=sv.ctr)
        x1 = e(R, d)
        K.gemm(y, Wo, R, d, d, bias=at.c_proj.bias, drop=(p_drop, sv.seed_attn[i]), resid=x, C=x1,
               seed_ptr=sv.ctr)
        a2, mu2, rs2 = e(R, d, dt=T_), e(R), e(R)
        K.layernorm_fwd(x1, blk.ln_2.weight, blk.ln_2.bias, blk.ln_2.eps, a2, mu2, rs2)
        if T_ == F32:   # exact mode: the pre-activation h, the backward evaluates GELU'(h) (h: f32)
            h, g = e(R, 4 * d, dt=T_), e(R, 4 * d, dt=T_)
            K.gemm(a2, Wfc, R, 4 * d, d, bias=mlp.c_fc.bias, act=K.AW_ACT_GELU_TANH, C=h, C2=g, c2_mode=1)
        else:
            # bf16: g = GELU(h) and GELU'(h) from one exponential (c2_mode 4), the derivative saved in place of h
            # (same bytes); the backward multiplies by it instead of evaluating GELU' of the bf16 pre-activation
            g, h = e(R, 4 * d, dt=T_), e(R, 4 * d, dt=T_)
            K.gemm(a2, Wfc, R, 4 * d, d, bias=mlp.c_fc.bias, act=K.AW_ACT_GELU_TANH, C=g, C2=h, c2_mode=4)
        x2 = e(R, d)
        K.gemm(g, Wp, R, d, 4 * d, bias=mlp.c_proj.bias, drop=(p_drop, sv.seed_mlp[i]), resid=x1, C=x2,
               seed_ptr=sv.ctr)
        blocks.append(dict(x=x, a=a, mu1=mu1, rs1=rs1, qkv=qkv, y=y, lse=lse, x1=x1, a2=a2, mu2=mu2, rs2=rs2, h=h, g=g,
                           Wqkv=Wqkv, Wo=Wo, Wfc=Wfc, Wp=Wp))
        x = x2
    lnf = m.transformer.ln_f
    xf_dt = T_ if generate else F32
    xf, muf, rsf = e(R, d, dt=xf_dt), e(R), e(R)
    K.layernorm_fwd(x, lnf.weight, lnf.bias, lnf.eps, xf, muf, rsf)
    sv.blocks, sv.x_last, sv.xf, sv.muf, sv.rsf = blocks, x, xf, muf, rsf
    if generate:
        Vp = _pad8(V)
        Wlm = ops["Wlm"]        # [Vp][d]: padded rows stay zero (K padding of the dgrad)
        logits_buf = e(R, Vp)
        logits = logits_buf[:, :V]
        # over the padded width: the zero rows of Wlm give exact zeros in the padding columns, and N = Vp (a
        # multiple of 8) takes the vectorised specialised epilogue instead of the generic one (N = V = 514)
        K.gemm(xf, Wlm, R, Vp, d, C=logits_buf)
        sv.Wlm, sv.logits_buf, sv.Vp = Wlm, logits_buf, Vp
        out = logits.view(B, T, V)
    else:
        ch = m.class_head
        s, out = e(R), e(B, 2)
        K.class_head_fwd(xf, B, T, ch.linear_1.weight, ch.linear_1.bias, ch.linear_2.weight, ch.linear_2.bias, s, out)
        sv.s = s
    return out, (sv if need_backward else None)


def late_parameters(m, generate):
    """Parameters whose gradients are final at backward()'s mid_hook: the task head, ln_f and blocks
    nb//2 .. nb-1 (the backward reaches them first; their weight gradients are issued before the hook)."""
    nb = len(m.transformer.h)
    ps = [m.lm_head.weight] if generate else list(m.class_head.parameters())
    ps += list(m.transformer.ln_f.parameters())
    for blk in list(m.transformer.h)[nb // 2:]:
        ps += list(blk.parameters())
    return ps


def backward(m, sv, g_out, slot, mid_hook=None):
    """g_out: gradient of the logits (B, T, V) f32 or of the class logits (B, 2).  ``mid_hook()`` runs once the
    gradients of late_parameters(m, generate) are final (a data-parallel step starts their all-reduce there, which
    then overlaps the backward of the earlier blocks)."""
    B, T, R, d, nh, V, T_ = sv.B, sv.T, sv.R, sv.d, sv.nh, sv.V, sv.Tdt
    dev = g_out.device
    e = lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
    lnf = m.transformer.ln_f
    nb = len(sv.blocks)
    if sv.generate:
        Vp = sv.Vp
        gl = getattr(sv, "gl", None)      # fused_step: the cross-entropy backward already wrote the padded operand
        if gl is None:
            gl = torch.zeros(R, Vp, device=dev, dtype=T_)
            # strided cast into the zero-padded operand: GEMM epilogue with an empty contraction (v = 0 + resid)
            K.gemm(gl, gl, R, V, 0, resid=g_out.reshape(R, V).contiguous(), C=gl[:, :V])
        # lm_head weight gradient [V][d] and input gradient (K padded to Vp with zero rows/columns)
        K.gemm(gl[:, :V], sv.xf, V, d, R, a_trans=True, b_trans=True, C=slot(m.lm_head.weight), accumulate=True)
        gxf = e(R, d)
        K.gemm(gl, sv.Wlm, R, d, Vp, b_trans=True, C=gxf)
    else:
        ch = m.class_head
        gxf = e(R, d)
        b1 = ch.linear_1.bias
        b2 = ch.linear_2.bias
        K.class_head_bwd(sv.xf, sv.s, g_out.contiguous(), B, T, ch.linear_1.weight, ch.linear_2.weight, gxf,
                         slot(ch.linear_1.weight), slot(b1) if b1 is not None else None,
                         slot(ch.linear_2.weight), slot(b2) if b2 is not None else None)
    # ln_f backward -> residual-stream gradient gx (f32) + masked operand for the last block's MLP projection
    gx = e(R, d)
    go = e(R, d, dt=T_)
    last = nb - 1
    K.layernorm_bwd(sv.x_last, gxf, lnf.weight, sv.muf, sv.rsf, gx, False, slot(lnf.weight), slot(lnf.bias),
                    dx2=go, drop=(sv.p_drop, sv.seed_mlp[last] if nb else 0), seed_ptr=sv.ctr)
    # the weight gradients are deferred and issued as one batch per half, the first before the mid-backward hook (a
    # data-parallel step reduces the later half's gradients while the earlier blocks run); with no collective
    # (m._wgrad_merge, set by the step graphs) or no hook, all blocks in one batch at the end (384 tiles split in two
    # pieces instead of 2 x 192 in four: a third of the split-K slab traffic and one launch fewer)
    wg = {"fc2": [], "fc1": [], "proj": [], "qkv": []}
    half = nb // 2
    for i in reversed(range(nb)):
        blk = m.transformer.h[i]
        at, mlp = blk.attn, blk.mlp
        c = sv.blocks[i]
        # ---- MLP
        gh = e(R, 4 * d, dt=T_)
        # c["h"]: the pre-activation (f32 mode) or its saved GELU' (bf16 mode, forward c2_mode 4)
        K.gemm(go, c["Wp"], R, 4 * d, d, b_trans=True, act=K.AW_ACT_GELU_TANH if T_ == F32 else K.AW_ACT_DERIV,
               pre=c["h"], C=gh)
        wg["fc2"].append((go, c["g"], d, 4 * d, R, dict(a_trans=True, b_trans=True, C=slot(mlp.c_proj.weight),
                                                         accumulate=True, a_rowsum=slot(mlp.c_proj.bias))))
        ga2 = e(R, d)
        K.gemm(gh, c["Wfc"], R, d, 4 * d, b_trans=True, C=ga2)
        wg["fc1"].append((gh, c["a2"], 4 * d, d, R, dict(a_trans=True, b_trans=True, C=slot(mlp.c_fc.weight),
                                                          accumulate=True, a_rowsum=slot(mlp.c_fc.bias))))
        go2 = e(R, d, dt=T_)
        K.layernorm_bwd(c["x1"], ga2, blk.ln_2.weight, c["mu2"], c["rs2"], gx, True, slot(blk.ln_2.weight),
                        slot(blk.ln_2.bias), dx2=go2, drop=(sv.p_drop, sv.seed_attn[i]),
                        seed_ptr=sv.ctr)
        # ---- attention
        gy = e(R, d, dt=T_)
        K.gemm(go2, c["Wo"], R, d, d, b_trans=True, C=gy)
        wg["proj"].append((go2, c["y"], d, d, R, dict(a_trans=True, b_trans=True, C=slot(at.c_proj.weight),
                                                       accumulate=True, a_rowsum=slot(at.c_proj.bias))))
        dqkv = e(R, 3 * d, dt=T_)
        ws = e(B * nh * T)
        K.attn_bwd(c["qkv"], c["y"], gy, c["lse"], B, T, nh, d, dqkv, ws, drop=(sv.p_att, sv.seed_probs[i]),
                   seed_ptr=sv.ctr)
        wg["qkv"].append((dqkv, c["a"], 3 * d, d, R, dict(a_trans=True, b_trans=True, C=slot(at.c_attn.weight),
                                                           accumulate=True, a_rowsum=slot(at.c_attn.bias))))
        ga = e(R, d)
        K.gemm(dqkv, c["Wqkv"], R, d, 3 * d, b_trans=True, C=ga)
        go = e(R, d, dt=T_) if i > 0 else None
        K.layernorm_bwd(c["x"], ga, blk.ln_1.weight, c["mu1"], c["rs1"], gx, True, slot(blk.ln_1.weight),
                        slot(blk.ln_1.bias), dx2=go, drop=(sv.p_drop, sv.seed_mlp[i - 1] if i > 0 else 0),
                        seed_ptr=sv.ctr)
        if i == half and mid_hook is not None:
            if not m.__dict__.get("_wgrad_merge", False):
                # the four kinds of the later half of the blocks: one batch (bf16) or one grouped launch per kind
                K.wgrad_issue([pb for kind in wg for pb in wg[kind]])
                wg = {kind: [] for kind in wg}
            mid_hook()
    K.wgrad_issue([pb for kind in wg for pb in wg[kind]])
    if nb == 0 and mid_hook is not None:
        mid_hook()
    # the table gradient by counting sort + one owner per element (aw_embed_bwd_sorted: 18 + 25 us against 48 us of
    # contended atomics at 16371 rows into 514; a side-stream sort at the forward measured slower, step +0.4 %)
    K.embed_bwd(sv_ids(sv), gx, slot(m.embedding.latent_embedding.weight))


def sv_ids(sv):
    return sv.ids


class DecoderFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, m, ids, generate, seed, *params):
        out, sv = forward(m, ids, generate, m.training, need_backward=True, seed=seed)
        sv.ids = ids.contiguous()
        ctx.m, ctx.sv, ctx.params = m, sv, params
        return out

    @staticmethod
    def backward(ctx, g_out):
        m, sv = ctx.m, ctx.sv
        sink = getattr(m, "_grad_sink", None)
        grads = {}

        def slot(p):
            if sink is not None and p in sink:
                return sink[p]
            g = grads.get(p)
            if g is None:
                g = torch.zeros_like(p, dtype=F32)
                grads[p] = g
            return g

        backward(m, sv, g_out.contiguous(), slot)
        ctx.sv = None
        return (None, None, None, None) + tuple(grads.get(p) for p in ctx.params)


class _CrossEntropy(torch.autograd.Function):
    """F.cross_entropy (mean over non-ignored rows) on the HIP kernels (transformer_decoder.py:226-230)."""

    @staticmethod
    def forward(ctx, logits2d, target, ignore_index):
        R, V = logits2d.shape
        lse = torch.empty(R, device=logits2d.device)
        s = torch.zeros(2, device=logits2d.device, dtype=torch.float64)
        K.ce_fwd(logits2d, V, target.contiguous(), ignore_index, s[0:1], s[1:2], lse)
        out = torch.empty((), device=logits2d.device)
        K.ce_finalize(s[0:1], s[1:2], out)
        ctx.save_for_backward(logits2d, target, lse, s)
        ctx.ignore = ignore_index
        return out

    @staticmethod
    def backward(ctx, g):
        logits2d, target, lse, s = ctx.saved_tensors
        R, V = logits2d.shape
        dl = torch.empty(R, V, device=logits2d.device)
        K.ce_bwd(logits2d, V, target.contiguous(), ctx.ignore, lse, s[1:2], g.reshape(1).contiguous(), dl)
        return dl, None, None


def fused_step(m, batch, scale, slot, mid_hook=None, groups=1):
    """forward + cross-entropy + backward of one micro-batch of the current task, without autograd: the work of
    training_step followed by (loss * scale).backward() (model/transformer_decoder.py:139-155, 226-230).  Returns
    (loss, logits).

    groups = G > 1: the batch is the G equal micro-batches of one accumulation group, concatenated along the
    sequences (accumulate_grad_batches, train_transformer_mtasks.py:32): each micro-batch's loss is its own mean
    over its own valid tokens (one cross-entropy reduction per group), so the summed gradient is Lightning's sum of
    the G micro-batch gradients; the returned loss is the mean of the G losses.  Every row draws its own dropout
    mask from the one counter range of this forward.  RNG stream: the G eager micro-steps draw G seeds (one
    _next_seed() each), the grouped step one, so with dropout > 0 an eager and a graphed run of the same seed draw
    different (equally distributed, independent per row) masks; runs are reproducible within either path, and the
    eager-vs-grouped equivalence tests run at dropout 0 (tests/test_training_regime.py)."""
    x, cond, y = batch
    generate = m.task == "generate"
    dev = x.device
    G = int(groups)
    if G < 1 or x.shape[0] % G:
        raise ValueError(f"fused_step: {x.shape[0]} sequences do not split into {G} equal micro-batches")
    sums = torch.empty(G, 2, device=dev, dtype=torch.float64)  # zeroed by the forward's dropout-counter launch
    out, sv = forward(m, x, generate, m.training, need_backward=True, seed=m._next_seed(), zero=sums)
    sv.ids = x.contiguous()
    if generate:
        logits2d = out.view(-1, out.shape[-1])          # rows of stride Vp (the padded logits buffer)
        target, ignore = y.reshape(-1).contiguous(), -1
    else:
        logits2d, target, ignore = out, cond.reshape(-1).contiguous(), -100
    R, V = logits2d.shape
    Rg = R // G
    rows = [slice(j * Rg, (j + 1) * Rg) for j in range(G)]
    lse = torch.empty(R, device=dev)
    for j, sl in enumerate(rows):
        K.ce_fwd(logits2d[sl], V, target[sl], ignore, sums[j, 0:1], sums[j, 1:2], lse[sl])
    losses = torch.empty(G, device=dev)
    for j in range(G):
        K.ce_finalize(sums[j, 0:1], sums[j, 1:2], losses[j:j + 1])
    loss = losses[0] if G == 1 else losses.mean()
    g = m._loss_scale_tensor(float(scale), dev) if hasattr(m, "_loss_scale_tensor") else \
        torch.full((1,), float(scale), device=dev)
    if generate:
        # the logits gradient straight into the zero-padded [R][Vp] operand of the lm_head GEMMs, in the operand
        # dtype (aw_ce_bwd zeroes the padding columns): no f32 copy, no strided cast launch
        gl = torch.empty(R, sv.Vp, device=dev, dtype=sv.Tdt)
        dl = gl[:, :V]
        sv.gl = gl
    else:
        dl = torch.empty(R, V, device=dev)
    for j, sl in enumerate(rows):
        K.ce_bwd(logits2d[sl], V, target[sl], ignore, lse[sl], sums[j, 1:2], g, dl[sl])
    backward(m, sv, dl.view(out.shape), slot, mid_hook=mid_hook)
    return loss, out


def cross_entropy(logits2d, target, ignore_index=-100):
    if logits2d.stride(-1) != 1:
        raise ValueError("logits rows must be contiguous")
    return _CrossEntropy.apply(logits2d, target, ignore_index)


class KVCache:
    """Per-block key/value cache for incremental decoding: (B, Tmax, 2d) rows [K | V] in the operand dtype, plus
    the operand copies of the block weights (cast once per generate call)."""

    def __init__(self, m, B, Tmax, dtype=None):
        self.T_ = operand_dtype(dtype)
        dev = m.lm_head.weight.device
        d = m.d_model
        self.B, self.Tmax = B, Tmax
        self.kv = [torch.empty(B, Tmax, 2 * d, device=dev, dtype=self.T_) for _ in m.transformer.h]
        self.wops, casts = [], []
        for blk in m.transformer.h:
            ws = []
            for lin in (blk.attn.c_attn, blk.attn.c_proj, blk.mlp.c_fc, blk.mlp.c_proj):
                w = lin.weight
                if self.T_ == w.dtype:
                    ws.append(w)
                else:
                    o = torch.empty(w.shape, device=dev, dtype=self.T_)
                    casts.append((w, w.shape[0], w.shape[1], 1, 0, 5, o))
                    ws.append(o)
            self.wops.append(ws)
        K.weight_relayout_batch(casts)
        V = m.n_classes
        self.Wlm = torch.zeros(_pad8(V), d, device=dev, dtype=self.T_)
        K.cast(m.lm_head.weight, self.Wlm[:V])


@torch.no_grad()
def forward_cached(m, ids_new, cache: KVCache, pos0: int):
    """Eval forward of n_new tokens per sequence at positions pos0 .. pos0+n_new-1 against the cached keys and
    values of positions < pos0 (appending their own); returns the logits of the LAST new position (B, V) f32.
    pos0 = 0 with the whole prompt is the prefill; n_new = 1 the decode step (model/transformer_decoder.py:203-224
    recomputes the whole prefix instead -- same values, the cached keys of a position never change while the
    context is not cropped)."""
    B, n = ids_new.shape
    d, nh, V = m.d_model, m.n_head, m.n_classes
    T_ = cache.T_
    if pos0 + n > cache.Tmax:
        raise RuntimeError(f"KV cache holds {cache.Tmax} positions, asked for {pos0 + n}")
    pe = m.embedding.positional_embedding.pe
    if pos0 + n > pe.shape[1]:
        raise RuntimeError(f"positions beyond the positional table ({pe.shape[1]} rows, model/embedding.py:49-50)")
    R = B * n
    dev = ids_new.device
    e = lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
    x = e(R, d)
    K.embed_fwd(ids_new.contiguous(), m.embedding.latent_embedding.weight, pe[0, pos0:], x)
    for i, blk in enumerate(m.transformer.h):
        at, mlp = blk.attn, blk.mlp
        Wqkv, Wo, Wfc, Wp = cache.wops[i]
        a, mu, rs = e(R, d, dt=T_), e(R), e(R)
        K.layernorm_fwd(x, blk.ln_1.weight, blk.ln_1.bias, blk.ln_1.eps, a, mu, rs)
        qkv = e(R, 3 * d, dt=T_)
        K.gemm(a, Wqkv, R, 3 * d, d, bias=at.c_attn.bias, C=qkv)
        y = e(R, d, dt=T_)
        K.attn_decode(qkv, B, n, pos0, nh, d, cache.kv[i], y)
        x1 = e(R, d)
        K.gemm(y, Wo, R, d, d, bias=at.c_proj.bias, resid=x, C=x1)
        a2 = e(R, d, dt=T_)
        K.layernorm_fwd(x1, blk.ln_2.weight, blk.ln_2.bias, blk.ln_2.eps, a2, mu, rs)
        h, g = e(R, 4 * d, dt=T_), e(R, 4 * d, dt=T_)
        K.gemm(a2, Wfc, R, 4 * d, d, bias=mlp.c_fc.bias, act=K.AW_ACT_GELU_TANH, C=h, C2=g, c2_mode=1)
        x2 = e(R, d)
        K.gemm(g, Wp, R, d, 4 * d, bias=mlp.c_proj.bias, resid=x1, C=x2)
        x = x2
    lnf = m.transformer.ln_f
    xf, muf, rsf = e(R, d, dt=T_), e(R), e(R)
    K.layernorm_fwd(x, lnf.weight, lnf.bias, lnf.eps, xf, muf, rsf)
    last = xf.view(B, n, d)[:, n - 1]                     # (B, d) rows of stride n*d: the GEMM takes lda
    logits = e(B, V)
    K.gemm(last, cache.Wlm, B, V, d, C=logits)
    return logits
