"""Autograd for the building blocks used on their own: PatchEmbedding, ResBlock stacks (CNNBlock), SepCNNBlock,
PatchEmbeddingInverse, Block, LatentEmbedding(Cond).

The training entry points run whole models as one fused node (arcweld.vqvae / arcweld.decoder); the reference's
sub-modules are ordinary autograd modules as well (model/vq_vae_patch_embedd.py:7-114, model/transformer_block.py,
model/embedding.py), so each one here has its own forward (saving what its backward reads) and backward on the same
HIP kernels -- the per-block pieces of the fused passes, with the weight operands built per call (the persistent,
optimizer-maintained copies belong to the fused models).

Every function takes and returns the reference's layouts: (B, C, S) channel-major for the conv blocks, (B, T, d) for
the transformer block.  Dropout draws a fresh host seed per call (the masks are counter-based; the backward
regenerates them from the seed).
"""
from __future__ import annotations

import torch

from . import kernels as K
from . import vqvae as engine
from .vqvae import _mix, operand_dtype

F32 = torch.float32


def _empty(dev):
    return lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731


def _seed(p):
    return int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0


def _tokens(x_bcs, T):
    """(B, C, S) channel-major -> token-major (B*S, C) contiguous in dtype T."""
    B, C, S = x_bcs.shape
    out = torch.empty(B * S, C, device=x_bcs.device, dtype=T)
    out.view(B, S, C).copy_(x_bcs.permute(0, 2, 1))
    return out


def _channel_major(t_nc, B, S):
    return t_nc.view(B, S, -1).permute(0, 2, 1)


def _masked_copy(g, T, p, seed):
    """Operand copy of g [N][H] (dtype T) with the dropout mask of (p, seed) applied: the GEMM epilogue over an
    empty contraction (v = 0 + resid, C2 = mask(v))."""
    N, H = g.shape
    out = torch.empty(N, H, device=g.device, dtype=T)
    dummy = torch.zeros(8, 8, device=g.device, dtype=T)
    K.gemm(dummy, dummy, N, H, 0, resid=g, C2=out, c2_mode=3, drop2=(p, seed))
    return out


def _cast(t, T):
    if t.dtype == T:
        return t.contiguous()
    out = torch.empty(t.shape, device=t.device, dtype=T)
    K.cast(t.contiguous(), out)
    return out


class _Saved:
    pass


class ModuleFunction(torch.autograd.Function):
    """(fwd, bwd, x, *params) -> fwd(x)[0]; backward: bwd(saved, g, slot, need_x) -> grad of x (or None) with the
    parameter gradients accumulated into slot(param)."""

    @staticmethod
    def forward(ctx, fwd, bwd, x, *params):
        out, saved = fwd(x, True)
        ctx.bwd, ctx.saved, ctx.params = bwd, saved, params
        return out

    @staticmethod
    def backward(ctx, g):
        grads = {}

        def slot(p):
            t = grads.get(p)
            if t is None:
                t = torch.zeros_like(p, dtype=F32)
                grads[p] = t
            return t

        gx = ctx.bwd(ctx.saved, g.contiguous(), slot, ctx.needs_input_grad[2])
        ctx.saved = None
        return (None, None, gx) + tuple(grads.get(p) for p in ctx.params)


def needs_graph(mod, *tensors):
    """True when the call must record an autograd node (grad mode on and anything requires grad)."""
    return torch.is_grad_enabled() and (any(t.requires_grad for t in tensors if t.is_floating_point()) or
                                        any(p.requires_grad for p in mod.parameters()))


def run(mod, fwd, bwd, x):
    """Forward of a sub-module: an autograd node when needed, otherwise the plain kernel forward."""
    if needs_graph(mod, x):
        params = tuple(p for p in mod.parameters())
        return ModuleFunction.apply(fwd, bwd, x, *params)
    with torch.no_grad():
        return fwd(x, False)[0]


# ------------------------------------------------------------------------------------------- PatchEmbedding
def patch_embed(mod, x):
    """(B, L, C) -> (B, H, S): channel-major flatten + Conv1d(1, H, k=P, s=P) (vq_vae_patch_embedd.py:7-17)."""
    P, H = mod.patch_size, mod.proj.out_channels
    T = operand_dtype()

    def fwd(x, save):
        x = x.contiguous().float()
        B, L, C = x.shape
        S = L * C // P
        ldp = (P + 7) // 8 * 8
        e = _empty(x.device)
        patches = e(B * S, ldp, dt=T)
        K.patchify(x, P, patches)
        W = torch.zeros(H, ldp, device=x.device, dtype=T)
        K.weight_relayout(mod.proj.weight, H, 1, P, 0, 4, W, ldo=ldp)
        out = e(B * S, H)
        K.gemm(patches, W, B * S, H, ldp, bias=mod.proj.bias, C=out)
        sv = _Saved()
        sv.shape, sv.patches, sv.W, sv.ldp = (B, L, C, S), patches, W, ldp
        return _channel_major(out, B, S), sv

    def bwd(sv, g, slot, need_x):
        B, L, C, S = sv.shape
        N = B * S
        gt = _tokens(g, T)
        K.gemm(gt, sv.patches, H, P, N, a_trans=True, b_trans=True, C=slot(mod.proj.weight).view(H, P),
               accumulate=True, a_rowsum=slot(mod.proj.bias))
        if not need_x:
            return None
        gp = torch.empty(N, sv.ldp, device=g.device)
        K.gemm(gt, sv.W, N, sv.ldp, H, b_trans=True, C=gp)
        # patches[b*S + t][j] = x[b, l, c] with t*P + j = c*L + l: the inverse is a view of the patch rows
        return gp[:, :P].reshape(B, C, L).permute(0, 2, 1).contiguous()

    return run(mod, fwd, bwd, x)


# ------------------------------------------------------------------------------------------- ResBlock stacks
def cnn_block(mod, x):
    """CNNBlock (vq_vae_patch_embedd.py:93-114): (B, H, S) -> (B, H, S).  seperate=True: every token on its own
    (centre taps), False: k=3 convolutions along the token axis; BatchNorm ResBlocks when batch_norm."""
    return _resblock_stack(mod, list(mod.shared_conv), mod.seperate, mod.batch_norm, mod.dropout_p, x)


def resblock(mod, x):
    """ResBlock.forward (vq_vae_patch_embedd.py:73-74): x + block(x) on (B, C, L), both convs k = 3 / pad = 1 along
    L (an L = 1 slice -- the per-token encoder -- leaves only the centre tap, as in the reference)."""
    c1 = mod.block[1]
    if tuple(c1.kernel_size) != (3,) or tuple(c1.stride) != (1,) or tuple(c1.padding) != (1,):
        raise NotImplementedError("ResBlock on the HIP path: kernel_size 3, stride 1, padding 1 (the reference's use)")
    bn = isinstance(mod.block[2], torch.nn.BatchNorm1d)
    return _resblock_stack(mod, [mod], False, bn, float(mod.block[6].p), x)


def _resblock_stack(mod, blocks, sep, batch_norm, dropout_p, x):
    """A stack of ResBlocks (the module `mod` owns their parameters) as one autograd node."""
    T = operand_dtype()

    def fwd(x, save):
        B, H, S = x.shape
        N = B * S
        e = _empty(x.device)
        training = mod.training
        p = dropout_p if training else 0.0
        seed = _seed(p)
        cur = _tokens(x, F32)
        a0 = _gelu_operand(cur, T)
        conv = None if sep else (H, S, 1, 0)
        kd = H if sep else 3 * H
        sv = _Saved()
        sv.shape, sv.p, sv.training, sv.blocks = (B, H, S), p, training, []
        for r, blk in enumerate(blocks):
            c1, c2 = blk.block[1], blk.block[4]
            if sep:
                w1, w2 = e(H, H, dt=T), e(H, H, dt=T)
                K.weight_relayout_batch([engine._centre_job(c1.weight, w1), engine._centre_job(c2.weight, w2)])
            else:
                w1, w2 = e(H, 3 * H, dt=T), e(H, 3 * H, dt=T)
                K.weight_relayout_batch([engine._conv3_job(c1.weight, 1, w1), engine._conv3_job(c2.weight, 1, w2)])
            sr = _mix(seed, r)
            if batch_norm:   # per-token statistics when the tokens run separately, over all positions otherwise
                gk = {} if conv is None else dict(conv=conv)
                y, an, bs = engine._bn_block_fwd(a0, cur, w1, w2, kd, gk, c1, c2, (blk.block[2], blk.block[5]),
                                                 S if sep else 1, training, p, sr, None, T)
            else:
                h, a1 = e(N, H, dt=T), e(N, H, dt=T)
                K.gemm(a0, w1, N, H, kd, conv=conv, bias=c1.bias, C=h, C2=a1, c2_mode=1)
                y, an = e(N, H), e(N, H, dt=T)
                K.gemm(a1, w2, N, H, kd, conv=conv, bias=c2.bias, drop=(p, sr), resid=cur, C=y, C2=an, c2_mode=1)
                bs = (h, a1)
            if save:
                sv.blocks.append((cur, a0, bs, w1, w2, sr))
            cur, a0 = y, an
        return _channel_major(cur, B, S), sv

    def bwd(sv, g, slot, need_x):
        B, H, S = sv.shape
        N = B * S
        p = sv.p
        e = _empty(g.device)
        kd = H if sep else 3 * H
        dconv = None if sep else (H, S, -1, 0)
        wconv = (H, S, 1, 1)

        def wg(c, A, Bm):
            if sep:
                Cw, cm = engine._centre_grad(slot(c.weight))
                return (A, Bm, H, H, N, dict(a_trans=True, b_trans=True, C=Cw, accumulate=True, col_map=cm,
                                             a_rowsum=slot(c.bias)))
            Cw, cm = engine._conv3_grad(slot(c.weight))
            return (A, Bm, H, 3 * H, N, dict(a_trans=True, b_trans=True, conv=wconv, C=Cw, accumulate=True,
                                             col_map=cm, a_rowsum=slot(c.bias)))

        gy = _tokens(g, F32)
        nb = len(blocks)
        go = _masked_copy(gy, T, p, sv.blocks[-1][5]) if (nb and not batch_norm) else None
        wgrads = []
        for r in reversed(range(nb)):
            blk = blocks[r]
            c1, c2 = blk.block[1], blk.block[4]
            xr, a0, bs, w1, w2, sr = sv.blocks[r]
            if sep:
                W1d, W2d = w1, w2
            else:   # dgrad operands [3O][I]
                W1d, W2d = e(3 * H, H, dt=T), e(3 * H, H, dt=T)
                K.weight_relayout_batch([engine._conv3_job(c1.weight, 2, W1d), engine._conv3_job(c2.weight, 2, W2d)])
            if batch_norm:
                gk = {} if dconv is None else dict(conv=dconv)
                gy, _ = engine._bn_block_bwd(gy, xr, a0, bs, W1d, W2d, kd, gk, wg, c1, c2, (blk.block[2], blk.block[5]),
                                             S if sep else 1, sv.training, p, sr, None, T, slot, wgrads,
                                             need_copy=False)
                continue
            h, a1 = bs
            gh = e(N, H, dt=T)
            K.gemm(go, W2d, N, H, kd, b_trans=True, conv=dconv, pre=h, C=gh)
            wgrads.append(wg(c2, go, a1))
            gyn = e(N, H)
            gon = e(N, H, dt=T) if r > 0 else None
            K.gemm(gh, W1d, N, H, kd, b_trans=True, conv=dconv, pre=xr, resid=gy, C=gyn, C2=gon,
                   c2_mode=3 if r > 0 else 0, drop2=(p, sv.blocks[r - 1][5] if r > 0 else 0))
            wgrads.append(wg(c1, gh, a0))
            gy, go = gyn, gon
        K.gemm_grouped(wgrads)
        if not need_x:
            return None
        if nb == 0:
            return g
        return _channel_major(gy, B, S).contiguous()

    return run(mod, fwd, bwd, x)


def _gelu_operand(x, T):
    N, H = x.shape
    out = torch.empty(N, H, device=x.device, dtype=T)
    dummy = torch.zeros(8, 8, device=x.device, dtype=T)
    K.gemm(dummy, dummy, N, H, 0, resid=x, C2=out, c2_mode=1)
    return out


# ------------------------------------------------------------------------------------------- SepCNNBlock
def sep_cnn(mod, x):
    """SepCNNBlock (vq_vae_patch_embedd.py:77-91): (B, H, S) -> (B, S, D), per-token Conv1d(H, D, 1)."""
    T = operand_dtype()
    conv = mod.shared_conv
    D = conv.out_channels

    def fwd(x, save):
        B, H, S = x.shape
        N = B * S
        xt = _tokens(x, T)
        W = torch.empty(D, H, device=x.device, dtype=T)
        K.weight_relayout(conv.weight, D, H, 1, 0, 0, W)
        z = torch.empty(N, D, device=x.device)
        K.gemm(xt, W, N, D, H, bias=conv.bias, C=z)
        sv = _Saved()
        sv.shape, sv.xt, sv.W = (B, H, S), xt, W
        return z.view(B, S, D), sv

    def bwd(sv, g, slot, need_x):
        B, H, S = sv.shape
        N = B * S
        gz = _cast(g.reshape(N, D), T)
        K.gemm(gz, sv.xt, D, H, N, a_trans=True, b_trans=True, C=slot(conv.weight).view(D, H), accumulate=True,
               a_rowsum=slot(conv.bias))
        if not need_x:
            return None
        gx = torch.empty(N, H, device=g.device)
        K.gemm(gz, sv.W, N, H, D, b_trans=True, C=gx)
        return _channel_major(gx, B, S).contiguous()

    return run(mod, fwd, bwd, x)


# ------------------------------------------------------------------------------------------- PatchEmbeddingInverse
def patch_unembed(mod, x):
    """PatchEmbeddingInverse (vq_vae_patch_embedd.py:19-57): ConvT(H, H, k1) -> BatchNorm1d -> GELU ->
    ConvT(H, 1, 5, 5); (B, H, S) -> (B, L, input_dim)."""
    T = operand_dtype()
    k1 = mod.k1
    t1, bn, t2 = mod.proj[0], mod.proj[1], mod.proj[3]

    def fwd(x, save):
        B, H, S = x.shape
        N = B * S
        e = _empty(x.device)
        xt = _tokens(x, T)
        W = e(k1 * H, H, dt=T)
        K.weight_relayout(t1.weight, H, H, k1, 0, 3, W)
        Y = e(N, k1 * H)
        training = mod.training
        cs = torch.zeros(2 * H, device=x.device, dtype=torch.float64) if training else None
        K.gemm(xt, W, N, k1 * H, H, bias=t1.bias, bias_mod=H, C=Y, colstats=cs, stats_mod=H)
        stats = e(4 * H)
        K.bn_finalize(cs, N * k1, H, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                      bn.num_batches_tracked if training else None, bn.eps,
                      bn.momentum if bn.momentum is not None else 0.1, training, stats)
        Q = S * k1
        out = e(B, Q * 5 // mod.input_dim, mod.input_dim)
        K.unpatch_head_fwd(Y.view(N * k1, H), Q, stats, t2.weight.view(H, 5), t2.bias, out)
        sv = _Saved()
        sv.shape, sv.xt, sv.W, sv.Y, sv.stats, sv.training = (B, H, S), xt, W, Y, stats, training
        return out, sv

    def bwd(sv, g, slot, need_x):
        B, H, S = sv.shape
        N = B * S
        e = _empty(g.device)
        Y2 = sv.Y.view(N * k1, H)
        gsums = torch.zeros(2 * H, device=g.device, dtype=torch.float64)
        w2 = t2.weight.view(H, 5)
        K.unpatch_head_bwd1(Y2, S * k1, sv.stats, w2, g, gsums, slot(t2.weight).view(H, 5), slot(t2.bias),
                            slot(bn.weight), slot(bn.bias))
        gY = e(N * k1, H, dt=T)
        K.unpatch_head_bwd2(Y2, S * k1, sv.stats, w2, g, gsums, sv.training, gY, slot(t1.bias))
        gY2 = gY.view(N, k1 * H)
        K.gemm(sv.xt, gY2, H, k1 * H, N, a_trans=True, b_trans=True, C=slot(t1.weight).view(H, H * k1),
               accumulate=True, col_map=(H, k1, 0))
        if not need_x:
            return None
        gx = e(N, H)
        K.gemm(gY2, sv.W, N, H, k1 * H, b_trans=True, C=gx)
        return _channel_major(gx, B, S).contiguous()

    return run(mod, fwd, bwd, x)


# ------------------------------------------------------------------------------------------- transformer pieces
def causal_self_attention(mod, x):
    """CausalSelfAttention.forward (transformer_block.py:40-63): resid_drop(c_proj(softmax(mask(q k^T / sqrt(hs)))
    v)) on (B, T, d) -- QKV GEMM, flash attention (probability dropout inside the kernel), c_proj GEMM with the
    residual dropout in its epilogue."""
    Td = operand_dtype()
    nh = mod.n_head

    def fwd(x, save):
        B, T, d = x.shape
        R = B * T
        e = _empty(x.device)
        training = mod.training
        p = float(mod.resid_dropout.p) if training else 0.0
        pa = float(mod.attn_pdrop) if training else 0.0
        s_res, s_probs = _seed(p), _seed(pa)
        xa = _cast(x.reshape(R, d), Td)
        Wqkv, Wo = _cast(mod.c_attn.weight, Td), _cast(mod.c_proj.weight, Td)
        qkv = e(R, 3 * d, dt=Td)
        K.gemm(xa, Wqkv, R, 3 * d, d, bias=mod.c_attn.bias, C=qkv)
        y, lse = e(R, d, dt=Td), e(B * nh * T)
        K.attn_fwd(qkv, B, T, nh, d, y, lse, drop=(pa, s_probs))
        out = e(R, d)
        K.gemm(y, Wo, R, d, d, bias=mod.c_proj.bias, drop=(p, s_res), C=out)
        sv = _Saved()
        sv.shape, sv.p, sv.pa, sv.seeds = (B, T, d), p, pa, (s_res, s_probs)
        if save:
            sv.c = dict(xa=xa, qkv=qkv, y=y, lse=lse, Wqkv=Wqkv, Wo=Wo)
        return out.view(B, T, d), sv

    def bwd(sv, g, slot, need_x):
        B, T, d = sv.shape
        R = B * T
        e = _empty(g.device)
        c = sv.c
        s_res, s_probs = sv.seeds
        go = _masked_copy(g.reshape(R, d).float().contiguous(), Td, sv.p, s_res)
        gy = e(R, d, dt=Td)
        K.gemm(go, c["Wo"], R, d, d, b_trans=True, C=gy)
        K.gemm(go, c["y"], d, d, R, a_trans=True, b_trans=True, C=slot(mod.c_proj.weight), accumulate=True,
               a_rowsum=slot(mod.c_proj.bias))
        dqkv = e(R, 3 * d, dt=Td)
        ws = e(B * nh * T)
        K.attn_bwd(c["qkv"], c["y"], gy, c["lse"], B, T, nh, d, dqkv, ws, drop=(sv.pa, s_probs))
        K.gemm(dqkv, c["xa"], 3 * d, d, R, a_trans=True, b_trans=True, C=slot(mod.c_attn.weight), accumulate=True,
               a_rowsum=slot(mod.c_attn.bias))
        if not need_x:
            return None
        gx = e(R, d)
        K.gemm(dqkv, c["Wqkv"], R, d, 3 * d, b_trans=True, C=gx)
        return gx.view(B, T, d)

    return run(mod, fwd, bwd, x)


def mlp(mod, x):
    """Block.mlpf (transformer_block.py:81-83): dropout(c_proj(NewGELU(c_fc(x)))) on (..., d); `mod` is the block's
    ``mlp`` ModuleDict.  The tanh-GELU and the dropout run in the GEMM epilogues."""
    Td = operand_dtype()

    def fwd(x, save):
        shape = x.shape
        d = shape[-1]
        R = x.numel() // d
        e = _empty(x.device)
        training = mod.training
        p = float(mod["dropout"].p) if training else 0.0
        s = _seed(p)
        xa = _cast(x.reshape(R, d), Td)
        Wfc, Wp = _cast(mod["c_fc"].weight, Td), _cast(mod["c_proj"].weight, Td)
        dh = Wfc.shape[0]
        h, gl = e(R, dh, dt=Td), e(R, dh, dt=Td)
        K.gemm(xa, Wfc, R, dh, d, bias=mod["c_fc"].bias, act=K.AW_ACT_GELU_TANH, C=h, C2=gl, c2_mode=1)
        out = e(R, d)
        K.gemm(gl, Wp, R, d, dh, bias=mod["c_proj"].bias, drop=(p, s), C=out)
        sv = _Saved()
        sv.shape, sv.p, sv.seed = shape, p, s
        if save:
            sv.c = dict(xa=xa, h=h, g=gl, Wfc=Wfc, Wp=Wp)
        return out.view(shape), sv

    def bwd(sv, g, slot, need_x):
        d = sv.shape[-1]
        R = g.numel() // d
        e = _empty(g.device)
        c = sv.c
        dh = c["Wfc"].shape[0]
        go = _masked_copy(g.reshape(R, d).float().contiguous(), Td, sv.p, sv.seed)
        gh = e(R, dh, dt=Td)
        K.gemm(go, c["Wp"], R, dh, d, b_trans=True, act=K.AW_ACT_GELU_TANH, pre=c["h"], C=gh)
        K.gemm(go, c["g"], d, dh, R, a_trans=True, b_trans=True, C=slot(mod["c_proj"].weight), accumulate=True,
               a_rowsum=slot(mod["c_proj"].bias))
        K.gemm(gh, c["xa"], dh, d, R, a_trans=True, b_trans=True, C=slot(mod["c_fc"].weight), accumulate=True,
               a_rowsum=slot(mod["c_fc"].bias))
        if not need_x:
            return None
        gx = e(R, d)
        K.gemm(gh, c["Wfc"], R, d, dh, b_trans=True, C=gx)
        return gx.view(sv.shape)

    return run(mod, fwd, bwd, x)


# ------------------------------------------------------------------------------------------- transformer Block
def block(mod, x):
    """Block (transformer_block.py:66-88): x + drop(attn(ln_1(x))); x + drop(mlp(ln_2(x))), (B, T, d)."""
    Td = operand_dtype()
    at, mlp = mod.attn, mod.mlp
    nh = at.n_head

    def fwd(x, save):
        B, T, d = x.shape
        R = B * T
        e = _empty(x.device)
        training = mod.training
        p = float(mod.res_dropout) if training else 0.0
        pa = float(at.attn_pdrop) if training else 0.0
        s_attn, s_mlp, s_probs = _seed(p), _seed(p), _seed(pa)
        xr = x.reshape(R, d).contiguous().float()
        Wqkv, Wo = _cast(at.c_attn.weight, Td), _cast(at.c_proj.weight, Td)
        Wfc, Wp = _cast(mlp.c_fc.weight, Td), _cast(mlp.c_proj.weight, Td)
        a, mu1, rs1 = e(R, d, dt=Td), e(R), e(R)
        K.layernorm_fwd(xr, mod.ln_1.weight, mod.ln_1.bias, mod.ln_1.eps, a, mu1, rs1)
        qkv = e(R, 3 * d, dt=Td)
        K.gemm(a, Wqkv, R, 3 * d, d, bias=at.c_attn.bias, C=qkv)
        y, lse = e(R, d, dt=Td), e(B * nh * T)
        K.attn_fwd(qkv, B, T, nh, d, y, lse, drop=(pa, s_probs))
        x1 = e(R, d)
        K.gemm(y, Wo, R, d, d, bias=at.c_proj.bias, drop=(p, s_attn), resid=xr, C=x1)
        a2, mu2, rs2 = e(R, d, dt=Td), e(R), e(R)
        K.layernorm_fwd(x1, mod.ln_2.weight, mod.ln_2.bias, mod.ln_2.eps, a2, mu2, rs2)
        h, gl = e(R, 4 * d, dt=Td), e(R, 4 * d, dt=Td)
        K.gemm(a2, Wfc, R, 4 * d, d, bias=mlp.c_fc.bias, act=K.AW_ACT_GELU_TANH, C=h, C2=gl, c2_mode=1)
        x2 = e(R, d)
        K.gemm(gl, Wp, R, d, 4 * d, bias=mlp.c_proj.bias, drop=(p, s_mlp), resid=x1, C=x2)
        sv = _Saved()
        sv.shape, sv.p, sv.pa, sv.seeds = (B, T, d), p, pa, (s_attn, s_mlp, s_probs)
        if save:
            sv.c = dict(x=xr, a=a, mu1=mu1, rs1=rs1, qkv=qkv, y=y, lse=lse, x1=x1, a2=a2, mu2=mu2, rs2=rs2, h=h,
                        g=gl, Wqkv=Wqkv, Wo=Wo, Wfc=Wfc, Wp=Wp)
        return x2.view(B, T, d), sv

    def bwd(sv, g, slot, need_x):
        B, T, d = sv.shape
        R = B * T
        e = _empty(g.device)
        c = sv.c
        p, pa = sv.p, sv.pa
        s_attn, s_mlp, s_probs = sv.seeds
        gx = g.reshape(R, d).float().clone()     # residual-stream gradient; the LayerNorm backwards add into it
        go = _masked_copy(gx, Td, p, s_mlp)
        # ---- MLP
        gh = e(R, 4 * d, dt=Td)
        K.gemm(go, c["Wp"], R, 4 * d, d, b_trans=True, act=K.AW_ACT_GELU_TANH, pre=c["h"], C=gh)
        K.gemm(go, c["g"], d, 4 * d, R, a_trans=True, b_trans=True, C=slot(mlp.c_proj.weight), accumulate=True,
               a_rowsum=slot(mlp.c_proj.bias))
        ga2 = e(R, d)
        K.gemm(gh, c["Wfc"], R, d, 4 * d, b_trans=True, C=ga2)
        K.gemm(gh, c["a2"], 4 * d, d, R, a_trans=True, b_trans=True, C=slot(mlp.c_fc.weight), accumulate=True,
               a_rowsum=slot(mlp.c_fc.bias))
        go2 = e(R, d, dt=Td)
        K.layernorm_bwd(c["x1"], ga2, mod.ln_2.weight, c["mu2"], c["rs2"], gx, True, slot(mod.ln_2.weight),
                        slot(mod.ln_2.bias), dx2=go2, drop=(p, s_attn))
        # ---- attention
        gy = e(R, d, dt=Td)
        K.gemm(go2, c["Wo"], R, d, d, b_trans=True, C=gy)
        K.gemm(go2, c["y"], d, d, R, a_trans=True, b_trans=True, C=slot(at.c_proj.weight), accumulate=True,
               a_rowsum=slot(at.c_proj.bias))
        dqkv = e(R, 3 * d, dt=Td)
        ws = e(B * nh * T)
        K.attn_bwd(c["qkv"], c["y"], gy, c["lse"], B, T, nh, d, dqkv, ws, drop=(pa, s_probs))
        K.gemm(dqkv, c["a"], 3 * d, d, R, a_trans=True, b_trans=True, C=slot(at.c_attn.weight), accumulate=True,
               a_rowsum=slot(at.c_attn.bias))
        ga = e(R, d)
        K.gemm(dqkv, c["Wqkv"], R, d, 3 * d, b_trans=True, C=ga)
        K.layernorm_bwd(c["x"], ga, mod.ln_1.weight, c["mu1"], c["rs1"], gx, True, slot(mod.ln_1.weight),
                        slot(mod.ln_1.bias))
        return gx.view(B, T, d) if need_x else None

    return run(mod, fwd, bwd, x)


# ------------------------------------------------------------------------------------------- embeddings
def latent_embedding(mod, ids, cond=None, cond_weight=None):
    """latent_embedding(ids) + pe[:T] (+ cond_embedding(cond) on every position, LatentEmbeddingCond;
    model/embedding.py:27-59).  The gradients go to the embedding tables (scatter-add per token)."""
    W = mod.latent_embedding.weight
    pe = mod.positional_embedding.pe

    def fwd(ids, save):
        B, T = ids.shape
        if T > pe.shape[1]:
            raise RuntimeError(f"The size of tensor a ({T}) must match the size of tensor b ({pe.shape[1]}) at "
                               "non-singleton dimension 1")
        R = B * T
        ids = ids.contiguous()
        out = torch.empty(R, W.shape[1], device=ids.device)
        K.embed_fwd(ids, W, pe[0], out)
        cids = None
        if cond is not None:      # + cond_embedding(cond)[b] on each of the T positions of window b
            cids = cond.reshape(B, 1).expand(B, T).reshape(1, R).contiguous()
            out2 = torch.empty_like(out)
            K.embed_fwd(cids, cond_weight, out, out2)     # "positional" rows = the R rows just written
            out = out2
        sv = _Saved()
        sv.ids, sv.cids, sv.shape = ids, cids, (B, T)
        return out.view(B, T, -1), sv

    def bwd(sv, g, slot, need_x):
        B, T = sv.shape
        g2 = g.reshape(B * T, -1).float().contiguous()
        K.embed_bwd(sv.ids, g2, slot(W))
        if sv.cids is not None:
            K.embed_bwd(sv.cids, g2, slot(cond_weight))
        return None

    return run(mod, fwd, bwd, ids)
