"""Fused VQ-VAE-Patch training path on the HIP kernels (model/vq_vae_patch_embedd.py:117-167).

Activations are TOKEN-MAJOR: a batch of B windows is N = B*S token rows of H channels, row = b*S + t, with the
reference's channel-major patch order (tokens 0..S/2-1 voltage, S/2..S-1 current).  Every dense contraction is
one ``aw_gemm`` launch:

  patch embed   (N x ldp) . Wp^T            -> x0 (f32) + gelu(x0) (operand dtype)
  enc ResBlock  a0 . W1c^T -> h, gelu(h);  a1 . W2c^T + b, dropout, + x  -> x', gelu(x')   (centre taps only)
  sep conv      x_R . Ws^T                  -> z (f32)
  VQ            aw_vq_forward (fp32, bit-exact argmin)
  dec 1x1       zq . Wd0^T                  -> y0, gelu(y0)
  dec ResBlock  implicit k=3 conv GEMMs (K = 3H, rows shifted within each window)
  ConvT(H->H)   y_R . Wt1r^T (N = k1*H)     -> Y (f32) + BatchNorm column statistics in the epilogue
  head          BN -> GELU -> ConvT(H->1) -> x_hat, one wave per position

The backward mirrors it (input-gradient GEMMs with the GELU' and dropout masks fused in the epilogues,
weight-gradient GEMMs with the bias gradient fused as an A-row-sum).  Operands are exact fp32 MFMA by default
(the reference's numerics on MI355X); bf16 MFMA with fp32 accumulation is an explicit opt-in (arcweld.precision).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import _native as nat
from . import kernels as K
from . import operands
from .precision import operand_dtype  # noqa: F401  (re-exported: model/ and arcweld.decoder import it from here)

F32 = torch.float32


def _mix(seed: int, salt: int) -> int:
    z = (seed * 0x9E3779B97F4A7C15 + salt * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    z ^= z >> 31
    z = (z * 0xD6E8FEB86659FD93) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 32)


def rng_snapshot(m, dev, p_drop, zero=None):
    """Advance the module's device-side dropout counter and return a device copy of it for this forward (None
    when no dropout is active).  The kernels mix it into the host seeds (aw_gemm_args.seed_ptr), so a captured
    HIP graph draws fresh masks on every replay and the backward regenerates exactly the forward's masks.
    `zero` (a float64 block, the forward's accumulators) is zeroed by the same launch."""
    if p_drop <= 0.0:
        if zero is not None:
            zero.zero_()
        return None
    ctr = getattr(m, "_rng_counter", None)
    if ctr is None or ctr.device != dev:
        ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        m._rng_counter = ctr
    snap = torch.empty(1, dtype=torch.int64, device=dev)
    K.counter_add_snapshot(ctr, snap, zero=zero)      # advance, snapshot (and zero) in one launch
    return snap


# partial code histograms of the VQ forward (aw_vq_forward_ex2): workgroup b adds into partial b % 8, so no more
# than N / (64 * 8) workgroups add into one address (at 1, every workgroup's adds into the same 2 KB serialised at
# the memory-side atomic units: 2.5 us of the configs[1] kernel)
VQ_COUNT_GROUPS = 8


def accumulators(m, dev, K, H, zero=True):
    """Device accumulators of one forward, carved from one persistent f64 block (zeroed by ONE launch: here, or by
    rng_snapshot's when zero=False and the caller passes it the "block"): VQ sqerr (f64), MSE sqerr (f64,
    fused_train_step), BN column statistics (2H f64) and the VQ code counts (VQ_COUNT_GROUPS partial histograms of K
    f32, summed by aw_vq_finalize_ex).  Each is consumed inside the call that filled it (never across a
    forward/backward boundary)."""
    key = (dev, K, H)
    st = m.__dict__.get("_acc_block")
    if st is None or st[0] != key:
        st = (key, torch.empty(2 + 4 * H + (VQ_COUNT_GROUPS * K + 1) // 2, dtype=torch.float64, device=dev))
        m.__dict__["_acc_block"] = st
    buf = st[1]
    if zero:
        buf.zero_()
    return dict(block=buf, vq_sq=buf[0:1], mse_sq=buf[1:2], colstats=buf[2:2 + 2 * H], head_gsums=buf[2 + 2 * H:2 + 4 * H],
                counts=buf[2 + 4 * H:].view(torch.float32)[:VQ_COUNT_GROUPS * K])


def resid_dtype(m, T):
    """dtype of the ResBlock residual streams (the activations x, y and their gradients) of the fused step.

    Exact-fp32 operands keep them in fp32 (the reference's numerics).  In the bf16 operand mode they are bf16, which
    is what the reference under bf16 autocast holds: its conv outputs are bf16, so x + block(x) and its gradient are
    bf16 tensors (model/vq_vae_patch_embedd.py:73-74) -- half the epilogue bytes of the 32 residual launches per step.
    ``--batchnorm 1`` keeps fp32 streams (its BatchNorm kernels read f32), as does ARCWELD_RESID_F32=1 (A/B)."""
    if T == F32 or m.batch_norm or os.environ.get("ARCWELD_RESID_F32", "0") == "1":
        return F32
    return T


class VQVAEShapes:
    def __init__(self, m, B):
        self.B = B
        self.H, self.D, self.K = m.hidden_dim, m.embedding_dim, m.num_embeddings
        self.R = m.n_resblocks
        self.P, self.L, self.C = m.patch_size, m.seq_len, m.input_dim
        self.S = self.L * self.C // self.P
        self.N = B * self.S
        self.k1 = m.reverse_patch_embed.k1
        self.Q = self.S * self.k1
        self.ldp = (self.P + 7) // 8 * 8


def _params(m):
    """Reference-layout parameter tensors of a VQVAEPatch, by role."""
    enc = [(blk.block[1], blk.block[4]) for blk in m.encoder[0].shared_conv]
    dec = [(blk.block[1], blk.block[4]) for blk in m.decoder[1].shared_conv]
    # --batchnorm 1: the BatchNorm1d after each ResBlock conv (block[2], block[5]); None with Identity
    enc_bn = [(blk.block[2], blk.block[5]) if m.batch_norm else None for blk in m.encoder[0].shared_conv]
    dec_bn = [(blk.block[2], blk.block[5]) if m.batch_norm else None for blk in m.decoder[1].shared_conv]
    rp = m.reverse_patch_embed.proj
    # the residual VQ (--use-improved-vq) keeps EMA codebook buffers, no codebook parameter
    E = None if getattr(m, "use_improved_vq", False) else m.vector_quantization.embedding.weight
    return dict(pe=m.patch_embed.proj, enc=enc, sep=m.encoder[1].shared_conv, E=E,
                dec0=m.decoder[0], dec=dec, t1=rp[0], bn=rp[1], t2=rp[3], enc_bn=enc_bn, dec_bn=dec_bn)


class Saved:
    pass


def _centre_job(w, out):
    """Relayout job: the centre tap of a per-token encoder conv weight (O, I, 3) -> [O][I].  The weight is either
    the reference's contiguous layout or the optimizer's tap-major view (arcweld.optim.RAdam.declare_centre_tap),
    whose centre tap is already a contiguous [O][I] matrix."""
    O, I = w.shape[0], w.shape[1]
    c = w[:, :, 1]
    if w.is_contiguous():
        return (w, O, I, 3, 1, 0, out)
    if not c.is_contiguous():
        raise ValueError("encoder conv weight: unsupported layout")
    return (c, O, I, 1, 0, 0, out)


def _operand_jobs(m, T):
    """Every weight operand of the training step (forward and backward): arcweld.operands.OperandJob list."""
    from .operands import OperandJob as J
    sh = VQVAEShapes(m, 1)
    H, D, R, P, k1 = sh.H, sh.D, sh.R, sh.P, sh.k1
    pr = _params(m)
    dev = pr["pe"].weight.device
    e = lambda *s: torch.empty(*s, device=dev, dtype=T)  # noqa: E731
    jobs = [J("Wp", pr["pe"].weight, H, 1, P, 0, 4, torch.zeros(H, sh.ldp, device=dev, dtype=T),
              sh.ldp)]
    centre = lambda w: _centre_job(w, None)[:6]  # noqa: E731  (the centre tap of the CURRENT storage)
    for r, (c1, c2) in enumerate(pr["enc"]):
        for nm, c in (("1", c1), ("2", c2)):
            jobs.append(J(f"enc{r}_{nm}", c.weight, H, H, 1, 0, 0, e(H, H), derive=centre))
    jobs.append(J("Ws", pr["sep"].weight, D, H, 1, 0, 0, e(D, H)))
    jobs.append(J("Wd0", pr["dec0"].weight, H, D, 1, 0, 0, e(H, D)))
    for r, (c1, c2) in enumerate(pr["dec"]):
        for nm, c in (("1", c1), ("2", c2)):
            jobs.append(J(f"dec{r}_{nm}", c.weight, H, H, 3, 0, 1, e(H, 3 * H)))     # forward [O][3I]
            jobs.append(J(f"dgw{r}_{nm}", c.weight, H, H, 3, 0, 2, e(3 * H, H)))     # dgrad [3O][I]
    jobs.append(J("Wt1", pr["t1"].weight, H, H, k1, 0, 3, e(k1 * H, H)))
    return jobs


def operand_set(m, T=None):
    """The OperandSet the training step of `m` reads (for arcweld.optim.RAdam.attach_operands)."""
    T = operand_dtype(T)
    return operands.peek(m, ("vqvae", T), lambda: _operand_jobs(m, T))


def _centre_grad(g):
    """Where the encoder conv weight-gradient GEMM writes: (C [O][ldc], col_map) for either weight layout."""
    O, I = g.shape[0], g.shape[1]
    if g.is_contiguous():
        return g.view(O, 3 * I), (0, 3, 1)
    c = g[:, :, 1]
    if not c.is_contiguous():
        raise ValueError("encoder conv gradient: unsupported layout")
    return c, (0, 1, 0)


def _conv3_job(w, mode, out):
    """Relayout job of a decoder k = 3 conv weight (mode 1: [O][3I] forward, mode 2: [3O][I] input gradient) for
    either storage order of the weight (contiguous (O, I, 3), or the optimizer's tap-major (O, 3, I))."""
    from .operands import OperandJob
    return OperandJob("", w, w.shape[0], w.shape[1], 3, 0, mode, out).relayout_job()


def _conv3_grad(g):
    """Where a decoder k = 3 conv weight-gradient GEMM (columns j*I + i) writes: (C [O][3I], col_map).  The
    reference's contiguous (O, I, 3) layout takes the columns through the (I, 3) column map; the optimizer's tap-major
    storage (arcweld.optim.RAdam.declare_tap_major, (O, 3, I)) is [O][3I] itself, written by contiguous atomics."""
    O, I = g.shape[0], g.shape[1]
    if g.is_contiguous():
        return g.view(O, 3 * I), (I, 3, 0)
    st = g.permute(0, 2, 1)
    if not st.is_contiguous():
        raise ValueError("decoder conv gradient: unsupported layout")
    return st.reshape(O, 3 * I), (0, 1, 0)


def _bn_stats(h, G, bn, training):
    """BatchNorm statistics [4][G][H] of h [N][H] (rows grouped by row % G); training moves the running stats."""
    N, H = h.shape
    sums = None
    if training and N // G <= 1:
        # torch BatchNorm1d refuses it too (a ragged last batch of one window under --batchnorm 1)
        raise ValueError(f"Expected more than 1 value per channel when training, got input size "
                         f"torch.Size([{N // G}, {H}])")
    if training:
        sums = torch.zeros(2, G, H, device=h.device, dtype=torch.float64)
        K.bn_group_stats(h, G, sums)
    st = torch.empty(4, G, H, device=h.device)
    K.bn_group_finalize(sums, N // G, H, G, bn, training, st)
    return st


def _bn_block_fwd(a0, x, w1, w2, Kd, gemm_kw, c1, c2, bns, G, training, p_drop, seed, ctr, T, last=False):
    """One `--batchnorm 1` ResBlock: x + Drop(BN2(Conv2(GELU(BN1(Conv1(GELU x)))))) (vq_vae_patch_embedd.py:60-74).
    a0 = GELU(x) in the operand dtype.  Returns (y f32, operand copy of GELU(y) -- of y itself for the last block,
    whose output feeds the next conv directly --, saved)."""
    N, H = x.shape
    bn1, bn2 = bns
    e = lambda *s, dt=F32: torch.empty(*s, device=x.device, dtype=dt)  # noqa: E731
    h1 = e(N, H)
    K.gemm(a0, w1, N, H, Kd, bias=c1.bias, C=h1, **gemm_kw)
    st1 = _bn_stats(h1, G, bn1, training)
    hn1, a1 = e(N, H), e(N, H, dt=T)
    K.bn_apply(h1, G, st1, 0, hn1, op=a1)
    h2 = e(N, H)
    K.gemm(a1, w2, N, H, Kd, bias=c2.bias, C=h2, **gemm_kw)
    st2 = _bn_stats(h2, G, bn2, training)
    y, an = e(N, H), e(N, H, dt=T)
    K.bn_apply(h2, G, st2, 2 if last else 1, y, op=an, resid=x, drop=(p_drop, seed), seed_ptr=ctr)
    return y, an, dict(h1=h1, hn1=hn1, a1=a1, h2=h2, st1=st1, st2=st2)


def _bn_block_bwd(gy, x, a0, bs, w1d, w2d, Kd, dgemm_kw, wg, c1, c2, bns, G, training, p_drop, seed, ctr, T, slot,
                  wgrads, need_copy):
    """Backward of _bn_block_fwd from gy (f32 gradient of y).  Appends the two weight-gradient problems to
    ``wgrads`` (wg(c, A, B) builds one) and returns (gx f32, bf16/f32 copy of gx or None)."""
    N, H = gy.shape
    bn1, bn2 = bns
    dev = gy.device
    e = lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
    n = N // G
    sums2 = torch.zeros(2, G, H, device=dev, dtype=torch.float64)
    K.bn_bwd_reduce(bs["h2"], G, bs["st2"], gy, sums2, drop=(p_drop, seed), seed_ptr=ctr)
    dh2 = e(N, H, dt=T)
    K.bn_bwd_apply(bs["h2"], G, bs["st2"], gy, sums2, n, training, dh2, slot(bn2.weight), slot(bn2.bias),
                   drop=(p_drop, seed), seed_ptr=ctr)
    t1 = e(N, H)   # gradient of BN1's output: (dh2 . W2) * GELU'(BN1(h1))
    K.gemm(dh2, w2d, N, H, Kd, b_trans=True, pre=bs["hn1"], C=t1, **dgemm_kw)
    wgrads.append(wg(c2, dh2, bs["a1"]))
    sums1 = torch.zeros(2, G, H, device=dev, dtype=torch.float64)
    K.bn_bwd_reduce(bs["h1"], G, bs["st1"], t1, sums1)
    dh1 = e(N, H, dt=T)
    K.bn_bwd_apply(bs["h1"], G, bs["st1"], t1, sums1, n, training, dh1, slot(bn1.weight), slot(bn1.bias))
    gx = e(N, H)
    gxo = e(N, H, dt=T) if need_copy else None
    K.gemm(dh1, w1d, N, H, Kd, b_trans=True, pre=x, resid=gy, C=gx, C2=gxo, c2_mode=2 if need_copy else 0,
           **dgemm_kw)
    wgrads.append(wg(c1, dh1, a0))
    return gx, gxo


def _chain_fwd(ws, convs, a0, x0, N, H, T, RT, p_drop, seeds, ctr, need_backward, taps, seg):
    """Forward of a ResBlock stack through aw_res_chain_fwd (encoder: taps 1, decoder: taps 3).  ws: the R pairs of
    optimizer-maintained operand copies ([O][I] or [O][3I]); convs: the R (conv1, conv2) modules.  Returns (GELU'(h),
    a1, GELU'(x), a lists -- a1 and a as the per-conv loop makes them, the saved derivatives in place of its h and x
    (the chain's backward multiplies by them), None without a backward --, the operand copies the backward packs its
    weights from or None, the dropout keep bits for the backward or None)."""
    R = len(ws)
    dev = a0.device
    e = lambda dt: torch.empty(N, H, device=dev, dtype=dt)  # noqa: E731
    sb = need_backward
    hs = [e(T) if sb else None for _ in range(R)]
    a1s = [e(T) if sb else None for _ in range(R)]
    xo = [e(RT) if sb and r < R - 1 else None for r in range(R)]
    ao = [e(T) for _ in range(R)]
    # fragment-packed weight copies, from the operand copies, packed right before the chain that streams them (the
    # backward's by _chain_bwd, right before the backward chain): the pack's writes are still in the caches when the
    # chain starts reading
    wsrc = [w for pair in ws for w in pair]
    pk = [torch.empty(H, taps * H, device=dev, dtype=T) for _ in wsrc]
    K.res_pack_weights(wsrc, pk, None, taps=taps)
    pk_bwd = wsrc if sb else None      # the sources of the backward's packed copies
    masks = K.res_dropout_masks_empty(N, R, dev) if sb and p_drop > 0 and R > 1 else None
    K.res_chain_fwd(a0, x0, pk[0::2], pk[1::2], [c1.bias for c1, _ in convs], [c2.bias for _, c2 in convs], hs, a1s,
                    xo, ao, drop=(p_drop, seeds), seed_ptr=ctr, masks=masks, taps=taps, seg=seg)
    return hs, a1s, xo, ao, pk_bwd, masks


def _chain_bwd(sv, convs, gx, gxo, hs, xs, a0s, a1s, pk_bwd, masks, wgrad_target, slot, taps, seg):
    """Backward of a ResBlock stack through aw_res_chain_bwd; returns (weight-gradient problems in the per-conv
    loop's order, the stack input's operand gradient gxo_out[0]).  wgrad_target(c) = (C, col_map) of conv c's
    weight gradient, taps 3 adds the implicit conv form (wconv) to each problem."""
    N, H = gx.shape
    R = len(hs)
    dev = gx.device
    T = gxo.dtype
    gh = [torch.empty(N, H, device=dev, dtype=T) for _ in range(R)]
    go = [torch.empty(N, H, device=dev, dtype=T) for _ in range(R)]
    wsrc, pk_bwd = pk_bwd, [torch.empty(H, taps * H, device=dev, dtype=T) for _ in pk_bwd]
    K.res_pack_weights(wsrc, None, pk_bwd, taps=taps)
    # hs / xs[1:]: the forward chain's saved GELU'(h_r) / GELU'(x_r); xs[0] = x_0, the stack input
    K.res_chain_bwd(gx, gxo, pk_bwd[0::2], pk_bwd[1::2], hs, xs[0], [None] + list(xs[1:R]), gh, go, drop_p=sv.p_drop,
                    masks=masks, taps=taps, seg=seg)
    extra = dict(conv=(H, seg, 1, 1)) if taps == 3 else {}
    wgrads = []
    for r in reversed(range(R)):
        c1, c2 = convs[r]
        gin = gxo if r == R - 1 else go[r + 1]
        for c, A, B in ((c2, gin, a1s[r]), (c1, gh[r], a0s[r])):
            Cw, cm = wgrad_target(c)
            wgrads.append((A, B, H, taps * H, N, dict(a_trans=True, b_trans=True, C=Cw, accumulate=True, col_map=cm,
                                                      a_rowsum=slot(c.bias), **extra)))
    return wgrads, go[0]


# The step's GEMM chain stores its epilogue outputs write-through (aw_gemm_args.store_policy): with 64 dependent
# class-A launches per step, each launch otherwise waits for the previous one's end-of-kernel L2 write-back of up to
# 32 MB of dirty output lines (same-box A/B: +3 % windows/s)
@K.store_policy(nat.AW_STORE_WT)
def forward(m, x, training: bool, need_backward: bool, dtype=None, seed: int = 0, head=True):
    """Returns (emb_loss (), x_hat (B, L, C), perplexity (), indices (N,), saved-or-None).

    ``head=False`` (the fused training step, need_backward only) stops after the BN statistics of the ConvT output:
    x_hat is returned unwritten, and the caller runs the head forward fused with the loss gradient and the first
    head-backward pass (``head_train``)."""
    T = operand_dtype(dtype)
    if x.dtype != F32 or x.dim() != 3:
        raise ValueError("VQVAEPatch expects float32 windows of shape (B, seq_len, input_dim)")
    x = x.contiguous()
    sh = VQVAEShapes(m, x.shape[0])
    H, D, N, S, R, P, k1 = sh.H, sh.D, sh.N, sh.S, sh.R, sh.P, sh.k1
    if x.shape[1] != sh.L or x.shape[2] != sh.C:
        raise ValueError(f"expected windows (B, {sh.L}, {sh.C}), got {tuple(x.shape)}")
    pr = _params(m)
    dev = x.device
    p_drop = float(m.dropout_p) if training else 0.0
    e = lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
    sv = Saved()
    sv.sh, sv.T, sv.p_drop, sv.training = sh, T, p_drop, training
    RT = sv.RT = resid_dtype(m, T)
    sv.enc_seed = [_mix(seed, 100 + r) for r in range(R)]
    sv.dec_seed = [_mix(seed, 200 + r) for r in range(R)]
    acc = accumulators(m, dev, sh.K, H, zero=False)
    sv.ctr = rng_snapshot(m, dev, p_drop, zero=acc["block"])
    sv.acc = acc
    # the head-backward sums of the block belong to one saved forward at a time: the owner is held by a weak
    # reference, released by its backward -- or by its collection when it is never backpropagated
    owner = m.__dict__.get("_acc_owner")
    owned = owner is not None and owner() is not None
    sv.head_gsums = acc["head_gsums"] if not owned else torch.zeros(2 * H, device=dev, dtype=torch.float64)
    if need_backward and not owned:
        m.__dict__["_acc_owner"] = weakref.ref(sv)

    # ---- operand copies of the weights (relayout + cast): persistent, refreshed by one batched relayout only when
    #      a weight changed outside the optimizer (the flat RAdam rewrites them in its update kernel)
    ops = operands.get(m, ("vqvae", T), lambda: _operand_jobs(m, T))
    Wp, Ws, Wd0, Wt1 = ops["Wp"], ops["Ws"], ops["Wd0"], ops["Wt1"]
    enc_w = [(ops[f"enc{r}_1"], ops[f"enc{r}_2"]) for r in range(R)]
    dec_w = [(ops[f"dec{r}_1"], ops[f"dec{r}_2"]) for r in range(R)]
    sv.ops = ops

    # ---- patch embed
    patches = e(N, sh.ldp, dt=T)
    K.patchify(x, P, patches)
    x0, a0 = e(N, H, dt=RT), e(N, H, dt=T)
    K.gemm(patches, Wp, N, H, sh.ldp, bias=pr["pe"].bias, C=x0, C2=a0, c2_mode=1, flops=2 * N * H * P)

    # ---- encoder ResBlocks (per-token: centre taps)
    xs, a0s, hs, a1s = [x0], [a0], [], []
    sv.enc_bs, sv.dec_bs = [], []
    sv.enc_chain = R > 0 and pr["enc_bn"][0] is None and K.res_chain_ok(H, R, T, RT)
    if sv.enc_chain:
        # bf16: the whole ResBlock stack as ONE persistent launch (csrc/reschain.hip), the same tensors bit for bit
        hs, a1s, xo, ao, sv.enc_pk_bwd, sv.enc_masks = _chain_fwd(enc_w, pr["enc"], a0, x0, N, H, T, RT, p_drop,
                                                                  sv.enc_seed, sv.ctr, need_backward, 1, S)
        xs += xo
        a0s += ao
    for r, (c1, c2) in enumerate(pr["enc"] if not sv.enc_chain else []):
        if pr["enc_bn"][r] is not None:   # BatchNorm ResBlocks: per-token statistics (G = S)
            xn, an, bs = _bn_block_fwd(a0s[r], xs[r], enc_w[r][0], enc_w[r][1], H, {}, c1, c2, pr["enc_bn"][r], S,
                                       training, p_drop, sv.enc_seed[r], sv.ctr, T, last=r == R - 1)
            xs.append(xn)
            a0s.append(an)
            sv.enc_bs.append(bs)
            continue
        h, a1 = e(N, H, dt=T), e(N, H, dt=T)   # pre-activation kept in the operand dtype
        K.gemm(a0s[r], enc_w[r][0], N, H, H, bias=c1.bias, C=h, C2=a1, c2_mode=1)
        if r < R - 1:
            xn, an = e(N, H, dt=RT), e(N, H, dt=T)
            K.gemm(a1, enc_w[r][1], N, H, H, bias=c2.bias, drop=(p_drop, sv.enc_seed[r]), seed_ptr=sv.ctr,
                   resid=xs[r], C=xn, C2=an,
                   c2_mode=1)
        else:  # last block: only the operand copy of x_R is consumed (sep conv)
            xn, an = None, e(N, H, dt=T)
            K.gemm(a1, enc_w[r][1], N, H, H, bias=c2.bias, drop=(p_drop, sv.enc_seed[r]), seed_ptr=sv.ctr,
                   resid=xs[r], C=an)
        xs.append(xn)
        a0s.append(an)
        hs.append(h)
        a1s.append(a1)
    xR_T = a0s[R] if R > 0 else (x0 if x0.dtype == T else _cast(x0, T))

    # ---- SepCNNBlock -> z (B, S, D)
    z = e(N, D)
    K.gemm(xR_T, Ws, N, D, H, bias=pr["sep"].bias, C=z)

    # ---- vector quantizer
    Kc = sh.K
    if pr["E"] is None:
        # residual VQ with EMA codebooks (vector_quantizer.py:9-56): commitment loss, no perplexity (:39)
        rvq = m.vector_quantization.vq
        zq, idx2, losses, sv.rvq = rvq.quantize_rows(z, training, save=need_backward)
        idx = idx2[:, 0] if rvq.num_quantizers == 1 else idx2
        emb_loss = losses.view(()) if rvq.num_quantizers == 1 else losses.sum()
        perplexity = None
    else:
        zq = e(N, D)
        idx = e(N, dt=torch.int64)
        counts, sq = acc["counts"], acc["vq_sq"]
        zq_T = None if T == F32 else e(N, D, dt=T)    # the operand copy comes out of the VQ kernel itself
        K.vq_forward(z, pr["E"], zq, idx, counts, sq, zq_copy=zq_T, count_groups=VQ_COUNT_GROUPS)
        emb_loss, perplexity = e(()), e(())
        K.vq_finalize(counts, sq, N, Kc, D, m.vector_quantization.beta, emb_loss, perplexity,
                      count_groups=VQ_COUNT_GROUPS)
    if pr["E"] is None or T == F32:
        zq_T = zq if T == F32 else _cast(zq, T)

    # ---- decoder: 1x1 conv + ResBlocks with k=3 convs along the window
    y0, ya0 = e(N, H, dt=RT), e(N, H, dt=T)
    K.gemm(zq_T, Wd0, N, H, D, bias=pr["dec0"].bias, C=y0, C2=ya0, c2_mode=1)
    conv = (H, S, 1, 0)
    ys, ya0s, dhs, da1s = [y0], [ya0], [], []
    sv.dec_chain = R > 0 and pr["dec_bn"][0] is None and K.res_chain_ok(H, R, T, RT, 3, S, "DEC")
    if sv.dec_chain:
        # bf16: the decoder's k = 3 ResBlock stack as one persistent launch (csrc/reschain.hip, taps = 3)
        dhs, da1s, yo, yao, sv.dec_pk_bwd, sv.dec_masks = _chain_fwd(dec_w, pr["dec"], ya0, y0, N, H, T, RT, p_drop,
                                                                     sv.dec_seed, sv.ctr, need_backward, 3, S)
        ys += yo
        ya0s += yao
    for r, (c1, c2) in enumerate(pr["dec"] if not sv.dec_chain else []):
        if pr["dec_bn"][r] is not None:   # BatchNorm ResBlocks: statistics over all B*S positions (G = 1)
            yn, an, bs = _bn_block_fwd(ya0s[r], ys[r], dec_w[r][0], dec_w[r][1], 3 * H, dict(conv=conv), c1, c2,
                                       pr["dec_bn"][r], 1, training, p_drop, sv.dec_seed[r], sv.ctr, T,
                                       last=r == R - 1)
            ys.append(yn)
            ya0s.append(an)
            sv.dec_bs.append(bs)
            continue
        h, a1 = e(N, H, dt=T), e(N, H, dt=T)   # pre-activation kept in the operand dtype
        K.gemm(ya0s[r], dec_w[r][0], N, H, 3 * H, conv=conv, bias=c1.bias, C=h, C2=a1, c2_mode=1)
        if r < R - 1:
            yn, an = e(N, H, dt=RT), e(N, H, dt=T)
            K.gemm(a1, dec_w[r][1], N, H, 3 * H, conv=conv, bias=c2.bias, drop=(p_drop, sv.dec_seed[r]),
                   seed_ptr=sv.ctr, resid=ys[r],
                   C=yn, C2=an, c2_mode=1)
        else:
            yn, an = None, e(N, H, dt=T)
            K.gemm(a1, dec_w[r][1], N, H, 3 * H, conv=conv, bias=c2.bias, drop=(p_drop, sv.dec_seed[r]),
                   seed_ptr=sv.ctr, resid=ys[r],
                   C=an)
        ys.append(yn)
        ya0s.append(an)
        dhs.append(h)
        da1s.append(a1)
    yR_T = ya0s[R] if R > 0 else (y0 if y0.dtype == T else _cast(y0, T))

    # ---- un-patch: ConvT(H->H, k1) with BN statistics in the epilogue, then the fused head
    bn = pr["bn"]
    # In the bf16 operand mode the ConvT output Y is bf16 (what autocast keeps for a ConvTranspose1d output; the BN
    # statistics still come from the f32 values in the epilogue): half the bytes of the GEMM's output and of the head's
    # passes over Y.  Round 3 measured it even over the step (the head passes are VALU-bound); on the round-4 step it
    # measured 3.162 / 3.155 / 3.157 vs 3.170 / 3.170 / 3.193 ms for an f32 Y (alternating, same box).
    # ARCWELD_HEAD_BF16=0 keeps Y in f32.
    bf_y = T != F32 and K.head_bf16_ok(H) and os.environ.get("ARCWELD_HEAD_BF16", "1") == "1"
    Y = e(N, k1 * H, dt=T if bf_y else F32)
    colstats = acc["colstats"] if training else None
    K.gemm(yR_T, Wt1, N, k1 * H, H, bias=pr["t1"].bias, bias_mod=H, C=Y, colstats=colstats, stats_mod=H)
    stats = e(4 * H)
    K.bn_finalize(colstats, N * k1, H, bn.weight, bn.bias, bn.running_mean if training else bn.running_mean,
                  bn.running_var, bn.num_batches_tracked if training else None, bn.eps,
                  bn.momentum if bn.momentum is not None else 0.1, training, stats)
    x_hat = e(sh.B, sh.L, sh.C)
    Y2 = Y.view(N * k1, H)
    sv.head_fused = not head and need_backward and fused_head_ok(H)
    if not sv.head_fused:
        K.unpatch_head_fwd(Y2, sh.Q, stats, pr["t2"].weight.view(H, 5), pr["t2"].bias, x_hat)

    if not need_backward:
        return emb_loss, x_hat, perplexity, idx, None
    sv.patches, sv.xs, sv.a0s, sv.hs, sv.a1s, sv.xR_T = patches, xs, a0s, hs, a1s, xR_T
    sv.z, sv.idx, sv.zq_T = z, idx, zq_T
    sv.ys, sv.ya0s, sv.dhs, sv.da1s, sv.yR_T = ys, ya0s, dhs, da1s, yR_T
    sv.Y2, sv.stats = Y2, stats
    sv.enc_w, sv.Ws, sv.Wd0, sv.Wt1 = enc_w, Ws, Wd0, Wt1
    return emb_loss, x_hat, perplexity, idx, sv


def fused_head_ok(H):
    """aw_unpatch_head_fwd_bwd1 serves H == 512 (the reference's hidden size)."""
    return H == 512


def head_train(m, sv, x, gscale, x_hat, sqerr, slot):
    """Head forward + MSE value and gradient + head-backward pass 1 in one read of the ConvT output (the fused
    training step; ``forward(..., head=False)`` left x_hat for it).  Returns g_xhat; ``backward`` then skips pass 1."""
    sh, H = sv.sh, sv.sh.H
    pr = _params(m)
    bn = pr["bn"]
    g_xhat = torch.empty_like(x_hat)
    K.unpatch_head_fwd_bwd1(sv.Y2, sh.Q, sv.stats, pr["t2"].weight.view(H, 5), pr["t2"].bias, x, gscale, x_hat,
                            g_xhat, sqerr, sv.head_gsums, slot(pr["t2"].weight).view(H, 5), slot(pr["t2"].bias),
                            slot(bn.weight), slot(bn.bias))
    sv.head_pass1_done = True
    return g_xhat


@torch.no_grad()
def encode(m, x, dtype=F32):
    """Frozen-encoder tokenization: windows (W, L, C) f32 -> (codebook indices (W*S,) int64, z (W*S, D) f32).

    patch embed -> encoder ResBlocks (eval: no dropout) -> sep conv -> VQ argmin; the decoder is never run
    (latentspace_dataloader.py:154-161 calls only patch_embed/encoder/vector_quantization).  Operands are exact
    fp32 unless ``dtype`` says otherwise, so the indices are the reference's bit for bit; ``dtype=torch.bfloat16``
    trades that for speed.
    """
    T = F32 if dtype is None else operand_dtype(dtype)
    if x.dtype != F32 or x.dim() != 3:
        raise ValueError("expected float32 windows of shape (W, seq_len, input_dim)")
    x = x.contiguous()
    sh = VQVAEShapes(m, x.shape[0])
    H, D, N, R, P = sh.H, sh.D, sh.N, sh.R, sh.P
    if x.shape[1] != sh.L or x.shape[2] != sh.C:
        raise ValueError(f"expected windows (W, {sh.L}, {sh.C}), got {tuple(x.shape)}")
    pr = _params(m)
    e = lambda *s, dt=F32: torch.empty(*s, device=x.device, dtype=dt)  # noqa: E731
    Wp = e(H, sh.ldp, dt=T)
    K.weight_relayout(pr["pe"].weight, H, 1, P, 0, 4, Wp, ldo=sh.ldp)
    patches = e(N, sh.ldp, dt=T)
    K.patchify(x, P, patches)
    xr, a = e(N, H), e(N, H, dt=T)
    K.gemm(patches, Wp, N, H, sh.ldp, bias=pr["pe"].bias, C=xr, C2=a, c2_mode=1, flops=2 * N * H * P)
    ew = [(e(H, H, dt=T), e(H, H, dt=T)) for _ in range(R)]
    Ws = e(D, H, dt=T)
    K.weight_relayout_batch([jb for r, (c1, c2) in enumerate(pr["enc"])
                             for jb in (_centre_job(c1.weight, ew[r][0]), _centre_job(c2.weight, ew[r][1]))]
                            + [(pr["sep"].weight, D, H, 1, 0, 0, Ws)])
    h, a1 = e(N, H, dt=T), e(N, H, dt=T)   # pre-activation kept in the operand dtype
    for r, (c1, c2) in enumerate(pr["enc"]):
        w1, w2 = ew[r]
        if pr["enc_bn"][r] is not None:   # BatchNorm ResBlocks (module mode decides batch vs running statistics)
            xr, a, _ = _bn_block_fwd(a, xr, w1, w2, H, {}, c1, c2, pr["enc_bn"][r], sh.S, m.training, 0.0, 0, None,
                                     T, last=r == R - 1)
            continue
        K.gemm(a, w1, N, H, H, bias=c1.bias, C=h, C2=a1, c2_mode=1)
        if r < R - 1:   # x <- x + conv2(gelu(h)) in place (row-local epilogue), a <- gelu(x)
            K.gemm(a1, w2, N, H, H, bias=c2.bias, resid=xr, C=xr, C2=a, c2_mode=1)
        else:           # the sep conv consumes x_R itself (no GELU): write it in the operand dtype
            K.gemm(a1, w2, N, H, H, bias=c2.bias, resid=xr, C=a)
    xR_T = a if R > 0 else (xr if T == F32 else _cast(xr, T))
    z = e(N, D)
    K.gemm(xR_T, Ws, N, D, H, bias=pr["sep"].bias, C=z)
    if pr["E"] is None:   # residual VQ: eval-mode assignment (no EMA), one token per position needs nq == 1
        rvq = m.vector_quantization.vq
        if rvq.num_quantizers != 1:
            raise ValueError("tokenization needs a single quantizer (ResidualVQ num_quantizers == 1)")
        _, idx2, _, _ = rvq.quantize_rows(z, False)
        return idx2[:, 0].contiguous(), z
    zq, idx = e(N, D), e(N, dt=torch.int64)
    counts = torch.zeros(sh.K, device=x.device)
    sq = torch.zeros(1, device=x.device, dtype=torch.float64)
    K.vq_forward(z, pr["E"], zq, idx, counts, sq)
    return idx, z


def _cast(t, T):
    out = torch.empty(t.shape, device=t.device, dtype=T)
    K.cast(t, out)
    return out


@K.store_policy(nat.AW_STORE_WT)
def backward(m, sv, g_emb, g_xhat, slot, mid_hook=None):
    """Accumulate parameter gradients into ``slot(param)`` (f32 tensors shaped like the parameter).

    ``mid_hook()`` runs once the decoder side is done (head, ConvT, decoder ResBlocks, decoder 1x1, codebook): those
    gradients are final there, which lets a data-parallel step reduce them while the encoder backward runs."""
    sh, T, p_drop = sv.sh, sv.T, sv.p_drop
    H, D, N, S, R, P, k1 = sh.H, sh.D, sh.N, sh.S, sh.R, sh.P, sh.k1
    pr = _params(m)
    dev = g_xhat.device
    e = lambda *s, dt=F32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
    g_xhat = g_xhat.contiguous()
    bn = pr["bn"]

    # ---- head + BN backward
    gsums = sv.head_gsums
    owner = m.__dict__.get("_acc_owner")
    if owner is not None and owner() is sv:
        m.__dict__["_acc_owner"] = None
    if not getattr(sv, "head_pass1_done", False):
        K.unpatch_head_bwd1(sv.Y2, sh.Q, sv.stats, pr["t2"].weight.view(H, 5), g_xhat, gsums,
                            slot(pr["t2"].weight).view(H, 5), slot(pr["t2"].bias), slot(bn.weight), slot(bn.bias))
    gY = e(N * k1, H, dt=T)
    K.unpatch_head_bwd2(sv.Y2, sh.Q, sv.stats, pr["t2"].weight.view(H, 5), g_xhat, gsums, sv.training, gY,
                        slot(pr["t1"].bias))
    gY2 = gY.view(N, k1 * H)
    # ConvT1 weight gradient, computed as [i][(j,o)] and accumulated straight into the (H_in, H_out, k1) layout
    K.gemm(sv.yR_T, gY2, H, k1 * H, N, a_trans=True, b_trans=True, C=slot(pr["t1"].weight).view(H, H * k1),
           accumulate=True, col_map=(H, k1, 0))
    # ConvT1 input gradient -> grad of the decoder output, plus the dropout-masked operand for its last block
    RT = sv.RT
    gy, go = e(N, H, dt=RT), e(N, H, dt=T)
    last = R - 1
    bnm = m.batch_norm and R > 0    # BatchNorm ResBlocks: each block applies its own dropout mask to gy
    K.gemm(gY2, sv.Wt1, N, H, k1 * H, b_trans=True, C=gy, C2=None if bnm else go, c2_mode=0 if bnm else
           (3 if R > 0 else 2), drop2=(p_drop, sv.dec_seed[last] if R > 0 else 0), seed_ptr=sv.ctr)

    # ---- decoder ResBlocks (reverse)
    dconv_in = (H, S, -1, 0)
    wconv = (H, S, 1, 1)
    # weight gradients of the whole ResBlock stack are deferred and issued as ONE grouped launch (every tile runs
    # the full token reduction: no split-K, no slab reduce); their operands stay alive until then
    wgrads = []
    dgw = [(sv.ops[f"dgw{r}_1"], sv.ops[f"dgw{r}_2"]) for r in range(R)]
    def wg_dec(c, A, B):
        Cw, cm = _conv3_grad(slot(c.weight))
        return (A, B, H, 3 * H, N, dict(a_trans=True, b_trans=True, conv=wconv, C=Cw, accumulate=True, col_map=cm,
                                        a_rowsum=slot(c.bias)))

    if getattr(sv, "dec_chain", False):
        wgrads, go = _chain_bwd(sv, pr["dec"], gy, go, sv.dhs, sv.ys, sv.ya0s, sv.da1s, sv.dec_pk_bwd, sv.dec_masks,
                                lambda c: _conv3_grad(slot(c.weight)), slot, 3, S)
        sv.dec_pk_bwd = sv.dec_masks = None
    for r in reversed(range(R)) if not getattr(sv, "dec_chain", False) else ():
        c1, c2 = pr["dec"][r]
        W1d, W2d = dgw[r]
        if bnm:
            gy, go = _bn_block_bwd(gy, sv.ys[r], sv.ya0s[r], sv.dec_bs[r], W1d, W2d, 3 * H, dict(conv=dconv_in),
                                   wg_dec, c1, c2, pr["dec_bn"][r], 1, sv.training, p_drop, sv.dec_seed[r], sv.ctr,
                                   T, slot, wgrads, need_copy=r == 0)
            continue
        gh = e(N, H, dt=T)
        K.gemm(go, W2d, N, H, 3 * H, b_trans=True, conv=dconv_in, pre=sv.dhs[r], C=gh)
        wgrads.append(wg_dec(c2, go, sv.da1s[r]))
        gyn, gon = e(N, H, dt=RT), e(N, H, dt=T)
        K.gemm(gh, W1d, N, H, 3 * H, b_trans=True, conv=dconv_in, pre=sv.ys[r], resid=gy, C=gyn, C2=gon,
               c2_mode=3 if r > 0 else 2, drop2=(p_drop, sv.dec_seed[r - 1] if r > 0 else 0),
               seed_ptr=sv.ctr)
        wgrads.append(wg_dec(c1, gh, sv.ya0s[r]))
        gy, go = gyn, gon
    K.gemm_grouped(wgrads)

    # ---- decoder 1x1 conv (weight (H, D, 1) is a contiguous [H][D] matrix)
    K.gemm(go, sv.zq_T, H, D, N, a_trans=True, b_trans=True, C=slot(pr["dec0"].weight).view(H, D), accumulate=True,
           a_rowsum=slot(pr["dec0"].bias))
    gzq = e(N, D)
    K.gemm(go, sv.Wd0, N, D, H, b_trans=True, C=gzq)

    # ---- vector quantizer (straight-through + codebook/commitment loss)
    dz = e(N, D)
    dz_T = dz if T == F32 else None
    if pr["E"] is None:   # residual VQ: straight-through + commitment terms, codebooks are EMA buffers
        res, qs = sv.rvq
        nq = res.shape[0]
        K.rvq_backward(res, qs, gzq, g_emb if nq == 1 else g_emb.expand(nq).contiguous(), dz)
    else:
        dz_T = dz if T == F32 else e(N, D, dt=T)    # operand copy written by the VQ backward kernel
        K.vq_backward(sv.z, pr["E"], sv.idx, gzq, g_emb, m.vector_quantization.beta, dz, slot(pr["E"]),
                      dz_copy=None if T == F32 else dz_T)
    if mid_hook is not None:
        with K.store_policy(nat.AW_STORE_NT):     # the hook's own launches (e.g. collectives) keep the default policy
            mid_hook()
    if dz_T is None:
        dz_T = _cast(dz, T)

    # ---- SepCNNBlock
    K.gemm(dz_T, sv.xR_T, D, H, N, a_trans=True, b_trans=True, C=slot(pr["sep"].weight).view(D, H), accumulate=True,
           a_rowsum=slot(pr["sep"].bias))
    gx, gxo = e(N, H, dt=RT), e(N, H, dt=T)
    K.gemm(dz_T, sv.Ws, N, H, D, b_trans=True, C=gx, C2=None if bnm else gxo, c2_mode=0 if bnm else
           (3 if R > 0 else 2), drop2=(p_drop, sv.enc_seed[R - 1] if R > 0 else 0), seed_ptr=sv.ctr)

    # ---- encoder ResBlocks (reverse); weight gradients deferred into one grouped launch as in the decoder
    wgrads = []

    def wg_enc(c, A, B):
        Cw, cm = _centre_grad(slot(c.weight))
        return (A, B, H, H, N, dict(a_trans=True, b_trans=True, C=Cw, accumulate=True, col_map=cm,
                                    a_rowsum=slot(c.bias)))

    if getattr(sv, "enc_chain", False):
        # bf16: the input-gradient chain of all R blocks in one launch, on the packed backward weight copies the
        # forward made
        wgrads, gxo = _chain_bwd(sv, pr["enc"], gx, gxo, sv.hs, sv.xs, sv.a0s, sv.a1s, sv.enc_pk_bwd, sv.enc_masks,
                                 lambda c: _centre_grad(slot(c.weight)), slot, 1, S)
        sv.enc_pk_bwd = sv.enc_masks = None
    for r in reversed(range(R)) if not getattr(sv, "enc_chain", False) else ():
        c1, c2 = pr["enc"][r]
        w1, w2 = sv.enc_w[r]
        if bnm:
            gx, gxo = _bn_block_bwd(gx, sv.xs[r], sv.a0s[r], sv.enc_bs[r], w1, w2, H, {}, wg_enc, c1, c2,
                                    pr["enc_bn"][r], S, sv.training, p_drop, sv.enc_seed[r], sv.ctr, T, slot, wgrads,
                                    need_copy=r == 0)
            continue
        gh = e(N, H, dt=T)
        K.gemm(gxo, w2, N, H, H, b_trans=True, pre=sv.hs[r], C=gh)
        C2w, cm2 = _centre_grad(slot(c2.weight))
        wgrads.append((gxo, sv.a1s[r], H, H, N, dict(a_trans=True, b_trans=True, C=C2w, accumulate=True, col_map=cm2,
                                                     a_rowsum=slot(c2.bias))))
        gxn, gxon = e(N, H, dt=RT), e(N, H, dt=T)
        K.gemm(gh, w1, N, H, H, b_trans=True, pre=sv.xs[r], resid=gx, C=gxn, C2=gxon, c2_mode=3 if r > 0 else 2,
               drop2=(p_drop, sv.enc_seed[r - 1] if r > 0 else 0), seed_ptr=sv.ctr)
        C1w, cm1 = _centre_grad(slot(c1.weight))
        wgrads.append((gh, sv.a0s[r], H, H, N, dict(a_trans=True, b_trans=True, C=C1w, accumulate=True, col_map=cm1,
                                                    a_rowsum=slot(c1.bias))))
        gx, gxo = gxn, gxon
    K.wgrad_issue(wgrads)      # the 16 per-token conv weight gradients: one stream-K batch (bf16) or one grouped launch

    # ---- patch embed weight/bias
    K.gemm(gxo, sv.patches, H, P, N, a_trans=True, b_trans=True, C=slot(pr["pe"].weight).view(H, P),
           accumulate=True, a_rowsum=slot(pr["pe"].bias))


class VQVAEPatchFunction(torch.autograd.Function):
    """autograd boundary of the fused path: inputs (x, *params) -> (emb_loss, x_hat, perplexity)."""

    @staticmethod
    def forward(ctx, m, x, seed, *params):
        training = m.training
        need = torch.is_grad_enabled() or any(p.requires_grad for p in params)
        emb, x_hat, perp, idx, sv = forward(m, x, training, need_backward=True, seed=seed)
        ctx.m, ctx.sv, ctx.params = m, sv, params
        if perp is not None:          # None for the residual VQ (vector_quantizer.py:39)
            ctx.mark_non_differentiable(perp)
        m._last_indices = idx
        return emb, x_hat, perp

    @staticmethod
    def backward(ctx, g_emb, g_xhat, g_perp):
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

        if g_emb is None:
            g_emb = torch.zeros(1, device=g_xhat.device)
        if g_xhat is None:
            g_xhat = torch.zeros(sv.sh.B, sv.sh.L, sv.sh.C, device=g_emb.device)
        backward(m, sv, g_emb.reshape(1).contiguous(), g_xhat, slot)
        ctx.sv = None
        return (None, None, None) + tuple(grads.get(p) for p in ctx.params)
