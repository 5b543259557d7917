"""VQVAEPatch and its building blocks -- drop-in for model/vq_vae_patch_embedd.py of the reference.

The module tree (and therefore every state_dict key and shape) matches the reference exactly:
patch_embed.proj, encoder.0.shared_conv.{r}.block.{1,4}, encoder.1.shared_conv, vector_quantization.embedding,
decoder.0, decoder.1.shared_conv.{r}.block.{1,4}, reverse_patch_embed.proj.{0,1,3}.

``VQVAEPatch.forward`` runs the whole network as ONE fused HIP pass (arcweld.vqvae) behind a single autograd
Function.  The sub-modules keep working on their own in the reference's channel-major layout (B, C, S) for
inference (the latent tokenizer calls patch_embed -> encoder -> vector_quantization,
dataloader/latentspace_dataloader.py:154-161); their standalone forwards run the same kernels.
"""
import torch
from torch import nn

from arcweld import kernels as K
from arcweld import vqvae as engine
from model.autencoder_lightning_base import Autoencoder
from model.vector_quantizer import ResidualVQLightning, VectorQuantizer


def _need_no_grad(mod, *tensors):
    if torch.is_grad_enabled() and (any(t.requires_grad for t in tensors) or
                                    any(p.requires_grad for p in mod.parameters())):
        raise NotImplementedError(
            f"{type(mod).__name__}.forward on its own is inference-only on the HIP path; train through "
            "VQVAEPatch.forward (one fused autograd node) or wrap the call in torch.no_grad()")


def _tokens(x_bcs, T):
    """(B, C, S) channel-major -> token-major (B*S, C) contiguous in operand dtype T."""
    B, C, S = x_bcs.shape
    t = x_bcs.permute(0, 2, 1)
    if t.dtype != T or not t.is_contiguous():
        out = torch.empty(B * S, C, device=x_bcs.device, dtype=T)
        out.view(B, S, C).copy_(t)
        return out
    return t.reshape(B * S, C)


class PatchEmbedding(nn.Module):
    """(B, L, C) -> (B, H, L*C/P): channel-major flatten + Conv1d(1, H, k=P, s=P) (reference :7-17)."""

    def __init__(self, patch_size, embed_dim):
        super().__init__()
        self.patch_size = patch_size
        self.proj = nn.Conv1d(1, embed_dim, kernel_size=patch_size, stride=patch_size)

    def forward(self, x):
        _need_no_grad(self, x)
        B, L, C = x.shape
        P, H = self.patch_size, self.proj.out_channels
        S = L * C // P
        ldp = (P + 7) // 8 * 8
        T = engine.operand_dtype()
        patches = torch.empty(B * S, ldp, device=x.device, dtype=T)
        K.patchify(x.contiguous(), P, patches)
        W = torch.empty(H, ldp, device=x.device, dtype=T)
        K.weight_relayout(self.proj.weight, H, 1, P, 0, 4, W, ldo=ldp)
        out = torch.empty(B * S, H, device=x.device)
        K.gemm(patches, W, B * S, H, ldp, bias=self.proj.bias, C=out)
        return out.view(B, S, H).permute(0, 2, 1)


class PatchEmbeddingInverse(nn.Module):
    """ConvT(H->H, k1, s1) -> BatchNorm1d -> GELU -> ConvT(H->1, 5, 5) -> (B, L, input_dim) (reference :19-57)."""

    _K1 = {25: 5, 10: 2, 50: 10}

    def __init__(self, patch_size, embed_dim, input_dim):
        super().__init__()
        self.patch_size = patch_size
        if patch_size not in self._K1:
            raise NotImplementedError(f"Patch size not implemented: {patch_size}")
        self.k1 = self._K1[patch_size]
        self.proj = nn.Sequential(
            nn.ConvTranspose1d(embed_dim, embed_dim, kernel_size=self.k1, stride=self.k1),
            nn.BatchNorm1d(embed_dim),
            nn.GELU(),
            nn.ConvTranspose1d(embed_dim, 1, kernel_size=5, stride=5),
        )
        self.input_dim = input_dim

    def forward(self, x):
        _need_no_grad(self, x)
        B, H, S = x.shape
        T = engine.operand_dtype()
        xt = _tokens(x, T)
        N, k1 = B * S, self.k1
        W = torch.empty(k1 * H, H, device=x.device, dtype=T)
        K.weight_relayout(self.proj[0].weight, H, H, k1, 0, 3, W)
        Y = torch.empty(N, k1 * H, device=x.device)
        bn = self.proj[1]
        cs = torch.zeros(2 * H, device=x.device, dtype=torch.float64) if self.training else None
        K.gemm(xt, W, N, k1 * H, H, bias=self.proj[0].bias, bias_mod=H, C=Y, colstats=cs, stats_mod=H)
        stats = torch.empty(4 * H, device=x.device)
        K.bn_finalize(cs, N * k1, H, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                      bn.num_batches_tracked if self.training else None, bn.eps, bn.momentum or 0.1, self.training,
                      stats)
        out = torch.empty(B, S * k1 * 5 // self.input_dim, self.input_dim, device=x.device)
        K.unpatch_head_fwd(Y.view(N * k1, H), S * k1, stats, self.proj[3].weight.view(H, 5), self.proj[3].bias, out)
        return out


class ResBlock(nn.Module):
    """x + Drop(BN?(Conv(GELU(BN?(Conv(GELU(x))))))) (reference :60-74)."""

    def __init__(self, channels: int, kernel_size: int = 3, stride: int = 1, padding: int = 1, dropout_p: float = 0.1,
                 batch_norm: bool = True):
        super().__init__()
        self.block = nn.Sequential(
            nn.GELU(),
            nn.Conv1d(channels, channels, kernel_size=kernel_size, stride=stride, padding=padding),
            nn.BatchNorm1d(channels) if batch_norm else nn.Identity(),
            nn.GELU(),
            nn.Conv1d(channels, channels, kernel_size=kernel_size, stride=stride, padding=padding),
            nn.BatchNorm1d(channels) if batch_norm else nn.Identity(),
            nn.Dropout(p=dropout_p),
        )


class SepCNNBlock(nn.Module):
    """Per-token Conv1d(H -> D, k=1) then permute to (B, S, D) (reference :77-91)."""

    def __init__(self, hidden_dim: int, embedding_dim: int) -> None:
        super().__init__()
        self.shared_conv = nn.Conv1d(hidden_dim, embedding_dim, kernel_size=1, stride=1, padding=0)

    def forward(self, x):
        _need_no_grad(self, x)
        B, H, S = x.shape
        D = self.shared_conv.out_channels
        T = engine.operand_dtype()
        xt = _tokens(x, T)
        W = torch.empty(D, H, device=x.device, dtype=T)
        K.weight_relayout(self.shared_conv.weight, D, H, 1, 0, 0, W)
        z = torch.empty(B * S, D, device=x.device)
        K.gemm(xt, W, B * S, D, H, bias=self.shared_conv.bias, C=z)
        return z.view(B, S, D)


class CNNBlock(nn.Module):
    """Stack of ResBlocks; seperate=True runs each token on its own (k=3/pad=1 on a length-1 slice -> only the
    centre tap contributes), seperate=False convolves along the token axis (reference :93-114)."""

    def __init__(self, embed_dim: int, seperate: bool = True, kernel_size: int = 3, stride: int = 1, padding: int = 1,
                 dropout_p: float = 0.1, batch_norm: bool = True, n_resblocks: int = 1):
        super().__init__()
        self.seperate = seperate
        self.batch_norm = batch_norm
        self.dropout_p = dropout_p
        self.shared_conv = nn.Sequential(*[
            ResBlock(channels=embed_dim, kernel_size=kernel_size, stride=stride, padding=padding, dropout_p=dropout_p,
                     batch_norm=batch_norm) for _ in range(n_resblocks)])

    def forward(self, x):
        _need_no_grad(self, x)
        B, H, S = x.shape
        N = B * S
        T = engine.operand_dtype()
        cur = x.permute(0, 2, 1).contiguous().view(N, H)
        a0 = _gelu_operand(cur, T)
        p = self.dropout_p if self.training else 0.0
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        for r, blk in enumerate(self.shared_conv):
            c1, c2 = blk.block[1], blk.block[4]
            if self.seperate:
                w1, w2 = (torch.empty(H, H, device=x.device, dtype=T) for _ in range(2))
                K.weight_relayout_batch([engine._centre_job(c1.weight, w1), engine._centre_job(c2.weight, w2)])
                kd, conv = H, None
            else:
                w1, w2 = (torch.empty(H, 3 * H, device=x.device, dtype=T) for _ in range(2))
                K.weight_relayout(c1.weight, H, H, 3, 0, 1, w1)
                K.weight_relayout(c2.weight, H, H, 3, 0, 1, w2)
                kd, conv = 3 * H, (H, S, 1, 0)
            if self.batch_norm:   # BatchNorm ResBlocks: per-token statistics when the tokens run separately
                gk = {} if conv is None else dict(conv=conv)
                cur, a0, _ = engine._bn_block_fwd(a0, cur, w1, w2, kd, gk, c1, c2, (blk.block[2], blk.block[5]),
                                                  S if self.seperate else 1, self.training, p, engine._mix(seed, r),
                                                  None, T)
                continue
            a1 = torch.empty(N, H, device=x.device, dtype=T)
            K.gemm(a0, w1, N, H, kd, conv=conv, bias=c1.bias, C2=a1, c2_mode=1)
            nxt = torch.empty(N, H, device=x.device)
            an = torch.empty(N, H, device=x.device, dtype=T)
            K.gemm(a1, w2, N, H, kd, conv=conv, bias=c2.bias, drop=(p, engine._mix(seed, r)), resid=cur, C=nxt, C2=an,
                   c2_mode=1)
            cur, a0 = nxt, an
        return cur.view(B, S, H).permute(0, 2, 1)


def _gelu_operand(x, T):
    """GELU(x) in operand dtype T through the GEMM epilogue with an empty contraction (K = 0):
    v = 0 + resid = x, C2 = gelu(v)."""
    N, H = x.shape
    out = torch.empty(N, H, device=x.device, dtype=T)
    dummy = torch.zeros(8, 8, device=x.device, dtype=T)
    K.gemm(dummy, dummy, N, H, 0, resid=x, C2=out, c2_mode=1)
    return out


class VQVAEPatch(Autoencoder):
    """VQ-VAE with patch embedding (reference model/vq_vae_patch_embedd.py:117-167)."""

    def __init__(self, hidden_dim: int, input_dim: int, num_embeddings: int, embedding_dim: int, n_resblocks: int,
                 learning_rate: float, dropout_p: float = 0.1, patch_size: int = 25, seq_len: int = 200,
                 batch_norm: bool = True, beta: float = 0.25, use_improved_vq: bool = False, kmeans_iters: int = 0,
                 threshold_ema_dead_code: int = 2):
        super().__init__(hidden_dim=hidden_dim, input_dim=input_dim, num_embeddings=num_embeddings,
                         embedding_dim=embedding_dim, n_resblocks=n_resblocks, learning_rate=learning_rate,
                         seq_len=seq_len, dropout_p=dropout_p)
        self.use_improved_vq = bool(use_improved_vq)
        self.patch_embed = PatchEmbedding(patch_size=patch_size, embed_dim=hidden_dim)
        self.encoder = nn.Sequential(
            CNNBlock(embed_dim=hidden_dim, n_resblocks=n_resblocks, dropout_p=dropout_p, batch_norm=batch_norm),
            SepCNNBlock(hidden_dim=hidden_dim, embedding_dim=embedding_dim),
        )
        if use_improved_vq:   # vq_vae_patch_embedd.py:132-136: one EMA quantizer, k-means init, dead-code reset
            self.vector_quantization = ResidualVQLightning(num_quantizers=1, e_dim=embedding_dim, n_e=num_embeddings,
                                                           kmeans_init=True, kmeans_iters=kmeans_iters,
                                                           threshold_ema_dead_code=threshold_ema_dead_code)
        else:
            self.vector_quantization = VectorQuantizer(n_e=num_embeddings, e_dim=embedding_dim, beta=beta)
        self.decoder = nn.Sequential(
            nn.Conv1d(embedding_dim, hidden_dim, kernel_size=1, stride=1, padding=0),
            CNNBlock(embed_dim=hidden_dim, seperate=False, n_resblocks=n_resblocks, dropout_p=dropout_p,
                     batch_norm=batch_norm),
        )
        self.reverse_patch_embed = PatchEmbeddingInverse(patch_size=patch_size, embed_dim=hidden_dim,
                                                         input_dim=input_dim)
        self.enc_out_len = seq_len // patch_size * input_dim
        self.patch_size = patch_size
        self.batch_norm = batch_norm
        self.apply(self.weights_init)
        self._last_indices = None

    def _next_seed(self):
        """Host part of the dropout seed: fixed per (torch seed, rank).  The per-call variation comes from the
        module's device-side counter (arcweld.vqvae.rng_snapshot), so eager calls and replays of a captured step
        graph draw the same sequence of masks."""
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        return (torch.initial_seed() * 1000003 + 1 + (rank << 40)) & 0x7FFFFFFFFFFFFFFF

    def forward(self, x):
        """(B, seq_len, input_dim) -> (embedding_loss, x_hat (B, seq_len, input_dim), perplexity)."""
        params = tuple(self.parameters())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return engine.VQVAEPatchFunction.apply(self, x, self._next_seed(), *params)
        emb, x_hat, perp, idx, _ = engine.forward(self, x, self.training, need_backward=False,
                                                  seed=self._next_seed())
        self._last_indices = idx
        return emb, x_hat, perp

    @torch.no_grad()
    def fused_train_step(self, x, scale, mid_hook=None):
        """One training micro-step on the kernels without autograd: the same work as ``training_step`` followed by
        ``(loss * scale).backward()`` (loss = mse(x_hat, x) + embedding loss, autencoder_lightning_base.py:80-97).
        Gradients accumulate into each parameter's ``.grad`` (the flat optimizer views when a Trainer installed
        ``_grad_sink``).  ``mid_hook`` is called between the decoder-side and the encoder-side backward (see
        arcweld.vqvae.backward): the data-parallel step starts the decoder-side all-reduce there.  Returns the loss."""
        x = x.contiguous()
        emb, x_hat, perp, idx, sv = engine.forward(self, x, self.training, need_backward=True, seed=self._next_seed())
        self._last_indices = idx
        sq = sv.acc["mse_sq"]            # zeroed with the forward's other accumulators (one fill launch)
        K.mse_fwd(x_hat, x, sq)
        recon = torch.empty((), device=x.device)
        K.mse_finalize(sq, x.numel(), recon)
        loss = torch.empty((), device=x.device)
        K.scalar_add(recon.reshape(1), emb.reshape(1), loss)
        g = self._loss_scale_tensor(float(scale), x.device)
        g_xhat = torch.empty_like(x_hat)
        K.mse_bwd(x_hat, x, g, g_xhat)
        sink = getattr(self, "_grad_sink", None)

        def slot(p):
            if sink is not None and p in sink:
                return sink[p]
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            return p.grad

        engine.backward(self, sv, g, g_xhat, slot, mid_hook=mid_hook)
        self.log('train/loss', loss, prog_bar=True)
        self.log('train/recon_error', recon)
        self.last_recon = (x[:1], x_hat[:1])
        return loss

    def _loss_scale_tensor(self, scale, dev):
        """Persistent device scalar holding the loss scale (refilled only when the value changes)."""
        st = self.__dict__.get("_gscale")
        if st is None or st[0] != scale or st[1].device != dev:
            st = (scale, torch.full((1,), scale, device=dev))
            self.__dict__["_gscale"] = st
        return st[1]

    def operand_set(self):
        """The persistent GEMM operand copies of the training step (arcweld.operands), for the optimizer to keep
        current (arcweld.optim.RAdam.attach_operands)."""
        return engine.operand_set(self)

    def centre_tap_parameters(self):
        """The encoder ResBlock conv weights: k = 3, pad = 1 convs applied per token to length-1 inputs
        (vq_vae_patch_embedd.py:93-114, loop :108-110), so only weight[:, :, 1] is used and the side taps receive
        an exactly-zero gradient.  The optimizer keeps those taps out of the all-reduce, clip norm and update."""
        return [blk.block[i].weight for blk in self.encoder[0].shared_conv for i in (1, 4)]

    def backward_split_parameter(self):
        """First parameter (in registration order) whose gradient is final at fused_train_step's mid_hook (the
        residual VQ's codebooks are EMA buffers: the decoder's 1x1 conv comes first then)."""
        if self.use_improved_vq:
            return self.decoder[0].weight
        return self.vector_quantization.embedding.weight

    def backward_late_parameters(self):
        """Parameters whose gradients are final at fused_train_step's mid_hook: the codebook and everything after
        it in registration order (decoder 1x1 conv, decoder ResBlocks, un-patch head)."""
        ps = list(self.parameters())
        cut = next(i for i, p in enumerate(ps) if p is self.backward_split_parameter())
        return ps[cut:]

    @torch.no_grad()
    def encode_ids(self, x):
        """Frozen-encoder tokenization (latentspace_dataloader.py:154-161): windows (B, L, C) -> ids (B, S) int64,
        fused patch_embed -> encoder -> VQ on the HIP path (eval-mode semantics of the current module state)."""
        from arcweld import tokenize
        return tokenize.encode_ids(self, x)
