"""VQVAEPatch and its building blocks -- drop-in for model/vq_vae_patch_embedd.py of the reference.

The module tree (and therefore every state_dict key and shape) matches the reference exactly:
patch_embed.proj, encoder.0.shared_conv.{r}.block.{1,4}, encoder.1.shared_conv, vector_quantization.embedding,
decoder.0, decoder.1.shared_conv.{r}.block.{1,4}, reverse_patch_embed.proj.{0,1,3}.

``VQVAEPatch.forward`` runs the whole network as ONE fused HIP pass (arcweld.vqvae) behind a single autograd
Function.  The sub-modules also work on their own in the reference's channel-major layout (B, C, S) -- the latent
tokenizer calls patch_embed -> encoder -> vector_quantization (dataloader/latentspace_dataloader.py:154-161) -- and
are trainable there too: each records its own autograd node whose backward runs the same kernels
(arcweld.modules).
"""
import torch
from torch import nn

from arcweld import kernels as K
from arcweld import modules
from arcweld import vqvae as engine
from model.autencoder_lightning_base import Autoencoder
from model.vector_quantizer import ResidualVQLightning, VectorQuantizer


class PatchEmbedding(nn.Module):
    """(B, L, C) -> (B, H, L*C/P): channel-major flatten + Conv1d(1, H, k=P, s=P) (reference :7-17)."""

    def __init__(self, patch_size, embed_dim):
        super().__init__()
        self.patch_size = patch_size
        self.proj = nn.Conv1d(1, embed_dim, kernel_size=patch_size, stride=patch_size)

    def forward(self, x):
        return modules.patch_embed(self, x)


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
        return modules.patch_unembed(self, x)


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

    def forward(self, x):
        """(B, C, L) -> x + block(x): an autograd node of its own on the per-block kernels (arcweld.modules)."""
        return modules.resblock(self, x)


class SepCNNBlock(nn.Module):
    """Per-token Conv1d(H -> D, k=1) then permute to (B, S, D) (reference :77-91)."""

    def __init__(self, hidden_dim: int, embedding_dim: int) -> None:
        super().__init__()
        self.shared_conv = nn.Conv1d(hidden_dim, embedding_dim, kernel_size=1, stride=1, padding=0)

    def forward(self, x):
        return modules.sep_cnn(self, x)


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
        return modules.cnn_block(self, x)


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
        sink = getattr(self, "_grad_sink", None)

        def slot(p):
            if sink is not None and p in sink:
                return sink[p]
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            return p.grad

        # the head forward runs fused with the MSE gradient and the first head-backward pass (engine.head_train)
        emb, x_hat, perp, idx, sv = engine.forward(self, x, self.training, need_backward=True, seed=self._next_seed(),
                                                   head=False)
        self._last_indices = idx
        sq = sv.acc["mse_sq"]            # zeroed with the forward's other accumulators (one fill launch)
        g = self._loss_scale_tensor(float(scale), x.device)
        if sv.head_fused:
            g_xhat = engine.head_train(self, sv, x, g, x_hat, sq, slot)
        else:
            K.mse_fwd(x_hat, x, sq)
            g_xhat = torch.empty_like(x_hat)
            K.mse_bwd(x_hat, x, g, g_xhat)
        recon = torch.empty((), device=x.device)
        loss = torch.empty((), device=x.device)
        K.mse_finalize_add(sq, x.numel(), emb.reshape(1), recon, loss)

        engine.backward(self, sv, g, g_xhat, slot, mid_hook=mid_hook)
        self.log('train/loss', loss, prog_bar=True)
        self.log('train/recon_error', recon)
        self.last_recon = (x[:1], x_hat[:1])
        return loss

    def _loss_scale_tensor(self, scale, dev):
        """Persistent device scalar holding the loss scale, one per (scale, device) and never freed (a captured step
        graph keeps reading the one it was made with)."""
        cache = self.__dict__.setdefault("_gscale", {})
        key = (float(scale), str(dev))
        if key not in cache:
            cache[key] = torch.full((1,), scale, device=dev)
        return cache[key]

    def operand_set(self):
        """The persistent GEMM operand copies of the training step (arcweld.operands), for the optimizer to keep
        current (arcweld.optim.RAdam.attach_operands)."""
        return engine.operand_set(self)

    def centre_tap_parameters(self):
        """The encoder ResBlock conv weights: k = 3, pad = 1 convs applied per token to length-1 inputs
        (vq_vae_patch_embedd.py:93-114, loop :108-110), so only weight[:, :, 1] is used and the side taps receive
        an exactly-zero gradient.  The optimizer keeps those taps out of the all-reduce, clip norm and update."""
        return [blk.block[i].weight for blk in self.encoder[0].shared_conv for i in (1, 4)]

    def tap_major_parameters(self):
        """The decoder ResBlock k = 3 conv weights (vq_vae_patch_embedd.py:142-145 with :60-74): the optimizer stores
        them (O, 3, I) so their weight-gradient GEMM writes contiguous rows (arcweld.optim.RAdam.declare_tap_major)."""
        return [blk.block[i].weight for blk in self.decoder[1].shared_conv for i in (1, 4)]

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
