"""VectorQuantizer and ResidualVQLightning -- drop-ins for model/vector_quantizer.py of the reference.

VectorQuantizer (:59-131): forward and backward run on the HIP kernels (aw_vq_forward / aw_vq_finalize /
aw_vq_backward / aw_vq_onehot): exact fp32 distances with the reference's expression and first-index argmin, so the
codebook indices are bit-identical to the reference on identical inputs.

ResidualVQLightning (:9-56): the EMA residual quantizer of vector-quantize-pytorch restated on the HIP kernels
(arcweld/residual_vq.py; parity against the third-party library unpinned).
"""
import torch
from torch import nn

from arcweld import kernels as K
from arcweld.lightning import LightningModule
from arcweld.residual_vq import ResidualVQ


class _VQFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, E, beta, want_onehot):
        D = E.shape[1]
        z2 = z.reshape(-1, D).contiguous()
        N, Kc = z2.shape[0], E.shape[0]
        zq = torch.empty_like(z2)
        idx = torch.empty(N, dtype=torch.int64, device=z.device)
        counts = torch.zeros(Kc, device=z.device)
        sq = torch.zeros(1, dtype=torch.float64, device=z.device)
        K.vq_forward(z2, E.contiguous(), zq, idx, counts, sq)
        loss = torch.empty((), device=z.device)
        perp = torch.empty((), device=z.device)
        K.vq_finalize(counts, sq, N, Kc, D, beta, loss, perp)
        onehot = torch.empty(N, Kc, device=z.device)
        if want_onehot:
            K.vq_onehot(idx, Kc, onehot)
        ctx.save_for_backward(z2, E, idx)
        ctx.beta, ctx.zshape = beta, z.shape
        idx2 = idx.view(N, 1)
        ctx.mark_non_differentiable(perp, onehot, idx2)
        return loss, zq.view(z.shape), perp, onehot, idx2

    @staticmethod
    def backward(ctx, g_loss, g_zq, g_perp, g_onehot, g_idx):
        z2, E, idx = ctx.saved_tensors
        dz = torch.empty_like(z2)
        dE = torch.zeros_like(E)
        gl = (g_loss if g_loss is not None else torch.zeros((), device=z2.device)).reshape(1).contiguous()
        gz = g_zq.reshape(z2.shape).contiguous() if g_zq is not None else None
        K.vq_backward(z2, E, idx, gz, gl, ctx.beta, dz, dE)
        return dz.view(ctx.zshape), dE, None, None


class VectorQuantizer(LightningModule):
    """Discretization bottleneck of the VQ-VAE (reference model/vector_quantizer.py:59-131).

    n_e: number of embeddings, e_dim: embedding dim, beta: weight of the codebook-side term (the reference
    weights the z-side term by 1 and the codebook side by beta, vector_quantizer.py:107-108).
    """

    def __init__(self, n_e, e_dim, beta):
        super().__init__()
        self.n_e = n_e
        self.e_dim = e_dim
        self.beta = beta
        self.embedding = nn.Embedding(self.n_e, self.e_dim)
        self.embedding.weight.data.uniform_(-1.0 / self.n_e, 1.0 / self.n_e)
        self.materialize_onehot = True

    def forward(self, z):
        """z (..., e_dim) -> (loss, z_q (straight-through), perplexity, min_encodings (N, n_e), indices (N, 1))."""
        return _VQFunction.apply(z, self.embedding.weight, float(self.beta), self.materialize_onehot)

    def get_embedding_from_one_hot(self, min_encoding_indices, target_shape):
        idx = min_encoding_indices.reshape(-1).to(torch.int64).contiguous()
        out = torch.empty(idx.numel(), self.e_dim, device=idx.device)
        K.vq_gather(self.embedding.weight.detach().contiguous(), idx, out)
        return out.view(target_shape).contiguous()


class ResidualVQLightning(LightningModule):
    """Improved VQ (reference model/vector_quantizer.py:9-56): ResidualVQ with k-means init and EMA dead-code
    replacement.  forward(x (B, S, e_dim)) -> (commit_loss (1, nq), z_q (B, S, e_dim), None, None, indices
    (B, S, nq)), the reference's tuple order (:37-39)."""

    def __init__(self, n_e: int, e_dim: int, kmeans_init: bool = False, kmeans_iters: int = 0,
                 threshold_ema_dead_code: int = 2, num_quantizers: int = 1):
        super().__init__()
        self.n_e = n_e
        self.e_dim = e_dim
        self.kmeans_init = kmeans_init
        self.kmeans_iters = kmeans_iters
        self.threshold_ema_dead_code = threshold_ema_dead_code
        self.num_quantizers = num_quantizers
        self.vq = ResidualVQ(num_quantizers=num_quantizers, dim=e_dim, codebook_size=n_e, kmeans_init=kmeans_init,
                             kmeans_iters=kmeans_iters, threshold_ema_dead_code=threshold_ema_dead_code)
        self.save_hyperparameters()

    def forward(self, x):
        z_q, indices, commit_loss = self.vq(x)
        return commit_loss, z_q, None, None, indices

    def forward_ood(self, x):
        """(loss_OOD (B,) = mean over (S, D) of (z_q - x)^2, z_q, indices, commit_loss) (:41-56)."""
        z_q, indices, commit_loss = self.vq(x)
        d = (z_q.detach() - x) ** 2
        return d.mean(dim=[1, 2]), z_q, indices, commit_loss
