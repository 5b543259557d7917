"""Residual VQ with EMA codebooks on the HIP kernels -- the quantizer behind ResidualVQLightning.

The reference (model/vector_quantizer.py:9-56) wraps ``vector_quantize_pytorch.ResidualVQ`` (third-party, unpinned,
not installed here).  This module restates that library's published algorithm with its module tree and buffer names
(``layers.<i>._codebook.{initted, cluster_size, embed_avg, embed}``), so a state_dict written by the library loads
here and vice versa; the arithmetic runs on csrc/vq.hip (nearest code) and csrc/rvq.hip (cluster sums, k-means,
EMA update, dead-code replacement, residual bookkeeping, backward).  Parity against the library is UNPINNED; the GPU
path is pinned to the CPU restatement in oracle/residual_vq.py (tests/test_residual_vq.py).

Per layer i on residual r_i (float32, (N, D)):
  * first call: k-means init (kmeans_iters Lloyd steps from K batch rows) -- eager, one time;
  * q_i = embed[argmin |r_i - e|^2] (aw_vq_forward; counts = bins, sqerr -> commitment loss mse(q_i, r_i));
  * training: EMA of cluster_size / embed_avg, Laplace-smoothed normalisation, expired codes (cluster_size <
    threshold_ema_dead_code) replaced by batch rows -- all on the device (graph-capturable, no host sync);
  * r_{i+1} = r_i - q_i, out += q_i.
Backward (straight-through): dz = nq * g_out + sum_i g_loss_i * 2 (r_i - q_i) / (N D); the codebooks are buffers.

Data parallel: with torch.distributed initialised, bins and per-code sums are all-reduced before the EMA (the
library's distributed codebook sync), and rank 0's codebook state is broadcast after a dead-code replacement.
"""
from __future__ import annotations

import torch
from torch import nn

from . import kernels as K

F32 = torch.float32


def _world(sync=None):
    """Ranks the codebooks synchronise over: the process group's size, or 1 when ``sync`` is False (a Trainer that
    runs each rank as an independent replica, ``devices=1``, sets ``ResidualVQ.sync_codebooks = False``)."""
    if sync is False:
        return 1
    d = torch.distributed
    return d.get_world_size() if d.is_available() and d.is_initialized() else 1


class EuclideanCodebook(nn.Module):
    """One codebook (vector-quantize-pytorch EuclideanCodebook, num_codebooks 1): buffers embed (1, K, D),
    embed_avg (1, K, D), cluster_size (1, K), initted (1,)."""

    def __init__(self, dim, codebook_size, kmeans_init=False, kmeans_iters=10, decay=0.8, eps=1e-5,
                 threshold_ema_dead_code=0):
        super().__init__()
        self.dim, self.codebook_size = dim, codebook_size
        self.kmeans_iters, self.decay, self.eps = kmeans_iters, decay, eps
        self.threshold_ema_dead_code = threshold_ema_dead_code
        if kmeans_init:
            embed = torch.zeros(1, codebook_size, dim)
        else:   # the library's uniform_init: kaiming_uniform_ on the (K, D) table
            embed = torch.empty(1, codebook_size, dim)
            nn.init.kaiming_uniform_(embed[0])
        self.register_buffer("initted", torch.tensor([float(not kmeans_init)]))
        self.register_buffer("cluster_size", torch.zeros(1, codebook_size))
        self.register_buffer("embed_avg", embed.clone())
        self.register_buffer("embed", embed)
        self._initted_host = None      # host mirror of `initted` (read once, then kept in step with it)
        self._ws = None
        self.sync_codebooks = None     # None: follow the process group; False: this rank's codebook only
        self.init_rows = None          # fixed k-means init rows (tests); None draws them like the library

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self._initted_host = None

    def is_initted(self):
        if self._initted_host is None:
            self._initted_host = bool(self.initted.item() > 0)
        return self._initted_host

    @torch.no_grad()
    def kmeans_init(self, r):
        """EuclideanCodebook.init_embed_: k-means on the first batch (rows r (N, D))."""
        if self.kmeans_iters < 1:
            raise ValueError("kmeans_init needs kmeans_iters >= 1 (vector-quantize-pytorch's kmeans returns the "
                             "cluster sizes of its last iteration; with 0 iterations it has none)")
        N, D = r.shape
        Kc, dev = self.codebook_size, r.device
        rows = self.init_rows        # None: the library's draw (randperm(N)[:K], or randint when N < K)
        if rows is None:
            rows = torch.randperm(N, device=dev)[:Kc] if N >= Kc else torch.randint(0, N, (Kc,), device=dev)
        rows = rows.to(dev, torch.int64)
        ws = _world(self.sync_codebooks)
        if ws > 1:
            torch.distributed.broadcast(rows, 0)        # one set of initial means (rank 0's rows ...)
        means = torch.empty(Kc, D, device=dev)
        K.vq_gather(r, rows.contiguous(), means)
        if ws > 1:
            torch.distributed.broadcast(means, 0)       # ... and rank 0's samples
        counts = torch.zeros(Kc, device=dev)
        zq, idx = torch.empty_like(r), torch.empty(N, dtype=torch.int64, device=dev)
        sq = torch.zeros(1, dtype=torch.float64, device=dev)
        for it in range(self.kmeans_iters):
            counts.zero_()
            sq.zero_()
            K.vq_forward(r, means, zq, idx, counts, sq)
            sums = torch.zeros(Kc, D, device=dev)
            K.vq_cluster_sums(r, idx, Kc, sums)
            if ws > 1:
                torch.distributed.all_reduce(counts)
                torch.distributed.all_reduce(sums)
            last = it == self.kmeans_iters - 1
            K.kmeans_update(means, sums, counts, avg=self.embed_avg[0] if last else None)   # embed_avg = means * bins
        self.embed[0].copy_(means)
        self.cluster_size[0].copy_(counts)
        self.initted.fill_(1.0)
        self._initted_host = True

    @torch.no_grad()
    def quantize(self, r, training, salt, seed_ptr):
        """r (N, D) -> (zq (N, D) straight-through values, idx (N,), loss () f32).  Training: EMA update after the
        assignment (the returned rows come from the codebook before the update)."""
        if not self.is_initted():
            self.kmeans_init(r)
        N, D = r.shape
        Kc, dev = self.codebook_size, r.device
        E = self.embed[0]
        zq, idx = torch.empty_like(r), torch.empty(N, dtype=torch.int64, device=dev)
        counts = torch.zeros(Kc, device=dev)
        sq = torch.zeros(1, dtype=torch.float64, device=dev)
        K.vq_forward(r, E, zq, idx, counts, sq)
        loss, perp = torch.zeros((), device=dev), torch.empty((), device=dev)
        if training:
            K.vq_finalize(counts, sq, N, Kc, D, 0.0, loss, perp)     # mse(q, r): commitment_weight 1
            sums = torch.zeros(Kc, D, device=dev)
            K.vq_cluster_sums(r, idx, Kc, sums)
            ws = _world(self.sync_codebooks)
            if ws > 1:
                torch.distributed.all_reduce(counts)
                torch.distributed.all_reduce(sums)
            if self._ws is None or self._ws.device != dev:
                self._ws = torch.empty(2 * Kc, device=dev)
            K.rvq_ema_update(E, self.embed_avg[0], self.cluster_size[0], counts, sums, r, self.decay, self.eps,
                             float(self.threshold_ema_dead_code), salt, seed_ptr, self._ws)
            if ws > 1 and self.threshold_ema_dead_code > 0:
                for t in (self.embed, self.embed_avg, self.cluster_size):
                    torch.distributed.broadcast(t, 0)    # replaced codes came from rank 0's rows
        return zq, idx, loss


class VectorQuantize(nn.Module):
    """vector-quantize-pytorch VectorQuantize with the defaults ResidualVQ uses (no projection, EMA codebook,
    commitment_weight 1)."""

    def __init__(self, dim, codebook_size, kmeans_init=False, kmeans_iters=10, threshold_ema_dead_code=0,
                 decay=0.8, eps=1e-5, commitment_weight=1.0):
        super().__init__()
        self.commitment_weight = commitment_weight
        self._codebook = EuclideanCodebook(dim, codebook_size, kmeans_init, kmeans_iters, decay, eps,
                                           threshold_ema_dead_code)

    @property
    def codebook(self):
        return self._codebook.embed[0]


class ResidualVQ(nn.Module):
    """vector-quantize-pytorch ResidualVQ(num_quantizers, dim, codebook_size, kmeans_init, kmeans_iters,
    threshold_ema_dead_code): forward(x (B, S, D)) -> (quantized (B, S, D), indices (B, S, nq), losses (1, nq))."""

    def __init__(self, num_quantizers, dim, codebook_size, kmeans_init=False, kmeans_iters=10,
                 threshold_ema_dead_code=0, **kw):
        super().__init__()
        self.num_quantizers, self.dim, self.codebook_size = num_quantizers, dim, codebook_size
        self.layers = nn.ModuleList([VectorQuantize(dim, codebook_size, kmeans_init, kmeans_iters,
                                                    threshold_ema_dead_code, **kw) for _ in range(num_quantizers)])
        self._rng_counter = None

    @property
    def sync_codebooks(self):
        """Whether the codebooks all-reduce their EMA statistics across ranks (None: whenever torch.distributed is
        initialised).  Set by arcweld.trainer.Trainer from its data-parallel mode."""
        return self.layers[0]._codebook.sync_codebooks if len(self.layers) else None

    @sync_codebooks.setter
    def sync_codebooks(self, value):
        for layer in self.layers:
            layer._codebook.sync_codebooks = value

    def seed_counter(self, dev):
        """Device counter mixed into the dead-code sampling seed; advanced once per training forward, so captured
        graphs draw fresh rows on every replay."""
        if self._rng_counter is None or self._rng_counter.device != dev:
            self._rng_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        K.counter_add(self._rng_counter, 1)
        return self._rng_counter

    @torch.no_grad()
    def quantize_rows(self, z, training, save=False):
        """z (N, D) f32 contiguous -> (out (N, D), idx (N, nq) int64, losses (nq,) f32, saved (res, q) or None)."""
        N, D = z.shape
        nq, dev = self.num_quantizers, z.device
        ctr = self.seed_counter(dev) if training else None
        out = torch.empty_like(z)
        idx = torch.empty(N, nq, dtype=torch.int64, device=dev)
        losses = torch.empty(nq, device=dev)
        res = torch.empty(nq, N, D, device=dev) if save else None
        qs = torch.empty(nq, N, D, device=dev) if save else None
        r = z
        for i, layer in enumerate(self.layers):
            zq, ii, loss = layer._codebook.quantize(r, training, salt=0x5EED + 7919 * i, seed_ptr=ctr)
            idx[:, i].copy_(ii)
            losses[i:i + 1].copy_(loss.reshape(1))
            if save:
                res[i].copy_(r)
                qs[i].copy_(zq)
            nxt = torch.empty_like(z) if i + 1 < nq else None
            K.rvq_residual(r, zq, out, first=i == 0, r_next=nxt)
            r = nxt
        return out, idx, losses, ((res, qs) if save else None)

    def forward(self, x):
        shape = x.shape
        z = x.reshape(-1, self.dim).to(F32).contiguous()
        out, idx, losses = _RVQFunction.apply(z, self, self.training)
        return out.view(shape), idx.view(*shape[:-1], self.num_quantizers), losses.view(1, self.num_quantizers)


class _RVQFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, rvq, training):
        out, idx, losses, saved = rvq.quantize_rows(z, training, save=True)
        ctx.saved = saved
        ctx.mark_non_differentiable(idx)
        return out, idx, losses

    @staticmethod
    def backward(ctx, g_out, g_idx, g_losses):
        res, qs = ctx.saved
        ctx.saved = None
        nq, N, D = res.shape
        dz = torch.empty(N, D, device=res.device)
        gl = g_losses.reshape(nq).contiguous() if g_losses is not None else torch.zeros(nq, device=res.device)
        K.rvq_backward(res, qs, g_out.contiguous() if g_out is not None else None, gl, dz)
        return dz, None, None
