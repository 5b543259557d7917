"""CPU restatement (numpy, float32) of the residual VQ with EMA codebooks behind ResidualVQLightning.

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module.

PARITY UNPINNED.  The reference (model/vector_quantizer.py:9-56; used by model/vq_vae_patch_embedd.py:132-136 when
``--use-improved-vq``) wraps ``vector_quantize_pytorch.ResidualVQ`` (environment.yaml:34, no version pin).  That
library is not installed here and the reference holds no test, fixture or output of it, so this module restates the
library's published algorithm (ResidualVQ -> VectorQuantize -> EuclideanCodebook, defaults decay 0.8, eps 1e-5,
commitment_weight 1, no learnable codebook, EMA update on) and the GPU path is checked against THIS restatement:

* ResidualVQ.forward            residual r_0 = x;  per layer: (q_i, idx_i, loss_i) = layer(r_i);
                                r_{i+1} = r_i - q_i (detached); out = sum q_i; losses stacked (1, nq)
* EuclideanCodebook.init_embed_ k-means init on the first call: means = rows sampled from the batch, kmeans_iters
                                Lloyd steps with -cdist argmax assignment, empty clusters keep their mean;
                                embed = means, cluster_size = bins of the last step, embed_avg = means * bins
* EuclideanCodebook.forward     idx = argmin |x - e|^2 (first index on ties), q = embed[idx] (before the update);
                                training: cs = ema(cs, bins), avg = ema(avg, sum_n onehot x), embed = avg /
                                laplace(cs) * sum(cs); expire codes with cs < threshold
* VectorQuantize.forward        q_ste = x + (q - x).detach();  training: loss = mse(q.detach(), x), eval: 0

Two places where the library draws random numbers are inputs here: the k-means init rows (``init_rows``, the
library's randperm(N)[:K] / randint) and the dead-code replacement rows, which the HIP kernel draws from a counter
hash (stratified: the expired code of rank j takes a row of the j-th of n_exp equal strata) -- restated bit for bit
by ``dead_code_rows`` below, so the two paths replace codes with the same rows.
"""
from __future__ import annotations

import numpy as np

DECAY = 0.8
EPS = 1e-5
M64 = (1 << 64) - 1


def _hash_group(seed: int, g: int) -> int:
    """aw_hash_group (csrc/common.h): one splitmix64 draw."""
    z = (seed + (g + 1) * 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _seed_mix(salt: int, ctr: int) -> int:
    """aw_seed_mix_value (csrc/common.h)."""
    z = (salt ^ ((ctr * 0xD1B54A32D192ED03 + 0x8CB92BA72F3D8DD7) & M64)) & M64
    z = ((z ^ (z >> 32)) * 0xD6E8FEB86659FD93) & M64
    return z ^ (z >> 32)


def dead_code_rows(expired: np.ndarray, N: int, salt: int, ctr: int | None) -> np.ndarray:
    """Row index per code (-1 when not expired), the rule of aw_rvq_ema_update."""
    seed = _seed_mix(salt & M64, ctr) if ctr is not None else salt & M64
    n_exp = int(expired.sum())
    rows = np.full(expired.shape[0], -1, dtype=np.int64)
    for j, k in enumerate(np.flatnonzero(expired)):
        h = _hash_group(seed, j)
        if n_exp <= N:
            lo, hi = j * N // n_exp, (j + 1) * N // n_exp
            rows[k] = lo + h % (hi - lo)
        else:
            rows[k] = h % N
    return rows


def assign(x: np.ndarray, embed: np.ndarray) -> np.ndarray:
    """Nearest code, first index on ties (squared Euclidean distance in float64: the restatement's tie margin is
    far below float32 rounding, so index checks use inputs without near-ties)."""
    d = ((x.astype(np.float64)[:, None, :] - embed.astype(np.float64)[None, :, :]) ** 2).sum(-1)
    return d.argmin(1)


def kmeans(samples: np.ndarray, K: int, iters: int, init_rows: np.ndarray):
    if iters < 1:
        raise ValueError("kmeans_iters must be >= 1 (the library's kmeans returns the bins of its last iteration)")
    means = samples[init_rows].astype(np.float32).copy()
    bins = None
    for _ in range(iters):
        idx = assign(samples, means)
        bins = np.bincount(idx, minlength=K).astype(np.float32)
        sums = np.zeros((K, samples.shape[1]), np.float32)
        np.add.at(sums, idx, samples.astype(np.float32))
        new = sums / np.maximum(bins, 1)[:, None]
        means = np.where((bins == 0)[:, None], means, new).astype(np.float32)
    return means, bins


class Codebook:
    """State of one EuclideanCodebook (embed, embed_avg (K, D), cluster_size (K,), initted)."""

    def __init__(self, K, D, kmeans_iters, threshold):
        self.K, self.D, self.iters, self.threshold = K, D, kmeans_iters, float(threshold)
        self.embed = np.zeros((K, D), np.float32)
        self.embed_avg = np.zeros((K, D), np.float32)
        self.cluster_size = np.zeros(K, np.float32)
        self.initted = False

    def init(self, x, init_rows):
        means, bins = kmeans(x, self.K, self.iters, init_rows)
        self.embed, self.cluster_size = means, bins
        self.embed_avg = (means * bins[:, None]).astype(np.float32)
        self.initted = True

    def forward(self, x, training, init_rows=None, salt=0, ctr=None):
        """x (N, D) float32 -> (quantized (N, D) from the pre-update codebook, idx (N,), loss, raw codebook rows)."""
        if not self.initted:
            self.init(x, init_rows)
        idx = assign(x, self.embed)
        q = self.embed[idx].copy()
        q_ste = (x + (q - x)).astype(np.float32) if training else q       # eval: no straight-through
        loss = float(np.mean((q.astype(np.float64) - x) ** 2)) if training else 0.0   # mse(quantize.detach(), x)
        if training:
            bins = np.bincount(idx, minlength=self.K).astype(np.float32)
            sums = np.zeros((self.K, self.D), np.float32)
            np.add.at(sums, idx, x.astype(np.float32))
            cs = (self.cluster_size * DECAY + bins * (1 - DECAY)).astype(np.float32)
            avg = (self.embed_avg * DECAY + sums * (1 - DECAY)).astype(np.float32)
            tot = cs.sum(dtype=np.float32)
            smooth = ((cs + EPS) / (tot + self.K * EPS) * tot).astype(np.float32)
            embed = (avg / smooth[:, None]).astype(np.float32)
            expired = (cs < self.threshold) if self.threshold > 0 else np.zeros(self.K, bool)
            rows = dead_code_rows(expired, x.shape[0], salt, ctr)
            for k in np.flatnonzero(expired):
                embed[k] = x[rows[k]]
                avg[k] = x[rows[k]] * self.threshold
                cs[k] = self.threshold
            self.embed, self.embed_avg, self.cluster_size = embed, avg, cs
        return q_ste, idx, loss, q


def residual_vq_forward(books, x, training, init_rows=None, salts=None, ctr=None):
    """ResidualVQ.forward over a list of Codebook: returns (out (N, D), idx (N, nq), losses (nq,), residuals
    (nq, N, D), raw codebook rows (nq, N, D))."""
    r = x.astype(np.float32)
    out = np.zeros_like(r)
    idxs, losses, res, qs = [], [], [], []
    for i, cb in enumerate(books):
        q, idx, loss, raw = cb.forward(r, training, None if init_rows is None else init_rows[i],
                                       0 if salts is None else salts[i], ctr)
        res.append(r)
        qs.append(raw)
        out = (out + q).astype(np.float32)
        r = (r - q).astype(np.float32)
        idxs.append(idx)
        losses.append(loss)
    return out, np.stack(idxs, -1), np.array(losses, np.float32), np.stack(res), np.stack(qs)


def residual_vq_backward(res, qs, g_out, g_losses, commitment=1.0):
    """dx of sum(out * g_out) + sum(g_losses * losses): nq * g_out + sum_i g_i * c * 2 (r_i - q_i) / (N D)."""
    nq, N, D = res.shape
    dz = nq * g_out.astype(np.float64)
    for i in range(nq):
        dz = dz + g_losses[i] * commitment * 2.0 * (res[i].astype(np.float64) - qs[i]) / (N * D)
    return dz.astype(np.float32)


def torch_quantizer(embeds, commitment=1.0):
    """The residual VQ's forward as a torch-autograd quantizer for oracle/vqvae.vqvae_forward: codebooks fixed
    (embeds: list of (K, D) arrays, the state before the step), z_q = sum of straight-through layer outputs,
    loss = sum_i commitment * mse(q_i.detach(), r_i) (for one quantizer the reference's (1, 1) loss), perplexity None,
    idx of the first layer."""
    import torch

    Es = [torch.tensor(np.asarray(e, np.float32)) for e in embeds]

    def q(z):
        D = z.shape[-1]
        r = z.reshape(-1, D)
        out = torch.zeros_like(r)
        loss = torch.zeros(())
        first = None
        for E in Es:
            idx = torch.tensor(assign(r.detach().numpy(), E.numpy()))
            raw = E[idx]
            ste = r + (raw - r).detach()
            loss = loss + commitment * torch.mean((raw.detach() - r) ** 2)
            out = out + ste
            r = r - ste.detach()
            first = idx if first is None else first
        return loss, out.view(z.shape), None, first

    return q
