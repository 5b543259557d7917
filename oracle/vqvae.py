"""CPU restatement (fp32, torch autograd on CPU) of the reference VQ-VAE-Patch training path.

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module.

Parity pin: every function below is checked against golden vectors produced by the reference itself
(``tests/golden/make_golden.py`` imports /root/reference/model/*.py through a stub shim) in
``tests/test_oracle.py``.

Written functionally on a reference-layout ``state_dict`` with a TOKEN-MAJOR activation layout
(B, S, H) instead of the reference's (B, H, S); the arithmetic is the same:

* patchify           model/vq_vae_patch_embedd.py:13-17   channel-major flatten, Conv1d(1->H, k=P, s=P)
* encoder ResBlocks  model/vq_vae_patch_embedd.py:60-74, 103-114 (seperate=True: each token alone, so a
                     k=3/pad=1 conv on a length-1 slice sees only its centre tap weight[:, :, 1])
* SepCNNBlock        model/vq_vae_patch_embedd.py:77-91   per-token Conv1d(H->D, k=1), then (B,S,D)
* VectorQuantizer    model/vector_quantizer.py:76-119     expanded L2, first-index argmin, STE, perplexity
* decoder            model/vq_vae_patch_embedd.py:142-145 Conv1d(D->H, k=1), ResBlocks with real k=3 convs
                     along the token axis (zero padded per window)
* un-patchify        model/vq_vae_patch_embedd.py:19-57   ConvT(H->H) -> BatchNorm1d(train stats) -> GELU(erf)
                     -> ConvT(H->1, k5, s5) -> reshape (B,200,2) interleaved
* loss               model/autencoder_lightning_base.py:80-84  mse(x_hat, x) + embedding loss
"""
from __future__ import annotations

import math

import numpy as np

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def gelu_erf(x):
    return 0.5 * x * (1.0 + torch.erf(x * (1.0 / math.sqrt(2.0))))


def _bn_train(x, gamma, beta, run_mean, run_var, axes):
    """BatchNorm1d in training mode: biased batch variance for normalisation, unbiased for running var."""
    n = 1
    for a in axes:
        n *= x.shape[a]
    mean = x.mean(dim=axes, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=axes, keepdim=True)
    y = (x - mean) / torch.sqrt(var + BN_EPS) * gamma + beta
    if run_mean is not None:
        with torch.no_grad():
            run_mean.mul_(1 - BN_MOMENTUM).add_(BN_MOMENTUM * mean.reshape(-1))
            run_var.mul_(1 - BN_MOMENTUM).add_(BN_MOMENTUM * var.reshape(-1) * n / max(n - 1, 1))
    return y


def _bn_eval(x, gamma, beta, run_mean, run_var):
    return (x - run_mean) / torch.sqrt(run_var + BN_EPS) * gamma + beta


def vq_quantize(z, E, beta):
    """model/vector_quantizer.py:76-119.  z (..., D) -> (loss, z_q_ste, perplexity, idx (N,) int64, counts (K,))."""
    D = E.shape[1]
    zf = z.reshape(-1, D)
    dist = (zf ** 2).sum(1, keepdim=True) + (E ** 2).sum(1) - 2 * zf @ E.t()
    idx = torch.argmin(dist, dim=1)
    zq = E[idx].view(z.shape)
    loss = torch.mean((zq.detach() - z) ** 2) + beta * torch.mean((zq - z.detach()) ** 2)
    zq_ste = z + (zq - z).detach()
    counts = torch.bincount(idx, minlength=E.shape[0]).to(z.dtype)
    p = counts / zf.shape[0]
    perplexity = torch.exp(-torch.sum(p * torch.log(p + 1e-10)))
    return loss, zq_ste, perplexity, idx, counts


class VQVAEConfig:
    def __init__(self, hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25,
                 seq_len=200, input_dim=2, batch_norm=False, beta=0.25, dropout_p=0.0):
        self.H, self.K, self.D, self.R = hidden_dim, num_embeddings, embedding_dim, n_resblocks
        self.P, self.L, self.C = patch_size, seq_len, input_dim
        self.bn, self.beta, self.dropout_p = batch_norm, beta, dropout_p
        self.S = seq_len // patch_size * input_dim           # tokens per window (enc_out_len)
        self.k1 = {25: 5, 10: 2, 50: 10}[patch_size]         # first ConvT kernel = stride


def _resblock(x, sd, pre, taps, cfg, train, token_axis_conv):
    """ResBlock (model/vq_vae_patch_embedd.py:60-74) on token-major x (B, S, H)."""
    def conv(a, w, b):
        if not token_axis_conv:                          # length-1 slices: centre tap only
            return a @ w[:, :, 1].t() + b
        ap = F.pad(a, (0, 0, 1, 1))                      # zero-pad one token each side, per window
        S = a.shape[1]
        return sum(ap[:, j:j + S, :] @ w[:, :, j].t() for j in range(3)) + b

    def bn(a, idx):
        if not cfg.bn:
            return a
        g, bb = sd[f"{pre}.block.{idx}.weight"], sd[f"{pre}.block.{idx}.bias"]
        rm, rv = sd[f"{pre}.block.{idx}.running_mean"], sd[f"{pre}.block.{idx}.running_var"]
        if not train:
            return _bn_eval(a, g, bb, rm, rv)
        if token_axis_conv:                              # decoder: stats over (B, S)
            return _bn_train(a, g, bb, rm, rv, axes=(0, 1))
        # encoder: the shared ResBlock runs once per token slice -> per-slice stats over B and
        # 16 sequential running-stat updates in token order (vq_vae_patch_embedd.py:108-110)
        outs = [_bn_train(a[:, t:t + 1, :], g, bb, rm, rv, axes=(0, 1)) for t in range(a.shape[1])]
        return torch.cat(outs, dim=1)

    h = conv(gelu_erf(x), sd[f"{pre}.block.1.weight"], sd[f"{pre}.block.1.bias"])
    h = bn(h, 2)
    o = conv(gelu_erf(h), sd[f"{pre}.block.4.weight"], sd[f"{pre}.block.4.bias"])
    o = bn(o, 5)
    return x + o


def vqvae_forward(sd, x, cfg: VQVAEConfig, train=True, capture=None, quantizer=None):
    """Returns (embedding_loss, x_hat, perplexity) like VQVAEPatch.forward (vq_vae_patch_embedd.py:155-167).
    ``quantizer(z) -> (loss, z_q_ste, perplexity, idx)`` replaces the VectorQuantizer (e.g. the residual VQ of
    oracle/residual_vq.torch_quantizer for --use-improved-vq)."""
    B = x.shape[0]
    h = patch_embed(sd, x, cfg, "patch_embed.")                                 # (B,S,H)
    for r in range(cfg.R):
        h = _resblock(h, sd, f"encoder.0.shared_conv.{r}", None, cfg, train, token_axis_conv=False)
    z = h @ sd["encoder.1.shared_conv.weight"][:, :, 0].t() + sd["encoder.1.shared_conv.bias"]  # (B,S,D)
    if quantizer is None:
        emb_loss, zq, perplexity, idx, _ = vq_quantize(z, sd["vector_quantization.embedding.weight"], cfg.beta)
    else:
        emb_loss, zq, perplexity, idx = quantizer(z)
    if capture is not None:
        capture["z_e"] = z
        capture["idx"] = idx
    h = zq @ sd["decoder.0.weight"][:, :, 0].t() + sd["decoder.0.bias"]
    for r in range(cfg.R):
        h = _resblock(h, sd, f"decoder.1.shared_conv.{r}", None, cfg, train, token_axis_conv=True)
    x_hat = unpatch(sd, h, cfg, train, "reverse_patch_embed.")
    return emb_loss, x_hat, perplexity


def patch_embed(sd, x, cfg: VQVAEConfig, p):
    """PatchEmbedding (vq_vae_patch_embedd.py:7-17): windows (B, L, C) -> token-major (B, S, H)."""
    B = x.shape[0]
    flat = x.transpose(1, 2).reshape(B, cfg.L * cfg.C)                         # channel-major
    patches = flat.view(B, cfg.S, cfg.P)
    return patches @ sd[p + "proj.weight"][:, 0, :].t() + sd[p + "proj.bias"]


def unpatch(sd, h, cfg: VQVAEConfig, train, p):
    """PatchEmbeddingInverse (vq_vae_patch_embedd.py:19-57): token-major (B, S, H) -> (B, L, C)."""
    B = h.shape[0]
    # ConvT(H->H, k=k1, s=k1): position k1*t + j, channel o
    w1 = sd[p + "proj.0.weight"]                                               # (H_in, H_out, k1)
    y = torch.einsum("bti,ioj->btjo", h, w1).reshape(B, h.shape[1] * cfg.k1, -1) + sd[p + "proj.0.bias"]
    g, bb = sd[p + "proj.1.weight"], sd[p + "proj.1.bias"]
    rm, rv = sd[p + "proj.1.running_mean"], sd[p + "proj.1.running_var"]
    y = _bn_train(y, g, bb, rm, rv, axes=(0, 1)) if train else _bn_eval(y, g, bb, rm, rv)
    a = gelu_erf(y)
    w2 = sd[p + "proj.3.weight"]                                               # (H, 1, 5)
    out = torch.einsum("bqo,oj->bqj", a, w2[:, 0, :]).reshape(B, -1) + sd[p + "proj.3.bias"]
    return out.view(B, -1, cfg.C)                                              # interleaved reshape


def vqvae_train_step_grads(sd_np, x_np, cfg: VQVAEConfig, train=True, quantizer=None):
    """fwd + bwd of loss = mse(x_hat, x) + emb_loss (autencoder_lightning_base.py:80-84). Returns outputs,
    gradients keyed by reference parameter name, and the post-forward state (BN running stats)."""
    sd = {k: torch.tensor(v).clone() for k, v in sd_np.items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items()
              if not (k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"))}
    x = torch.tensor(x_np)
    cap = {}
    emb_loss, x_hat, perp = vqvae_forward(sd, x, cfg, train=train, capture=cap, quantizer=quantizer)
    recon = F.mse_loss(x_hat, x)
    loss = recon + emb_loss
    loss.backward()
    grads = {k: (p.grad.numpy() if p.grad is not None else None) for k, p in params.items()}
    state = {k: v.detach().numpy() for k, v in sd.items()
             if k.endswith("running_mean") or k.endswith("running_var")}
    out = dict(x_hat=x_hat.detach().numpy(), emb_loss=emb_loss.detach().numpy(),
               perplexity=None if perp is None else perp.detach().numpy(),
               recon=recon.detach().numpy(), loss=loss.detach().numpy(), idx=cap["idx"].numpy(),
               z_e=cap["z_e"].detach().numpy())
    return out, grads, state


def reference_state_dict_shapes(cfg: VQVAEConfig):
    """Parameter/buffer names and shapes of a reference VQVAEPatch state_dict (vq_vae_patch_embedd.py:117-151)."""
    H, D, K, P, k1 = cfg.H, cfg.D, cfg.K, cfg.P, cfg.k1
    shapes = {"patch_embed.proj.weight": (H, 1, P), "patch_embed.proj.bias": (H,)}
    for stack in ("encoder.0", "decoder.1"):
        for r in range(cfg.R):
            for i in (1, 4):
                shapes[f"{stack}.shared_conv.{r}.block.{i}.weight"] = (H, H, 3)
                shapes[f"{stack}.shared_conv.{r}.block.{i}.bias"] = (H,)
            if cfg.bn:
                for i in (2, 5):
                    p = f"{stack}.shared_conv.{r}.block.{i}"
                    shapes[p + ".weight"] = (H,)
                    shapes[p + ".bias"] = (H,)
                    shapes[p + ".running_mean"] = (H,)
                    shapes[p + ".running_var"] = (H,)
                    shapes[p + ".num_batches_tracked"] = ()
    shapes["encoder.1.shared_conv.weight"] = (D, H, 1)
    shapes["encoder.1.shared_conv.bias"] = (D,)
    shapes["vector_quantization.embedding.weight"] = (K, D)
    shapes["decoder.0.weight"] = (H, D, 1)
    shapes["decoder.0.bias"] = (H,)
    shapes["reverse_patch_embed.proj.0.weight"] = (H, H, k1)
    shapes["reverse_patch_embed.proj.0.bias"] = (H,)
    shapes["reverse_patch_embed.proj.1.weight"] = (H,)
    shapes["reverse_patch_embed.proj.1.bias"] = (H,)
    shapes["reverse_patch_embed.proj.1.running_mean"] = (H,)
    shapes["reverse_patch_embed.proj.1.running_var"] = (H,)
    shapes["reverse_patch_embed.proj.1.num_batches_tracked"] = ()
    shapes["reverse_patch_embed.proj.3.weight"] = (H, 1, 5)
    shapes["reverse_patch_embed.proj.3.bias"] = (1,)
    return shapes


def det_state_dict(cfg: VQVAEConfig, base: int):
    from oracle import gen
    return {k: gen.param_value(base, k, s) for k, s in reference_state_dict_shapes(cfg).items()}


def encode_ids(sd, x, cfg: VQVAEConfig, n_cycles: int):
    """Frozen-encoder tokenization, restating the reference loop (latentspace_dataloader.py:154-161, 228-250):
    for each window i: patch_embed -> encoder -> VQ idx (B*S,) -> (B, S); stack (n_cycles, B, S), swap to
    (B, n_cycles, S) and flatten the trailing axes (:261).  x: (B, n_cycles*L, C) numpy f32 -> int64 (B, n_cycles*S).
    Eval semantics: torch.no_grad, dropout off (encoder BN off, --batchnorm 0)."""
    st = {k: torch.as_tensor(v) for k, v in sd.items()}
    t_x = []
    with torch.no_grad():
        for i in range(n_cycles):
            xi = torch.as_tensor(np.ascontiguousarray(x[:, i * cfg.L:(i + 1) * cfg.L, :]))
            cap = {}
            vqvae_forward(st, xi, cfg, train=False, capture=cap)
            t_x.append(cap["idx"].numpy().reshape(xi.shape[0], -1))
    return np.array(t_x).swapaxes(0, 1).reshape(x.shape[0], -1).astype(np.int64)


def autoregressive_pairs(data):
    """MyLatentAutoregressiveDataset (base_dataloader.py:84-97): start = max+1, end = max+2, classes = max+3;
    x = [start, ids], y = [ids, end]."""
    mx = int(np.max(data))
    n = len(data)
    x = np.concatenate([np.full((n, 1), mx + 1), data], axis=1)
    y = np.concatenate([data, np.full((n, 1), mx + 2)], axis=1)
    return x, y, mx + 3
