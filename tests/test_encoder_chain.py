"""The fused encoder ResBlock chain (csrc/encoder_chain.hip, aw_encoder_chain_fwd) against the per-block GEMM
launches it replaces (ARCWELD_ENCODER_CHAIN=0): every saved tensor of the forward (h, gelu(h), x, gelu(x) per
block), the dropout masks (the GEMM epilogue's counter hash), the train step's outputs and every gradient, in bf16
operands at the bench shape and on a ragged token count."""
import os

import numpy as np
import pytest
import torch

from oracle import gen
from oracle import vqvae as ov

pytestmark = pytest.mark.gpu
KW = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)


def _model(seed, dropout):
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=dropout, batch_norm=False, **KW)
    sd = ov.det_state_dict(ov.VQVAEConfig(**KW), seed)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().train()


def _run(m, x, chain, monkeypatch):
    from arcweld import vqvae as V
    from arcweld.functional import mse_loss
    from arcweld import kernels as K
    monkeypatch.setenv("ARCWELD_ENCODER_CHAIN", "1" if chain else "0")
    calls = []
    monkeypatch.setattr(K, "encoder_chain_fwd", lambda *a, _f=K.encoder_chain_fwd, **k: calls.append(1) or _f(*a, **k))
    m._rng_counter = torch.zeros(1, dtype=torch.int64, device="cuda")     # same dropout masks for both runs
    m.zero_grad()
    emb, x_hat, _, idx, sv = V.forward(m, x, True, need_backward=True, seed=7)
    saved = {"h": [t.float() for t in sv.hs], "a1": [t.float() for t in sv.a1s],
             "x": [t for t in sv.xs[1:-1]], "a0": [t.float() for t in sv.a0s[1:]]}
    m._rng_counter = torch.zeros(1, dtype=torch.int64, device="cuda")
    emb, x_hat, perp = m(x)
    (mse_loss(x_hat, x) + emb).backward()
    assert len(calls) == (2 if chain else 0)      # the fused launch is what ran (or did not)
    return saved, x_hat.detach(), m._last_indices.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("B,dropout", [(1024, 0.1), (37, 0.0)])
def test_encoder_chain_matches_per_block_launches_bf16(B, dropout, monkeypatch):
    from arcweld.precision import operands
    m = _model(2101, dropout)
    x = torch.tensor(gen.windows(2102, B), device="cuda")
    with operands(torch.bfloat16):
        a = _run(m, x, True, monkeypatch)
        b = _run(m, x, False, monkeypatch)
    for k in a[0]:
        for r, (u, v) in enumerate(zip(a[0][k], b[0][k])):
            # same bf16 operands and MFMA instruction; only the order of the partial sums may differ
            torch.testing.assert_close(u, v, rtol=2e-2, atol=2e-2, msg=f"{k}[{r}]")
            assert (u - v).norm() / (v.norm() + 1e-20) < 5e-3, (k, r)
    rel = ((a[1] - b[1]).norm() / b[1].norm()).item()
    assert rel < 5e-3, rel
    assert (a[2] == b[2]).float().mean().item() > 0.99
    for n, g in b[3].items():
        if n == "reverse_patch_embed.proj.0.bias":
            continue
        rel = ((a[3][n] - g).norm() / (g.norm() + 1e-20)).item()
        assert rel < 2e-2, (n, rel)
