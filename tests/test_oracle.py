"""The CPU oracle (oracle/*.py) against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  No GPU needed."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import gen
from oracle import vqvae as ov
from oracle import decoder as od
from oracle import optim as oo


def test_generator_is_stable():
    # counter-based: identical across calls and a prefix of a longer draw
    a = gen.uniform(7, (10,), -1, 1)
    b = gen.uniform(7, (20,), -1, 1)[:10]
    assert np.array_equal(a, b)
    assert gen.splitmix64(0, 1)[0] == np.uint64(0xE220A8397B1DCDAF)


def test_vq_small_matches_reference():
    g = golden("vq_small.npz")
    E = torch.tensor(gen.uniform(101, (64, 16), -0.5, 0.5), requires_grad=True)
    z = torch.tensor(gen.normal(102, (16, 16, 16), 0.5), requires_grad=True)
    g_zq = torch.tensor(gen.normal(103, (16, 16, 16), 1.0))
    loss, zq, perp, idx, counts = ov.vq_quantize(z, E, 0.25)
    (float(g["g_loss"]) * loss + (zq * g_zq).sum()).backward()
    assert np.array_equal(idx.numpy(), g["idx"].reshape(-1))
    np.testing.assert_allclose(zq.detach().numpy(), g["z_q"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-6)
    np.testing.assert_allclose(perp.item(), g["perplexity"], rtol=1e-6)
    np.testing.assert_allclose(z.grad.numpy(), g["dz"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(E.grad.numpy(), g["dE"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("tag,K,D,N,eseed,estd", [
    ("K512_D64_init", 512, 64, 16384, 201, None),
    ("K512_D64_trained", 512, 64, 16384, 202, 0.08),
    ("K8192_D256_trained", 8192, 256, 4096, 203, 0.05),
])
def test_vq_indices_bit_exact(tag, K, D, N, eseed, estd):
    g = golden("vq_idx.npz")
    z = gen.normal(210 + K, (N, D), 0.08)
    E = gen.uniform(eseed, (K, D), -1.0 / K, 1.0 / K) if estd is None else gen.normal(eseed, (K, D), estd)
    _, _, perp, idx, _ = ov.vq_quantize(torch.tensor(z), torch.tensor(E), 0.25)
    ref = g[f"idx_{tag}"].astype(np.int64)
    assert np.array_equal(idx.numpy(), ref), f"{(idx.numpy() != ref).sum()} mismatches"
    np.testing.assert_allclose(perp.item(), g[f"perplexity_{tag}"], rtol=1e-5)


VQVAE_CASES = [
    ("vqvae_small.npz", dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25,
                             batch_norm=False), 8, 301, 302),
    ("vqvae_small_bn.npz", dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25,
                                batch_norm=True), 8, 303, 304),
    ("vqvae_small_p10.npz", dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=1, patch_size=10,
                                 batch_norm=False), 4, 305, 306),
    ("vqvae_small_p50.npz", dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=1, patch_size=50,
                                 batch_norm=False), 4, 307, 308),
]


@pytest.mark.parametrize("fname,kw,B,wseed,xseed", VQVAE_CASES)
def test_vqvae_train_step_matches_reference(fname, kw, B, wseed, xseed):
    g = golden(fname)
    cfg = ov.VQVAEConfig(**kw)
    sd = ov.det_state_dict(cfg, wseed)
    x = gen.windows(xseed, B)
    out, grads, state = ov.vqvae_train_step_grads(sd, x, cfg)
    assert np.array_equal(out["idx"], g["idx"])
    np.testing.assert_allclose(out["x_hat"], g["x_hat"], rtol=1e-5, atol=1e-5)
    for k in ("emb_loss", "perplexity", "recon", "loss"):
        np.testing.assert_allclose(out[k], g[k], rtol=1e-5, err_msg=k)
    for k, v in grads.items():
        np.testing.assert_allclose(v, g["grad/" + k], rtol=1e-4, atol=1e-6, err_msg=k)
    assert set("grad/" + k for k in grads) == set(f for f in g.files if f.startswith("grad/"))
    for k, v in state.items():
        np.testing.assert_allclose(v, g["state/" + k], rtol=1e-5, atol=1e-6, err_msg=k)
    # eval mode uses the (updated) running statistics
    sd2 = dict(sd)
    sd2.update(state)
    with torch.no_grad():
        e2, xh2, _ = ov.vqvae_forward({k: torch.tensor(v) for k, v in sd2.items()}, torch.tensor(x), cfg, train=False)
    np.testing.assert_allclose(xh2.numpy(), g["eval_x_hat"], rtol=1e-5, atol=1e-5)


def test_vqvae_full_size_matches_reference():
    g = golden("vqvae_full_b4.npz")
    cfg = ov.VQVAEConfig()
    sd = ov.det_state_dict(cfg, 309)
    out, grads, _ = ov.vqvae_train_step_grads(sd, gen.windows(310, 4), cfg)
    assert np.array_equal(out["idx"], g["idx"])
    np.testing.assert_allclose(out["x_hat"], g["x_hat"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["loss"], g["loss"], rtol=1e-5)
    for k, v in grads.items():
        # atol floor: the ConvT bias feeding train-mode BN has an exactly-zero gradient (rounding noise ~1e-8)
        np.testing.assert_allclose(np.linalg.norm(v.astype(np.float64)), g["gnorm/" + k], rtol=1e-4, atol=1e-6,
                                   err_msg=k)
        sl = g["gslice/" + k]
        np.testing.assert_allclose(v.reshape(-1)[:64], sl, rtol=1e-3, atol=1e-4 * np.abs(sl).max() + 1e-7, err_msg=k)


DEC_CASES = [
    ("decoder_small.npz", dict(d_model=64, n_classes=34, seq_len=33, n_blocks=2), 4, 4, 401, 402, False),
    ("decoder_small_bias.npz", dict(d_model=64, n_classes=34, seq_len=33, n_blocks=2), 4, 3, 403, 404, True),
]


def _dec_inputs(B, T, V, xseed):
    x = gen.randint(xseed, (B, T), 0, V)
    y = gen.randint(xseed + 1, (B, T), 0, V)
    y[:, -3:] = -1
    cond = gen.randint(xseed + 2, (B,), 0, 2)
    return x, y, cond


@pytest.mark.parametrize("fname,kw,n_head,B,wseed,xseed,bias", DEC_CASES)
def test_decoder_matches_reference(fname, kw, n_head, B, wseed, xseed, bias):
    g = golden(fname)
    sd = od.det_state_dict(wseed, class_h_bias=bias, **kw)
    x, y, cond = _dec_inputs(B, kw["seq_len"], kw["n_classes"], xseed)
    for task, t in (("generate", "gen"), ("classification", "cls")):
        loss, logits, grads = od.decoder_step_grads(sd, x, y, cond, n_head, task)
        np.testing.assert_allclose(loss, g[f"{t}/loss"], rtol=1e-5)
        np.testing.assert_allclose(logits, g[f"{t}/logits"], rtol=1e-5, atol=1e-5)
        assert sorted(grads) == sorted(g[f"{t}/grad_names"].tolist())
        for k, v in grads.items():
            np.testing.assert_allclose(v, g[f"{t}/grad/{k}"], rtol=1e-4, atol=1e-6, err_msg=k)


def test_decoder_full_size_matches_reference():
    g = golden("decoder_full_b2.npz")
    kw = dict(d_model=512, n_classes=514, seq_len=321, n_blocks=8)
    sd = od.det_state_dict(405, **kw)
    x, y, cond = _dec_inputs(2, 321, 514, 406)
    loss, logits, grads = od.decoder_step_grads(sd, x, y, cond, 8, "generate")
    np.testing.assert_allclose(loss, g["gen/loss"], rtol=1e-5)
    np.testing.assert_allclose(logits[:, :, :32], g["gen/logits_slice"], rtol=1e-4, atol=1e-5)
    for k, v in grads.items():
        np.testing.assert_allclose(np.linalg.norm(v.astype(np.float64)), g["gen/gnorm/" + k], rtol=1e-4, err_msg=k)


def test_pe_cap_at_512_rows():
    sd = od.det_state_dict(1, d_model=64, n_classes=10, seq_len=600, n_blocks=1)
    with pytest.raises(RuntimeError):
        od.decoder_forward({k: torch.tensor(v) for k, v in sd.items()}, torch.zeros(1, 600, dtype=torch.long), 4)


@pytest.mark.parametrize("tag,betas,groups", [
    ("vqvae", (0.9, 0.999), [(0.0, [0, 1, 2])]),
    ("decoder", (0.9, 0.95), [(0.1, [0, 2]), (0.0, [1])]),
])
def test_radam_and_clip_match_reference(tag, betas, groups):
    g = golden("radam.npz")
    shapes = [(33, 7), (7,), (5, 3, 2)]
    params = [gen.normal(500 + i, s, 0.3) for i, s in enumerate(shapes)]
    wd = [0.0] * 3
    for w, idx in groups:
        for i in idx:
            wd[i] = w
    st = oo.RAdamState(shapes)
    for step in range(8):
        grads = [gen.normal(600 + 17 * step + i, s, 1.0) for i, s in enumerate(shapes)]
        tot = oo.clip_grad_norm(grads, 0.7)
        np.testing.assert_allclose(tot, g[f"{tag}/prenorm_{step}"], rtol=1e-6)
        oo.radam_step(params, grads, st, 1e-3, betas, 1e-8, wd)
        for i, p in enumerate(params):
            np.testing.assert_allclose(p, g[f"{tag}/p{i}_step{step}"], rtol=1e-6, atol=1e-7)
