"""Frozen-encoder tokenization: oracle pinned on the reference's fixture indices; the fused GPU
encoder + VQ pass is bit-exact against the oracle for multi-cycle sequences."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import gen
from oracle import vqvae as ov

SMALL = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
FULL = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)


def test_oracle_encode_ids_matches_reference_fixture():
    g = golden("vqvae_small.npz")
    cfg = ov.VQVAEConfig(**SMALL)
    sd = ov.det_state_dict(cfg, 301)
    x = gen.windows(302, 8)
    ids = ov.encode_ids(sd, x, cfg, n_cycles=1)
    assert ids.shape == (8, 16) and ids.dtype == np.int64
    assert np.array_equal(ids.reshape(-1), g["idx"])


def test_oracle_encode_ids_cycle_order():
    cfg = ov.VQVAEConfig(**SMALL)
    sd = ov.det_state_dict(cfg, 301)
    a, b = gen.windows(302, 3), gen.windows(303, 3)
    ids = ov.encode_ids(sd, np.concatenate([a, b], axis=1), cfg, n_cycles=2)
    assert np.array_equal(ids[:, :16], ov.encode_ids(sd, a, cfg, 1))
    assert np.array_equal(ids[:, 16:], ov.encode_ids(sd, b, cfg, 1))


def test_autoregressive_dataset_matches_oracle():
    from arcweld.tokenize import MyLatentAutoregressiveDataset
    data = gen.randint(7, (5, 32), 0, 500)
    labels = gen.randint(8, (5,), 0, 2)
    ds = MyLatentAutoregressiveDataset(data, labels)
    x, y, nc = ov.autoregressive_pairs(data)
    assert ds.num_classes == nc == int(data.max()) + 3
    for i in range(5):
        xi, ci, yi = ds[i]
        assert xi.dtype == torch.long and yi.dtype == torch.long
        assert np.array_equal(xi.numpy(), x[i]) and np.array_equal(yi.numpy(), y[i]) and int(ci) == labels[i]
    ds2 = MyLatentAutoregressiveDataset(data)
    assert ds2[0][1].shape == (1,) and int(ds2[0][1][0]) == 0


def _model(kw, wseed):
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.1, batch_norm=False, **kw)
    sd = ov.det_state_dict(ov.VQVAEConfig(**kw), wseed)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().eval(), sd


@pytest.mark.gpu
def test_encode_ids_full_size_matches_reference_fixture():
    g = golden("vqvae_full_b4.npz")
    m, _ = _model(FULL, 309)
    ids = m.encode_ids(torch.tensor(gen.windows(310, 4), device="cuda"))
    assert ids.shape == (4, 16)
    assert np.array_equal(ids.cpu().numpy().reshape(-1), g["idx"])


@pytest.mark.gpu
def test_encode_ids_multicycle_bit_exact_vs_oracle():
    from arcweld.tokenize import encode_ids
    m, sd = _model(FULL, 309)
    nc, B = 20, 3
    x = np.concatenate([gen.windows(900 + i, B) for i in range(nc)], axis=1)
    ids = encode_ids(m, torch.tensor(x, device="cuda"))
    ref = ov.encode_ids(sd, x, ov.VQVAEConfig(**FULL), n_cycles=nc)
    assert ids.shape == (B, nc * 16)
    assert np.array_equal(ids.cpu().numpy(), ref), f"{(ids.cpu().numpy() != ref).sum()} mismatches"


@pytest.mark.gpu
def test_encode_ids_bf16_mostly_agrees():
    from arcweld.tokenize import encode_ids
    m, _ = _model(FULL, 309)
    x = torch.tensor(gen.windows(77, 256), device="cuda")
    a = encode_ids(m, x)
    b = encode_ids(m, x, dtype=torch.bfloat16)
    assert (a == b).float().mean().item() > 0.9
