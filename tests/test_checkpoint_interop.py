"""Lightning checkpoints written from the REFERENCE modules (tests/golden/ref_*.ckpt: the .ckpt layout --
state_dict, hyper_parameters, epoch, global_step, ... -- built by tests/golden/make_golden.py from the reference's
own VQVAEPatch / MyTransformerDecoder) load into the drop-in through load_from_checkpoint (utils.py:30,
train_transformer_mtasks.py:171; torch.load(weights_only=True): tensors and plain values only), keep every
state_dict entry, and reproduce the reference's eval outputs (fp32)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden


def _load(cls_name, fname):
    from model.transformer_decoder import MyTransformerDecoder
    from model.vq_vae_patch_embedd import VQVAEPatch
    cls = {"vqvae": VQVAEPatch, "decoder": MyTransformerDecoder}[cls_name]
    path = os.path.join(GOLDEN, fname)
    return cls.load_from_checkpoint(path), torch.load(path, map_location="cpu", weights_only=True)


@pytest.mark.parametrize("kind,fname", [("vqvae", "ref_vqvae_small.ckpt"), ("decoder", "ref_decoder_small.ckpt")])
def test_reference_checkpoint_loads_with_every_key(kind, fname):
    m, ck = _load(kind, fname)
    sd = m.state_dict()
    assert set(sd) == set(ck["state_dict"])
    for k, v in ck["state_dict"].items():
        assert torch.equal(sd[k].cpu(), v), k
    for k, v in ck["hyper_parameters"].items():
        if k in m.hparams:
            assert m.hparams[k] == v, k


@pytest.mark.gpu
def test_reference_checkpoint_reproduces_reference_outputs():
    from arcweld.precision import operands
    from oracle import gen
    g = golden("ref_ckpt_outputs.npz")
    with operands(torch.float32):
        m, _ = _load("vqvae", "ref_vqvae_small.ckpt")
        m = m.cuda().eval()
        x = torch.tensor(gen.windows(1602, 4), device="cuda")
        with torch.no_grad():
            e, xh, p = m(x)
            ids = m.encode_ids(x)
        np.testing.assert_allclose(xh.cpu().numpy(), g["vq_x_hat"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(e.item(), g["vq_emb_loss"], rtol=1e-4)
        np.testing.assert_allclose(p.item(), g["vq_perplexity"], rtol=1e-4)
        assert np.array_equal(ids.reshape(-1).cpu().numpy(), g["vq_idx"])
        d, _ = _load("decoder", "ref_decoder_small.ckpt")
        d = d.cuda().eval()
        ids = torch.tensor(gen.randint(1604, (3, 17), 0, 20), device="cuda")
        with torch.no_grad():
            lg = d(ids)
            cl = d(ids, generate=False)
        np.testing.assert_allclose(lg.cpu().numpy(), g["dec_logits"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(cl.cpu().numpy(), g["dec_class_logits"], rtol=1e-4, atol=1e-4)
